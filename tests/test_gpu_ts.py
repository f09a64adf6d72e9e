"""Tailstorm on the device (through the C ABI) against the CPU oracle — needs an MI355X.

Every record field is bit-identical: per-node rewards are accumulated in the reference's
fp64 order (set_rewards adds r per confirmed vote; the head's defender reward is the left
fold over nodes), heights are integers and event times follow the same IEEE operation
sequence on both sides. Episodes in which the reference raises (the oracle catches the
exception and records CPR_ST_REFERENCE_RAISES) or whose optimal quorum search would pass
its budget (pruned, so not reached at these configurations; CPR_ST_CAPACITY on both
sides) must be flagged identically on the device; the lane's own capacities must never be hit at these configurations, and flagged
episodes stay out of the summary (cpr_summary.invalid).
"""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f not in ("status",)]
BAD = 32 | 64


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def _cfg(**kw):
    kw.setdefault("protocol", L.PROTO_TAILSTORM)
    kw.setdefault("k", 8)
    kw.setdefault("reward_scheme", L.REWARD_DISCOUNT)
    kw.setdefault("subblock_selection", L.SELECT_HEURISTIC)
    return device.make_config(**kw)


def _compare(cfg, keep, n, first=0):
    b = device.Batch(cfg, keep=keep)
    s, rec = b.run(n, first_episode=first, records=True)
    ok = (rec["status"] & BAD) == 0
    ref = O.run_episodes(cfg, first, n, threads=8)
    # flags: exactly the episodes the oracle flags (reference exception, quorum budget)
    assert np.array_equal(rec["status"] & BAD, ref["status"] & BAD), (
        np.nonzero((rec["status"] & BAD) != (ref["status"] & BAD))[0][:8])
    for f in FIELDS:
        bad = np.nonzero((rec[f] != ref[f]) & ok)[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])
    assert s.episodes == int(ok.sum()) and s.invalid == n - int(ok.sum())
    flagged = n - int(ok.sum())
    if flagged:
        print(f"{flagged}/{n} episodes flagged identically on both sides "
              f"(raises {int(((rec['status'] & 64) != 0).sum())})")
    return s, rec, ok


GYM = [
    # alpha, gamma, policy, scheme, selection, k, steps, episodes
    (0.33, 0.5, L.TS_POLICY_HONEST, L.REWARD_DISCOUNT, L.SELECT_HEURISTIC, 8, 2048, 128),
    (0.33, 0.5, L.TS_POLICY_AVOID_LOSS, L.REWARD_DISCOUNT, L.SELECT_HEURISTIC, 8, 2048, 128),
    (0.25, 0.0, L.TS_POLICY_GET_AHEAD, L.REWARD_CONSTANT, L.SELECT_ALTRUISTIC, 8, 600, 256),
    (0.40, 0.9, L.TS_POLICY_LONG_DELAY, L.REWARD_HYBRID, L.SELECT_HEURISTIC, 8, 600, 256),
    (0.33, 0.8, L.TS_POLICY_MINOR_DELAY, L.REWARD_PUNISH, L.SELECT_HEURISTIC, 13, 600, 64),
    (0.30, 0.5, L.TS_POLICY_AVOID_LOSS_A, L.REWARD_CONSTANT, L.SELECT_OPTIMAL, 8, 400, 128),
    (0.20, 0.5, L.TS_POLICY_AVOID_LOSS_B, L.REWARD_DISCOUNT, L.SELECT_HEURISTIC, 3, 600, 256),
]


@pytest.mark.parametrize("alpha,gamma,policy,scheme,sel,k,steps,n", GYM)
def test_ts_gym_records_match_oracle(ctx, alpha, gamma, policy, scheme, sel, k, steps, n):
    cfg, keep = _cfg(alpha=alpha, gamma=gamma, policy=policy, reward_scheme=scheme,
                     subblock_selection=sel, k=k, max_steps=steps, seed=0x7A110000)
    s, rec, ok = _compare(cfg, keep, n)
    assert (rec["n_steps"][ok] == steps).all()


@pytest.mark.parametrize("policy", [0, 1, 3, 6])
def test_ts_two_agents_loop_matches_oracle(ctx, policy):
    # BASELINE configs[3]: two agents, k = 8, discount, heuristic
    cfg, keep = _cfg(alpha=0.33, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP, activations=10000,
                     policy=policy, seed=11)
    _, _, ok = _compare(cfg, keep, 64)
    assert ok.all()


def test_ts_lockstep_matches_oracle_step_by_step(ctx):
    n, steps = 12, 200
    cfg, keep = _cfg(alpha=0.33, gamma=0.5, max_steps=steps, seed=99, n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    envs = [O.TsGymEnv(cfg, episode=i) for i in range(n)]
    assert np.array_equal(obs, np.array([e.reset() for e in envs]))
    rnd = np.random.default_rng(0)
    for t in range(steps):
        acts = rnd.integers(0, 8, size=n).astype(np.int32)
        acts[::2] = [O.ts_policy("avoid-loss", e.fields(), 8) for e in envs[::2]]
        obs, rew, done, info = b.step(acts)
        for i, e in enumerate(envs):
            o, r, d, inf = e.step(int(acts[i]))
            assert np.array_equal(obs[i], o), (t, i)
            assert rew[i] == r and done[i] == d, (t, i)
            for key in ["episode_reward_attacker", "episode_reward_defender",
                        "episode_progress", "episode_chain_time", "episode_sim_time",
                        "episode_n_steps", "episode_n_activations", "head_height"]:
                assert info[key][i] == inf[key], (t, i, key)
    assert done.all()


def test_ts_policy_decoding(ctx):
    n = 6
    cfg, keep = _cfg(alpha=0.4, gamma=0.5, max_steps=200, seed=5, n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    envs = [O.TsGymEnv(cfg, episode=i) for i in range(n)]
    for e in envs:
        e.reset()
    for t in range(80):
        assert np.array_equal(b.observe_fields(), np.array([e.fields() for e in envs]))
        for name, pid in device.policy_registry(L.PROTO_TAILSTORM):
            assert b.policy_actions(pid, obs).tolist() == [
                O.ts_policy(name, e.fields(), 8) for e in envs], name
        acts = np.array([O.ts_policy("minor-delay", e.fields(), 8) for e in envs], np.int32)
        obs, _, _, _ = b.step(acts, with_info=False)
        for i, e in enumerate(envs):
            e.step(int(acts[i]))


def test_ts_rollout_matches_sequential_oracle_episodes(ctx):
    n, T, ms = 16, 200, 60
    cfg, keep = _cfg(alpha=0.33, gamma=0.5, policy=L.TS_POLICY_GET_AHEAD, max_steps=ms, seed=7,
                     n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    s, obs, rew, done = b.rollout(T, outputs=True)
    assert s.steps == n * T
    finished = 0
    acts_total = 0
    for i in range(n):
        ep = i
        e = O.TsGymEnv(cfg, episode=ep)
        e.reset()
        for t in range(T):
            o, r, d, info = e.step(O.ts_policy("get-ahead", e.fields(), 8))
            assert rew[t, i] == r and done[t, i] == d, (i, t)
            if d:
                finished += 1
                acts_total += int(info["episode_n_activations"])
                ep += n
                e = O.TsGymEnv(cfg, episode=ep)
                o = e.reset()
            assert np.array_equal(obs[t, i], o), (i, t)
        assert not d  # T is no multiple of max_steps: every lane ends mid-episode
        acts_total += int(info["episode_n_activations"])
    assert s.episodes == finished
    assert s.activations == acts_total, (s.activations, acts_total)
    # the same rollout in two launches (lanes resume at their decision point)
    b2 = device.Batch(cfg, keep=keep)
    sa, obs_a, rew_a, done_a = b2.rollout(77, outputs=True)
    sb, obs_b, rew_b, done_b = b2.rollout(T - 77, outputs=True)
    assert np.array_equal(np.concatenate([obs_a, obs_b]), obs)
    assert np.array_equal(np.concatenate([rew_a, rew_b]), rew)
    assert np.array_equal(np.concatenate([done_a, done_b]), done)
    assert sa.activations + sb.activations == s.activations
    assert sa.episodes + sb.episodes == s.episodes


def test_ts_spec_registry_and_validation(ctx):
    assert [x for x, _ in device.policy_registry(L.PROTO_TAILSTORM)] == [
        "long-delay", "avoid-loss-b", "avoid-loss-a", "avoid-loss", "minor-delay", "get-ahead",
        "honest"]
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, max_steps=10)
    assert device.Batch(cfg, keep=keep).observation_spec()[:2] == (10, 8)
    for bad in [dict(k=0), dict(reward_scheme=L.REWARD_BLOCK), dict(subblock_selection=5)]:
        cfg, keep = _cfg(alpha=0.3, gamma=0.5, max_steps=10, **bad)
        with pytest.raises(L.CprError) as e:
            device.Batch(cfg, keep=keep)
        assert e.value.code == L.CPR_E_INVALID_ARG


# ---- table-driven tailstorm_ssz policy (CPR_TS_POLICY_TABLE)

def _ts_table(k, dim=5, seed=4):
    return np.random.default_rng(seed).integers(0, 8, size=dim * dim * (k + 1) ** 2 * 3).astype(
        np.uint8)


@pytest.mark.parametrize("mode", ["gym", "loop"])
def test_ts_table_policy_matches_oracle(ctx, mode):
    k = 8
    table = _ts_table(k)
    if mode == "gym":
        cfg, keep = _cfg(alpha=0.33, gamma=0.5, table=table, k=k, max_steps=400, seed=0x7AB1E)
    else:
        cfg, keep = _cfg(alpha=0.33, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP,
                         activations=3000, table=table, k=k, seed=0x7AB1E)
    assert cfg.policy == L.TS_POLICY_TABLE
    _compare(cfg, keep, 128)


def test_ts_table_policy_decoding_and_rollout(ctx):
    k = 4
    table = _ts_table(k, dim=4, seed=11)
    n, T, ms = 12, 120, 40
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, table=table, k=k, max_steps=ms, seed=22, n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    fields = b.observe_fields()
    assert b.policy_actions(L.TS_POLICY_TABLE, obs).tolist() == [
        O.ts_policy(L.TS_POLICY_TABLE, f, k, table=table) for f in fields]
    b2 = device.Batch(cfg, keep=keep)
    s, _, rew, done = b2.rollout(T, outputs=True)
    for i in range(4):
        e, ep = O.TsGymEnv(cfg, episode=i), i
        e.reset()
        for t in range(T):
            _, r, d, _ = e.step(O.ts_policy(L.TS_POLICY_TABLE, e.fields(), k, table=table))
            assert rew[t, i] == r and done[t, i] == d, (i, t)
            if d:
                ep += n
                e = O.TsGymEnv(cfg, episode=ep)
                e.reset()


def test_ts_rollout_envs_per_wave_ragged(ctx, monkeypatch):
    """As test_bk_rollout_envs_per_wave_ragged, for the Tailstorm rollout."""
    n, T, ms = 100, 40, 25
    cfg, keep = _cfg(alpha=0.33, gamma=0.5, policy=L.TS_POLICY_GET_AHEAD, max_steps=ms,
                     seed=654, n_lanes=n)
    outs = {}
    for w in ("64", "32", "16", None):
        if w is None:
            monkeypatch.delenv("CPR_ROLL_LPW", raising=False)
        else:
            monkeypatch.setenv("CPR_ROLL_LPW", w)
        b = device.Batch(cfg, keep=keep)
        s, obs, rew, done = b.rollout(T, outputs=True)
        outs[w] = (s.steps, s.episodes, s.activations, obs, rew, done)
    ref = outs["64"]
    for w, o in outs.items():
        assert o[:3] == ref[:3], w
        for a, r in zip(o[3:], ref[3:]):
            assert np.array_equal(a, r), w
    _, _, _, obs, rew, done = ref
    for i in (0, 15, 16, 63, 64, 95, 96, 99):
        ep = i
        e = O.TsGymEnv(cfg, episode=ep)
        e.reset()
        for t in range(T):
            o, r, d, info = e.step(O.ts_policy("get-ahead", e.fields(), 8))
            assert rew[t, i] == r and done[t, i] == d, (i, t)
            if d:
                ep += n
                e = O.TsGymEnv(cfg, episode=ep)
                o = e.reset()
            assert np.array_equal(obs[t, i], o), (i, t)


@pytest.mark.parametrize("twin", ["0", "2"])
def test_ts_list_record_window_equals_ring(ctx, monkeypatch, twin):
    # configs[3]'s shape at 2,048 episodes: the fused kernel with the list records of each
    # lane's newest 8 vertices in LDS (the default, TsMem.tl) gives the summary, field for
    # field, that it gives with every record read from the ring in HBM (CPR_TS_TWIN=0) and
    # with a 2-row window that wraps every other append
    cfg, keep = _cfg(alpha=0.33, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP, activations=2000,
                     policy=L.TS_POLICY_AVOID_LOSS, seed=0x7A11)
    b = device.Batch(cfg, keep=keep)
    monkeypatch.delenv("CPR_TS_TWIN", raising=False)
    s_win = b.run(2048, first_episode=0)
    monkeypatch.setenv("CPR_TS_TWIN", twin)
    s_alt = b.run(2048, first_episode=0)
    assert s_win.episodes == 2048 and s_win.invalid == 0
    for f in L.Summary.FIELDS:
        assert getattr(s_win, f) == getattr(s_alt, f), f
    assert list(s_win.hist) == list(s_alt.hist)
