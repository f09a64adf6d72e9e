"""B_k on the device (through the C ABI) against the CPU oracle — needs an MI355X.

Every record field is bit-identical: rewards are integers (1 per confirmed vote for
`Constant`, k per block for `Block`), heights are integers and event times follow the
same IEEE operation sequence on both sides (keyed stream, fdlibm log,
-ffp-contract=off). The lockstep API is compared step by step (observation floats,
reward, done, info), and the fused rollout (BASELINE configs[4]) step by step for
every lane against sequential oracle episodes with the same auto-reset ids.
"""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f not in ("status",)]
CAPACITY = 32


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def _cfg(**kw):
    kw.setdefault("protocol", L.PROTO_BK)
    kw.setdefault("k", 8)
    return device.make_config(**kw)


def _compare(cfg, keep, n, first=0):
    b = device.Batch(cfg, keep=keep)
    s, rec = b.run(n, first_episode=first, records=True)
    ref = O.run_episodes(cfg, first, n, threads=8)
    ok = (rec["status"] & CAPACITY) == 0
    for f in FIELDS:
        bad = np.nonzero((rec[f] != ref[f]) & ok)[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])
    return s, rec, ok


GYM = [
    # alpha, gamma, policy, scheme, k, steps, episodes
    (0.33, 0.5, L.BK_POLICY_HONEST, L.REWARD_CONSTANT, 8, 2048, 128),
    (0.33, 0.5, L.BK_POLICY_MINOR_DELAY, L.REWARD_BLOCK, 8, 2048, 128),
    (0.25, 0.0, L.BK_POLICY_GET_AHEAD, L.REWARD_CONSTANT, 8, 600, 256),
    (0.40, 0.9, L.BK_POLICY_AVOID_LOSS, L.REWARD_BLOCK, 8, 600, 256),
    (0.33, 0.3, L.BK_POLICY_MINOR_DELAY, L.REWARD_CONSTANT, 42, 600, 64),
    (0.20, 0.5, L.BK_POLICY_AVOID_LOSS, L.REWARD_CONSTANT, 2, 600, 256),
]


@pytest.mark.parametrize("alpha,gamma,policy,scheme,k,steps,n", GYM)
def test_bk_gym_records_match_oracle(ctx, alpha, gamma, policy, scheme, k, steps, n):
    cfg, keep = _cfg(alpha=alpha, gamma=gamma, policy=policy, reward_scheme=scheme, k=k,
                     max_steps=steps, seed=0xB0B00000)
    s, rec, ok = _compare(cfg, keep, n)
    assert ok.all()
    assert s.episodes == n and (rec["n_steps"] == steps).all()
    assert (rec["reward_attacker"] + rec["reward_defender"] == rec["progress"]).all()


def test_bk_table_policy_matches_oracle(ctx):
    k, dim = 8, 4
    rnd = np.random.default_rng(5)
    table = rnd.integers(0, 8, size=dim * dim * (k + 1) * (k + 1) * 3).astype(np.uint8)
    cfg, keep = _cfg(alpha=0.33, gamma=0.5, table=table, max_steps=600, seed=17)
    assert cfg.policy == L.BK_POLICY_TABLE and cfg.policy_table_dim == dim
    _compare(cfg, keep, 128)


@pytest.mark.parametrize("policy", [0, 1, 2, 3])
def test_bk_two_agents_loop_matches_oracle(ctx, policy):
    cfg, keep = _cfg(alpha=0.3, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP, activations=4000,
                     policy=policy, seed=11)
    _compare(cfg, keep, 64)


def test_bk_summary_independent_of_chunking(ctx):
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, policy=L.BK_POLICY_MINOR_DELAY, max_steps=400,
                     seed=3)
    b = device.Batch(cfg, keep=keep)
    whole = b.run(2000, first_episode=0)
    a = b.run(700, first_episode=0)
    c = b.run(1300, first_episode=700)
    for f in ["episodes", "steps", "activations", "reward_attacker_fx", "reward_defender_fx",
              "progress_fx", "rel_revenue_fx", "orphans"]:
        assert getattr(whole, f) == getattr(a, f) + getattr(c, f), f


def test_bk_lockstep_matches_oracle_step_by_step(ctx):
    n, steps = 16, 250
    cfg, keep = _cfg(alpha=0.33, gamma=0.5, max_steps=steps, seed=99, n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    envs = [O.BkGymEnv(cfg, episode=i) for i in range(n)]
    ref = np.array([e.reset() for e in envs])
    assert np.array_equal(obs, ref)
    rnd = np.random.default_rng(0)
    for t in range(steps):
        acts = rnd.integers(0, 8, size=n).astype(np.int32)
        acts[::3] = [O.bk_policy("avoid-loss", e.fields(), 8) for e in envs[::3]]
        obs, rew, done, info = b.step(acts)
        for i, e in enumerate(envs):
            o, r, d, inf = e.step(int(acts[i]))
            assert np.array_equal(obs[i], o), (t, i)
            assert rew[i] == r and done[i] == d, (t, i)
            for key in ["episode_reward_attacker", "episode_reward_defender",
                        "episode_progress", "episode_chain_time", "episode_sim_time",
                        "episode_n_steps", "episode_n_activations", "head_height",
                        "head_miner"]:
                assert info[key][i] == inf[key], (t, i, key)
    assert done.all()


def test_bk_observe_fields_and_policy_decoding(ctx):
    n = 8
    cfg, keep = _cfg(alpha=0.4, gamma=0.5, max_steps=300, seed=5, n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    envs = [O.BkGymEnv(cfg, episode=i) for i in range(n)]
    for e in envs:
        e.reset()
    for t in range(120):
        f = b.observe_fields()
        assert np.array_equal(f, np.array([e.fields() for e in envs]))
        for name, pid in device.policy_registry(L.PROTO_BK):
            dev = b.policy_actions(pid, obs)
            assert dev.tolist() == [O.bk_policy(name, e.fields(), 8) for e in envs], name
        acts = np.array([O.bk_policy("minor-delay", e.fields(), 8) for e in envs], np.int32)
        obs, _, _, _ = b.step(acts, with_info=False)
        for i, e in enumerate(envs):
            e.step(int(acts[i]))


def test_bk_rollout_matches_sequential_oracle_episodes(ctx):
    n, T, ms = 32, 300, 70
    cfg, keep = _cfg(alpha=0.33, gamma=0.5, policy=L.BK_POLICY_AVOID_LOSS, max_steps=ms,
                     seed=123, n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    s, obs, rew, done = b.rollout(T, outputs=True)
    assert s.steps == n * T
    finished = 0
    acts_total = 0
    for i in range(n):
        ep = i
        e = O.BkGymEnv(cfg, episode=ep)
        e.reset()
        for t in range(T):
            a = O.bk_policy("avoid-loss", e.fields(), 8)
            o, r, d, info = e.step(a)
            assert rew[t, i] == r and bool(done[t, i]) == d, (i, t)
            if d:
                finished += 1
                acts_total += int(info["episode_n_activations"])
                ep += n
                e = O.BkGymEnv(cfg, episode=ep)
                o = e.reset()
            assert np.array_equal(obs[t, i], o), (i, t)
        assert not d  # T is no multiple of max_steps: every lane ends mid-episode
        acts_total += int(info["episode_n_activations"])
    assert s.episodes == finished
    # every activation of the rollout: finished episodes + the lanes' current ones
    assert s.activations == acts_total, (s.activations, acts_total)
    # the same rollout in two launches (lanes resume at their decision point)
    b2 = device.Batch(cfg, keep=keep)
    sa, obs_a, rew_a, done_a = b2.rollout(123, outputs=True)
    sb, obs_b, rew_b, done_b = b2.rollout(T - 123, outputs=True)
    assert np.array_equal(np.concatenate([obs_a, obs_b]), obs)
    assert np.array_equal(np.concatenate([rew_a, rew_b]), rew)
    assert np.array_equal(np.concatenate([done_a, done_b]), done)
    assert sa.activations + sb.activations == s.activations
    assert sa.episodes + sb.episodes == s.episodes
    # a further call continues from the lanes' state
    s2 = b.rollout(10)
    assert s2.steps == n * 10


def test_bk_spec_registry_and_validation(ctx):
    assert [x for x, _ in device.policy_registry(L.PROTO_BK)] == [
        "avoid-loss", "minor-delay", "get-ahead", "honest"]
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, max_steps=10)
    b = device.Batch(cfg, keep=keep)
    n_obs, n_act, lo, hi = b.observation_spec()
    assert (n_obs, n_act) == (8, 8)
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, max_steps=10, unit_observation=False)
    _, _, lo, hi = device.Batch(cfg, keep=keep).observation_spec()
    rlo, rhi = O.bk_obs_range(False)
    assert np.array_equal(lo, rlo) and np.array_equal(hi, rhi)
    for bad in [dict(k=0), dict(reward_scheme=L.REWARD_DISCOUNT)]:
        cfg, keep = _cfg(alpha=0.3, gamma=0.5, max_steps=10, **bad)
        with pytest.raises(L.CprError) as e:
            device.Batch(cfg, keep=keep)
        assert e.value.code == L.CPR_E_INVALID_ARG


class _HipBuffer:
    """Device memory through the HIP runtime (ctypes), for rollout outputs too large to
    stage through the host."""

    def __init__(self, nbytes):
        import ctypes

        self.hip = ctypes.CDLL("libamdhip64.so")
        self.p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(self.p), ctypes.c_size_t(nbytes)) == 0
        self.nbytes = nbytes

    def rows(self, dtype, shape, lanes):
        """host copy of columns `lanes` of a [T][n] row-major device array"""
        import ctypes

        T, n = shape
        item = np.dtype(dtype).itemsize
        out = np.zeros((T, len(lanes)), dtype)
        host = np.zeros(n, dtype)
        for t in range(T):
            src = ctypes.c_void_p(self.p.value + t * n * item)
            assert self.hip.hipMemcpy(host.ctypes.data_as(ctypes.c_void_p), src,
                                      ctypes.c_size_t(n * item), 2) == 0  # DeviceToHost
            out[t] = host[lanes]
        return out

    def free(self):
        self.hip.hipFree(self.p)


def test_configs4_full_size_table_rollout(ctx):
    # BASELINE configs[4]: 65,536 lockstep B_k k=8 envs (bk(k=8, reward="constant") +
    # bk_ssz, alpha .33, gamma .5, d = 2) stepped by an on-device table policy for 2048-step
    # episodes (experiments/train/configs/bk-8.yaml:7-8, ppo.py:278-285); T = 2,200 steps so
    # every lane finishes its first episode and auto-resets
    n, T, ms, K, D = 65536, 2200, 2048, 8, 4
    table = np.random.default_rng(41).integers(0, 8, size=D * D * (K + 1) ** 2 * 3).astype(
        np.uint8)
    cfg, keep = _cfg(alpha=0.33, gamma=0.5, table=table, k=K, max_steps=ms, seed=4,
                     n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    rew = _HipBuffer(T * n * 8)
    done = _HipBuffer(T * n)
    try:
        s = b.rollout(T, device_outputs=(None, rew.p.value, done.p.value))
        assert s.steps == n * T and s.invalid == 0
        assert s.episodes >= n  # every lane finished at least one 2048-step episode
        assert s.activations > s.steps * 0.5
        # sampled lanes, bit for bit against sequential oracle episodes (auto-reset ids
        # lane, lane + n, ...)
        lanes = [0, 1, 777, 40000, n - 1]
        r = rew.rows(np.float64, (T, n), lanes)
        d = done.rows(np.uint8, (T, n), lanes)
        for c, i in enumerate(lanes):
            ep = i
            e = O.BkGymEnv(cfg, episode=ep)
            e.reset()
            ret = 0.0
            for t in range(T):
                _, rr, dd, info = e.step(O.bk_policy(L.BK_POLICY_TABLE, e.fields(), K,
                                                     table=table, dim=D))
                assert r[t, c] == rr and bool(d[t, c]) == dd, (i, t)
                ret += rr
                if dd:
                    # reward conservation: the step rewards sum to the episode's reward
                    assert ret == info["episode_reward_attacker"], (i, t)
                    assert info["episode_n_steps"] == ms
                    ep += n
                    e = O.BkGymEnv(cfg, episode=ep)
                    e.reset()
                    ret = 0.0
        print(f"configs[4]: {s.steps} env-steps, {s.activations} activations, "
              f"{s.episodes} finished episodes")
    finally:
        rew.free()
        done.free()


def test_bk_rollout_envs_per_wave_ragged(ctx, monkeypatch):
    """A ragged batch (100 envs: the last wave partly used) gives the same outputs at 64, 32
    and 16 envs per wave (CPR_ROLL_LPW; the default picks 16 here), and sampled lanes equal
    sequential oracle episodes."""
    n, T, ms = 100, 40, 25
    cfg, keep = _cfg(alpha=0.33, gamma=0.5, policy=L.BK_POLICY_AVOID_LOSS, max_steps=ms,
                     seed=321, n_lanes=n)
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
        e = O.BkGymEnv(cfg, episode=ep)
        e.reset()
        for t in range(T):
            o, r, d, info = e.step(O.bk_policy("avoid-loss", e.fields(), 8))
            assert rew[t, i] == r and bool(done[t, i]) == d, (i, t)
            if d:
                ep += n
                e = O.BkGymEnv(cfg, episode=ep)
                o = e.reset()
            assert np.array_equal(obs[t, i], o), (i, t)
