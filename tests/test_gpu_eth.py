"""Ethereum on the device (through the C ABI) against the CPU oracle — needs an MI355X.

Every record field is bit-identical: rewards are dyadic (multiples of 1/32 for both
incentive schemes), heights/work are integers and event times follow the same IEEE
operation sequence on both sides (keyed stream, fdlibm log, -ffp-contract=off).
"""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f not in ("status",)]


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def _cfg(**kw):
    kw.setdefault("protocol", L.PROTO_ETHEREUM)
    return device.make_config(**kw)


def _compare(cfg, keep, n, first=0):
    b = device.Batch(cfg, keep=keep)
    s, rec = b.run(n, first_episode=first, records=True)
    ref = O.run_episodes(cfg, first, n, threads=8)
    ok = (rec["status"] & 32) == 0
    # the lane's capacities (block ring, event heap) must hold at the tested configurations
    assert ok.all(), f"{int((~ok).sum())}/{n} episodes hit CPR_ST_CAPACITY"
    assert s.episodes == n and s.invalid == 0
    for f in FIELDS:
        bad = np.nonzero((rec[f] != ref[f]) & ok)[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])
    return s, rec, ok


GYM = [
    # alpha, gamma, policy, scheme, steps, episodes
    (0.35, 0.5, L.ETH_POLICY_FN19, L.REWARD_CONSTANT, 300, 256),
    (0.35, 0.5, L.ETH_POLICY_FN19PKEL, L.REWARD_DISCOUNT, 300, 256),
    (0.25, 0.0, L.ETH_POLICY_SELFISH_RELEASE, L.REWARD_CONSTANT, 300, 256),
    (0.40, 0.9, L.ETH_POLICY_SELFISH_DISCARD, L.REWARD_DISCOUNT, 300, 256),
    (0.10, 0.75, L.ETH_POLICY_HONEST, L.REWARD_CONSTANT, 300, 256),
    (0.45, 0.5, L.ETH_POLICY_FN19, L.REWARD_DISCOUNT, 2016, 128),
]


@pytest.mark.parametrize("alpha,gamma,policy,scheme,steps,n", GYM)
def test_eth_gym_records_match_oracle(ctx, alpha, gamma, policy, scheme, steps, n):
    cfg, keep = _cfg(alpha=alpha, gamma=gamma, policy=policy, reward_scheme=scheme,
                     max_steps=steps, seed=0xE7E70000)
    s, rec, ok = _compare(cfg, keep, n)
    assert (rec["n_steps"] == steps).all()


@pytest.mark.parametrize("policy", [0, 1, 2, 3, 4])
def test_eth_two_agents_loop_matches_oracle(ctx, policy):
    cfg, keep = _cfg(alpha=0.3, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP, activations=10000,
                     policy=policy, reward_scheme=L.REWARD_DISCOUNT, seed=11)
    _compare(cfg, keep, 64)


def test_eth_summary_independent_of_chunking(ctx):
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, policy=L.ETH_POLICY_FN19, max_steps=500, seed=3)
    b = device.Batch(cfg, keep=keep)
    whole = b.run(3000, first_episode=0)
    a = b.run(1000, first_episode=0)
    c = b.run(2000, first_episode=1000)
    for f in ["episodes", "activations", "reward_attacker_fx", "reward_defender_fx",
              "progress_fx", "rel_revenue_fx", "orphans"]:
        assert getattr(whole, f) == getattr(a, f) + getattr(c, f), f


def test_eth_policy_registry_and_spec(ctx):
    assert [n for n, _ in device.policy_registry(L.PROTO_ETHEREUM)] == [
        "fn19pkel", "fn19", "selfish_discard", "selfish_release", "honest"]
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, max_steps=10)
    b = device.Batch(cfg, keep=keep)
    n_obs, n_act, lo, hi = b.observation_spec()
    assert (n_obs, n_act) == (10, 24)
    assert list(lo) == [0.0] * 10 and list(hi) == [1.0] * 10


# ---------------------------------------------------------------- lockstep gym lanes


def test_eth_lockstep_matches_oracle_step_by_step(ctx):
    # engine.ml reset/step over device lanes vs the oracle's engine, every output field;
    # random actions over all 24 (action, uncle-rule) pairs plus a policy on every third lane
    n, steps = 16, 250
    for unit in (True, False):
        cfg, keep = _cfg(alpha=0.35, gamma=0.5, max_steps=steps, seed=77, n_lanes=n,
                         reward_scheme=L.REWARD_DISCOUNT, unit_observation=unit)
        b = device.Batch(cfg, keep=keep)
        obs = b.reset()
        envs = [O.EthGymEnv(cfg, episode=i) for i in range(n)]
        ref = np.array([e.reset() for e in envs])
        assert np.array_equal(obs, ref)
        rnd = np.random.default_rng(1)
        for t in range(steps):
            acts = rnd.integers(0, 24, size=n).astype(np.int32)
            acts[::3] = [O.eth_policy("fn19", e.fields()) for e in envs[::3]]
            obs, rew, done, info = b.step(acts)
            for i, e in enumerate(envs):
                o, r, d, inf = e.step(int(acts[i]))
                assert np.array_equal(obs[i], o), (t, i, obs[i], o)
                assert rew[i] == r and done[i] == d, (t, i)
                for key in ["episode_reward_attacker", "episode_reward_defender",
                            "episode_progress", "episode_chain_time", "episode_sim_time",
                            "episode_n_steps", "episode_n_activations", "head_height",
                            "head_miner"]:
                    assert info[key][i] == inf[key], (t, i, key)
        assert done.all()


def test_eth_observe_fields_and_policy_decoding(ctx):
    n = 8
    for unit in (True, False):
        cfg, keep = _cfg(alpha=0.4, gamma=0.5, max_steps=300, seed=6, n_lanes=n,
                         unit_observation=unit)
        b = device.Batch(cfg, keep=keep)
        obs = b.reset()
        envs = [O.EthGymEnv(cfg, episode=i) for i in range(n)]
        for e in envs:
            e.reset()
        for t in range(100):
            f = b.observe_fields()
            assert np.array_equal(f, np.array([e.fields() for e in envs]))
            for name, pid in device.policy_registry(L.PROTO_ETHEREUM):
                dev = b.policy_actions(pid, obs)
                assert dev.tolist() == [O.eth_policy(name, e.fields()) for e in envs], name
            acts = np.array([O.eth_policy("selfish_release", e.fields()) for e in envs],
                            np.int32)
            obs, _, _, _ = b.step(acts, with_info=False)
            for i, e in enumerate(envs):
                e.step(int(acts[i]))


def test_eth_rollout_matches_sequential_oracle_episodes(ctx):
    n, T, ms = 32, 240, 60
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, policy=L.ETH_POLICY_FN19, max_steps=ms, seed=31,
                     n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    s, obs, rew, done = b.rollout(T, outputs=True)
    assert s.steps == n * T
    finished = 0
    for i in range(n):
        ep = i
        e = O.EthGymEnv(cfg, episode=ep)
        e.reset()
        for t in range(T):
            o, r, d, _ = e.step(O.eth_policy("fn19", e.fields()))
            assert rew[t, i] == r and bool(done[t, i]) == d, (i, t)
            if d:
                finished += 1
                ep += n
                e = O.EthGymEnv(cfg, episode=ep)
                o = e.reset()
            assert np.array_equal(obs[t, i], o), (i, t)
    assert s.episodes == finished
    assert b.rollout(10).steps == n * 10


# ---- table-driven ethereum_ssz policy (CPR_ETH_POLICY_TABLE)

def _eth_table(dim=6, seed=3):
    return np.random.default_rng(seed).integers(0, 24, size=dim * dim * 2).astype(np.uint8)


@pytest.mark.parametrize("mode", ["gym", "loop"])
def test_eth_table_policy_matches_oracle(ctx, mode):
    table = _eth_table()
    if mode == "gym":
        cfg, keep = _cfg(alpha=0.35, gamma=0.5, table=table, reward_scheme=L.REWARD_CONSTANT,
                         max_steps=400, seed=0x7AB1E)
    else:
        cfg, keep = _cfg(alpha=0.35, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP,
                         activations=1200, table=table, reward_scheme=L.REWARD_DISCOUNT,
                         seed=0x7AB1E)
    assert cfg.policy == L.ETH_POLICY_TABLE
    s, rec, ok = _compare(cfg, keep, 256)
    assert s.episodes == 256


def test_eth_table_policy_decoding_and_rollout(ctx):
    table = _eth_table(dim=4, seed=9)
    n, T, ms = 12, 120, 40
    cfg, keep = _cfg(alpha=0.3, gamma=0.5, table=table, max_steps=ms, seed=21, n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    fields = b.observe_fields()
    assert b.policy_actions(L.ETH_POLICY_TABLE, obs).tolist() == [
        O.eth_policy(L.ETH_POLICY_TABLE, f, table=table) for f in fields]
    b2 = device.Batch(cfg, keep=keep)
    s, _, rew, done = b2.rollout(T, outputs=True)
    for i in range(4):
        e, ep = O.EthGymEnv(cfg, episode=i), i
        e.reset()
        for t in range(T):
            _, r, d, _ = e.step(O.eth_policy(L.ETH_POLICY_TABLE, e.fields(), table=table))
            assert rew[t, i] == r and done[t, i] == d, (i, t)
            if d:
                ep += n
                e = O.EthGymEnv(cfg, episode=ep)
                e.reset()


# ---- the window lane (eth_window.h): Ethereum gym episodes on the selfish-mining network
# run a window at a time; what it cannot vouch for is re-run on the event engine

WINDOW = [
    # alpha, gamma, policy, scheme, propagation delay, episodes
    (0.45, 0.0, L.ETH_POLICY_FN19, L.REWARD_CONSTANT, 1e-9, 256),
    (0.45, 0.9, L.ETH_POLICY_FN19, L.REWARD_CONSTANT, 1e-9, 256),
    (0.35, 0.5, L.ETH_POLICY_SELFISH_RELEASE, L.REWARD_CONSTANT, 1e-9, 256),
    # tiny delay: same-instant races are common (tie replay through the skew heap)
    (0.40, 0.5, L.ETH_POLICY_FN19, L.REWARD_DISCOUNT, 1e-13, 256),
    (0.45, 0.9, L.ETH_POLICY_FN19PKEL, L.REWARD_CONSTANT, 1e-13, 256),
    # long delay: activations inside deliveries, re-run on the event engine
    (0.40, 0.5, L.ETH_POLICY_FN19, L.REWARD_CONSTANT, 0.05, 128),
    (0.35, 0.9, L.ETH_POLICY_SELFISH_DISCARD, L.REWARD_DISCOUNT, 0.01, 128),
]


@pytest.mark.parametrize("alpha,gamma,policy,scheme,prop,n", WINDOW)
def test_eth_window_lane_matches_oracle(ctx, alpha, gamma, policy, scheme, prop, n):
    cfg, keep = _cfg(alpha=alpha, gamma=gamma, policy=policy, reward_scheme=scheme,
                     max_steps=2016, propagation_delay=prop, seed=0xE7E71000)
    s, rec, ok = _compare(cfg, keep, n)
    st = rec["status"]
    if prop < 1e-12:
        assert ((st & L.ST_TIE) != 0).sum() > 0  # ties occurred and were replayed
    if prop > 1e-3:
        rerun = (st & L.ST_EXACT_RERUN) != 0
        assert rerun.sum() > n // 4  # most episodes overlapped and were re-run exactly
        assert ((st[rerun] & L.ST_OVERLAP) != 0).all()
    # the summary is the sum of the records (re-runs replace the flagged episodes)
    assert s.episodes == n and s.steps == int(rec["n_steps"].sum())
    assert s.activations == int(rec["n_activations"].sum())
    assert s.reward_attacker_fx == int(np.rint(rec["reward_attacker"] * 2**20).sum())
    assert s.progress_fx == int(np.rint(rec["progress"] * 2**20).sum())


# status_tie / status_overlap are route diagnostics (include/cpr_hip.h cpr_summary): the
# window lane counts its tie replays and hand-backs, the event engine sets neither bit
ROUTE_FIELDS = ("status_tie", "status_overlap")


@pytest.mark.parametrize("gamma,prop", [(0.0, 1e-9), (0.5, 1e-9), (0.9, 1e-9), (0.5, 0.05)])
def test_eth_window_lane_equals_event_engine(ctx, gamma, prop, monkeypatch):
    # the bench's configs[2] point at full episode length: the window lane's summary equals
    # the event engine's (CPR_ETH_WINDOW=0) field for field; at a 0.05 delay most episodes
    # overlap, so the window route's hand-backs (status_overlap) are many and every one was
    # re-run exactly (its records carry CPR_ST_EXACT_RERUN)
    cfg, keep = _cfg(alpha=0.45, gamma=gamma, policy=L.ETH_POLICY_FN19,
                     reward_scheme=L.REWARD_CONSTANT, max_steps=2016, seed=0x5EED0000,
                     propagation_delay=prop)
    b = device.Batch(cfg, keep=keep)
    n = 2048 if prop < 1e-3 else 256
    s_win, rec = b.run(n, first_episode=0, records=True)
    monkeypatch.setenv("CPR_ETH_WINDOW", "0")
    s_ev = b.run(n, first_episode=0)
    for f in L.Summary.FIELDS:
        if f in ROUTE_FIELDS:
            continue
        assert getattr(s_win, f) == getattr(s_ev, f), f
    assert list(s_win.hist) == list(s_ev.hist)
    assert s_ev.status_tie == 0 and s_ev.status_overlap == 0
    handed = int(((rec["status"] & L.ST_OVERLAP) != 0).sum())
    assert s_win.status_overlap == handed
    assert ((rec["status"][(rec["status"] & L.ST_OVERLAP) != 0] & L.ST_EXACT_RERUN) != 0).all()
    if prop > 1e-3:
        assert handed > n // 4


def test_eth_long_episodes_stay_on_the_event_engine(ctx):
    # episodes longer than the window lane's block ring (2^15) go to the event engine, whose
    # ring wraps, instead of ending in a hand-back and a one-lane exact re-run each
    # (capi.hip eth_window_ok); every record equals the oracle's
    cfg, keep = _cfg(alpha=0.35, gamma=0.5, policy=L.ETH_POLICY_FN19,
                     reward_scheme=L.REWARD_CONSTANT, max_steps=33000, seed=0xE7E72000)
    s, rec, ok = _compare(cfg, keep, 32)
    assert not (rec["status"] & (L.ST_EXACT_RERUN | L.ST_OVERLAP)).any()
    assert (rec["n_steps"] == 33000).all() and s.status_overlap == 0
