"""engine.ml:209-214's done clause beyond max_steps — needs an MI355X.

An episode ends when ``not (steps < max_steps && progress < max_progress && now <
max_time)``: progress is ``Ref.progress`` of the head (height for Nakamoto, work for
Ethereum, the protocols' own measure for B_k and Tailstorm) and ``now`` the simulation
clock at the attacker's interaction. Every kernel family evaluates the clause itself
(kernels.hip run_gym, eth_window.h / ethereum_lane.h / bk_lane.h / ts_lane.h gym_step),
so each is compared here with the oracle (oracle/src: des.cpp, ethereum.cpp, bk.cpp,
tailstorm.cpp) on episodes that a finite max_time or max_progress ends before max_steps:
fused records field by field, lockstep steps (observation, reward, done, info) one by one,
and device rollouts' auto-resets against sequential oracle episodes. The two tests of the
reference's test_daa.py run on cpr_amd.envs at the end.
"""

import collections
import os

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device, envs, protocols

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f not in ("status",)]
INFO = ["episode_reward_attacker", "episode_reward_defender", "episode_progress",
        "episode_chain_time", "episode_sim_time", "episode_n_steps", "episode_n_activations",
        "head_height", "head_miner"]


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def _records(cfg, keep, n, first=0, bad_mask=0):
    b = device.Batch(cfg, keep=keep)
    s, rec = b.run(n, first_episode=first, records=True)
    ref = O.run_episodes(cfg, first, n, threads=8)
    ok = (rec["status"] & bad_mask) == 0 if bad_mask else np.ones(n, bool)
    if bad_mask:  # flags (capacity, reference exceptions) identical on both sides
        assert np.array_equal(rec["status"] & bad_mask, ref["status"] & bad_mask)
    for f in FIELDS:
        bad = np.nonzero((rec[f] != ref[f]) & ok)[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])
    return b, s, rec, ok


def _ended_early(rec, ok, max_steps, max_time, max_progress):
    """The clause really bit: most episodes stop before max_steps, each for a reason the
    clause names (time reached, or progress reached)."""
    early = (rec["n_steps"] < max_steps) & ok
    assert early.sum() >= ok.sum() // 2, (int(early.sum()), int(ok.sum()))
    why = np.zeros(len(rec), bool)
    if max_time is not None:
        why |= rec["sim_time"] >= max_time
    if max_progress is not None:
        why |= rec["progress"] >= max_progress
    assert why[early].all()
    return early


# ---------------------------------------------------------------- Nakamoto

NAK = [
    # alpha, gamma, policy, max_time, max_progress, propagation delay, episodes
    (0.33, 0.5, L.POLICY_SAPIRSHTEIN_2016_SM1, 300.0, None, 1e-9, 1024),
    (0.33, 0.5, L.POLICY_SAPIRSHTEIN_2016_SM1, None, 200.0, 1e-9, 1024),
    (0.25, 0.0, L.POLICY_HONEST, 300.0, None, 1e-9, 512),
    (0.45, 0.0, L.POLICY_SAPIRSHTEIN_2016_SM1, None, 150.0, 1e-9, 512),
    (0.45, 0.9, L.POLICY_EYAL_SIRER_2014, None, 150.0, 1e-9, 512),
    (0.40, 0.5, L.POLICY_EYAL_SIRER_2014, 250.0, 180.0, 1e-9, 512),
    # long delay: nearly every episode overlaps and is re-run on the exact event engine,
    # which evaluates the same clause (ethereum_lane.h gym_step in Nakamoto mode)
    (0.42, 0.5, L.POLICY_SAPIRSHTEIN_2016_SM1, 200.0, None, 0.05, 256),
    (0.42, 0.5, L.POLICY_SAPIRSHTEIN_2016_SM1, None, 120.0, 0.05, 256),
]


@pytest.mark.parametrize("alpha,gamma,policy,mt,mp,prop,n", NAK)
def test_nakamoto_fused_termination_matches_oracle(ctx, alpha, gamma, policy, mt, mp, prop, n):
    ms = 2016
    cfg, keep = device.make_config(alpha=alpha, gamma=gamma, policy=policy, max_steps=ms,
                                   max_time=mt, max_progress=mp, propagation_delay=prop,
                                   seed=0x7E2A0000)
    b, s, rec, ok = _records(cfg, keep, n)
    _ended_early(rec, ok, ms, mt, mp)
    if prop > 1e-3:
        assert ((rec["status"] & L.ST_EXACT_RERUN) != 0).sum() > n // 4
    # the summary-only specialisation (the bench's kernels) evaluates the clause too
    s0 = b.run(n, first_episode=0)
    for f in L.Summary.FIELDS:
        assert getattr(s0, f) == getattr(s, f), f
    assert s.steps == int(rec["n_steps"].sum())


@pytest.mark.parametrize("mt,mp", [(60.0, None), (None, 40.0)])
def test_nakamoto_lockstep_termination_step_by_step(ctx, mt, mp):
    n, ms = 32, 1000
    cfg, keep = device.make_config(alpha=0.4, gamma=0.5, max_steps=ms, max_time=mt,
                                   max_progress=mp, seed=0x7E2A0100, n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    es = [O.GymEnv(cfg, episode=i) for i in range(n)]
    assert np.array_equal(obs, np.array([e.reset() for e in es]))
    rng = np.random.default_rng(2)
    finished = np.zeros(n, bool)
    t = 0
    while not finished.all():
        acts = rng.integers(0, 4, size=n).astype(np.int32)
        obs, rew, done, info = b.step(acts)
        for i, e in enumerate(es):
            if finished[i]:
                continue
            o, r, d, inf = e.step(int(acts[i]))
            assert np.array_equal(obs[i], o), (t, i)
            assert rew[i] == r and done[i] == d, (t, i)
            for k in INFO:
                assert info[k][i] == inf[k], (t, i, k)
            if d:
                finished[i] = True
                assert inf["episode_n_steps"] < ms
        t += 1
        assert t < ms


# ---------------------------------------------------------------- Ethereum

ETH = [
    # alpha, gamma, policy, max_time, max_progress, propagation delay
    (0.35, 0.5, L.ETH_POLICY_FN19, 300.0, None, 1e-9),
    (0.45, 0.0, L.ETH_POLICY_FN19, None, 150.0, 1e-9),
    (0.40, 0.9, L.ETH_POLICY_SELFISH_RELEASE, 250.0, 200.0, 1e-9),
    (0.40, 0.5, L.ETH_POLICY_FN19, 200.0, None, 0.05),  # window lane hands back, re-runs
]


@pytest.mark.parametrize("route", ["window", "event"])
@pytest.mark.parametrize("alpha,gamma,policy,mt,mp,prop", ETH)
def test_ethereum_fused_termination_matches_oracle(ctx, monkeypatch, route, alpha, gamma,
                                                    policy, mt, mp, prop):
    # route "window": eth_window.h (episodes that fit its block ring), "event": the
    # per-lane event engine (CPR_ETH_WINDOW=0); both against the oracle's ethereum.cpp
    if route == "event":
        monkeypatch.setenv("CPR_ETH_WINDOW", "0")
    ms = 2016
    cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=alpha, gamma=gamma,
                                   policy=policy, max_steps=ms, max_time=mt, max_progress=mp,
                                   propagation_delay=prop, seed=0x7E2A0200)
    _, s, rec, ok = _records(cfg, keep, 256, bad_mask=L.ST_CAPACITY)
    assert ok.all()
    _ended_early(rec, ok, ms, mt, mp)
    assert s.episodes == 256 and s.steps == int(rec["n_steps"].sum())


def test_ethereum_lockstep_termination_step_by_step(ctx):
    n, ms = 16, 1000
    cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=0.35, gamma=0.5,
                                   max_steps=ms, max_time=80.0, seed=0x7E2A0300, n_lanes=n,
                                   reward_scheme=L.REWARD_DISCOUNT)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    es = [O.EthGymEnv(cfg, episode=i) for i in range(n)]
    assert np.array_equal(obs, np.array([e.reset() for e in es]))
    rng = np.random.default_rng(4)
    finished = np.zeros(n, bool)
    t = 0
    while not finished.all():
        acts = rng.integers(0, 24, size=n).astype(np.int32)
        obs, rew, done, info = b.step(acts)
        for i, e in enumerate(es):
            if finished[i]:
                continue
            o, r, d, inf = e.step(int(acts[i]))
            assert np.array_equal(obs[i], o), (t, i)
            assert rew[i] == r and done[i] == d, (t, i)
            for k in INFO:
                assert info[k][i] == inf[k], (t, i, k)
            finished[i] |= d
        t += 1
        assert t < ms


# ---------------------------------------------------------------- B_k and Tailstorm

def _bk_cfg(**kw):
    return device.make_config(protocol=L.PROTO_BK, k=8, **kw)


def _ts_cfg(**kw):
    kw.setdefault("reward_scheme", L.REWARD_DISCOUNT)
    kw.setdefault("subblock_selection", L.SELECT_HEURISTIC)
    return device.make_config(protocol=L.PROTO_TAILSTORM, k=8, **kw)


EVENT = [
    # protocol, policy, gamma, max_time, max_progress
    ("bk", L.BK_POLICY_MINOR_DELAY, 0.5, 300.0, None),
    ("bk", L.BK_POLICY_AVOID_LOSS, 0.0, None, 40.0),
    ("bk", L.BK_POLICY_HONEST, 0.5, 250.0, 30.0),
    ("ts", L.TS_POLICY_AVOID_LOSS, 0.5, 300.0, None),
    ("ts", L.TS_POLICY_GET_AHEAD, 0.0, None, 40.0),
    ("ts", L.TS_POLICY_HONEST, 0.5, 250.0, 30.0),
]


@pytest.mark.parametrize("proto,policy,gamma,mt,mp", EVENT)
def test_bk_ts_fused_termination_matches_oracle(ctx, proto, policy, gamma, mt, mp):
    ms = 2048
    mk = _bk_cfg if proto == "bk" else _ts_cfg
    cfg, keep = mk(alpha=0.33, gamma=gamma, policy=policy, max_steps=ms, max_time=mt,
                   max_progress=mp, seed=0x7E2A0400)
    _, s, rec, ok = _records(cfg, keep, 128, bad_mask=L.ST_CAPACITY | L.ST_REFERENCE_RAISES)
    _ended_early(rec, ok, ms, mt, mp)
    assert s.episodes == int(ok.sum())


@pytest.mark.parametrize("proto", ["bk", "ts"])
def test_bk_ts_lockstep_termination_step_by_step(ctx, proto):
    n, ms = 16, 2000
    mk, Env, na = ((_bk_cfg, O.BkGymEnv, 8) if proto == "bk" else (_ts_cfg, O.TsGymEnv, 8))
    cfg, keep = mk(alpha=0.33, gamma=0.5, max_steps=ms, max_time=60.0, seed=0x7E2A0500,
                   n_lanes=n)
    b = device.Batch(cfg, keep=keep)
    obs = b.reset()
    es = [Env(cfg, episode=i) for i in range(n)]
    assert np.array_equal(obs, np.array([e.reset() for e in es]))
    rng = np.random.default_rng(6)
    finished = np.zeros(n, bool)
    t = 0
    while not finished.all():
        acts = rng.integers(0, na, size=n).astype(np.int32)
        obs, rew, done, info = b.step(acts)
        for i, e in enumerate(es):
            if finished[i]:
                continue
            o, r, d, inf = e.step(int(acts[i]))
            assert np.array_equal(obs[i], o), (t, i)
            assert rew[i] == r and done[i] == d, (t, i)
            for k in INFO:
                assert info[k][i] == inf[k], (t, i, k)
            finished[i] |= d
        t += 1
        assert t < ms


@pytest.mark.parametrize("proto", ["bk", "ts"])
def test_bk_ts_rollout_termination_auto_resets(ctx, proto):
    # cpr_rollout's VecEnv auto-reset on a done the progress clause raises: every lane's
    # rewards and dones equal sequential oracle episodes with the same auto-reset ids
    n, T, ms = 16, 400, 5000
    if proto == "bk":
        cfg, keep = _bk_cfg(alpha=0.33, gamma=0.5, policy=L.BK_POLICY_MINOR_DELAY,
                            max_steps=ms, max_progress=24.0, seed=0x7E2A0600, n_lanes=n)
        Env, pol = O.BkGymEnv, (lambda e: O.bk_policy("minor-delay", e.fields(), 8))
    else:
        cfg, keep = _ts_cfg(alpha=0.33, gamma=0.5, policy=L.TS_POLICY_AVOID_LOSS,
                            max_steps=ms, max_progress=24.0, seed=0x7E2A0600, n_lanes=n)
        Env, pol = O.TsGymEnv, (lambda e: O.ts_policy("avoid-loss", e.fields(), 8))
    b = device.Batch(cfg, keep=keep)
    s, obs, rew, done = b.rollout(T, outputs=True)
    finished = 0
    for i in range(n):
        ep = i
        e = Env(cfg, episode=ep)
        e.reset()
        for t in range(T):
            o, r, d, _ = e.step(pol(e))
            assert rew[t, i] == r and bool(done[t, i]) == d, (i, t)
            if d:
                finished += 1
                ep += n
                e = Env(cfg, episode=ep)
                o = e.reset()
            assert np.array_equal(obs[t, i], o), (i, t)
    assert finished >= n  # the progress clause ended episodes inside the rollout
    assert s.episodes == finished


# ---------------------------------------------------------------- test_daa.py

def test_daa_max_time():
    # gym/ocaml/test/test_daa.py:61-77: max_time stops the episode (max_steps high enough
    # not to), honest play, chain time within 10 of the limit
    os.environ["CPR_SEED"] = "4242"
    try:
        target = 42 * 10
        env = envs.make("cpr_gym:core-v0", proto=protocols.nakamoto(unit_observation=True),
                        max_time=target, max_steps=int(target * 2), activation_delay=1)
        obs = env.reset()
        done = False
        while not done:
            obs, _, done, info = env.step(env.policy(obs, "honest"))
        assert info["episode_chain_time"] >= target - 10
        assert info["episode_sim_time"] >= target and info["episode_n_steps"] < 2 * target
    finally:
        del os.environ["CPR_SEED"]


def test_daa_converges():
    # gym/ocaml/test/test_daa.py:7-58: selfish mining at alpha 1/3, gamma .5 orphans
    # blocks, so the observed block interval misses the target; a moving-average difficulty
    # adjustment over 200 episodes brings it within 600 +- 25. Each env gets its own seed
    # (the reference self-inits OCaml's Random per process; CPR_SEED keeps this repeatable)
    target, eps = 600, 25
    seeds = iter(range(0xDAA0000, 0xDAA0000 + 1000))

    def env_with_activation_delay(x):
        os.environ["CPR_SEED"] = str(next(seeds))
        env = envs.make("cpr_gym:core-v0", proto=protocols.nakamoto(unit_observation=True),
                        max_steps=100, alpha=1 / 3, gamma=0.5, defenders=2,
                        activation_delay=x)
        return env, (lambda obs: env.policy(obs, "sapirshtein-2016-sm1"))

    def episode(env, p):
        obs = env.reset()
        done = False
        while not done:
            obs, _, done, info = env.step(p(obs))
        return info

    try:
        env, p = env_with_activation_delay(target)
        info = episode(env, p)
        observed = info["episode_chain_time"] / info["episode_progress"]
        assert not target - eps < observed < target + eps
        ad = collections.deque([target], maxlen=100)
        ct = collections.deque([info["episode_chain_time"]], maxlen=100)
        pr = collections.deque([info["episode_progress"]], maxlen=100)
        for _ in range(200):
            next_ad = target * np.mean(np.array(ad) / np.array(ct) * np.array(pr))
            ad.append(next_ad)
            env, p = env_with_activation_delay(next_ad)
            info = episode(env, p)
            ct.append(info["episode_chain_time"])
            pr.append(info["episode_progress"])
        observed = np.sum(ct) / np.sum(pr)
        assert target - eps < observed < target + eps, observed
    finally:
        os.environ.pop("CPR_SEED", None)
