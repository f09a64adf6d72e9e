"""Parity of the HIP path (through the C ABI) with the CPU oracle — needs an MI355X.

Integer/index results must be bit-identical; event times (f64) too, because both sides
evaluate the keyed stream and the clock with the same IEEE operation sequence
(-ffp-contract=off, fdlibm log). Observation floats of the lockstep API are compared
exactly as well (host-tabulated libm atan on both sides).
"""

import math

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device

pytestmark = pytest.mark.gpu

# every outcome field; `status` holds engine-specific diagnostics (the oracle flags any
# same-instant equal-height delivery, the device only the races it replays) and is
# checked separately
FIELDS = [f for f in L.RECORD_DTYPE.names if f not in ("status",)]


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def _records_equal(a, b):
    bad = {}
    for f in FIELDS:
        neq = np.nonzero(a[f] != b[f])[0]
        if len(neq):
            bad[f] = (int(neq[0]), a[f][neq[0]], b[f][neq[0]], len(neq))
    return bad


def test_stream_fill_matches_oracle(ctx):
    for seed, ep, tag in [(0, 0, 0), (0x5EED0000, 12345, 0), (2**63 + 7, 2**40 + 3, 0x10000002)]:
        blocks, ex = ctx.stream_fill(seed, ep, 17, tag, 4096, with_exp=True)
        for i in [0, 1, 2, 100, 4095]:
            assert blocks[i].tolist() == O.keyed_block(seed, ep, 17 + i, tag).tolist()
        for i in range(0, 4096, 7):
            u = O.u53(int(blocks[i][2]), int(blocks[i][3]))
            assert ex[i] == (-1.0 * 1.0) * O.cpr_log(u)


GRID = [
    # alpha, gamma, policy, steps, episodes
    (0.33, 0.5, L.POLICY_SAPIRSHTEIN_2016_SM1, 300, 512),
    (0.45, 0.5, L.POLICY_EYAL_SIRER_2014, 300, 512),
    (0.25, 0.0, L.POLICY_SAPIRSHTEIN_2016_SM1, 300, 256),
    (0.25, 0.3, L.POLICY_SIMPLE, 300, 256),
    (0.10, 0.75, L.POLICY_HONEST, 300, 256),
    (0.40, 0.9, L.POLICY_SAPIRSHTEIN_2016_SM1, 300, 256),
    (0.50, 0.5, L.POLICY_SIMPLE, 300, 256),
    (0.05, 0.5, L.POLICY_HONEST, 300, 256),
    (0.35, 0.5, L.POLICY_EYAL_SIRER_2014, 2016, 512),
]


@pytest.mark.parametrize("alpha,gamma,policy,steps,n", GRID)
def test_gym_episodes_bit_exact(ctx, alpha, gamma, policy, steps, n):
    cfg, keep = device.make_config(alpha=alpha, gamma=gamma, policy=policy, max_steps=steps,
                                   seed=0x5EED0000)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(n, first_episode=1000, records=True)
    ref = O.run_episodes(cfg, 1000, n, threads=8)
    assert _records_equal(rec, ref) == {}
    assert s.episodes == n
    assert s.activations == int(ref["n_activations"].sum())
    assert (rec["n_activations"] == steps + 1).all()


def test_gym_many_defenders_and_table_policy(ctx):
    rng = np.random.default_rng(3)
    table = rng.integers(0, 4, size=16 * 16 * 2).astype(np.uint8)
    for kw in [dict(alpha=0.3, gamma=0.95, defenders=42, policy=L.POLICY_SAPIRSHTEIN_2016_SM1),
               dict(alpha=0.3, gamma=0.6, defenders=5, table=table)]:
        cfg, keep = device.make_config(max_steps=400, seed=99, **kw)
        b = device.Batch(cfg, ctx=ctx, keep=keep)
        _, rec = b.run(256, first_episode=0, records=True)
        ref = O.run_episodes(cfg, 0, 256, threads=8)
        assert _records_equal(rec, ref) == {}


def test_tie_windows_replayed_exactly(ctx):
    # Match-heavy play: equal-time deliveries (fp64 ties) occur in ~1% of long episodes;
    # the device replays those windows through the skew heap and must agree exactly
    cfg, keep = device.make_config(alpha=0.33, gamma=0.5, policy=L.POLICY_EYAL_SIRER_2014,
                                   max_steps=2016, seed=0xABCDEF)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    _, rec = b.run(3072, first_episode=0, records=True)
    ref = O.run_episodes(cfg, 0, 3072, threads=8)
    assert _records_equal(rec, ref) == {}
    ties = (rec["status"] & L.ST_TIE) != 0
    assert ties.sum() > 0  # the case is actually exercised
    # every race the device replayed is one the oracle saw as a same-instant tie
    assert ((ref["status"][ties] & L.ST_TIE) != 0).all()
    assert int(((rec["status"] & L.ST_TIE_UNRESOLVED) != 0).sum()) == 0


@pytest.mark.parametrize("policy", [L.POLICY_EYAL_SIRER_2014, L.POLICY_SAPIRSHTEIN_2016_SM1])
@pytest.mark.parametrize("gamma,prop", [(0.0, 1e-9), (0.5, 1e-9), (0.0, 1e-5)])
def test_summary_only_kernels_equal_record_kernels(ctx, gamma, prop, policy):
    # cpr_run_episodes without records runs the summary-only specialisations of
    # k_run_episodes (no block-time bookkeeping; gamma = 0 compiled without arrivals and
    # with the lazy clock, which draws no delay while the uniform rules out an overlap; at
    # d = 2 ties by the closed-form rule, a tie it does not cover re-run exactly); with
    # records, the general kernel (heap replay). Match-heavy play at the bench's sizes of
    # episode: every summary field, ties and overlaps included, must be identical. A 1e-5
    # delay sends ~2.5e-5 of activations down the lazy clock's exact branch and makes
    # overlaps (and their exact re-runs) ~1 % of episodes.
    cfg, keep = device.make_config(alpha=0.33, gamma=gamma, policy=policy, max_steps=2016,
                                   seed=0x5A11, propagation_delay=prop)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    n = 65536
    s1, _ = b.run(n, first_episode=0, records=True)
    s0 = b.run(n, first_episode=0)
    for f in L.Summary.FIELDS:
        assert getattr(s0, f) == getattr(s1, f), f
    assert list(s0.hist) == list(s1.hist)
    if gamma > 0:
        assert s1.status_tie > 0  # ties occurred and took the closed-form rule
    if prop > 1e-6:
        assert s1.status_overlap > n // 100  # the exact branch found real overlaps


def test_summary_only_kernel_long_delay_matches_oracle(ctx):
    # propagation delay 20 x the activation delay at gamma = 0: lazy_threshold is 0 there,
    # so lazy_clock_ok must keep the summary-only kernel on the eager clock (with the lazy
    # one its skip test wrapped and missed every overlap, reporting closed-form results);
    # nearly every episode overlaps and is re-run exactly, and the summary must equal the
    # oracle's episodes summed
    cfg, keep = device.make_config(alpha=0.33, gamma=0.0, policy=L.POLICY_SAPIRSHTEIN_2016_SM1,
                                   max_steps=256, seed=0x1A2E, propagation_delay=20.0)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    n = 512
    s0 = b.run(n, first_episode=0)
    s1, rec = b.run(n, first_episode=0, records=True)
    ref = O.run_episodes(cfg, 0, n, threads=8)
    assert _records_equal(rec, ref) == {}
    for f in L.Summary.FIELDS:
        assert getattr(s0, f) == getattr(s1, f), f
    assert s0.status_overlap > n // 2


@pytest.mark.parametrize("n", [65536, 65536 + 37])
@pytest.mark.parametrize("policy", [L.POLICY_EYAL_SIRER_2014, L.POLICY_SAPIRSHTEIN_2016_SM1])
def test_deferred_races_tie_heavy(ctx, policy, n):
    # gamma = .5 defers its races (k_run_episodes TT = 2); a 1e-10 propagation
    # delay over 2016-step episodes (clock ~1e3, ulp ~1e-13) makes same-instant ties common,
    # so many episodes are flagged and rerun by the eager second pass, some over several
    # rounds of its grid: the summary must still equal the record kernel's (heap replay).
    # n not a multiple of 64: in the launch's last round part of a wave has left the loop,
    # and the lanes still there must verify every entry of the wave's list
    # (nakamoto_lane.h races_check)
    cfg, keep = device.make_config(alpha=0.4, gamma=0.5, policy=policy, max_steps=2016,
                                   propagation_delay=1e-10, seed=0x7E5)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s1, _ = b.run(n, first_episode=0, records=True)
    s0 = b.run(n, first_episode=0)
    for f in L.Summary.FIELDS:
        assert getattr(s0, f) == getattr(s1, f), f
    assert list(s0.hist) == list(s1.hist)
    assert s1.status_tie > n // 50


@pytest.mark.parametrize("alpha,policy,table", [(0.35, L.POLICY_SAPIRSHTEIN_2016_SM1, False),
                                                (0.5, L.POLICY_SAPIRSHTEIN_2016_SM1, False),
                                                (0.35, L.POLICY_EYAL_SIRER_2014, False),
                                                (0.45, L.POLICY_TABLE, True)])
def test_overlapping_windows_rerun_exactly(ctx, alpha, policy, table):
    # Activations that fire while the previous window's messages are in flight: with the
    # gym's 1e-9 propagation delay ~1e-9 of activations, here made common by a 0.05 delay
    # (network.ml selfish_mining ~propagation_delay). The closed-form lane flags them and
    # the library re-runs those episodes on the exact event engine (Nakamoto mode of the
    # Ethereum lane); every record must equal the oracle's, which follows the reference's
    # event queue, and the summary must equal the sum over the records.
    tab = None
    if table:
        tab = np.random.default_rng(3).integers(0, 4, size=12 * 12 * 2).astype(np.uint8)
    cfg, keep = device.make_config(alpha=alpha, gamma=0.5, policy=policy, max_steps=400,
                                   seed=0x0E7, propagation_delay=0.05, table=tab)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(768, first_episode=0, records=True)
    ref = O.run_episodes(cfg, 0, 768, threads=8)
    assert _records_equal(rec, ref) == {}
    flagged = (rec["status"] & L.ST_OVERLAP) != 0
    assert flagged.sum() > 100  # the case is actually exercised
    assert ((rec["status"][flagged] & L.ST_EXACT_RERUN) != 0).all()
    assert ((ref["status"][flagged] & L.ST_OVERLAP) != 0).all()
    assert s.episodes == 768 and s.status_overlap == int(flagged.sum())
    assert s.steps == int(rec["n_steps"].sum())
    assert s.activations == int(rec["n_activations"].sum())
    assert s.reward_attacker_fx == int((rec["reward_attacker"] * 2**20).sum())
    assert s.orphans == int((rec["n_activations"] - rec["head_height"]).sum())
    assert s.status_other == 0


@pytest.mark.parametrize("gamma,prop,policy", [(0.5, 0.05, L.POLICY_SAPIRSHTEIN_2016_SM1),
                                               (0.5, 0.3, L.POLICY_HONEST),
                                               (0.75, 0.05, L.POLICY_EYAL_SIRER_2014)])
def test_hybrid_reruns_equal_whole_episode_reruns(ctx, gamma, prop, policy, monkeypatch):
    # hybrid re-runs (cpr_amd/csrc/nak_hybrid.h: the closed form, the event engine only
    # between quiescent trivial points around each flagged window) against whole-episode
    # re-runs on the event engine (CPR_RERUN_HYBRID=0), on the device: every record field,
    # status included, for 2016-step episodes at delays where nearly every episode
    # overlaps, many times over
    cfg, keep = device.make_config(alpha=0.4, gamma=gamma, policy=policy, max_steps=2016,
                                   seed=0x4B1D, propagation_delay=prop)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    r0 = ctx.rerun_stats()
    _, hyb = b.run(256, first_episode=0, records=True)
    r1 = ctx.rerun_stats()
    monkeypatch.setenv("CPR_RERUN_HYBRID", "0")
    _, whole = b.run(256, first_episode=0, records=True)
    r2 = ctx.rerun_stats()
    assert _records_equal(hyb, whole) == {}
    assert np.array_equal(hyb["status"], whole["status"])
    assert ((hyb["status"] & L.ST_EXACT_RERUN) != 0).sum() > 200
    # and against the oracle (the reference's event-driven restatement on the same keyed
    # stream), not only against the device's own whole-episode engine: every record field
    ref = O.run_episodes(cfg, 0, 256, threads=8)
    assert _records_equal(hyb, ref) == {}
    # both re-ran the same episodes; the hybrid's flush is the shorter by far (the engine
    # simulates only the stretches around the flagged windows)
    assert r1[0] - r0[0] == r2[0] - r1[0]
    print(f"re-run flush ms: hybrid {r1[2] - r0[2]:.1f}, whole episodes {r2[2] - r1[2]:.1f}")
    assert r1[2] - r0[2] < r2[2] - r1[2]


@pytest.mark.parametrize("lds_max", [None, 40960])
def test_gamma0_reruns_exact_with_lds_heap(ctx, lds_max, monkeypatch):
    # gamma = 0 re-runs keep the +inf messages in the event heap (thousands of nodes in a
    # 2016-step episode): the re-run kernel holds the heap in LDS with the capacity that
    # fits and re-runs an episode that outgrows it in HBM (kernels_eth.hip). 40 KiB of LDS
    # forces both paths; every record must equal the oracle's
    if lds_max is not None:
        monkeypatch.setenv("CPR_RERUN_LDS_MAX", str(lds_max))
    cfg, keep = device.make_config(alpha=0.45, gamma=0.0, policy=L.POLICY_SAPIRSHTEIN_2016_SM1,
                                   max_steps=2016, seed=0x0E70, propagation_delay=0.05)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    r0 = ctx.rerun_hbm_retries()
    s, rec = b.run(192, first_episode=0, records=True)
    retries = ctx.rerun_hbm_retries() - r0
    ref = O.run_episodes(cfg, 0, 192, threads=8)
    assert _records_equal(rec, ref) == {}
    flagged = (rec["status"] & L.ST_EXACT_RERUN) != 0
    assert flagged.sum() > 50, int(flagged.sum())
    assert not (rec["status"] & L.ST_CAPACITY).any()
    assert s.episodes == 192
    if lds_max is not None:  # the HBM retry really ran (and its records equal the oracle's)
        assert retries > 0, retries
    print(f"lds_max {lds_max}: {int(flagged.sum())} re-runs, {retries} HBM retries")


def test_gym_overlaps_at_the_reference_delay(ctx):
    # at the gym's own 1e-9 delay overlaps are rare (~1 per 5e8 activations at gamma 0.5);
    # whatever the device flags in 2^16 full episodes was re-run and matches the oracle
    cfg, keep = device.make_config(alpha=0.45, gamma=0.5, policy=L.POLICY_SAPIRSHTEIN_2016_SM1,
                                   max_steps=2016, seed=0x5EED0000)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    _, rec = b.run(1 << 16, first_episode=0, records=True)
    idx = np.nonzero(rec["status"] & (L.ST_OVERLAP | L.ST_EXACT_RERUN))[0]
    for e in idx[:8]:
        ref = O.run_episodes(cfg, int(e), 1, threads=1)
        assert _records_equal(rec[e:e + 1], ref) == {}, int(e)


@pytest.mark.parametrize("policy", [0, 1, 2, 3])
@pytest.mark.parametrize("alpha", [0.1, 0.33, 0.45])
def test_loop_two_agents_bit_exact(ctx, alpha, policy):
    cfg, keep = device.make_config(alpha=alpha, gamma=0.0, network=L.NET_TWO_AGENTS,
                                   mode=L.MODE_LOOP, activations=10000, policy=policy, seed=5)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    _, rec = b.run(64, first_episode=0, records=True)
    for e in range(0, 64, 9):
        o = O.two_agents_task(alpha, policy, 10000, seed=5, episode=e)
        assert rec["reward_attacker"][e] == o["reward"][0]
        assert rec["reward_defender"][e] == o["reward"][1]
        assert rec["chain_time"][e] == o["head_time"]
        assert rec["head_height"][e] == o["head_height"]
        assert rec["n_activations"][e] == sum(o["activations"])


def test_lockstep_matches_oracle_step_by_step(ctx):
    n = 48
    cfg, keep = device.make_config(alpha=0.35, gamma=0.5, max_steps=150, seed=77,
                                   unit_observation=True, n_lanes=n)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    obs = b.reset()
    envs = [O.GymEnv(cfg, episode=i) for i in range(n)]
    ref_obs = np.array([e.reset() for e in envs])
    assert np.array_equal(obs, ref_obs)
    rng = np.random.default_rng(0)
    for t in range(150):
        acts = rng.integers(0, 4, size=n).astype(np.int32)
        obs, rew, done, info = b.step(acts)
        for i, e in enumerate(envs):
            o, r, d, inf = e.step(int(acts[i]))
            assert np.array_equal(obs[i], o), (t, i)
            assert rew[i] == r and done[i] == d
            for k in ["episode_reward_attacker", "episode_reward_defender", "episode_progress",
                      "episode_chain_time", "episode_sim_time", "episode_n_steps",
                      "episode_n_activations", "head_height", "head_miner"]:
                assert info[k][i] == inf[k], (t, i, k)
    assert done.all()


@pytest.mark.parametrize("policy", ["random", "sm1"])
def test_lockstep_overlaps_exact_on_event_engine(ctx, policy):
    # propagation delay 0.05: nearly every episode has an activation inside a delivery
    # window, where the closed form does not hold; such a lane moves to the exact event
    # engine (replaying its logged actions) and stays there, so every step of every lane
    # equals the oracle's engine.ml; a second episode per lane reuses the freed slots
    n, T = 64, 120
    cfg, keep = device.make_config(alpha=0.42, gamma=0.5, max_steps=T, seed=901,
                                   propagation_delay=0.05, unit_observation=False, n_lanes=n)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    rng = np.random.default_rng(5)
    moved = 0
    for rnd in range(2):
        ids = np.arange(n, dtype=np.uint64) + rnd * n
        obs = b.reset(episode_ids=ids)
        envs = [O.GymEnv(cfg, episode=int(i)) for i in ids]
        ref_obs = np.array([e.reset() for e in envs])
        assert np.array_equal(obs, ref_obs)
        for t in range(T):
            if policy == "random":
                acts = rng.integers(0, 4, size=n).astype(np.int32)
            else:
                acts = np.array([O.nak_policy(L.POLICY_SAPIRSHTEIN_2016_SM1, e.fields())
                                 for e in envs], dtype=np.int32)
            obs, rew, done, info = b.step(acts)
            st = info["status"]
            assert not ((st & L.ST_LOCKSTEP_INEXACT != 0) & (st & L.ST_EXACT_RERUN == 0)).any()
            for i, e in enumerate(envs):
                o, r, d, inf = e.step(int(acts[i]))
                assert np.array_equal(obs[i], o), (rnd, t, i, obs[i], o)
                assert rew[i] == r and done[i] == d, (rnd, t, i)
                for k in ["episode_reward_attacker", "episode_reward_defender",
                          "episode_progress", "episode_chain_time", "episode_sim_time",
                          "episode_n_steps", "episode_n_activations", "head_height",
                          "head_miner"]:
                    assert info[k][i] == inf[k], (rnd, t, i, k)
            assert np.array_equal(b.observe_fields(), np.array([e.fields() for e in envs]))
        assert done.all()
        moved += int(((st & L.ST_EXACT_RERUN) != 0).sum())
    assert moved >= n  # most lanes of both rounds took the exact path


def test_lockstep_partial_reset_keeps_exact_lanes(ctx):
    # a masked cpr_reset returns every lane's observation: the reset lanes' fresh ones and
    # the others' current ones, which for a lane on the exact event engine are that
    # engine's (kernels.hip k_reset); stepping on afterwards stays equal to the oracle
    n, T = 64, 120
    cfg, keep = device.make_config(alpha=0.42, gamma=0.5, max_steps=T, seed=903,
                                   propagation_delay=0.05, unit_observation=False, n_lanes=n)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    ids = np.arange(n, dtype=np.uint64)
    b.reset(episode_ids=ids)
    envs = [O.GymEnv(cfg, episode=int(i)) for i in ids]
    last = np.array([e.reset() for e in envs])

    def step_all(k):
        nonlocal last
        st = None
        for _ in range(k):
            acts = np.array([O.nak_policy(L.POLICY_SAPIRSHTEIN_2016_SM1, e.fields())
                             for e in envs], dtype=np.int32)
            obs, rew, done, info = b.step(acts)
            st = info["status"]
            ref = [e.step(int(acts[i])) for i, e in enumerate(envs)]
            last = np.array([r[0] for r in ref])
            assert np.array_equal(obs, last)
            assert np.array_equal(rew, np.array([r[1] for r in ref]))
        return st

    st = step_all(T // 2)
    exact = (st & L.ST_EXACT_RERUN) != 0
    mask = (np.arange(n) % 2 == 0).astype(np.uint8)
    assert (exact & (mask == 0)).sum() > 4  # unreset lanes on the exact engine exist
    new_ids = ids + 1000
    obs = b.reset(mask=mask, episode_ids=new_ids)
    for i in np.nonzero(mask)[0]:
        envs[i] = O.GymEnv(cfg, episode=int(new_ids[i]))
        last[i] = envs[i].reset()
    assert np.array_equal(obs, last)
    assert np.array_equal(b.observe_fields(), np.array([e.fields() for e in envs]))
    step_all(T // 4)


def test_policy_actions_decode(ctx):
    cfg, keep = device.make_config(alpha=0.3, gamma=0.5, n_lanes=1)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    fields = [[h, a, a - h, ev] for h in range(0, 7) for a in range(0, 9) for ev in (0, 1)]
    obs = np.array([O.obs_to_floats(f, True) for f in fields])
    for name, pid in device.policy_registry():
        got = b.policy_actions(pid, obs)
        want = [O.nak_policy(pid, f) for f in fields]
        assert got.tolist() == want, name


def test_invalid_configs_rejected(ctx):
    bad = [
        dict(alpha=1.5, gamma=0.5),  # engine.ml:42
        dict(alpha=0.3, gamma=0.9, defenders=2),  # network.ml:69-72
        dict(alpha=0.3, gamma=0.5, defenders=1),  # network.ml:63-64
        dict(alpha=float("nan"), gamma=0.5),
    ]
    for kw in bad:
        cfg, keep = device.make_config(max_steps=10, **kw)
        with pytest.raises(L.CprError) as e:
            device.Batch(cfg, ctx=ctx, keep=keep)
        assert e.value.code == L.CPR_E_INVALID_ARG


def test_summary_is_reduction_of_records(ctx):
    cfg, keep = device.make_config(alpha=0.4, gamma=0.5, max_steps=500, seed=1)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(20000, first_episode=0, records=True)
    h = rec["head_height"].astype(np.int64)
    ra = rec["reward_attacker"].astype(np.int64)
    assert s.episodes == 20000
    assert s.activations == int(rec["n_activations"].sum())
    assert s.reward_attacker_fx == int(ra.sum()) << 20
    assert s.progress_fx == int(h.sum()) << 20
    rel = np.where(h > 0, ra / np.maximum(h, 1), 0.0)
    assert s.rel_revenue_fx == int(np.rint(rel * 2**32).astype(np.uint64).sum())
    bins = np.clip((rel * 64).astype(np.int64), 0, 63)
    assert list(s.hist) == np.bincount(bins, minlength=64).tolist()


def test_full_size_properties(ctx):
    """BASELINE configs[1] size per point (2016 steps), checked by size-free properties."""
    cfg, keep = device.make_config(alpha=1 / 3, gamma=0.5, max_steps=2016, seed=0x5EED0000)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    n = 1 << 18
    s1 = b.run(n, first_episode=0)
    # shard invariance: two halves sum to the whole, bit for bit
    s2 = L.Summary()
    b.run(n // 2, first_episode=0, summary=s2)
    b.run(n // 2, first_episode=n // 2, summary=s2)
    assert s1.to_array().tolist() == s2.to_array().tolist()
    assert s1.activations == n * 2017 and s1.steps == n * 2016
    assert (s1.reward_attacker_fx + s1.reward_defender_fx) == s1.progress_fx
    assert s1.orphans == s1.activations - (s1.progress_fx >> 20)
    assert s1.status_other == 0
    # SM1 at alpha=1/3, gamma=0.5: Eyal-Sirer closed form 0.384615; 2016-step episodes
    # are within 2e-3 of the stationary value (finite-horizon start/end effects)
    m = s1.rel_revenue_fx / 2**32 / n
    assert abs(m - 0.384615) < 2e-3, m


def test_configs0_honest_episodes_match_oracle(ctx):
    # BASELINE configs[0]: cpr-nakamoto-v0 honest policy, alpha 0.33, gamma 0.5 (d = 2),
    # 2016-step episodes (2017 activations), every record field against the oracle
    cfg, keep = device.make_config(alpha=0.33, gamma=0.5, policy=L.POLICY_HONEST,
                                   max_steps=2016, seed=0x5EED0000)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(2048, records=True)
    ref = O.run_episodes(cfg, 0, 2048, threads=8)
    assert _records_equal(rec, ref) == {}
    assert (rec["n_activations"] == 2017).all() and s.episodes == 2048
    # honest play: the head chain is every block but the 1e-9-delay races' orphans, and
    # the attacker's share is alpha (normalised reward ~ 1)
    assert (rec["progress"] >= 2010).all()
    share = rec["reward_attacker"].sum() / rec["progress"].sum()
    assert abs(share - 0.33) < 0.005


def test_lockstep_65536_lanes_all_exact_at_long_delay(ctx):
    # engine.ml's step is exact for every env: with a 0.05 propagation delay nearly every
    # lane leaves the closed form, and every one of 65,536 lanes gets an exact-engine slot
    # (capi.hip ensure_lockstep sizes the pool to the lanes), so no step's outputs carry
    # inexact bits without CPR_ST_EXACT_RERUN; sampled lanes equal the oracle step by step
    n, T = 65536, 200
    cfg, keep = device.make_config(alpha=0.42, gamma=0.5, max_steps=T, seed=905,
                                   propagation_delay=0.05, unit_observation=False, n_lanes=n)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    obs = b.reset()
    sample = np.arange(0, n, n // 16)
    envs = {int(i): O.GymEnv(cfg, episode=int(i)) for i in sample}
    for i, e in envs.items():
        assert np.array_equal(obs[i], e.reset())
    moved = 0
    for t in range(T):
        acts = b.policy_actions(L.POLICY_SAPIRSHTEIN_2016_SM1, obs)
        obs, rew, done, info = b.step(acts)
        st = info["status"]
        inexact = (st & L.ST_LOCKSTEP_INEXACT) != 0
        assert not (inexact & ((st & L.ST_EXACT_RERUN) == 0)).any(), t
        moved = max(moved, int(((st & L.ST_EXACT_RERUN) != 0).sum()))
        for i, e in envs.items():
            o, r, d, _ = e.step(int(acts[i]))
            assert np.array_equal(obs[i], o) and rew[i] == r and done[i] == d, (t, i)
    assert moved > n // 2, moved  # most lanes ran on the exact engine


@pytest.mark.parametrize("cap", [0, 7])
def test_full_rerun_queue_flushes_not_capacity(ctx, cap, monkeypatch):
    # a flagged episode that finds the exact re-run queue full waits in its launch's
    # overflow flags and is re-run after the queue (kernels_eth.hip k_rerun_overflow): no
    # CPR_ST_CAPACITY, every record equal to the oracle's (a forced capacity of 0 / 7)
    monkeypatch.setenv("CPR_RERUN_QUEUE_CAP", str(cap))
    cfg, keep = device.make_config(alpha=0.45, gamma=0.5, policy=L.POLICY_SAPIRSHTEIN_2016_SM1,
                                   max_steps=400, seed=0x0E7, propagation_delay=0.05)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(512, first_episode=0, records=True)
    ref = O.run_episodes(cfg, 0, 512, threads=8)
    assert _records_equal(rec, ref) == {}
    assert not (rec["status"] & L.ST_CAPACITY).any()
    assert ((rec["status"] & L.ST_EXACT_RERUN) != 0).sum() > 100
    assert s.episodes == 512 and s.invalid == 0
    # the Ethereum window lane's re-runs take the same path
    cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=0.4, gamma=0.5,
                                   policy=L.ETH_POLICY_FN19, max_steps=400, seed=0x0E8,
                                   propagation_delay=0.05)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(256, first_episode=0, records=True)
    ref = O.run_episodes(cfg, 0, 256, threads=8)
    assert _records_equal(rec, ref) == {}
    assert not (rec["status"] & L.ST_CAPACITY).any() and s.invalid == 0
