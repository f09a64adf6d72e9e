"""Boundary behaviour of libcpr_hip on the device — needs an MI355X.

Status surfacing (ABI v6): a lockstep lane whose episode reaches a point where the
reference raises reports CPR_ST_REFERENCE_RAISES in cpr_step_info.status at the same step
the oracle raises, and the Python engine.step raises there; invalid episodes stay out of
summaries. Resource hygiene: policy queries do not leak device memory. Trace validation:
a clique trace naming a node outside the clique is rejected before it reaches a lane.
"""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device, engine, protocols

pytestmark = pytest.mark.gpu

# Tailstorm k = 1, optimal sub-block selection, avoid-loss: the reference raises
# (List.for_all2 in summary dedup / assert in tailstorm.ml) in these episodes of seed
# 0x7A110000 (found with the oracle, which records CPR_ST_REFERENCE_RAISES for them)
TS_RAISE = dict(protocol=L.PROTO_TAILSTORM, alpha=0.4, gamma=0.5, policy=L.TS_POLICY_AVOID_LOSS,
                reward_scheme=L.REWARD_DISCOUNT, subblock_selection=L.SELECT_OPTIMAL, k=1,
                max_steps=300, seed=0x7A110000)
RAISING = [55, 97, 122]


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def test_fused_flags_match_oracle_and_stay_out_of_summary(ctx):
    cfg, keep = device.make_config(**TS_RAISE)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(256, records=True)
    ref = O.run_episodes(cfg, 0, 256, threads=8)
    flagged = np.nonzero(rec["status"] & L.ST_REFERENCE_RAISES)[0]
    assert set(RAISING) <= set(flagged.tolist())
    assert np.array_equal(rec["status"] & (L.ST_REFERENCE_RAISES | L.ST_CAPACITY),
                          ref["status"] & (L.ST_REFERENCE_RAISES | L.ST_CAPACITY))
    ok = (rec["status"] & L.ST_INVALID) == 0
    assert s.invalid == len(flagged) and s.episodes == int(ok.sum())
    ra = rec["reward_attacker"][ok].sum()
    assert s.reward_attacker_fx == int(round(ra * 2**20))


def test_step_status_and_engine_raise_at_the_oracle_step(ctx):
    ep = RAISING[0]
    cfg, keep = device.make_config(n_lanes=1, **TS_RAISE)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    b.reset(episode_ids=np.array([ep], dtype=np.uint64))
    oracle_env = O.TsGymEnv(cfg, episode=ep)
    oracle_env.reset()
    raised_at = None
    for t in range(400):
        a = O.ts_policy("avoid-loss", oracle_env.fields(), 1)
        try:
            oracle_env.step(a)
        except RuntimeError:
            raised_at = t
        _, _, done, info = b.step(np.array([a], dtype=np.int32))
        if raised_at is not None:
            assert info["status"][0] & L.ST_REFERENCE_RAISES and done[0]
            break
        assert info["status"][0] & L.ST_INVALID == 0, t
    assert raised_at is not None
    # the drop-in engine raises at the same step
    env = engine.create(proto=protocols.tailstorm(reward="discount", k=1,
                                                  subblock_selection="optimal",
                                                  unit_observation=False),
                        alpha=0.4, gamma=0.5, defenders=2, activation_delay=1.0,
                        max_steps=300, seed=0x7A110000)
    env.episode = ep
    obs = engine.reset(env)
    pol = engine.policies(env)["avoid-loss"]
    with pytest.raises(RuntimeError, match="reference simulator raises"):
        for _ in range(raised_at + 1):
            obs, _, _, _ = engine.step(env, pol(obs))


def _hip_free_bytes():
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    free, total = ctypes.c_size_t(), ctypes.c_size_t()
    assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
    return free.value


@pytest.mark.parametrize("protocol,kw", [
    (L.PROTO_NAKAMOTO, {}),
    (L.PROTO_ETHEREUM, {}),
    (L.PROTO_BK, dict(k=8)),
    (L.PROTO_TAILSTORM, dict(k=8)),
])
def test_policy_queries_do_not_leak(ctx, protocol, kw):
    cfg, keep = device.make_config(protocol=protocol, alpha=0.3, gamma=0.5, max_steps=50,
                                   seed=1, n_lanes=4, policy=0, **kw)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    obs = b.reset()
    b.policy_actions(0, obs)
    free0 = _hip_free_bytes()
    for _ in range(20000):
        b.policy_actions(0, obs)
    free1 = _hip_free_bytes()
    assert free0 - free1 < 64 << 20, (free0, free1)


def test_clique_trace_rejects_node_outside_the_clique(ctx):
    n = 4
    cfg, keep = device.make_config(alpha=0.0, gamma=0.0, defenders=n, network=L.NET_HONEST_CLIQUE,
                                   mode=L.MODE_LOOP, activations=200, seed=3, policy=0)
    trace, _ = O.export_traces(cfg, 0, 2)
    trace.act_miner[5] = n  # a clique of n nodes has ids 0 .. n - 1
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    with pytest.raises(L.CprError) as e:
        b.replay(trace)
    assert e.value.code == L.CPR_E_INVALID_ARG and "act_miner" in str(e.value)
