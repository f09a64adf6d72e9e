"""cpr_replay on the device against the CPU oracle — needs an MI355X.

The north star's first correctness tier: per-episode outcomes match bit for bit when both
engines replay the same exported activation/delay trace. Traces come from the oracle,
either on the keyed stream (then the device's replay must also equal its own keyed run of
the same episode ids) or on the OCaml 4.12 `Random` replica — the reference's own stream —
including the 28 two-agents Nakamoto rows of data/withholding.tsv, which the device then
reproduces from their traces.
"""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device
from test_trace import CONFIGS, EXP_CONFIGS, check_withholding_record, withholding_traces

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f != "status"]
BAD = L.ST_CAPACITY | L.ST_REFERENCE_RAISES | L.ST_TRACE_MISS


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def _same(a, b, fields=FIELDS):
    for f in fields:
        bad = np.nonzero(a[f] != b[f])[0]
        assert len(bad) == 0, (f, int(bad[0]), a[f][bad[0]], b[f][bad[0]])


@pytest.mark.parametrize("name,kw", CONFIGS + EXP_CONFIGS,
                         ids=[c[0] for c in CONFIGS + EXP_CONFIGS])
def test_replay_keyed_trace_matches_oracle_and_keyed_run(ctx, name, kw):
    cfg, keep = device.make_config(**kw)
    n = 96
    trace, ref = O.export_traces(cfg, 500, n)
    b = device.Batch(cfg, keep=keep)
    _, rec = b.replay(trace)
    assert not (rec["status"] & BAD).any()
    _same(rec, ref)
    # the same draws from the keyed stream directly: identical records, status included
    _, keyed = b.run(n, first_episode=500, records=True)
    _same(rec, keyed, FIELDS + ["status"])


@pytest.mark.parametrize("name,kw", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_replay_ocaml_stream_trace_matches_oracle(ctx, name, kw):
    cfg, keep = device.make_config(**kw)
    trace, ref = O.export_traces(cfg, 0, 48, rng=O.OcamlRandom(2024))
    _, rec = device.Batch(cfg, keep=keep).replay(trace)
    assert not (rec["status"] & BAD).any()
    _same(rec, ref)


def test_replay_full_size_sm1_episodes(ctx):
    # cpr-nakamoto-v0 episodes of BASELINE configs[1] size (2016 steps), OCaml stream
    for alpha, gamma in [(0.33, 0.5), (0.45, 0.0), (0.25, 0.75)]:
        cfg, _ = device.make_config(alpha=alpha, gamma=gamma, max_steps=2016)
        trace, ref = O.export_traces(cfg, 0, 128, rng=O.OcamlRandom(int(alpha * 1000)))
        _, rec = device.Batch(cfg).replay(trace)
        assert not (rec["status"] & BAD).any()
        _same(rec, ref)


def test_replay_reproduces_withholding_rows(ctx):
    for row, cfg, trace, _ in withholding_traces():
        _, rec = device.Batch(cfg).replay(trace)
        assert rec["status"][0] & BAD == 0
        check_withholding_record(row, rec)


def test_replay_batches_many_episodes_and_summary(ctx):
    cfg, _ = device.make_config(alpha=0.35, gamma=0.5, max_steps=256, seed=99)
    trace, ref = O.export_traces(cfg, 0, 1500)
    s, rec = device.Batch(cfg).replay(trace)
    _same(rec, ref)
    assert s.episodes == 1500 and s.activations == int(ref["n_activations"].sum())
    # single-episode slices replay to the same records
    for e in (0, 777, 1499):
        _, one = device.Batch(cfg).replay(trace.episode(e))
        _same(one, rec[e:e + 1])


def test_replay_flags_truncated_trace(ctx):
    cfg, _ = device.make_config(alpha=0.35, gamma=0.5, max_steps=100, seed=3)
    trace, _ = O.export_traces(cfg, 0, 2)
    n0 = int(trace.act_offset[1])
    # episode 0 loses half its activations, episode 1 loses its link delays
    a = np.r_[trace.act_miner[: n0 // 2], trace.act_miner[n0:]]
    d = np.r_[trace.act_delay[: n0 // 2], trace.act_delay[n0:]]
    short = L.Trace(act_offset=[0, n0 // 2, n0 // 2 + (len(trace.act_miner) - n0)],
                    act_miner=a, act_delay=d, pow_offset=[0, 0, 0], pow_hash=[],
                    link_offset=[0, trace.link_offset[1], trace.link_offset[1]],
                    link_key=trace.link_key[: trace.link_offset[1]],
                    link_delay=trace.link_delay[: trace.link_offset[1]])
    _, rec = device.Batch(cfg).replay(short)
    assert rec["status"][0] & L.ST_TRACE_MISS
    if trace.link_offset[2] > trace.link_offset[1]:
        assert rec["status"][1] & L.ST_TRACE_MISS


def test_replay_rejects_invalid_traces(ctx):
    cfg, _ = device.make_config(alpha=0.35, gamma=0.5, max_steps=100, seed=3)
    trace, _ = O.export_traces(cfg, 0, 1)
    b = device.Batch(cfg)

    def with_(**over):
        arrays = {n: getattr(trace, n) for n, _ in L.Trace.ARRAYS}
        arrays.update(over)
        return L.Trace(**arrays)

    bad_miner = trace.act_miner.copy()
    bad_miner[3] = cfg.defenders + 1
    bad_delay = trace.act_delay.copy()
    bad_delay[2] = np.nan
    cases = [with_(act_miner=bad_miner), with_(act_delay=bad_delay),
             with_(act_offset=[1, len(trace.act_miner)])]
    if len(trace.link_key) >= 2:
        cases.append(with_(link_key=trace.link_key[::-1].copy()))
    for t in cases:
        with pytest.raises(L.CprError) as e:
            b.replay(t)
        assert e.value.code == L.CPR_E_INVALID_ARG
