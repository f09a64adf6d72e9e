"""Activation/delay traces (cpr_trace) on the CPU oracle.

The oracle logs every draw an episode consumes by keyed coordinate (activation j's miner
and clock delay, vertex pow bits, message delays); replaying that trace through the oracle
must reproduce every record field bit for bit, whether the draws came from the keyed
Philox stream or from the OCaml 4.12 `Random` replica (the reference's own stream). The
28 two-agents Nakamoto rows the reference recorded in data/withholding.tsv are reproduced
from their OCaml-stream traces. The device replays the same traces in test_gpu_replay.py.
"""

import json
import pathlib

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device

FIELDS = list(L.RECORD_DTYPE.names)
GOLDEN = pathlib.Path(__file__).parent / "golden"

# (name, make_config kwargs); small episodes so the whole module runs in seconds
CONFIGS = [
    ("nak-sm1-g05", dict(alpha=0.35, gamma=0.5, max_steps=300, seed=11)),
    ("nak-sm1-g09-d10", dict(alpha=0.4, gamma=0.9, max_steps=300, seed=12)),
    ("nak-es-g0", dict(alpha=0.3, gamma=0.0, policy=L.POLICY_EYAL_SIRER_2014, max_steps=300,
                       seed=13)),
    ("nak-loop", dict(alpha=0.33, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP, activations=500,
                      policy=L.POLICY_SAPIRSHTEIN_2016_SM1, seed=14)),
    ("eth-fn19", dict(protocol=L.PROTO_ETHEREUM, alpha=0.35, gamma=0.5, max_steps=200,
                      policy=L.ETH_POLICY_FN19, reward_scheme=L.REWARD_DISCOUNT, seed=15)),
    ("eth-release-g09", dict(protocol=L.PROTO_ETHEREUM, alpha=0.4, gamma=0.9, max_steps=150,
                             policy=L.ETH_POLICY_SELFISH_RELEASE, seed=16)),
    ("bk-avoid-loss", dict(protocol=L.PROTO_BK, k=8, alpha=0.33, gamma=0.5, max_steps=200,
                           policy=L.BK_POLICY_AVOID_LOSS, seed=17)),
    ("bk-loop", dict(protocol=L.PROTO_BK, k=4, alpha=0.4, network=L.NET_TWO_AGENTS,
                     mode=L.MODE_LOOP, activations=300, policy=L.BK_POLICY_GET_AHEAD, seed=18)),
    ("ts-avoid-loss", dict(protocol=L.PROTO_TAILSTORM, k=8, alpha=0.33, gamma=0.5,
                           max_steps=200, policy=L.TS_POLICY_AVOID_LOSS,
                           reward_scheme=L.REWARD_DISCOUNT, seed=19)),
    ("ts-loop", dict(protocol=L.PROTO_TAILSTORM, k=8, alpha=0.33, network=L.NET_TWO_AGENTS,
                     mode=L.MODE_LOOP, activations=300, policy=L.TS_POLICY_GET_AHEAD,
                     reward_scheme=L.REWARD_DISCOUNT, seed=20)),
]


# the reference's policy-test network (exponential-delay clique, attacker on node 0),
# keyed traces only (their oracle tasks draw from the keyed stream)
EXP_CONFIGS = [
    ("exp-nak-sm1", dict(protocol=L.PROTO_NAKAMOTO, alpha=0.0, gamma=0.0,
                         network=L.NET_EXP_CLIQUE, mode=L.MODE_LOOP, defenders=2,
                         activation_delay=2.0, propagation_delay=1.0, activations=300,
                         policy=L.POLICY_SAPIRSHTEIN_2016_SM1, seed=21)),
    ("exp-eth-fn19", dict(protocol=L.PROTO_ETHEREUM, alpha=0.0, gamma=0.0,
                          network=L.NET_EXP_CLIQUE, mode=L.MODE_LOOP, defenders=2,
                          activation_delay=2.0, propagation_delay=1.0, activations=300,
                          policy=L.ETH_POLICY_FN19, seed=22)),
    ("exp-bk", dict(protocol=L.PROTO_BK, k=4, alpha=0.0, gamma=0.0, network=L.NET_EXP_CLIQUE,
                    mode=L.MODE_LOOP, defenders=1, activation_delay=5.0,
                    propagation_delay=1.0, activations=300, policy=L.BK_POLICY_GET_AHEAD,
                    seed=23)),
    ("exp-ts", dict(protocol=L.PROTO_TAILSTORM, k=8, alpha=0.0, gamma=0.0,
                    network=L.NET_EXP_CLIQUE, mode=L.MODE_LOOP, defenders=1,
                    activation_delay=10.0, propagation_delay=1.0, activations=300,
                    policy=L.TS_POLICY_GET_AHEAD, reward_scheme=L.REWARD_DISCOUNT, seed=24)),
]


def _assert_same(a, b):
    for f in FIELDS:
        bad = np.nonzero(a[f] != b[f])[0]
        assert len(bad) == 0, (f, int(bad[0]), a[f][bad[0]], b[f][bad[0]])


@pytest.mark.parametrize("name,kw", CONFIGS + EXP_CONFIGS,
                         ids=[c[0] for c in CONFIGS + EXP_CONFIGS])
def test_keyed_trace_replays_exactly(name, kw):
    cfg, _ = device.make_config(**kw)
    trace, rec = O.export_traces(cfg, 100, 12)
    # recording changes nothing: the records equal an unrecorded oracle run
    _assert_same(rec, O.run_episodes(cfg, 100, 12))
    rep = O.replay(cfg, trace)
    assert not (rep["status"] & L.ST_TRACE_MISS).any()
    _assert_same(rep, rec)


@pytest.mark.parametrize("name,kw", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_ocaml_stream_trace_replays_exactly(name, kw):
    cfg, _ = device.make_config(**kw)
    trace, rec = O.export_traces(cfg, 0, 8, rng=O.OcamlRandom(7))
    rep = O.replay(cfg, trace)
    assert not (rep["status"] & L.ST_TRACE_MISS).any()
    _assert_same(rep, rec)


def test_trace_layout():
    cfg, _ = device.make_config(alpha=0.35, gamma=0.5, max_steps=100, seed=3)
    trace, rec = O.export_traces(cfg, 0, 5)
    assert trace.n_episodes == 5
    for arr in ("act_offset", "pow_offset", "link_offset"):
        off = getattr(trace, arr)
        assert off[0] == 0 and (np.diff(off) >= 0).all()
    # one clock per activation plus the clock scheduled after the last one
    assert (np.diff(trace.act_offset) == rec["n_activations"] + 1).all()
    for e in range(5):
        k = trace.link_key[trace.link_offset[e]:trace.link_offset[e + 1]]
        assert (np.diff(k.astype(np.float64)) > 0).all() or len(k) < 2
    assert ((trace.act_miner >= 0) & (trace.act_miner <= cfg.defenders)).all()
    assert (trace.act_delay > 0).all()


def test_truncated_trace_is_flagged():
    cfg, _ = device.make_config(alpha=0.35, gamma=0.5, max_steps=100, seed=3)
    trace, _ = O.export_traces(cfg, 0, 1)
    n = int(trace.act_offset[1])
    short = L.Trace(act_offset=[0, n // 2], act_miner=trace.act_miner[: n // 2],
                    act_delay=trace.act_delay[: n // 2], pow_offset=trace.pow_offset,
                    pow_hash=trace.pow_hash, link_offset=trace.link_offset,
                    link_key=trace.link_key, link_delay=trace.link_delay)
    rep = O.replay(cfg, short)
    assert rep["status"][0] & L.ST_TRACE_MISS


def test_trace_save_load_round_trip(tmp_path):
    cfg, _ = device.make_config(protocol=L.PROTO_BK, k=4, alpha=0.3, gamma=0.5, max_steps=50,
                                policy=L.BK_POLICY_GET_AHEAD, seed=5)
    trace, rec = O.export_traces(cfg, 0, 3)
    assert len(trace.pow_hash) > 0 and len(trace.link_key) > 0
    trace.save(tmp_path / "t.npz")
    back = L.Trace.load(tmp_path / "t.npz")
    for name, _ in L.Trace.ARRAYS:
        assert np.array_equal(getattr(back, name), getattr(trace, name))
    _assert_same(O.replay(cfg, back.episode(1)), rec[1:2])


def _withholding_rows():
    return json.loads((GOLDEN / "withholding_nakamoto_two_agents.json").read_text())["rows"]


def withholding_traces():
    """OCaml-stream traces of the 28 two-agents Nakamoto rows of data/withholding.tsv:
    [(row, config, trace, oracle record)], the RNG state carried as in test_oracle_kat."""
    out = []
    for row in _withholding_rows():
        rng = O.OcamlRandom()
        for _ in range(row["prior_tasks"]):
            O.two_agents_task(0.25, "honest", row["activations"], rng=rng)
        cfg, _ = device.make_config(alpha=row["alpha"], network=L.NET_TWO_AGENTS,
                                    mode=L.MODE_LOOP, activations=row["activations"],
                                    policy=O.POLICIES[row["policy"]])
        trace, rec = O.export_traces(cfg, 0, 1, rng=rng)
        out.append((row, cfg, trace, rec))
    return out


def check_withholding_record(row, rec):
    assert [int(x) for x in [rec["n_activations"][0]]] == [sum(row["activations_per_node"])]
    assert [float(rec["reward_attacker"][0]), float(rec["reward_defender"][0])] == row["reward"]
    assert "%.12g" % rec["chain_time"][0] == row["head_time"]
    assert float(rec["progress"][0]) == row["head_progress"]


def test_withholding_rows_from_ocaml_traces():
    for row, cfg, trace, rec in withholding_traces():
        check_withholding_record(row, rec)
        check_withholding_record(row, O.replay(cfg, trace))


def test_ocaml_recorder_format_round_trips(tmp_path):
    # integration/ocaml/trace_hooks.ml `write` (uncompiled here: no OCaml) emits the binary
    # layout Trace.load reads. Its array order and element widths are checked against the
    # reader statically; Trace.save_binary mirrors the writer byte for byte, and traces of
    # the OCaml Random stream (the reference's own draws) and of the keyed stream survive
    # the round trip and replay to the same records
    ml = (pathlib.Path(__file__).parents[1] / "integration" / "ocaml" / "trace_hooks.ml").read_text()
    writes = __import__("re").findall(r"^  arr (i64|u32|f64) ", ml, flags=__import__("re").M)
    width = {"i64": 8, "u32": 4, "f64": 8}
    assert [width[w] for w in writes] == [np.dtype(L.Trace._WIRE[n]).itemsize
                                         for n, _ in L.Trace.ARRAYS]
    assert [w == "f64" for w in writes] == [np.dtype(L.Trace._WIRE[n]).kind == "f"
                                           for n, _ in L.Trace.ARRAYS]
    assert 'Buffer.add_string buf "CPRTRACE"' in ml
    cases = [
        (dict(alpha=0.33, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP, activations=400,
              policy=L.POLICY_SAPIRSHTEIN_2016_SM1), O.OcamlRandom()),
        (dict(alpha=0.35, gamma=0.5, max_steps=200, seed=3), None),
        (dict(protocol=L.PROTO_BK, k=4, alpha=0.3, gamma=0.5, max_steps=60,
              policy=L.BK_POLICY_GET_AHEAD, seed=5), None),
    ]
    for i, (kw, rng) in enumerate(cases):
        cfg, _ = device.make_config(**kw)
        trace, rec = O.export_traces(cfg, 0, 3 if rng is None else 1, rng=rng)
        path = tmp_path / f"t{i}.cprtrace"
        trace.save_binary(path)
        assert open(path, "rb").read(8) == b"CPRTRACE"
        back = L.Trace.load(path)
        for name, _ in L.Trace.ARRAYS:
            assert np.array_equal(getattr(back, name), getattr(trace, name)), name
        _assert_same(O.replay(cfg, back), rec)
    # a truncated file is rejected
    raw = open(tmp_path / "t0.cprtrace", "rb").read()
    (tmp_path / "bad.cprtrace").write_bytes(raw[:-8])
    with pytest.raises(ValueError):
        L.Trace.load(tmp_path / "bad.cprtrace")
