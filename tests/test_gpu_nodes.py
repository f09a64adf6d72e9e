"""Per-node outputs on the device (cpr_node_outputs) — needs an MI355X.

The `activations` and `reward` columns of a csv_runner.ml:56-98 row (per-node activation
counts, the head's per-node reward array of simulator.ml:377-388) for every loop-task
network the device runs: honest cliques of all four protocols, the selfish-mining network
(Nakamoto, gamma in {0, 0.5, 0.9}) and two agents. Keyed episodes equal the oracle's
per-node vectors bit for bit; replayed traces of the reference's own data/honest_net.tsv
rows equal the row's `activations` and `reward` columns exactly.
"""

import json
import pathlib

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f not in ("status", "head_miner")]
GOLDEN = pathlib.Path(__file__).parent / "golden"


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def _clique(protocol, n, ad, acts, k=8, scheme=L.REWARD_DISCOUNT, sel=L.SELECT_HEURISTIC,
            seed=21):
    return device.make_config(alpha=0.0, gamma=0.0, defenders=n, network=L.NET_HONEST_CLIQUE,
                              mode=L.MODE_LOOP, protocol=protocol, reward_scheme=scheme, k=k,
                              subblock_selection=sel, activation_delay=ad, activations=acts,
                              seed=seed, policy=0)


CASES = {
    "nak-clique": lambda: _clique(L.PROTO_NAKAMOTO, 10, 30.0, 2000),
    "eth-clique": lambda: _clique(L.PROTO_ETHEREUM, 7, 2.0, 1500),
    "eth-clique-constant": lambda: _clique(L.PROTO_ETHEREUM, 5, 10.0, 1500,
                                           scheme=L.REWARD_CONSTANT),
    "bk-clique-constant": lambda: _clique(L.PROTO_BK, 6, 2.0, 1500, k=8, scheme=L.REWARD_CONSTANT),
    "bk-clique-block": lambda: _clique(L.PROTO_BK, 4, 10.0, 1500, k=4, scheme=L.REWARD_BLOCK),
    "ts-clique-discount": lambda: _clique(L.PROTO_TAILSTORM, 6, 2.0, 1200, k=8),
    "ts-clique-hybrid": lambda: _clique(L.PROTO_TAILSTORM, 3, 0.5, 1200, k=3,
                                        scheme=L.REWARD_HYBRID, sel=L.SELECT_ALTRUISTIC),
    "nak-sm-gamma0.5": lambda: device.make_config(alpha=0.35, gamma=0.5, mode=L.MODE_LOOP,
                                                  activations=3000, seed=5),
    "nak-sm-gamma0": lambda: device.make_config(alpha=0.35, gamma=0.0, mode=L.MODE_LOOP,
                                                activations=3000, seed=6,
                                                propagation_delay=1e-4),
    "nak-sm-gamma0.9": lambda: device.make_config(alpha=0.3, gamma=0.9, mode=L.MODE_LOOP,
                                                  activations=3000, seed=7,
                                                  propagation_delay=1e-4),
    "nak-two-agents": lambda: device.make_config(alpha=0.33, gamma=0.0,
                                                 network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP,
                                                 activations=3000, seed=8),
    "eth-two-agents": lambda: device.make_config(alpha=0.3, network=L.NET_TWO_AGENTS,
                                                 mode=L.MODE_LOOP, activations=3000, seed=9,
                                                 protocol=L.PROTO_ETHEREUM,
                                                 policy=L.ETH_POLICY_FN19,
                                                 reward_scheme=L.REWARD_DISCOUNT),
    "bk-two-agents": lambda: device.make_config(alpha=0.3, network=L.NET_TWO_AGENTS,
                                                mode=L.MODE_LOOP, activations=3000, seed=10,
                                                protocol=L.PROTO_BK, k=4,
                                                policy=L.BK_POLICY_AVOID_LOSS),
    "ts-two-agents": lambda: device.make_config(alpha=0.33, network=L.NET_TWO_AGENTS,
                                                mode=L.MODE_LOOP, activations=2000, seed=12,
                                                protocol=L.PROTO_TAILSTORM, k=8,
                                                policy=L.TS_POLICY_AVOID_LOSS,
                                                reward_scheme=L.REWARD_DISCOUNT),
}


@pytest.mark.parametrize("case", list(CASES))
def test_node_outputs_match_oracle(ctx, case):
    cfg, keep = CASES[case]()
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    n = 48
    rec, acts, rews = b.node_outputs(n, 100)
    orec, oacts, orews, ohm = O.node_outputs(cfg, b.n_nodes, first=100, n=n)
    ok = (rec["status"] & L.ST_INVALID) == 0
    assert ok.mean() > 0.9, case
    assert np.array_equal(acts[ok], oacts[ok]), case
    bad = np.nonzero((rews != orews).any(axis=1) & ok)[0]
    assert len(bad) == 0, (case, int(bad[0]), rews[bad[0]].tolist(), orews[bad[0]].tolist())
    known = ok & (ohm != -2)
    assert np.array_equal(rec["head_miner"][known], ohm[known]), case
    # records equal cpr_run_episodes' records (and the oracle's) except head_miner
    _, run = b.run(n, 100, records=True)
    for f in FIELDS:
        assert np.array_equal(rec[f][ok], run[f][ok]), (case, f)
        assert np.array_equal(rec[f][ok], orec[f][ok]), (case, f)
    # the rows decompose the records
    assert np.array_equal(acts.sum(axis=1)[ok], rec["n_activations"][ok])
    assert np.array_equal(rews[ok, 0], rec["reward_attacker"][ok])


def test_node_outputs_arguments(ctx):
    cfg, keep = CASES["nak-clique"]()
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    with pytest.raises(L.CprError, match="n_nodes"):
        nn = b.n_nodes
        rec = np.zeros(4, dtype=L.RECORD_DTYPE)
        a = np.zeros((4, nn + 1), np.int64)
        r = np.zeros((4, nn + 1))
        L.check(L.lib().cpr_node_outputs(b.handle, 4, 0, None, nn + 1, L.ptr(rec), L.ptr(a),
                                         L.ptr(r)))
    fc, fkeep = device.make_config(alpha=0.3, gamma=0.5, protocol=L.PROTO_FC16, max_steps=100,
                                     policy=L.FC16_POLICY_HONEST)
    fb = device.Batch(fc, ctx=ctx, keep=fkeep)
    with pytest.raises(L.CprError, match="FC16"):
        fb.node_outputs(4)


def test_gym_mode_rows_decompose_records(ctx):
    # gym episodes (cpr-nakamoto-v0, SM1) on the exact engine: the rows add up to the record
    cfg, keep = device.make_config(alpha=0.33, gamma=0.5, max_steps=500, seed=3)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    rec, acts, rews = b.node_outputs(256)
    _, run = b.run(256, records=True)
    for f in FIELDS:
        assert np.array_equal(rec[f], run[f]), f
    assert np.array_equal(acts.sum(axis=1), rec["n_activations"])
    assert np.array_equal(rews[:, 0], rec["reward_attacker"])
    assert np.array_equal(rews[:, 1:].sum(axis=1), rec["reward_defender"])


ROWS = json.loads((GOLDEN / "honest_net_clique.json").read_text())["rows"]


@pytest.mark.parametrize("row", ROWS, ids=[f"line{r['line']}" for r in ROWS])
def test_honest_net_rows_per_node(ctx, row):
    # data/honest_net.tsv rows: the reference's own `activations` and `reward` columns,
    # reproduced per node by replaying the OCaml Random draws the oracle records for them
    scheme = L.REWARD_DISCOUNT if row["incentive_scheme"] == "discount" else L.REWARD_CONSTANT
    proto = L.PROTO_ETHEREUM if row["protocol"] == "ethereum" else L.PROTO_NAKAMOTO
    cfg, keep = _clique(proto, row["nodes"], row["activation_delay"], row["activations"],
                        scheme=scheme, seed=11)
    trace, _ = O.export_traces(cfg, 0, 1, rng=O.OcamlRandom())
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    rec, acts, rews = b.node_outputs(trace=trace)
    assert not (rec["status"] & L.ST_TRACE_MISS).any()
    assert acts[0].tolist() == row["activations_per_node"]
    assert rews[0].tolist() == row["reward"]
    assert rec["head_height"][0] == row["head_height"]


CHAIN_ROWS = json.loads((GOLDEN / "honest_net_chains.json").read_text())["rows"]

# per-node outputs of a chained row's replayed trace, shared by the two tests below when they
# build byte-identical configurations (a Tailstorm row is one latency-bound lane, ~7 s)
_NODE_OUT = {}


def _chained_node_outputs(ctx, cfg, keep, row):
    from test_oracle_clique import chained_rng

    key = (row["line"], bytes(cfg))
    if key not in _NODE_OUT:
        trace, _ = O.export_traces(cfg, 0, 1, rng=chained_rng(row))
        b = device.Batch(cfg, ctx=ctx, keep=keep)
        _NODE_OUT[key] = b.node_outputs(trace=trace)
    return _NODE_OUT[key]


@pytest.mark.parametrize("row", CHAIN_ROWS, ids=lambda r: f"line{r['line']}-{r['protocol']}")
def test_chained_honest_net_rows_per_node(ctx, row):
    from test_oracle_clique import chained_rng

    proto = {"nakamoto": L.PROTO_NAKAMOTO, "ethereum": L.PROTO_ETHEREUM, "bk": L.PROTO_BK,
             "tailstorm": L.PROTO_TAILSTORM}[row["protocol"]]
    scheme = {None: L.REWARD_CONSTANT, "constant": L.REWARD_CONSTANT,
              "block": L.REWARD_BLOCK, "discount": L.REWARD_DISCOUNT}[row["incentive_scheme"]]
    sel = {None: 0, "altruistic": 0, "heuristic": 1, "optimal": 2}[row.get("subblock_selection")]
    cfg, keep = _clique(proto, row["nodes"], row["activation_delay"], row["activations"],
                        k=row.get("k") or 8, scheme=scheme, sel=sel, seed=11)
    rec, acts, rews = _chained_node_outputs(ctx, cfg, keep, row)
    assert not (rec["status"] & L.ST_TRACE_MISS).any()
    assert acts[0].tolist() == row["activations_per_node"]
    assert rews[0].tolist() == row["reward"]


# ---------------------------------------------------------------- TSV rows (csv_runner)

TSV_LINES = sorted(int(k) for k in json.loads((GOLDEN / "honest_net_tsv_lines.json")
                                               .read_text())["rows"])


@pytest.mark.parametrize("line", TSV_LINES)
def test_device_rows_reproduce_reference_text(ctx, line):
    # data/honest_net.tsv text, every column but version / machine_duration_s, from the
    # device's per-node outputs of the row's replayed OCaml Random draws
    from test_csv_runner import CHAINS, SKIP, TSV, _fields, _task
    from test_oracle_clique import chained_rng

    from cpr_amd import csv_runner as C

    row = CHAINS[line]
    task = _task(row)
    cfg, keep = C.config_of(task, seed=11)
    rec, acts, rews = _chained_node_outputs(ctx, cfg, keep, row)
    got = _fields(C.result_row(task, rec[0], acts[0], rews[0], 0.0), TSV["header"])
    for col, g, r in zip(TSV["header"], got, TSV["rows"][str(line)]):
        if col not in SKIP:
            assert g == r, (line, col, g, r)


def test_csv_runner_end_to_end(ctx, tmp_path):
    from cpr_amd import csv_runner as C

    tasks = C.honest_net_tasks(2000)[::13] + C.withholding_tasks(2000)[::61]
    rows = C.run(tasks, ctx=ctx, seed=3)
    out = tmp_path / "rows.tsv"
    C.save_rows_as_tsv(out, rows)
    lines = out.read_text().rstrip("\n").split("\n")
    header = lines[0].split("\t")
    assert len(lines) == len(tasks) + 1
    errors = 0
    for t, ln in zip(tasks, lines[1:]):
        d = dict(zip(header, ln.split("\t")))
        assert d["network"] == t.network.key and d["number_activations"] == "2000"
        if d.get("error"):
            errors += 1
            continue
        acts = [int(x) for x in d["activations"].split("|")]
        rews = [float(x) for x in d["reward"].split("|")]
        assert len(acts) == len(rews) == len(t.network.compute)
        assert sum(acts) == 2000
        assert float(d["head_progress"]) > 0 and float(d["head_time"]) > 0
    assert errors <= len(tasks) // 20, errors
    print(f"{len(tasks)} tasks, {errors} error rows")
