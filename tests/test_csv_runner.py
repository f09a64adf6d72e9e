"""The TSV writer of cpr_amd.csv_runner against the reference's own output (CPU).

Info.pp_rows / string_of_float semantics (simulator/lib/info.ml:24-70), and the rows of
data/honest_net.tsv the honest_net fixtures pin: each task's per-node outputs (from the
oracle, driven by the OCaml Random draws recovered for the row) formatted by
csv_runner.result_row must reproduce the reference's text field for field — every column
except `version` and the wall-clock `machine_duration_s` — and pp_rows over the rows must
reproduce the reference's header. Fixture: tests/golden/honest_net_tsv_lines.json
(make_honest_net_tsv_fixture.py).
"""

import json
import pathlib

import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import csv_runner as C

GOLDEN = pathlib.Path(__file__).parent / "golden"
TSV = json.loads((GOLDEN / "honest_net_tsv_lines.json").read_text())
CHAINS = {r["line"]: r for r in json.loads((GOLDEN / "honest_net_chains.json").read_text())["rows"]}
SKIP = {"version", "machine_duration_s"}


def test_string_of_float():
    cases = {1.0: "1.", 600.0: "600.", 0.25: "0.25", 1 - 0.33: "0.67", 1e6: "1000000.",
             1e-4: "0.0001", 5972265.794553: "5972265.79455", -2.0: "-2.",
             0.5 / 11: "0.0454545454545", 1e20: "1e+20", float("inf"): "inf",
             float("-inf"): "-inf", float("nan"): "nan", 0.0: "0."}
    for x, s in cases.items():
        assert C.string_of_float(x) == s, x


def test_pp_rows_expect():
    # info.ml:60-70 expect test; the formatter writes every field, so a row missing the
    # last key ends in a separator (the expect block trims trailing whitespace)
    rows = [[("a", 1), ("b", 2.0)], [("a", 7), ("b", 42.0)], [("a", 1), ("c", 5.0)]]
    assert C.pp_rows(rows) == "a\tb\tc\n1\t2.\t\n7\t42.\t\n1\t\t5.\n"
    assert C.pp_rows([[("x", True), ("x", "last")]]) == "x\nlast\n"


def _task(row):
    p = {"nakamoto": lambda: C.nakamoto(),
         "ethereum": lambda: C.ethereum(row["incentive_scheme"]),
         "bk": lambda: C.bk(row["k"], row["incentive_scheme"]),
         "tailstorm": lambda: C.tailstorm(row["k"], row["incentive_scheme"],
                                          row["subblock_selection"])}[row["protocol"]]()
    return C.Task(row["activations"], C.honest_clique(row["nodes"], row["activation_delay"]), p)


def _oracle_row(line):
    from test_oracle_clique import chained_rng

    row = CHAINS[line]
    task = _task(row)
    cfg, _keep = C.config_of(task, seed=11)
    trace, _ = O.export_traces(cfg, 0, 1, rng=chained_rng(row))
    rec, acts, rews, hm = O.node_outputs(cfg, row["nodes"], trace=trace)
    if hm[0] != -2:
        rec["head_miner"][0] = hm[0]
    return task, rec[0], acts[0], rews[0]


def _fields(row_pairs, header):
    d = {k: C.string_of_value(v) for k, v in row_pairs}
    return [d.get(k, "") for k in header]


@pytest.mark.parametrize("line", sorted(int(k) for k in TSV["rows"]))
def test_rows_reproduce_reference_text(line):
    task, rec, acts, rews = _oracle_row(line)
    ref = TSV["rows"][str(line)]
    got = _fields(C.result_row(task, rec, acts, rews, 0.0), TSV["header"])
    for col, g, r in zip(TSV["header"], got, ref):
        if col not in SKIP:
            assert g == r, (line, col, g, r)


def test_header_matches_reference():
    lines = sorted(int(k) for k in TSV["rows"])
    rows = [C.result_row(*_oracle_row(ln), 0.0) for ln in lines]
    text = C.pp_rows(rows)
    assert text.split("\n")[0].split("\t") == TSV["header"]
    assert len(text.rstrip("\n").split("\n")) == len(rows) + 1


def test_task_lists():
    hn = C.honest_net_tasks(10000)
    assert len(hn) == 5 * (2 + 6 * 4)  # (nakamoto, ethereum, 6 k x (2 B_k + 2 Tailstorm)) x 5
    wh = C.withholding_tasks(10000)
    nak, eth = 4, 5
    assert len(wh) == 7 * nak + 28 * nak + 7 * eth + 28 * eth + 6 * 2 * 7 * 4 + 6 * 2 * 7 * 7
    t = [x for x in wh if x.network.key == "gamma-0.9"][0]
    # 1 / (1 - 0.9) = 10.000000000000002 in floating point: 11 defenders, as the
    # reference's gamma-0.9 rows of data/withholding.tsv have
    assert t.network.cfg["defenders"] == 11 and len(t.network.compute) == 12
    assert t.attack.key == "ssz-unitobs-honest"
    r = C.prepare_row(t)
    assert dict(r)["compute"].split("|")[1] == C.string_of_float(0.9 / 11)
    assert dict(r)["network_description"] == (
        "1 attacker, alpha=0.1, 11 symmetric defenders, constant propagation delays "
        "modeling gamma=0.9. with defender message delay 0.0001)")


def test_error_row():
    t = C.honest_net_tasks(100)[0]
    import numpy as np

    rec = np.zeros(1, dtype=L.RECORD_DTYPE)[0]
    rec["status"] = L.ST_REFERENCE_RAISES
    r = dict(C.result_row(t, rec, [0] * 10, [0.0] * 10, 0.5))
    assert r["error"].startswith("the reference simulator raises") and "reward" not in r
