"""Honest cliques (experiments/simulate/models.ml:3-28) in the oracle, pinned by the
reference's own recorded outputs: every Nakamoto and Ethereum row of data/honest_net.tsv
(10 nodes, compute 1..10, uniform 0.5..1.5 delays, 10,000 activations; each task starts from
OCaml's default Random state) reproduces bit for bit with the OCaml 4.12 Random replica —
activations and reward of every node, head time to the TSV's 12 digits, head progress and
height. Fixture: tests/golden/honest_net_clique.json (make_honest_net_fixture.py)."""

import json
import pathlib

import numpy as np
import pytest

import oracle_py as O

ROWS = json.loads((pathlib.Path(__file__).parent / "golden" / "honest_net_clique.json")
                  .read_text())["rows"]


def _scheme(row):
    return 1 if row["incentive_scheme"] == "discount" else 0


@pytest.mark.parametrize("row", ROWS, ids=[f"line{r['line']}" for r in ROWS])
def test_honest_net_rows_exact(row):
    out = O.clique_task(row["protocol"], row["nodes"], row["activation_delay"],
                        row["activations"], scheme=_scheme(row), rng=O.OcamlRandom())
    assert out["activations"] == row["activations_per_node"]
    assert out["reward"] == row["reward"]
    assert float("%.12g" % out["head_time"]) == float(row["head_time"])
    assert out["head_progress"] == row["head_progress"]
    assert out["head_height"] == row["head_height"]


def test_keyed_clique_statistics_match_reference_rows():
    # the keyed stream is a different random source for the same model: orphan rates and
    # reward shares of 24 keyed tasks bracket the reference's rows
    for row in [r for r in ROWS if r["activation_delay"] in (30.0, 600.0)]:
        orph, share = [], []
        for ep in range(24):
            out = O.clique_task(row["protocol"], row["nodes"], row["activation_delay"],
                                row["activations"], scheme=_scheme(row), seed=7, episode=ep)
            orph.append(1 - out["head_height"] / row["activations"])
            share.append(out["reward"][-1] / sum(out["reward"]))
        ref_orph = 1 - row["head_height"] / row["activations"]
        ref_share = row["reward"][-1] / sum(row["reward"])
        for xs, ref in ((orph, ref_orph), (share, ref_share)):
            m, sd = float(np.mean(xs)), float(np.std(xs, ddof=1))
            assert abs(ref - m) <= 4 * sd + 1e-4, (row["line"], ref, m, sd)


# ---------------------------------------------------------------- Parany worker chains
#
# csv_runner.ml:105-131 runs honest_net.ml's tasks on forked Parany workers whose Random state
# carries from task to task. make_honest_net_chains.py recovered, for 23 rows, the earlier rows
# their worker ran first; replaying that chain from the default state reproduces the row bit
# for bit — including 10 B_k (k = 1, 2) and 3 Tailstorm (k = 1) rows, both incentive schemes; the chains of
# later rows pass through spar/stree tasks, which are out of scope).

import importlib.util  # noqa: E402

_spec = importlib.util.spec_from_file_location(
    "make_honest_net_chains", pathlib.Path(__file__).parent / "golden" / "make_honest_net_chains.py")
CH = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(CH)
CHAINS = json.loads((pathlib.Path(__file__).parent / "golden" / "honest_net_chains.json")
                    .read_text())["rows"]
BY_LINE = {r["line"]: r for r in CHAINS}


_CHAIN_END = {}


def chained_rng(row):
    """OCaml's default Random state advanced over the row's recovered worker chain (a copy of
    a per-process memo: several GPU tests start from the same row's state)."""
    key = tuple(row["chain"])
    if key not in _CHAIN_END:
        rng = O.OcamlRandom()
        for ln in row["chain"]:
            CH.run(BY_LINE[ln], rng)
        _CHAIN_END[key] = rng
    return _CHAIN_END[key].copy()


def test_chain_fixture_covers_bk_and_tailstorm():
    protos = [r["protocol"] for r in CHAINS]
    assert protos.count("bk") == 10 and protos.count("tailstorm") == 3
    assert {r["incentive_scheme"] for r in CHAINS if r["protocol"] == "bk"} == {"block", "constant"}


@pytest.mark.parametrize("row", [r for r in CHAINS if r["protocol"] in ("bk", "tailstorm")],
                         ids=lambda r: f"line{r['line']}-{r['protocol']}")
def test_honest_net_chained_rows_exact(row):
    out = CH.run(row, chained_rng(row))
    assert out["activations"] == row["activations_per_node"]
    assert out["reward"] == row["reward"]
    assert float("%.12g" % out["head_time"]) == float(row["head_time"])
    assert out["head_progress"] == row["head_progress"]
    assert out["head_height"] == row["head_height"]


BKTS_ROWS = json.loads((pathlib.Path(__file__).parent / "golden" / "honest_net_bk_ts_rows.json")
                       .read_text())["rows"]


def test_keyed_bk_ts_cliques_bracket_reference_rows():
    # the 24 B_k / Tailstorm rows (k = 4, 8, 16) whose worker states are unknown: orphan rate
    # (1 - progress / activations) and the strongest node's reward share of each row lie
    # within 4 sigma of 10 keyed oracle tasks of the same configuration
    schemes = {"constant": 0, "block": 2, "discount": 1}
    for row in BKTS_ROWS:
        orph, share = [], []
        for ep in range(10):
            kw = dict(net="honest-clique", n_nodes=row["nodes"],
                      activation_delay=row["activation_delay"],
                      scheme=schemes[row["incentive_scheme"]], seed=7, episode=ep)
            if row["protocol"] == "bk":
                out = O.bk_loop(row["k"], row["activations"], **kw)
            else:
                out = O.ts_loop(row["k"], row["activations"],
                                selection=O.TS_SELECTIONS[row["subblock_selection"]], **kw)
            orph.append(1 - out["head_progress"] / row["activations"])
            share.append(out["reward"][-1] / sum(out["reward"]))
        ref_orph = 1 - row["head_progress"] / row["activations"]
        ref_share = row["reward"][-1] / sum(row["reward"])
        for xs, ref in ((orph, ref_orph), (share, ref_share)):
            m, sd = float(np.mean(xs)), float(np.std(xs, ddof=1))
            assert abs(ref - m) <= 4 * sd + 1e-4, (row["line"], ref, m, sd)
