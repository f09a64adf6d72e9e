"""Per-node outputs of the oracle (the checker behind cpr_node_outputs), on the CPU.

The oracle's per-node rows decompose its own records for every loop-task network the
device runs, and its trace path reproduces the `activations` / `reward` columns of the
reference's data/honest_net.tsv rows (csv_runner.ml:74-79) exactly.
"""

import json
import pathlib

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from test_gpu_nodes import CASES, _clique

ROWS = json.loads((pathlib.Path(__file__).parent / "golden" / "honest_net_clique.json")
                  .read_text())["rows"]


def _nodes(cfg):
    if cfg.network == L.NET_TWO_AGENTS:
        return 2
    return cfg.defenders if cfg.network == L.NET_HONEST_CLIQUE else cfg.defenders + 1


@pytest.mark.parametrize("case", list(CASES))
def test_rows_decompose_records(case):
    cfg, _keep = CASES[case]()
    n = 4
    rec, acts, rews, hm = O.node_outputs(cfg, _nodes(cfg), first=100, n=n)
    ref = O.run_episodes(cfg, 100, n)
    ok = (rec["status"] & L.ST_INVALID) == 0
    for f in ("reward_attacker", "reward_defender", "progress", "n_activations", "head_height"):
        assert np.array_equal(rec[f], ref[f]), f
    assert np.array_equal(acts.sum(axis=1)[ok], rec["n_activations"][ok])
    assert np.array_equal(rews[ok, 0], rec["reward_attacker"][ok])
    # sums in node order, as run_loop_episode adds the defenders
    dsum = np.array([sum(r[1:].tolist(), 0.0) for r in rews])
    assert np.array_equal(dsum[ok], rec["reward_defender"][ok])


@pytest.mark.parametrize("row", ROWS[:6], ids=[f"line{r['line']}" for r in ROWS[:6]])
def test_trace_rows_reproduce_honest_net(row):
    scheme = L.REWARD_DISCOUNT if row["incentive_scheme"] == "discount" else L.REWARD_CONSTANT
    proto = L.PROTO_ETHEREUM if row["protocol"] == "ethereum" else L.PROTO_NAKAMOTO
    cfg, _keep = _clique(proto, row["nodes"], row["activation_delay"], row["activations"],
                         scheme=scheme, seed=11)
    trace, _ = O.export_traces(cfg, 0, 1, rng=O.OcamlRandom())
    rec, acts, rews, hm = O.node_outputs(cfg, row["nodes"], trace=trace)
    assert acts[0].tolist() == row["activations_per_node"]
    assert rews[0].tolist() == row["reward"]
    assert rec["head_height"][0] == row["head_height"]
