"""Honest cliques (experiments/simulate/models.ml:3-28) on the device — needs an MI355X.

Nakamoto (the event engine in Nakamoto mode) and Ethereum lanes on n honest nodes with
compute 1..n and uniform link delays, Simulator.loop tasks: every record bit-identical to
the oracle on the keyed stream, and the reference's own data/honest_net.tsv rows reproduced
on the device by replaying the OCaml 4.12 Random stream the oracle records for them.
"""

import json
import pathlib

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f != "status"]
ROWS = json.loads((pathlib.Path(__file__).parent / "golden" / "honest_net_clique.json")
                  .read_text())["rows"]


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


def _cfg(protocol, n, ad, acts, scheme=L.REWARD_DISCOUNT, seed=11, **kw):
    return device.make_config(
        alpha=0.0, gamma=0.0, defenders=n, network=L.NET_HONEST_CLIQUE, mode=L.MODE_LOOP,
        protocol=L.PROTO_ETHEREUM if protocol == "ethereum" else L.PROTO_NAKAMOTO,
        reward_scheme=scheme, activation_delay=ad, activations=acts, seed=seed,
        policy=0, **kw)


@pytest.mark.parametrize("protocol", ["nakamoto", "ethereum"])
@pytest.mark.parametrize("n,ad", [(10, 30.0), (10, 600.0), (3, 2.0), (33, 10.0)])
def test_clique_records_match_oracle(ctx, protocol, n, ad):
    cfg, keep = _cfg(protocol, n, ad, 2000)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(96, records=True)
    ref = O.run_episodes(cfg, 0, 96, threads=8)
    for f in FIELDS:
        bad = np.nonzero(rec[f] != ref[f])[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])
    assert not (rec["status"] & L.ST_CAPACITY).any()
    assert s.episodes == 96 and s.activations == int(rec["n_activations"].sum())


def test_clique_custom_delays(ctx):
    cfg, keep = _cfg("nakamoto", 5, 1.0, 1500, delay_lo=0.2, delay_hi=3.0)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    _, rec = b.run(64, records=True)
    ref = O.run_episodes(cfg, 0, 64, threads=8)
    for f in FIELDS:
        assert np.array_equal(rec[f], ref[f]), f


@pytest.mark.parametrize("row", ROWS, ids=[f"line{r['line']}" for r in ROWS])
def test_replay_reproduces_honest_net_rows(ctx, row):
    scheme = L.REWARD_DISCOUNT if row["incentive_scheme"] == "discount" else L.REWARD_CONSTANT
    cfg, keep = _cfg(row["protocol"], row["nodes"], row["activation_delay"], row["activations"],
                     scheme=scheme)
    trace, ref = O.export_traces(cfg, 0, 1, rng=O.OcamlRandom())
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    _, rec = b.replay(trace)
    assert not (rec["status"] & L.ST_TRACE_MISS).any()
    for f in FIELDS:
        assert rec[f][0] == ref[f][0], f
    assert rec["reward_attacker"][0] == row["reward"][0]
    assert rec["reward_defender"][0] == sum(row["reward"][1:])
    assert rec["n_activations"][0] == sum(row["activations_per_node"])
    assert float("%.12g" % rec["chain_time"][0]) == float(row["head_time"])
    assert rec["head_height"][0] == row["head_height"]
    assert rec["progress"][0] == row["head_progress"]


# ---------------------------------------------------------------- B_k and Tailstorm cliques

def _cfg_bkts(protocol, n, ad, acts, k, scheme, selection=L.SELECT_HEURISTIC, seed=13):
    return device.make_config(
        alpha=0.0, gamma=0.0, defenders=n, network=L.NET_HONEST_CLIQUE, mode=L.MODE_LOOP,
        protocol=L.PROTO_BK if protocol == "bk" else L.PROTO_TAILSTORM, reward_scheme=scheme,
        k=k, subblock_selection=selection, activation_delay=ad, activations=acts, seed=seed,
        policy=0)


@pytest.mark.parametrize("protocol,k,scheme,selection", [
    ("bk", 8, L.REWARD_CONSTANT, 0), ("bk", 4, L.REWARD_BLOCK, 0),
    ("tailstorm", 8, L.REWARD_DISCOUNT, L.SELECT_HEURISTIC),
    ("tailstorm", 4, L.REWARD_CONSTANT, L.SELECT_OPTIMAL),
    ("tailstorm", 3, L.REWARD_HYBRID, L.SELECT_ALTRUISTIC)])
@pytest.mark.parametrize("n,ad", [(10, 30.0), (10, 2.0), (3, 0.5), (2, 600.0)])
def test_bk_ts_clique_records_match_oracle(ctx, protocol, k, scheme, selection, n, ad):
    cfg, keep = _cfg_bkts(protocol, n, ad, 1500, k, scheme, selection)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    s, rec = b.run(64, records=True)
    ref = O.run_episodes(cfg, 0, 64, threads=8)
    for f in FIELDS:
        bad = np.nonzero(rec[f] != ref[f])[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])
    assert not (rec["status"] & L.ST_CAPACITY).any()
    assert s.episodes == 64 and s.activations == int(rec["n_activations"].sum())


CHAIN_ROWS = json.loads((pathlib.Path(__file__).parent / "golden" / "honest_net_chains.json")
                        .read_text())["rows"]


@pytest.mark.parametrize("row", [r for r in CHAIN_ROWS if r["protocol"] in ("bk", "tailstorm")],
                         ids=lambda r: f"line{r['line']}-{r['protocol']}")
def test_replay_reproduces_chained_bk_ts_rows(ctx, row):
    # the OCaml Random state the row's Parany worker had (test_oracle_clique.chained_rng),
    # then the row's own draws exported as a trace and replayed on the device
    from test_oracle_clique import chained_rng

    scheme = {"constant": L.REWARD_CONSTANT, "block": L.REWARD_BLOCK,
              "discount": L.REWARD_DISCOUNT}[row["incentive_scheme"]]
    sel = {None: 0, "altruistic": 0, "heuristic": 1, "optimal": 2}[row["subblock_selection"]]
    cfg, keep = _cfg_bkts(row["protocol"], row["nodes"], row["activation_delay"],
                          row["activations"], row["k"], scheme, sel)
    trace, ref = O.export_traces(cfg, 0, 1, rng=chained_rng(row))
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    _, rec = b.replay(trace)
    assert not (rec["status"] & L.ST_TRACE_MISS).any()
    for f in FIELDS:
        assert rec[f][0] == ref[f][0], f
    assert rec["reward_attacker"][0] == row["reward"][0]
    assert rec["reward_defender"][0] == sum(row["reward"][1:])
    assert rec["n_activations"][0] == sum(row["activations_per_node"])
    assert float("%.12g" % rec["chain_time"][0]) == float(row["head_time"])
    assert rec["head_height"][0] == row["head_height"]
    assert rec["progress"][0] == row["head_progress"]
