"""The headline network on the device against the reference's own data — needs an MI355X.

The gym's selfish-mining network (Network.T.selfish_mining, network.ml:61-105) is the path
BASELINE configs[1] runs on. Its semantics are pinned here two ways:

1. Simulator.loop rows of data/withholding.tsv (`gamma-*`, 112 Nakamoto rows: 7 alphas x
   gamma {0, .5, .75, .9} x 4 nakamoto_ssz policies, 10,000 activations, defender message
   delay 1e-4, models.ml:54-84, withholding.ml:29-52). Device records equal the oracle's
   bit for bit on sampled rows; every row's attacker reward, defender reward, progress and
   head time lie within 4 sigma of 1,024 device tasks (rank statistic, tests/gamma_stats.py).
2. experiments/rl-eval/rl-results.csv `gamma*_seq_hc` (cpr-v0 Nakamoto gym, defenders 42,
   2048-step episodes, best of SM1/honest mean reward per progress over 100 episodes,
   eval-policies.ipynb): within 3 sigma of 4,096 device episodes per point.
Fixtures: tests/golden/make_gamma_fixtures.py.
"""

import pathlib
import time

import numpy as np
import pytest

import gamma_stats as G
import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f != "status"]
N_TASKS = 512


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


SAMPLED = [(0.0, 0.45, "sapirshtein-2016-sm1"), (0.0, 0.33, "honest"),
           (0.5, 0.33, "sapirshtein-2016-sm1"), (0.5, 0.1, "eyal-sirer-2014"),
           (0.75, 0.4, "simple"), (0.75, 0.5, "sapirshtein-2016-sm1"),
           (0.9, 0.45, "sapirshtein-2016-sm1"), (0.9, 0.25, "honest")]


@pytest.mark.parametrize("gamma,alpha,policy", SAMPLED)
def test_gamma_loop_records_match_oracle(ctx, gamma, alpha, policy):
    row = next(r for r in G.withholding_rows()
               if (r["gamma"], r["alpha"], r["policy"]) == (gamma, alpha, policy))
    cfg = G.row_config(device.make_config, L, row, seed=0xB17)
    b = device.Batch(cfg, ctx=ctx)
    s, rec = b.run(48, records=True)
    ref = O.run_episodes(cfg, 0, 48, threads=8)
    assert not (rec["status"] & (L.ST_CAPACITY | L.ST_TRACE_MISS)).any()
    for f in FIELDS:
        bad = np.nonzero(rec[f] != ref[f])[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])
    assert s.episodes == 48 and s.activations == 48 * 10000


def test_gamma_loop_rows_within_4_sigma(ctx, say, tmp_path):
    # rows are latency-bound (one batch of dependent chains each), so they run side by side:
    # 4 worker processes x 4 streams (tests/gamma_rows_worker.py), the slow many-defender
    # rows spread over the workers first
    import subprocess
    import sys

    rows = G.withholding_rows()
    order = sorted(range(len(rows)), key=lambda i: -rows[i]["defenders"])
    shares = [order[w::4] for w in range(4)]
    t0 = time.perf_counter()
    procs = []
    for w, share in enumerate(shares):
        out = tmp_path / f"w{w}.npz"
        procs.append((out, subprocess.Popen(
            [sys.executable, str(pathlib.Path(__file__).parent / "gamma_rows_worker.py"),
             str(out), str(N_TASKS), *map(str, share)],
            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    done = 0
    log = []
    import selectors

    sel = selectors.DefaultSelector()
    for _, p in procs:
        sel.register(p.stdout, selectors.EVENT_READ)
    open_streams = len(procs)
    while open_streams:
        for key, _ in sel.select(timeout=30):
            line = key.fileobj.readline()
            if not line:
                sel.unregister(key.fileobj)
                open_streams -= 1
            elif not line.startswith("row "):
                log.append(line)
            else:
                done += 1
                if done % 8 == 0:
                    say(f"  gamma rows: {done} of {len(rows)} ({time.perf_counter() - t0:.0f} s)")
    results = []
    for out, p in procs:
        assert p.wait() == 0, f"worker failed ({out}): {''.join(log)[-3000:]}"
        z = np.load(out)
        results += [(rows[int(k[1:])], z[k]) for k in z.files]
    assert len(results) == len(rows)
    worst = (0.0, None)
    zs = []
    for row, rec in results:
        assert not (rec["status"] & L.ST_CAPACITY).any(), row
        for k, z in G.withholding_z(row, rec, stat=G.rank_z).items():
            zs.append(abs(z))
            if abs(z) > worst[0]:
                worst = (abs(z), (row["line"], row["gamma"], row["alpha"], row["policy"], k))
    print(f"{len(zs)} comparisons, worst |z| = {worst[0]:.2f} at {worst[1]}, "
          f"{sum(z > 3 for z in zs)} above 3")
    assert worst[0] < 4.0, worst


def test_rl_results_seq_hc_within_3_sigma(ctx, say):
    # 15 points: 3 sigma per point, and the family-wise band (Bonferroni, 1% over 15
    # two-sided tests: |z| < 3.40) for the single worst point
    from statistics import NormalDist

    band = NormalDist().inv_cdf(1.0 - 0.01 / (2 * len(G.rl_rows())))
    zs = []
    worst = (0.0, None)
    for row in G.rl_rows():
        rpp = {}
        for name, pid in (("sapirshtein-2016-sm1", L.POLICY_SAPIRSHTEIN_2016_SM1),
                          ("honest", L.POLICY_HONEST)):
            cfg, _ = device.make_config(alpha=row["alpha"], gamma=row["gamma"], defenders=42,
                                        policy=pid, max_steps=2048, seed=0x41E5)
            b = device.Batch(cfg, ctx=ctx)
            _, rec = b.run(4096, records=True)
            b.close()
            assert (rec["n_steps"] == 2048).all()
            rpp[name] = rec["reward_attacker"] / rec["progress"]
        best, mean, z = G.rpp_z(row["rpp_mean"], rpp)
        zs.append(abs(z))
        say(f"  alpha {row['alpha']} gamma {row['gamma']}: best {best} {mean:.4f} vs "
            f"reference {row['rpp_mean']:.4f}, z = {z:+.2f}")
        if abs(z) > worst[0]:
            worst = (abs(z), (row["alpha"], row["gamma"], best, mean, row["rpp_mean"]))
    print(f"worst |z| = {worst[0]:.2f} at {worst[1]}; {sum(z > 3 for z in zs)} of {len(zs)} "
          f"above 3; family-wise band {band:.2f}")
    assert sum(z > 3.0 for z in zs) <= 1 and worst[0] < band, worst


@pytest.mark.parametrize("gamma", [0.5, 0.9])
@pytest.mark.parametrize("policy", [L.POLICY_SAPIRSHTEIN_2016_SM1, L.POLICY_EYAL_SIRER_2014])
def test_gamma_loop_closed_form_matches_oracle(ctx, gamma, policy):
    # loop tasks at the gym's 1e-9 propagation delay stay on the closed-form lane (overlaps
    # re-run exactly); the oracle restates Simulator.loop on the same network
    cfg, _ = device.make_config(alpha=0.42, gamma=gamma, policy=policy, mode=L.MODE_LOOP,
                                activations=3000, propagation_delay=1e-9, seed=0xC10)
    b = device.Batch(cfg, ctx=ctx)
    _, rec = b.run(512, records=True)
    ref = O.run_episodes(cfg, 0, 512, threads=8)
    for f in FIELDS:
        bad = np.nonzero(rec[f] != ref[f])[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])
