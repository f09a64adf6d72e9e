"""The oracle on the selfish-mining (gamma) network against the reference's own recorded
Simulator.loop rows (data/withholding.tsv `gamma-*`, models.ml:54-84, withholding.ml:29-52;
fixture tests/golden/withholding_nakamoto_gamma.json made by make_gamma_fixtures.py).

Those rows started from unrecoverable OCaml Random states, so they pin the oracle
statistically: every row's progress and head time, and (gamma > 0) the attacker's and the
defenders' rewards, lie within 4 sigma of 32 keyed oracle tasks of the same configuration.
At gamma = 0 the rewards are heavy tailed (the attacker's share is the private fork still
ahead when the loop ends); tests/test_gpu_gamma.py checks them on 1,024 device tasks per
row with a rank statistic.
"""

import numpy as np
import pytest

import gamma_stats as G
import oracle_py
from cpr_amd import _lib as L
from cpr_amd import device

N_TASKS = 32
BOUND = 4.0


def test_fixture_covers_the_sweep():
    rows = G.withholding_rows()
    assert len(rows) == 112  # 7 alphas x 4 gammas x 4 policies (withholding.ml:4,29)
    keys = {(r["alpha"], r["gamma"], r["policy"]) for r in rows}
    assert len(keys) == 112
    for r in rows:
        d = max(2, int(np.ceil(1.0 / (1.0 - r["gamma"]))))  # withholding.ml:44-46
        assert r["defenders"] == d
        assert len(r["reward"]) == d + 1 and r["activations"] == 10000
        # Nakamoto: progress = height = rewards along the head chain
        assert r["head_progress"] == r["head_height"] == sum(r["reward"])


def test_oracle_matches_reference_gamma_rows():
    worst = (0.0, None)
    for i, row in enumerate(G.withholding_rows()):
        cfg = G.row_config(device.make_config, L, row, seed=0x6A330000 + i)
        rec = oracle_py.run_episodes(cfg, 0, N_TASKS, threads=8)
        outs = G.OUTPUTS if row["gamma"] > 0 else ("progress", "head_time")
        for k, z in G.withholding_z(row, rec, outputs=outs).items():
            if abs(z) > worst[0]:
                worst = (abs(z), (row["line"], k))
            assert abs(z) < BOUND, (row, k, z)
    print(f"worst |z| = {worst[0]:.2f} at {worst[1]}")


def test_honest_policy_never_forks_on_gamma_network():
    # ssz-honest rows: every block of the attacker is shared at once, so with gamma > 0 the
    # head chain holds all but the orphans of 1e-4-delay races (progress ~ activations)
    row = next(r for r in G.withholding_rows()
               if r["policy"] == "honest" and r["gamma"] == 0.5 and r["alpha"] == 0.33)
    cfg = G.row_config(device.make_config, L, row, seed=7)
    rec = oracle_py.run_episodes(cfg, 0, 8, threads=8)
    assert (rec["progress"] >= 9990).all() and (rec["n_activations"] == 10000).all()
    assert row["head_progress"] == 10000.0


@pytest.mark.parametrize("gamma", [0.0, 0.9])
def test_gamma_loop_rejects_like_reference(gamma):
    # Network.T.selfish_mining raises for gamma > (d - 1) / d (network.ml:63-72)
    cfg, _ = device.make_config(alpha=0.3, gamma=gamma, defenders=2, mode=L.MODE_LOOP,
                                activations=100, propagation_delay=1e-4, seed=1)
    if gamma <= 0.5:
        rec = oracle_py.run_episodes(cfg, 0, 2)
        assert (rec["n_activations"] == 100).all()
    else:
        with pytest.raises(RuntimeError, match="gamma must not be greater"):
            oracle_py.run_episodes(cfg, 0, 2)
