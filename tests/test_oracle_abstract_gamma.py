"""The oracle's flagged abstract-gamma mode (CPR_NET_ABSTRACT_GAMMA), CPU only.

Not a reference network (the reference rejects gamma = 1): oracle/src/des.cpp NakHonest
decides a match race against the defender block mined at the same instant by the keyed
coin U(k, 0, j) < gamma, with every delay zero. Pinned by the Eyal-Sirer closed form
(FC'14) for sapirshtein-2016-sm1, and by gamma = 0 reproducing first-received (the miner
and every defender keep the defender block). The device lane is compared with this oracle
record by record in tests/test_gpu_abstract_gamma.py and step by step on the host in
tests/native/lane_vs_oracle.cpp.
"""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device


def es14(alpha, gamma):
    a, g = alpha, gamma
    return (a * (1 - a) ** 2 * (4 * a + g * (1 - 2 * a)) - a ** 3) / (1 - a * (1 + (2 - a) * a))


@pytest.mark.parametrize("alpha,gamma", [(0.35, 1.0), (0.3, 0.5), (0.4, 0.0)])
def test_oracle_abstract_gamma_sm1_matches_eyal_sirer(alpha, gamma):
    n, steps = 64, 16384
    cfg, _ = device.make_config(alpha=alpha, gamma=gamma, network=L.NET_ABSTRACT_GAMMA,
                                defenders=2, max_steps=steps, seed=0x0AB5)
    rec = O.run_episodes(cfg, 0, n, threads=8)
    ra, h = rec["reward_attacker"], rec["progress"]
    r = ra.sum() / h.sum()
    se = np.sqrt(np.var(ra - r * h, ddof=1) / n) / h.mean()
    z = (r - es14(alpha, gamma)) / se
    assert abs(z) < 4, (r, es14(alpha, gamma), se, z)
    assert (rec["n_activations"] == steps + 1).all()


def test_oracle_abstract_gamma_one_beats_reference_gamma():
    # gamma = 1 is strictly better for the attacker than the gym's best representable
    # gamma with two defenders (0.5): the flag changes the outcome, not just the label
    cfg1, _ = device.make_config(alpha=0.3, gamma=1.0, network=L.NET_ABSTRACT_GAMMA,
                                 defenders=2, max_steps=4096, seed=5)
    cfg5, _ = device.make_config(alpha=0.3, gamma=0.5, max_steps=4096, seed=5)
    r1 = O.run_episodes(cfg1, 0, 32, threads=8)
    r5 = O.run_episodes(cfg5, 0, 32, threads=8)
    assert r1["reward_attacker"].sum() / r1["progress"].sum() > \
        r5["reward_attacker"].sum() / r5["progress"].sum() + 0.02
