"""The FC'16 abstract-model kernel (gym/rust/src/fc16.rs FC16SSZwPT).

CPU: the exact chain value of a table policy (cpr_amd.mdp.fc16_policy_value) against the
pure-Python episode oracle (tests/oracle_py.py fc16_episode) within 4 sigma, and the
MDP-derived table beating honest and SM1 in expectation. GPU: device records equal the
oracle's bit for bit on the keyed stream, and 2^20 device episodes match the exact value
within 4 sigma.
"""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import mdp


def _table(alpha=0.35, gamma=0.5, horizon=30):
    return mdp.fc16_table(alpha, gamma, horizon=horizon, maximum_fork_length=12)


def test_fc16_oracle_matches_exact_value():
    tab = _table()
    ev, eg = mdp.fc16_policy_value(0.35, 0.5, 30, tab)
    out = np.array([O.fc16_episode(7, e, 0.35, 0.5, 30, 2, tab)[:2] for e in range(1500)],
                   dtype=float)
    for i, want in enumerate((ev, eg)):
        z = (out[:, i].mean() - want) / (out[:, i].std(ddof=1) / np.sqrt(len(out)))
        assert abs(z) < 4, (i, out[:, i].mean(), want, z)


def test_fc16_mdp_table_beats_built_in_policies():
    # expected reward per episode: the MDP's table >= SM1 and honest at alpha .35, gamma .5
    tab = _table()
    honest = np.zeros(13 * 13 * 3, np.uint8)
    for a in range(13):
        for h in range(13):
            honest[(a * 13 + h) * 3:(a * 13 + h) * 3 + 3] = (
                O.FC16_OVERRIDE if a > h else (O.FC16_ADOPT if h > a else O.FC16_WAIT))
    v_tab, g_tab = mdp.fc16_policy_value(0.35, 0.5, 30, tab)
    v_hon, g_hon = mdp.fc16_policy_value(0.35, 0.5, 30, honest)
    assert v_tab / g_tab > v_hon / g_hon
    assert abs(v_hon / g_hon - 0.35) < 0.01  # honest play earns its share


@pytest.mark.gpu
def test_fc16_device_matches_oracle_and_value():
    from cpr_amd import device

    tab = _table()
    cfg, keep = device.make_config(protocol=L.PROTO_FC16, alpha=0.35, gamma=0.5, horizon=30,
                                   table=tab, seed=7)
    b = device.Batch(cfg, keep=keep)
    s, rec = b.run(256, records=True)
    ref = np.array([O.fc16_episode(7, e, 0.35, 0.5, 30, 2, tab) for e in range(256)])
    assert np.array_equal(rec["reward_attacker"], ref[:, 0])
    assert np.array_equal(rec["progress"], ref[:, 1])
    assert np.array_equal(rec["n_steps"], ref[:, 2])
    for pol in (L.FC16_POLICY_HONEST, L.FC16_POLICY_SM1):
        cfg2, _ = device.make_config(protocol=L.PROTO_FC16, alpha=0.4, gamma=0.9, horizon=20,
                                     policy=pol, seed=3)
        _, rec2 = device.Batch(cfg2).run(128, records=True)
        ref2 = np.array([O.fc16_episode(3, e, 0.4, 0.9, 20, pol) for e in range(128)])
        assert np.array_equal(rec2["reward_attacker"], ref2[:, 0]), pol
        assert np.array_equal(rec2["n_steps"], ref2[:, 2]), pol
    # 2^20 episodes against the exact chain value
    n = 1 << 20
    s, rec = b.run(n, first_episode=1 << 32, records=True)
    ev, eg = mdp.fc16_policy_value(0.35, 0.5, 30, tab)
    r = rec["reward_attacker"]
    z = (r.mean() - ev) / (r.std(ddof=1) / np.sqrt(n))
    assert abs(z) < 4, (r.mean(), ev, z)
    assert s.episodes == n and s.invalid == 0
