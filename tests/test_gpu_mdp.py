"""MDP-derived table policies (cpr_amd.mdp) on the device — needs an
MI355X. The value-iteration table for the SSZ'16 Bitcoin model drives CPR_POLICY_TABLE in
cpr-nakamoto-v0 episodes: every record bit-identical to the oracle on the keyed stream, and at
alpha >= 0.35, gamma = 0.5 it earns more than sapirshtein-2016-sm1 on the same stream (oracle
sample, 4000 episodes: 0.4228 vs 0.4155 at alpha = 0.35, 0.5663 vs 0.5250 at 0.4)."""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device, mdp

pytestmark = pytest.mark.gpu

FIELDS = [f for f in L.RECORD_DTYPE.names if f != "status"]


@pytest.fixture(scope="module")
def ctx():
    return device.default_context()


@pytest.mark.parametrize("alpha,gamma", [(0.4, 0.5), (0.3, 0.0), (0.45, 0.9)])
def test_mdp_table_records_match_oracle(ctx, alpha, gamma):
    table = mdp.policy_table(alpha, gamma, maximum_fork_length=20)
    cfg, keep = device.make_config(alpha=alpha, gamma=gamma, max_steps=2016, seed=0xD0,
                                   policy=L.POLICY_TABLE, table=table)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    _, rec = b.run(512, records=True)
    ref = O.run_episodes(cfg, 0, 512, threads=8)
    for f in FIELDS:
        bad = np.nonzero(rec[f] != ref[f])[0]
        assert len(bad) == 0, (f, int(bad[0]), rec[f][bad[0]], ref[f][bad[0]])


def _rel(ctx, alpha, n, **kw):
    cfg, keep = device.make_config(alpha=alpha, gamma=0.5, max_steps=2016, seed=0xD1, **kw)
    b = device.Batch(cfg, ctx=ctx, keep=keep)
    _, rec = b.run(n, records=True)
    rel = rec["reward_attacker"] / (rec["reward_attacker"] + rec["reward_defender"])
    return rel.mean(), rel.std() / np.sqrt(n)


@pytest.mark.parametrize("alpha", [0.35, 0.4, 0.45])
def test_mdp_table_beats_sm1(ctx, alpha):
    n = 1 << 16
    table = mdp.policy_table(alpha, 0.5, maximum_fork_length=20)
    m, sm = _rel(ctx, alpha, n, policy=L.POLICY_TABLE, table=table)
    s, ss = _rel(ctx, alpha, n, policy=L.POLICY_SAPIRSHTEIN_2016_SM1)
    assert m > s + 5 * np.hypot(sm, ss), (alpha, m, s)
