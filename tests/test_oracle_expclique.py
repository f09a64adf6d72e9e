"""The oracle's exponential-delay clique with an attacker (CPR_NET_EXP_CLIQUE), on the CPU:
the config-driven loop task equals oracle_bk_loop / oracle_ts_loop on the same network
(cpr_protocols.ml:200-210,478-485) episode by episode, and the reference's policy-test
orphan limit (cpr_protocols.ml:554-617: honest policy, 3 nodes, activation delay 100,
exponential(1) links, 1000 activations, orphan rate <= 0.01) holds on average.
"""

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from test_gpu_expclique import RANDOM_CASES, exp_clique


@pytest.mark.parametrize("proto,pol", [(L.PROTO_BK, L.BK_POLICY_AVOID_LOSS),
                                       (L.PROTO_TAILSTORM, L.TS_POLICY_AVOID_LOSS)])
def test_config_task_equals_loop_task(proto, pol):
    scheme = L.REWARD_DISCOUNT if proto == L.PROTO_TAILSTORM else L.REWARD_CONSTANT
    cfg, _ = exp_clique(proto, 2, pol, 500, k=8, scheme=scheme, ad=10.0, seed=4)
    rec, a, r, _ = O.node_outputs(cfg, 3, first=2, n=3)
    for e in range(3):
        if proto == L.PROTO_BK:
            o = O.bk_loop(8, 500, net="clique", n_nodes=3, activation_delay=10.0, prop_ev=1.0,
                          policy=pol, scheme=0, seed=4, episode=2 + e)
        else:
            o = O.ts_loop(8, 500, net="clique", n_nodes=3, activation_delay=10.0, prop_ev=1.0,
                          policy=pol, scheme="discount", seed=4, episode=2 + e)
        assert a[e].tolist() == o["activations"] and r[e].tolist() == o["reward"]
        assert rec["head_height"][e] == o["head_height"]
        assert rec["progress"][e] == o["head_progress"]


@pytest.mark.parametrize("proto,k,scheme,sel", [
    (L.PROTO_BK, 8, L.REWARD_BLOCK, 0),
    (L.PROTO_TAILSTORM, 8, L.REWARD_CONSTANT, L.SELECT_OPTIMAL),
    (L.PROTO_TAILSTORM, 8, L.REWARD_DISCOUNT, L.SELECT_HEURISTIC),
])
def test_policy_test_orphan_limit(proto, k, scheme, sel):
    cfg, _ = exp_clique(proto, 2, 0, 1000, k=k, scheme=scheme, sel=sel, ad=100.0, seed=7)
    rec = O.run_episodes(cfg, 0, 64, threads=8)
    orphan = (1000.0 - rec["progress"]) / 1000.0
    assert orphan.mean() <= 0.01 and (orphan <= 0.01).mean() > 0.9


def test_exp_clique_config():
    cfg, _ = exp_clique(L.PROTO_TAILSTORM, 1, L.TS_POLICY_HONEST, 100)
    assert cfg.network == L.NET_EXP_CLIQUE and cfg.defenders == 1
    assert cfg.propagation_delay == 1.0 and cfg.mode == L.MODE_LOOP


# the reference's `random` policy tests (cpr_protocols.ml:658-782): node 0 takes a uniformly
# random action of its attack space at every decision (Random.int A.Action.n; here the
# keyed draw of include/cpr_hip.h *_POLICY_RANDOM), 3-node symmetric clique, activation
# delay 100, exponential(1) links, 1000 activations; the orphan rate must stay <= 0.5
# (RANDOM_CASES: test_gpu_expclique.py). Every episode completes: the optimal selection's
# large searches (OCaml's overflowed n_choose_k) run pruned (oracle/src/tailstorm.cpp)
@pytest.mark.parametrize("name,proto,pol,k,scheme,sel", RANDOM_CASES)
def test_random_attacker_orphan_limit(name, proto, pol, k, scheme, sel):
    cfg, _ = exp_clique(proto, 2, pol, 1000, k=k, scheme=scheme, sel=sel, ad=100.0, seed=9)
    rec = O.run_episodes(cfg, 0, 32, threads=8)
    assert not (rec["status"] & L.ST_INVALID).any(), name
    orphan = (1000.0 - rec["progress"]) / 1000.0
    assert orphan.max() <= 0.5, (name, orphan.max())
    # the draws are the keyed stream's: another seed gives other episodes
    cfg2, _ = exp_clique(proto, 2, pol, 1000, k=k, scheme=scheme, sel=sel, ad=100.0, seed=10)
    rec2 = O.run_episodes(cfg2, 0, 8, threads=8)
    assert not np.array_equal(rec2["reward_attacker"], rec["reward_attacker"][:8]), name
