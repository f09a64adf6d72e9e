"""Ethereum part of the CPU oracle against the reference's own known answers.

Pinned by: Compare.at_most_first KATs (simulator/lib/compare_test.ml:40-41), the uncle
validity KATs (simulator/protocols/ethereum_test.ml:82-168, all 28 cases), the action
table bijection (ethereum_ssz.ml:265-276) and the policy definitions
(ethereum_ssz.ml:444-521). The tie order of OCaml's heap sort among equal keys is
restated from the OCaml stdlib algorithm; no reference vector exercises it (parity
unpinned for that detail).
"""

import math
import random

import numpy as np
import pytest

import oracle_py as O
from cpr_amd import _lib as L
from cpr_amd import device


# ---------------------------------------------------------------- Compare / Array.sort


def test_at_most_first_kats():
    # compare_test.ml:40-41
    assert O.at_most_first([1, 7, 3, 5, 0, 2], 2) == [0, 1]
    assert O.at_most_first([7, 1], 3) == [1, 7]


def test_ocaml_sort_sorts():
    rnd = random.Random(7)
    for n in list(range(0, 12)) + [31, 100, 257]:
        xs = [rnd.randrange(-5, 5) for _ in range(n)]
        assert O.ocaml_sort(xs) == sorted(xs)


def test_ocaml_sort_tie_order_is_a_permutation():
    rnd = random.Random(3)
    for n in range(1, 20):
        keys = [rnd.randrange(3) for _ in range(n)]
        out = O.ocaml_sort_pairs(keys, list(range(n)))
        assert [k for k, _ in out] == sorted(keys)
        assert sorted(t for _, t in out) == list(range(n))


def test_ocaml_sort_is_not_stable():
    # heap sort: equal keys do not keep input order (e.g. three equal keys)
    out = O.ocaml_sort_pairs([0, 0, 0], [0, 1, 2])
    assert [t for _, t in out] != [0, 1, 2]


# ---------------------------------------------------------------- uncle validity


def test_ethereum_validity_kats():
    # ethereum_test.ml:44-168 (root height 43, work 47; mine = parent + uncles)
    d = O.EthDag(43, 47)

    def mine(p, u=()):
        return d.mine(p, u)

    def mine_exn(p, u=()):
        b, ok = mine(p, u)
        assert ok, "invalid block"
        return b

    a = [None] * 10
    a[9] = d.root
    for i in range(8, -1, -1):
        a[i] = mine_exn(a[i + 1])
    b = [None] * 9
    for i in range(8, -1, -1):
        b[i] = mine_exn(a[i + 1])
    c = [None] * 8
    for i in range(7, -1, -1):
        c[i] = mine_exn(b[i + 1])

    def works(p, u):
        assert mine(p, u)[1], (p, u)

    def fails(p, u):
        assert not mine(p, u)[1], (p, u)

    works(a[1], [])
    fails(a[1], [a[1]])
    fails(a[1], [a[2]])
    fails(a[1], [a[9]])
    fails(a[1], [a[9]])
    fails(a[1], [b[0]])
    for i in range(1, 7):
        works(a[1], [b[i]])
    fails(a[1], [b[7]])
    fails(a[1], [b[8]])
    works(a[1], [b[2], b[3]])
    fails(a[1], [b[2], b[2]])
    fails(a[1], [b[2], b[3], b[4]])
    for i in range(8):
        fails(a[1], [c[i]])

    # indirect double inclusion
    a9 = d.root
    a8 = mine_exn(a9)
    a7 = mine_exn(a8)
    a6 = mine_exn(a7)
    a5 = mine_exn(a6)
    a4 = mine_exn(a5)
    b4 = mine_exn(a5)
    a3 = mine_exn(a4, [b4])
    fails(a3, [b4])
    a2 = mine_exn(a3)
    fails(a2, [b4])
    a1 = mine_exn(a2)
    fails(a1, [b4])
    mine_exn(a1)


# ---------------------------------------------------------------- attack space


def test_action_table_bijection():
    # ethereum_ssz.ml:249-276: 6 actions x 4 mining rules, index = rank * 4 + own * 2 + foreign
    seen = set()
    for rank in range(6):
        for own in (0, 1):
            for foreign in (0, 1):
                seen.add(rank * 4 + own * 2 + foreign)
    assert seen == set(range(24))


def _obs(ph=0, pw=None, qh=0, qw=None, ev=0, po=0, poi=0, poe=0):
    pw = ph if pw is None else pw
    qw = qh if qw is None else qw
    # field order: public_height public_work private_height private_work diff_height
    # diff_work public_orphans private_orphans_inclusive private_orphans_exclusive event
    return [ph, pw, qh, qw, qh - ph, qw - pw, po, poi, poe, ev]


def A(rank, own, foreign):
    return rank * 4 + own * 2 + foreign


@pytest.mark.parametrize(
    "policy,obs,expect",
    [
        ("honest", _obs(ph=1), A(1, 1, 1)),
        ("honest", _obs(ph=0, qh=1), A(2, 1, 1)),
        ("selfish_release", _obs(ph=2, qh=1), A(1, 1, 0)),
        ("selfish_discard", _obs(ph=2, qh=1), A(0, 1, 0)),
        ("selfish_release", _obs(ph=0, qh=0), A(5, 1, 0)),
        ("selfish_release", _obs(ph=0, qh=3), A(5, 1, 0)),
        ("selfish_release", _obs(ph=1, qh=2), A(2, 1, 0)),
        ("fn19", _obs(ph=1, qh=2, ev=0), A(2, 1, 1)),
        ("fn19", _obs(ph=1, qh=3, ev=0), A(5, 1, 1)),
        ("fn19", _obs(ph=2, qh=1, ev=1), A(0, 1, 1)),
        ("fn19", _obs(ph=1, qh=1, ev=1), A(3, 1, 1)),
        ("fn19", _obs(ph=1, qh=2, ev=1), A(2, 1, 1)),
        ("fn19", _obs(ph=1, qh=4, ev=1), A(4, 1, 1)),
        ("fn19pkel", _obs(ph=2, qh=1, ev=1), A(1, 1, 0)),
        ("fn19pkel", _obs(ph=1, qh=4, ev=1), A(4, 1, 0)),
    ],
)
def test_eth_policy_spot_checks(policy, obs, expect):
    assert O.eth_policy(policy, obs) == expect


@pytest.mark.parametrize("unit", [False, True])
def test_eth_observation_round_trip(unit):
    rnd = random.Random(1)
    for _ in range(200):
        f = [rnd.randrange(0, 40) for _ in range(10)]
        f[4] = rnd.randrange(-30, 30)
        f[5] = rnd.randrange(-30, 30)
        f[9] = rnd.randrange(2)
        x = O.eth_obs_to_floats(f, unit)
        if unit:
            assert all(0.0 <= v <= 1.0 for v in x)
        assert O.eth_obs_of_floats(x, unit).tolist() == f


# ---------------------------------------------------------------- gym engine


def _cfg(**kw):
    kw.setdefault("protocol", L.PROTO_ETHEREUM)
    c, _ = device.make_config(**kw)
    return c


@pytest.mark.parametrize("policy", list(O.ETH_POLICIES))
@pytest.mark.parametrize("scheme", [L.REWARD_CONSTANT, L.REWARD_DISCOUNT])
def test_eth_gym_episode_invariants(policy, scheme):
    # every appended block passes the referee's validity check inside the oracle (it
    # raises otherwise); check the engine's accounting on top
    c = _cfg(alpha=0.35, gamma=0.5, max_steps=300, policy=O.ETH_POLICIES[policy],
             reward_scheme=scheme, unit_observation=False)
    for ep in range(4):
        env = O.EthGymEnv(c, episode=ep)
        obs = env.reset()
        done = False
        n = 0
        while not done:
            a = O.eth_policy(policy, env.fields())
            obs, r, done, info = env.step(a)
            n += 1
            assert info["episode_progress"] == info["head_work"]
            assert info["head_work"] >= info["head_height"]
        assert n == 300 and info["episode_n_activations"] == 301
        tot = info["episode_reward_attacker"] + info["episode_reward_defender"]
        # every block pays 1 + n_uncles/32 to its miner plus at most 1 per uncle
        assert tot >= info["head_height"]
        assert tot <= info["head_height"] + 2.0 * (info["head_work"] - info["head_height"])
        # dyadic rewards: multiples of 1/32
        assert (tot * 32) == int(tot * 32)


def test_eth_gym_random_actions_never_invalid():
    c = _cfg(alpha=0.4, gamma=0.75, max_steps=400, unit_observation=True)
    rnd = random.Random(5)
    for ep in range(6):
        env = O.EthGymEnv(c, episode=ep)
        env.reset()
        done = False
        while not done:
            _, _, done, _ = env.step(rnd.randrange(24))


def test_eth_gym_rejects_bad_action():
    c = _cfg(alpha=0.3, gamma=0.5, max_steps=10)
    env = O.EthGymEnv(c)
    env.reset()
    with pytest.raises(RuntimeError):
        env.step(24)


def test_eth_honest_share_close_to_alpha():
    # honest attacker on the gamma network: relative reward ~ alpha
    c = _cfg(alpha=0.3, gamma=0.5, max_steps=2000, policy=O.ETH_POLICIES["honest"],
             reward_scheme=L.REWARD_DISCOUNT)
    rec = O.run_episodes(c, 0, 16, threads=4)
    rel = rec["reward_attacker"] / (rec["reward_attacker"] + rec["reward_defender"])
    assert abs(rel.mean() - 0.3) < 0.02


def test_eth_two_agents_selfish_beats_honest_at_high_alpha():
    # withholding.tsv Ethereum rows: selfish policies gain at alpha=0.45 on two agents
    hon = O.eth_two_agents_task(0.45, "honest", 10000, scheme=1, seed=1, episode=0)
    sel = O.eth_two_agents_task(0.45, "selfish_release", 10000, scheme=1, seed=1, episode=0)
    share = lambda r: r["reward"][0] / sum(r["reward"])
    assert share(sel) > share(hon)
    assert abs(share(hon) - 0.45) < 0.05


def _eth_rows():
    import json
    import pathlib

    p = pathlib.Path(__file__).parent / "golden" / "withholding_ethereum_two_agents.json"
    return json.loads(p.read_text())["rows"]


def test_eth_withholding_rows_statistical():
    # each recorded row (data/withholding.tsv, one 10k-activation sample from an
    # unrecoverable OCaml Random state) must lie within 4 sigma of the oracle's
    # distribution over 32 keyed-stream episodes of the same task
    rows = _eth_rows()
    assert len(rows) == 35
    worst = 0.0
    for r in rows:
        scheme = L.REWARD_DISCOUNT if r["incentive_scheme"] == "discount" else L.REWARD_CONSTANT
        c, _ = device.make_config(alpha=r["alpha"], network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP,
                                  activations=r["activations"], protocol=L.PROTO_ETHEREUM,
                                  reward_scheme=scheme, policy=O.ETH_POLICIES[r["policy"]],
                                  seed=0xE7E7)
        rec = O.run_episodes(c, 0, 32, threads=8)
        for field, want in [("reward_attacker", r["reward"][0]),
                            ("reward_defender", r["reward"][1]),
                            ("progress", r["head_progress"]),
                            ("head_height", r["head_height"])]:
            x = np.asarray(rec[field], dtype=np.float64)
            if x.std() == 0:
                assert want == x[0], (r["line"], field)
                continue
            z = abs(want - x.mean()) / x.std()
            worst = max(worst, z)
            assert z < 4.0, (r["line"], r["policy"], field, z)
    assert worst > 0.5  # the comparison is not vacuous
