"""Pin the CPU oracle to the reference's own known-answer data (no GPU needed).

* data/withholding.tsv: all 28 two-agents Nakamoto rows (4 SSZ policies x 7 alphas,
  10,000 activations, OCaml Random carried over between tasks) — rewards per node,
  activations per node, head time (12 significant digits as written by
  string_of_float) and head progress must match exactly.
* ssz_tools.ml:82-228 observation-encoding expect tests (unit and raw).
* Philox4x32-10 known-answer vectors (Random123 kat_vectors) for the keyed stream.
"""

import json
import math
import pathlib
import struct

import numpy as np
import pytest

import oracle_py as O

GOLD = pathlib.Path(__file__).parent / "golden"


def _fixture():
    return json.loads((GOLD / "withholding_nakamoto_two_agents.json").read_text())["rows"]


@pytest.mark.parametrize("row", _fixture(), ids=lambda r: f"tsv{r['line']}")
def test_withholding_two_agents_rows(row):
    rng = O.OcamlRandom()  # OCaml's unseeded default state (full_init [|27182818|])
    for _ in range(row["prior_tasks"]):  # earlier tasks of the same Parany worker
        O.two_agents_task(0.25, "honest", row["activations"], rng=rng)
    out = O.two_agents_task(row["alpha"], row["policy"], row["activations"], rng=rng)
    assert out["activations"] == row["activations_per_node"]
    assert out["reward"] == row["reward"]
    assert "%.12g" % out["head_time"] == row["head_time"]
    assert out["head_progress"] == row["head_progress"]


def test_withholding_fixture_covers_all_rows():
    rows = _fixture()
    assert len(rows) == 28
    assert {r["policy"] for r in rows} == set(O.POLICIES)


def test_ocaml_random_int_and_float_ranges():
    r = O.OcamlRandom(42)
    xs = [r.int(7) for _ in range(2000)]
    assert min(xs) == 0 and max(xs) == 6
    fs = [r.float(1.0) for _ in range(2000)]
    assert 0.0 <= min(fs) and max(fs) < 1.0
    assert 0.45 < np.mean(fs) < 0.55


# ssz_tools.ml:101-152 (unit) and :175-226 (raw), scale 1 as used by nakamoto_ssz.ml:35-38
@pytest.mark.parametrize(
    "fields,unit,expect",
    [
        ([0, 0, 0, 0], True, [0.0, 0.0, 0.5, 0.0]),
        ([1, 1, 1, 1], True, [0.5, 0.5, 0.75, 1.0]),
        ([0, 0, -1, 0], True, [0.0, 0.0, 0.25, 0.0]),
        ([0, 42, -42, 1], False, [0.0, 42.0, -42.0, 1.0]),
        ([1, 0, 1, 0], False, [1.0, 0.0, 1.0, 0.0]),
    ],
)
def test_observation_encoding_kats(fields, unit, expect):
    assert O.obs_to_floats(fields, unit).tolist() == expect


def test_observation_encoding_max_int():
    big = 2**31 - 1
    f = O.obs_to_floats([big, big, big, 1], True)
    assert f[0] == pytest.approx(1.0, abs=1e-9) and f[2] == pytest.approx(1.0, abs=1e-9)
    f = O.obs_to_floats([0, 0, -big, 0], True)
    assert f[2] == pytest.approx(0.0, abs=1e-9)


@pytest.mark.parametrize("x", [0, 1, 2, 256])
@pytest.mark.parametrize("unit", [True, False])
def test_observation_round_trip(x, unit):
    for signed in (x, -x):
        fields = [x, x, signed, 1]
        back = O.obs_of_floats(O.obs_to_floats(fields, unit), unit)
        assert back.tolist() == fields


# Random123 kat_vectors, philox4x32 10 rounds
@pytest.mark.parametrize(
    "ctr,key,out",
    [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        (
            [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
            [0xA4093822, 0x299F31D0],
            [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1],
        ),
    ],
)
def test_philox_kat(ctr, key, out):
    assert O.philox(ctr, key).tolist() == out


def _ulp_diff(a, b):
    ia = struct.unpack("<q", struct.pack("<d", a))[0]
    ib = struct.unpack("<q", struct.pack("<d", b))[0]
    return abs(ia - ib)


def test_cpr_log_accuracy():
    # keyed stream v2 table log (oracle/src/keyed_stream.h) against the exactly rounded
    # natural log (50-digit decimal): within 2 ulp, correctly rounded for most inputs
    import decimal

    decimal.getcontext().prec = 50
    rng = np.random.default_rng(7)
    us = np.concatenate([rng.random(20000), [2.0**-53, 0.5, 1 - 2.0**-53, 0.999999, 1e-300]])
    d = [_ulp_diff(O.cpr_log(float(u)), float(decimal.Decimal(float(u)).ln())) for u in us]
    assert max(d) <= 2
    assert sum(x == 0 for x in d) > 0.6 * len(d)
    assert O.cpr_log(0.0) == -math.inf
    assert O.cpr_log(1.0) == 0.0


def test_u53_grid():
    assert O.u53(0, 0) == 0.0
    assert O.u53(0xFFFFFFFF, 0xFFFFFFFF) == 1.0 - 2.0**-53


def test_keyed_stream_is_order_free():
    a = O.keyed_block(1, 2, 3, 0)
    b = O.keyed_block(1, 2, 4, 0)
    assert a.tolist() == O.keyed_block(1, 2, 3, 0).tolist()
    assert a.tolist() != b.tolist()


# nakamoto_ssz.ml:274-340 spot checks (policy table of the reference)
@pytest.mark.parametrize(
    "policy,h,a,act",
    [
        ("sapirshtein-2016-sm1", 2, 1, 0),  # h > a -> Adopt
        ("sapirshtein-2016-sm1", 1, 1, 2),  # (1,1) -> Match
        ("sapirshtein-2016-sm1", 1, 2, 1),  # h = a - 1, h >= 1 -> Override
        ("sapirshtein-2016-sm1", 0, 3, 3),  # otherwise Wait
        ("eyal-sirer-2014", 2, 5, 2),  # lead > 2 -> Match
        ("eyal-sirer-2014", 3, 4, 1),  # lead 1 after h > 0 -> Override
        ("honest", 0, 1, 1),
        ("honest", 1, 0, 0),
        ("simple", 1, 3, 1),
    ],
)
def test_policy_spot_checks(policy, h, a, act):
    assert O.nak_policy(O.POLICIES[policy], [h, a, a - h, 1]) == act


def _cfg(**kw):
    from cpr_amd import device

    c, keep = device.make_config(**kw)
    return c


def test_gym_engine_smoke():
    # gym/ocaml/test/test_engine.py:4-30
    env = O.GymEnv(_cfg(alpha=0.33, gamma=0.5, defenders=2, unit_observation=False))
    env.reset()
    obs, r, done, info = env.step(0)
    assert not done
    env = O.GymEnv(_cfg(alpha=0.33, gamma=0.5, defenders=2))
    env.reset()
    for _ in range(600):
        obs, r, done, info = env.step(3)
    assert not done
    assert info["episode_n_activations"] == 601  # reset consumes activation #1


def test_gym_episode_accounting():
    env = O.GymEnv(_cfg(alpha=0.3, gamma=0.5, max_steps=100))
    env.reset()
    done = False
    n = 0
    while not done:
        f = env.fields()
        obs, r, done, info = env.step(O.nak_policy(0, f))
        n += 1
    assert n == 100 and info["episode_n_steps"] == 100 and info["episode_n_activations"] == 101
    assert info["episode_reward_attacker"] + info["episode_reward_defender"] == info["head_height"]


def test_gym_gamma_one_rejected():
    # network.ml:69-72 rejects gamma > (d-1)/d
    with pytest.raises(ValueError):
        O.GymEnv(_cfg(alpha=0.3, gamma=1.0, defenders=2))
