"""Host-side checks of bench.py's contract (no GPU): the headline workload is BASELINE
configs[1] at its stated size, the other configs are BASELINE's, the committed profiles the
line reads its measured traffic from parse, and the closed form it prints beside the
abstract-gamma column is Eyal and Sirer's."""

import json
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_headline_is_configs1_at_its_stated_size():
    # 20 whole rounds of the 262,144-lane resident grid per point, and the driver's 20 steps
    # make BASELINE's 10^8 episodes per (alpha, gamma) point
    src = (ROOT / "bench.py").read_text()
    assert "default=5242880" in src
    assert 5242880 % 262144 == 0 and 5242880 * 20 >= 10**8
    assert bench.ALPHAS[0] == 0.05 and bench.ALPHAS[-1] == 0.50 and len(bench.ALPHAS) == 10
    assert bench.GAMMAS == [0.0, 0.5]  # gamma = 1 runs apart, in the flagged abstract mode
    assert bench.STEPS_PER_EPISODE == 2016


def test_other_configs_cover_baseline():
    specs = bench.other_config_specs()
    keys = [s[0] for s in specs]
    assert keys == ["configs[0]", "configs[2]", "configs[3]", "configs[3]_exp", "configs[4]"]
    by = {s[0]: s for s in specs}
    from cpr_amd import _lib as L

    # configs[2]: Ethereum with whitepaper (constant) uncle rewards, selfish_release and
    # fn19 over alpha x gamma
    pts = by["configs[2]"][4]
    assert {p["protocol"] for p in pts} == {L.PROTO_ETHEREUM}
    assert {p["reward_scheme"] for p in pts} == {L.REWARD_CONSTANT}
    assert sorted({p["gamma"] for p in pts}) == [0.0, 0.5, 0.9]
    assert {p["policy"] for p in pts} == {L.ETH_POLICY_SELFISH_RELEASE, L.ETH_POLICY_FN19}
    assert len({p["alpha"] for p in pts}) >= 2 and len(pts) == 12
    # configs[0]: at least 10^6 episodes
    assert by["configs[0]"][5] >= 10**6
    # configs[3]: Tailstorm k = 8, discount, withholding (two attack policies), 10^4 activations
    for p in by["configs[3]"][4] + by["configs[3]_exp"][4]:
        assert p["protocol"] == L.PROTO_TAILSTORM and p["k"] == 8
        assert p["reward_scheme"] == L.REWARD_DISCOUNT and p["activations"] == 10000
    assert by["configs[3]_exp"][4][0]["network"] == L.NET_EXP_CLIQUE
    # configs[4]: 65,536 lockstep B_k k = 8 envs with a table policy
    (p4,) = by["configs[4]"][4]
    assert p4["protocol"] == L.PROTO_BK and p4["k"] == 8 and p4["n_lanes"] == 65536
    assert p4["table"] is not None and by["configs[4]"][6] > 0


def test_committed_profiles_parse():
    pmc = bench.config_pmc()
    assert set(pmc) >= {"configs[0]", "configs[2]", "configs[3]", "configs[3]_exp", "configs[4]"}
    for v in pmc.values():
        assert v["hbm_bytes_per_activation"] > 0 and v["source"].startswith("profiles/")
    traffic, src, valu = bench.pmc_traffic(5242880)
    assert traffic and traffic > 0 and src.startswith("profiles/") and 100 < valu < 400


@pytest.mark.parametrize("alpha,gamma,want", [(1 / 3, 0.5, 0.384615), (0.25, 0.95, 0.2994),
                                              (0.25, 1.0, 0.3049)])
def test_eyal_sirer_closed_form(alpha, gamma, want):
    assert bench.es14(alpha, gamma) == pytest.approx(want, abs=1e-4)


def test_driver_record_shape():
    # the last driver record of the previous round has the fields the contract asks for
    recs = sorted(ROOT.glob("BENCH_r*.json"))
    if not recs:
        pytest.skip("no driver record yet")
    d = json.loads(recs[-1].read_text())
    line = d.get("parsed") or {}
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "roofline", "cpu_baseline", "config"):
        assert k in line, k


def _bench_cmd(args, env_drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")):
    import os
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in env_drop}
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, cwd=str(ROOT),
                          env=env, capture_output=True, text=True, timeout=300)


def test_bench_starts_its_own_ranks():
    # `bench.py --gpus 4` with no torchrun around it starts 4 rank processes itself (before
    # anything touches a GPU); the collective sees all of them and rank 0 alone prints
    p = _bench_cmd(["--gpus", "4", "--backend", "gloo", "--launch-check", "--steps", "3"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["ranks_summed"] == 1 + 2 + 3 + 4 and d["value"] is None


def test_bench_rejects_a_world_size_other_than_gpus():
    # under a launcher whose WORLD_SIZE disagrees with --gpus the bench stops (it used to
    # warn and time one rank)
    import os
    import subprocess

    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--backend",
                        "gloo", "--launch-check"], cwd=str(ROOT), env=env, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr
