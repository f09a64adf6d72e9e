"""Differential fuzz of the device lane state machine against the oracle, on the CPU.

tests/native/lane_vs_oracle.cpp compiles cpr_amd/csrc/nakamoto_lane.h for the host and
runs it step by step beside the oracle's event-driven simulator on the same keyed stream:
every observation and every head (rewards, height, chain time, clock, activations,
miner) must match, for the four SSZ policies and two random-action fuzz policies over
alpha x gamma (defenders 2..42) and for Simulator.loop on the two-agents network.
(The GPU runs the same header; tests/test_gpu_parity.py checks device == oracle.)
"""

import json
import os
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parent.parent


def test_lane_matches_oracle_fuzz():
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "lane_vs_oracle"
    p = subprocess.run([str(exe), "6", "600"], capture_output=True, text=True, timeout=600)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["mismatches"] == 0 and out["hazard_mismatches"] == 0, p.stderr[-2000:]
    assert out["unresolved"] == 0
    assert out["episodes"] > 1000
    assert out["tie_rule_episodes"] > 100  # two-defender episodes run with the tie rule
    # ring, spill and replay scratch filled with garbage first (tests/native/garbage.h)
    p = subprocess.run([str(exe), "1", "400"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, GARBAGE="19"))
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0 and out["mismatches"] == 0, p.stderr[-2000:]


def test_tie_rule_equals_heap_replay():
    # the closed-form tie outcome of the d = 2 summary-only kernels (nakamoto_lane.h
    # tie_table_d2) against the heap replay over every case it covers
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    p = subprocess.run([str(ROOT / "tests" / "native" / "build" / "tie_table")],
                       capture_output=True, text=True, timeout=120)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["mismatches"] == 0 and out["cases"] == 320 and 0 < out["on_top"] < 320


def test_deferred_races_equal_eager():
    # tests/native/defer_vs_eager.cpp: the d = 2 summary-only kernel's deferred races (listed
    # per wave, verified in batches across the wave's lanes) end every episode in the eager
    # closed form's state, word for word (one lane, and emulated waves whose lanes share the
    # list), unless the verification flagged the episode for the eager second pass (a race
    # the release did not win, or a tie the closed-form rule decides otherwise); the
    # configurations make such races and same-instant ties common so every path runs
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    p = subprocess.run([str(ROOT / "tests" / "native" / "build" / "defer_vs_eager"), "60", "600"],
                       capture_output=True, text=True, timeout=300)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["mismatches"] == 0 and out["episodes"] == 4800
    assert out["redo_flags"] > 1000 and out["redo_episodes"] > 100 and out["drains"] > 10000
    assert out["ties_kept"] > 100 and out["tie_episodes"] > 100  # ties kept without a redo
    assert out["redo_episodes_release_wins"] == 0  # dmax < delta: nothing to redo
    # waves of 8 lanes sharing one list, verified across lanes on each owner's stream
    assert out["wave_mismatches"] == 0 and out["wave_episodes"] == 2560


def test_lazy_clock_equals_eager():
    # tests/native/lazy_vs_eager.cpp: the gamma = 0 summary-only kernel's lazy clock
    # (NakLane LZ: no log while the uniform rules out an overlap) against the eager lane,
    # word for word after every step, status bits included; long delays make the exact
    # branch and real overlaps common, and some episodes draw a +inf clock delay
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    p = subprocess.run([str(ROOT / "tests" / "native" / "build" / "lazy_vs_eager"), "20", "400"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["mismatches"] == 0 and out["episodes"] == 3600
    assert out["lazy_branch_activations"] > 100000 and out["overlap_episodes"] > 1000
    assert out["inf_clock_episodes"] == 720
    # the gamma = .5 kernel (deferred races): the lazy run flags a superset of the eager
    # run's episodes for the second pass and otherwise ends in the same state
    assert out["tt2_mismatches"] == 0 and out["tt2_episodes"] == 2400
    assert out["tt2_lazy_redo"] >= out["tt2_eager_redo"] > 0
    assert out["tt2_overlap_episodes"] > 100 and out["tt2_tie_episodes"] > 50
    # delta / ev >= 14.8 zeroes lazy_threshold: lazy_clock_ok must refuse the lazy clock
    # (round-5 advisor finding: u_lazy - 1 wrapped and skipped every overlap check); run
    # anyway, the lazy lane misses overlaps, so the guard is what keeps it exact
    assert out["guard_failures"] == 0 and out["forced_zero_threshold_mismatches"] > 0


def test_ethereum_lane_matches_oracle_fuzz():
    # tests/native/eth_vs_oracle.cpp: cpr_amd/csrc/ethereum_lane.h (host build) vs the
    # oracle's ethereum.cpp, every step: 10 observation fields incl. the three dry-run
    # uncle selections, rewards, height, work, chain time, clock, activations, head miner;
    # 5 policies + 2 random-action fuzzers x 2 reward schemes x alpha x gamma, and
    # Simulator.loop tasks on the two-agents network; plus the lane in Nakamoto mode on
    # Simulator.loop tasks of the selfish-mining network (withholding.ml gamma-* tasks,
    # gamma 0 .. 0.9, defender delays 1e-4 and 0.05) against the oracle's oracle_sm_task;
    # and loop tasks on the exponential-delay clique (Ethereum and Nakamoto mode, 1..7
    # defenders, mean link delay 0.05 and 0.6) against the oracle's public entry
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "eth_vs_oracle"
    p = subprocess.run([str(exe), "6", "400"], capture_output=True, text=True, timeout=600)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["mismatches"] == 0, p.stderr[-2000:]
    assert out["episodes"] > 1000 and out["steps"] > 300000
    assert out["capacity"] == 0  # heap bound: d messages per block (capi.hip validate_eth)
    # from garbage-filled lane regions (tests/native/garbage.h: pooled device memory)
    p = subprocess.run([str(exe), "1", "300"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, GARBAGE="11"))
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0 and out["mismatches"] == 0, p.stderr[-2000:]


def test_bk_lane_matches_oracle_fuzz():
    # tests/native/bk_vs_oracle.cpp: cpr_amd/csrc/bk_lane.h (host build) vs the oracle's
    # bk.cpp, every step: the 8 bk_ssz observation fields, the policy action, rewards,
    # height, chain time, clock, activations, head signer and the vertex count; 4 policies
    # + a random table + 2 random-action fuzzers x 2 reward schemes x alpha x gamma, and
    # Simulator.loop tasks on the two-agents network; k = 8 and k = 3
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "bk_vs_oracle"
    for k, steps in [("8", "400"), ("3", "250")]:
        p = subprocess.run([str(exe), "4", steps, k], capture_output=True, text=True,
                           timeout=600)
        out = json.loads(p.stdout.strip().splitlines()[-1])
        assert p.returncode == 0, p.stderr[-2000:]
        assert out["mismatches"] == 0, p.stderr[-2000:]
        assert out["episodes"] > 700 and out["capacity"] == 0
    # the device kernels' LDS paths (event-heap slab, visibility window) in host buffers,
    # the lane's region filled with garbage first (tests/native/garbage.h)
    p = subprocess.run([str(exe), "2", "400", "8"], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, SLABTEST="1", GARBAGE="13"))
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0 and out["mismatches"] == 0, p.stderr[-2000:]


def test_tailstorm_lane_matches_oracle_fuzz():
    # tests/native/ts_vs_oracle.cpp: cpr_amd/csrc/ts_lane.h (host build) vs the oracle's
    # tailstorm.cpp, every step: 10 observation fields, the policy action, per-node fp64
    # rewards, height, chain time, clock, activations and vertex count; 7 policies + 2
    # random-action fuzzers x 4 reward schemes x alpha x gamma, plus Simulator.loop tasks;
    # heuristic, altruistic and optimal sub-block selection. Episodes where the reference
    # raises, or its optimal quorum would brute-force beyond the budget, must be flagged at
    # the same step by both engines.
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "ts_vs_oracle"
    for args in [("3", "400", "8", "1"), ("2", "300", "8", "0"), ("2", "300", "3", "2")]:
        p = subprocess.run([str(exe), *args], capture_output=True, text=True, timeout=600)
        out = json.loads(p.stdout.strip().splitlines()[-1])
        assert p.returncode == 0, p.stderr[-2000:]
        assert out["mismatches"] == 0, p.stderr[-2000:]
        assert out["episodes"] > 250 and out["capacity"] == 0
    # the device kernels' LDS paths (event-heap slab, visibility rows, list-record window from
    # garbage-filled buffers: the fused kernel's 8 rows, and 2 rows, which wrap every other
    # append) in host buffers
    for twin in ("8", "2"):
        p = subprocess.run([str(exe), "2", "300", "8", "1"], capture_output=True, text=True,
                           timeout=600,
                           env=dict(os.environ, SLABTEST="1", TWIN=twin, GARBAGE="17"))
        out = json.loads(p.stdout.strip().splitlines()[-1])
        assert p.returncode == 0 and out["mismatches"] == 0, p.stderr[-2000:]


def test_device_log_and_philox_match_oracle():
    # tests/native/log_vs_oracle.cpp: the device's cpr_log (branch-free fdlibm tails) and
    # Philox4x32-10 (gfx950 v_bitop3 xors) compiled for the host, bit for bit against the
    # oracle's line-by-line fdlibm and keyed blocks: 2e7 uniform inputs plus 480k inputs
    # near 1, near powers of two and subnormal
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "log_vs_oracle"
    p = subprocess.run([str(exe), "20000000"], capture_output=True, text=True, timeout=600)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["log_mismatches"] == 0 and out["philox_mismatches"] == 0
    assert out["checked"] > 20_000_000


def test_ethereum_window_lane_matches_oracle_fuzz():
    # tests/native/ethwin_vs_oracle.cpp: the Ethereum window lane (cpr_amd/csrc/eth_window.h,
    # host build) vs the oracle's event-driven ethereum.cpp, every step (10 observation
    # fields, rewards, height, work, chain time, clock, activations, head miner, done);
    # 5 policies + 2 random-action fuzzers x alpha x gamma (defenders per the gym's rule),
    # more defenders, and tie-heavy (1e-13 / 1e-12 delays: same-instant races replayed
    # through the skew heap) and overlap-heavy (0.05 / 0.01) networks, whose flagged
    # episodes stop being compared at the flag (the kernel re-runs them exactly)
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "ethwin_vs_oracle"
    p = subprocess.run([str(exe), "5", "500"], capture_output=True, text=True, timeout=600)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["mismatches"] == 0, p.stderr[-2000:]
    assert out["episodes"] > 1000 and out["steps"] > 400000
    assert out["tie_episodes"] > 20 and out["overlaps"] > 20  # both hazards exercised
    # the lane's region filled with pseudo-random bytes first (the device's pooled memory
    # holds what the previous launch left): the same outputs, so nothing reads a byte the
    # lane did not write
    p = subprocess.run([str(exe), "2", "400"], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, GARBAGE="7"))
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0 and out["mismatches"] == 0, p.stderr[-2000:]


def test_hybrid_rerun_equals_whole_episode_engine():
    # tests/native/hybrid_vs_exact.cpp: the hybrid exact re-run (cpr_amd/csrc/nak_hybrid.h:
    # the closed-form lane, the event engine from the last quiescent trivial point before a
    # flagged window to the first one after it) against the whole episode on the event
    # engine in Nakamoto mode (the re-run it replaces), host builds on the same keyed
    # stream: rewards, height, chain time, head miner, steps, activations, sim time and the
    # engine's status for 5 alphas x 3 gammas x 4 propagation delays (up to 0.3, where most
    # windows overlap) x 5 policies (a random table among them)
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "hybrid_vs_exact"
    p = subprocess.run([str(exe), "8", "2016"], capture_output=True, text=True, timeout=600)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["mismatches"] == 0, p.stderr[-2000:]
    assert out["episodes"] == 2400 and out["activations"] > 4_000_000
    # both directions exercised many times: the engine entered and left again
    assert out["entered"] > 1000 and out["entries"] > 50_000 and out["ended_closed"] > 1000
    # the re-run kernel's layout (hring apart, the engine's rest in the LDS-sized buffer with
    # the heap reduced where it does not fit, summary-only and records runs) gives the same
    # outputs, and no region is written past its end (canary tails)
    assert out["layout_mismatches"] == 0 and out["canary_hits"] == 0
    assert out["split_configs"] == 300 and out["reduced_heap_configs"] > 0
    # and under host AddressSanitizer + UBSan (round-5 verdict: the re-run fault study), its
    # regions filled with garbage first (tests/native/garbage.h)
    p = subprocess.run([str(exe) + "_asan", "1", "2016"], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, GARBAGE="23"))
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["mismatches"] == 0 and out["canary_hits"] == 0 and out["episodes"] == 300


def test_optimal_quorum_pruned_search_equals_literal():
    # Tailstorm's optimal sub-block selection (tailstorm.ml:418-507): both engines enumerate
    # the reference's k-subsets in its lexicographic order but skip prefixes that cannot be
    # connected or cannot beat the best reward so far. OPTCHECK makes the oracle recompute
    # every selection with the reference's literal enumeration (here up to 3e7 choices) and
    # compare, while tests/native/ts_vs_oracle.cpp compares the lane with the oracle step by
    # step: (1) the random-attacker exp-clique case of tests/test_gpu_expclique.py (seed 9,
    # constant rewards, 1000 activations; its large searches used to exceed the old 1e5
    # budget in ~1 % of episodes), (2) gym episodes with optimal selection
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "ts_vs_oracle"
    env = dict(os.environ, OPTCHECK="30000000", TSCASE="2,10,0,100,1.0,1000,9,0,256")
    p = subprocess.run([str(exe), "1", "1", "8", "2"], capture_output=True, text=True,
                       timeout=600, env=env)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["mismatches"] == 0 and out["capacity"] == 0 and out["episodes"] == 256
    assert out["opt_mismatches"] == 0 and out["opt_unverified"] == 0
    assert out["opt_compared"] > 100_000 and out["opt_large"] > 0
    env = dict(os.environ, OPTCHECK="30000000")
    p = subprocess.run([str(exe), "2", "300", "8", "2"], capture_output=True, text=True,
                       timeout=600, env=env)
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert p.returncode == 0, p.stderr[-2000:]
    assert out["mismatches"] == 0 and out["budget"] == 0
    assert out["opt_mismatches"] == 0 and out["opt_compared"] > 100_000


def test_tailstorm_optimal_budget_flags_same_searches():
    # round-5 advisor finding: the oracle's pruned search counted prefixes that cannot reach
    # k positions (i <= n - 1) while ts_lane.h counts only i <= n - (k - j), so a search near
    # the budget could flag in one engine only. Both now count the same prefixes; with the
    # budget lowered to 10 / 20 / 40 visits in both (OPTBUDGET) many searches run out of it,
    # and every episode must be flagged by both engines or by neither (the old count
    # disagreed on 34 / 25 / 5 episodes of this run)
    subprocess.run(["make", "-s", "-C", str(ROOT / "tests" / "native")], check=True)
    exe = ROOT / "tests" / "native" / "build" / "ts_vs_oracle"
    for budget, least in [("10", 100), ("20", 40), ("40", 1)]:
        p = subprocess.run([str(exe), "1", "200", "8", "2"], capture_output=True, text=True,
                           timeout=600, env=dict(os.environ, OPTBUDGET=budget))
        out = json.loads(p.stdout.strip().splitlines()[-1])
        assert p.returncode == 0, p.stderr[-2000:]
        assert out["mismatches"] == 0 and out["budget"] >= least, out
