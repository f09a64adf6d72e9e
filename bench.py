"""Headline benchmark: simulated block activations/s for the Nakamoto SM1 alpha x gamma
sweep of BASELINE.json configs[1], one process per GPU.

A step = one pass of the sweep: for every (alpha, gamma) point each GPU simulates its own
E gym episodes of 2016 steps (cpr-nakamoto-v0 semantics: selfish-mining network with
d = max(2, ceil(1/(1-gamma))) defenders, policy sapirshtein-2016-sm1, 2017 activations per
episode), fused into one kernel launch per point; the batch summary is integer-exact and
all-reduced once over RCCL. Weak scaling: E is per GPU.

gamma = 1 is rejected by the reference (gym/ocaml/cpr_gym/envs.py:73-75,
network.ml:69-72), so the timed sweep runs gamma in {0, 0.5}; the gamma = 1 column runs
after it, untimed for `value`, in the flagged abstract-gamma mode (CPR_NET_ABSTRACT_GAMMA,
include/cpr_hip.h) and is reported separately ("abstract_gamma_1") beside the Eyal-Sirer
closed form.

Prints one JSON line (rank 0).
"""

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

ALPHAS = [0.05, 0.10, 0.15, 0.20, 0.25, 0.30, 0.35, 0.40, 0.45, 0.50]
GAMMAS = [0.0, 0.5]
STEPS_PER_EPISODE = 2016
OPS_PER_ACTIVATION = 40  # build-defined algorithmic VALU cost
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 256 CU x 4 SIMD32 x 32 lanes/clk x 2.4 GHz
SEED = 0x5EED0000


def _host_cores():
    """Cores this process may use: the affinity mask, capped by the job's CPU share when
    the environment states one (the GPU box exports OMP_NUM_THREADS = its per-GPU share;
    nproc there counts the whole machine)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = os.environ.get("OMP_NUM_THREADS")
    cores = min(aff, int(share)) if share and share.isdigit() and int(share) > 0 else aff
    return max(1, cores), aff


def es14(alpha, gamma):
    """Eyal & Sirer (FC'14) relative revenue of selfish mining (alpha < 1/2)."""
    a, g = alpha, gamma
    return (a * (1 - a) ** 2 * (4 * a + g * (1 - 2 * a)) - a ** 3) / (1 - a * (1 + (2 - a) * a))


def cpu_baseline(seconds, points):
    """The CPU oracle (faithful DES restatement, oracle/src/des.cpp) on the host: one run on
    every core this job may use and one on a single core, each a bounded sample of the
    same sweep points (all-core and single-process numbers)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
    import oracle_py
    from cpr_amd import device

    cores, aff = _host_cores()

    def sample(threads, budget, base):
        per_point = 4 * threads
        acts = eps = i = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget:
            alpha, gamma = points[i % len(points)]
            cfg, _ = device.make_config(alpha=alpha, gamma=gamma, max_steps=STEPS_PER_EPISODE,
                                        seed=SEED)
            rec = oracle_py.run_episodes(cfg, base + i * per_point, per_point, threads=threads)
            acts += int(rec["n_activations"].sum())
            eps += per_point
            i += 1
        return acts, eps, time.perf_counter() - t0

    acts, eps, dt = sample(cores, seconds * 0.6, 10**9)
    acts1, eps1, dt1 = sample(1, seconds * 0.4, 2 * 10**9)
    return {
        "value": acts / dt,
        "unit": "activations/s",
        "cores": cores,
        "kind": "port",
        "sample": f"{eps} episodes x {STEPS_PER_EPISODE} steps of the same sweep points "
                  f"({dt:.1f} s on {cores} threads; the host's affinity mask holds {aff} cores, "
                  f"the job's CPU share is {cores}; oracle/src/des.cpp event-driven DES)",
        "episodes_per_s": eps / dt,
        "single_core": {"value": acts1 / dt1, "unit": "activations/s", "cores": 1,
                        "sample": f"{eps1} episodes ({dt1:.1f} s)"},
        "affinity_cores": aff,
    }


# algorithmic HBM bytes of k_run_episodes: the Monte-Carlo outputs,
# ~48 B per episode (rewards, progress, status; the summary's share is negligible)
ALG_BYTES_PER_EPISODE = 48.0
HBM_PEAK_GBS = 8000.0


def pmc_traffic(episodes):
    """HBM bytes per k_run_episodes launch from the newest committed rocprofv3 PMC summary
    of this same bench command (tools/profile.sh -> tools/summarize_profile.py:
    FETCH_SIZE x1024 x2 gfx950 correction + WRITE_SIZE x1024), or None when no summary
    for this launch size exists."""
    import glob

    for path in sorted(glob.glob(os.path.join(HERE, "profiles", "*_pmc_summary.json")),
                       reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("kernel") != "k_run_episodes" or d.get("episodes_per_dispatch") != episodes:
            continue
        rd = d.get("hbm_read_bytes_per_dispatch (FETCH_SIZE x1024 x2, gfx950 correction)")
        wr = d.get("hbm_write_bytes_per_dispatch (WRITE_SIZE x1024)")
        if rd is None or wr is None:
            continue
        return rd + wr, os.path.relpath(path, HERE), d.get("valu_wave_instr_per_activation")
    return None, None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--episodes", type=int, default=393216, help="per GPU per sweep point")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend (nccl = RCCL; gloo only for the one-GPU "
                         "multi-rank test, tests/test_gpu_distributed.py)")
    args = ap.parse_args()

    import torch

    from cpr_amd import _lib as L
    from cpr_amd import device, parallel

    rank, ws, local = parallel.init(args.backend)
    if ws != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
    # one GPU per rank; under gloo several ranks may share one GPU (rank-sharing test)
    gpu = local if args.backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    tdev = torch.device("cuda", gpu)
    cdev = tdev if args.backend == "nccl" else None  # where collectives' tensors live
    ctx = device.Context(gpu)
    points = [(a, g) for g in GAMMAS for a in ALPHAS]
    batches = []
    for a, g in points:
        cfg, keep = device.make_config(alpha=a, gamma=g, max_steps=STEPS_PER_EPISODE, seed=SEED)
        batches.append(device.Batch(cfg, ctx=ctx, keep=keep))
    E = args.episodes
    sbytes = ctypes.sizeof(L.Summary)

    def one_step(step_idx, sums_dev):
        # every point's episodes submitted asynchronously on the library's streams (the
        # flagged-episode re-runs go to its second stream); summaries accumulate on the
        # device and are read after the synchronize that closes the timed region
        base = (step_idx * ws + rank) * E  # disjoint episode ids per rank and step
        for b, sd in zip(batches, sums_dev):
            b.run_async(E, base, sd.data_ptr())

    def read(sums_dev):
        return [L.Summary.from_buffer_copy(sd.cpu().numpy().tobytes()) for sd in sums_dev]

    def new_sums():
        return [torch.zeros(sbytes // 8, dtype=torch.int64, device=tdev) for _ in points]

    for w in range(args.warmup):
        one_step(10**6 + w, new_sums())
    ctx.synchronize()
    sums_dev = new_sums()
    parallel.barrier(cdev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(k, sums_dev)
    ctx.synchronize()
    torch.cuda.synchronize()
    parallel.barrier(cdev)
    dt = parallel.allreduce_max(time.perf_counter() - t0, cdev)
    sums = read(sums_dev)
    totals = [parallel.allreduce_summary(s, cdev) for s in sums]
    acts = sum(int(s.activations) for s in totals)
    episodes = sum(int(s.episodes) for s in totals)

    # dominant kernel = k_run_episodes; achieved from HIP events recorded by the library
    # around the last launch of every point, on the stream the kernel runs on; activations
    # per launch = E episodes x (max_steps + 1) (every gym episode is exactly that long)
    kms = np.array([b.last_launch()[0] for b in batches])

    # configs[1]'s gamma = 1 column in the flagged abstract-gamma mode, after the timed
    # region: same kernel, zero delays, match races decided by gamma coins; its own clock
    abatches = []
    for a in ALPHAS:
        cfg, keep = device.make_config(alpha=a, gamma=1.0, network=L.NET_ABSTRACT_GAMMA,
                                       defenders=2, max_steps=STEPS_PER_EPISODE, seed=SEED)
        abatches.append(device.Batch(cfg, ctx=ctx, keep=keep))
    asums = new_sums()
    parallel.barrier(cdev)
    torch.cuda.synchronize()
    ta = time.perf_counter()
    for b, sd in zip(abatches, asums):
        b.run_async(E, rank * E, sd.data_ptr())
    ctx.synchronize()
    torch.cuda.synchronize()
    parallel.barrier(cdev)
    dta = parallel.allreduce_max(time.perf_counter() - ta, cdev)
    atotals = [parallel.allreduce_summary(s, cdev) for s in read(asums[:len(abatches)])]
    traffic, traffic_src, valu_meas = pmc_traffic(E)
    kacts = np.full(len(batches), float(E * (STEPS_PER_EPISODE + 1)))
    act_per_s_kernel = float(kacts.sum() / (kms.sum() / 1e3))
    achieved = act_per_s_kernel * OPS_PER_ACTIVATION / 1e12
    if rank == 0:
        sweep = {}
        for (a, g), s in zip(points, totals):
            st = parallel.summary_stats(s)
            sweep[f"{a:.2f},{g:.1f}"] = [round(st["mean"], 6), round(st["stderr"], 6)]
        ties = sum(int(s.status_tie) for s in totals)
        overlaps = sum(int(s.status_overlap) for s in totals)
        other = sum(int(s.status_other) for s in totals)
        out = {
            "metric": "simulated block activations/sec (whole node) at 1/2/4/8 MI355X; episodes/sec",
            "value": acts / dt,
            "unit": "activations/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32 state machine + f64 event times",
            "data": "synthetic: keyed Philox4x32-10 stream (DESIGN.md §3), seed 0x5eed0000",
            "config": {
                "workload": "BASELINE configs[1]: Nakamoto SM1 (sapirshtein-2016-sm1) selfish "
                            "mining, alpha 0.05..0.50 x gamma {0, 0.5} (gamma=1 is rejected by "
                            "the reference), 2016-step cpr-nakamoto-v0 episodes",
                "episodes_per_point_per_gpu": E,
                "points": len(points),
                "activations_per_episode": STEPS_PER_EPISODE + 1,
                "parallelism": f"dp{ws} (episode shards, 1 {'RCCL' if args.backend == 'nccl' else 'gloo'} "
                               f"all-reduce of the summary)",
            },
            "episodes_per_s": episodes / dt,
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": VALU_PEAK_TOPS,
                "unit": "Tops/s (VALU lane-ops, 40 ops/activation cost model)",
                "frac": achieved / VALU_PEAK_TOPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                # SQ_INSTS_VALU x 64 / activations from the same PMC summary: the VALU
                # lane-instructions the kernel really issues per activation, beside the
                # 40-op cost model `achieved` is priced at
                "measured_valu_lane_ops_per_activation": valu_meas,
                "algorithmic_bytes_per_launch": ALG_BYTES_PER_EPISODE * E,
                "hbm_frac_algorithmic": ALG_BYTES_PER_EPISODE * E / (kms.mean() / 1e3)
                / (HBM_PEAK_GBS * 1e9),
                "kernel": "k_run_episodes",
                "kernel_ms_mean": float(kms.mean()),
                "kernel_activations_per_s": act_per_s_kernel,
            },
            "status": {"tie_episodes": ties, "overlap_episodes": overlaps, "other": other},
            "sweep_mean_rel_revenue": sweep,
            "abstract_gamma_1": {
                "mode": "FLAGGED abstract-gamma (CPR_NET_ABSTRACT_GAMMA): not the reference's "
                        "network, which rejects gamma = 1; zero delays, 2 defenders, a match "
                        "race goes to the attacker's release at every defender (coin < 1)",
                "activations_per_s": sum(int(s.activations) for s in atotals) / dta,
                "episodes_per_point": E * ws,
                "mean_rel_revenue_vs_es14": {
                    f"{a:.2f}": [round(parallel.summary_stats(s)["mean"], 6),
                                 round(parallel.summary_stats(s)["stderr"], 6),
                                 round(es14(a, 1.0), 6) if a < 0.5 else None]
                    for a, s in zip(ALPHAS, atotals)},
                "invalid_episodes": sum(int(s.invalid) for s in atotals),
            },
        }
        if not args.no_cpu and ws == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, points)
        print(json.dumps(out), flush=True)
    for b in batches + abatches:
        b.close()
    ctx.close()
    if ws > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
