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


# ---------------------------------------------------------------- BASELINE configs[0, 2-4]
CONFIG0_EPISODES = 1 << 20  # >= 10^6 episodes
CONFIG2_ALPHAS = (0.35, 0.45)
# build-defined VALU cost model per activation
OPS_BY_PROTOCOL = {"nakamoto": 40, "ethereum": 60, "bk": 80, "tailstorm": 120}


def other_config_specs():
    """The other BASELINE.json configs, each as (key, description, protocol, kernel, [points],
    episodes per point (None = the kernel's resident lanes), rollout steps or None).
    A point is a device.make_config keyword dict."""
    from cpr_amd import _lib as L

    specs = [(
        "configs[0]", "Nakamoto honest, alpha .33, gamma .5 (d = 2), 2016-step cpr-nakamoto-v0 "
        "episodes (the reference's CPU-runnable case)", "nakamoto", "k_run_episodes",
        [dict(alpha=0.33, gamma=0.5, policy=L.POLICY_HONEST, max_steps=STEPS_PER_EPISODE)],
        CONFIG0_EPISODES, None)]
    # configs[2]: Ethereum Byzantium, whitepaper (constant) uncle rewards, ethereum_ssz
    # selfish_release and fn19 over alpha x gamma, 2016-step gym episodes (the window lane,
    # eth_window.h; one launch of the resident lanes per point)
    eth = [dict(protocol=L.PROTO_ETHEREUM, alpha=a, gamma=g, policy=pol,
                reward_scheme=L.REWARD_CONSTANT, max_steps=STEPS_PER_EPISODE)
           for pol in (L.ETH_POLICY_SELFISH_RELEASE, L.ETH_POLICY_FN19)
           for a in CONFIG2_ALPHAS for g in (0.0, 0.5, 0.9)]
    specs.append(("configs[2]", "Ethereum-PoW uncle-aware selfish mining, Byzantium + whitepaper "
                  "(constant) uncle rewards, ethereum_ssz selfish_release and fn19 (Feng & Niu "
                  "'19), alpha {.35, .45} x gamma {0, .5, .9}, 2016-step gym episodes",
                  "ethereum", "k_eth_win_episodes", eth, None, None))
    # configs[3]: Tailstorm k = 8, discount, heuristic sub-block selection, withholding
    # attack on the two-agents network (Simulator.loop tasks of 10^4 activations,
    # withholding.ml:68-90), get-ahead and avoid-loss; the exp(1)-propagation variant apart
    ts = dict(protocol=L.PROTO_TAILSTORM, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP,
              activations=10000, k=8, reward_scheme=L.REWARD_DISCOUNT,
              subblock_selection=L.SELECT_HEURISTIC)
    specs.append(("configs[3]", "Tailstorm k=8, discount rewards, heuristic quorums, get-ahead "
                  "and avoid-loss withholding, two-agents network (alpha .33), 10^4-activation "
                  "Simulator.loop tasks", "tailstorm", "k_ts_run_episodes",
                  [dict(ts, alpha=0.33, policy=L.TS_POLICY_GET_AHEAD),
                   dict(ts, alpha=0.33, policy=L.TS_POLICY_AVOID_LOSS)], None, None))
    specs.append(("configs[3]_exp", "the same on 2 miners of equal compute with exponential(1) "
                  "link delays (cpr_protocols.ml:478-485), activation delay 10, get-ahead",
                  "tailstorm", "k_ts_run_episodes",
                  [dict(ts, alpha=0.0, network=L.NET_EXP_CLIQUE, defenders=1,
                        activation_delay=10.0, propagation_delay=1.0,
                        policy=L.TS_POLICY_GET_AHEAD)], None, None))
    # configs[4]: 65,536 lockstep B_k k = 8 gym envs, constant rewards, table policy, 2048-step
    # episodes, VecEnv auto-reset; the rollout steps every lane 512 times
    K, D = 8, 4
    table = np.random.default_rng(0).integers(0, 8, size=D * D * (K + 1) ** 2 * 3).astype(np.uint8)
    specs.append(("configs[4]", "65,536 parallel bk_ssz gym envs (B_k k=8, constant rewards, "
                  "alpha .33, gamma .5, d = 2) stepped in lockstep by an on-device random table "
                  "policy, 2048-step episodes, VecEnv auto-reset; every step's observation, "
                  "reward and done written to device buffers [step][lane] (an RL consumer's "
                  "input)", "bk", "k_bk_rollout",
                  [dict(protocol=L.PROTO_BK, alpha=0.33, gamma=0.5, k=K, table=table,
                        reward_scheme=L.REWARD_CONSTANT, max_steps=2048, n_lanes=65536)],
                  None, 512))
    return specs


def _cpu_sample(cfg, seconds, threads, per_call):
    """oracle run_episodes on cfg for about `seconds`: activations, steps, episodes, time"""
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import oracle_py

    acts = steps = eps = i = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        rec = oracle_py.run_episodes(cfg, 3 * 10**9 + i * per_call, per_call, threads=threads)
        acts += int(rec["n_activations"].sum())
        steps += int(rec["n_steps"].sum())
        eps += per_call
        i += 1
    return acts, steps, eps, time.perf_counter() - t0


def run_other_configs(ctx, cpu_seconds, with_cpu, pmc, keys=None):
    """One launch per point at the kernel's resident lane count (configs[0]: the headline's
    episode count), timed by the library's HIP events (cpr_last_launch) and by the host
    clock around each synchronous call; roofline at the §8d cost model; measured HBM bytes
    from the committed PMC summary of the same launch (tools/profile_configs.sh); a bounded
    oracle sample of the same config on this host."""
    from cpr_amd import device

    cores, aff = _host_cores()
    out = {}
    for key, desc, proto, kernel, points, eps, roll in other_config_specs():
        if keys is not None and key not in keys:
            continue
        acts = steps = episodes = invalid = 0
        wall = kms = 0.0
        lanes_l, res_l, point_ms = [], [], []
        # per point: episodes handed to the exact re-run (Ethereum window-lane hand-backs,
        # Nakamoto overlaps) and the re-run kernels' ms, beside the point's status counts
        pt_reruns, pt_rerun_ms, pt_overlap, pt_tie = [], [], [], []
        for pt in points:
            r0 = ctx.rerun_stats()
            cfg, keep = device.make_config(seed=SEED, **pt)
            b = device.Batch(cfg, ctx=ctx, keep=keep)
            n = eps
            if n is None and roll is None:
                n = b.launch_shape()[1] * int(os.environ.get("CPR_CFG_ROUNDS", "1"))
            t0 = time.perf_counter()
            if roll is not None:
                import torch

                b.rollout(8)  # reset + a few steps, untimed
                # obs / reward / done of every step into device memory, as a VecEnv consumer
                # reads them (~5 MB per step)
                nl, ol = b.n_lanes, b.obs_len
                dev = torch.device("cuda", ctx.device)
                o_t = torch.empty((roll, nl, ol), dtype=torch.float64, device=dev)
                r_t = torch.empty((roll, nl), dtype=torch.float64, device=dev)
                d_t = torch.empty((roll, nl), dtype=torch.uint8, device=dev)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                s = b.rollout(roll, device_outputs=(o_t.data_ptr(), r_t.data_ptr(),
                                                    d_t.data_ptr()))
                out_bytes = o_t.numel() * 8 + r_t.numel() * 8 + d_t.numel()
            else:
                s = b.run(n, first_episode=0)
            wall += time.perf_counter() - t0
            ms, _ = b.last_launch()
            kms += ms
            point_ms.append(round(ms, 3))
            ln, res = b.launch_shape()
            lanes_l.append(ln)
            res_l.append(res)
            r1 = ctx.rerun_stats()
            pt_reruns.append(r1[0] - r0[0])
            pt_rerun_ms.append(round(r1[2] - r0[2], 3))
            pt_overlap.append(int(s.status_overlap))
            pt_tie.append(int(s.status_tie))
            acts += int(s.activations)
            steps += int(s.steps)
            episodes += int(s.episodes)
            invalid += int(s.invalid)
            b.close()
        ops = OPS_BY_PROTOCOL[proto]
        kact = acts / (kms / 1e3)
        ach = kact * ops / 1e12
        entry = {
            "workload": desc,
            "points": len(points),
            "activations": acts,
            "activations_per_s": acts / wall,
            "kernel_ms": kms,
            "kernel_ms_per_point": point_ms,
            "exact_reruns_per_point": pt_reruns,
            "exact_rerun_ms_per_point": pt_rerun_ms,
            "status_overlap_per_point": pt_overlap,
            "status_tie_per_point": pt_tie,
            "kernel_activations_per_s": kact,
            "lanes_per_launch": lanes_l[0],
            "resident_lanes": res_l[0],
            "lanes_over_resident": lanes_l[0] / res_l[0] if res_l[0] else None,
            # episodes whose outputs are not valid (CPR_ST_INVALID: capacity, reference
            # exception, trace miss): their work is counted, their outputs are not
            "invalid": invalid,
            "roofline": {"bound": "valu", "kernel": kernel, "achieved": ach,
                         "peak": VALU_PEAK_TOPS,
                         "unit": f"Tops/s (VALU lane-ops, {ops} ops/activation cost model)",
                         "frac": ach / VALU_PEAK_TOPS},
        }
        if roll is not None:
            entry["env_steps_per_s"] = steps / wall
            entry["env_steps"] = steps
            entry["rollout_steps_per_lane"] = roll
            entry["device_output_bytes"] = out_bytes
            entry["device_output_gb_per_s"] = out_bytes / wall / 1e9
        else:
            entry["episodes_per_s"] = episodes / wall
        t = pmc.get(key) if pmc else None
        if t and t.get("kernel") not in (None, kernel):
            t = None  # a profile of another kernel (an older build of this config)
        if t:
            entry["roofline"]["traffic"] = t["hbm_bytes_per_activation"] * acts
            entry["roofline"]["traffic_source"] = t["source"]
            entry["roofline"]["hbm_bytes_per_activation"] = t["hbm_bytes_per_activation"]
            entry["roofline"]["measured_valu_lane_ops_per_activation"] = t.get("valu_lane_ops_per_activation")
        else:
            entry["roofline"]["traffic"] = None
        if with_cpu:
            cfg, _ = device.make_config(seed=SEED, **dict(points[0], n_lanes=0))
            a, st, e, dt = _cpu_sample(cfg, cpu_seconds, cores, 2 * cores)
            entry["cpu_baseline"] = {
                "value": a / dt, "unit": "activations/s", "cores": cores, "kind": "port",
                "sample": f"{e} episodes of the first point ({dt:.1f} s on {cores} threads; "
                          f"oracle/src event-driven restatement)",
                "env_steps_per_s": st / dt}
        out[key] = entry
    return out


def config_pmc():
    """Newest committed profiles/*_config_pmc.json (tools/summarize_configs.py): per config
    key, HBM bytes and VALU lane-ops per activation of the same launches."""
    import glob

    for path in sorted(glob.glob(os.path.join(HERE, "profiles", "*_config_pmc.json")), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        for v in d.values():
            v["source"] = os.path.relpath(path, HERE)
        return d
    return {}


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
        valu = d.get("valu_lane_instr_per_activation", d.get("valu_wave_instr_per_activation"))
        return rd + wr, os.path.relpath(path, HERE), valu
    return None, None, None


def _spawn_ranks(n, argv):
    """`--gpus N` without a launcher (no WORLD_SIZE in the environment): start N fresh rank
    processes of this script, one per GPU, with the torchrun variables set, as the
    reference's batch runner forks its own workers (csv_runner.ml:105-131). The parent
    touches neither torch nor the GPU; the ranks inherit stdout, so rank 0's JSON line is
    the output. Returns the first non-zero exit status of a rank (the others are ended)."""
    import signal
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench: rank {procs.index(p)} exited with {c}; stopping the others",
                      file=sys.stderr)
                for q in live:  # the exact processes this parent started
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def launch_check(args, rank, ws):
    """--launch-check: the rank/collective skeleton of main() with no GPU work"""
    from cpr_amd import _lib as L
    from cpr_amd import parallel

    parallel.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    parallel.barrier()
    dt = parallel.allreduce_max(time.perf_counter() - t0)
    s = L.Summary()
    s.episodes = rank + 1
    tot = parallel.allreduce_summaries([s])[0]
    if rank == 0:
        print(json.dumps({"launch_check": True, "value": None, "n_gpus": ws,
                          "steps": args.steps, "ranks_summed": int(tot.episodes),
                          "max_dt_s": dt, "backend": args.backend}), flush=True)
    import torch.distributed as dist

    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    # 20 x 262,144 = a whole number of rounds of the resident grid (4 or 5 waves/SIMD on
    # 256 CUs: 262,144 or 327,680 lanes), and the driver's 20 steps make BASELINE configs[1]'s
    # 10^8 episodes per (alpha, gamma) point on every GPU
    ap.add_argument("--episodes", type=int, default=5242880, help="per GPU per sweep point")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip BASELINE configs[0], [2]-[4] (other_configs)")
    ap.add_argument("--config-cpu-seconds", type=float, default=2.0)
    ap.add_argument("--gammas", default=",".join(str(g) for g in GAMMAS),
                    help="sweep gammas (A/B runs; the headline is the default)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend (nccl = RCCL; gloo for the one-GPU multi-rank "
                         "test, tests/test_gpu_distributed.py, and the CPU launcher check)")
    ap.add_argument("--launch-check", action="store_true",
                    help="CPU check of the rank launch (tests/test_bench_host.py): start the "
                         "ranks, init the collective, time and all-reduce EMPTY steps without "
                         "touching a GPU; the line says so and has no value")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start the ranks ourselves, before anything touches a GPU
        sys.exit(_spawn_ranks(args.gpus, sys.argv[1:]))

    import torch

    from cpr_amd import _lib as L
    from cpr_amd import device, parallel

    rank, ws, local = parallel.init(args.backend)
    if ws != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} but WORLD_SIZE={ws}: every GPU is one rank "
                 f"(start with --gpus N alone, or under torchrun --nproc-per-node N)")
    import torch.distributed as dist

    if dist.is_initialized():
        ws = dist.get_world_size()
    if args.launch_check:
        return launch_check(args, rank, ws)
    # one GPU per rank; under gloo several ranks may share one GPU (rank-sharing test)
    gpu = local if args.backend == "nccl" else local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    tdev = torch.device("cuda", gpu)
    cdev = tdev if args.backend == "nccl" else None  # where collectives' tensors live
    ctx = device.Context(gpu)
    gammas = [float(g) for g in args.gammas.split(",")]
    points = [(a, g) for g in gammas for a in ALPHAS]
    # CPR_BENCH_STREAMS (A/B only): point i on context i % S, i.e. its own HIP stream
    nstreams = int(os.environ.get("CPR_BENCH_STREAMS", "1"))
    smap = os.environ.get("CPR_BENCH_STREAM_MAP", "gamma")
    ctxs = [ctx] + [device.Context(gpu) for _ in range(nstreams - 1)]
    batches = []
    for i, (a, g) in enumerate(points):
        cfg, keep = device.make_config(alpha=a, gamma=g, max_steps=STEPS_PER_EPISODE, seed=SEED)
        si = (i // len(ALPHAS)) % nstreams if smap == "gamma" else i % nstreams
        batches.append(device.Batch(cfg, ctx=ctxs[si], keep=keep))
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

    def sync_all():
        for c in ctxs:
            c.synchronize()

    def rerun_all():
        st = [c.rerun_stats() for c in ctxs]
        return tuple(sum(x[i] for x in st) for i in range(3))

    for w in range(args.warmup):
        one_step(10**6 + w, new_sums())
    sync_all()
    rr0 = rerun_all()
    sums_dev = new_sums()
    parallel.barrier(cdev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        one_step(k, sums_dev)
    sync_all()
    torch.cuda.synchronize()
    parallel.barrier(cdev)
    dt_local = time.perf_counter() - t0
    dt = parallel.allreduce_max(dt_local, cdev)
    rr1 = rerun_all()  # this rank's exact re-runs of the timed region
    sums = read(sums_dev)
    totals = parallel.allreduce_summaries(sums, cdev)  # one packed collective
    acts = sum(int(s.activations) for s in totals)
    episodes = sum(int(s.episodes) for s in totals)

    # dominant kernel = k_run_episodes; achieved from HIP events recorded by the library
    # around the last launch of every point, on the stream the kernel runs on; activations
    # per launch = E episodes x (max_steps + 1) (every gym episode is exactly that long)
    kms = np.array([b.last_launch()[0] for b in batches])
    # every rank's own clock, kernel time and re-runs (csv_runner.ml:105-131 reports each
    # worker's tasks): a 1->8 GPU series that is not linear then shows which rank was slow
    # and why; the local wall includes the barrier wait, so the slowest rank has the least
    # wait (kernel ms = the last step's launches, rerun counts = the timed region's)
    local_acts = sum(int(s.activations) for s in sums)
    rows = parallel.gather_rows([rank, dt_local, float(kms.sum()), local_acts,
                                 rr1[0] - rr0[0], rr1[2] - rr0[2], float(gpu)], cdev)

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
    atotals = parallel.allreduce_summaries(read(asums[:len(abatches)]), cdev)
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
                "episodes_per_point_timed": E * args.steps * ws,
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
                # SURVEY §8d's unit figure: 48 B of per-episode outputs; the sweep reduces
                # them on chip to one summary per launch, so `traffic` is below it
                "algorithmic_bytes_per_launch": ALG_BYTES_PER_EPISODE * E,
                "hbm_frac_algorithmic": ALG_BYTES_PER_EPISODE * E / (kms.mean() / 1e3)
                / (HBM_PEAK_GBS * 1e9),
                "kernel": "k_run_episodes",
                "kernel_ms_mean": float(kms.mean()),
                "kernel_ms_per_point": {f"{a:.2f},{g:.1f}": round(float(m), 3)
                                        for (a, g), m in zip(points, kms)},
                "kernel_activations_per_s": act_per_s_kernel,
            },
            "status": {"tie_episodes": ties, "overlap_episodes": overlaps, "other": other,
                       # rank 0's timed region: episodes re-run exactly, and those kernels'
                       # ms on the context's stream (they overlap the sweep's launches)
                       "exact_reruns_rank0": rr1[0] - rr0[0],
                       "exact_rerun_flushes_rank0": rr1[1] - rr0[1],
                       "exact_rerun_ms_rank0": round(rr1[2] - rr0[2], 3)},
            "per_rank": [{"rank": int(r[0]), "gpu": int(r[6]), "wall_s": round(r[1], 4),
                          "kernel_ms_last_step": round(r[2], 3),
                          "activations": int(r[3]),
                          "activations_per_s_local": r[3] / r[1] if r[1] > 0 else None,
                          "exact_reruns": int(r[4]), "exact_rerun_ms": round(r[5], 3)}
                         for r in rows],
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
        if not args.no_cpu:
            # host only, after every collective of the timed region: at N > 1 rank 0
            # measures the same bounded oracle sample, so every line of a 1/2/4/8-GPU series
            # carries the CPU baseline of its own job (north_star)
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, points)
        if not args.no_configs and ws == 1:
            # the other BASELINE configs on this GPU, after the headline's timed region
            out["other_configs"] = run_other_configs(ctx, args.config_cpu_seconds,
                                                     not args.no_cpu, config_pmc())
        print(json.dumps(out), flush=True)
    for b in batches + abatches:
        b.close()
    for c in ctxs:
        c.close()
    if ws > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
