"""Two HIP ranks through the multi-GPU path on the box's one GPU.

Each rank is its own process with its own libcpr_hip context on the GPU; the episode range
is sharded across ranks and the integer summaries are all-reduced once (gloo here: RCCL
needs one GPU per rank, and the round-end 8-GPU bench runs the same code over RCCL). The
all-reduced totals must equal one process running the whole range bit for bit, and
bench.py's own multi-rank path (barrier, max-over-ranks time, summary all-reduce) must
print its JSON line with n_gpus = 2 and the whole-job episode count.
"""

import json
import os
import subprocess
import sys

import pytest

from cpr_amd import device, parallel

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _launch(args, port, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port)] + args
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_two_ranks_allreduce_equals_one_process(tmp_path):
    sys.path.insert(0, HERE)
    import dist_gpu_worker as W

    out = tmp_path / "totals.json"
    p = _launch([os.path.join(HERE, "dist_gpu_worker.py"), str(out)], 29600 + os.getpid() % 200)
    assert p.returncode == 0, p.stderr[-4000:]
    got = json.load(open(out))
    assert got["world_size"] == 2
    assert got["shards"] == [[0, W.EPISODES // 2], [W.EPISODES // 2, W.EPISODES]]
    ctx = device.Context(0)
    try:
        whole = parallel.sweep(W.POINTS, W.EPISODES, ctx=ctx, steps=W.STEPS)
    finally:
        ctx.close()
    for a, g in W.POINTS:
        ref = whole[(a, g)].to_array().tolist()
        assert got["totals"][f"{a},{g}"] == ref, (a, g)
        assert whole[(a, g)].episodes == W.EPISODES


def test_bench_two_ranks_gloo():
    p = _launch([os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                 "--episodes", "8192", "--no-cpu", "--backend", "gloo"],
                29800 + os.getpid() % 200)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2
    # 20 sweep points x 8192 episodes per rank x 2 ranks x 2 timed steps
    assert round(d["episodes_per_s"] * d["ms_per_step"] * d["steps"] / 1e3) == 20 * 8192 * 2 * 2
    assert d["value"] > 0 and "gloo" in d["config"]["parallelism"]


def test_bench_starts_two_ranks_itself():
    # no torchrun: `bench.py --gpus 2` starts its two ranks itself (both on the box's one
    # GPU under gloo) and reports the whole job
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    # reports the whole job, with rank 0's bounded CPU baseline (measured after the timed
    # region) in the N-GPU line too
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
                        "2", "--warmup", "1", "--episodes", "8192", "--cpu-seconds", "2",
                        "--backend", "gloo"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert round(d["episodes_per_s"] * d["ms_per_step"] * d["steps"] / 1e3) == 20 * 8192 * 2 * 2
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
    assert "other_configs" not in d  # GPU work beyond the headline stays at N = 1
    # every rank's clock, kernel time, activations and re-runs (round-5 verdict item 7)
    pr = d["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1]
    assert all(r["wall_s"] > 0 and r["kernel_ms_last_step"] > 0 for r in pr)
    assert sum(r["activations"] for r in pr) == round(d["value"] * d["ms_per_step"] * d["steps"] / 1e3)
