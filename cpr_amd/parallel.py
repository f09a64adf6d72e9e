"""Multi-GPU execution: one process per GPU, episodes sharded by index range, one RCCL
all-reduce of the integer batch summary at the end.

Episodes are independent (the reference farms them to Parany fork workers,
experiments/simulate/csv_runner.ml:105-131), so the data path has no collective; the
keyed stream makes episode e's result identical on any GPU, and the summary is integer
fixed point, so totals are bit-identical for 1/2/4/8 GPUs. Backend "nccl" is RCCL over
xGMI on ROCm; "gloo" is used for CPU tests.
"""

import os

import numpy as np

from . import _lib as L


def world():
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend="nccl"):
    import torch
    import torch.distributed as dist

    rank, ws, local = world()
    if ws > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=ws)
    return rank, ws, local


def shard(n_episodes, rank, world_size):
    """Contiguous episode range [lo, hi) of one rank."""
    lo = n_episodes * rank // world_size
    hi = n_episodes * (rank + 1) // world_size
    return lo, hi


def allreduce_summary(summary, device=None):
    """Sum a cpr_summary over all ranks (int64 vector, one collective)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return summary
    t = torch.from_numpy(summary.to_array())
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return L.Summary.from_array(t.cpu().numpy())


def allreduce_summaries(summaries, device=None):
    """Sum a list of cpr_summary over all ranks with ONE collective: the int64 vectors are
    packed into one tensor (one all-reduce of the batch summaries)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return list(summaries)
    arrs = [s.to_array() for s in summaries]
    t = torch.from_numpy(np.concatenate(arrs))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    flat = t.cpu().numpy()
    out, o = [], 0
    for a in arrs:
        out.append(L.Summary.from_array(flat[o:o + len(a)].copy()))
        o += len(a)
    return out


def barrier(device=None):
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        if device is not None:
            dist.barrier(device_ids=[device.index] if device.index is not None else None)
        else:
            dist.barrier()


def allreduce_max(x, device=None):
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(row, device=None):
    """Every rank's row of floats (same length everywhere), in rank order: one all_gather
    of a small f64 tensor (bench.py's per-rank diagnostics). One rank: [row]."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [list(map(float, row))]
    t = torch.tensor([float(x) for x in row], dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def sweep(points, episodes_per_point, first_episode=0, rank=0, world_size=1, ctx=None,
          steps=2016, policy=L.POLICY_SAPIRSHTEIN_2016_SM1, seed=0x5EED0000, records=False):
    """Run an alpha x gamma sweep; this rank runs its shard of every point.

    points: [(alpha, gamma)]. Returns {point: Summary (local shard)} and, if records,
    {point: record array}.
    """
    from . import device

    out, recs = {}, {}
    lo, hi = shard(episodes_per_point, rank, world_size)
    for alpha, gamma in points:
        cfg, keep = device.make_config(alpha=alpha, gamma=gamma, policy=policy, max_steps=steps,
                                       seed=seed)
        b = device.Batch(cfg, ctx=ctx, keep=keep)
        if records:
            s, r = b.run(hi - lo, first_episode + lo, records=True)
            recs[(alpha, gamma)] = r
        else:
            s = b.run(hi - lo, first_episode + lo)
        out[(alpha, gamma)] = s
        b.close()
    return (out, recs) if records else out


def summary_stats(s):
    """Mean relative revenue with its standard error from an integer summary."""
    n = max(1, s.episodes)
    m = s.rel_revenue_fx / 2**32 / n
    m2 = s.rel_revenue_sq_fx / 2**32 / n
    var = max(0.0, m2 - m * m)
    return dict(episodes=int(s.episodes), mean=m, stderr=float(np.sqrt(var / n)),
                activations=int(s.activations))
