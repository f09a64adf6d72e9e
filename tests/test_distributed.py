"""Multi-process path on the CPU (gloo, world size 2): episode sharding and the summary
all-reduce of cpr_amd.parallel give exactly the single-process totals.

Each rank summarises its shard of oracle episode records the way k_run_episodes does
(integer fixed point), then all-reduces; the result must equal the whole-range summary
bit for bit — the property that makes 1/2/4/8-GPU bench totals identical.
"""

import os

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from cpr_amd import _lib as L
from cpr_amd import device, parallel


def summarize(rec):
    s = L.Summary()
    h = rec["head_height"].astype(np.int64)
    ra = rec["reward_attacker"].astype(np.int64)
    s.episodes = len(rec)
    s.steps = int(rec["n_steps"].sum())
    s.activations = int(rec["n_activations"].sum())
    s.reward_attacker_fx = int(ra.sum()) << 20
    s.reward_defender_fx = int((h - ra).sum()) << 20
    s.progress_fx = int(h.sum()) << 20
    rel = np.where(h > 0, ra / np.maximum(h, 1), 0.0)
    s.rel_revenue_fx = int(np.rint(rel * 2**32).astype(np.uint64).sum())
    s.rel_revenue_sq_fx = int(np.rint(rel * rel * 2**32).astype(np.uint64).sum())
    s.orphans = int((rec["n_activations"] - h).sum())
    for i, c in enumerate(np.bincount(np.clip((rel * 64).astype(np.int64), 0, 63), minlength=64)):
        s.hist[i] = int(c)
    return s


N = 96


def _records():
    import oracle_py

    cfg, _ = device.make_config(alpha=0.35, gamma=0.5, max_steps=200, seed=11)
    return oracle_py.run_episodes(cfg, 0, N)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = parallel.shard(N, rank, world)
    rec = _records()[lo:hi]
    tot = parallel.allreduce_summary(summarize(rec))
    q.put((rank, tot.to_array().tolist(), lo, hi))
    dist.destroy_process_group()


def test_shard_covers_range():
    for n in [1, 7, 96, 1000]:
        for w in [1, 2, 3, 8]:
            parts = [parallel.shard(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))


def test_summary_array_round_trip():
    s = L.Summary()
    s.rel_revenue_fx = (1 << 64) - 5
    s.hist[3] = 7
    t = L.Summary.from_array(s.to_array())
    assert t.rel_revenue_fx == s.rel_revenue_fx and t.hist[3] == 7


def test_gloo_world2_allreduce_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    whole = summarize(_records()).to_array().tolist()
    for rank, arr, lo, hi in outs:
        assert arr == whole


# bench.py's episode bases: step k of rank r runs episodes [(k * ws + r) * E, + E) of every
# sweep point, and the summaries of all points go through ONE packed all-reduce
# (parallel.allreduce_summaries). Over K steps the ranks together cover [0, K * ws * E)
# exactly once, so the all-reduced totals must equal one process's summary of that range,
# bit for bit, at any world size.
E_BENCH, K_BENCH = 6, 2
BENCH_POINTS = [(0.3, 0.5), (0.45, 0.0)]


def _bench_records(point, first, n):
    import oracle_py

    cfg, _ = device.make_config(alpha=point[0], gamma=point[1], max_steps=120, seed=0x5EED0000)
    return oracle_py.run_episodes(cfg, first, n)


def _bench_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sums = []
    for pt in BENCH_POINTS:
        recs = [_bench_records(pt, (k * world + rank) * E_BENCH, E_BENCH) for k in range(K_BENCH)]
        sums.append(summarize(np.concatenate(recs)))
    tot = parallel.allreduce_summaries(sums)
    # bench.py's per_rank rows: one all_gather, every rank's row in rank order everywhere
    rows = parallel.gather_rows([rank, 10.0 * rank + 0.5, world])
    assert rows == [[float(r), 10.0 * r + 0.5, float(world)] for r in range(world)], rows
    q.put((rank, [t.to_array().tolist() for t in tot]))
    dist.destroy_process_group()


def _run_world(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + world * 7 + os.getpid() % 500
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return outs


def test_gloo_bench_bases_world4_and_world8_equal_single_process():
    for world in (4, 8):
        outs = _run_world(world)
        whole = [summarize(_bench_records(pt, 0, K_BENCH * world * E_BENCH)).to_array().tolist()
                 for pt in BENCH_POINTS]
        assert len(outs) == world
        for rank, arrs in outs:
            assert arrs == whole, (world, rank)
