"""One rank of tests/test_gpu_distributed.py: the bench's multi-rank path on HIP lanes.

Started by torch.distributed.run (RANK / WORLD_SIZE / LOCAL_RANK in the environment).
Every rank runs its shard of an alpha x gamma sweep on libcpr_hip device lanes
(cpr_amd.parallel.sweep: disjoint episode ranges), all-reduces the integer summaries over
gloo (ranks share the box's one GPU; RCCL needs one GPU per rank), and rank 0 writes the
totals as JSON to argv[1].
"""

import json
import sys

from cpr_amd import device, parallel

POINTS = [(0.33, 0.5), (0.45, 0.0), (0.25, 0.9)]
EPISODES = 6000
STEPS = 2016


def main(out):
    rank, ws, _ = parallel.init("gloo")
    ctx = device.Context(0)
    local = parallel.sweep(POINTS, EPISODES, rank=rank, world_size=ws, ctx=ctx, steps=STEPS)
    totals = {f"{a},{g}": parallel.allreduce_summary(local[(a, g)]).to_array().tolist()
              for a, g in POINTS}
    lo, hi = parallel.shard(EPISODES, rank, ws)
    shards = [None] * ws
    import torch.distributed as dist

    dist.all_gather_object(shards, (lo, hi))
    if rank == 0:
        json.dump({"world_size": ws, "totals": totals, "shards": shards}, open(out, "w"))
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
