"""Exact re-runs of flagged Nakamoto episodes on the device: how many, their status bits,
and what they cost (GPU; writes to stdout)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from cpr_amd import _lib as L  # noqa: E402
from cpr_amd import device  # noqa: E402


def main():
    ctx = device.default_context()
    # latency of one re-run: every episode overlaps at a 0.05 propagation delay
    for a in (0.35, 0.5):
        for n in (1, 8, 64):
            cfg, keep = device.make_config(alpha=a, gamma=0.5, max_steps=2016, seed=1,
                                           propagation_delay=0.05)
            b = device.Batch(cfg, ctx=ctx, keep=keep)
            b.run(n, records=True)
            t = time.perf_counter()
            _, rec = b.run(n, first_episode=1000, records=True)
            dt = time.perf_counter() - t
            st = np.bitwise_or.reduce(rec["status"])
            print(f"alpha={a} n={n}: {dt * 1e3:.1f} ms, status bits {st:#x}, "
                  f"capacity {(rec['status'] & L.ST_CAPACITY != 0).sum()}", flush=True)
    # the bench's points at the gym delay
    for a in (0.35, 0.45, 0.5):
        cfg, keep = device.make_config(alpha=a, gamma=0.5, max_steps=2016, seed=0x5EED0000)
        b = device.Batch(cfg, ctx=ctx, keep=keep)
        t = time.perf_counter()
        _, rec = b.run(393216 * 3, records=True)
        dt = time.perf_counter() - t
        f = rec["status"][(rec["status"] & L.ST_EXACT_RERUN) != 0]
        print(f"bench point alpha={a}: {dt * 1e3:.1f} ms, reruns {len(f)}, statuses "
              f"{[hex(x) for x in f[:12]]}", flush=True)


if __name__ == "__main__":
    main()
