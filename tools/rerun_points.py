"""Exact re-runs per bench sweep point (GPU diagnostic, not a test): for a few alpha x gamma
points of bench.py's sweep, how many episodes of one launch the library re-ran exactly and
what the launch plus its re-run launch cost (one synchronous run each).
"""
import sys, time
sys.path.insert(0, ".")
import numpy as np
from cpr_amd import _lib as L, device
ctx = device.default_context()
E = 393216
for g in (0.0, 0.5):
    for a in (0.05, 0.25, 0.45, 0.5):
        cfg, keep = device.make_config(alpha=a, gamma=g, max_steps=2016, seed=0x5eed0000)
        b = device.Batch(cfg, ctx=ctx, keep=keep)
        b.run(4096)
        t = time.perf_counter(); s, rec = b.run(E, first_episode=0, records=True); dt = time.perf_counter() - t
        n = int(((rec["status"] & L.ST_EXACT_RERUN) != 0).sum())
        print(f"gamma {g} alpha {a}: reruns {n}, run+rerun {dt*1e3:.1f} ms, kernel {b.last_launch()[0]:.2f} ms", flush=True)
        b.close()
