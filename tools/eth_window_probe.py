"""Speed probe of the Ethereum window lane (eth_window.h) on BASELINE configs[2]'s points:
one launch per point at the kernel's resident lane count (or --episodes), kernel time from
the library's HIP events, wall time around the synchronous call (incl. exact re-runs).
usage: python tools/eth_window_probe.py [--episodes N] [--engine]  (--engine: event engine)"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cpr_amd import _lib as L  # noqa: E402
from cpr_amd import device  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--episodes", type=int, default=0)
ap.add_argument("--engine", action="store_true")
ap.add_argument("--points", default="fn19:0.45:0,fn19:0.45:0.5,fn19:0.45:0.9,sr:0.35:0.5")
args = ap.parse_args()
if args.engine:
    os.environ["CPR_ETH_WINDOW"] = "0"
pol = {"fn19": L.ETH_POLICY_FN19, "sr": L.ETH_POLICY_SELFISH_RELEASE}
for spec in args.points.split(","):
    p, a, g = spec.split(":")
    cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=float(a), gamma=float(g),
                                   policy=pol[p], reward_scheme=L.REWARD_CONSTANT,
                                   max_steps=2016, seed=0x5EED0000)
    b = device.Batch(cfg, keep=keep)
    b.run(256)
    n = args.episodes or b.launch_shape()[1]
    t0 = time.perf_counter()
    s = b.run(n, first_episode=0)
    wall = time.perf_counter() - t0
    ms, _ = b.last_launch()
    lanes, res = b.launch_shape()
    print(json.dumps({"point": spec, "episodes": n, "lanes": lanes, "resident": res,
                      "kernel_ms": round(ms, 2), "wall_s": round(wall, 3),
                      "kernel_act_per_s": s.activations / (ms / 1e3),
                      "wall_act_per_s": s.activations / wall, "invalid": int(s.invalid),
                      "ties": int(s.status_tie), "overlap": int(s.status_overlap),
                      "rel": s.rel_revenue_fx / 2**32 / max(1, s.episodes)}), flush=True)
    b.close()
