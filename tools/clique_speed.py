"""Honest-clique throughput probe (experiments/simulate/honest_net.ml task shape: 10 nodes,
compute 1..10, U(0.5, 1.5) links, 10,000-activation Simulator.loop tasks) for the four
protocols on one GPU. The reference records its own per-task wall time in
data/honest_net.tsv (machine_duration_s, one OCaml process per task)."""
import sys
import time

sys.path.insert(0, '.')
from cpr_amd import _lib as L, device

RUNS = [("nakamoto", L.PROTO_NAKAMOTO, L.REWARD_CONSTANT, 8, 600.0, 16384),
        ("ethereum", L.PROTO_ETHEREUM, L.REWARD_DISCOUNT, 8, 600.0, 16384),
        ("bk8", L.PROTO_BK, L.REWARD_CONSTANT, 8, 600.0, 16384),
        ("tailstorm8", L.PROTO_TAILSTORM, L.REWARD_DISCOUNT, 8, 600.0, 4096)]
for name, proto, sch, k, ad, n in RUNS:
    cfg, keep = device.make_config(alpha=0.0, gamma=0.0, defenders=10,
                                   network=L.NET_HONEST_CLIQUE, mode=L.MODE_LOOP,
                                   protocol=proto, reward_scheme=sch, k=k, subblock_selection=2,
                                   activation_delay=ad, activations=10000, seed=3, policy=0)
    b = device.Batch(cfg, keep=keep)
    b.run(256)
    t = time.time()
    s = b.run(n)
    dt = time.time() - t
    print(f"{name}: {n} tasks x 10000 activations in {dt:.3f} s -> {s.activations / dt:.3e} "
          f"act/s, {n / dt:.1f} tasks/s; status_other {s.status_other}", flush=True)
