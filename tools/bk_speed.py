"""B_k throughput probe (BASELINE configs[4] shape): fused 2048-step episodes and the
lockstep device rollout over 65,536 lanes with a table policy. Prints one line per run."""
import sys
import time

sys.path.insert(0, '.')
import numpy as np

from cpr_amd import _lib as L, device

K = 8
for pol, n in [(L.BK_POLICY_MINOR_DELAY, 262144), (L.BK_POLICY_HONEST, 262144)]:
    cfg, keep = device.make_config(alpha=0.33, gamma=0.5, policy=pol, k=K, max_steps=2048,
                                   seed=1, protocol=L.PROTO_BK)
    b = device.Batch(cfg, keep=keep)
    b.run(2048)
    t = time.time(); s = b.run(n); dt = time.time() - t
    ms, acts = b.last_launch()
    print(f"fused pol={pol}: {s.steps/dt:.3e} steps/s {s.activations/dt:.3e} act/s wall, "
          f"kernel {ms:.1f} ms -> {acts/ms*1e3:.3e} act/s; eps {s.episodes} other {s.status_other} "
          f"rel {s.rel_revenue_fx/2**32/s.episodes:.4f}", flush=True)

rnd = np.random.default_rng(0)
D = 4
table = rnd.integers(4, 8, size=D * D * (K + 1) ** 2 * 3).astype(np.uint8)
for lanes, T in [(65536, 64), (65536, 256)]:
    cfg, keep = device.make_config(alpha=0.33, gamma=0.5, table=table, k=K, max_steps=2048,
                                   seed=2, protocol=L.PROTO_BK, n_lanes=lanes)
    b = device.Batch(cfg, keep=keep)
    b.rollout(8)
    t = time.time(); s = b.rollout(T); dt = time.time() - t
    ms, acts = b.last_launch()
    print(f"rollout lanes={lanes} T={T}: {s.steps/dt:.3e} env-steps/s {s.activations/dt:.3e} act/s wall,"
          f" kernel {ms:.1f} ms -> {s.steps/ms*1e3:.3e} steps/s; finished eps {s.episodes} other {s.status_other}",
          flush=True)

# Tailstorm: BASELINE configs[3] (two agents, k=8, discount, heuristic, 10^4-activation
# Simulator.loop tasks) and 2048-step gym episodes
for pol, n in [(L.TS_POLICY_GET_AHEAD, 131072), (L.TS_POLICY_AVOID_LOSS, 131072)]:
    cfg, keep = device.make_config(alpha=0.33, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP,
                                   activations=2000, policy=pol, k=8,
                                   reward_scheme=L.REWARD_DISCOUNT,
                                   subblock_selection=L.SELECT_HEURISTIC, seed=3,
                                   protocol=L.PROTO_TAILSTORM)
    b = device.Batch(cfg, keep=keep)
    b.run(1024)
    t = time.time(); s = b.run(n); dt = time.time() - t
    ms, acts = b.last_launch()
    print(f"tailstorm loop pol={pol}: {s.activations/dt:.3e} act/s wall, kernel {ms:.1f} ms -> "
          f"{acts/ms*1e3:.3e} act/s; eps {s.episodes} other {s.status_other} "
          f"rel {s.rel_revenue_fx/2**32/s.episodes:.4f}", flush=True)
cfg, keep = device.make_config(alpha=0.33, gamma=0.5, policy=L.TS_POLICY_AVOID_LOSS, k=8,
                               reward_scheme=L.REWARD_DISCOUNT, max_steps=2048, seed=4,
                               protocol=L.PROTO_TAILSTORM)
b = device.Batch(cfg, keep=keep)
b.run(1024)
t = time.time(); s = b.run(131072); dt = time.time() - t
ms, acts = b.last_launch()
print(f"tailstorm gym avoid-loss: {s.steps/dt:.3e} steps/s {s.activations/dt:.3e} act/s wall, "
      f"kernel {ms:.1f} ms; eps {s.episodes} other {s.status_other}", flush=True)
