"""One warm-up plus one measured launch of an event-engine kernel, for rocprofv3 passes
(tools/profile_events.sh). Prints one JSON line: kernel, launch size, activations,
kernel time (HIP events) and activations/s.

  python tools/event_probe.py eth          k_eth_run_episodes: Ethereum fn19, whitepaper
                                           (constant) uncle rewards, alpha .35, gamma .5,
                                           2016-step gym episodes (BASELINE configs[2])
  python tools/event_probe.py eth45        k_eth_run_episodes: a bench configs[2] point (fn19,
                                           alpha .45, gamma .5)
  python tools/event_probe.py eth_honest   k_eth_run_episodes: honest, gamma 0, discount
  python tools/event_probe.py bk           k_bk_run_episodes: B_k k=8 minor-delay, 2048 steps
  python tools/event_probe.py ts           k_ts_run_episodes: Tailstorm k=8 discount heuristic
                                           get-ahead, two agents, 10^4-activation loop tasks
                                           (BASELINE configs[3])
  python tools/event_probe.py ts_exp       k_ts_run_episodes: the same on configs[3]'s exp(1)
                                           clique variant (activation delay 10)
  python tools/event_probe.py bk_rollout   k_bk_rollout: 65,536 B_k k=8 lanes, table policy,
                                           64 lockstep steps (BASELINE configs[4])
  python tools/event_probe.py replay       cpr_replay: Nakamoto two-agents loop tasks from a
                                           synthetic activation trace (exponential delays,
                                           alpha-weighted miners), k_run_episodes<TraceSource>
"""

import json
import sys
import time

sys.path.insert(0, ".")
import numpy as np

from cpr_amd import _lib as L
from cpr_amd import device

N = None

def fused(cfg, keep, n):
    """One launch of n episodes; n = 0: the kernel's resident lane count (one episode per
    resident lane, the grid full), found from a small warm-up launch (cpr_launch_shape)."""
    b = device.Batch(cfg, keep=keep)
    b.run(256, first_episode=1 << 40)
    _, resident = b.launch_shape()
    if n <= 0:  # 0: resident lanes; -k: k episodes per resident lane (work-queue refills)
        n = resident * max(1, -n)
    t = time.perf_counter()
    s = b.run(n)
    wall = time.perf_counter() - t
    ms, acts = b.last_launch()
    lanes, _ = b.launch_shape()
    return dict(episodes=n, activations=int(s.activations), steps=int(s.steps), kernel_ms=ms,
                wall_s=wall, invalid=int(s.invalid), lanes=lanes, resident_lanes=resident)


def main():
    which = sys.argv[1]
    global N
    N = int(sys.argv[2]) if len(sys.argv) > 2 else None  # episodes; 0 = resident lanes
    if which == "eth":
        cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=0.35, gamma=0.5,
                                       policy=L.ETH_POLICY_FN19, reward_scheme=L.REWARD_CONSTANT,
                                       max_steps=2016, seed=1)
        out = fused(cfg, keep, 131072 if N is None else N)
        out["kernel"] = "k_eth_run_episodes"
    elif which == "eth45":
        # a configs[2] point (bench.py other_configs): fn19, alpha .45, gamma .5
        cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=0.45, gamma=0.5,
                                       policy=L.ETH_POLICY_FN19, reward_scheme=L.REWARD_CONSTANT,
                                       max_steps=2016, seed=1)
        out = fused(cfg, keep, 131072 if N is None else N)
        out["kernel"] = "k_eth_run_episodes"
    elif which == "eth_honest":
        cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=0.25, gamma=0.0,
                                       policy=L.ETH_POLICY_HONEST, reward_scheme=L.REWARD_DISCOUNT,
                                       max_steps=2016, seed=1)
        out = fused(cfg, keep, 131072 if N is None else N)
        out["kernel"] = "k_eth_run_episodes"
    elif which == "bk":
        cfg, keep = device.make_config(protocol=L.PROTO_BK, alpha=0.33, gamma=0.5, k=8,
                                       policy=L.BK_POLICY_MINOR_DELAY, max_steps=2048, seed=1)
        out = fused(cfg, keep, 131072 if N is None else N)
        out["kernel"] = "k_bk_run_episodes"
    elif which == "ts_exp":
        # configs[3]'s exp(1)-propagation variant: attacker + 1 defender, exponential links
        cfg, keep = device.make_config(protocol=L.PROTO_TAILSTORM, alpha=0.0, gamma=0.0,
                                       network=L.NET_EXP_CLIQUE, mode=L.MODE_LOOP, defenders=1,
                                       activation_delay=10.0, propagation_delay=1.0,
                                       activations=10000, k=8, reward_scheme=L.REWARD_DISCOUNT,
                                       subblock_selection=L.SELECT_HEURISTIC,
                                       policy=L.TS_POLICY_GET_AHEAD, seed=1)
        out = fused(cfg, keep, 65536 if N is None else N)
        out["kernel"] = "k_ts_run_episodes"
    elif which == "ts":
        cfg, keep = device.make_config(protocol=L.PROTO_TAILSTORM, alpha=0.33,
                                       network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP,
                                       activations=10000, k=8, reward_scheme=L.REWARD_DISCOUNT,
                                       subblock_selection=L.SELECT_HEURISTIC,
                                       policy=L.TS_POLICY_GET_AHEAD, seed=1)
        out = fused(cfg, keep, 32768 if N is None else N)
        out["kernel"] = "k_ts_run_episodes"
    elif which == "bk_rollout":
        K, D, lanes = 8, 4, 65536
        table = np.random.default_rng(0).integers(0, 8, size=D * D * (K + 1) ** 2 * 3)
        cfg, keep = device.make_config(protocol=L.PROTO_BK, alpha=0.33, gamma=0.5, k=K,
                                       table=table.astype(np.uint8), max_steps=2048, seed=2,
                                       n_lanes=lanes)
        b = device.Batch(cfg, keep=keep)
        b.rollout(8)
        t = time.perf_counter()
        s = b.rollout(64)
        wall = time.perf_counter() - t
        ms, _ = b.last_launch()
        out = dict(kernel="k_bk_rollout", lanes=lanes, steps=int(s.steps),
                   activations=int(s.activations), kernel_ms=ms, wall_s=wall)
    elif which == "replay":
        n, acts, alpha = 16384, 10000, 0.33
        rng = np.random.default_rng(5)
        miner = (rng.random(n * acts) >= alpha).astype(np.int32)
        delay = rng.exponential(1.0, size=n * (acts + 1))
        off = np.arange(n + 1, dtype=np.int64)
        trace = L.Trace(act_offset=off * acts, act_miner=miner, act_delay=delay[: n * acts],
                        pow_offset=np.zeros(n + 1, np.int64), pow_hash=np.zeros(0, np.int32),
                        link_offset=np.zeros(n + 1, np.int64),
                        link_key=np.zeros(0, np.uint64), link_delay=np.zeros(0))
        cfg, keep = device.make_config(alpha=alpha, network=L.NET_TWO_AGENTS, mode=L.MODE_LOOP,
                                       activations=acts - 1,
                                       policy=L.POLICY_SAPIRSHTEIN_2016_SM1, seed=1)
        b = device.Batch(cfg, keep=keep)
        b.replay(trace.episode(0), records=False)
        t = time.perf_counter()
        s = b.replay(trace, records=False)
        wall = time.perf_counter() - t
        ms, _ = b.last_launch()
        out = dict(kernel="k_run_episodes<TraceSource> (cpr_replay)", episodes=n, activations=int(s.activations),
                   kernel_ms=ms, wall_s=wall, invalid=int(s.invalid),
                   trace_bytes=int(trace.act_miner.nbytes + trace.act_delay.nbytes))
    else:
        raise SystemExit(f"unknown probe {which}")
    out["probe"] = which
    out["activations_per_s_kernel"] = out["activations"] / (out["kernel_ms"] / 1e3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
