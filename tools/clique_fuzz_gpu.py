"""Randomised device-vs-oracle sweep over honest-clique configurations (all four protocols):
n in 2..24 nodes, random U(lo, hi) link delays and activation delays, random k, reward
scheme and sub-block selection; every record field compared bit for bit for 32 keyed
episodes per configuration. Prints one line per configuration and a final tally; exit 1 on
any mismatch. Needs an MI355X (device) and the built oracle (checker)."""
import sys

sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import numpy as np

import oracle_py as O
from cpr_amd import _lib as L, device

FIELDS = [f for f in L.RECORD_DTYPE.names if f != "status"]
rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 2024)
n_cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 40
bad_total = 0
for i in range(n_cfg):
    proto = [L.PROTO_NAKAMOTO, L.PROTO_ETHEREUM, L.PROTO_BK, L.PROTO_TAILSTORM][i % 4]
    n = int(rng.integers(2, 25))
    lo = float(rng.choice([0.0, 0.1, 0.5, 1.0]))
    hi = lo + float(rng.choice([0.0, 0.5, 1.0, 4.0]))
    ad = float(rng.choice([0.2, 1.0, 5.0, 30.0, 600.0]))
    k = int(rng.integers(1, 9))
    sch = {L.PROTO_NAKAMOTO: L.REWARD_CONSTANT,
           L.PROTO_ETHEREUM: int(rng.choice([L.REWARD_CONSTANT, L.REWARD_DISCOUNT])),
           L.PROTO_BK: int(rng.choice([L.REWARD_CONSTANT, L.REWARD_BLOCK])),
           L.PROTO_TAILSTORM: int(rng.choice([L.REWARD_CONSTANT, L.REWARD_DISCOUNT,
                                              L.REWARD_PUNISH, L.REWARD_HYBRID]))}[proto]
    sel = int(rng.integers(0, 3))
    acts = int(rng.choice([200, 1000, 3000]))
    cfg, keep = device.make_config(alpha=0.0, gamma=0.0, defenders=n,
                                   network=L.NET_HONEST_CLIQUE, mode=L.MODE_LOOP, protocol=proto,
                                   reward_scheme=sch, k=k, subblock_selection=sel,
                                   activation_delay=ad, activations=acts, seed=1000 + i, policy=0,
                                   delay_lo=lo, delay_hi=hi)
    b = device.Batch(cfg, keep=keep)
    _, rec = b.run(32, records=True)
    ref = O.run_episodes(cfg, 0, 32, threads=8)
    bad = sum(int((rec[f] != ref[f]).sum()) for f in FIELDS)
    cap = int((rec["status"] & L.ST_CAPACITY).astype(bool).sum())
    bad_total += bad
    print(f"cfg {i:3d} proto={proto} n={n:2d} k={k} scheme={sch} sel={sel} delays=[{lo},{hi}] "
          f"ad={ad} acts={acts}: mismatching fields {bad}, capacity {cap}", flush=True)
print(f"TOTAL mismatching fields {bad_total} over {n_cfg} configurations x 32 episodes")
sys.exit(1 if bad_total else 0)
