import sys, numpy as np
sys.path[:0] = ["/root/repo", "/root/repo/tests"]
from cpr_amd import _lib as L, device
TS_RAISE = dict(protocol=L.PROTO_TAILSTORM, alpha=0.4, gamma=0.5, policy=L.TS_POLICY_AVOID_LOSS,
                reward_scheme=L.REWARD_DISCOUNT, subblock_selection=L.SELECT_OPTIMAL, k=1,
                max_steps=300, seed=0x7A110000)
cfg, keep = device.make_config(**TS_RAISE)
b = device.Batch(cfg, keep=keep)
s, rec = b.run(256, records=True)
print("status values", np.unique(rec["status"], return_counts=True))
print("steps", rec["n_steps"][:8], "acts", rec["n_activations"][:8])
print("flag eps", np.nonzero(rec["status"])[0][:20])
