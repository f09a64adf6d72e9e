# bounded diagnostic of the window lane's LDS window (prints as it goes)
import os, sys, time
sys.path[:0] = ["/root/repo", "/root/repo/tests"]
from cpr_amd import _lib as L, device
print("start", os.environ.get("CPR_WIN_LDS"), flush=True)
for n, steps in [(4, 50), (256, 300)]:
    cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=0.35, gamma=0.5,
                                   policy=L.ETH_POLICY_FN19, reward_scheme=L.REWARD_CONSTANT,
                                   max_steps=steps, seed=0xE7E70000)
    b = device.Batch(cfg, keep=keep)
    t = time.time()
    s, rec = b.run(n, records=True)
    print(n, steps, "ok %.3f s" % (time.time() - t), int(s.episodes), int(s.activations), flush=True)
    b.close()
