# bounded diagnostic: which step of a window-lane launch blocks
import ctypes, os, sys, time, faulthandler
faulthandler.dump_traceback_later(25, exit=True)
sys.path[:0] = ["/root/repo", "/root/repo/tests"]
import torch
from cpr_amd import _lib as L, device
torch.cuda.set_device(0)
print("torch ok", flush=True)
ctx = device.Context(0)
cfg, keep = device.make_config(protocol=L.PROTO_ETHEREUM, alpha=0.35, gamma=0.5,
                               policy=L.ETH_POLICY_FN19, reward_scheme=L.REWARD_CONSTANT,
                               max_steps=50, seed=0xE7E70000)
b = device.Batch(cfg, ctx=ctx, keep=keep)
print("batch ok", b.launch_shape(), flush=True)
sd = torch.zeros(ctypes.sizeof(L.Summary) // 8, dtype=torch.int64, device="cuda")
t = time.time()
b.run_async(4, 0, sd.data_ptr())
print("run_async returned %.3f" % (time.time() - t), flush=True)
ctx.synchronize()
print("synchronized %.3f" % (time.time() - t), flush=True)
t = time.time()
s, rec = b.run(4, first_episode=0, records=True)
print("records run %.3f" % (time.time() - t), int(s.episodes), flush=True)
