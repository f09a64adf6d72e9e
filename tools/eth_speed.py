import sys, time
sys.path.insert(0, '.')
from cpr_amd import _lib as L, device
for (a, g, pol, sch, n) in [(0.35, 0.5, L.ETH_POLICY_FN19, L.REWARD_CONSTANT, 65536*4), (0.35, 0.9, L.ETH_POLICY_SELFISH_RELEASE, L.REWARD_CONSTANT, 65536*2), (0.25, 0.0, L.ETH_POLICY_HONEST, L.REWARD_DISCOUNT, 65536*2)]:
    cfg, keep = device.make_config(alpha=a, gamma=g, policy=pol, reward_scheme=sch, max_steps=2016, seed=1, protocol=L.PROTO_ETHEREUM)
    b = device.Batch(cfg, keep=keep)
    b.run(4096)
    t = time.time(); s = b.run(n); dt = time.time() - t
    ms, acts = b.last_launch()
    print(f"a={a} g={g} pol={pol}: {s.activations/dt:.3e} act/s wall, kernel {ms:.1f} ms -> {acts/ms*1e3:.3e} act/s; eps {s.episodes} other {s.status_other} rel {s.rel_revenue_fx/2**32/s.episodes:.4f}", flush=True)
