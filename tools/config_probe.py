"""Run one or more of bench.py's other BASELINE configs (configs[0], [2]-[4]) on the GPU
without the CPU leg, one launch per point as bench.py does, and print their entries as one
JSON line. Profiled by tools/profile_configs.sh (one rocprofv3 pass set per key).

usage: python tools/config_probe.py 'configs[2]' ['configs[3]' ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402
from cpr_amd import device  # noqa: E402

if __name__ == "__main__":
    import torch

    # torch's HIP runtime first, then the library's context on the same device (bench.py's
    # order: a context opened before torch leaves torch without a device)
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    ctx = device.Context(0)
    out = bench.run_other_configs(ctx, 0.0, False, {}, keys=set(sys.argv[1:]))
    print(json.dumps(out), flush=True)
    ctx.close()
