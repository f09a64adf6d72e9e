"""One worker process of tests/test_gpu_gamma.py::test_gamma_loop_rows_within_4_sigma.

Each `data/withholding.tsv` gamma row is one batch of dependent 10,000-activation chains,
so a row's time is one lane's chain latency and rows only go faster side by side. A
process gets 4 hardware queues (GPU_MAX_HW_QUEUES), so the test starts 4 of these workers
(16 rows in flight); each runs its share of the rows on 4 threads with a context (HIP
stream) per thread and writes the records to an .npz.

usage: python tests/gamma_rows_worker.py <out.npz> <n_tasks> <row index> [<row index> ...]
"""

import sys
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_HERE = __file__.rsplit("/", 1)[0]
sys.path.insert(0, _HERE)
sys.path.insert(0, _HERE + "/..")  # the repository root: cpr_amd

import gamma_stats as G  # noqa: E402
from cpr_amd import _lib as L  # noqa: E402
from cpr_amd import device  # noqa: E402


def main(out, n_tasks, idx):
    rows = G.withholding_rows()
    local = threading.local()
    ctxs, batches = [], []

    def one(i):
        if not hasattr(local, "ctx"):
            local.ctx = device.Context(0)
            ctxs.append(local.ctx)
        cfg = G.row_config(device.make_config, L, rows[i], seed=0x6A330000 + i)
        b = device.Batch(cfg, ctx=local.ctx)
        _, rec = b.run(n_tasks, records=True)
        batches.append(b)  # closed at the end: hipFree would synchronize the device
        print(f"row {i}", flush=True)
        return i, rec

    with ThreadPoolExecutor(4) as pool:
        res = dict(pool.map(one, idx))
    for b in batches:
        b.close()
    for c in ctxs:
        c.close()
    np.savez(out, **{f"r{i}": rec for i, rec in res.items()})


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), [int(x) for x in sys.argv[3:]])
