#!/bin/bash
# A/B of the Ethereum window lane's LDS block window (CPR_WIN_LDS=1, default) against
# every block read from the ring in HBM (0): bench.py's configs[2] entry
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 0 1}; do
  CPR_WIN_LDS=$v timeout -k 10 300 python tools/config_probe.py 'configs[2]' > gpurun_out/r6m_win_$v.json 2> gpurun_out/r6m_win_$v.err || exit 1
  python - "$v" >> gpurun_out/r6m_win_ab.log <<'PY'
import json, sys
v = sys.argv[1]
d = json.load(open(f"gpurun_out/r6m_win_{v}.json"))["configs[2]"]
print(f"win_lds {v} act/s {d['activations_per_s']:.4e} kernel {d['kernel_activations_per_s']:.4e} ms/pt {d['kernel_ms_per_point']}")
PY
done
