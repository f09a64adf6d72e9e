#!/bin/bash
# A/B of configs[2] / configs[3] with R rounds of the resident lanes per launch and the
# work queue on (WQ=1) or off: VARIANTS = "R:WQ ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-1:0 1:1 4:1}; do
  IFS=: read R WQ <<< "$v"
  CPR_NAK_WQ=$WQ CPR_CFG_ROUNDS=$R timeout -k 10 400 python tools/config_probe.py ${KEYS:-configs[2]} > gpurun_out/r6g_cfg_${R}_wq$WQ.json 2> gpurun_out/r6g_cfg_${R}_wq$WQ.err || exit 1
  python - "$R" "$WQ" >> gpurun_out/r6g_cfg_ab.log <<'PY'
import json, sys
R, W = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/r6g_cfg_{R}_wq{W}.json"))
for k, v in d.items():
    print(f"rounds {R} wq {W} {k} act/s {v['activations_per_s']:.4e} kernel {v['kernel_activations_per_s']:.4e} ms/pt {v['kernel_ms_per_point']}")
PY
done
