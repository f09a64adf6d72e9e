#!/bin/bash
# A/B of the Ethereum window lane's LDS block window: VARIANTS = "LIB:WIN ..." with LIB a
# build/var/<LIB>.so from tools/build_variants.py (or "default" = the tree's library) and
# WIN = CPR_WIN_LDS (1 window, 0 every block read from the ring in HBM); bench.py's
# configs[2] entry through tools/config_probe.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-default:0 default:1}; do
  IFS=: read LIB WIN <<< "$v"
  if [[ $LIB == default ]]; then unset CPR_HIP_LIB; else export CPR_HIP_LIB=build/var/$LIB.so; fi
  CPR_WIN_LDS=$WIN timeout -k 10 300 python tools/config_probe.py 'configs[2]' > gpurun_out/r6m_win_${LIB}_$WIN.json 2> gpurun_out/r6m_win_${LIB}_$WIN.err || exit 1
  python - "$LIB" "$WIN" >> gpurun_out/r6m_win_ab.log <<'PY'
import json, sys
lib, win = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/r6m_win_{lib}_{win}.json"))["configs[2]"]
print(f"{lib} win_lds {win} act/s {d['activations_per_s']:.4e} kernel {d['kernel_activations_per_s']:.4e} lanes {d['lanes_per_launch']} ms/pt {d['kernel_ms_per_point']}")
PY
done
