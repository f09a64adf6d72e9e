#!/bin/bash
# A/B of the Tailstorm fused kernel's list-record LDS window (CPR_TS_TWIN rows, 0 = none;
# CPR_EV_VWIN visibility rows): VARIANTS = "TWIN:VWIN ...", VWIN "-" = the planner's;
# bench.py's configs[3] entries through tools/config_probe.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0:- 8:-}; do
  IFS=: read TW VW <<< "$v"
  if [[ $VW == - ]]; then unset CPR_EV_VWIN; else export CPR_EV_VWIN=$VW; fi
  CPR_TS_TWIN=$TW timeout -k 10 300 python tools/config_probe.py 'configs[3]' 'configs[3]_exp' > gpurun_out/r6q_twin_${TW}_$VW.json 2> gpurun_out/r6q_twin_${TW}_$VW.err || exit 1
  python - "$TW" "$VW" >> gpurun_out/r6q_twin_ab.log <<'PY'
import json, sys
tw, vw = sys.argv[1], sys.argv[2]
d = json.load(open(f"gpurun_out/r6q_twin_{tw}_{vw}.json"))
for k in ("configs[3]", "configs[3]_exp"):
    e = d[k]
    print(f"twin {tw} vwin {vw} {k} act/s {e['activations_per_s']:.4e} kernel {e['kernel_activations_per_s']:.4e} invalid {e['invalid']}")
PY
done
