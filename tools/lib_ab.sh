#!/bin/bash
# A/B of two builds of the library on the headline sweep: VARIANTS = "LIB ..." with LIB a
# build/var/<LIB>.so or "default" (the tree's); bench.py --no-cpu --no-configs, STEPS steps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${VARIANTS:-prev default prev default}; do
  if [[ $lib == default ]]; then unset CPR_HIP_LIB; else export CPR_HIP_LIB=build/var/$lib.so; fi
  timeout -k 10 300 python bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu --no-configs > gpurun_out/${TAG:-lab}_$lib.json 2> gpurun_out/${TAG:-lab}_$lib.err || exit 1
  python - "$lib" >> gpurun_out/${TAG:-lab}_ab.log <<PY
import json, sys
d = json.load(open("gpurun_out/${TAG:-lab}_" + sys.argv[1] + ".json"))
r = d["roofline"]
print(sys.argv[1], "value %.4e" % d["value"], "kernel %.4e" % r["kernel_activations_per_s"], "g0 %.2f" % (sum(v for k, v in r["kernel_ms_per_point"].items() if k.endswith(",0.0")) / 10), "g5 %.2f" % (sum(v for k, v in r["kernel_ms_per_point"].items() if k.endswith(",0.5")) / 10))
PY
done
