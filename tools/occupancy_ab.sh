#!/bin/bash
# A/B of k_run_episodes occupancy variants (build/var/w{4,5,6}.so: amdgpu_waves_per_eu 4/5/6
# for the gym kernel): the default bench workload without the CPU leg, one run per variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp cpr_amd/libcpr_hip.so gpurun_out/orig.so
for v in w4 w5 w6 w5 w4; do
  cp build/var/$v.so cpr_amd/libcpr_hip.so
  timeout -k 10 180 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/ab_$v.log 2>&1
  rc=$?; echo "$v rc=$rc" >> gpurun_out/ab_status.log; [[ $rc -eq 0 ]] || exit $rc
  python - "$v" >> gpurun_out/ab_status.log <<'PY'
import json, sys
v = sys.argv[1]
line = [l for l in open(f"gpurun_out/ab_{v}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(v, "value %.4e" % d["value"], "kernel_ms %.3f" % d["roofline"]["kernel_ms_mean"])
PY
done
cp gpurun_out/orig.so cpr_amd/libcpr_hip.so
