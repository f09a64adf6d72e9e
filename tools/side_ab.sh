#!/bin/bash
# A/B of the deferred-race second pass on the context's side stream (CPR_SIDE_PASS=1,
# the default) against the same stream (0): the headline bench without configs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 0 1}; do
  CPR_SIDE_PASS=$v timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu --no-configs > gpurun_out/r6k_side_$v.log 2>&1 || exit 1
  python - "$v" >> gpurun_out/r6k_side_ab.log <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/r6k_side_{v}.log") if l.startswith("{")][-1])
print("side %s value %.4e kernel_ms_mean %.2f ms_per_step %.1f ties %d overlaps %d" % (v, d["value"], d["roofline"]["kernel_ms_mean"], d["ms_per_step"], d["status"]["tie_episodes"], d["status"]["overlap_episodes"]))
PY
done
