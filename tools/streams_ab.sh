#!/bin/bash
# A/B of the headline sweep's launches on one or several HIP streams (contexts):
# VARIANTS = "S:MAP:GRID ..." (MAP gamma = one stream per gamma column, rr = round robin;
# GRID = percent of the resident grid per launch, 100 = all; WQ = 1 work queue, 0 static)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-1:gamma:100:1 2:gamma:100:1}; do
  IFS=: read S MAP GRID WQ <<< "$v"
  tag=${S}_${MAP}_${GRID}_wq$WQ
  CPR_NAK_WQ=$WQ CPR_GRID_SCALE=$GRID CPR_BENCH_STREAMS=$S CPR_BENCH_STREAM_MAP=$MAP timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu --no-configs ${BENCH_ARGS:-} > gpurun_out/r6e_streams_$tag.log 2>&1 || exit 1
  python - "$tag" >> gpurun_out/r6e_streams_ab.log <<'PY'
import json, sys
t = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/r6e_streams_{t}.log") if l.startswith("{")][-1])
print("%s value %.4e kernel_ms_mean %.2f ms_per_step %.1f" % (t, d["value"], d["roofline"]["kernel_ms_mean"], d["ms_per_step"]))
PY
done
