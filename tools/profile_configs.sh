#!/bin/bash
# rocprofv3 evidence for bench.py's other_configs (BASELINE configs[0], [2]-[4]): per key a
# kernel-trace/stats pass and PMC passes of their own (no --sys-trace with --pmc):
# instruction mix, HBM bytes (FETCH_SIZE, WRITE_SIZE). Output: gpurun_out/cf_<n>_<pass>/.
# Summarise with tools/summarize_configs.py <tag> -> profiles/<tag>_config_pmc.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
KEYS="${KEYS:-0 2 3 3_exp 4}"
run() {  # name, key, rocprofv3 args...
  local name=$1 key=$2; shift 2
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d gpurun_out/$name -o run -- python3 tools/config_probe.py "$key" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/cf_status.log
  return $rc
}
for K in $KEYS; do
  if [[ $K == 3_exp ]]; then KEY="configs[3]_exp"; else KEY="configs[$K]"; fi
  run cf_${K}_trace "$KEY" --kernel-trace --stats || exit 1
  run cf_${K}_sq "$KEY" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
  run cf_${K}_fetch "$KEY" --pmc FETCH_SIZE || exit 1
  run cf_${K}_write "$KEY" --pmc WRITE_SIZE || exit 1
done
