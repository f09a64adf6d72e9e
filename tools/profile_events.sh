#!/bin/bash
# rocprofv3 evidence for the event-engine kernels (tools/event_probe.py): per probe one
# kernel-trace/stats pass and PMC passes of their own (no --sys-trace with --pmc):
# instruction mix and waits, LDS use and bank conflicts, HBM bytes, L2 hit rate.
# Output: gpurun_out/ev_<probe>_<pass>/. Summarise with tools/summarize_events.py <tag>.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PROBES="${PROBES:-eth eth_honest bk ts bk_rollout replay}"
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" --output-format csv -d gpurun_out/$name -o run -- python3 tools/event_probe.py $P > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/ev_status.log
  return $rc
}
for P in $PROBES; do
  run ev_${P}_trace --kernel-trace --stats || exit 1
  run ev_${P}_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES || exit 1
  run ev_${P}_fetch --pmc FETCH_SIZE || exit 1
  run ev_${P}_write --pmc WRITE_SIZE || exit 1
  run ev_${P}_tcc --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
done
