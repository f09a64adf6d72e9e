#!/bin/bash
# Memory-system counters of the event engines' launches (tools/config_probe.py), one pass
# per counter set: L1 address translation (UTCL1 hits / misses), L1->L2 read latency and
# requests, L2 hits / misses. KEYS: config keys (default configs[4]); TAG names the output.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-diag}
n=0
for key in ${KEYS:-configs[4]}; do
  n=$((n + 1))
  DEFAULT_PASSES=("TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES")
  # PASSES: counter sets separated by ';' (one rocprofv3 pass each) instead of the above
  if [[ -n "${PASSES:-}" ]]; then IFS=';' read -ra SETS <<< "$PASSES"; else SETS=("${DEFAULT_PASSES[@]}"); fi
  for pass in "${SETS[@]}"; do
    p=$(echo ${pass%% *} | tr 'A-Z' 'a-z')
    timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/${TAG}_${n}_$p -o run -- python3 tools/config_probe.py "$key" > gpurun_out/${TAG}_${n}_$p.log 2>&1
    rc=$?; echo "$key $p rc=$rc" | tee -a gpurun_out/${TAG}_status.log; [[ $rc -eq 0 ]] || exit $rc
  done
done
