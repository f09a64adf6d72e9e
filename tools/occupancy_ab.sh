#!/bin/bash
# A/B of the event-engine kernels' occupancy (tools/build_variants.py: build/var/ev<w>.so,
# CPR_EV_WAVES = w) on the event probes at resident capacity (tools/event_probe.py <p> 0).
# Usage: VARIANTS="0 2 4" PROBES="eth bk ts_exp" bash tools/occupancy_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-0 2 4}; do
  lib=cpr_amd/libcpr_hip.so
  [[ $v != 0 ]] && lib=build/var/ev$v.so
  for P in ${PROBES:-eth bk ts_exp}; do
    CPR_HIP_LIB=$PWD/$lib timeout -k 10 ${PROBE_TIMEOUT:-150} python tools/event_probe.py $P 0 > gpurun_out/ab_ev${v}_$P.json 2>gpurun_out/ab_ev${v}_$P.err
    rc=$?; echo "ev$v $P rc=$rc $(cat gpurun_out/ab_ev${v}_$P.json)" | tee -a gpurun_out/ab_status.log
    [[ $rc -eq 0 ]] || exit $rc
  done
done
