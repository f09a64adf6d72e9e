#!/bin/bash
# Tailstorm kernel A/B: event_probe ts / ts_exp with the tree's library and build/var/tsold.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for P in ts ts_exp; do
  for v in new old new old; do
    if [[ $v == old ]]; then export CPR_HIP_LIB=build/var/tsold.so; else unset CPR_HIP_LIB; fi
    timeout -k 10 300 python tools/event_probe.py $P > gpurun_out/tsab_${P}_$v.log 2>&1
    rc=$?; echo "$P $v rc=$rc $(tail -1 gpurun_out/tsab_${P}_$v.log)" >> gpurun_out/tsab_status.log
    [[ $rc -eq 0 ]] || exit $rc
  done
done
