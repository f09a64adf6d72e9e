#!/bin/bash
# Round-4 GPU session: the tests touched this round, then probes. Each GPU step has its
# own time limit; a fault, abort or timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r04}
ok() { local rc=$1; [[ $rc -eq 0 || $rc -eq 1 ]]; }
timeout -k 10 ${PYTEST_LIMIT:-600} python -u -m pytest -x -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_eth.py tests/test_gpu_expclique.py} > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/${TAG}_status.log; ok $rc || exit $rc
for v in ${VARIANTS:-}; do
  if [[ $v == default ]]; then L=cpr_amd/libcpr_hip.so; else L=build/var/$v.so; fi
  echo "== $v" >> gpurun_out/${TAG}_probe.log
  CPR_HIP_LIB=$L timeout -k 10 300 python tools/eth_window_probe.py ${PROBE_ARGS:-} >> gpurun_out/${TAG}_probe.log 2>&1
  rc=$?; echo "probe $v rc=$rc" | tee -a gpurun_out/${TAG}_status.log; [[ $rc -eq 0 ]] || exit $rc
done
# BASELINE's other configs with and without the event-heap LDS slab (CPR_EV_SLAB=0: every
# heap node in HBM)
for s in ${SLABS:-}; do
  echo "== slab $s" >> gpurun_out/${TAG}_configs.log
  if [[ $s == default ]]; then E=""; else E="CPR_EV_SLAB=$s"; fi
  env $E timeout -k 10 400 python tools/config_probe.py ${CONFIGS:-'configs[3]' 'configs[4]'} >> gpurun_out/${TAG}_configs.log 2>&1
  rc=$?; echo "configs $s rc=$rc" | tee -a gpurun_out/${TAG}_status.log; [[ $rc -eq 0 ]] || exit $rc
done
