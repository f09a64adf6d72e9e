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
# k_run_episodes variants (tools/nak_probe_variants.py) on the default sweep, per gamma
for v in ${NAK_VARIANTS:-}; do
  for g in ${NAK_GAMMAS:-0.5 0}; do
    CPR_HIP_LIB=build/var/$v.so timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --no-configs --gammas $g > gpurun_out/${TAG}_nak_${v}_$g.log 2>&1
    rc=$?; echo "nak $v $g rc=$rc" | tee -a gpurun_out/${TAG}_status.log; [[ $rc -eq 0 ]] || exit $rc
  done
done
# per-gamma PMC instruction mix of k_run_episodes (SQ counters, one pass per gamma)
export TMPDIR=/tmp
for g in ${PMC_GAMMAS:-}; do
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/${TAG}_pmc_g$g -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-configs --gammas $g > gpurun_out/${TAG}_pmc_g$g.log 2>&1
  rc=$?; echo "pmc $g rc=$rc" | tee -a gpurun_out/${TAG}_status.log; [[ $rc -eq 0 ]] || exit $rc
done
# BASELINE's other configs under library variants (build/var/<name>.so; default = the tree's)
for v in ${LIBS:-}; do
  if [[ $v == default ]]; then L=cpr_amd/libcpr_hip.so; else L=build/var/$v.so; fi
  echo "== lib $v" >> gpurun_out/${TAG}_libs.log
  CPR_HIP_LIB=$L timeout -k 10 400 python tools/config_probe.py ${CONFIGS:-'configs[3]'} >> gpurun_out/${TAG}_libs.log 2>&1
  rc=$?; echo "lib $v rc=$rc" | tee -a gpurun_out/${TAG}_status.log; [[ $rc -eq 0 ]] || exit $rc
done
