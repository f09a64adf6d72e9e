#!/bin/bash
# A/B of lanes per wave: lockstep rollouts (CPR_ROLL_LPW) and fused event kernels
# (CPR_EV_LPW), on the tree's library or occupancy variants (build/var/ev<w>.so,
# tools/build_variants.py). AB: "lib:roll_lpw:ev_lpw" triples; CONFIGS: config_probe keys.
# Parity first: PARITY_TESTS under PARITY_LIB with PARITY_ENV.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=${TAG:-r05g}
if [[ -n ${PARITY_TESTS:-} ]]; then
  env ${PARITY_ENV:-} CPR_HIP_LIB=${PARITY_LIB:-cpr_amd/libcpr_hip.so} timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread $PARITY_TESTS > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest rc=$?"; exit 1; }
  echo "pytest ok"
fi
for ab in ${AB:-default:32:64}; do
  IFS=: read v rw ew <<< "$ab"
  if [[ $v == default ]]; then L=cpr_amd/libcpr_hip.so; else L=build/var/$v.so; fi
  echo "== lib $v roll_lpw $rw ev_lpw $ew" >> gpurun_out/${TAG}_lpw.log
  CPR_HIP_LIB=$L CPR_ROLL_LPW=$rw CPR_EV_LPW=$ew timeout -k 10 300 python tools/config_probe.py ${CONFIGS:-'configs[4]'} >> gpurun_out/${TAG}_lpw.log 2>&1 || { echo "probe $ab failed"; exit 1; }
done
