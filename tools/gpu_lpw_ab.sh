#!/bin/bash
# configs[4] A/B of the lockstep rollout's envs per wave (CPR_ROLL_LPW) and occupancy
# variants (build/var/ev<w>.so, tools/build_variants.py): LPW=32 on the tree's library, then
# "lib:lpw" pairs from AB (default "ev4:16 ev4:32"); parity of the rollout tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
TAG=${TAG:-r05g}
for w in ${PARITY_LPW:-16}; do
  CPR_HIP_LIB=${PARITY_LIB:-cpr_amd/libcpr_hip.so} CPR_ROLL_LPW=$w timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_bk.py tests/test_gpu_ts.py -k "rollout or lockstep" > gpurun_out/${TAG}_pytest_$w.log 2>&1 || { echo "pytest $w rc=$?"; exit 1; }
  echo "pytest $w ok"
done
for ab in default:32 ${AB:-ev4:16 ev4:32} default:32; do
  v=${ab%%:*}; w=${ab##*:}
  if [[ $v == default ]]; then L=cpr_amd/libcpr_hip.so; else L=build/var/$v.so; fi
  echo "== lib $v lpw $w" >> gpurun_out/${TAG}_lpw.log
  CPR_HIP_LIB=$L CPR_ROLL_LPW=$w timeout -k 10 300 python tools/config_probe.py ${CONFIGS:-'configs[4]'} >> gpurun_out/${TAG}_lpw.log 2>&1 || { echo "probe $ab failed"; exit 1; }
done
