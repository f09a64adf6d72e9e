#!/bin/bash
# r03f: Nakamoto parity incl. exact lockstep lanes, the k_run_episodes cost-centre A/B, the
# event engines' occupancy A/B under wave-coherent dispatch, then rocprofv3 evidence for the
# headline (tools/profile.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_python_api.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [[ $rc -le 1 ]] || exit $rc
VARIANTS="base cheap_rng cheap_log cheap_link unroll2" EPISODES="5242880" bash tools/nak_probe_ab.sh || exit 1
VARIANTS="0 2 4" PROBES="eth eth_honest bk ts_exp" PROBE_TIMEOUT=120 bash tools/occupancy_ab.sh || exit 1
bash tools/profile.sh || exit 1
