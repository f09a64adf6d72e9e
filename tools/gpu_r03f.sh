#!/bin/bash
# r03f: Nakamoto parity incl. exact lockstep lanes, then rocprofv3 evidence for the headline
# (tools/profile.sh) and the other BASELINE configs (tools/profile_configs.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_python_api.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [[ $rc -le 1 ]] || exit $rc
bash tools/profile.sh || exit 1
bash tools/profile_configs.sh || exit 1
