#!/bin/bash
# GPU session for B_k: parity tests, then the throughput probe. Each GPU step has its own
# time limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [[ $rc -eq 0 || $rc -eq 1 ]]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bk.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_bk.log 2>&1
rc=$?; echo "pytest_bk rc=$rc" | tee -a gpurun_out/status.log; ok $rc || exit $rc
timeout -k 10 300 python -u tools/bk_speed.py > gpurun_out/bk_speed.log 2>&1
rc=$?; echo "bk_speed rc=$rc" | tee -a gpurun_out/status.log; exit $rc
