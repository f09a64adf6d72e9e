#!/bin/bash
# Full GPU session: smoke, every -m gpu test, B_k probe. Stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [[ $rc -eq 0 || $rc -eq 1 ]]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/status.log; ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/status.log; ok $rc || exit $rc
timeout -k 10 500 python -u tools/bk_speed.py > gpurun_out/bk_speed.log 2>&1
rc=$?; echo "bk_speed rc=$rc" | tee -a gpurun_out/status.log; exit $rc
