#!/bin/bash
# GPU session for the event-engine protocols: B_k + Tailstorm parity tests, then the probe.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [[ $rc -eq 0 || $rc -eq 1 ]]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bk.py tests/test_gpu_ts.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ev.log 2>&1
rc=$?; echo "pytest_ev rc=$rc" | tee -a gpurun_out/status.log; ok $rc || exit $rc
timeout -k 10 600 python -u tools/bk_speed.py > gpurun_out/bk_speed.log 2>&1
rc=$?; echo "bk_speed rc=$rc" | tee -a gpurun_out/status.log; exit $rc
