#!/bin/bash
# One GPU session: smoke, GPU parity tests, a short bench. Each GPU step has its own time
# limit; a fault/abort/timeout (124, 134, 137, 139) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [[ $rc -eq 0 || $rc -eq 1 ]]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/status.log; ok $rc || exit $rc
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/status.log; ok $rc || exit $rc
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/status.log; exit $rc
