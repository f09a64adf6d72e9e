#!/bin/bash
# Round-end style GPU session: smoke, every -m gpu test, the default bench line, then the
# rocprofv3 passes of tools/profile.sh. Each GPU step has its own time limit; a fault,
# abort or timeout (124, 134, 137, 139) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ok() { local rc=$1; [[ $rc -eq 0 || $rc -eq 1 ]]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/status.log; ok $rc || exit $rc
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/status.log; ok $rc || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
[[ -n "${SKIP_PROFILE:-}" ]] && exit 0
bash tools/profile.sh
