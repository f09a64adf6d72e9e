#!/bin/bash
# Nakamoto kernel iteration session: smoke, the Nakamoto/replay/boundary/API GPU tests
# (plus any extra test files in $EXTRA_TESTS), the default bench line, then the rocprofv3
# passes of tools/profile.sh. Each GPU step has its own time limit; a fault, abort or
# timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_replay.py tests/test_gpu_boundary.py tests/test_python_api.py ${EXTRA_TESTS:-} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_perf.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
[[ -n "${SKIP_PROFILE:-}" ]] && exit 0
bash tools/profile.sh
