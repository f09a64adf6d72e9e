#!/bin/bash
# Nakamoto closed-form lane session: its GPU tests, the default bench line and the
# rocprofv3 passes of tools/profile.sh. Each GPU step has its own time limit; a fault,
# abort or timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu --deselect tests/test_gpu_gamma.py::test_gamma_loop_rows_within_4_sigma --deselect tests/test_gpu_gamma.py::test_rl_results_seq_hc_within_3_sigma -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_nak.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
bash tools/profile.sh
