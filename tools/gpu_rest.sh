#!/bin/bash
# Second half of a GPU session: the -m gpu test files from $FROM_TESTS (default: the
# statistical and replay files), then optional kernel A/B variants ($VARIANTS, see
# tools/nak_probe_ab.sh) and the rocprofv3 passes of tools/profile.sh ($PROFILE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
F="${FROM_TESTS:-tests/test_gpu_gamma.py tests/test_gpu_mdp.py tests/test_gpu_nodes.py tests/test_gpu_parity.py tests/test_gpu_replay.py tests/test_gpu_ts.py tests/test_python_api.py tests/test_trace.py}"
timeout -k 10 900 python -u -m pytest $F -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_rest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [[ $rc -eq 0 || $rc -eq 1 ]] || exit $rc
if [[ -n "${VARIANTS:-}" ]]; then bash tools/nak_probe_ab.sh || exit $?; fi
if [[ -n "${PROFILE:-}" ]]; then bash tools/profile.sh; fi
