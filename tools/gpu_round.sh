#!/bin/bash
# Round-end style GPU session: smoke, every -m gpu test, the default bench line, then the
# rocprofv3 passes of tools/profile.sh and (PROFILE_CONFIGS=1) tools/profile_configs.sh.
# Each GPU step has its own time limit; a fault, abort or timeout (124, 134, 137, 139)
# stops the script. TAG names the logs (gpurun_out/<TAG>_*); SKIP_TESTS=1 / SKIP_BENCH=1 /
# SKIP_PROFILE=1 leave steps out; TESTS overrides the test selection.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-round}
ok() { local rc=$1; [[ $rc -eq 0 || $rc -eq 1 ]]; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a gpurun_out/${TAG}_status.log; ok $rc || exit $rc
if [[ -z "${SKIP_TESTS:-}" ]]; then
  timeout -k 10 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" | tee -a gpurun_out/${TAG}_status.log; ok $rc || exit $rc
fi
if [[ -z "${SKIP_BENCH:-}" ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1
  rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/${TAG}_status.log; [[ $rc -eq 0 ]] || exit $rc
fi
[[ -n "${SKIP_PROFILE:-}" ]] && exit 0
bash tools/profile.sh || exit 1
[[ -n "${PROFILE_CONFIGS:-}" ]] && bash tools/profile_configs.sh
exit 0
