cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
F="tests/test_gpu_expclique.py tests/test_gpu_gamma.py tests/test_gpu_mdp.py tests/test_gpu_nodes.py tests/test_gpu_parity.py tests/test_gpu_replay.py tests/test_gpu_ts.py tests/test_host.py tests/test_lane_fuzz.py tests/test_mdp.py tests/test_python_api.py tests/test_trace.py"
timeout -k 10 900 python -u -m pytest $F -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_rest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/status.log
