set -o pipefail
mkdir -p gpurun_out
for P in eth eth_honest bk ts ts_exp bk_rollout; do timeout -k 10 150 python tools/event_probe.py $P >> gpurun_out/r03b_probes.jsonl 2>>gpurun_out/r03b_probes.err || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_expclique.py tests/test_gpu_ts.py tests/test_gpu_eth.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1
