set -o pipefail
mkdir -p gpurun_out
for P in eth eth_honest bk ts_exp; do timeout -k 10 170 python tools/event_probe.py $P 0 >> gpurun_out/r03d_probes.jsonl 2>>gpurun_out/r03d_probes.err || exit 1; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_ts.py tests/test_gpu_bk.py tests/test_gpu_eth.py tests/test_gpu_expclique.py tests/test_gpu_replay.py tests/test_gpu_nodes.py tests/test_gpu_clique.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest.log 2>&1
