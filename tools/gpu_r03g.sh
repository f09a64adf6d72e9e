#!/bin/bash
# r03g: Nakamoto and event-engine parity after the arrive specialisation, equal-round lane
# counts, the event kernels' work-queue refill and per-protocol occupancy; the configs[2]
# probe at 1/2/4 episodes per resident lane and the event probes; a short headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_ts.py tests/test_gpu_bk.py tests/test_gpu_eth.py tests/test_gpu_expclique.py tests/test_gpu_replay.py tests/test_gpu_nodes.py tests/test_gpu_clique.py -x -q --timeout 300 --timeout-method thread --durations=10 > gpurun_out/pt_ev.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu --no-configs > gpurun_out/bench_short.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
for N in 0 -2 -4; do
  timeout -k 10 150 python tools/event_probe.py eth45 $N >> gpurun_out/probes.jsonl 2>>gpurun_out/probes.err
  rc=$?; echo "eth45 $N rc=$rc" >> gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
done
for P in eth eth_honest bk ts_exp; do
  timeout -k 10 150 python tools/event_probe.py $P 0 >> gpurun_out/probes.jsonl 2>>gpurun_out/probes.err
  rc=$?; echo "$P rc=$rc" >> gpurun_out/status.log; [[ $rc -eq 0 ]] || exit $rc
done
