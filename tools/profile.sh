#!/bin/bash
# rocprofv3 evidence for the dominant kernel (k_run_episodes): kernel-trace stats, then
# PMC counters in separate passes (no --sys-trace with --pmc). Output: gpurun_out/prof_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ARGS="--steps 1 --warmup 0 --no-cpu --no-configs ${BENCH_ARGS:-}"
step() { local rc=$1 name=$2; echo "$name rc=$rc" | tee -a gpurun_out/prof_status.log; [[ $rc -eq 0 ]]; }
timeout -k 10 120 rocprofv3 -L > gpurun_out/prof_counters.txt 2>&1
step $? list || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_trace -o run -- python3 bench.py $ARGS > gpurun_out/prof_trace.log 2>&1
step $? trace || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/prof_pmc_sq -o run -- python3 bench.py $ARGS > gpurun_out/prof_pmc_sq.log 2>&1
step $? pmc_sq || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_pmc_fetch -o run -- python3 bench.py $ARGS > gpurun_out/prof_pmc_fetch.log 2>&1
step $? pmc_fetch || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_pmc_write -o run -- python3 bench.py $ARGS > gpurun_out/prof_pmc_write.log 2>&1
step $? pmc_write || exit 1
# LDS evidence for the deferred-race kernel (gamma = .5: race lists in LDS): LDS
# instructions and bank-conflict cycles, in a pass of their own
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d gpurun_out/prof_pmc_lds -o run -- python3 bench.py $ARGS > gpurun_out/prof_pmc_lds.log 2>&1
step $? pmc_lds || exit 1
