// Ethereum episode kernel for gfx950: one lane = one episode of the ethereum_ssz attack
// space (gym mode: engine.ml reset/step loop with an on-device policy; loop mode:
// Simulator.loop ~activations), driven by the exact per-lane event engine of
// ethereum_lane.h. Each resident lane owns one contiguous HBM region (block ring, node
// visibility, event heap, scratch) reused for every episode it runs.
#include <hip/hip_runtime.h>

#include "../../include/cpr_hip.h"
#include "ethereum_lane.h"
#include "kernels.h"
#include "summary.h"

#pragma clang fp contract(off)

namespace cpr {

template <class Src>
__global__ __launch_bounds__(kBlock) void k_eth_run_episodes(
    eth::EthParams P, Src src, int64_t n_eps, uint8_t* mem,
    int64_t lane_bytes, cpr_episode_record* recs, cpr_summary* sum) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  const eth::EthMem M = eth::eth_mem_at(mem + tid * lane_bytes, P.cap_b, P.cap_e, P.n);
  Acc acc = {};
  eth::EthLane L;
  for (int64_t e = tid; e < n_eps; e += nthreads) {
    const auto S = src.at(e);
    int32_t hd;
    if (P.mode == CPR_MODE_GYM) {
      L.gym_reset(P, S, M);
      bool done = L.dead != 0;
      hd = 0;
      while (!done) {
        const eth::EthObs o = L.observe(P, M, false);
        hd = L.gym_step(P, S, M, eth::eth_policy(P.policy, o), &done);
      }
    } else {
      hd = L.loop(P, S, M);
    }
    L.status |= Src::missed(S);
    const eth::EBlock& h = L.B(P, M, hd);
    const int32_t ra = h.rew_att, rd = h.rew_def;
    const double rel = (ra + rd) != 0 ? (double)ra / (double)(ra + rd) : 0.0;
    acc_episode(acc, (int64_t)ra << 15, (int64_t)rd << 15, (int64_t)h.work << 20, rel, h.height,
                L.steps, L.c_act, L.status, hist);
    if (recs) {
      cpr_episode_record r;
      r.reward_attacker = (double)ra / 32.0;
      r.reward_defender = (double)rd / 32.0;
      r.progress = (double)h.work;
      r.chain_time = h.time;
      r.sim_time = P.mode == CPR_MODE_GYM ? L.now : 0.0;
      r.n_steps = L.steps;
      r.n_activations = L.c_act;
      r.head_height = h.height;
      r.head_miner = P.mode == CPR_MODE_GYM ? h.miner : -1;
      r.status = L.status;
      r.head_work = h.work;
      recs[e] = r;
    }
  }
  __syncthreads();
  block_flush(acc, hist, sum);
}

hipError_t launch_eth_run_episodes(const eth::EthParams& P, uint64_t seed, uint64_t first,
                                   int64_t n_eps, uint8_t* mem, int64_t lane_bytes,
                                   int64_t lanes, cpr_episode_record* recs, cpr_summary* sum,
                                   hipStream_t st) {
  const unsigned blocks = (unsigned)(lanes / kBlock);
  hipLaunchKernelGGL(k_eth_run_episodes<SeedSource>, dim3(blocks), dim3(kBlock), 0, st, P, SeedSource{seed, first}, n_eps, mem, lane_bytes, recs, sum);
  return hipGetLastError();
}

hipError_t launch_eth_replay_episodes(const eth::EthParams& P, const TraceSource& src, int64_t n_eps,
                                 uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                 cpr_episode_record* recs, cpr_summary* sum, hipStream_t st) {
  hipLaunchKernelGGL(k_eth_run_episodes<TraceSource>, dim3((unsigned)(lanes / kBlock)),
                     dim3(kBlock), 0, st, P, src, n_eps, mem, lane_bytes, recs, sum);
  return hipGetLastError();
}

int eth_blocks_per_cu() {
  int blocks = 0;
  hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_eth_run_episodes<SeedSource>, kBlock, 0);
  if (e != hipSuccess || blocks <= 0) blocks = 2;
  return blocks;
}

}  // namespace cpr
