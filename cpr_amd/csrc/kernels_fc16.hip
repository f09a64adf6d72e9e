// FC'16 abstract-model kernel for gfx950 (fc16_lane.h): one lane = one probabilistically
// terminating episode of gym/rust/src/fc16.rs, grid-stride over episodes, policy (honest,
// SM1 or an (a, h, fork) table from cpr_amd.mdp) evaluated in the lane. Integer state and
// 32-bit threshold draws only; outcomes reduced like every episode kernel (summary.h).
#include <hip/hip_runtime.h>

#include "../../include/cpr_hip.h"
#include "fc16_lane.h"
#include "kernels.h"
#include "summary.h"

namespace cpr {

__global__ __launch_bounds__(kBlock) void k_fc16_episodes(fc16::Fc16Params P, SeedSource src,
                                                          int64_t n_eps,
                                                          cpr_episode_record* recs,
                                                          cpr_summary* sum) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  Acc acc = {};
  for (int64_t e = tid; e < n_eps; e += nthreads) {
    const fc16::Fc16Out o = fc16::fc16_episode(P, src.at(e));
    const int64_t ra = o.reward, rd = o.progress - o.reward;
    const double rel = o.progress != 0 ? (double)ra / (double)o.progress : 0.0;
    // activations: the start block plus one per step (every step mines one block)
    acc_episode(acc, ra << 20, rd << 20, o.progress << 20, rel, o.progress, o.steps,
                o.steps + 1, o.status, hist);
    if (recs) {
      cpr_episode_record r;
      r.reward_attacker = (double)ra;
      r.reward_defender = (double)rd;
      r.progress = (double)o.progress;
      r.chain_time = 0.0;
      r.sim_time = 0.0;
      r.n_steps = o.steps;
      r.n_activations = o.steps + 1;
      r.head_height = (int32_t)o.progress;
      r.head_miner = -1;
      r.status = o.status;
      r.head_work = 0;
      recs[e] = r;
    }
  }
  __syncthreads();
  block_flush(acc, hist, sum);
}

hipError_t launch_fc16_episodes(const fc16::Fc16Params& P, uint64_t seed, uint64_t first,
                                int64_t n_eps, int64_t lanes, cpr_episode_record* recs,
                                cpr_summary* sum, hipStream_t st) {
  const unsigned blocks = (unsigned)(lanes / kBlock);
  hipLaunchKernelGGL(k_fc16_episodes, dim3(blocks), dim3(kBlock), 0, st, P,
                     SeedSource{seed, first}, n_eps, recs, sum);
  return hipGetLastError();
}

}  // namespace cpr
