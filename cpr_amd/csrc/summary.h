// Episode-summary reduction shared by the episode kernels (kernels.hip, kernels_eth.hip):
// per-lane integer accumulators, wave shuffles, one LDS pass per workgroup, then one
// 64-bit atomic per field per workgroup. Integer arithmetic only, so the totals do not
// depend on scheduling or on how episodes are sharded over GPUs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cpr_hip.h"
#include "cpr_stream.h"

#pragma clang fp contract(off)

namespace cpr {

constexpr int kBlock = 256;

__device__ inline int64_t wave_sum(int64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

struct Acc {
  int64_t episodes, steps, activations, ra_fx, rd_fx, prog_fx, orphans, tie, overlap, other;
  uint64_t rel_fx, rel_sq_fx;
  int64_t invalid;
};

// cpr_summary word index of `invalid` (after the histogram)
constexpr int kInvalidWord = 12 + CPR_HIST_BINS;

// one finished episode; rewards and progress in 2^-20 fixed point, rel = attacker share
// of the head's rewards (wrappers.py:14-26 SparseRelativeRewardWrapper)
__device__ inline void acc_episode(Acc& a, int64_t ra_fx, int64_t rd_fx, int64_t prog_fx,
                                   double rel, int64_t head_height, int64_t steps,
                                   int64_t acts, uint32_t status, int32_t* hist_lds) {
  if (status & CPR_ST_INVALID) {  // outputs not valid: work counted, nothing else
    a.steps += steps;
    a.activations += acts;
    a.invalid += 1;
    return;
  }
  a.episodes += 1;
  a.steps += steps;
  a.activations += acts;
  a.ra_fx += ra_fx;
  a.rd_fx += rd_fx;
  a.prog_fx += prog_fx;
  a.orphans += acts - head_height;
  a.tie += (status & CPR_ST_TIE) ? 1 : 0;
  a.overlap += (status & CPR_ST_OVERLAP) ? 1 : 0;
  a.other += (status & ~(uint32_t)(CPR_ST_TIE | CPR_ST_OVERLAP | CPR_ST_EXACT_RERUN)) ? 1 : 0;
  a.rel_fx += (uint64_t)__builtin_rint(rel * 4294967296.0);
  a.rel_sq_fx += (uint64_t)__builtin_rint(rel * rel * 4294967296.0);
  int bin = (int)(rel * (double)CPR_HIST_BINS);
  bin = bin < 0 ? 0 : (bin >= CPR_HIST_BINS ? CPR_HIST_BINS - 1 : bin);
  atomicAdd(&hist_lds[bin], 1);
}

__device__ inline void block_flush(const Acc& a, int32_t* hist_lds, cpr_summary* out) {
  __shared__ int64_t red[kBlock / 64][13];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t v[13] = {a.episodes, a.steps,   a.activations, a.ra_fx,
                   a.rd_fx,    a.prog_fx, a.orphans,     a.tie,
                   a.overlap,  a.other,   (int64_t)a.rel_fx, (int64_t)a.rel_sq_fx,
                   a.invalid};
#pragma unroll
  for (int i = 0; i < 13; ++i) v[i] = wave_sum(v[i]);
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 13; ++i) red[wave][i] = v[i];
  __syncthreads();
  if (threadIdx.x < 13) {
    int64_t s = 0;
    for (int w = 0; w < kBlock / 64; ++w) s += red[w][threadIdx.x];
    unsigned long long* base = (unsigned long long*)out;
    // cpr_summary word index of each accumulator (rel sums sit before orphans)
    const int idx[13] = {0, 1, 2, 3, 4, 5, 8, 9, 10, 11, 6, 7, kInvalidWord};
    if (s) atomicAdd(base + idx[threadIdx.x], (unsigned long long)s);
  }
  if (threadIdx.x < CPR_HIST_BINS && hist_lds[threadIdx.x])
    atomicAdd((unsigned long long*)&out->hist[threadIdx.x],
              (unsigned long long)hist_lds[threadIdx.x]);
}

// Accumulators in LDS instead of registers (the Nakamoto lane's 24 VGPRs of int64 sums
// would otherwise stay live through every activation): one ds atomic per field per
// finished episode into the workgroup's 12 words, then one global atomic per field.
// Word order is cpr_summary's.
struct LdsAcc {
  unsigned long long* w;  // 13 words in LDS (word 12 = invalid)
  __device__ inline void init() {
    if (threadIdx.x < 13) w[threadIdx.x] = 0ull;
  }
  __device__ inline void episode(int64_t ra_fx, int64_t rd_fx, int64_t prog_fx, double rel,
                                 int64_t head_height, int64_t steps, int64_t acts,
                                 uint32_t status, int32_t* hist_lds) {
    auto add = [&](int i, int64_t v) {
      if (v) atomicAdd(&w[i], (unsigned long long)v);
    };
    if (status & CPR_ST_INVALID) {  // outputs not valid: work counted, nothing else
      add(1, steps);
      add(2, acts);
      add(12, 1);
      return;
    }
    add(0, 1);
    add(1, steps);
    add(2, acts);
    add(3, ra_fx);
    add(4, rd_fx);
    add(5, prog_fx);
    add(6, (int64_t)__builtin_rint(rel * 4294967296.0));
    add(7, (int64_t)__builtin_rint(rel * rel * 4294967296.0));
    add(8, acts - head_height);
    add(9, (status & CPR_ST_TIE) ? 1 : 0);
    add(10, (status & CPR_ST_OVERLAP) ? 1 : 0);
    add(11, (status & ~(uint32_t)(CPR_ST_TIE | CPR_ST_OVERLAP | CPR_ST_EXACT_RERUN)) ? 1 : 0);
    int bin = (int)(rel * (double)CPR_HIST_BINS);
    bin = bin < 0 ? 0 : (bin >= CPR_HIST_BINS ? CPR_HIST_BINS - 1 : bin);
    atomicAdd(&hist_lds[bin], 1);
  }
  // after __syncthreads()
  __device__ inline void flush(const int32_t* hist_lds, cpr_summary* out) const {
    if (threadIdx.x < 13 && w[threadIdx.x])
      atomicAdd((unsigned long long*)out + (threadIdx.x < 12 ? threadIdx.x : kInvalidWord),
                w[threadIdx.x]);
    if (threadIdx.x < CPR_HIST_BINS && hist_lds[threadIdx.x])
      atomicAdd((unsigned long long*)&out->hist[threadIdx.x],
                (unsigned long long)hist_lds[threadIdx.x]);
  }
};

__device__ inline Stream make_stream(uint64_t seed, uint64_t ep) {
  Stream S;
  S.k0 = (uint32_t)seed;
  S.k1 = (uint32_t)(seed >> 32);
  S.e0 = (uint32_t)ep;
  S.e1 = (uint32_t)(ep >> 32);
  return S;
}

// Where a fused episode kernel gets the draws of its e-th episode: the keyed stream of
// episode first + e (cpr_run_episodes), or episode e of a device copy of a cpr_trace
// (cpr_replay). missed() is the status bit a lane adds to its record.
// size(n): the episodes a launch of n runs; index(e): the launch-relative index of its e-th
struct SeedSource {
  uint64_t seed, first;
  __device__ inline Stream at(int64_t e) const { return make_stream(seed, first + (uint64_t)e); }
  __device__ inline int64_t size(int64_t n) const { return n; }
  __device__ inline int64_t index(int64_t e) const { return e; }
  __device__ static inline uint32_t missed(const Stream&) { return 0u; }
};

// the episodes a deferred-race launch (k_run_episodes, TT = 2) handed to its eager second
// pass: count, then launch-relative indices, in that launch's spill buffer
struct ListSource {
  SeedSource base;
  const uint32_t* count;
  const int64_t* list;
  __device__ inline Stream at(int64_t i) const { return base.at(list[i]); }
  __device__ inline int64_t size(int64_t n) const {
    const int64_t c = (int64_t)*count;
    return c < n ? c : n;
  }
  __device__ inline int64_t index(int64_t i) const { return list[i]; }
  __device__ static inline uint32_t missed(const Stream&) { return 0u; }
};

struct TraceSource {
  const int64_t* act_off;
  const int32_t* act_miner;
  const double* act_delay;
  const int64_t* pow_off;
  const int32_t* pow_hash;
  const int64_t* link_off;
  const uint64_t* link_key;
  const double* link_delay;
  __device__ inline TraceStream at(int64_t e) const {
    TraceStream S;
    const int64_t a0 = act_off[e], p0 = pow_off[e], l0 = link_off[e];
    S.act_miner = act_miner + a0;
    S.act_delay = act_delay + a0;
    S.n_act = (int32_t)(act_off[e + 1] - a0);
    S.pow_hash = pow_hash + p0;
    S.n_pow = (int32_t)(pow_off[e + 1] - p0);
    S.key = link_key + l0;
    S.delay = link_delay + l0;
    S.n_link = (int32_t)(link_off[e + 1] - l0);
    S.miss = 0u;
    return S;
  }
  __device__ inline int64_t size(int64_t n) const { return n; }
  __device__ inline int64_t index(int64_t e) const { return e; }
  __device__ static inline uint32_t missed(const TraceStream& S) {
    return S.miss ? (uint32_t)CPR_ST_TRACE_MISS : 0u;
  }
};


}  // namespace cpr
