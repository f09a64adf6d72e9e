// Ethereum episode kernel for gfx950: one lane = one episode of the ethereum_ssz attack
// space (gym mode: engine.ml reset/step loop with an on-device policy; loop mode:
// Simulator.loop ~activations), driven by the exact per-lane event engine of
// ethereum_lane.h. Each resident lane owns one contiguous HBM region (block ring, node
// visibility, event heap, scratch) reused for every episode it runs.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <cstdlib>

#include "../../include/cpr_hip.h"
#include "eth_window.h"
#include "ethereum_lane.h"
#include "kernels.h"
#include "nak_hybrid.h"
#include "summary.h"
#include "wave_sched.h"

#pragma clang fp contract(off)

namespace cpr {


// one finished episode: summary, record, per-node row
template <class Src, class St>
__device__ inline void eth_finish(const eth::EthParams& P, eth::EthLane& L, const eth::EthMem& M,
                                  const St& S, int64_t e, int32_t hd, Acc& acc, int32_t* hist,
                                  cpr_episode_record* recs, const NodeOut& no) {
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
    r.head_work = P.nak ? 0 : h.work;
    recs[e] = r;
  }
  if (no.acts) {  // csv_runner.ml:74-79: sim.activations and (Dag.data head).rewards
    const int32_t* hr = M.nrew + (int64_t)(hd & (P.cap_b - 1)) * P.n;
    for (int32_t j = 0; j < P.n; ++j) {
      no.acts[e * P.n + j] = M.nact[j];
      no.rews[e * P.n + j] = (double)hr[j] / 32.0;
    }
    no.head_miner[e] = h.miner;
  }
}

// wave_sched.h adapter for ethereum_lane.h (also the Nakamoto-mode engine)
struct EthAdapter {
  using Lane = eth::EthLane;
  using Par = eth::EthParams;
  using Mem = eth::EthMem;
  template <class St>
  __device__ static void begin(Lane& L, const Par& P, const St& S, const Mem& M) {
    L.init(P, S, M);
  }
  __device__ static bool gym(const Par& P) { return P.mode == CPR_MODE_GYM; }
  __device__ static bool loop_attacker(const Par& P) { return P.net != 2; }
  __device__ static bool pow0(uint32_t ev) { return (ev & 7u) == eth::EV_DAG && (ev >> 5) == 0u; }
  template <class St>
  __device__ static void run_pow0(Lane& L, const Par& P, const St&, const Mem& M, int32_t) {
    const eth::Payload d = L.payload(P, M, 0, L.priv, eth::F_MINING, L.own, L.foreign);
    const int32_t v = L.append(P, M, 0, d);
    L.push_now(P, M, eth::mkev(eth::EV_MV, 0, eth::KD_POW), v);
  }
  __device__ static void act(Lane& L, const Par& P, const Mem& M) {
    const eth::EthObs o = L.observe(P, M, false);
    const int32_t sh = L.apply(P, M, eth::lane_action(P, o));
    if (sh >= 0) L.share(P, M, 0, sh);
    ++L.steps;
  }
  __device__ static int32_t head_gym(Lane& L, const Par& P, const Mem& M, int32_t att) {
    return L.head(P, M, att);
  }
  __device__ static int32_t head_loop(Lane& L, const Par& P, const Mem& M) {
    return L.head(P, M, P.net == 2 ? M.tips[0] : L.priv);
  }
  __device__ static bool gym_done(Lane& L, const Par& P, const Mem& M, int32_t hd) {
    const double progress = (double)L.B(P, M, hd).work;
    return L.dead || !(L.steps < P.max_steps && progress < P.max_progress && L.now < P.max_time);
  }
};

template <class Src>
__global__ __launch_bounds__(kBlock) CPR_EV_OCC void k_eth_run_episodes(
    eth::EthParams P, Src src, int64_t n_eps, uint8_t* mem,
    int64_t lane_bytes, cpr_episode_record* recs, cpr_summary* sum, NodeOut no) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  eth::EthMem M = eth::eth_mem_at(mem + tid * lane_bytes, P.cap_b, P.cap_e, P.n);
  if (no.mem) eth::eth_node_mem(M, no.mem + tid * no.lane_bytes, P.n);
  Acc acc = {};
  eth::EthLane L;
#if CPR_EV_SCHED
  int64_t e = tid;  // wave-coherent dispatch (wave_sched.h), episodes from a work queue
  auto S = src.at(e < n_eps ? e : 0);
  EvCursor c;
  c.cls = -1;
  c.phase = PH_IDLE;
  if (e < n_eps) ev_begin<EthAdapter>(L, P, S, M, c);
  for (;;) {
    while (c.phase != PH_IDLE && c.cls < 0) {
      if (c.phase != PH_OVER) ev_fetch<EthAdapter>(L, P, S, M, c);
      if (c.phase == PH_OVER) {
        eth_finish<Src>(P, L, M, S, e, c.hd, acc, hist, recs, no);
        e = ev_next_episode(P.next, e, nthreads);
        if (e < n_eps) {
          S = src.at(e);
          ev_begin<EthAdapter>(L, P, S, M, c);
        } else {
          c.phase = PH_IDLE;
        }
      }
    }
    const int32_t k = ev_choose(c.cls);
    if (k < 0) break;
    if (c.cls == k) ev_exec<EthAdapter>(L, P, S, M, c);
  }
#else
  for (int64_t e = tid; e < n_eps; e += nthreads) {
    const auto S = src.at(e);
    int32_t hd;
    if (P.mode == CPR_MODE_GYM) {
      L.gym_reset(P, S, M);
      bool done = L.dead != 0;
      hd = 0;
      while (!done) {
        const eth::EthObs o = L.observe(P, M, false);
        hd = L.gym_step(P, S, M, eth::lane_action(P, o), &done);
      }
    } else {
      hd = L.loop(P, S, M);
    }
    eth_finish<Src>(P, L, M, S, e, hd, acc, hist, recs, no);
  }
#endif
  __syncthreads();
  block_flush(acc, hist, sum);
}

// Ethereum gym episodes on the selfish-mining network, a window at a time (eth_window.h):
// one lane per episode, grid-stride over the launch's episodes, outputs as
// k_eth_run_episodes. An episode the window lane cannot vouch for (W_REDO) goes to the
// context's exact re-run queue instead, like the Nakamoto lane's (k_nak_exact_rerun runs it
// again from its first draw on the event engine at the next synchronization point). Each
// lane leaves its loop at its own done (max_steps, max_progress or max_time, engine.ml:
// 209-214); with max_steps alone the lanes of a wave run the same number of windows.
#ifdef CPR_EW_WAVES  // occupancy A/B (tools/build_variants.py --ew)
#define CPR_EW_OCC __attribute__((amdgpu_waves_per_eu(CPR_EW_WAVES)))
#else
#define CPR_EW_OCC
#endif
template <int REC>
__global__ __launch_bounds__(kBlock) CPR_EW_OCC void k_eth_win_episodes(
    eth::EthParams P, SeedSource src, int64_t n_eps, uint8_t* mem, int64_t lane_bytes,
    cpr_episode_record* recs, cpr_summary* sum, int64_t* redo, uint32_t* redo_n,
    uint32_t launch_id, int64_t redo_cap, uint8_t* ovf) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  __shared__ unsigned long long acc_w[13];
  LdsAcc acc{acc_w};
  acc.init();
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  const ethw::WinMem M = ethw::win_mem_at(mem + tid * lane_bytes, P.cap_b);
  if (!REC) recs = nullptr;
  ethw::WinLane W;
  // a lane that finishes takes the next episode from the work queue (P.next, wave_sched.h)
  for (int64_t e = tid; e < n_eps; e = ev_next_episode(P.next, e, nthreads)) {
    const Stream S = src.at(e);
    W.gym_reset(P, S, M);
    bool done = W.dead != 0;
    int32_t hd = 0;
    while (!done) hd = W.gym_step(P, S, M, eth::lane_action(P, W.observe(P, M, false)), &done);
    uint32_t status = W.status;
    if (status & ethw::W_REDO) {
      const uint32_t r = atomicAdd(redo_n, 1u);
      if ((int64_t)r < redo_cap)
        redo[r] = ((int64_t)launch_id << 40) | (e << 8) | (int64_t)(status & 0xffu);
      else  // queue full: the launch's overflow flags (k_rerun_overflow)
        ovf[e] = (uint8_t)(0x80u | (status & 0x7fu));
      continue;
    }
    const ethw::WBlock& h = W.B(P, M, hd);
    const int32_t ra = h.rew_att, rd = h.rew_def;
    const double rel = (ra + rd) != 0 ? (double)ra / (double)(ra + rd) : 0.0;
    acc.episode((int64_t)ra << 15, (int64_t)rd << 15, (int64_t)h.work << 20, rel, h.height,
                W.steps, W.c_act, status, hist);
    if (REC && recs) {
      cpr_episode_record r;
      r.reward_attacker = (double)ra / 32.0;
      r.reward_defender = (double)rd / 32.0;
      r.progress = (double)h.work;
      r.chain_time = W.time_of(P, M, hd);
      r.sim_time = W.now;
      r.n_steps = W.steps;
      r.n_activations = W.c_act;
      r.head_height = h.height;
      r.head_miner = h.miner;
      r.status = status;
      r.head_work = h.work;
      recs[e] = r;
    }
  }
  __syncthreads();
  acc.flush(hist, sum);
}

using EthWinFn = void (*)(eth::EthParams, SeedSource, int64_t, uint8_t*, int64_t,
                          cpr_episode_record*, cpr_summary*, int64_t*, uint32_t*, uint32_t,
                          int64_t, uint8_t*);
static EthWinFn eth_win_fn(bool recs) {
  return recs ? k_eth_win_episodes<1> : k_eth_win_episodes<0>;
}

hipError_t launch_eth_win_episodes(const eth::EthParams& P, uint64_t seed, uint64_t first,
                                   int64_t n_eps, uint8_t* mem, int64_t lane_bytes,
                                   int64_t lanes, cpr_episode_record* recs, cpr_summary* sum,
                                   int64_t* redo, uint32_t* redo_n, uint32_t launch_id,
                                   int64_t redo_cap, uint8_t* ovf, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, ethw::win_lane_bytes(P.cap_b));
  hipLaunchKernelGGL(eth_win_fn(recs != nullptr), dim3((unsigned)(lanes / kBlock)), dim3(kBlock),
                     0, st, P, SeedSource{seed, first}, n_eps, mem, lane_bytes, recs, sum, redo,
                     redo_n, launch_id, redo_cap, ovf);
  return hipGetLastError();
}

int eth_win_blocks_per_cu(bool recs) {
  int blocks = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &blocks, (const void*)eth_win_fn(recs), kBlock, 0);
  if (e != hipSuccess || blocks <= 0) blocks = 2;
  return blocks;
}

// Exact re-run of the Nakamoto episodes the closed-form lane flagged.
// Episode kernels queue (launch << 40) | (episode index << 8) | status bits instead of
// accumulating such an episode; at the next synchronization point this kernel simulates
// every queued episode again from its first draw on this event engine in Nakamoto mode
// (P.nak), which follows every event of the reference's queue, so messages still in
// flight at an activation are exact. Its record and summary contribution replace the
// flagged ones; status keeps the lane's bits and adds CPR_ST_EXACT_RERUN.
//
// One episode per one-wave workgroup (lane 0 runs it: a re-run is one dependent chain, the
// other lanes would only diverge); all queued episodes run concurrently. The summary is
// updated with per-episode atomics (episodes of different launches go to different
// summaries; there are ~1e-5 of them per episode kernel at the gym's delays).
template <class St>
__device__ inline int32_t nak_rerun_one(const eth::EthParams& P, const St& S,
                                        const eth::EthMem& M, eth::EthLane& L) {
  if (P.mode != CPR_MODE_GYM) return L.loop(P, S, M);
  L.gym_reset(P, S, M);
  bool done = L.dead != 0;
  int32_t hd = 0;
  while (!done) hd = L.gym_step(P, S, M, eth::lane_action(P, L.observe(P, M, false)), &done);
  return hd;
}

// one episode into a summary with per-episode atomics; rewards and progress in 2^-20
// fixed point, as acc_episode
__device__ inline void summary_add_episode(cpr_summary* out, int64_t ra_fx, int64_t rd_fx,
                                           int64_t prog_fx, double rel, int64_t height,
                                           int64_t steps, int64_t acts, uint32_t status) {
  auto add = [](int64_t* p, int64_t v) {
    if (v) atomicAdd((unsigned long long*)p, (unsigned long long)v);
  };
  if (status & CPR_ST_INVALID) {  // outputs not valid: work counted, nothing else
    add(&out->steps, steps);
    add(&out->activations, acts);
    add(&out->invalid, 1);
    return;
  }
  add(&out->episodes, 1);
  add(&out->steps, steps);
  add(&out->activations, acts);
  add(&out->reward_attacker_fx, ra_fx);
  add(&out->reward_defender_fx, rd_fx);
  add(&out->progress_fx, prog_fx);
  add((int64_t*)&out->rel_revenue_fx, (int64_t)__builtin_rint(rel * 4294967296.0));
  add((int64_t*)&out->rel_revenue_sq_fx, (int64_t)__builtin_rint(rel * rel * 4294967296.0));
  add(&out->orphans, acts - height);
  add(&out->status_tie, (status & CPR_ST_TIE) ? 1 : 0);
  add(&out->status_overlap, (status & CPR_ST_OVERLAP) ? 1 : 0);
  add(&out->status_other,
      (status & ~(uint32_t)(CPR_ST_TIE | CPR_ST_OVERLAP | CPR_ST_EXACT_RERUN)) ? 1 : 0);
  int bin = (int)(rel * (double)CPR_HIST_BINS);
  bin = bin < 0 ? 0 : (bin >= CPR_HIST_BINS ? CPR_HIST_BINS - 1 : bin);
  add(&out->hist[bin], 1);
}

// one queued episode on the lane region M (params P): the episode's own stream or trace
__device__ inline int32_t nak_rerun_entry(const RerunLaunch& RL, int64_t e,
                                          const eth::EthParams& P, const eth::EthMem& M,
                                          eth::EthLane& L, uint32_t* miss) {
  if (RL.is_trace) {
    auto S = RL.tr.at(e);
    const int32_t hd = nak_rerun_one(P, S, M, L);
    *miss = TraceSource::missed(S);
    return hd;
  }
  *miss = 0;
  return nak_rerun_one(P, make_stream(RL.seed, RL.first + (uint64_t)e), M, L);
}

// the re-run episode's record and summary contribution (replacing the flagged ones):
// Nakamoto episodes of the closed-form lane (P.nak: one reward per block, progress =
// height) and Ethereum episodes of the window lane (eth_window.h) alike. The flags the
// re-run resolved (a fast lane's capacity or unresolved tie) leave the status.
__device__ inline void nak_rerun_finish(const RerunLaunch& RL, int64_t e,
                                        const eth::EthParams& P, const eth::EthMem& M,
                                        eth::EthLane& L, int32_t hd, uint32_t flags) {
  const uint32_t resolved =
      CPR_ST_DEEP_FORK | CPR_ST_TIE_UNRESOLVED | CPR_ST_STALE_TIME | CPR_ST_CAPACITY;
  const uint32_t status = (flags & ~(uint32_t)CPR_ST_CAPACITY) | L.status | CPR_ST_EXACT_RERUN;
  const eth::EBlock& h = L.B(P, M, hd);
  const int32_t ra = h.rew_att, rd = h.rew_def;  // units of 1/32
  const double rel = (ra + rd) != 0 ? (double)ra / (double)(ra + rd) : 0.0;
  const int64_t steps = P.mode == CPR_MODE_GYM ? L.steps : 0;
  summary_add_episode(RL.sum, (int64_t)ra << 15, (int64_t)rd << 15, (int64_t)h.work << 20, rel,
                      h.height, steps, L.c_act,
                      (flags & ~resolved) | L.status | CPR_ST_EXACT_RERUN);
  if (RL.recs) {
    cpr_episode_record rc;
    rc.reward_attacker = (double)ra / 32.0;
    rc.reward_defender = (double)rd / 32.0;
    rc.progress = (double)h.work;
    rc.chain_time = h.time;
    rc.sim_time = P.mode == CPR_MODE_GYM ? L.now : 0.0;
    rc.n_steps = steps;
    rc.n_activations = L.c_act;
    rc.head_height = h.height;
    rc.head_miner = P.mode == CPR_MODE_GYM ? h.miner : -1;
    rc.status = status;
    rc.head_work = P.nak ? 0 : h.work;
    RL.recs[e] = rc;
  }
}

// a hybrid re-run that ended on the closed form: the record and summary the engine would
// have written for the same head (nak_rerun_finish's fields; rewards in units of 1/32)
__device__ inline void nak_hybrid_finish(const RerunLaunch& RL, int64_t e, const Stream& S,
                                         const HybridResult& R, uint32_t flags,
                                         uint32_t est) {
  const uint32_t resolved =
      CPR_ST_DEEP_FORK | CPR_ST_TIE_UNRESOLVED | CPR_ST_STALE_TIME | CPR_ST_CAPACITY;
  const uint32_t status = (flags & ~(uint32_t)CPR_ST_CAPACITY) | est | CPR_ST_EXACT_RERUN;
  const int32_t ra = R.hd.ra * 32, rd = (R.hd.h - R.hd.ra) * 32;
  const double rel = (ra + rd) != 0 ? (double)ra / (double)(ra + rd) : 0.0;
  summary_add_episode(RL.sum, (int64_t)ra << 15, (int64_t)rd << 15, (int64_t)R.hd.h << 20, rel,
                      R.hd.h, R.steps, R.acts, (flags & ~resolved) | est | CPR_ST_EXACT_RERUN);
  if (RL.recs) {
    cpr_episode_record rc;
    rc.reward_attacker = (double)ra / 32.0;
    rc.reward_defender = (double)rd / 32.0;
    rc.progress = (double)R.hd.h;
    rc.chain_time = R.hd.tm;
    rc.sim_time = R.now;
    rc.n_steps = R.steps;
    rc.n_activations = R.acts;
    rc.head_height = R.hd.h;
    rc.head_miner = miner_of(RL.NP, S, R.hd.k);
    rc.status = status;
    rc.head_work = 0;
    RL.recs[e] = rc;
  }
}

// one flagged episode again on the event engine, lane region `base` (HBM) and lane_lds:
// everything but the block ring (visibility, event heap, tips, scratch) in LDS. A lane
// whose heap capacity does not fit runs with the capacity that does (the heap's node order
// does not depend on it) and, only if its episode outgrows that, again in HBM. gamma = 0
// re-runs are the case: +inf messages stay in the heap (ethereum_lane.h), a few thousand
// nodes, whose dependent walks are L2 round trips in HBM
__device__ inline void rerun_episode(const RerunLaunch& RL, int64_t e, uint32_t flags,
                                     uint8_t* base, uint8_t* lane_lds, int64_t lds_bytes,
                                     const uint32_t* queue_n, double* hring = nullptr) {
  const eth::EthParams P = RL.P;
  // attempt 0: LDS (full or reduced heap capacity); attempt 1 (only after the reduced
  // heap overflowed): the lane's HBM region
  int32_t lds_cap_e = -1;  // heap capacity in LDS, -1 = HBM
  if (lds_bytes > 0) {
    const int64_t heap = eth::align128((int64_t)P.cap_e * 24);
    const int64_t other = eth::eth_rest_bytes(P.cap_b, P.cap_e, P.n) - heap;
    const int64_t room = (lds_bytes - other) / 128 * 128;
    if (room >= heap)
      lds_cap_e = P.cap_e;
    else if (room >= 256 * 24)
      lds_cap_e = (int32_t)(room / 24);
  }
  for (int attempt = lds_cap_e < 0 ? 1 : 0; attempt < 2; ++attempt) {
    eth::EthParams PA = P;
    if (attempt == 0) PA.cap_e = lds_cap_e;
    const eth::EthMem M = attempt == 0
                              ? eth::eth_mem_split(base, lane_lds, PA.cap_b, PA.cap_e, PA.n)
                              : eth::eth_mem_at(base, P.cap_b, P.cap_e, P.n);
    eth::EthLane L;
    if (RL.hybrid && !RL.is_trace) {
      // the closed form with the engine around the flagged windows (nak_hybrid.h); its
      // lane state after the engine's region
      const Stream S = make_stream(RL.seed, RL.first + (uint64_t)e);
      LaneMem LM = hybrid_mem(base + eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n), RL.NP.cap);
      // block times feed only the record's chain_time: a summary-only launch skips them;
      // the private-chain ring in the workgroup's LDS (hring) rather than HBM
      LM.times = RL.recs != nullptr;
      if (hring) LM.ring = hring;
      NakLane NL;
      const HybridResult R = nak_hybrid_episode(RL.NP, PA, S, LM, M, L, NL);
      if (attempt == 0 && R.entries && L.dead == 2 && PA.cap_e < P.cap_e) {
        atomicAdd(const_cast<uint32_t*>(queue_n) + 1, 1u);
        continue;
      }
      const uint32_t est = R.entries ? L.status : 0u;
      if (R.closed)
        nak_hybrid_finish(RL, e, S, R, flags, est);
      else
        nak_rerun_finish(RL, e, P, M, L, R.ehd, flags);
      break;
    }
    uint32_t miss = 0;
    const int32_t hd = nak_rerun_entry(RL, e, PA, M, L, &miss);
    if (attempt == 0 && L.dead == 2 && PA.cap_e < P.cap_e) {  // outgrew LDS: count, redo
      atomicAdd(const_cast<uint32_t*>(queue_n) + 1, 1u);  // cpr_rerun_hbm_retries
      continue;
    }
    nak_rerun_finish(RL, e, P, M, L, hd, flags | miss);
    break;
  }
}

__global__ __launch_bounds__(64) void k_nak_exact_rerun(const RerunLaunch* launches,
                                                         const int64_t* queue,
                                                         const uint32_t* queue_n,
                                                         int64_t queue_cap, uint8_t* mem,
                                                         int64_t lane_bytes, int64_t lds_bytes) {
  extern __shared__ __attribute__((aligned(128))) uint8_t lane_lds[];
  __shared__ double hring[RING];  // a hybrid's private-chain ring (nak_hybrid.h)
  int64_t nq = (int64_t)*queue_n;
  nq = nq < queue_cap ? nq : queue_cap;
  uint8_t* base = mem + (int64_t)blockIdx.x * lane_bytes;
  if (threadIdx.x != 0) return;  // one dependent chain per episode: lane 0 runs it
  for (int64_t r = blockIdx.x; r < nq; r += gridDim.x) {
    const int64_t q = queue[r];
    rerun_episode(launches[q >> 40], (q >> 8) & 0xffffffffll, (uint32_t)(q & 0xff), base,
                  lane_lds, lds_bytes, queue_n, hring);
  }
}

// The episodes that found the queue full (their launch's overflow flags, nonzero bytes):
// only when the count passed the capacity. The workgroup's 64 lanes scan 64 flags at a
// time; lane 0 re-runs the flagged ones.
__global__ __launch_bounds__(64) void k_rerun_overflow(const RerunLaunch* launches,
                                                        int64_t n_launches,
                                                        const uint32_t* queue_n,
                                                        int64_t queue_cap, uint8_t* mem,
                                                        int64_t lane_bytes, int64_t lds_bytes) {
  extern __shared__ __attribute__((aligned(128))) uint8_t lane_lds[];
  if ((int64_t)*queue_n <= queue_cap) return;
  uint8_t* base = mem + (int64_t)blockIdx.x * lane_bytes;
  for (int64_t li = 0; li < n_launches; ++li) {
    const RerunLaunch& RL = launches[li];
    if (!RL.ovf) continue;
    for (int64_t b0 = (int64_t)blockIdx.x * 64; b0 < RL.n_eps; b0 += (int64_t)gridDim.x * 64) {
      const int64_t e = b0 + threadIdx.x;
      const uint32_t f = e < RL.n_eps ? RL.ovf[e] : 0u;
      uint64_t set = __ballot(f != 0u);
      if (threadIdx.x == 0) {
        while (set) {
          const int32_t k = __builtin_ctzll(set);
          set &= set - 1;
          const uint32_t fk = RL.ovf[b0 + k];
          rerun_episode(RL, b0 + k, fk & 0x7fu, base, lane_lds, lds_bytes, queue_n);
        }
      }
    }
  }
}

// LDS per one-wave workgroup: up to a whole CU's 160 KiB when the launch needs it, less the
// kernels' static LDS (k_nak_exact_rerun's hybrid ring, 128 B): lds_dynamic_max, so that
// static + dynamic never exceeds the CU (CPR_LDS_GUARD, kernels.h)
hipError_t launch_nak_exact_rerun(const RerunLaunch* launches, int64_t n_launches,
                                  const int64_t* queue, const uint32_t* queue_n,
                                  int64_t queue_cap, uint8_t* mem, int64_t lane_bytes,
                                  int64_t lds_bytes, int64_t lanes, hipStream_t st) {
  const int64_t room = std::min(lds_dynamic_max((const void*)k_nak_exact_rerun),
                                lds_dynamic_max((const void*)k_rerun_overflow)) / 128 * 128;
  int64_t cap = room;
  if (const char* v = getenv("CPR_RERUN_LDS_MAX"))  // tests: force the reduced-heap paths
    cap = std::min<int64_t>(cap, std::max<int64_t>(0, atoll(v)));
  int64_t lds = lds_bytes < cap ? lds_bytes : cap;
  if (lds > 64 * 1024) {
    // the attribute is per device: granted LDS cached per device id (0 = not yet asked),
    // concurrent first callers may both ask, which is harmless
    static std::atomic<int64_t> granted[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::atomic<int64_t>& g = granted[dev & 63];
    int64_t have = g.load(std::memory_order_acquire);
    if (have == 0) {
      const bool a = hipFuncSetAttribute((const void*)k_nak_exact_rerun,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)room) == hipSuccess;
      const bool b = hipFuncSetAttribute((const void*)k_rerun_overflow,
                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)room) == hipSuccess;
      have = a && b ? room : 64 * 1024 - 128;
      (void)hipGetLastError();
      g.store(have, std::memory_order_release);
    }
    if (lds > have) lds = have;
  }
  if (lds < 0) lds = 0;
  CPR_LDS_GUARD(k_nak_exact_rerun, lds);
  CPR_LDS_GUARD(k_rerun_overflow, lds);
  hipLaunchKernelGGL(k_nak_exact_rerun, dim3((unsigned)lanes), dim3(64), (size_t)lds, st,
                     launches, queue, queue_n, queue_cap, mem, lane_bytes, lds);
  hipLaunchKernelGGL(k_rerun_overflow, dim3((unsigned)lanes), dim3(64), (size_t)lds, st,
                     launches, n_launches, queue_n, queue_cap, mem, lane_bytes, lds);
  return hipGetLastError();
}

hipError_t launch_eth_run_episodes(const eth::EthParams& P, uint64_t seed, uint64_t first,
                                   int64_t n_eps, uint8_t* mem, int64_t lane_bytes,
                                   int64_t lanes, cpr_episode_record* recs, cpr_summary* sum,
                                   hipStream_t st, const NodeOut& no) {
  CPR_LAYOUT_GUARD(lane_bytes, eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  const unsigned blocks = (unsigned)(lanes / kBlock);
  hipLaunchKernelGGL(k_eth_run_episodes<SeedSource>, dim3(blocks), dim3(kBlock), 0, st, P,
                     SeedSource{seed, first}, n_eps, mem, lane_bytes, recs, sum, no);
  return hipGetLastError();
}

hipError_t launch_eth_replay_episodes(const eth::EthParams& P, const TraceSource& src, int64_t n_eps,
                                 uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                 cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                 const NodeOut& no) {
  CPR_LAYOUT_GUARD(lane_bytes, eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  hipLaunchKernelGGL(k_eth_run_episodes<TraceSource>, dim3((unsigned)(lanes / kBlock)),
                     dim3(kBlock), 0, st, P, src, n_eps, mem, lane_bytes, recs, sum, no);
  return hipGetLastError();
}

int eth_blocks_per_cu() {
  int blocks = 0;
  hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_eth_run_episodes<SeedSource>, kBlock, 0);
  if (e != hipSuccess || blocks <= 0) blocks = 2;
  return blocks;
}

// ---------------------------------------------------------------- lockstep gym lanes
// engine.ml reset/step with host actions (cpr_reset / cpr_step) and the on-device rollout,
// one lane region of eth_lane_bytes per env; reward = Δ head.rewards[0] (engine.ml:223)
struct EthSlot {
  eth::EthLane L;
  uint64_t ep;
  double last_ra;
  int32_t live;
};

// ethereum_ssz.ml:43-56 normalizers through ssz_tools.ml NormalizeObs.to_float; the unit
// encodings use host-tabulated libm values (tabs = [2/pi atan(i) | 0.5 + atan(i - N)/pi],
// i < N), the lanes' state decides the orphan fields with the three dry-run payloads
__device__ inline void eth_write_obs(const eth::EthObs& o, int unit, const double* tabs,
                                     int32_t tn, double* out) {
  const int32_t v[10] = {o.public_height,  o.public_work,
                         o.private_height, o.private_work,
                         o.diff_height,    o.diff_work,
                         o.public_orphans, o.private_orphans_inclusive,
                         o.private_orphans_exclusive, o.event};
  const double pi = 3.141592653589793;
  for (int j = 0; j < 10; ++j) {
    const int32_t x = v[j];
    if (!unit || j == 9) {
      out[j] = (double)x;
    } else if (j == 4 || j == 5) {
      out[j] = (x > -tn && x < tn) ? tabs[2 * tn + x] : 0.5 + (1.0 / pi * atan((double)x / 1.0));
    } else {
      out[j] = x < tn ? tabs[x] : 2.0 / pi * atan((double)x / 1.0);
    }
  }
}

__device__ inline void eth_slot_reset(const eth::EthParams& P, uint64_t seed, const eth::EthMem& M,
                                      EthSlot& SL, uint64_t ep) {
  SL.ep = ep;
  SL.last_ra = 0.0;
  SL.live = 1;
  SL.L.gym_reset(P, make_stream(seed, ep), M);
}

__device__ inline eth::EthMem eth_lane_mem(const eth::EthParams& P, uint8_t* mem,
                                           int64_t lane_bytes, int64_t i) {
  return eth::eth_mem_at(mem + i * lane_bytes, P.cap_b, P.cap_e, P.n);
}

__global__ __launch_bounds__(kBlock) void k_eth_reset(eth::EthParams P, uint64_t seed,
                                                       uint8_t* mem, int64_t lane_bytes,
                                                       EthSlot* slots, int64_t n,
                                                       const uint8_t* mask, const uint64_t* eps,
                                                       int unit, const double* tabs, int32_t tn,
                                                       double* obs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const eth::EthMem M = eth_lane_mem(P, mem, lane_bytes, i);
  EthSlot SL = slots[i];
  if (mask == nullptr || mask[i]) eth_slot_reset(P, seed, M, SL, eps ? eps[i] : (uint64_t)i);
  eth_write_obs(SL.L.observe(P, M, true), unit, tabs, tn, obs + 10 * i);
  slots[i] = SL;
}

__device__ inline void eth_info(const eth::EthParams& P, const eth::EthMem& M, EthSlot& SL,
                                int32_t hd, int64_t i, const StepBuffers& out) {
  const eth::EBlock& h = SL.L.B(P, M, hd);
  out.era[i] = (double)h.rew_att / 32.0;
  out.erd[i] = (double)h.rew_def / 32.0;
  out.eprog[i] = (double)h.work;
  out.ect[i] = h.time;
  out.est[i] = SL.L.now;
  out.esteps[i] = SL.L.steps;
  out.eacts[i] = SL.L.c_act;
  out.hh[i] = h.height;
  out.hm[i] = h.miner;
}

__global__ __launch_bounds__(kBlock) void k_eth_step(eth::EthParams P, uint64_t seed,
                                                      uint8_t* mem, int64_t lane_bytes,
                                                      EthSlot* slots, int64_t n,
                                                      const int32_t* actions, int unit,
                                                      const double* tabs, int32_t tn,
                                                      StepBuffers out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const eth::EthMem M = eth_lane_mem(P, mem, lane_bytes, i);
  EthSlot SL = slots[i];
  bool done = false;
  const int32_t hd = SL.L.gym_step(P, make_stream(seed, SL.ep), M, actions[i], &done);
  const double ra = (double)SL.L.B(P, M, hd).rew_att / 32.0;
  out.reward[i] = ra - SL.last_ra;  // engine.ml:223
  out.done[i] = done ? 1 : 0;
  out.status[i] = SL.L.status;
  if (out.era) eth_info(P, M, SL, hd, i, out);
  SL.last_ra = ra;
  eth_write_obs(SL.L.observe(P, M, true), unit, tabs, tn, out.obs + 10 * i);
  slots[i] = SL;
}

// n_steps lockstep steps per lane with the batch policy on the device, VecEnv auto-reset
// (episode id + n), as k_bk_rollout
__global__ __launch_bounds__(kBlock) CPR_EV_OCC void k_eth_rollout(eth::EthParams P, uint64_t seed,
                                                         uint8_t* mem, int64_t lane_bytes,
                                                         EthSlot* slots, int64_t n,
                                                         int64_t n_steps, int unit,
                                                         const double* tabs, int32_t tn,
                                                         double* obs, double* reward,
                                                         uint8_t* done_out, cpr_summary* sum) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Acc acc = {};
  int64_t steps_all = 0, acts_all = 0;
  if (i < n) {
    const eth::EthMem M = eth_lane_mem(P, mem, lane_bytes, i);
    EthSlot SL = slots[i];
    if (!SL.live) {
      eth_slot_reset(P, seed, M, SL, (uint64_t)i);
      acts_all += SL.L.c_act;
    }
    for (int64_t t = 0; t < n_steps; ++t) {
      const eth::EthObs o = SL.L.observe(P, M, false);
      const int32_t c0 = SL.L.c_act;
      bool done = false;
      const int32_t hd =
          SL.L.gym_step(P, make_stream(seed, SL.ep), M, eth::lane_action(P, o), &done);
      acts_all += SL.L.c_act - c0;
      ++steps_all;
      const eth::EBlock& h = SL.L.B(P, M, hd);
      const double ra = (double)h.rew_att / 32.0;
      const int64_t k = t * n + i;
      if (reward) reward[k] = ra - SL.last_ra;
      if (done_out) done_out[k] = done ? 1 : 0;
      SL.last_ra = ra;
      if (done) {
        const int32_t a = h.rew_att, d = h.rew_def;
        const double rel = (a + d) != 0 ? (double)a / (double)(a + d) : 0.0;
        acc_episode(acc, (int64_t)a << 15, (int64_t)d << 15, (int64_t)h.work << 20, rel,
                    h.height, SL.L.steps, SL.L.c_act, SL.L.status, hist);
        eth_slot_reset(P, seed, M, SL, SL.ep + (uint64_t)n);
        acts_all += SL.L.c_act;
      }
      if (obs) eth_write_obs(SL.L.observe(P, M, true), unit, tabs, tn, obs + 10 * k);
    }
    slots[i] = SL;
  }
  acc.steps = steps_all;
  acc.activations = acts_all;
  __syncthreads();
  block_flush(acc, hist, sum);
}

__global__ void k_eth_observe_fields(eth::EthParams P, uint8_t* mem, int64_t lane_bytes,
                                     const EthSlot* slots, int64_t n, int32_t* f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const eth::EthMem M = eth_lane_mem(P, mem, lane_bytes, i);
  eth::EthLane L = slots[i].L;
  const eth::EthObs o = L.observe(P, M, true);
  int32_t* g = f + 10 * i;
  g[0] = o.public_height;
  g[1] = o.public_work;
  g[2] = o.private_height;
  g[3] = o.private_work;
  g[4] = o.diff_height;
  g[5] = o.diff_work;
  g[6] = o.public_orphans;
  g[7] = o.private_orphans_inclusive;
  g[8] = o.private_orphans_exclusive;
  g[9] = o.event;
}

// engine.ml:258-261: decode (ssz_tools.ml NormalizeObs.of_float) and apply the policy
__global__ void k_eth_policy(int32_t policy, int unit, const double* obs, int64_t n,
                             const uint8_t* table, int32_t dim, int32_t* actions) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* x = obs + 10 * i;
  const double pi = 3.141592653589793;
  int32_t v[10];
  for (int j = 0; j < 10; ++j) {
    if (j == 9)
      v[j] = (int32_t)floor(x[j] * 1.0);
    else if (!unit)
      v[j] = (int32_t)x[j];
    else if (j == 4 || j == 5)
      v[j] = (int32_t)__builtin_round(tan(pi * (x[j] - 0.5)) * 1.0);
    else
      v[j] = (int32_t)__builtin_round(tan(pi / 2.0 * x[j]) * 1.0);
  }
  eth::EthObs o;
  o.public_height = v[0];
  o.public_work = v[1];
  o.private_height = v[2];
  o.private_work = v[3];
  o.diff_height = v[4];
  o.diff_work = v[5];
  o.public_orphans = v[6];
  o.private_orphans_inclusive = v[7];
  o.private_orphans_exclusive = v[8];
  o.event = v[9];
  actions[i] = eth::eth_policy_t(policy, o, table, dim);
}

static unsigned eth_grid_of(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

hipError_t launch_eth_reset(const eth::EthParams& P, uint64_t seed, uint8_t* mem,
                            int64_t lane_bytes, void* slots, int64_t n, const uint8_t* mask,
                            const uint64_t* eps, int unit, const double* tabs, int32_t tn,
                            double* obs, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  hipLaunchKernelGGL(k_eth_reset, dim3(eth_grid_of(n)), dim3(kBlock), 0, st, P, seed, mem,
                     lane_bytes, (EthSlot*)slots, n, mask, eps, unit, tabs, tn, obs);
  return hipGetLastError();
}

hipError_t launch_eth_step(const eth::EthParams& P, uint64_t seed, uint8_t* mem,
                           int64_t lane_bytes, void* slots, int64_t n, const int32_t* actions,
                           int unit, const double* tabs, int32_t tn, const StepBuffers& b,
                           hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  hipLaunchKernelGGL(k_eth_step, dim3(eth_grid_of(n)), dim3(kBlock), 0, st, P, seed, mem,
                     lane_bytes, (EthSlot*)slots, n, actions, unit, tabs, tn, b);
  return hipGetLastError();
}

hipError_t launch_eth_rollout(const eth::EthParams& P, uint64_t seed, uint8_t* mem,
                              int64_t lane_bytes, void* slots, int64_t n, int64_t n_steps,
                              int unit, const double* tabs, int32_t tn, double* obs,
                              double* reward, uint8_t* done, cpr_summary* sum, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  hipLaunchKernelGGL(k_eth_rollout, dim3(eth_grid_of(n)), dim3(kBlock), 0, st, P, seed, mem,
                     lane_bytes, (EthSlot*)slots, n, n_steps, unit, tabs, tn, obs, reward, done,
                     sum);
  return hipGetLastError();
}

hipError_t launch_eth_observe_fields(const eth::EthParams& P, uint8_t* mem, int64_t lane_bytes,
                                     const void* slots, int64_t n, int32_t* f, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  hipLaunchKernelGGL(k_eth_observe_fields, dim3(eth_grid_of(n)), dim3(kBlock), 0, st, P, mem,
                     lane_bytes, (const EthSlot*)slots, n, f);
  return hipGetLastError();
}

hipError_t launch_eth_policy(int32_t policy, int unit, const double* obs, int64_t n,
                             const uint8_t* table, int32_t dim, int32_t* actions,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_eth_policy, dim3(eth_grid_of(n)), dim3(kBlock), 0, st, policy, unit, obs,
                     n, table, dim, actions);
  return hipGetLastError();
}

size_t eth_slot_bytes() { return sizeof(EthSlot); }

}  // namespace cpr
