// HIP kernels for gfx950 (MI355X): one lane = one independent episode / gym env.
//
// Work is integer/branch (VALU) bound; nothing is a contraction, so no MFMA. Per-lane
// state lives in VGPRs; the mining times of the last 16 private-chain blocks live in LDS
// (32 KB per workgroup), deeper ones spill to HBM; every other block the lane can name
// carries its own mining time, so an activation stores nothing to HBM.
// Episode outcomes are reduced wave-wide with shuffles, then per workgroup in LDS, then
// one 64-bit atomic per field per workgroup, all in integer arithmetic so totals are
// independent of scheduling and of how episodes are sharded over GPUs.
// every kernel of this file takes one seed for the whole grid (cpr_stream.h)
#define CPR_UNIFORM_SEED 1
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/cpr_hip.h"
#include "kernels.h"
#include "nakamoto_lane.h"
#include "summary.h"

#pragma clang fp contract(off)

namespace cpr {

__device__ inline void acc_add(Acc& a, const BRef& hd, int64_t steps, int64_t acts,
                               uint32_t status, int32_t* hist_lds) {
  const double rel = hd.h != 0 ? (double)hd.ra / (double)hd.h : 0.0;
  acc_episode(a, (int64_t)hd.ra << 20, (int64_t)(hd.h - hd.ra) << 20, (int64_t)hd.h << 20, rel,
              hd.h, steps, acts, status, hist_lds);
}
__device__ inline void acc_add(LdsAcc& a, const BRef& hd, int64_t steps, int64_t acts,
                               uint32_t status, int32_t* hist_lds) {
  const double rel = hd.h != 0 ? (double)hd.ra / (double)hd.h : 0.0;
  a.episode((int64_t)hd.ra << 20, (int64_t)(hd.h - hd.ra) << 20, (int64_t)hd.h << 20, rel, hd.h,
            steps, acts, status, hist_lds);
}

// One gym episode (engine.ml:164-249): reset = first activation up to the attacker's
// interaction; step = apply, deliveries, next activation, observe; head at the end.
// LZ: the lazy clock (NakLane::lazy_overlap_check; 2 = with deferred races, races_check),
// launched only when the host's lazy_clock_ok holds and only max_steps ends the episode
template <int POL, int TT, class St, int LZ = 0>
__device__ inline CPR_AI BRef run_gym(NakLane& L, const NakParams& P, const St& S, const LaneMem& M,
                               int64_t* steps_out) {
  L.init();
  L.activate<St, LZ>(P, S, M);
  const bool check_prog = P.max_progress < __builtin_inf();
  int64_t steps = 0;
  if (LZ || (!check_prog && !(P.max_time < __builtin_inf()))) {
    // only max_steps ends the episode: the trip count is the same in every lane of the
    // wave, so the loop exit is uniform and no lane state is merged at a divergent exit
    do {
      const NakLane::Draw dr = L.draw<St, LZ>(P, S);
      L.apply(L.policy_action<POL>(P));
      L.resolve<St, POL >= 0 ? 0 : -1, TT>(P, S, M);
      if constexpr (TT == 2) enqueue_race<LZ>(L, M);
      L.activate<St, LZ>(P, S, M, dr);
      ++steps;
      // the lanes of the wave verify together once the wave's list is nearly full
      if constexpr (TT == 2) {
        if (races_due(L, M)) verify_races<St, LZ>(L, P, S, M);
      }
    } while (steps < P.max_steps);
    if constexpr (TT == 2) verify_races<St, LZ>(L, P, S, M);
    *steps_out = steps;
    return L.head(P, M);
  }
  for (;;) {
    const int32_t a = L.policy_action<POL>(P);
    L.apply(a);
    L.resolve<St, POL >= 0 ? 0 : -1, TT == 2 ? 1 : TT>(P, S, M);
    L.activate(P, S, M);
    ++steps;
    bool go = steps < P.max_steps && L.t < P.max_time;
    if (check_prog && go) go = (double)L.head(P, M).h < P.max_progress;
    if (!go) break;
  }
  *steps_out = steps;
  return L.head(P, M);
}

// Simulator.loop ~activations with the SSZ attacker as node 0 (simulator.ml:519-533,
// nakamoto_ssz.ml:262-272); all messages delivered before the head is taken.
template <int POL, class St>
__device__ inline CPR_AI BRef run_loop(NakLane& L, const NakParams& P, const St& S, const LaneMem& M,
                                int64_t activations) {
  L.init();
  for (int64_t i = 0; i < activations; ++i) {
    L.activate(P, S, M);
    L.apply(L.policy_action<POL>(P));
    L.resolve(P, S, M);
  }
  return L.head(P, M);
}

// The episode after e (k_run_episodes): with a work-queue counter, the wave's live lanes
// take the next 64 episodes together (one atomic by the lowest live lane, broadcast), so a
// wave that runs ahead takes more episodes and a launch ends within about one episode of
// its slowest wave instead of after a fixed share per wave; the lanes of a wave keep
// consecutive episodes started together, so their activation counts stay equal (the keyed
// counter and the deferred races' wave list rely on it). Without: the static grid stride
__device__ inline CPR_AI int64_t nak_next_episode(unsigned long long* next, int64_t e,
                                                  int64_t nthreads) {
  if (next == nullptr) return e + nthreads;
  const uint64_t live = __ballot(1);
  const int32_t leader = __builtin_ctzll(live);
  const int32_t lane = (int32_t)(threadIdx.x % WAVE);
  unsigned long long base = 0ull;
  if (lane == leader) base = atomicAdd(next, (unsigned long long)WAVE);
  base = __shfl(base, leader);
  return nthreads + (int64_t)base + lane;
}

// lane status bits whose episodes the closed form cannot vouch for
constexpr uint32_t kInexact = ST_OVERLAP | ST_DEEP_FORK | ST_TIE_UNRESOLVED | ST_STALE_TIME;

// POL: nakamoto_ssz policy fixed at compile time (P_HONEST .. P_SM1; these kernels never
// run the abstract-gamma mode), or -1 for P.policy (and P.abstract_g)
// REC: 1 = per-episode records may be written (block mining times tracked for chain_time);
// 0 = summary only (recs is null): the lane's time bookkeeping compiles out (LaneMem.times)
// ARR: P.arrive fixed at compile time (0: attacker messages never reach the defenders, the
// gym's gamma = 0 network, so the second defender tip, the races and the tie replay drop
// out; 1: they do), or -1 to read it from P
// TT: 1 = launched for d = 2 only: ties take the closed-form rule (tie_table_d2) instead
// of the inlined heap replay, whose registers otherwise stay live across the whole loop;
// 2 = as 1, and the races are deferred and verified in batches (verify_races; REC = 0 only:
// the race lists take the LDS ring); an episode a race went otherwise in is listed in
// `list` (count, then episode indices) for the eager second pass (ListSource, TT = 1)
// LZ: lazy clock (REC = 0 only; 1 at ARR = 0, 2 with the deferred races TT = 2)
template <int MODE, class Src, int POL, int REC = 1, int ARR = -1, int TT = 0, int LZ = 0>
#ifndef CPR_G0_WAVES
#define CPR_G0_WAVES 8  // the gamma = 0 kernel: 61 VGPRs fit 8 waves/SIMD (7 unasked)
#endif
#ifndef CPR_TT_WAVES
#define CPR_TT_WAVES 5  // the d = 2 tie-rule kernels (96 VGPRs)
#endif
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ARR == 0 ? CPR_G0_WAVES : (TT ? CPR_TT_WAVES : 4)))) void k_run_episodes(
    NakParams P, Src src, int64_t n_eps, int64_t activations,
    double* spill, uint8_t* replay, cpr_episode_record* recs, cpr_summary* sum,
    int64_t* redo, uint32_t* redo_n, uint32_t launch_id, int64_t redo_cap, int64_t* list,
    uint8_t* ovf) {
  // the race lists take the LDS ring, which only the summary-only kernels leave free
  static_assert(TT != 2 || REC == 0, "deferred races need the summary-only kernel");
  static_assert(!LZ || (REC == 0 && MODE == CPR_MODE_GYM && (LZ == 1 ? ARR == 0 : TT == 2)),
                "the lazy clock is for the summary-only gym kernels (gamma = 0, deferred races)");
  if (ARR >= 0) P.arrive = ARR;
  if (TT) P.d = 2;  // launched for two defenders only (gym_run_fn): masks and loops fold
  __shared__ int32_t hist[CPR_HIST_BINS];
  // TT = 2 (summary only): the ring holds the race queue alone, sized so that five
  // workgroups fit a CU's LDS
  __shared__ double ring[(REC || TT != 2 ? RING : 2 * RQ_LANE) * kBlock];
  __shared__ int32_t rflag[TT == 2 ? kBlock : 1];
  __shared__ uint32_t rep[TT == 2 ? 2 * kBlock : 1];
  __shared__ unsigned long long acc_w[13];
  LdsAcc acc{acc_w};
  acc.init();
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  LaneMem M;
  M.ring = ring + threadIdx.x;
  M.ring_stride = kBlock;
  // spill per lane, contiguous: a lane's evictions are consecutive words, which the L2
  // merges into whole lines over time. (Interleaving it [slot][lane] like the LDS ring was
  // measured 9 % slower per launch: lanes of a wave evict at different depths, so their
  // words rarely share a line anyway; profiles/r03e_nak_ab.log)
  M.spill = spill + tid * P.cap;
  M.spill_stride = 1;
  M.cap = P.cap;
  M.replay = ReplayMem::at(replay + tid * REPLAY_BYTES);
  M.times = REC != 0;
  if (!REC) recs = nullptr;
  if (TT == 2) {
    // summary-only: the ring holds no block times; each wave's race list takes its share
    M.rq = reinterpret_cast<uint4*>(ring) + (threadIdx.x / WAVE) * (RQ_LANE * WAVE);
    M.rq_cap = RQ_LANE * WAVE;
    M.rflag = rflag + (threadIdx.x / WAVE) * WAVE;
    M.rep = rep + (threadIdx.x / WAVE) * (2 * WAVE);
    M.lane = (int32_t)(threadIdx.x % WAVE);
    M.wave = WAVE;
    M.rflag[M.lane] = 0;
  }
  NakLane L;
  const int64_t n_run = src.size(n_eps);
  for (int64_t e = tid; e < n_run; e = nak_next_episode(P.next, e, nthreads)) {
    const auto S = src.at(e);
    int64_t steps = 0;
    const BRef hd = MODE == CPR_MODE_GYM ? run_gym<POL, TT, std::remove_const_t<decltype(S)>, LZ>(L, P, S, M, &steps)
                                         : run_loop<POL>(L, P, S, M, activations);
    if constexpr (TT == 2) {
      if (L.status & ST_RACE_REDO) {
        // a deferred race went otherwise: the eager pass runs this episode again (list:
        // count, then episode indices; room for every episode of the launch)
        const uint32_t r = atomicAdd(reinterpret_cast<uint32_t*>(list), 1u);
        list[1 + r] = src.index(e);
        continue;
      }
    }
    const double tm = L.time_of(M, hd);
    const uint32_t status = L.status | Src::missed(S);
    uint32_t st_out = status;
    if (redo != nullptr && !P.abstract_g && (status & kInexact) != 0u) {
      // the closed form does not hold for this episode: hand it to the exact event engine
      // (k_nak_exact_rerun), which writes its record and summary contribution
      const uint32_t r = atomicAdd(redo_n, 1u);
      if ((int64_t)r < redo_cap) {
        redo[r] = ((int64_t)launch_id << 40) | (src.index(e) << 8) | (int64_t)(status & 0xffu);
      } else {
        // queue full: the episode waits in the launch's overflow flags, which the re-run
        // pass scans after the queue (k_rerun_overflow)
        ovf[src.index(e)] = (uint8_t)(0x80u | (status & 0x7fu));
      }
      continue;
    } else if (P.abstract_g && (status & kInexact) != 0u) {
      st_out |= CPR_ST_CAPACITY;  // the exact event engine has no abstract-gamma mode
    }
    acc_add(acc, hd, steps, L.k, st_out, hist);
    if (REC && recs) {
      cpr_episode_record r;
      r.reward_attacker = (double)hd.ra;
      r.reward_defender = (double)(hd.h - hd.ra);
      r.progress = (double)hd.h;
      r.chain_time = tm;
      r.sim_time = MODE == CPR_MODE_GYM ? L.t : 0.0;
      r.n_steps = steps;
      r.n_activations = L.k;
      r.head_height = hd.h;
      r.head_miner = MODE == CPR_MODE_GYM ? miner_of(P, S, hd.k) : -1;
      r.status = st_out;
      r.head_work = 0;
      recs[src.index(e)] = r;
    }
  }
  __syncthreads();
  acc.flush(hist, sum);
}

// ---- lockstep gym lanes (engine.reset / engine.step over n lanes)

struct LockLane {
  NakLane L;
  uint64_t ep;
  int64_t steps;
  double last_ra;
  int32_t live;
  int32_t exact;  // 1 + the exact-engine slot this lane runs on, 0 = the closed form
};

// nakamoto_ssz action (0 Adopt .. 3 Wait) -> the Nakamoto-mode Ethereum lane's action index
// (eth::lane_action's mapping)
__device__ inline int32_t nak_to_eth_action(int32_t a) {
  constexpr int32_t map[4] = {eth::A_ADOPT_DISCARD, eth::A_OVERRIDE, eth::A_MATCH, eth::A_WAIT};
  return map[a & 3] * 4;
}

__device__ inline LaneMem lock_mem(const NakParams& P, const LockBuffers& B, int64_t i, int64_t n) {
  LaneMem M;
  M.ring = B.ring + i;
  M.ring_stride = n;
  M.spill = B.spill + i * P.cap;  // per lane, contiguous, as the fused kernel's
  M.spill_stride = 1;
  M.cap = P.cap;
  M.replay = ReplayMem::at(B.replay + i * REPLAY_BYTES);
  return M;
}

__device__ inline void write_obs_fields(int32_t h, int32_t a, int32_t d, int32_t ev, int unit,
                                        const double* tab_nn, const double* tab_sg,
                                        int32_t tab_n, double* o) {
  if (unit) {
    // ssz_tools.ml:29-40; host-tabulated (libm) for |x| < tab_n
    o[0] = h < tab_n ? tab_nn[h] : 2.0 / 3.141592653589793 * atan((double)h / 1.0);
    o[1] = a < tab_n ? tab_nn[a] : 2.0 / 3.141592653589793 * atan((double)a / 1.0);
    o[2] = (d > -tab_n && d < tab_n) ? tab_sg[d + tab_n]
                                     : 0.5 + (1.0 / 3.141592653589793 * atan((double)d / 1.0));
    o[3] = (double)ev / 1.0;
  } else {
    o[0] = (double)h;
    o[1] = (double)a;
    o[2] = (double)d;
    o[3] = (double)ev;
  }
}

__device__ inline void write_obs(const NakLane& L, int unit, const double* tab_nn,
                                 const double* tab_sg, int32_t tab_n, double* o) {
  int32_t h, a, d, ev;
  L.observe(&h, &a, &d, &ev);
  write_obs_fields(h, a, d, ev, unit, tab_nn, tab_sg, tab_n, o);
}

// a lockstep lane's slot on the exact event engine (k_lock_exact)
__device__ inline eth::EthMem lock_exact_mem(const eth::EthParams& EP, const LockBuffers& B,
                                             int32_t slot) {
  return eth::eth_mem_at(B.emem + (int64_t)slot * B.elane_bytes, EP.cap_b, EP.cap_e, EP.n);
}

__global__ __launch_bounds__(kBlock) void k_reset(NakParams P, eth::EthParams EP, uint64_t seed,
                                                   LockBuffers B, int64_t n, const uint8_t* mask,
                                                   const uint64_t* eps, int unit,
                                                   const double* tab_nn, const double* tab_sg,
                                                   int32_t tab_n, double* obs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  LockLane& LL = ((LockLane*)B.lanes)[i];
  if (mask != nullptr && !mask[i] && LL.exact > 0) {
    // a lane left unreset that runs on the exact engine: its observation is the exact
    // lane's (engine.ml:122-170 returns every env's current observation)
    eth::EthLane E = ((eth::EthLane*)B.eslots)[LL.exact - 1];
    const eth::EthObs o = E.observe(EP, lock_exact_mem(EP, B, LL.exact - 1), false);
    write_obs_fields(o.public_height, o.private_height, o.diff_height, o.event, unit, tab_nn,
                     tab_sg, tab_n, obs + 4 * i);
    return;
  }
  if (mask == nullptr || mask[i]) {
    if (LL.exact > 0) {  // the lane's exact-engine slot goes back to the free stack
      const int32_t t = atomicAdd(B.efree + B.n_slots, 1);
      B.efree[t] = LL.exact - 1;
    }
    LL.exact = 0;
    const LaneMem M = lock_mem(P, B, i, n);
    NakLane L;
    L.init();
    const uint64_t ep = eps ? eps[i] : (uint64_t)i;
    L.activate(P, make_stream(seed, ep), M);
    LL.L = L;
    LL.ep = ep;
    LL.steps = 0;
    LL.last_ra = 0.0;
    LL.live = 1;
  }
  write_obs(LL.L, unit, tab_nn, tab_sg, tab_n, obs + 4 * i);
}

__global__ __launch_bounds__(kBlock) void k_step(NakParams P, uint64_t seed, LockBuffers B,
                                                  int64_t n, const int32_t* actions, int unit,
                                                  const double* tab_nn, const double* tab_sg,
                                                  int32_t tab_n, StepBuffers out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  LockLane& LL = ((LockLane*)B.lanes)[i];
  if (B.alog && LL.steps < B.alog_cap) B.alog[i * B.alog_cap + LL.steps] = (uint8_t)actions[i];
  if (LL.exact) return;  // stepped on the exact engine by k_lock_exact
  NakLane L = LL.L;
  const LaneMem M = lock_mem(P, B, i, n);
  const Stream S = make_stream(seed, LL.ep);
  L.apply(actions[i]);
  L.resolve(P, S, M);
  L.activate(P, S, M);
  LL.steps += 1;
  const BRef hd = L.head(P, M);
  const double progress = (double)hd.h;
  const bool done = !(LL.steps < P.max_steps && progress < P.max_progress && L.t < P.max_time);
  const double ra = (double)hd.ra;
  out.reward[i] = ra - LL.last_ra;  // engine.ml:223
  out.done[i] = done ? 1 : 0;
  out.status[i] = L.status;
  if (out.era) {
    out.era[i] = ra;
    out.erd[i] = (double)(hd.h - hd.ra);
    out.eprog[i] = progress;
    out.ect[i] = L.time_of(M, hd);
    out.est[i] = L.t;
    out.esteps[i] = LL.steps;
    out.eacts[i] = L.k;
    out.hh[i] = hd.h;
    out.hm[i] = miner_of(P, S, hd.k);
  }
  LL.last_ra = ra;
  LL.L = L;
  write_obs(L, unit, tab_nn, tab_sg, tab_n, out.obs + 4 * i);
}

// lockstep lanes that left the closed form: engine.ml's step is always
// exact (engine.ml:176-249), so a lane whose step set CPR_ST_LOCKSTEP_INEXACT bits is
// simulated again on the exact event engine (Ethereum lane, Nakamoto mode) from its first
// draw with the actions it was given, and stays there until its next reset; this step's
// outputs are rewritten from that lane (status: the closed form's bits | EXACT_RERUN)

__global__ __launch_bounds__(kBlock) void k_lock_exact(eth::EthParams EP, uint64_t seed,
                                                        LockBuffers B, int64_t n,
                                                        const int32_t* actions, int unit,
                                                        const double* tab_nn,
                                                        const double* tab_sg, int32_t tab_n,
                                                        StepBuffers out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  LockLane& LL = ((LockLane*)B.lanes)[i];
  eth::EthLane* slots = (eth::EthLane*)B.eslots;
  const Stream S = make_stream(seed, LL.ep);
  int32_t hd;
  bool done = false;
  int32_t slot;
  eth::EthLane E;
  double prev_ra = LL.last_ra;  // attacker reward after the previous step
  if (LL.exact) {
    slot = LL.exact - 1;
    E = slots[slot];
    hd = E.gym_step(EP, S, lock_exact_mem(EP, B, slot), nak_to_eth_action(actions[i]), &done);
    LL.steps += 1;
  } else {
    if (!(LL.L.status & kInexact) || LL.steps > B.alog_cap) return;
    const int32_t t = atomicSub(B.efree + B.n_slots, 1) - 1;
    if (t < 0) {  // every slot taken: the lane keeps its flags (inexact outputs)
      atomicAdd(B.efree + B.n_slots, 1);
      return;
    }
    slot = B.efree[t];
    // k_step already advanced last_ra by this step's closed-form reward (whole blocks:
    // exact in fp64), so the previous step's value is the difference
    prev_ra = LL.last_ra - out.reward[i];
    const eth::EthMem M = lock_exact_mem(EP, B, slot);
    E.gym_reset(EP, S, M);
    hd = 0;
    for (int64_t s = 0; s < LL.steps; ++s)
      hd = E.gym_step(EP, S, M, nak_to_eth_action(B.alog[i * B.alog_cap + s]), &done);
    LL.exact = slot + 1;
  }
  const eth::EthMem M = lock_exact_mem(EP, B, slot);
  const eth::EBlock h = E.B(EP, M, hd);
  const double ra = (double)(h.rew_att / 32);  // 1 per block in Nakamoto mode
  out.reward[i] = ra - prev_ra;  // engine.ml:223
  out.done[i] = done ? 1 : 0;
  out.status[i] = LL.L.status | E.status | CPR_ST_EXACT_RERUN;
  if (out.era) {
    out.era[i] = ra;
    out.erd[i] = (double)(h.rew_def / 32);
    out.eprog[i] = (double)h.height;
    out.ect[i] = h.time;
    out.est[i] = E.now;
    out.esteps[i] = E.steps;
    out.eacts[i] = E.c_act;
    out.hh[i] = h.height;
    out.hm[i] = h.miner;
  }
  LL.last_ra = ra;
  const eth::EthObs o = E.observe(EP, M, false);
  slots[slot] = E;
  write_obs_fields(o.public_height, o.private_height, o.diff_height, o.event, unit, tab_nn,
                   tab_sg, tab_n, out.obs + 4 * i);
}

__global__ void k_observe_fields(eth::EthParams EP, LockBuffers B, int64_t n, int32_t* f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const LockLane& LL = ((const LockLane*)B.lanes)[i];
  if (LL.exact) {
    eth::EthLane E = ((eth::EthLane*)B.eslots)[LL.exact - 1];
    const eth::EthObs o = E.observe(EP, lock_exact_mem(EP, B, LL.exact - 1), false);
    f[4 * i] = o.public_height;
    f[4 * i + 1] = o.private_height;
    f[4 * i + 2] = o.diff_height;
    f[4 * i + 3] = o.event;
    return;
  }
  LL.L.observe(f + 4 * i, f + 4 * i + 1, f + 4 * i + 2, f + 4 * i + 3);
}

// engine.ml:258-261: decode the observation (ssz_tools.ml:42-59), apply the policy
__global__ void k_policy(int32_t policy, int unit, const double* obs, int64_t n,
                         const uint8_t* table, int32_t dim, int32_t* actions) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* o = obs + 4 * i;
  int32_t h, a, ev;
  if (unit) {
    h = (int32_t)__builtin_round(tan(3.141592653589793 / 2.0 * o[0]) * 1.0);
    a = (int32_t)__builtin_round(tan(3.141592653589793 / 2.0 * o[1]) * 1.0);
    ev = (int32_t)floor(o[3] * 1.0);
  } else {
    h = (int32_t)o[0];
    a = (int32_t)o[1];
    ev = (int32_t)o[3];
  }
  actions[i] = nak_policy(policy, h, a, ev, table, dim);
}

__global__ void k_stream_fill(uint64_t seed, uint64_t ep, uint32_t idx0, uint32_t tag, int64_t n,
                              uint32_t* out, double* exp_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Stream S = make_stream(seed, ep);
  const Words4 w = S.block(idx0 + (uint32_t)i, tag);
  out[4 * i] = w.w0;
  out[4 * i + 1] = w.w1;
  out[4 * i + 2] = w.w2;
  out[4 * i + 3] = w.w3;
  if (exp_out) exp_out[i] = (-1.0 * 1.0) * cpr_log(u53(w.w2, w.w3));
}

// ---------------------------------------------------------------- launchers

// the k_run_episodes instantiation a launch runs (keyed stream): the built-in policies get
// their own specialisation, and summary-only ones (no records asked for: no block-time
// bookkeeping) for either kind of network; the flagged abstract-gamma mode, tables and loop
// tasks run the generic kernel. Template arguments do not change the signature.
using RunFn = void (*)(NakParams, SeedSource, int64_t, int64_t, double*, uint8_t*,
                       cpr_episode_record*, cpr_summary*, int64_t*, uint32_t*, uint32_t, int64_t,
                       int64_t*, uint8_t*);
// deferred races (TT = 2) pay where the release always reaches the non-miner defender no
// later than the defender block (dmax <= delta: the gym's gamma <= .5 networks), so that a
// verification almost never sends an episode to the second pass; they need release indices
// that fit a list entry (the second pass's list has its own buffer, run_episodes_list_bytes)
#ifndef CPR_DEFER_RACES
#define CPR_DEFER_RACES 1
#endif
#ifndef CPR_LAZY_CLOCK  // 0: the gamma = 0 summary kernel draws every clock (A/B runs)
#define CPR_LAZY_CLOCK 1
#endif
static bool deferred_races_ok(const NakParams& P) {
  return CPR_DEFER_RACES && P.dmax <= P.delta && P.cap <= 4096;
}
using ListFn = void (*)(NakParams, ListSource, int64_t, int64_t, double*, uint8_t*,
                        cpr_episode_record*, cpr_summary*, int64_t*, uint32_t*, uint32_t, int64_t,
                        int64_t*, uint8_t*);
template <int POL>
static RunFn gym_run_fn(const NakParams& P, bool recs, bool defer, ListFn* second) {
  if (recs) return k_run_episodes<CPR_MODE_GYM, SeedSource, POL, 1, -1>;
  if (!P.arrive && lazy_clock_ok(P) && CPR_LAZY_CLOCK)
    return k_run_episodes<CPR_MODE_GYM, SeedSource, POL, 0, 0, 0, 1>;
  if (!P.arrive) return k_run_episodes<CPR_MODE_GYM, SeedSource, POL, 0, 0>;
  if (P.d != 2) return k_run_episodes<CPR_MODE_GYM, SeedSource, POL, 0, 1>;
  if (!defer) return k_run_episodes<CPR_MODE_GYM, SeedSource, POL, 0, 1, 1>;
  if (second) *second = k_run_episodes<CPR_MODE_GYM, ListSource, POL, 0, 1, 1>;
  if (lazy_clock_ok(P) && CPR_LAZY_CLOCK)
    return k_run_episodes<CPR_MODE_GYM, SeedSource, POL, 0, 1, 2, 2>;
  return k_run_episodes<CPR_MODE_GYM, SeedSource, POL, 0, 1, 2>;
}
// second: set to the eager second pass when the launch defers its races (else untouched)
static RunFn run_fn(const NakParams& P, int32_t mode, bool recs, bool defer = false,
                    ListFn* second = nullptr) {
  if (mode != CPR_MODE_GYM) return k_run_episodes<CPR_MODE_LOOP, SeedSource, -1>;
  if (P.abstract_g) return k_run_episodes<CPR_MODE_GYM, SeedSource, -1>;
  switch (P.policy) {
    case P_HONEST: return gym_run_fn<P_HONEST>(P, recs, defer, second);
    case P_SIMPLE: return gym_run_fn<P_SIMPLE>(P, recs, defer, second);
    case P_ES2014: return gym_run_fn<P_ES2014>(P, recs, defer, second);
    case P_SM1: return gym_run_fn<P_SM1>(P, recs, defer, second);
    default: return k_run_episodes<CPR_MODE_GYM, SeedSource, -1>;
  }
}

hipError_t launch_run_episodes(const NakParams& P0, uint64_t seed, uint64_t first, int64_t n_eps,
                               int32_t mode, int64_t activations, double* spill,
                               uint8_t* replay, int64_t* list, int64_t lanes,
                               cpr_episode_record* recs, cpr_summary* sum, int64_t* redo,
                               uint32_t* redo_n, uint32_t launch_id, int64_t redo_cap,
                               uint8_t* ovf, hipStream_t st, const SidePass* side) {
  const unsigned blocks = (unsigned)(lanes / kBlock);
  const SeedSource src{seed, first};
  if (side) *side->ran = false;
  ListFn second = nullptr;
  const RunFn fn = run_fn(P0, mode, recs != nullptr, list != nullptr && deferred_races_ok(P0),
                          &second);
  NakParams P = P0;
  P.u_lazy = lazy_clock_ok(P0) ? lazy_threshold(P0) : 0ull;
  // deferred races: `list` (1 + n_eps words) receives the episodes for the eager second
  // pass, its count first
  if (second) {
    const hipError_t er = hipMemsetAsync(list, 0, sizeof(int64_t), st);
    if (er != hipSuccess) return er;
  }
  hipLaunchKernelGGL(fn, dim3(blocks), dim3(kBlock), 0, st, P, src, n_eps, activations, spill,
                     replay, recs, sum, redo, redo_n, launch_id, redo_cap, list, ovf);
  if (second) {
    // a few episodes in a hundred (~1 % eager, ~3.5 % with the lazy clock, whose races
    // near a tie cannot be decided without the clock): the whole grid runs them in one round
    // (more take more rounds of the same grid-stride loop); blocks without an episode exit
    // at once
    const ListSource ls{src, reinterpret_cast<const uint32_t*>(list), list + 1};
    const unsigned b2 = blocks;
    P.next = nullptr;  // the second pass: the static grid stride over the listed episodes
    hipStream_t s2 = st;
    if (side) {
      // on the side stream, behind this launch's main kernel: it overlaps the next launch
      // on `st`. The summary-only d = 2 kernels touch neither the spill nor the tie-replay
      // scratch (no block times; ties by tie_table_d2), which the next launch may use, so
      // the second pass gets neither
      hipError_t e = hipEventRecord(side->main_done, st);
      if (e == hipSuccess) e = hipStreamWaitEvent(side->stream, side->main_done, 0);
      if (e != hipSuccess) return e;
      s2 = side->stream;
      spill = nullptr;
      replay = nullptr;
    }
    hipLaunchKernelGGL(second, dim3(b2), dim3(kBlock), 0, s2, P, ls, n_eps, activations, spill,
                       replay, recs, sum, redo, redo_n, launch_id, redo_cap, list, ovf);
    if (side) {
      const hipError_t e = hipEventRecord(side->done, s2);
      if (e != hipSuccess) return e;
      *side->ran = true;
    }
  }
  return hipGetLastError();
}

// the second pass's list of a launch of n_eps episodes (0: no deferred races for P)
int64_t run_episodes_list_bytes(const NakParams& P, int32_t mode, bool recs, int64_t n_eps) {
  if (mode != CPR_MODE_GYM || recs || !deferred_races_ok(P)) return 0;
  return (n_eps + 1) * (int64_t)sizeof(int64_t);
}

hipError_t launch_replay_episodes(const NakParams& P, const TraceSource& src, int64_t n_eps,
                                  int32_t mode, int64_t activations, double* spill,
                                  uint8_t* replay, int64_t lanes,
                                  cpr_episode_record* recs, cpr_summary* sum, int64_t* redo,
                                  uint32_t* redo_n, uint32_t launch_id, int64_t redo_cap,
                                  uint8_t* ovf, hipStream_t st) {
  const unsigned blocks = (unsigned)(lanes / kBlock);
  if (mode == CPR_MODE_GYM)
    hipLaunchKernelGGL((k_run_episodes<CPR_MODE_GYM, TraceSource, -1>), dim3(blocks), dim3(kBlock), 0,
                       st, P, src, n_eps, activations, spill, replay, recs, sum, redo, redo_n, launch_id, redo_cap,
                       nullptr, ovf);
  else
    hipLaunchKernelGGL((k_run_episodes<CPR_MODE_LOOP, TraceSource, -1>), dim3(blocks), dim3(kBlock),
                       0, st, P, src, n_eps, activations, spill, replay, recs, sum, redo, redo_n, launch_id, redo_cap,
                       nullptr, ovf);
  return hipGetLastError();
}

hipError_t launch_reset(const NakParams& P, const eth::EthParams& EP, uint64_t seed,
                        const LockBuffers& B, int64_t n, const uint8_t* mask, const uint64_t* eps,
                        int unit, const double* tab_nn, const double* tab_sg, int32_t tab_n,
                        double* obs, hipStream_t st) {
  const unsigned blocks = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_reset, dim3(blocks), dim3(kBlock), 0, st, P, EP, seed, B, n, mask, eps,
                     unit, tab_nn, tab_sg, tab_n, obs);
  return hipGetLastError();
}

hipError_t launch_step(const NakParams& P, uint64_t seed, const LockBuffers& B, int64_t n,
                       const int32_t* actions, int unit, const double* tab_nn,
                       const double* tab_sg, int32_t tab_n, const StepBuffers& b,
                       hipStream_t st) {
  const unsigned blocks = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_step, dim3(blocks), dim3(kBlock), 0, st, P, seed, B, n, actions, unit,
                     tab_nn, tab_sg, tab_n, b);
  return hipGetLastError();
}

hipError_t launch_lock_exact(const eth::EthParams& EP, uint64_t seed, const LockBuffers& B,
                             int64_t n, const int32_t* actions, int unit, const double* tab_nn,
                             const double* tab_sg, int32_t tab_n, const StepBuffers& b,
                             hipStream_t st) {
  if (!B.alog) return hipSuccess;
  const unsigned blocks = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_lock_exact, dim3(blocks), dim3(kBlock), 0, st, EP, seed, B, n, actions,
                     unit, tab_nn, tab_sg, tab_n, b);
  return hipGetLastError();
}

hipError_t launch_observe_fields(const eth::EthParams& EP, const LockBuffers& B, int64_t n,
                                 int32_t* f, hipStream_t st) {
  const unsigned blocks = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_observe_fields, dim3(blocks), dim3(kBlock), 0, st, EP, B, n, f);
  return hipGetLastError();
}

hipError_t launch_policy(int32_t policy, int unit, const double* obs, int64_t n,
                         const uint8_t* table, int32_t dim, int32_t* actions, hipStream_t st) {
  const unsigned blocks = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_policy, dim3(blocks), dim3(kBlock), 0, st, policy, unit, obs, n, table,
                     dim, actions);
  return hipGetLastError();
}

hipError_t launch_stream_fill(uint64_t seed, uint64_t ep, uint32_t idx0, uint32_t tag, int64_t n,
                              uint32_t* out, double* exp_out, hipStream_t st) {
  const unsigned blocks = (unsigned)((n + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_stream_fill, dim3(blocks), dim3(kBlock), 0, st, seed, ep, idx0, tag, n,
                     out, exp_out);
  return hipGetLastError();
}

size_t lock_lane_bytes() { return sizeof(LockLane); }

// occupancy of the instantiation a launch runs (the deferred-race kernel holds more LDS)
int run_episodes_blocks_per_cu(const NakParams& P, int32_t mode, bool recs) {
  int blocks = 0;
  ListFn second = nullptr;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &blocks, (const void*)run_fn(P, mode, recs, deferred_races_ok(P), &second), kBlock, 0);
  if (e != hipSuccess || blocks <= 0) blocks = 2;
  return blocks;
}

}  // namespace cpr
