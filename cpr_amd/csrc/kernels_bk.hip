// B_k kernels for gfx950: one lane = one episode / gym env of the bk_ssz attack space,
// driven by the exact per-lane event engine of bk_lane.h. Each lane owns one contiguous
// HBM region (vertex ring, per-node visibility and times, quorums, drafts, event heap,
// scratch) reused for every episode it runs.
//
//   k_bk_run_episodes  fused reset/(policy, step)* episodes, or Simulator.loop tasks
//   k_bk_reset/k_bk_step  lockstep gym API (engine.ml reset / step) with host actions
//   k_bk_rollout       lockstep rollout on the device: every lane takes n_steps steps with
//                      the batch policy (built-in or table), auto-resetting finished
//                      episodes like a gym VecEnv (BASELINE configs[4])
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "../../include/cpr_hip.h"
#include "bk_lane.h"
#include "kernels.h"
#include "summary.h"
#include "wave_sched.h"

#pragma clang fp contract(off)

namespace cpr {

// engine.ml reward = Δ head.rewards[0]; episode ids of lane i in a rollout: i, i + n, ...
struct BkSlot {
  bk::BkLane L;
  uint64_t ep;
  double last_ra;
  int32_t head;
  int32_t live;
};

__device__ inline void bk_acc(Acc& acc, const bk::BkParams& P, const bk::BkLane& L,
                              const bk::BVtx& h, int32_t* hist) {
  const int32_t ra = h.rew_att, rd = h.rew_def;
  const double rel = (ra + rd) != 0 ? (double)ra / (double)(ra + rd) : 0.0;
  // orphans: activations (votes) not confirmed by the head's chain
  acc_episode(acc, (int64_t)ra << 20, (int64_t)rd << 20, (int64_t)h.height * P.k << 20, rel,
              (int64_t)h.height * P.k, L.steps, L.c_act, L.status, hist);
}

// one finished episode: summary, record, per-node row
template <class Src, class St>
__device__ inline void bk_finish(const bk::BkParams& P, bk::BkLane& L, const bk::BkMem& M,
                                 const St& S, int64_t e, int32_t hd, Acc& acc, int32_t* hist,
                                 cpr_episode_record* recs, const NodeOut& no) {
  L.status |= Src::missed(S);
  const bk::BVtx& h = L.X(P, M, hd);
  bk_acc(acc, P, L, h, hist);
  if (recs) {
    cpr_episode_record r;
    r.reward_attacker = (double)h.rew_att;
    r.reward_defender = (double)h.rew_def;
    r.progress = (double)(h.height * P.k);
    r.chain_time = h.time;
    r.sim_time = P.mode == CPR_MODE_GYM ? L.now : 0.0;
    r.n_steps = L.steps;
    r.n_activations = L.c_act;
    r.head_height = h.height;
    r.head_miner = h.who;
    r.status = L.status;
    r.head_work = 0;
    recs[e] = r;
  }
  if (no.acts) {  // csv_runner.ml:74-79: sim.activations and (Dag.data head).rewards
    const int32_t* hr =
        h.qslot < 0 ? nullptr : M.nrew + (int64_t)(h.qslot & (P.cap_q - 1)) * P.n;
    for (int32_t j = 0; j < P.n; ++j) {
      no.acts[e * P.n + j] = M.nact[j];
      no.rews[e * P.n + j] = hr ? (double)hr[j] : 0.0;
    }
    no.head_miner[e] = h.who;
  }
}

// wave_sched.h adapter for bk_lane.h
struct BkAdapter {
  using Lane = bk::BkLane;
  using Par = bk::BkParams;
  using Mem = bk::BkMem;
  template <class St>
  __device__ static void begin(Lane& L, const Par& P, const St& S, const Mem& M) {
    L.init(P, S, M);
  }
  __device__ static bool gym(const Par& P) { return P.mode == CPR_MODE_GYM; }
  __device__ static bool loop_attacker(const Par& P) { return P.net != 2; }
  __device__ static bool pow0(uint32_t ev) {
    return (ev & 7u) == bk::EV_DAG && (ev >> 5) == 0u && ((ev >> 3) & 3u) == bk::KD_POW;
  }
  template <class St>
  __device__ static void run_pow0(Lane& L, const Par& P, const St& S, const Mem& M, int32_t) {
    const int32_t v = L.append_vote(P, S, M, 0, L.priv);
    L.push_now(P, M, bk::mkev(bk::EV_MV, 0, bk::KD_POW), v);
  }
  __device__ static void act(Lane& L, const Par& P, const Mem& M) {
    L.apply(P, M, bk::bk_policy(P, L.observe(P, M)));
    ++L.steps;
  }
  __device__ static int32_t head_gym(Lane& L, const Par& P, const Mem& M, int32_t att) {
    return L.head(P, M, att);
  }
  __device__ static int32_t head_loop(Lane& L, const Par& P, const Mem& M) {
    return L.head(P, M, P.net == 2 ? M.tips[0] : L.priv);
  }
  __device__ static bool gym_done(Lane& L, const Par& P, const Mem& M, int32_t hd) {
    const double progress = (double)(L.X(P, M, hd).height * P.k);
    return L.dead || !(L.steps < P.max_steps && progress < P.max_progress && L.now < P.max_time);
  }
};

// the heap slab of a workgroup (dynamic LDS): kl nodes per lane, node-major
extern __shared__ __attribute__((aligned(16))) bk::HNode bk_slab[];

template <class Src>
__global__ __launch_bounds__(kBlock) CPR_EV_OCC void k_bk_run_episodes(
    bk::BkParams P, Src src, int64_t n_eps, uint8_t* mem,
    int64_t lane_bytes, cpr_episode_record* recs, cpr_summary* sum, NodeOut no, int32_t kl,
    int32_t vw) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
  bk::BkMem M = bk::bk_mem_at(mem + tid * lane_bytes, P);
  // every episode starts with an empty heap and a fresh window (init): the slab needs no
  // load or store
  bk::bk_heap_slab(M, bk_slab, (int32_t)threadIdx.x, (int32_t)blockDim.x, kl);
  bk::bk_vis_window(M, (uint8_t*)(bk_slab + (size_t)kl * blockDim.x), (int32_t)threadIdx.x, vw);
  if (no.mem) bk::bk_node_mem(M, no.mem + tid * no.lane_bytes, P);
  Acc acc = {};
  bk::BkLane L;
#if CPR_EV_SCHED
  int64_t e = tid;  // wave-coherent dispatch (wave_sched.h), episodes from a work queue
  auto S = src.at(e < n_eps ? e : 0);
  EvCursor c;
  c.cls = -1;
  c.phase = PH_IDLE;
  if (e < n_eps) ev_begin<BkAdapter>(L, P, S, M, c);
  for (;;) {
    while (c.phase != PH_IDLE && c.cls < 0) {
      if (c.phase != PH_OVER) ev_fetch<BkAdapter>(L, P, S, M, c);
      if (c.phase == PH_OVER) {
        bk_finish<Src>(P, L, M, S, e, c.hd, acc, hist, recs, no);
        e = ev_next_episode(P.next, e, nthreads);
        if (e < n_eps) {
          S = src.at(e);
          ev_begin<BkAdapter>(L, P, S, M, c);
        } else {
          c.phase = PH_IDLE;
        }
      }
    }
    const int32_t k = ev_choose(c.cls);
    if (k < 0) break;
    if (c.cls == k) ev_exec<BkAdapter>(L, P, S, M, c);
  }
#else
  for (int64_t e = tid; e < n_eps; e += nthreads) {
    const auto S = src.at(e);
    int32_t hd;
    if (P.mode == CPR_MODE_GYM) {
      L.gym_reset(P, S, M);
      bool done = L.dead != 0;
      hd = 0;
      while (!done) hd = L.gym_step(P, S, M, bk::bk_policy(P, L.observe(P, M)), &done);
    } else {
      hd = L.loop(P, S, M);
    }
    bk_finish<Src>(P, L, M, S, e, hd, acc, hist, recs, no);
  }
#endif
  __syncthreads();
  block_flush(acc, hist, sum);
}

// ssz_tools.ml:1-74 with bk_ssz.ml:37-48 normalizers; unit encodings use host-tabulated
// libm values (tabs = [2/pi atan(i) | 0.5 + atan(i - N)/pi | 2/pi atan(i/k)], i < N)
__device__ inline void bk_write_obs(const bk::BkObs& o, int unit, const double* tabs,
                                    int32_t tn, int32_t k, double* out) {
  const double pi = 3.141592653589793;
  if (!unit) {
    out[0] = (double)o.public_blocks;
    out[1] = (double)o.private_blocks;
    out[2] = (double)o.diff_blocks;
    out[3] = (double)o.public_votes;
    out[4] = (double)o.private_votes_inclusive;
    out[5] = (double)o.private_votes_exclusive;
    out[6] = o.lead ? 1.0 : 0.0;
    out[7] = (double)o.event;
    return;
  }
  auto nn1 = [&](int32_t x) { return x < tn ? tabs[x] : 2.0 / pi * atan((double)x / 1.0); };
  auto nnk = [&](int32_t x) {
    return x < tn ? tabs[3 * tn + x] : 2.0 / pi * atan((double)x / (double)k);
  };
  out[0] = nn1(o.public_blocks);
  out[1] = nn1(o.private_blocks);
  const int32_t d = o.diff_blocks;
  out[2] = (d > -tn && d < tn) ? tabs[tn + d + tn] : 0.5 + (1.0 / pi * atan((double)d / 1.0));
  out[3] = nnk(o.public_votes);
  out[4] = nnk(o.private_votes_inclusive);
  out[5] = nnk(o.private_votes_exclusive);
  out[6] = o.lead ? 1.0 : 0.0;
  out[7] = (double)o.event / 2.0;
}

__device__ inline void bk_slot_reset(const bk::BkParams& P, uint64_t seed, const bk::BkMem& M,
                                     BkSlot& SL, uint64_t ep) {
  SL.ep = ep;
  SL.last_ra = 0.0;
  SL.head = 0;
  SL.live = 1;
  SL.L.gym_reset(P, make_stream(seed, ep), M);
}

__global__ __launch_bounds__(kBlock) void k_bk_reset(bk::BkParams P, uint64_t seed,
                                                      uint8_t* mem, int64_t lane_bytes,
                                                      BkSlot* slots, int64_t n,
                                                      const uint8_t* mask, const uint64_t* eps,
                                                      int unit, const double* tabs, int32_t tn,
                                                      double* obs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bk::BkMem M = bk::bk_mem_at(mem + i * lane_bytes, P);
  BkSlot SL = slots[i];
  if (mask == nullptr || mask[i]) bk_slot_reset(P, seed, M, SL, eps ? eps[i] : (uint64_t)i);
  bk_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, obs + 8 * i);
  slots[i] = SL;
}

__global__ __launch_bounds__(kBlock) void k_bk_step(bk::BkParams P, uint64_t seed, uint8_t* mem,
                                                     int64_t lane_bytes, BkSlot* slots,
                                                     int64_t n, const int32_t* actions, int unit,
                                                     const double* tabs, int32_t tn,
                                                     StepBuffers out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bk::BkMem M = bk::bk_mem_at(mem + i * lane_bytes, P);
  BkSlot SL = slots[i];
  const Stream S = make_stream(seed, SL.ep);
  bool done = false;
  const int32_t hd = SL.L.gym_step(P, S, M, actions[i], &done);
  SL.head = hd;
  const bk::BVtx& h = SL.L.X(P, M, hd);
  const double ra = (double)h.rew_att;
  out.reward[i] = ra - SL.last_ra;  // engine.ml:223
  out.done[i] = done ? 1 : 0;
  out.status[i] = SL.L.status;
  if (out.era) {
    out.era[i] = ra;
    out.erd[i] = (double)h.rew_def;
    out.eprog[i] = (double)(h.height * P.k);
    out.ect[i] = h.time;
    out.est[i] = SL.L.now;
    out.esteps[i] = SL.L.steps;
    out.eacts[i] = SL.L.c_act;
    out.hh[i] = h.height;
    out.hm[i] = h.who;
  }
  SL.last_ra = ra;
  bk_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, out.obs + 8 * i);
  slots[i] = SL;
}

// n_steps lockstep steps per lane with the batch's on-device policy; finished episodes are
// summarised and the lane restarts with episode id ep + n (VecEnv auto-reset: the
// observation written at a done step is the new episode's first observation).
// summary.steps / .activations count every step / activation of the rollout; the other
// summary fields cover the episodes that finished in it.
// four waves per SIMD (128 VGPRs): rollout_lanes_per_wave spreads a small batch over them
#ifndef CPR_ROLL_WAVES
#define CPR_ROLL_WAVES 4
#endif
#if CPR_EV_WAVES > 0
#define CPR_ROLL_OCC CPR_EV_OCC
#else
#define CPR_ROLL_OCC __attribute__((amdgpu_waves_per_eu(CPR_ROLL_WAVES)))
#endif
__global__ __launch_bounds__(kBlock) CPR_ROLL_OCC void k_bk_rollout(bk::BkParams P, uint64_t seed,
                                                        uint8_t* mem, int64_t lane_bytes,
                                                        BkSlot* slots, int64_t n,
                                                        int64_t n_steps, int unit,
                                                        const double* tabs, int32_t tn,
                                                        double* obs, double* reward,
                                                        uint8_t* done_out, cpr_summary* sum,
                                                        int32_t kl, int32_t vw, int32_t lpw) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  // lpw envs per wave (lanes lpw..63 idle): fewer envs per wave, more waves per SIMD to hide
  // the dependent loads (rollout_lanes_per_wave); the slab holds the used lanes' columns
  const int32_t wl = (int32_t)(threadIdx.x & 63u);
  const int32_t wpb = (int32_t)(blockDim.x >> 6);
  const int32_t col = (int32_t)(threadIdx.x >> 6) * lpw + (wl < lpw ? wl : 0);
  const int64_t i = wl < lpw ? (int64_t)blockIdx.x * wpb * lpw + col : n;
  Acc acc = {};
  int64_t steps_all = 0, acts_all = 0;
#if CPR_EV_SCHED
  // wave-coherent dispatch (wave_sched.h roll_fetch): the plain loop below split into items;
  // every lane's own sequence of events, actions and outputs is the plain loop's
  bk::BkMem M = bk::bk_mem_at(mem + (i < n ? i : 0) * lane_bytes, P);
  bk::bk_heap_slab(M, bk_slab, col, wpb * lpw, kl);
  bk::bk_vis_window(M, (uint8_t*)(bk_slab + (size_t)kl * wpb * lpw), col, vw);
  BkSlot SL;
  EvCursor c;
  c.cls = -1;
  c.phase = PH_IDLE;
  int64_t ts = 0;  // steps of this launch taken
  int32_t a0 = 0;  // activations of the current episode before this launch
  Stream S = make_stream(seed, 0);
  if (i < n) {
    SL = slots[i];
    bk::bk_heap_load(M, SL.L.hused);
    bk::bk_vis_load(M, P, SL.L.newest);
    if (!SL.live)
      bk_slot_reset(P, seed, M, SL, (uint64_t)i);
    else
      a0 = SL.L.c_act;
    S = make_stream(seed, SL.ep);
    if (n_steps > 0) {
      BkAdapter::act(SL.L, P, M);
      c.att = SL.L.priv;
      c.phase = PH_RUN;
    }
  }
#ifdef CPR_EV_CLOCKS
  // diagnostic build: shader-clock cycles of the wave per item class (the exec that follows
  // the choice), of fetching and of choosing; printed by lane 0 of a few workgroups
  uint64_t clk[WK_N + 2] = {};
  uint64_t sub[5] = {};  // the attack item: prepare, head/done, obs write, observe, apply
  uint32_t cnt[WK_N] = {};
  uint64_t tprev = clock64();
  int32_t last = -1;
#endif
  for (;;) {
#ifdef CPR_EV_CLOCKS
    {
      const uint64_t tn = clock64();
      if (last >= 0) clk[last] += tn - tprev;
      tprev = tn;
    }
#endif
    if (c.phase != PH_IDLE && c.cls < 0) roll_fetch<BkAdapter>(SL.L, M, c);
#ifdef CPR_EV_CLOCKS
    {
      const uint64_t tn = clock64();
      clk[WK_N] += tn - tprev;
      tprev = tn;
    }
#endif
    const int32_t kc = ev_choose(c.cls);
#ifdef CPR_EV_CLOCKS
    {
      const uint64_t tn = clock64();
      clk[WK_N + 1] += tn - tprev;
      tprev = tn;
      last = kc;
      if (kc >= 0) cnt[kc] += 1;
    }
#endif
    if (kc < 0) break;
    if (c.cls != kc) continue;
    c.cls = -1;
    if (kc == WK_POW0) {
      BkAdapter::run_pow0(SL.L, P, S, M, c.s);
      continue;
    }
    if (kc != WK_ATTACK) {
      SL.L.handle(P, S, M, c.ev, c.s);
      continue;
    }
    if (c.ev != kRollFail) SL.L.prepare(P, M, (c.ev >> 3) & 3u, c.s);
#ifdef CPR_EV_CLOCKS
    uint64_t ta = clock64();
    sub[0] += ta - tprev;  // prepare
#endif
    if (c.phase == PH_FRESH) {
      // the reset after a done step reached its first interaction: that step's observation
      c.phase = PH_RUN;
      if (obs) bk_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, obs + 8 * ((ts - 1) * n + i));
    } else {
      const int32_t hd = BkAdapter::head_gym(SL.L, P, M, c.att);
      const bool done = BkAdapter::gym_done(SL.L, P, M, hd);
#ifdef CPR_EV_CLOCKS
      {
        const uint64_t tb = clock64();
        sub[1] += tb - ta;  // head, done
        ta = tb;
      }
#endif
      const bk::BVtx& h = SL.L.X(P, M, hd);
      const double ra = (double)h.rew_att;
      const int64_t k = ts * n + i;
      if (reward) reward[k] = ra - SL.last_ra;
      if (done_out) done_out[k] = done ? 1 : 0;
      SL.last_ra = ra;
      ++ts;
      if (done) {
        bk_acc(acc, P, SL.L, h, hist);
        acts_all += SL.L.c_act - a0;
        a0 = 0;
        SL.ep += (uint64_t)n;  // bk_slot_reset, its events run as items
        SL.last_ra = 0.0;
        SL.head = 0;
        SL.live = 1;
        S = make_stream(seed, SL.ep);
        SL.L.init(P, S, M);
        c.phase = PH_FRESH;
        continue;
      }
      if (obs) bk_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, obs + 8 * k);
    }
#ifdef CPR_EV_CLOCKS
    {
      const uint64_t tb = clock64();
      sub[2] += tb - ta;  // observation written
      ta = tb;
    }
#endif
    if (ts >= n_steps) {
      c.phase = PH_IDLE;  // at the decision point of the next launch's first step
      continue;
    }
#ifdef CPR_EV_CLOCKS
    {
      const bk::BkObs o = SL.L.observe(P, M);
      const uint64_t tb = clock64();
      sub[3] += tb - ta;  // observe (the policy's)
      ta = tb;
      SL.L.apply(P, M, bk::bk_policy(P, o));
      ++SL.L.steps;
      sub[4] += clock64() - ta;  // policy + apply
    }
#else
    BkAdapter::act(SL.L, P, M);
#endif
    c.att = SL.L.priv;
  }
  if (i < n) {
    acts_all += SL.L.c_act - a0;
    steps_all = n_steps;
    bk::bk_heap_store(M, SL.L.hused);
    slots[i] = SL;
  }
#ifdef CPR_EV_CLOCKS
  if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 77 || blockIdx.x == 200)) {
    uint64_t tot = 0;
    for (int32_t q = 0; q < WK_N + 2; ++q) tot += clk[q];
    printf("EVCLK block %d total %llu fetch %llu choose %llu | clock %llu/%u dag %llu/%u "
           "tx %llu/%u rx %llu/%u on %llu/%u mv %llu/%u mdv %llu/%u attack %llu/%u "
           "pow0 %llu/%u\n",
           (int)blockIdx.x, (unsigned long long)tot, (unsigned long long)clk[WK_N],
           (unsigned long long)clk[WK_N + 1], (unsigned long long)clk[0], cnt[0],
           (unsigned long long)clk[1], cnt[1], (unsigned long long)clk[2], cnt[2],
           (unsigned long long)clk[3], cnt[3], (unsigned long long)clk[4], cnt[4],
           (unsigned long long)clk[5], cnt[5], (unsigned long long)clk[6], cnt[6],
           (unsigned long long)clk[7], cnt[7], (unsigned long long)clk[8], cnt[8]);
    printf("EVCLK block %d attack: prepare %llu head %llu obs %llu observe %llu apply %llu\n",
           (int)blockIdx.x, (unsigned long long)sub[0], (unsigned long long)sub[1],
           (unsigned long long)sub[2], (unsigned long long)sub[3], (unsigned long long)sub[4]);
  }
#endif
#else
  if (i < n) {
    bk::BkMem M = bk::bk_mem_at(mem + i * lane_bytes, P);
    BkSlot SL = slots[i];
    // the lane's heap nodes 0 .. kl-1 move to the slab for this launch
    bk::bk_heap_slab(M, bk_slab, col, wpb * lpw, kl);
    bk::bk_vis_window(M, (uint8_t*)(bk_slab + (size_t)kl * wpb * lpw), col, vw);
    bk::bk_heap_load(M, SL.L.hused);
    bk::bk_vis_load(M, P, SL.L.newest);
    if (!SL.live) {
      bk_slot_reset(P, seed, M, SL, (uint64_t)i);
      acts_all += SL.L.c_act;
    }
    Stream S = make_stream(seed, SL.ep);
    for (int64_t t = 0; t < n_steps; ++t) {
      const bk::BkObs o = SL.L.observe(P, M);
      const int32_t c0 = SL.L.c_act;
      bool done = false;
      const int32_t hd = SL.L.gym_step(P, S, M, bk::bk_policy(P, o), &done);
      acts_all += SL.L.c_act - c0;
      ++steps_all;
      const bk::BVtx& h = SL.L.X(P, M, hd);
      const double ra = (double)h.rew_att;
      const int64_t k = t * n + i;
      if (reward) reward[k] = ra - SL.last_ra;
      if (done_out) done_out[k] = done ? 1 : 0;
      SL.last_ra = ra;
      if (done) {
        bk_acc(acc, P, SL.L, h, hist);
        bk_slot_reset(P, seed, M, SL, SL.ep + (uint64_t)n);
        acts_all += SL.L.c_act;
        S = make_stream(seed, SL.ep);
      }
      if (obs) bk_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, obs + 8 * k);
    }
    bk::bk_heap_store(M, SL.L.hused);
    slots[i] = SL;
  }
#endif
  // rollout totals: all steps and activations (acc.steps/activations hold finished
  // episodes only, so replace them before the block reduction)
  acc.steps = steps_all;
  acc.activations = acts_all;
  __syncthreads();
  block_flush(acc, hist, sum);
}

__global__ void k_bk_observe_fields(bk::BkParams P, uint8_t* mem, int64_t lane_bytes,
                                    const BkSlot* slots, int64_t n, int32_t* f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bk::BkMem M = bk::bk_mem_at(mem + i * lane_bytes, P);
  bk::BkLane L = slots[i].L;
  const bk::BkObs o = L.observe(P, M);
  int32_t* g = f + 8 * i;
  g[0] = o.public_blocks;
  g[1] = o.private_blocks;
  g[2] = o.diff_blocks;
  g[3] = o.public_votes;
  g[4] = o.private_votes_inclusive;
  g[5] = o.private_votes_exclusive;
  g[6] = o.lead;
  g[7] = o.event;
}

// engine.ml:258-261: decode (ssz_tools.ml:42-58 of_float) and apply the policy
__global__ void k_bk_policy(bk::BkParams P, int unit, const double* obs, int64_t n,
                            int32_t* actions) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* x = obs + 8 * i;
  const double pi = 3.141592653589793;
  int32_t v[8];
  for (int j = 0; j < 8; ++j) {
    if (j == 6) {
      v[j] = x[j] >= 0.5 ? 1 : 0;
    } else if (j == 7) {
      v[j] = unit ? (int32_t)floor(x[j] * 2.0) : (int32_t)x[j];
    } else if (!unit) {
      v[j] = (int32_t)x[j];
    } else {
      const double scale = j >= 3 ? (double)P.k : 1.0;
      v[j] = j == 2 ? (int32_t)__builtin_round(tan(pi * (x[j] - 0.5)) * scale)
                    : (int32_t)__builtin_round(tan(pi / 2.0 * x[j]) * scale);
    }
  }
  const bk::BkObs o{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
  actions[i] = bk::bk_policy(P, o);
}

// ---------------------------------------------------------------- launchers

static unsigned grid_of(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

int64_t lds_dynamic_max(const void* kernel) {
  struct Entry {
    const void* k;
    int dev;
    int64_t room;
  };
  static std::mutex mu;
  static std::vector<Entry> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(mu);
  for (const Entry& e : cache)
    if (e.k == kernel && e.dev == dev) return e.room;
  int lds = 0;
  if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess ||
      lds <= 0)
    lds = 64 * 1024;
  hipFuncAttributes fa{};
  if (hipFuncGetAttributes(&fa, kernel) != hipSuccess) {
    (void)hipGetLastError();
    return 0;  // unknown: no dynamic LDS (not cached, asked again next time)
  }
  const int64_t room = std::max<int64_t>(0, (int64_t)lds - (int64_t)fa.sharedSizeBytes);
  cache.push_back(Entry{kernel, dev, room});
  return room;
}

// heap nodes per lane in the LDS slab for a grid of `blocks` workgroups: the LDS a
// workgroup gets when the grid spreads over the device's CUs (160 KiB per CU), less the
// kernels' static LDS, at most 32 nodes (the gym's windows hold 14-30 live events);
// CPR_EV_SLAB overrides it (A/B runs; 0 = every node in HBM)
int32_t ev_slab_nodes(int64_t blocks, const void* kernel) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  if (const char* v = getenv("CPR_EV_SLAB")) return std::max(0, std::min(32, atoi(v)));
  const int64_t per_cu = std::max<int64_t>(1, (blocks + cus - 1) / cus);
  // 160 KiB less the kernel's static LDS (reserved as at least 2 KiB, the plans' rule)
  const int64_t room = std::min<int64_t>(lds_dynamic_max(kernel), 160 * 1024 - 2048);
  const int64_t bytes = std::min<int64_t>(room, (160 * 1024) / per_cu - (160 * 1024 - room));
  int32_t kl = (int32_t)std::min<int64_t>(32, std::max<int64_t>(0, bytes / (kBlock * 24)));
  if ((int64_t)kl * kBlock * 24 > 64 * 1024) {
    // more than the default 64 KiB of dynamic LDS: ask once per kernel
    if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)room) != hipSuccess) {
      (void)hipGetLastError();
      kl = (64 * 1024) / (kBlock * 24);
    }
  }
  return kl;
}

// envs per wave of a lockstep rollout of n envs on `kernel`: the widest of 64 / 32 / 16 whose
// waves fit the kernel's resident waves per SIMD (occupancy query), so that a small batch
// still runs several waves per SIMD, which hide each other's dependent loads (BASELINE
// configs[4], 65,536 B_k envs: one wave per SIMD at 64; 32 per wave +5.6 % env-steps/s,
// 16 per wave at the 4-wave budget of k_bk_rollout +3.7 % more;
// profiles/r05f_lpw.log, profiles/r05g_lpw.log). CPR_ROLL_LPW overrides it.
int32_t rollout_lanes_per_wave(int64_t n, const void* kernel) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  if (const char* v = getenv("CPR_ROLL_LPW")) {
    const int32_t w = atoi(v);
    if (w >= 1 && w <= 64) return w;
  }
  int per_cu = 0;  // workgroups of kBlock / 64 waves, i.e. waves per SIMD
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess ||
      per_cu <= 0) {
    (void)hipGetLastError();
    per_cu = 1;
  }
  const int64_t simds = (int64_t)cus * 4;
  for (int32_t w : {16, 32})
    if ((n + w * simds - 1) / (w * simds) <= per_cu) return w;
  return 64;
}

// lanes per wave that run episodes in the fused event-engine kernels (the others idle):
// 64 (CPR_EV_LPW overrides it for A/B runs: 32 with an occupancy variant runs the same
// lanes as twice the waves)
int32_t event_lanes_per_wave() {
  if (const char* v = getenv("CPR_EV_LPW")) {
    const int32_t w = atoi(v);
    if (w >= 1 && w <= 64) return w;
  }
  return 64;
}

// an event-engine kernel's slab: the heap's first kl nodes and the visibility rows of the
// newest vw vertices (BkMem.vl / TsMem.vl; 64, else 32, when they take at most a third of
// the workgroup's share of LDS; CPR_EV_VWIN overrides it, 0 = none); kl from what is left
// (ev_slab_nodes' rules)
EvSlab ev_slab_plan(int64_t blocks, const void* kernel, int32_t n, int32_t lanes,
                    int32_t trec_rows) {
  if (lanes <= 0) lanes = kBlock;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
  }
  const int64_t per_cu = std::max<int64_t>(1, (blocks + cus - 1) / cus);
  // 160 KiB less the kernel's static LDS (reserved as at least 2 KiB, the plans' rule)
  const int64_t room = std::min<int64_t>(lds_dynamic_max(kernel), 160 * 1024 - 2048);
  const int64_t avail = std::min<int64_t>(room, (160 * 1024) / per_cu - (160 * 1024 - room));
  int32_t vw = 0;
  for (int32_t w : {64, 32})
    if (vw == 0 && (int64_t)w * n * lanes * 3 <= avail) vw = w;
  if (const char* v = getenv("CPR_EV_VWIN")) {
    const int32_t w = atoi(v);
    vw = (w >= 1 && (w & (w - 1)) == 0 && w <= 256) ? w : 0;
  }
  int64_t rest = avail - (int64_t)vw * n * lanes;
  if (rest < 0) {
    vw = 0;
    rest = avail;
  }
  // the list-record window (after the visibility rows, 16-aligned; a 16-byte record per row
  // and lane) takes its share before the heap nodes
  int32_t tw = trec_rows > 0 && (trec_rows & (trec_rows - 1)) == 0 ? trec_rows : 0;
  while (tw > 0 && rest - 16 - (int64_t)tw * 16 * lanes < 0) tw >>= 1;
  if (tw > 0) rest -= 16 + (int64_t)tw * 16 * lanes;
  int32_t kl = (int32_t)std::min<int64_t>(32, std::max<int64_t>(0, rest / (lanes * 24)));
  if (const char* v = getenv("CPR_EV_SLAB")) kl = std::max(0, std::min(32, atoi(v)));
  auto layout = [&](EvSlab& s) {
    const size_t vis_end = (size_t)s.kl * lanes * 24 + (size_t)s.vw * n * lanes;
    s.tw_off = (vis_end + 15) / 16 * 16;
    s.bytes = s.tw > 0 ? s.tw_off + (size_t)s.tw * 16 * lanes : vis_end;
  };
  EvSlab sl{kl, vw, 0};
  sl.tw = tw;
  layout(sl);
  if (sl.bytes > 64 * 1024 &&
      hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)room) != hipSuccess) {
    (void)hipGetLastError();  // the default 64 KiB: the heap slab alone
    sl.vw = 0;
    sl.tw = 0;
    sl.kl = std::min(32, (64 * 1024) / (lanes * 24));
    layout(sl);
  }
  return sl;
}

hipError_t launch_bk_run_episodes(const bk::BkParams& P, uint64_t seed, uint64_t first,
                                  int64_t n_eps, uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                  cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                  const NodeOut& no) {
  CPR_LAYOUT_GUARD(lane_bytes, bk::bk_lane_bytes(P));
  const unsigned blocks = (unsigned)(lanes / kBlock);
  const EvSlab sl = ev_slab_plan(blocks, (const void*)k_bk_run_episodes<SeedSource>, P.n);
  CPR_LDS_GUARD(k_bk_run_episodes<SeedSource>, sl.bytes);
  hipLaunchKernelGGL(k_bk_run_episodes<SeedSource>, dim3(blocks), dim3(kBlock), sl.bytes, st, P,
                     SeedSource{seed, first}, n_eps, mem, lane_bytes, recs, sum, no, sl.kl,
                     sl.vw);
  return hipGetLastError();
}

hipError_t launch_bk_replay_episodes(const bk::BkParams& P, const TraceSource& src, int64_t n_eps,
                                 uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                 cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                  const NodeOut& no) {
  CPR_LAYOUT_GUARD(lane_bytes, bk::bk_lane_bytes(P));
  const unsigned blocks = (unsigned)(lanes / kBlock);
  const EvSlab sl = ev_slab_plan(blocks, (const void*)k_bk_run_episodes<TraceSource>, P.n);
  CPR_LDS_GUARD(k_bk_run_episodes<TraceSource>, sl.bytes);
  hipLaunchKernelGGL(k_bk_run_episodes<TraceSource>, dim3(blocks), dim3(kBlock), sl.bytes, st, P,
                     src, n_eps, mem, lane_bytes, recs, sum, no, sl.kl, sl.vw);
  return hipGetLastError();
}

hipError_t launch_bk_reset(const bk::BkParams& P, uint64_t seed, uint8_t* mem, int64_t lane_bytes,
                           void* slots, int64_t n, const uint8_t* mask, const uint64_t* eps,
                           int unit, const double* tabs, int32_t tn, double* obs,
                           hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, bk::bk_lane_bytes(P));
  hipLaunchKernelGGL(k_bk_reset, dim3(grid_of(n)), dim3(kBlock), 0, st, P, seed, mem, lane_bytes,
                     (BkSlot*)slots, n, mask, eps, unit, tabs, tn, obs);
  return hipGetLastError();
}

hipError_t launch_bk_step(const bk::BkParams& P, uint64_t seed, uint8_t* mem, int64_t lane_bytes,
                          void* slots, int64_t n, const int32_t* actions, int unit,
                          const double* tabs, int32_t tn, const StepBuffers& b, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, bk::bk_lane_bytes(P));
  hipLaunchKernelGGL(k_bk_step, dim3(grid_of(n)), dim3(kBlock), 0, st, P, seed, mem, lane_bytes,
                     (BkSlot*)slots, n, actions, unit, tabs, tn, b);
  return hipGetLastError();
}

hipError_t launch_bk_rollout(const bk::BkParams& P, uint64_t seed, uint8_t* mem,
                             int64_t lane_bytes, void* slots, int64_t n, int64_t n_steps,
                             int unit, const double* tabs, int32_t tn, double* obs,
                             double* reward, uint8_t* done, cpr_summary* sum, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, bk::bk_lane_bytes(P));
  const int32_t lpw = rollout_lanes_per_wave(n, (const void*)k_bk_rollout);
  const int64_t per_block = (int64_t)(kBlock / 64) * lpw;
  const unsigned blocks = (unsigned)((n + per_block - 1) / per_block);
  const EvSlab sl = ev_slab_plan(blocks, (const void*)k_bk_rollout, P.n, (int32_t)per_block);
  CPR_LDS_GUARD(k_bk_rollout, sl.bytes);
  hipLaunchKernelGGL(k_bk_rollout, dim3(blocks), dim3(kBlock), sl.bytes, st, P, seed, mem,
                     lane_bytes, (BkSlot*)slots, n, n_steps, unit, tabs, tn, obs, reward, done,
                     sum, sl.kl, sl.vw, lpw);
  return hipGetLastError();
}

hipError_t launch_bk_observe_fields(const bk::BkParams& P, uint8_t* mem, int64_t lane_bytes,
                                    const void* slots, int64_t n, int32_t* f, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, bk::bk_lane_bytes(P));
  hipLaunchKernelGGL(k_bk_observe_fields, dim3(grid_of(n)), dim3(kBlock), 0, st, P, mem,
                     lane_bytes, (const BkSlot*)slots, n, f);
  return hipGetLastError();
}

hipError_t launch_bk_policy(const bk::BkParams& P, int unit, const double* obs, int64_t n,
                            int32_t* actions, hipStream_t st) {
  hipLaunchKernelGGL(k_bk_policy, dim3(grid_of(n)), dim3(kBlock), 0, st, P, unit, obs, n,
                     actions);
  return hipGetLastError();
}

size_t bk_slot_bytes() { return sizeof(BkSlot); }

int bk_blocks_per_cu() {
  int blocks = 0;
  hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_bk_run_episodes<SeedSource>, kBlock, 0);
  if (e != hipSuccess || blocks <= 0) blocks = 2;
  return blocks;
}

}  // namespace cpr
