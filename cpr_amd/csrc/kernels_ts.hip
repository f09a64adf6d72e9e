// Tailstorm kernels for gfx950: one lane = one episode / gym env of the tailstorm_ssz
// attack space, driven by the exact per-lane event engine of ts_lane.h (same launch
// structure as kernels_bk.hip: fused episodes, lockstep reset/step, device rollout).
#include <hip/hip_runtime.h>

// occupancy of this TU's event-engine kernels (kernels.h CPR_EV_OCC): 2 waves/SIMD measured
// +35 % over the unconstrained build on the configs[3] exp-clique probe under wave-coherent
// dispatch (profiles/r03f_event_occupancy_ab.log); build_variants.py overrides it with -D
#ifndef CPR_EV_WAVES
#define CPR_EV_WAVES 2
#endif

#include "../../include/cpr_hip.h"
#include "kernels.h"
#include "summary.h"
#include "ts_lane.h"
#include "wave_sched.h"

#pragma clang fp contract(off)

namespace cpr {

struct TsSlot {
  ts::TsLane L;
  uint64_t ep;
  double last_ra;
  int32_t live;
};

// head rewards: engine.ml:215-219 folds head.rewards left to right
__device__ inline void ts_head_rewards(const ts::TsParams& P, ts::TsLane& L, const ts::TsMem& M,
                                       int32_t hd, double* ra, double* rd) {
  const ts::TVtx& h = L.X(P, M, hd);
  *ra = 0.0;
  *rd = 0.0;
  if (h.qslot < 0) return;
  const double* rw = L.R(P, M, h.qslot);
  *ra = rw[0];
  double s = 0.0;
  for (int32_t j = 1; j < P.n; ++j) s += rw[j];
  *rd = s;
}

__device__ inline void ts_acc(Acc& acc, const ts::TsParams& P, ts::TsLane& L,
                              const ts::TsMem& M, int32_t hd, int32_t* hist) {
  double ra, rd;
  ts_head_rewards(P, L, M, hd, &ra, &rd);
  const int32_t h = L.X(P, M, hd).height;
  const double rel = (ra + rd) != 0.0 ? ra / (ra + rd) : 0.0;
  acc_episode(acc, (int64_t)__builtin_rint(ra * 1048576.0), (int64_t)__builtin_rint(rd * 1048576.0),
              (int64_t)h * P.k << 20, rel, (int64_t)h * P.k, L.steps, L.c_act, L.status, hist);
}

// one finished episode: summary, record, per-node row
template <class Src, class St>
__device__ inline void ts_finish(const ts::TsParams& P, ts::TsLane& L, const ts::TsMem& M,
                                 const St& S, int64_t e, int32_t hd, Acc& acc, int32_t* hist,
                                 cpr_episode_record* recs, const NodeOut& no) {
  L.status |= Src::missed(S);
  ts_acc(acc, P, L, M, hd, hist);
  if (recs) {
    cpr_episode_record r;
    ts_head_rewards(P, L, M, hd, &r.reward_attacker, &r.reward_defender);
    const ts::TVtx& h = L.X(P, M, hd);
    r.progress = (double)(h.height * P.k);
    r.chain_time = h.time;
    r.sim_time = P.mode == CPR_MODE_GYM ? L.now : 0.0;
    r.n_steps = L.steps;
    r.n_activations = L.c_act;
    r.head_height = h.height;
    r.head_miner = -1;
    r.status = L.status;
    r.head_work = 0;
    recs[e] = r;
  }
  if (no.acts) {  // csv_runner.ml:74-79: sim.activations and (Dag.data head).rewards
    const ts::TVtx& h = L.X(P, M, hd);
    const double* hr = h.qslot < 0 ? nullptr : L.R(P, M, h.qslot);
    for (int32_t j = 0; j < P.n; ++j) {
      no.acts[e * P.n + j] = M.nact[j];
      no.rews[e * P.n + j] = hr ? hr[j] : 0.0;
    }
    no.head_miner[e] = -1;  // summaries have no miner (tailstorm.ml info: kind, height)
  }
}

// wave_sched.h adapter: gym episodes (engine.ml reset / step with the on-device policy) and
// Simulator.loop tasks of ts_lane.h
struct TsAdapter {
  using Lane = ts::TsLane;
  using Par = ts::TsParams;
  using Mem = ts::TsMem;
  template <class St>
  __device__ static void begin(Lane& L, const Par& P, const St& S, const Mem& M) {
    L.init(P, S, M);
  }
  __device__ static bool gym(const Par& P) { return P.mode == CPR_MODE_GYM; }
  __device__ static bool loop_attacker(const Par& P) { return P.net != 2; }
  __device__ static bool pow0(uint32_t ev) {
    return (ev & 7u) == ts::EV_DAG && (ev >> 5) == 0u && ((ev >> 3) & 3u) == ts::KD_POW;
  }
  template <class St>
  __device__ static void run_pow0(Lane& L, const Par& P, const St& S, const Mem& M, int32_t) {
    const int32_t v = L.append_vote(P, S, M, 0, L.payload_parent(P, M, 0, L.priv));
    L.push_now(P, M, bk::mkev(ts::EV_MV, 0, ts::KD_POW), v);
  }
  __device__ static void act(Lane& L, const Par& P, const Mem& M) {
    L.apply(P, M, ts::ts_policy_p(P, L.observe(P, M)));
    ++L.steps;
  }
  __device__ static int32_t head_gym(Lane& L, const Par& P, const Mem& M, int32_t att) {
    return L.dead ? 0 : L.head(P, M, att);
  }
  __device__ static int32_t head_loop(Lane& L, const Par& P, const Mem& M) {
    return L.dead ? 0 : L.head(P, M, P.net == 2 ? M.tips[0] : L.priv);
  }
  __device__ static bool gym_done(Lane& L, const Par& P, const Mem& M, int32_t hd) {
    const double progress = (double)(L.X(P, M, hd).height * P.k);
    return L.dead || !(L.steps < P.max_steps && progress < P.max_progress && L.now < P.max_time);
  }
};

// the heap slab of a workgroup (dynamic LDS): kl nodes per lane, node-major
extern __shared__ __attribute__((aligned(16))) bk::HNode ts_slab[];

template <class Src>
__global__ __launch_bounds__(kBlock) CPR_EV_OCC void k_ts_run_episodes(
    ts::TsParams P, Src src, int64_t n_eps, uint8_t* mem,
    int64_t lane_bytes, cpr_episode_record* recs, cpr_summary* sum, NodeOut no, int32_t kl,
    int32_t vw, int32_t lpw, int32_t tw, int32_t tw_off) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  // lpw lanes per wave run episodes (the others idle; event_lanes_per_wave)
  const int32_t wl = (int32_t)(threadIdx.x & 63u);
  const int32_t wpb = (int32_t)(blockDim.x >> 6);
  const bool used = wl < lpw;
  const int32_t col = (int32_t)(threadIdx.x >> 6) * lpw + (used ? wl : 0);
  const int64_t tid = (int64_t)blockIdx.x * wpb * lpw + col;
  const int64_t nthreads = (int64_t)gridDim.x * wpb * lpw;
  ts::TsMem M = ts::ts_mem_at(mem + tid * lane_bytes, P);
  if (no.mem) M.nact = (int64_t*)(no.mem + tid * no.lane_bytes);
  // every episode starts with an empty heap and a fresh window (init): the slab needs no
  // load or store
  ts::ts_heap_slab(M, ts_slab, col, wpb * lpw, kl);
  ts::ts_vis_window(M, (uint8_t*)(ts_slab + (size_t)kl * wpb * lpw), col, vw);
  if (tw > 0) ts::ts_trec_window(M, (ts::TRec*)((uint8_t*)ts_slab + tw_off), col, tw);
  Acc acc = {};
  ts::TsLane L;
#if CPR_EV_SCHED
  // wave-coherent dispatch (wave_sched.h): grid-stride over episodes, every iteration runs
  // the work class most lanes of the wave hold
  int64_t e = used ? tid : n_eps;
  auto S = src.at(e < n_eps ? e : 0);
  EvCursor c;
  c.cls = -1;
  c.phase = PH_IDLE;
  if (e < n_eps) ev_begin<TsAdapter>(L, P, S, M, c);
#ifdef CPR_EV_CLOCKS
  // diagnostic build: shader-clock cycles of the wave per item class (the exec after the
  // choice), of fetching / finishing episodes and of choosing; lane 0 of a few workgroups
  uint64_t clk[WK_N + 2] = {};
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
    while (c.phase != PH_IDLE && c.cls < 0) {
      if (c.phase != PH_OVER) ev_fetch<TsAdapter>(L, P, S, M, c);
      if (c.phase == PH_OVER) {
        ts_finish<Src>(P, L, M, S, e, c.hd, acc, hist, recs, no);
        e = ev_next_episode(P.next, e, nthreads);
        if (e < n_eps) {
          S = src.at(e);
          ev_begin<TsAdapter>(L, P, S, M, c);
        } else {
          c.phase = PH_IDLE;
        }
      }
    }
#ifdef CPR_EV_CLOCKS
    {
      const uint64_t tn = clock64();
      clk[WK_N] += tn - tprev;
      tprev = tn;
    }
#endif
    const int32_t k = ev_choose(c.cls);
#ifdef CPR_EV_CLOCKS
    {
      const uint64_t tn = clock64();
      clk[WK_N + 1] += tn - tprev;
      tprev = tn;
      last = k;
      if (k >= 0) cnt[k] += 1;
    }
#endif
    if (k < 0) break;
    if (c.cls == k) ev_exec<TsAdapter>(L, P, S, M, c);
  }
#ifdef CPR_EV_CLOCKS
  if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 77 || blockIdx.x == 200)) {
    uint64_t tot = 0;
    for (int32_t q = 0; q < WK_N + 2; ++q) tot += clk[q];
    printf("TSCLK block %d total %llu fetch %llu choose %llu | clock %llu/%u dag %llu/%u "
           "tx %llu/%u rx %llu/%u on %llu/%u mv %llu/%u mdv %llu/%u attack %llu/%u "
           "pow0 %llu/%u\n",
           (int)blockIdx.x, (unsigned long long)tot, (unsigned long long)clk[WK_N],
           (unsigned long long)clk[WK_N + 1], (unsigned long long)clk[0], cnt[0],
           (unsigned long long)clk[1], cnt[1], (unsigned long long)clk[2], cnt[2],
           (unsigned long long)clk[3], cnt[3], (unsigned long long)clk[4], cnt[4],
           (unsigned long long)clk[5], cnt[5], (unsigned long long)clk[6], cnt[6],
           (unsigned long long)clk[7], cnt[7], (unsigned long long)clk[8], cnt[8]);
  }
#endif
#else
  for (int64_t e = used ? tid : n_eps; e < n_eps; e += nthreads) {
    const auto S = src.at(e);
    int32_t hd;
    if (P.mode == CPR_MODE_GYM) {
      L.gym_reset(P, S, M);
      bool done = L.dead != 0;
      hd = 0;
      while (!done) hd = L.gym_step(P, S, M, ts::ts_policy_p(P, L.observe(P, M)), &done);
    } else {
      hd = L.loop(P, S, M);
    }
    ts_finish<Src>(P, L, M, S, e, hd, acc, hist, recs, no);
  }
#endif
  __syncthreads();
  block_flush(acc, hist, sum);
}

// tailstorm_ssz.ml:41-55 normalizers; tabs as in kernels_bk.hip
__device__ inline void ts_write_obs(const ts::TsObs& o, int unit, const double* tabs, int32_t tn,
                                    int32_t k, double* out) {
  const double pi = 3.141592653589793;
  const int32_t v[10] = {o.public_blocks,           o.private_blocks,
                         o.diff_blocks,             o.public_votes,
                         o.private_votes_inclusive, o.private_votes_exclusive,
                         o.public_depth,            o.private_depth_inclusive,
                         o.private_depth_exclusive, o.event};
  if (!unit) {
    for (int i = 0; i < 10; ++i) out[i] = (double)v[i];
    return;
  }
  for (int i = 0; i < 9; ++i) {
    const int32_t x = v[i];
    if (i == 2)
      out[i] = (x > -tn && x < tn) ? tabs[tn + x + tn] : 0.5 + (1.0 / pi * atan((double)x / 1.0));
    else if (i < 2)
      out[i] = x < tn ? tabs[x] : 2.0 / pi * atan((double)x / 1.0);
    else
      out[i] = x < tn ? tabs[3 * tn + x] : 2.0 / pi * atan((double)x / (double)k);
  }
  out[9] = (double)v[9] / 2.0;
}

__device__ inline void ts_slot_reset(const ts::TsParams& P, uint64_t seed, const ts::TsMem& M,
                                     TsSlot& SL, uint64_t ep) {
  SL.ep = ep;
  SL.last_ra = 0.0;
  SL.live = 1;
  SL.L.gym_reset(P, make_stream(seed, ep), M);
}

__global__ __launch_bounds__(kBlock) void k_ts_reset(ts::TsParams P, uint64_t seed, uint8_t* mem,
                                                      int64_t lane_bytes, TsSlot* slots,
                                                      int64_t n, const uint8_t* mask,
                                                      const uint64_t* eps, int unit,
                                                      const double* tabs, int32_t tn,
                                                      double* obs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ts::TsMem M = ts::ts_mem_at(mem + i * lane_bytes, P);
  TsSlot SL = slots[i];
  if (mask == nullptr || mask[i]) ts_slot_reset(P, seed, M, SL, eps ? eps[i] : (uint64_t)i);
  ts_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, obs + 10 * i);
  slots[i] = SL;
}

__global__ __launch_bounds__(kBlock) void k_ts_step(ts::TsParams P, uint64_t seed, uint8_t* mem,
                                                     int64_t lane_bytes, TsSlot* slots,
                                                     int64_t n, const int32_t* actions, int unit,
                                                     const double* tabs, int32_t tn,
                                                     StepBuffers out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ts::TsMem M = ts::ts_mem_at(mem + i * lane_bytes, P);
  TsSlot SL = slots[i];
  const Stream S = make_stream(seed, SL.ep);
  bool done = false;
  const int32_t hd = SL.L.gym_step(P, S, M, actions[i], &done);
  double ra, rd;
  ts_head_rewards(P, SL.L, M, hd, &ra, &rd);
  const ts::TVtx& h = SL.L.X(P, M, hd);
  out.reward[i] = ra - SL.last_ra;
  out.done[i] = done ? 1 : 0;
  out.status[i] = SL.L.status;
  if (out.era) {
    out.era[i] = ra;
    out.erd[i] = rd;
    out.eprog[i] = (double)(h.height * P.k);
    out.ect[i] = h.time;
    out.est[i] = SL.L.now;
    out.esteps[i] = SL.L.steps;
    out.eacts[i] = SL.L.c_act;
    out.hh[i] = h.height;
    out.hm[i] = -1;
  }
  SL.last_ra = ra;
  ts_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, out.obs + 10 * i);
  slots[i] = SL;
}

// see k_bk_rollout
__global__ __launch_bounds__(kBlock) CPR_EV_OCC void k_ts_rollout(ts::TsParams P, uint64_t seed,
                                                        uint8_t* mem, int64_t lane_bytes,
                                                        TsSlot* slots, int64_t n,
                                                        int64_t n_steps, int unit,
                                                        const double* tabs, int32_t tn,
                                                        double* obs, double* reward,
                                                        uint8_t* done_out, cpr_summary* sum,
                                                        int32_t kl, int32_t vw, int32_t lpw) {
  __shared__ int32_t hist[CPR_HIST_BINS];
  if (threadIdx.x < CPR_HIST_BINS) hist[threadIdx.x] = 0;
  __syncthreads();
  // lpw envs per wave, as k_bk_rollout
  const int32_t wl = (int32_t)(threadIdx.x & 63u);
  const int32_t wpb = (int32_t)(blockDim.x >> 6);
  const int32_t col = (int32_t)(threadIdx.x >> 6) * lpw + (wl < lpw ? wl : 0);
  const int64_t i = wl < lpw ? (int64_t)blockIdx.x * wpb * lpw + col : n;
  Acc acc = {};
  int64_t steps_all = 0, acts_all = 0;
#if CPR_EV_SCHED
  // wave-coherent dispatch, as k_bk_rollout
  ts::TsMem M = ts::ts_mem_at(mem + (i < n ? i : 0) * lane_bytes, P);
  ts::ts_heap_slab(M, ts_slab, col, wpb * lpw, kl);
  ts::ts_vis_window(M, (uint8_t*)(ts_slab + (size_t)kl * wpb * lpw), col, vw);
  TsSlot SL;
  EvCursor c;
  c.cls = -1;
  c.phase = PH_IDLE;
  int64_t tsn = 0;  // steps of this launch taken
  int32_t a0 = 0;   // activations of the current episode before this launch
  Stream S = make_stream(seed, 0);
  if (i < n) {
    SL = slots[i];
    ts::ts_heap_load(M, SL.L.hused);
    ts::ts_vis_load(M, P, SL.L.newest);
    if (!SL.live)
      ts_slot_reset(P, seed, M, SL, (uint64_t)i);
    else
      a0 = SL.L.c_act;
    S = make_stream(seed, SL.ep);
    if (n_steps > 0) {
      TsAdapter::act(SL.L, P, M);
      c.att = SL.L.priv;
      c.phase = PH_RUN;
    }
  }
  for (;;) {
    if (c.phase != PH_IDLE && c.cls < 0) roll_fetch<TsAdapter>(SL.L, M, c);
    const int32_t kc = ev_choose(c.cls);
    if (kc < 0) break;
    if (c.cls != kc) continue;
    c.cls = -1;
    if (kc == WK_POW0) {
      TsAdapter::run_pow0(SL.L, P, S, M, c.s);
      continue;
    }
    if (kc != WK_ATTACK) {
      SL.L.handle(P, S, M, c.ev, c.s);
      continue;
    }
    if (c.ev != kRollFail) SL.L.prepare(P, M, (c.ev >> 3) & 3u, c.s);
    if (c.phase == PH_FRESH) {
      c.phase = PH_RUN;
      if (obs)
        ts_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, obs + 10 * ((tsn - 1) * n + i));
    } else {
      const int32_t hd = TsAdapter::head_gym(SL.L, P, M, c.att);
      const bool done = TsAdapter::gym_done(SL.L, P, M, hd);
      double ra, rd;
      ts_head_rewards(P, SL.L, M, hd, &ra, &rd);
      const int64_t kk = tsn * n + i;
      if (reward) reward[kk] = ra - SL.last_ra;
      if (done_out) done_out[kk] = done ? 1 : 0;
      SL.last_ra = ra;
      ++tsn;
      if (done) {
        ts_acc(acc, P, SL.L, M, hd, hist);
        acts_all += SL.L.c_act - a0;
        a0 = 0;
        SL.ep += (uint64_t)n;  // ts_slot_reset, its events run as items
        SL.last_ra = 0.0;
        SL.live = 1;
        S = make_stream(seed, SL.ep);
        SL.L.init(P, S, M);
        c.phase = PH_FRESH;
        continue;
      }
      if (obs) ts_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, obs + 10 * kk);
    }
    if (tsn >= n_steps) {
      c.phase = PH_IDLE;
      continue;
    }
    TsAdapter::act(SL.L, P, M);
    c.att = SL.L.priv;
  }
  if (i < n) {
    acts_all += SL.L.c_act - a0;
    steps_all = n_steps;
    ts::ts_heap_store(M, SL.L.hused);
    slots[i] = SL;
  }
#else
  if (i < n) {
    ts::TsMem M = ts::ts_mem_at(mem + i * lane_bytes, P);
    TsSlot SL = slots[i];
    // the lane's heap nodes 0 .. kl-1 move to the slab for this launch
    ts::ts_heap_slab(M, ts_slab, col, wpb * lpw, kl);
    ts::ts_vis_window(M, (uint8_t*)(ts_slab + (size_t)kl * wpb * lpw), col, vw);
    ts::ts_heap_load(M, SL.L.hused);
    ts::ts_vis_load(M, P, SL.L.newest);
    if (!SL.live) {
      ts_slot_reset(P, seed, M, SL, (uint64_t)i);
      acts_all += SL.L.c_act;
    }
    Stream S = make_stream(seed, SL.ep);
    for (int64_t t = 0; t < n_steps; ++t) {
      const ts::TsObs o = SL.L.observe(P, M);
      const int32_t c0 = SL.L.c_act;
      bool done = false;
      const int32_t hd = SL.L.gym_step(P, S, M, ts::ts_policy_p(P, o), &done);
      acts_all += SL.L.c_act - c0;
      ++steps_all;
      double ra, rd;
      ts_head_rewards(P, SL.L, M, hd, &ra, &rd);
      const int64_t kk = t * n + i;
      if (reward) reward[kk] = ra - SL.last_ra;
      if (done_out) done_out[kk] = done ? 1 : 0;
      SL.last_ra = ra;
      if (done) {
        ts_acc(acc, P, SL.L, M, hd, hist);
        ts_slot_reset(P, seed, M, SL, SL.ep + (uint64_t)n);
        acts_all += SL.L.c_act;
        S = make_stream(seed, SL.ep);
      }
      if (obs) ts_write_obs(SL.L.observe(P, M), unit, tabs, tn, P.k, obs + 10 * kk);
    }
    ts::ts_heap_store(M, SL.L.hused);
    slots[i] = SL;
  }
#endif
  acc.steps = steps_all;
  acc.activations = acts_all;
  __syncthreads();
  block_flush(acc, hist, sum);
}

__global__ void k_ts_observe_fields(ts::TsParams P, uint8_t* mem, int64_t lane_bytes,
                                    const TsSlot* slots, int64_t n, int32_t* f) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ts::TsMem M = ts::ts_mem_at(mem + i * lane_bytes, P);
  ts::TsLane L = slots[i].L;
  const ts::TsObs o = L.observe(P, M);
  const int32_t v[10] = {o.public_blocks,           o.private_blocks,
                         o.diff_blocks,             o.public_votes,
                         o.private_votes_inclusive, o.private_votes_exclusive,
                         o.public_depth,            o.private_depth_inclusive,
                         o.private_depth_exclusive, o.event};
  for (int j = 0; j < 10; ++j) f[10 * i + j] = v[j];
}

// engine.ml:258-261 on encoded observations (ssz_tools.ml:42-58 of_float)
__global__ void k_ts_policy(int32_t policy, int32_t k, int unit, const double* obs, int64_t n,
                            const uint8_t* table, int32_t dim, int32_t* actions) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double* x = obs + 10 * i;
  const double pi = 3.141592653589793;
  int32_t v[10];
  for (int j = 0; j < 10; ++j) {
    if (j == 9) {
      v[j] = unit ? (int32_t)floor(x[j] * 2.0) : (int32_t)x[j];
    } else if (!unit) {
      v[j] = (int32_t)x[j];
    } else {
      const double scale = j >= 3 ? (double)k : 1.0;
      v[j] = j == 2 ? (int32_t)__builtin_round(tan(pi * (x[j] - 0.5)) * scale)
                    : (int32_t)__builtin_round(tan(pi / 2.0 * x[j]) * scale);
    }
  }
  const ts::TsObs o{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9]};
  actions[i] = ts::ts_policy_t(policy, k, o, table, dim);
}

// ---------------------------------------------------------------- launchers

static unsigned ts_grid(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// the fused kernel's list-record window rows (TsMem.tl, ev_slab_plan): 8 (configs[3] +2.6 %
// in kernel, the exp-delay variant +0.5 %, profiles/r6q_ts_trec_window_ab.log; 16 rows leave
// no heap slab and lose); CPR_TS_TWIN overrides (0 = none) for A/B runs
static int32_t ts_trec_rows() {
  if (const char* v = getenv("CPR_TS_TWIN")) return std::max(0, std::min(64, atoi(v)));
  return 8;
}

hipError_t launch_ts_run_episodes(const ts::TsParams& P, uint64_t seed, uint64_t first,
                                  int64_t n_eps, uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                  cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                  const NodeOut& no) {
  CPR_LAYOUT_GUARD(lane_bytes, ts::ts_lane_bytes(P));
  // the resident grid; lpw < 64 runs lanes * lpw / 64 episodes at a time in it
  const int32_t lpw = event_lanes_per_wave();
  const unsigned blocks = (unsigned)(lanes / kBlock);
  const EvSlab sl = ev_slab_plan(blocks, (const void*)k_ts_run_episodes<SeedSource>, P.n,
                                 (kBlock / 64) * lpw, ts_trec_rows());
  CPR_LDS_GUARD(k_ts_run_episodes<SeedSource>, sl.bytes);
  hipLaunchKernelGGL(k_ts_run_episodes<SeedSource>, dim3(blocks), dim3(kBlock), sl.bytes, st, P,
                     SeedSource{seed, first}, n_eps, mem, lane_bytes, recs, sum, no, sl.kl,
                     sl.vw, lpw, sl.tw, (int32_t)sl.tw_off);
  return hipGetLastError();
}

hipError_t launch_ts_replay_episodes(const ts::TsParams& P, const TraceSource& src, int64_t n_eps,
                                 uint8_t* mem, int64_t lane_bytes, int64_t lanes,
                                 cpr_episode_record* recs, cpr_summary* sum, hipStream_t st,
                                  const NodeOut& no) {
  CPR_LAYOUT_GUARD(lane_bytes, ts::ts_lane_bytes(P));
  // the resident grid; lpw < 64 runs lanes * lpw / 64 episodes at a time in it
  const int32_t lpw = event_lanes_per_wave();
  const unsigned blocks = (unsigned)(lanes / kBlock);
  const EvSlab sl = ev_slab_plan(blocks, (const void*)k_ts_run_episodes<TraceSource>, P.n,
                                 (kBlock / 64) * lpw, ts_trec_rows());
  CPR_LDS_GUARD(k_ts_run_episodes<TraceSource>, sl.bytes);
  hipLaunchKernelGGL(k_ts_run_episodes<TraceSource>, dim3(blocks), dim3(kBlock), sl.bytes, st, P,
                     src, n_eps, mem, lane_bytes, recs, sum, no, sl.kl, sl.vw, lpw, sl.tw,
                     (int32_t)sl.tw_off);
  return hipGetLastError();
}

hipError_t launch_ts_reset(const ts::TsParams& P, uint64_t seed, uint8_t* mem, int64_t lane_bytes,
                           void* slots, int64_t n, const uint8_t* mask, const uint64_t* eps,
                           int unit, const double* tabs, int32_t tn, double* obs,
                           hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, ts::ts_lane_bytes(P));
  hipLaunchKernelGGL(k_ts_reset, dim3(ts_grid(n)), dim3(kBlock), 0, st, P, seed, mem, lane_bytes,
                     (TsSlot*)slots, n, mask, eps, unit, tabs, tn, obs);
  return hipGetLastError();
}

hipError_t launch_ts_step(const ts::TsParams& P, uint64_t seed, uint8_t* mem, int64_t lane_bytes,
                          void* slots, int64_t n, const int32_t* actions, int unit,
                          const double* tabs, int32_t tn, const StepBuffers& b, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, ts::ts_lane_bytes(P));
  hipLaunchKernelGGL(k_ts_step, dim3(ts_grid(n)), dim3(kBlock), 0, st, P, seed, mem, lane_bytes,
                     (TsSlot*)slots, n, actions, unit, tabs, tn, b);
  return hipGetLastError();
}

hipError_t launch_ts_rollout(const ts::TsParams& P, uint64_t seed, uint8_t* mem,
                             int64_t lane_bytes, void* slots, int64_t n, int64_t n_steps,
                             int unit, const double* tabs, int32_t tn, double* obs,
                             double* reward, uint8_t* done, cpr_summary* sum, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, ts::ts_lane_bytes(P));
  const int32_t lpw = rollout_lanes_per_wave(n, (const void*)k_ts_rollout);
  const int64_t per_block = (int64_t)(kBlock / 64) * lpw;
  const unsigned blocks = (unsigned)((n + per_block - 1) / per_block);
  const EvSlab sl = ev_slab_plan(blocks, (const void*)k_ts_rollout, P.n, (int32_t)per_block);
  CPR_LDS_GUARD(k_ts_rollout, sl.bytes);
  hipLaunchKernelGGL(k_ts_rollout, dim3(blocks), dim3(kBlock), sl.bytes, st, P, seed, mem,
                     lane_bytes, (TsSlot*)slots, n, n_steps, unit, tabs, tn, obs, reward, done,
                     sum, sl.kl, sl.vw, lpw);
  return hipGetLastError();
}

hipError_t launch_ts_observe_fields(const ts::TsParams& P, uint8_t* mem, int64_t lane_bytes,
                                    const void* slots, int64_t n, int32_t* f, hipStream_t st) {
  CPR_LAYOUT_GUARD(lane_bytes, ts::ts_lane_bytes(P));
  hipLaunchKernelGGL(k_ts_observe_fields, dim3(ts_grid(n)), dim3(kBlock), 0, st, P, mem,
                     lane_bytes, (const TsSlot*)slots, n, f);
  return hipGetLastError();
}

hipError_t launch_ts_policy(int32_t policy, int32_t k, int unit, const double* obs, int64_t n,
                            const uint8_t* table, int32_t dim, int32_t* actions,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_ts_policy, dim3(ts_grid(n)), dim3(kBlock), 0, st, policy, k, unit, obs, n,
                     table, dim, actions);
  return hipGetLastError();
}

size_t ts_slot_bytes() { return sizeof(TsSlot); }

int ts_blocks_per_cu() {
  int blocks = 0;
  hipError_t e =
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_ts_run_episodes<SeedSource>, kBlock, 0);
  if (e != hipSuccess || blocks <= 0) blocks = 2;
  return blocks;
}

}  // namespace cpr
