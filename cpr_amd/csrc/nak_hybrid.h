// Hybrid exact re-runs of Nakamoto gym episodes: the closed-form lane
// (nakamoto_lane.h) runs the episode until it flags a window it cannot vouch for (an
// overlap, an unresolved tie, a deep fork), the exact event engine (ethereum_lane.h, Nakamoto
// mode) takes over from the last quiescent trivial point before that window, and hands the
// episode back at the first quiescent trivial point past it. Only the stretch around the
// flagged window runs on the event engine, so a re-run costs about the closed form's time
// on one lane instead of ~2,000 activations of event handling.
//
// A quiescent trivial point is a gym step's position after the window's deliveries, before
// the next activation's clock, where (a) no message is in flight: the reference's queue
// holds the next clock event alone (a one-node skew heap, so its shape, and the order of
// every later pop, is the reference's), and (b) every node's view reduces to one block x:
// every defender prefers x, which a defender mined (or genesis), and the attacker's
// private and public blocks are x with no share pending. Everything the reference does
// from there depends on x (height, rewards, mining time, miner), the activation count, the
// latest activation's time and the step count only: later blocks all descend from x, so
// no walk (common ancestors, release targets, ancestor queries) goes below it, and blocks
// off that chain (orphans, discarded private blocks) are never reached again.
//
// Both directions need (a) to be provable from the closed form: it is when the next
// activation raises no overlap (the previous window's last arrival is before its clock), so
// a closed-form checkpoint is committed only after that activation went through clean.
// Networks whose queue keeps never-arriving messages (gamma = 0: +inf events shape the
// heap) have no such point and keep the whole-episode re-run; so do trace sources, random
// policies and episodes ended by max_progress / max_time (the launcher's condition).
#pragma once
#include "ethereum_lane.h"
#include "nakamoto_lane.h"

namespace cpr {

// the lane status bits that hand an episode over (kernels.hip kInexact)
constexpr uint32_t kHybInexact = ST_OVERLAP | ST_DEEP_FORK | ST_TIE_UNRESOLVED | ST_STALE_TIME;

// per-lane HBM for the closed-form lane of a hybrid re-run: private-chain ring, spill,
// tie-replay heap
__host__ __device__ inline int64_t hybrid_bytes(int32_t cap) {
  return eth::align128((int64_t)RING * 8) + eth::align128((int64_t)cap * 8) +
         eth::align128(REPLAY_BYTES);
}
__host__ __device__ inline LaneMem hybrid_mem(uint8_t* base, int32_t cap) {
  LaneMem M;
  M.ring = (double*)base;
  M.ring_stride = 1;
  M.spill = (double*)(base + eth::align128((int64_t)RING * 8));
  M.spill_stride = 1;
  M.cap = cap;
  M.replay = ReplayMem::at(base + eth::align128((int64_t)RING * 8) +
                           eth::align128((int64_t)cap * 8));
  M.times = true;
  return M;
}

// the closed-form lane's state is trivial after resolve: no private block, nothing pending,
// every defender on D (a defender's block or genesis), the attacker's base and public view D
__host__ __device__ inline bool nak_trivial(const NakLane& L) {
  return L.n == 0 && L.rel == 0 && L.n_ba == 0 && L.pend < 0 && L.onA == 0ull &&
         L.D.k != K_PRIVATE && L.pub.k == L.D.k && L.pub.h == L.D.h && L.p0.k == L.D.k &&
         L.p0.h == L.D.h;
}

// a quiescent trivial point: block x, activations done, the latest one's time, gym steps
struct HybridCk {
  BRef x;
  int32_t k;
  double t;
  int64_t steps;
};

// the closed form from its current state until the episode ends or it flags a window,
// committing each quiescent trivial point it passes to *ck. Not inlined, on local copies,
// and with the policy fixed at compile time: its loop gets a register allocation of its
// own rather than one shared with the event engine's code in the same kernel
// TT = 1 (d = 2 only): ties
// by the closed-form rule (tie_table_d2), whose uncovered cases flag TIE_UNRESOLVED and go
// to the engine like any flagged window, instead of the inlined heap replay
template <int POL, int TT, class St>
__host__ __device__ __attribute__((noinline)) void hybrid_closed(const NakParams& NPr,
                                                                 const St& Sr,
                                                                 const LaneMem& LMr,
                                                                 NakLane* Lp, int64_t* steps_p,
                                                                 HybridCk* ck_p) {
  const NakParams NP = NPr;
  const St S = Sr;
  const LaneMem LM = LMr;
  NakLane L = *Lp;
  int64_t steps = *steps_p;
  HybridCk ck = *ck_p;
  while (steps < NP.max_steps) {
    const NakLane::Draw dr = L.draw(NP, S);
    L.apply(L.policy_action<POL>(NP));
    L.resolve<St, 0, TT>(NP, S, LM);
    const bool triv = nak_trivial(L);
    const BRef cx = L.D;
    const int32_t ckk = L.k;
    const double ckt = L.t;
    const int64_t cks = steps;
    L.activate(NP, S, LM, dr);
    ++steps;
    if (L.status & kHybInexact) break;
    if (triv) {  // activation ckk went through clean: that point was quiescent
      ck.x = cx;
      ck.k = ckk;
      ck.t = ckt;
      ck.steps = cks;
    }
  }
  *Lp = L;
  *steps_p = steps;
  *ck_p = ck;
}

struct HybridResult {
  int32_t closed;   // 1: the episode ended on the closed form (hd), 0: on the engine (ehd)
  BRef hd;
  int32_t ehd;
  int64_t steps;
  int32_t acts;
  double now;
  int32_t entries;  // times the engine took over
  int32_t eng_acts; // activations the engine simulated (from its entry points)
};

// one gym episode (engine.ml:164-249); NP: the closed-form parameters (cap: spill slots,
// enough that no deep fork occurs), EP: the same configuration on the engine
template <class St>
__host__ __device__ inline HybridResult nak_hybrid_episode(const NakParams& NP,
                                                           const eth::EthParams& EP,
                                                           const St& S, const LaneMem& LM,
                                                           const eth::EthMem& EM,
                                                           eth::EthLane& E, NakLane& L) {
  HybridResult R{};
  int64_t steps = 0;
  // checkpoint: the latest quiescent trivial point; k = 0 is the reset
  HybridCk ck{};
  E.status = 0u;
  E.steps = 0;
  L.init();
  L.activate(NP, S, LM);
  for (;;) {
    // ---- closed form
    if (!(L.status & kHybInexact)) {
      if (NP.d == 2) {
        switch (NP.policy) {
          case P_HONEST: hybrid_closed<P_HONEST, 1>(NP, S, LM, &L, &steps, &ck); break;
          case P_SIMPLE: hybrid_closed<P_SIMPLE, 1>(NP, S, LM, &L, &steps, &ck); break;
          case P_ES2014: hybrid_closed<P_ES2014, 1>(NP, S, LM, &L, &steps, &ck); break;
          case P_SM1: hybrid_closed<P_SM1, 1>(NP, S, LM, &L, &steps, &ck); break;
          default: hybrid_closed<-1, 1>(NP, S, LM, &L, &steps, &ck); break;
        }
      } else {
        switch (NP.policy) {
          case P_HONEST: hybrid_closed<P_HONEST, 0>(NP, S, LM, &L, &steps, &ck); break;
          case P_SIMPLE: hybrid_closed<P_SIMPLE, 0>(NP, S, LM, &L, &steps, &ck); break;
          case P_ES2014: hybrid_closed<P_ES2014, 0>(NP, S, LM, &L, &steps, &ck); break;
          case P_SM1: hybrid_closed<P_SM1, 0>(NP, S, LM, &L, &steps, &ck); break;
          default: hybrid_closed<-1, 0>(NP, S, LM, &L, &steps, &ck); break;
        }
      }
      if (!(L.status & kHybInexact)) {
        R.closed = 1;
        R.hd = L.head(NP, LM);
        R.steps = steps;
        R.acts = L.k;
        R.now = L.t;
        return R;
      }
    }
    // ---- the engine, from the checkpoint, until a quiescent trivial point past the
    // activations the closed form has done (the flagged window among them)
    const int32_t stop_k = L.k;
    ++R.entries;
    bool done;
    int32_t ehd = 0;
    int32_t back = -1;
    if (ck.k == 0) {
      E.gym_reset(EP, S, EM);
      done = E.dead != 0;
    } else {
      const int32_t xs = ck.x.k + 1;  // the block of activation k is serial k + 1
      E.enter_trivial(EP, S, EM, xs, ck.x.h, ck.x.ra * 32, (ck.x.h - ck.x.ra) * 32, ck.x.tm,
                      miner_of(NP, S, ck.x.k), ck.k, ck.t, ck.steps + 1);
      const int32_t att = E.priv;
      uint32_t kind;
      int32_t blk, xb;
      const int32_t r = E.skip_or_stop(EP, S, EM, &kind, &blk, stop_k, &xb);
      if (r == 0) E.prepare(EP, EM, kind, blk);
      ehd = E.head(EP, EM, att);
      done = E.dead || !(E.steps < EP.max_steps);
    }
    while (!done) {
      const int32_t a = eth::lane_action(EP, E.observe(EP, EM, false));
      const int32_t sh = E.apply(EP, EM, a);
      if (sh >= 0) E.share(EP, EM, 0, sh);
      ++E.steps;
      const int32_t att = E.priv;
      uint32_t kind;
      int32_t blk, xb;
      const int32_t r = E.skip_or_stop(EP, S, EM, &kind, &blk, stop_k, &xb);
      if (r == 1) {
        back = xb;
        break;
      }
      if (r == 0) E.prepare(EP, EM, kind, blk);
      ehd = E.head(EP, EM, att);
      done = E.dead || !(E.steps < EP.max_steps);
    }
    R.eng_acts += E.c_act - ck.k;
    if (back < 0) {
      R.closed = 0;
      R.ehd = ehd;
      R.steps = E.steps;
      R.acts = E.c_act;
      R.now = E.now;
      return R;
    }
    // ---- back to the closed form at that point, before activation E.c_act's clock; it is
    // the new checkpoint (quiescent by construction)
    const eth::EBlock& xr = E.B(EP, EM, back);
    BRef x;
    x.h = xr.height;
    x.ra = xr.rew_att / 32;
    x.k = back - 1;
    x.fork = x.h;
    x.tm = xr.time;
    L.init();
    L.p0 = L.pub = L.D = L.A = L.b = x;
    L.lca_da = x.h;
    L.t = E.tclk;
    L.k = E.c_act;
    steps = E.steps - 1;
    ck.x = x;
    ck.k = L.k;
    ck.t = L.t;
    ck.steps = steps;
    L.activate(NP, S, LM);  // init left no window to overlap
    ++steps;
  }
}

}  // namespace cpr
