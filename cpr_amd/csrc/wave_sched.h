// Wave-coherent event dispatch for the per-lane event engines (bk_lane.h, ethereum_lane.h,
// ts_lane.h).
//
// A lane of these engines is one episode: pop the next event of its skew heap, run its
// handler (simulator.ml:421-508), repeat. Run as a plain loop, the 64 lanes of a wave sit in
// different handlers, so every iteration executes (and waits on the dependent memory
// chains of) nearly every handler once, each with a few lanes active. Here each lane holds
// its next work item (an event, or a gym interaction), items are grouped into classes by
// handler, and every iteration runs the one class most lanes hold: lanes that hold another
// class wait, keeping their item. Each lane still processes its own events in its own
// order, so every output is identical to the plain loop's (the parity tests compare both
// to the oracle); only the wave's interleaving of lanes changes.
//
// The adapter A gives the protocol specifics: A::Lane, A::Par, A::Mem and
//   begin(L, P, S, M)            init (simulator.ml:233-332) for a fresh episode
//   gym(P)                       engine.ml gym episode (else Simulator.loop ~activations)
//   loop_attacker(P)             loop mode: node 0's OnNode runs the attack space
//   pow0(ev)                     gym: the attacker's own Dag PoW event (engine.ml:108-121
//                                substitutes the agent's payload)
//   run_pow0(L, P, S, M, s)      that substitution
//   act(L, P, M)                 gym: policy (observe) -> apply (+ share) -> ++steps
//   head_gym(L, P, M, att)       engine.ml:195-206 head of a finished gym step
//   head_loop(L, P, M)           Simulator.loop's head
//   gym_done(L, P, M, hd)        engine.ml:209-214
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cpr {

// work classes (event types of bk_lane.h / ethereum_lane.h / ts_lane.h, plus the attacker's
// interaction and the gym's PoW substitution)
enum : int32_t {
  WK_CLOCK = 0, WK_DAG = 1, WK_TX = 2, WK_RX = 3, WK_ON = 4, WK_MV = 5, WK_MDV = 6,
  WK_ATTACK = 7, WK_POW0 = 8, WK_N = 9
};
// the next episode of a lane that finished one: a work queue when the launch has a counter
// (lanes that drew short episodes take more of them, so a launch of several episodes per lane
// lasts about its mean work, not its slowest lane's), else the static grid stride. Totals do
// not depend on which lane ran an episode (integer summaries, records by episode id).
__device__ inline int64_t ev_next_episode(unsigned long long* next, int64_t e, int64_t nthreads) {
  if (next == nullptr) return e + nthreads;
  return nthreads + (int64_t)atomicAdd(next, 1ull);
}

// cursor phases
enum : int32_t { PH_FRESH = 0, PH_RUN = 1, PH_OVER = 2, PH_IDLE = 3 };

struct EvCursor {
  double t;
  uint32_t ev;
  int32_t s;
  int64_t left;   // loop mode: activations still to simulate
  int32_t att;    // gym: the attacker's preference when the current step began
  int32_t hd;     // head of the episode once it is over
  int32_t cls;    // class of the held item, -1 none
  int32_t phase;  // gym: PH_FRESH until the first interaction; PH_OVER, PH_IDLE
};

template <class A, class St>
__device__ inline void ev_begin(typename A::Lane& L, const typename A::Par& P, const St& S,
                                const typename A::Mem& M, EvCursor& c) {
  A::begin(L, P, S, M);
  c.left = P.activations;
  c.att = 0;
  c.hd = 0;
  c.cls = -1;
  c.phase = PH_FRESH;
}

// pop the lane's next work item (loop mode: clocks past the activation budget are
// drained, simulator.ml:519-533), or end the episode
template <class A, class St>
__device__ inline void ev_fetch(typename A::Lane& L, const typename A::Par& P, const St& S,
                                const typename A::Mem& M, EvCursor& c) {
  const bool gym = A::gym(P);
  for (;;) {
    double t;
    uint32_t ev;
    int32_t s;
    if (L.dead || !L.pop(M, &t, &ev, &s)) {
      if (gym) {
        if (!L.dead) L.fail(6);  // engine.ml:120 "simulation should continue forever"
        c.hd = c.phase == PH_FRESH ? 0 : A::head_gym(L, P, M, c.att);
      } else {
        c.hd = A::head_loop(L, P, M);
      }
      c.phase = PH_OVER;
      return;
    }
    L.now = t;
    const uint32_t ty = ev & 7u;
    const int32_t node = (int32_t)(ev >> 5);
    if (!gym && ty == 0u) {  // EV_CLOCK
      if (c.left <= 0) continue;
      --c.left;
    }
    c.ev = ev;
    c.s = s;
    if (ty == 4u && node == 0 && (gym || A::loop_attacker(P)))
      c.cls = WK_ATTACK;
    else if (gym && A::pow0(ev))
      c.cls = WK_POW0;
    else
      c.cls = (int32_t)ty;
    return;
  }
}

// run the held item
template <class A, class St>
__device__ inline void ev_exec(typename A::Lane& L, const typename A::Par& P, const St& S,
                               const typename A::Mem& M, EvCursor& c) {
  const int32_t cls = c.cls;
  c.cls = -1;
  if (cls == WK_ATTACK && A::gym(P)) {
    // engine.ml:176-249 split at the interaction: prepare; head / done of the step that
    // led here; then the next action (policy on the observation, apply)
    L.prepare(P, M, (c.ev >> 3) & 3u, c.s);
    if (c.phase == PH_FRESH) {
      c.phase = PH_RUN;
      if (L.dead) {
        c.hd = 0;
        c.phase = PH_OVER;
        return;
      }
    } else {
      c.hd = A::head_gym(L, P, M, c.att);
      if (A::gym_done(L, P, M, c.hd)) {
        c.phase = PH_OVER;
        return;
      }
    }
    A::act(L, P, M);
    c.att = L.priv;
    return;
  }
  if (cls == WK_POW0) {
    A::run_pow0(L, P, S, M, c.s);
    return;
  }
  L.handle(P, S, M, c.ev, c.s);
}

// ---- rollouts (k_bk_rollout / k_ts_rollout: lockstep steps with the on-device policy,
// VecEnv auto-reset) under the same dispatch. A lane starts a launch at the attacker's
// decision point (prepared); its items are the events up to the next interaction
// (engine.ml:108-121 skip_to_interaction, with the PoW substitution), and the interaction
// itself ends the step: head / done / reward, then the observation and the next action, or
// on done the reset (init, whose events up to the first interaction run as items as well).
// An empty heap or a dead lane ends the step as gym_step does (no prepare, done).
constexpr uint32_t kRollFail = 0xffffffffu;  // the step's interaction is an episode failure

template <class A>
__device__ inline void roll_fetch(typename A::Lane& L, const typename A::Mem& M, EvCursor& c) {
  double t;
  uint32_t ev;
  int32_t s;
  if (L.dead) {
    c.ev = kRollFail;
    c.cls = WK_ATTACK;
    return;
  }
  if (!L.pop(M, &t, &ev, &s)) {
    L.fail(6);  // engine.ml:120 "simulation should continue forever"
    c.ev = kRollFail;
    c.cls = WK_ATTACK;
    return;
  }
  L.now = t;
  c.ev = ev;
  c.s = s;
  if ((ev & 7u) == 4u && (ev >> 5) == 0u)  // EV_ON at node 0: the attacker's interaction
    c.cls = WK_ATTACK;
  else if (A::pow0(ev))
    c.cls = WK_POW0;
  else
    c.cls = (int32_t)(ev & 7u);
}

// the class the most lanes of this wave hold (-1: none), wave-uniform
__device__ inline int32_t ev_choose(int32_t cls) {
  int32_t best = -1, bn = 0;
#pragma unroll
  for (int32_t k = 0; k < WK_N; ++k) {
    const int32_t n = __popcll(__ballot(cls == k));
    if (n > bn) {
      bn = n;
      best = k;
    }
  }
  return __builtin_amdgcn_readfirstlane(best);
}

}  // namespace cpr
