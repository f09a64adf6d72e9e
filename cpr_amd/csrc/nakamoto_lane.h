// One GPU lane = one gym episode of the nakamoto_ssz attack space (SSZ'16, four actions)
// on the selfish-mining network the gym builds, or one Simulator.loop task on the
// two-agents network. The reference runs an event-driven simulator with a DAG, per-node
// views and a skew-heap event queue (simulator.ml:421-508); for Nakamoto on these
// networks every outcome-relevant fact fits in a few block references and counters, so
// the lane is a branch-light integer state machine driven by the keyed stream.
//
// What the lane tracks, and the reference code it stands for:
//   p0, n, rel      attacker private chain = p0 + n withheld/released blocks, released
//                   prefix rel (nakamoto_ssz.ml:156-260, simulator.ml:401-419 share)
//   pub             attacker's model of the defender head (deliver_private_to_public,
//                   nakamoto_ssz.ml:191-218), with its common-ancestor height `fork`
//   D, A, onA       defender tips: every defender holds D or A (bitmask); honest
//                   update_head (nakamoto.ml:85-95) with first-received tie breaking
//   b, wminer       the block of the activation the attacker is reacting to
//   BRef.ra         attacker reward count along the chain = rewards[0] (simulator.ml:377-388)
//   BRef.fork       height of the block's common ancestor with the private chain
//                   (Dagtools.common_ancestor, dagtools.ml:102-121)
//
// Per-lane memory (LaneMem): the private chain's mining times in a 16-slot ring (LDS in
// the fused kernel) with a global spill for deeper chains. Every other block the lane can
// name carries its mining time in its BRef, so the head's chain time needs no log.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpr_stream.h"

#pragma clang fp contract(off)

namespace cpr {

// Lane methods are inlined into the kernel before any optimisation: optimised on their own,
// `c ? this->x.f : this->y.f` becomes a load from a selected field address, which keeps
// the whole lane struct in scratch memory once inlined.
#define CPR_AI __attribute__((always_inline))

enum : int32_t { A_ADOPT = 0, A_OVERRIDE = 1, A_MATCH = 2, A_WAIT = 3 };
enum : int32_t { P_HONEST = 0, P_SIMPLE = 1, P_ES2014 = 2, P_SM1 = 3, P_TABLE = 4 };
enum : uint32_t {
  ST_TIE = 1u,
  ST_OVERLAP = 2u,
  ST_DEEP_FORK = 4u,
  ST_TIE_UNRESOLVED = 8u,
  ST_STALE_TIME = 16u,
  // internal (never output): a deferred race went otherwise than assumed; the episode is
  // listed and run again with the races decided eagerly (k_run_episodes, TT = 2)
  ST_RACE_REDO = 1u << 20
};

constexpr int32_t RING = 16;   // private-chain slots kept in the ring
constexpr int32_t RCAP = 512;  // tie-replay heap nodes per lane
constexpr int32_t RMAX = 16;   // released blocks per window the replay supports
constexpr int64_t REPLAY_BYTES = 8704;  // RCAP * 16 + 2 * (RMAX + 1) * 8, rounded

struct ReplayNode {
  double t;
  int32_t ev;
  int16_t l, r;
};

struct ReplayMem {
  ReplayNode* nodes;  // RCAP
  uint64_t* masks;    // 2 * (RMAX + 1): received, visible per block, bit j-1 = defender j
  __host__ __device__ static inline ReplayMem at(uint8_t* base) {
    ReplayMem m;
    m.nodes = (ReplayNode*)base;
    m.masks = (uint64_t*)(base + (int64_t)RCAP * sizeof(ReplayNode));
    return m;
  }
};

struct LaneMem {
  double* ring;       // ring[(m & (RING-1)) * ring_stride]: mining time of chain block m
  double* spill;      // spill[m * spill_stride], m < cap: chain blocks evicted from the ring
  int64_t ring_stride, spill_stride;
  int32_t cap;
  ReplayMem replay;
  // block mining times are tracked (BRef.tm, the ring and its spill): they feed only the
  // record's chain_time. A kernel that writes no records sets this to a compile-time false
  // and every time computation, ring store and spill store drops out of the inlined lane
  // (the summary does not depend on them).
  bool times = true;
  // deferred races (NakLane::resolve<.., TT = 2>, enqueue_race, verify_races): the wave's
  // dense list of unverified races (rq_cap entries, shared by its lanes), the wave's
  // outcome flags and episode words (the keyed stream's e0, e1: a race is verified on its
  // owner's stream), one and two per lane, and this lane's index in the wave
  uint4* rq = nullptr;
  int32_t rq_cap = 0;
  int32_t* rflag = nullptr;
  uint32_t* rep = nullptr;
  int32_t lane = 0;
  int32_t wave = 1;  // lanes that share the list (WAVE in the kernels; the host tests emulate more)
};

// deferred races: queue entries per lane of a wave (the list is the wave's: 64 times this)
#ifndef CPR_RQ_LANE
#define CPR_RQ_LANE 6
#endif
constexpr int32_t RQ_LANE = CPR_RQ_LANE;
// words of a NakLane without block times (NakLane::pack, the host tests' state comparison)
constexpr int32_t CK_WORDS = 38;

// wave primitives of the deferred races (a wave of one lane on the host)
#if defined(__HIP_DEVICE_COMPILE__)
constexpr int32_t WAVE = 64;
__device__ inline CPR_AI uint64_t wave_ballot(bool p) { return __ballot(p ? 1 : 0); }
__device__ inline CPR_AI int32_t lanes_below(uint64_t m) {
  return (int32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                            __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// LDS written by some lanes, then read by others of the same wave: keep the order
__device__ inline CPR_AI void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}
// several lanes may flag the same owner in one pass
__device__ inline CPR_AI void flag_or(int32_t* p, int32_t v) { atomicOr(p, v); }
#else
constexpr int32_t WAVE = 1;
inline uint64_t wave_ballot(bool p) { return p ? 1ull : 0ull; }
inline int32_t lanes_below(uint64_t) { return 0; }
inline void wave_lds_order() {}
inline void flag_or(int32_t* p, int32_t v) { *p |= v; }
#endif

constexpr int32_t K_GENESIS = -1, K_PRIVATE = -2;

struct BRef {
  int32_t h;     // height (nakamoto.ml:11-14)
  int32_t ra;    // attacker blocks on the chain up to here
  int32_t k;     // activation that mined it (DAG serial - 1); K_GENESIS; K_PRIVATE for the
                 // attacker's private-chain blocks (mined by node 0, named by chain index)
  int32_t fork;  // height of the common ancestor with the attacker's private chain
  double tm;     // mining time = Simulator.timestamp for these networks (simulator.ml:14-21)
};

// dst := c ? src : dst, field by field (a whole-struct conditional copy would make the
// compiler select between the two objects' addresses and put them in scratch memory)
__host__ __device__ inline CPR_AI void sel(BRef& dst, bool c, const BRef& src) {
  dst.h = c ? src.h : dst.h;
  dst.ra = c ? src.ra : dst.ra;
  dst.k = c ? src.k : dst.k;
  dst.fork = c ? src.fork : dst.fork;
  dst.tm = c ? src.tm : dst.tm;
}

struct NakParams {
  uint64_t t_att;       // floor(alpha * 2^32)
  int32_t d;            // defenders
  int32_t arrive;       // attacker messages reach defenders (gamma > 0 or two-agents)
  double ev;            // activation delay (expected block interval)
  double delta;         // defender -> defender delay (network.ml:93)
  double dmax;          // attacker -> defender uniform [0, dmax) (network.ml:68-75)
  int64_t max_steps;
  double max_progress;
  double max_time;
  int32_t policy;
  int32_t table_dim;
  const uint8_t* table;
  int32_t cap;          // spill slots per lane
  int32_t abstract_g;   // CPR_NET_ABSTRACT_GAMMA: match races decided by per-defender coins
  double gamma;         //   U(k, 0, j) < gamma (zero delays otherwise)
  // lazy clock (NakLane LZ): a clock uniform U (53-bit integer) below u_lazy draws a delay
  // > 2 delta, which no later window can overlap (set by the launcher, lazy_clock_ok)
  uint64_t u_lazy;
  // fused-episode launches (k_run_episodes): device counter of the episodes handed out
  // beyond the first round, in chunks of one wave (zeroed before the launch); null = the
  // static grid-stride assignment
  unsigned long long* next = nullptr;
};

// u_lazy = floor(exp(-2.5 delta / ev) 2^53): U < u_lazy gives dt > 2 delta with margin to
// spare for the log's rounding
inline uint64_t lazy_threshold(const NakParams& P) {
  return (uint64_t)std::floor(std::exp(-2.5 * P.delta / P.ev) * 9007199254740992.0);
}

// the lazy clock (NakLane LZ) is exact when a delay above 2 delta cannot overlap anywhere in
// the episode: ulp(t) <= delta / 4 for every reachable clock t (each delay is at most
// 53 ln 2 ev < 40 ev, or +inf, which the lane handles apart), and max_steps alone ends it
inline bool lazy_clock_ok(const NakParams& P) {
  if (!(P.delta > 0.0) || !std::isfinite(P.delta) || !(P.ev > 0.0) || !std::isfinite(P.ev))
    return false;
  if (P.max_progress < __builtin_inf() || P.max_time < __builtin_inf()) return false;
  // (<= 2^14 steps: the race kernel's clock bound esum, <= 150500 a step, stays in 32 bits)
  if (P.max_steps <= 0 || P.max_steps > (1ll << 14)) return false;
  const double tmax = ((double)P.max_steps + 2.0) * P.ev * 40.0;
  if (!(std::ldexp(1.0, std::ilogb(tmax) - 52) <= P.delta / 4.0)) return false;
  // delta > ~14.7 ev puts the threshold at 0: no uniform can skip the check, and the lane's
  // skip test (u - 1 >= u_lazy - 1) would wrap and skip every one of them instead
  return lazy_threshold(P) >= 2ull;
}

__host__ __device__ inline CPR_AI uint64_t all_mask(int32_t d) {
  return d >= 64 ? ~0ull : ((1ull << d) - 1ull);
}

// nakamoto_ssz.ml:274-340 (policy registry: sapirshtein-2016-sm1, eyal-sirer-2014,
// simple, honest)
__host__ __device__ inline CPR_AI int32_t nak_policy(int32_t policy, int32_t h, int32_t a, int32_t ev,
                                              const uint8_t* table, int32_t dim) {
  switch (policy) {
    case P_HONEST:
      return a > h ? A_OVERRIDE : (a < h ? A_ADOPT : A_WAIT);
    case P_SIMPLE:
      return h > 0 ? (a < h ? A_ADOPT : A_OVERRIDE) : A_WAIT;
    case P_ES2014:
      if (a < h) return A_ADOPT;
      if (h == 0 && a == 1) return A_WAIT;
      if (h == 1 && a == 1) return A_MATCH;
      if (h == 1 && a == 2) return A_OVERRIDE;
      if (h == 2 && a == 1) return A_ADOPT;
      if (h > 0) return (a - h == 1) ? A_OVERRIDE : A_MATCH;
      return A_WAIT;
    case P_SM1:
      if (h > a) return A_ADOPT;
      if (h == 1 && a == 1) return A_MATCH;
      if (h == a - 1 && h >= 1) return A_OVERRIDE;
      return A_WAIT;
    default: {
      const int32_t hp = h < 0 ? 0 : (h >= dim ? dim - 1 : h);
      const int32_t ap = a < 0 ? 0 : (a >= dim ? dim - 1 : a);
      return (int32_t)table[(hp * dim + ap) * 2 + ev];
    }
  }
}

// ---- exact replay of one delivery window (used only when two deliveries tie in fp64)
//
// At every activation the reference's event queue holds exactly one element, the clock
// (all earlier windows have drained; overlaps are flagged separately). So when a defender
// receives the fresh defender block and the attacker's matching release at the very same
// instant, the winner is fixed by replaying this window's events through the same skew
// heap (orderedQueue.ml:17-47) with the handlers of simulator.ml:421-508. Blocks of the
// window: x = 0 is the defender block b, x = 1..r the released chain a_rlo..a_rhi.

enum : int32_t { RE_SC = 0, RE_SC2 = 1, RE_DAG = 2, RE_MV = 3, RE_ON = 4, RE_MDV = 5, RE_TX = 6, RE_RX = 7 };

__host__ __device__ inline CPR_AI int32_t re_ev(int32_t ty, int32_t node, int32_t x) {
  return ty | (node << 3) | (x << 11);
}

struct SkewHeapLane {
  ReplayNode* n;
  int32_t root, freeh, used;
  bool ok;
  __host__ __device__ inline CPR_AI int32_t alloc(double t, int32_t ev) {
    int32_t i;
    if (freeh >= 0) {
      i = freeh;
      freeh = n[i].l;
    } else if (used < RCAP) {
      i = used++;
    } else {
      ok = false;
      return -1;
    }
    n[i].t = t;
    n[i].ev = ev;
    n[i].l = -1;
    n[i].r = -1;
    return i;
  }
  // orderedQueue.ml:17-26, iterative: new equal-time elements sink below existing ones
  __host__ __device__ inline CPR_AI void push(double t, int32_t ev) {
    int32_t parent = -1;
    int32_t node = root;
    for (;;) {
      if (node < 0) {
        const int32_t a = alloc(t, ev);
        if (parent < 0)
          root = a;
        else
          n[parent].l = (int16_t)a;
        return;
      }
      if (t < n[node].t) {
        const double ot = n[node].t;
        const int32_t oe = n[node].ev;
        n[node].t = t;
        n[node].ev = ev;
        t = ot;
        ev = oe;
      } else {
        const int16_t tmp = n[node].l;
        n[node].l = n[node].r;
        n[node].r = tmp;
      }
      parent = node;
      node = n[node].l;
    }
  }
  // orderedQueue.ml:28-47 (ties prefer the left subtree)
  __host__ __device__ inline CPR_AI bool pop(double* t, int32_t* ev) {
    if (root < 0) return false;
    *t = n[root].t;
    *ev = n[root].ev;
    int32_t parent = -1, side = 0, node = root;
    for (;;) {
      const int32_t l = n[node].l, r = n[node].r;
      int32_t repl = -2;
      if (r < 0)
        repl = l;
      else if (l < 0)
        repl = r;
      if (repl != -2) {
        if (parent < 0)
          root = repl;
        else if (side == 0)
          n[parent].l = (int16_t)repl;
        else
          n[parent].r = (int16_t)repl;
        n[node].l = (int16_t)freeh;
        freeh = node;
        return true;
      }
      if (n[l].t <= n[r].t) {
        n[node].t = n[l].t;
        n[node].ev = n[l].ev;
        parent = node;
        side = 0;
        node = l;
      } else {
        n[node].t = n[r].t;
        n[node].ev = n[r].ev;
        parent = node;
        side = 1;
        node = r;
      }
    }
  }
};

// Replay of a defender-mined window in which the attacker released a_rlo..a_rhi (shared
// at activation count kw, top first), the top one at the fresh block's height. Returns the
// non-miner defenders that end on the released top (first received wins,
// nakamoto.ml:85-89). *ok = false on capacity overflow.
template <class St>
__host__ __device__ inline CPR_AI uint64_t tie_replay(const NakParams& P, const St& S,
                                               const ReplayMem& M, int32_t miner, double t,
                                               int32_t rlo, int32_t rhi, int32_t kw, bool* ok) {
  const int32_t r = rhi - rlo + 1;
  if (r > RMAX) {
    *ok = false;
    return 0ull;
  }
  uint64_t* recv = M.masks;
  uint64_t* vis = M.masks + (RMAX + 1);
  for (int32_t x = 0; x <= r; ++x) recv[x] = vis[x] = 0ull;
  bool recv0 = false, vis0 = false;
  uint64_t decided = 0ull, on_top = 0ull;
  SkewHeapLane H{M.nodes, -1, -1, 0, true};
  H.push(t, re_ev(RE_SC, 0, 0));
  double now;
  int32_t ev;
  while (H.ok && H.pop(&now, &ev)) {
    const int32_t ty = ev & 7, j = (ev >> 3) & 255, x = ev >> 11;
    const uint64_t bit = j ? (1ull << (j - 1)) : 0ull;
    switch (ty) {
      case RE_SC:  // StochasticClock: Dag now, next clock later (simulator.ml:465-472)
        H.push(now, re_ev(RE_DAG, miner, 0));
        H.push(__builtin_inf(), re_ev(RE_SC2, 0, 0));
        break;
      case RE_SC2:
        *ok = true;
        return on_top;
      case RE_DAG:  // append, MakeVisible (:473-480)
        H.push(now, re_ev(RE_MV, miner, 0));
        break;
      case RE_MV: {  // :424-450
        if (j == 0) {
          if (!vis0) {
            vis0 = true;
            H.push(now, re_ev(RE_ON, 0, 0));
            H.push(now, re_ev(RE_MDV, 0, 0));
          }
          break;
        }
        const bool pvis = x <= 1 ? true : ((vis[x - 1] & bit) != 0ull);
        if (!(vis[x] & bit) && pvis) {
          vis[x] |= bit;
          H.push(now, re_ev(RE_ON, j, x));
          H.push(now, re_ev(RE_MDV, j, x));
        }
        break;
      }
      case RE_ON:  // :451-464
        if (j == 0) {
          // the attacker's interaction; its action shares a_rhi, recursing to a_rlo
          for (int32_t m = rhi; m >= rlo; --m) H.push(now, re_ev(RE_TX, 0, m - rlo + 1));
        } else if (j == miner && x == 0) {
          H.push(now, re_ev(RE_TX, miner, 0));  // honest PoW handler shares b
        } else if (j != miner && !(decided & bit)) {
          if (x == 0) {
            decided |= bit;
          } else if (x == r) {
            decided |= bit;
            on_top |= bit;
          }
        }
        break;
      case RE_MDV:  // :494-508, children of a_m is a_m+1 only
        if (j != 0 && x >= 1 && x < r && (recv[x + 1] & bit)) H.push(now, re_ev(RE_MV, j, x + 1));
        break;
      case RE_TX:  // :481-487, links in destination order
        if (x == 0) {
          H.push(now + 0.0, re_ev(RE_RX, 0, 0));
          for (int32_t jj = 1; jj <= P.d; ++jj)
            if (jj != miner) H.push(now + P.delta, re_ev(RE_RX, jj, 0));
        } else {
          const uint32_t off = (uint32_t)(r - x);  // share order: top first
          for (int32_t jj = 1; jj <= P.d; ++jj) {
            H.push(now + S.link((uint32_t)kw, off, (uint32_t)jj, P.dmax), re_ev(RE_RX, jj, x));
          }
        }
        break;
      case RE_RX:  // :488-493
        if (j == 0) {
          if (!recv0) {
            recv0 = true;
            H.push(now, re_ev(RE_MV, 0, 0));
          }
        } else if (!(recv[x] & bit)) {
          recv[x] |= bit;
          H.push(now, re_ev(RE_MV, j, x));
        }
        break;
    }
  }
  *ok = false;
  return 0ull;
}

// tie_replay's outcome in closed form for two defenders and one released block (the
// attacker matching with one block, the only tie SM1 and ES'14 make at d = 2): the window's
// events are then fixed, so the heap's order of the two equal-time deliveries at the
// non-miner defender j = 3 - miner depends only on the miner and on where the miner's own
// copy of the release lands relative to that instant: j ends on the released block iff
//   miner 1: that copy arrives at the tie instant too;
//   miner 2: it arrives no later than the tie instant.
// Tabulated by running tie_replay over both miners and the four orderings (arrival at t,
// inside (t, t + delta), at t + delta, after), for several t and delta
// (tests/native/tie_table.cpp, asserted in the CPU suite); the host fuzzer compares lanes
// that use it with the oracle (tests/native/lane_vs_oracle.cpp).
template <class St>
__host__ __device__ inline CPR_AI uint64_t tie_table_d2(const NakParams& P, const St& S,
                                                        int32_t miner, double t, int32_t kw) {
  const double tb = t + P.delta;
  const double vm = t + S.link((uint32_t)kw, 0u, (uint32_t)miner, P.dmax);
  const bool on = miner == 1 ? vm == tb : !(vm > tb);
  return on ? (1ull << (2 - miner)) : 0ull;  // bit j - 1, j = 3 - miner
}

struct NakLane {
  double t;          // time of the latest activation (clock.now at the interaction)
  int32_t k;         // activations so far (clock.c_activations); the same in every lane of
                     // a wave, so the keyed-stream counter and release keys stay uniform
  int32_t n;         // private blocks above p0 (observable state)
  int32_t rel;       // released prefix of the private chain
  int32_t n_ba;      // private length of the BetweenActions state (attacker's preferred)
  int32_t pend;      // pending private->public message: chain index, -1 = none
  int32_t wminer;    // miner of the current window's activation (0 = attacker)
  int32_t event;     // observation event: 0 ProofOfWork, 1 Network; bit 1: the window's
                     // defender block became pub (apply's `fresh`)
  int32_t rlo, rhi;  // chain indices released in the current window (shared at count k);
                     // kept until the next activation, whose overlap check reads them
  uint32_t status;
  BRef p0, pub, D, A, b;
  uint64_t onA;      // bit j-1: defender j prefers A (else D)
  int32_t lca_da;    // height of LCA(D, A)
  int32_t w_hasb;    // the window resolved last delivered a defender block
  double w_bound;    // conservative bound on that window's latest arrival
  int32_t qn;        // deferred races in the wave's list (TT = 2; the same in every lane)
  uint32_t rw;       // the race resolve<.., 2> took as decided: wminer | rlo << 2 |
                     // rhi << 14, 0 = none (enqueue_race lists it)
  int32_t tinf;      // LZ: a clock delay of +inf was drawn (the clock is +inf from then on)
  uint32_t esum;     // LZ = 2: sum over the activations so far of lz_term(U), so that
                     // t <= esum ev / 4096 (lz_term bounds -log(U 2^-53) in units of 2^-12)

  __host__ __device__ inline CPR_AI double chain_t(const LaneMem& M, int32_t m) const {
    if (!M.times) return 0.0;
    // two loads in their own address spaces (ds_read, then a rare global load) rather than
    // a select of pointers, which would compile to a generic flat load
    double v = M.ring[(m & (RING - 1)) * M.ring_stride];
    // volatile: stops the compiler from sinking both loads into one generic (flat) load
    if (m <= n - RING) v = *(volatile const double*)&M.spill[(int64_t)m * M.spill_stride];
    return v;
  }

  // chain block m (m >= 1) of the private chain; p0 for m <= 0
  __host__ __device__ inline CPR_AI BRef chain_ref(const LaneMem& M, int32_t m) const {
    BRef r;
    const bool above = m > 0;
    const int32_t mm = above ? m : 0;
    r.h = p0.h + mm;
    r.ra = p0.ra + mm;
    r.k = above ? K_PRIVATE : p0.k;
    r.fork = r.h;  // p0.fork == p0.h always (apply sets it on Adopt)
    r.tm = above ? chain_t(M, m) : p0.tm;
    return r;
  }

  __host__ __device__ inline CPR_AI void init() {
    BRef g;
    g.h = 0; g.ra = 0; g.k = K_GENESIS; g.fork = 0; g.tm = 0.0;
    p0 = pub = D = A = b = g;
    t = 0.0;
    k = 0; n = 0; rel = 0; n_ba = 0; pend = -1; wminer = 0; event = 0;
    rlo = 1; rhi = 0; status = 0u; onA = 0ull; lca_da = 0;
    w_hasb = 0; w_bound = -__builtin_inf();
    qn = 0; rw = 0u; tinf = 0; esum = 0u;
  }

  // the lane's state without block times (the summary-only kernels' whole state) as
  // CK_WORDS words
  __host__ __device__ inline CPR_AI void pack(uint32_t* c) const {
    int32_t f = 0;
    auto w = [&](uint32_t x) { c[f++] = x; };
    auto wd = [&](double x) { const uint64_t b = bitsd(x); w((uint32_t)b); w((uint32_t)(b >> 32)); };
    auto wb = [&](const BRef& r) { w((uint32_t)r.h); w((uint32_t)r.ra); w((uint32_t)r.k); w((uint32_t)r.fork); };
    wd(t); w((uint32_t)k); w((uint32_t)n); w((uint32_t)rel); w((uint32_t)n_ba); w((uint32_t)pend);
    w((uint32_t)wminer); w((uint32_t)event); w((uint32_t)rlo); w((uint32_t)rhi); w(status);
    wb(p0); wb(pub); wb(D); wb(A); wb(b);
    w((uint32_t)onA); w((uint32_t)(onA >> 32)); w((uint32_t)lca_da); w((uint32_t)w_hasb);
    wd(w_bound);
  }

  // latest finite arrival of the window resolved last (exact; only evaluated when the next
  // activation lands inside the conservative bound, ~1e-9 of activations in the gym). Its
  // coordinates are still live: t and k are the window's, rlo/rhi its release.
  template <class St>
  __host__ __device__ inline CPR_AI double window_last_arrival(const NakParams& P,
                                                        const St& S) const {
    return window_last_arrival_at(P, S, t);
  }
  // the same with the window's time given (the lazy clock recomputes it)
  template <class St>
  __host__ __device__ inline CPR_AI double window_last_arrival_at(const NakParams& P,
                                                                  const St& S, double tw) const {
    double last = -__builtin_inf();
    if (w_hasb && P.d >= 2) last = tw + P.delta;
    if (rhi >= rlo && P.arrive) {
      for (int32_t j = 1; j <= P.d; ++j)
        for (int32_t m = rlo; m <= rhi; ++m) {
          const double a = tw + S.link((uint32_t)k, (uint32_t)(rhi - m), (uint32_t)j, P.dmax);
          last = a > last ? a : last;
        }
    }
    return last;
  }

  // StochasticClock + Dag + the attacker's prepare (simulator.ml:465-480, engine.ml:108-121,
  // nakamoto_ssz.ml:191-218). Written as selects: the lanes of a wave take different
  // sides of every decision, so both sides run anyway and the merges cost no copies.
  struct Draw {
    double dt;
    int32_t miner;
    uint64_t u;  // LZ: the clock uniform as a 53-bit integer (dt not computed)
  };
  // the next activation's miner and clock delay: they depend on the activation count only,
  // so the gym loop draws them first and the Philox / log chain overlaps the policy and
  // apply selects of the same iteration
  template <class St, int LZ = 0>
  __host__ __device__ inline CPR_AI Draw draw(const NakParams& P, const St& S) const {
    return draw_at<St, LZ>(P, S, k);
  }
  // the draws of activation kk (kk = k: the next one)
  template <class St, int LZ = 0>
  __host__ __device__ inline CPR_AI Draw draw_at(const NakParams& P, const St& S,
                                                 int32_t kk) const {
    Draw d;
    if constexpr (LZ) {
      d.u = S.act_u((uint32_t)kk, P.t_att, P.d, &d.miner);
      d.dt = 0.0;
    } else {
      d.u = 0;
      d.dt = S.act((uint32_t)kk, P.t_att, P.d, P.ev, &d.miner);
    }
    return d;
  }

  // LZ = lazy clock, for the summary-only kernels (no records), where the clock feeds only
  // the overlap check and, at gamma = .5 (LZ = 2, deferred races), the races' same-instant
  // test. The overlap check can fire only when the previous window sent a message (its
  // defender block at t + delta, a release at t + U dmax <= t + delta) and the new activation
  // comes no later. A uniform below P.u_lazy draws dt > 2 delta, which (with the launcher's
  // bound ulp(t) <= delta / 4 over the whole episode) rules that out without the log, so the
  // clock is neither drawn nor summed. Only the rest, ~2.5 delta / ev of activations, takes
  // this branch: it sums the clock from the episode's first draw in the same order as the
  // eager lane and makes the same comparisons, so the status bits (and the exact re-run an
  // overlap sends the episode to) are the eager lane's. tinf: a zero uniform (delay +inf)
  // leaves the eager lane's clock at +inf, where every later window with a message
  // overlaps. LZ = 2 races: see races_check.
  template <class St>
  __host__ __device__ inline void lazy_overlap_check(const NakParams& P, const St& S,
                                                     uint64_t u) {
    const bool wb = w_hasb != 0 && P.d >= 2;
    const bool wr = rhi >= rlo && P.arrive;  // the previous window's release
    if (tinf) {
      if (wb || wr) status |= ST_OVERLAP;
      return;
    }
    if (u == 0ull) {  // this activation's delay is +inf: t + inf > every arrival
      tinf = 1;
      return;
    }
    if (!wb && !wr) return;
    double tp = 0.0;
    for (int32_t j = 0; j < k; ++j) tp = tp + S.clock((uint32_t)j, P.ev);
    const double tn = tp + S.clock((uint32_t)k, P.ev);
    double bound = wb ? tp + P.delta : -__builtin_inf();
    if (wr) {
      const double ub = tp + (P.dmax - 0.0);
      bound = ub > bound ? ub : bound;
    }
    if (tn <= bound) {
      if (tn <= window_last_arrival_at(P, S, tp)) status |= ST_OVERLAP;
    }
  }
  // an upper bound of -log(U 2^-53) in units of 2^-12: with uh = the top 24 bits of U
  // (U >> 29, so U >= uh 2^29), -log(U 2^-53) <= (24 - log2 uh) ln 2. log2 in f32 (the
  // hardware's v_log_f32 on the device, within a few 1e-6 of the true value; std::log2f on
  // the host: the bound need not be the same bits on both sides, only a bound) with ln 2
  // rounded up and a margin of 8 units for log2's and the f32 fma's rounding, plus 1 for
  // the truncation. uh = 0 (U < 2^29): 53 ln 2 and some. U = 0 (+inf) is tinf's case
  __host__ __device__ static inline CPR_AI uint32_t lz_term(uint64_t u) {
    const uint32_t uh = (uint32_t)(u >> 29);
#if defined(__HIP_DEVICE_COMPILE__)
    const float y = __builtin_amdgcn_logf((float)uh);
#else
    const float y = std::log2((float)uh);
#endif
    const float b = __builtin_fmaf(y, -2839.1309f, 68148.2f);  // 4096 ((24 - y) ln2) + 9
    return uh == 0u ? 150500u : (uint32_t)b;
  }

  template <class St, int LZ = 0>
  __host__ __device__ inline CPR_AI void activate(const NakParams& P, const St& S, const LaneMem& M) {
    activate<St, LZ>(P, S, M, draw<St, LZ>(P, S));
  }

  template <class St, int LZ = 0>
  __host__ __device__ inline CPR_AI void activate(const NakParams& P, const St& S, const LaneMem& M,
                                                  const Draw dr) {
    const int32_t miner = dr.miner;
    const double tn = t + dr.dt;
    if constexpr (LZ) {
      // u >= u_lazy, or u == 0 (unsigned wrap), or a +inf clock: the exact check
      if ((dr.u - 1ull) >= (P.u_lazy - 1ull) || tinf) lazy_overlap_check(P, S, dr.u);
      if constexpr (LZ == 2) esum += lz_term(dr.u);
    } else {
      if (tn <= w_bound) {
        if (tn <= window_last_arrival(P, S)) status |= ST_OVERLAP;
      }
      t = tn;
    }
    const int32_t ka = k;
    ++k;
    wminer = miner;
    rlo = 1;
    rhi = 0;
    // deliver the pending release to the attacker's public model (strict >)
    sel(pub, pend >= 0 && p0.h + pend > pub.h, chain_ref(M, pend));
    const bool att = miner == 0;
    if (att) {
      int32_t m = n + 1;
      if (m >= M.cap) {
        status |= ST_DEEP_FORK;
        m = M.cap - 1;
      }
      if (M.times) {
        double* slot = M.ring + (m & (RING - 1)) * M.ring_stride;
        if (m > RING) M.spill[(int64_t)(m - RING) * M.spill_stride] = *slot;  // evict
        *slot = tn;
      }
      n = m;
    }
    // the defender block (its fields are meaningless when the attacker mined)
    const bool par_a = ((onA >> ((miner - 1) & 63)) & 1ull) != 0ull;
    b.h = (par_a ? A.h : D.h) + 1;
    b.ra = par_a ? A.ra : D.ra;
    b.fork = par_a ? A.fork : D.fork;
    b.k = ka;
    b.tm = M.times ? tn : 0.0;
    const bool fresh = !att && b.h > pub.h;
    sel(pub, fresh, b);
    event = att ? 0 : (fresh ? 3 : 1);
  }

  __host__ __device__ inline CPR_AI void observe(int32_t* pub_blocks, int32_t* priv_blocks,
                                          int32_t* diff_blocks, int32_t* ev) const {
    const int32_t ca = pub.fork;
    const int32_t ph = p0.h + n;
    *pub_blocks = pub.h - ca;
    *priv_blocks = ph - ca;
    *diff_blocks = ph - pub.h;
    *ev = event & 1;
  }

  // Agent.apply (nakamoto_ssz.ml:232-260) + Simulator.handle_action share (:401-419).
  // Adopt: private := public (forks of the defender tips move to the new base); Match /
  // Override: release up to the public height (+1); Wait (and any out-of-range action,
  // rejected by the host) shares nothing.
  __host__ __device__ inline CPR_AI void apply(int32_t action) {
    const bool adopt = action == A_ADOPT;
    const bool relx = action == A_MATCH || action == A_OVERRIDE;
    const int32_t hp = pub.h;
    const bool fresh = (event & 2) != 0;  // pub is this window's defender block
    const bool onch = pub.fork == hp;                // pub lies on the private chain
    const int32_t bf = fresh ? b.h : (onch ? (b.fork < hp ? b.fork : hp) : b.fork);
    const int32_t df = fresh ? D.fork : (onch ? (D.fork < hp ? D.fork : hp) : D.h);
    const int32_t af = fresh ? A.fork : (onch ? (A.fork < hp ? A.fork : hp) : lca_da);
    const int32_t target = hp + (action == A_OVERRIDE ? 1 : 0);
    int32_t mf = target - p0.h;
    mf = mf < 0 ? 0 : (mf > n ? n : mf);
    const bool newrel = relx && mf > rel;
    rlo = newrel ? rel + 1 : rlo;
    rhi = newrel ? mf : rhi;
    rel = adopt ? 0 : (newrel ? mf : rel);
    pend = relx ? mf : -1;
    n_ba = adopt ? 0 : n;
    n = adopt ? 0 : n;
    b.fork = adopt ? bf : b.fork;
    D.fork = adopt ? df : D.fork;
    A.fork = adopt ? af : A.fork;
    BRef np = pub;  // value copy: the select below picks values, not field addresses
    np.fork = hp;
    sel(p0, adopt, np);
    pub.fork = adopt ? hp : pub.fork;
  }

  // deliveries of the window: the fresh defender block and the attacker's release reach
  // the defenders (simulator.ml:481-508 with update_head, nakamoto.ml:85-89)
  // AG: the abstract-gamma rule fixed at compile time (0 off, 1 on) or read from P (-1)
  // TT: 1 = ties resolved without the heap replay (tie_table_d2), for kernels that run only
  // d = 2 configurations; a tie that rule does not cover flags TIE_UNRESOLVED (the fused
  // kernel hands such an episode to the exact re-run). 0 = tie_replay.
  // 2 = deferred (d = 2 and dmax <= delta, the gym's gamma = .5 network): every release then
  // reaches the non-miner defender no later than the defender block, so the race's outcome
  // is decided, the release first, unless the two arrive at the same fp instant. The race is
  // taken as decided and noted (rw) for enqueue_race; verify_races checks the wave's list in
  // batches and flags the episode for an eager re-run when a tie decided otherwise.
  template <class St, int AG = -1, int TT = 0>
  __host__ __device__ inline CPR_AI void resolve(const NakParams& P, const St& S, const LaneMem& M) {
    const bool released = rhi >= rlo && P.arrive;
    const uint64_t all = all_mask(P.d);
    const bool dm = wminer != 0;
    const int32_t xh = p0.h + rhi;
    const int32_t hs = onA ? A.h : D.h;
    const int32_t lca_new = dm ? b.fork : D.fork;  // read before the race block splits this
    const bool newA = released && (dm ? xh >= b.h : xh > hs);
    uint64_t mask = all;
    const bool abstract_g = AG >= 0 ? AG != 0 : P.abstract_g != 0;
    if (released && dm && xh == b.h && abstract_g) {
      // flagged abstract-gamma mode: each defender, the miner included, mines on the
      // released block iff its coin falls below gamma (Eyal-Sirer'14's gamma)
      mask = 0ull;
      for (int32_t j = 1; j <= P.d; ++j)
        mask |= S.link((uint32_t)k, 0u, (uint32_t)j, 1.0) < P.gamma ? 1ull << (j - 1) : 0ull;
    } else if (TT == 2 && released && dm && xh == b.h) {
      mask = 1ull << (2 - wminer);  // j = 3 - wminer first reached by the release
      rw = (uint32_t)wminer | ((uint32_t)rlo << 2) | ((uint32_t)rhi << 14);
    } else if (released && dm && xh == b.h) {
      // race at every defender except the miner: first visible wins. One link draw per
      // (non-miner defender, released block); the defender index is per lane.
      const double tb = t + P.delta;
      mask = 0ull;
      bool tie = false;
      for (int32_t i = 0; i < P.d - 1; ++i) {
        const int32_t j = i + (i + 1 >= wminer ? 2 : 1);
        double v = -__builtin_inf();
        for (int32_t m = rlo; m <= rhi; ++m) {
          const double a = t + S.link((uint32_t)k, (uint32_t)(rhi - m), (uint32_t)j, P.dmax);
          v = a > v ? a : v;
        }
        mask |= v < tb ? 1ull << (j - 1) : 0ull;
        tie |= v == tb;
      }
      if (tie) {
        // same instant at some defender: the queue order decides
        status |= ST_TIE;
        if (TT) {
          if (P.d == 2 && rlo == rhi)
            mask = tie_table_d2(P, S, wminer, t, k);
          else
            status |= ST_TIE_UNRESOLVED;
        } else {
          bool ok = false;
          const uint64_t exact = tie_replay(P, S, M.replay, wminer, t, rlo, rhi, k, &ok);
          if (ok)
            mask = exact;
          else
            status |= ST_TIE_UNRESOLVED;
        }
      }
    }
    sel(A, newA, chain_ref(M, rhi));
    lca_da = newA ? lca_new : lca_da;
    onA = dm ? (newA ? mask : 0ull) : (newA ? all : onA);
    sel(D, dm, b);
    double bound = dm && P.d >= 2 ? t + P.delta : -__builtin_inf();
    if (released) {
      const double ub = t + (P.dmax - 0.0);
      bound = ub > bound ? ub : bound;
    }
    w_bound = bound;
    w_hasb = dm ? 1 : 0;
    wminer = 0;
  }

  // Ref.winner over [attacker preferred; defender tips 1..d] (engine.ml:195-206,
  // nakamoto.ml:43-48): first maximal height, attacker listed first
  __host__ __device__ inline CPR_AI BRef head(const NakParams& P, const LaneMem& M) const {
    BRef best = chain_ref(M, n_ba);
    const uint64_t all = all_mask(P.d);
    const uint64_t mb = wminer ? (1ull << (wminer - 1)) : 0ull;
    const uint64_t ma = onA & ~mb;
    const uint64_t md = all & ~onA & ~mb;
    // candidates in node order: the miner of b holds b, the first defender on A holds A,
    // the first on D holds D; the first maximal height wins (fold keeps earlier on ties)
    const int32_t ja = ma ? 1 + __builtin_ctzll(ma) : (1 << 30);
    const int32_t jd = md ? 1 + __builtin_ctzll(md) : (1 << 30);
    int32_t bh = wminer ? b.h : -1, bj = wminer ? wminer : (1 << 30);
    BRef cand = b;
    const bool ta = ma && (A.h > bh || (A.h == bh && ja < bj));
    sel(cand, ta, A);
    bh = ta ? A.h : bh;
    bj = ta ? ja : bj;
    const bool td = md && (D.h > bh || (D.h == bh && jd < bj));
    sel(cand, td, D);
    bh = td ? D.h : bh;
    sel(best, bh > best.h, cand);
    return best;
  }

  // Simulator.timestamp of a block = its mining time for these networks
  __host__ __device__ inline CPR_AI double time_of(const LaneMem&, const BRef& x) const { return x.tm; }

  // POL >= 0: the policy fixed at compile time (the fused kernel's specialisations), so
  // the policy switch and its table operands disappear from the activation loop
  template <int POL = -1>
  __host__ __device__ inline CPR_AI int32_t policy_action(const NakParams& P) const {
    int32_t h, a, dd, ev;
    observe(&h, &a, &dd, &ev);
    return nak_policy(POL >= 0 ? POL : P.policy, h, a, ev, P.table, P.table_dim);
  }
};

// TT = 2, after resolve: the lanes whose race was taken as decided append it to the wave's
// dense list (entry: window time, activation count, rw with the owner lane in bits 26..31),
// so that verify_races spreads the wave's races over all its lanes
// LZ = 2 (lazy clock): instead of the window time, its bound esum (t <= esum ln2 ev) and
// whether the clock is +inf
template <int LZ = 0>
__host__ __device__ inline CPR_AI uint4 race_entry(const NakLane& L, int32_t lane) {
  uint4 e;
  if constexpr (LZ == 2) {
    e.x = L.esum;
    e.y = (uint32_t)L.tinf;
  } else {
    const uint64_t tb = bitsd(L.t);
    e.x = (uint32_t)tb;
    e.y = (uint32_t)(tb >> 32);
  }
  e.z = (uint32_t)L.k;
  e.w = L.rw | ((uint32_t)lane << 26);
  return e;
}
template <int LZ = 0>
__host__ __device__ inline CPR_AI void enqueue_race(NakLane& L, const LaneMem& M) {
  const bool race = L.rw != 0u;
  const uint64_t bal = wave_ballot(race);
  if (race) M.rq[L.qn + lanes_below(bal)] = race_entry<LZ>(L, M.lane);
  L.qn += __builtin_popcountll(bal);
  L.rw = 0u;
}

// the wave's list must be verified before the next iteration could overflow it
__host__ __device__ inline CPR_AI bool races_due(const NakLane& L, const LaneMem& M) {
  return L.qn > M.rq_cap - M.wave;
}

// TT = 2: verifies the wave's deferred races, lane i taking entries i, i + 64, ... A race
// whose release does not strictly precede the defender block at the non-miner defender (a
// same-instant tie) was decided wrongly or by the queue order. A tie the closed-form rule
// (resolve<.., 1>) decides as assumed only marks the episode (ST_TIE); anything else flags
// it (ST_RACE_REDO): the kernel lists it, and a second pass runs it again with every race
// decided eagerly (tests/native/defer_vs_eager.cpp compares the two on the host).
// In three phases, each over the whole wave (the host tests emulate a wave phase by phase):
// publish the lane's episode; check entries lane, lane + wave, ...; settle the own flag
template <class St>
__host__ __device__ inline CPR_AI void races_publish(const St& S, const LaneMem& M) {
  M.rep[2 * M.lane] = S.e0;
  M.rep[2 * M.lane + 1] = S.e1;
}
// LZ = 2: the window time is not known, only a bound T >= t + delta (esum ev / 4096,
// widened by 1e-9 for the log's and the sum's rounding, plus delta). t + a and t + delta both round
// to the grid of spacing <= ulp(T), each within half of it, so a < delta - ulp(T) puts the
// release strictly first, as the eager check would find. Anything closer (~ulp(t) / delta,
// 1e-4 of races at the gym's delay; or a +inf clock) cannot be decided without t and flags
// the episode for the eager second pass, which decides it with t as the eager kernel does.
template <class St, int LZ = 0>
__host__ __device__ inline CPR_AI void races_check(const NakLane& L, const NakParams& P,
                                                  const St& S, const LaneMem& M) {
  // the entries are spread over the lanes that are here: in the last grid-stride round of
  // a launch some lanes of the wave have left the episode loop, and an entry assigned to
  // one of them would never be checked. (On the host a wave is emulated phase by phase
  // and every emulated lane takes part: lane / wave as given.)
  int32_t rank = M.lane, stride = M.wave;
#if defined(__HIP_DEVICE_COMPILE__)
  const uint64_t here = wave_ballot(true);
  rank = lanes_below(here);
  stride = __builtin_popcountll(here);
#endif
  for (int32_t i = rank; i < L.qn; i += stride) {
    const uint4 e = M.rq[i];
    const int32_t rlo = (int32_t)((e.w >> 2) & 0xfffu), rhi = (int32_t)((e.w >> 14) & 0xfffu);
    const uint32_t j = 3u - (e.w & 3u);
    const int32_t owner = (int32_t)(e.w >> 26);
    St so = S;  // the owner lane's episode
    so.e0 = M.rep[2 * owner];
    so.e1 = M.rep[2 * owner + 1];
    if constexpr (LZ == 2) {
      double a = -__builtin_inf();
      for (int32_t m = rlo; m <= rhi; ++m) {
        const double x = so.link(e.z, (uint32_t)(rhi - m), j, P.dmax);
        a = x > a ? x : a;
      }
      const double T = (double)e.x * (P.ev * (1.0 / 4096.0)) * (1.0 + 1e-9) + P.delta;
      const int32_t ex = (int32_t)((bitsd(T) >> 52) & 0x7ffu);  // T > 0, normal
      const double ulp = dbits((uint64_t)(ex > 52 ? ex - 52 : 1) << 52);
      if (e.y != 0u || !(a < P.delta - ulp)) flag_or(&M.rflag[owner], 2);
      continue;
    }
    const double t = dbits((uint64_t)e.x | ((uint64_t)e.y << 32));
    double v = -__builtin_inf();
    for (int32_t m = rlo; m <= rhi; ++m) {
      const double a = t + so.link(e.z, (uint32_t)(rhi - m), j, P.dmax);
      v = a > v ? a : v;
    }
    const double tb = t + P.delta;
    if (!(v < tb)) {
      // the release did not arrive first: a same-instant tie whose closed-form rule
      // (resolve<.., 1>) agrees with the assumed outcome only marks the episode (1);
      // anything else has it run again (2)
      const bool kept = v == tb && rlo == rhi &&
                        tie_table_d2(P, so, (int32_t)(e.w & 3u), t, (int32_t)e.z) != 0ull;
      flag_or(&M.rflag[owner], kept ? 1 : 2);
    }
  }
}
__host__ __device__ inline CPR_AI void races_settle(NakLane& L, const LaneMem& M) {
  const int32_t fl = M.rflag[M.lane];
  M.rflag[M.lane] = 0;
  L.qn = 0;
  L.status |= (fl & 1) ? ST_TIE : 0u;
  L.status |= (fl & 2) ? ST_RACE_REDO : 0u;
}
template <class St, int LZ = 0>
__host__ __device__ inline CPR_AI void verify_races(NakLane& L, const NakParams& P, const St& S,
                                                   const LaneMem& M) {
  races_publish(S, M);
  wave_lds_order();
  races_check<St, LZ>(L, P, S, M);
  wave_lds_order();
  races_settle(L, M);
}

// miner of activation index ka (for head_miner of the record)
template <class St>
__host__ __device__ inline CPR_AI int32_t miner_of(const NakParams& P, const St& S, int32_t ka) {
  if (ka == K_PRIVATE) return 0;
  if (ka < 0) return -1;
  return S.miner((uint32_t)ka, P.t_att, P.d);
}

}  // namespace cpr
