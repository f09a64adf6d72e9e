// Ethereum gym episodes on the gym's selfish-mining network, one activation window at a
// time: the fast lane of cpr_run_episodes for Ethereum.
//
// The exact per-lane event engine (ethereum_lane.h) pushes and pops every event of the
// reference's queue (simulator.ml:421-508): about 14 per activation with two defenders and
// 50 with eleven, each a walk of a skew heap in HBM. But on this network (network.ml:61-105:
// defender -> defender delay delta, defender -> attacker 0, attacker -> defender U(0, dmax))
// an activation's messages have all arrived before the next activation in all but ~1e-9 of
// windows, exactly as for Nakamoto (nakamoto_lane.h). At that point every defender holds
// the same set of blocks (all defender blocks and, when dmax is finite, every block the
// attacker has released), the attacker holds all of them, and the queue holds the next
// clock alone. So a window's outcome is a closed-form function of the block DAG:
//
//   activation   miner m, clock delay (keyed stream); Honest.puzzle_payload' (uncles from
//                the visible children of the tip's last six ancestors, ethereum.ml:234-277)
//                for defender m from its tip, or the agent's payload for the attacker;
//                append; the attacker's interaction (prepare, ethereum_ssz.ml:325-362)
//   action       Agent.apply (ethereum_ssz.ml:398-429), the release's closure shared
//                (simulator.ml:401-419)
//   deliveries   every defender ends on the first-visible block of maximal height among
//                its tip, the defender block b (t + delta) and the released top sh (the
//                latest arrival over sh's closure): update_head keeps strictly higher
//                blocks (ethereum.ml:279-283). Only a race of equal heights needs link draws.
//
// No event queue, no per-node visibility array: visibility at quiescence is a function of
// the block (miner, released). A same-instant race (fl(t + U_j) == fl(t + delta)) is
// decided by the queue's order: for a released chain the window is replayed through the
// skew heap exactly as the Nakamoto lane does (tie_replay, nakamoto_lane.h: the window's
// events are the same; uncles ride along in payloads only). Everything the closed form
// cannot vouch for — an activation inside the previous window's deliveries (OVERLAP), a
// tie on a release that is not a chain or exceeds the replay (TIE_UNRESOLVED), a candidate
// or frontier overflow (CAPACITY) — flags the episode, and the kernel re-runs it on the
// exact event engine. Parity: tests/native/ethwin_vs_oracle.cpp compares this lane with
// the oracle's event-driven ethereum.cpp step by step on the host; tests/test_gpu_eth.py with the oracle.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpr_stream.h"
#include "ethereum_lane.h"
#include "nakamoto_lane.h"

#pragma clang fp contract(off)

namespace cpr {
namespace ethw {

using eth::EthObs;
using eth::EthParams;
using eth::Payload;

// window-lane status bits the fused kernel hands to the exact event engine
constexpr uint32_t W_REDO = ST_OVERLAP | ST_TIE_UNRESOLVED | eth::EST_CAPACITY;

// 32 bytes: serials are < cap_b <= 2^15 (append stops the lane before the ring would wrap),
// so block references and heights fit 16 bits, and a 128-byte line holds four blocks (the
// lane's walks read neighbouring serials: chains, children lists). The append time, read
// only for the head's chain time at the end, lives in a separate array (WinMem.tm)
struct WBlock {
  int16_t p[3];    // parent, uncles (-1: none)
  int16_t child;   // newest block whose first parent this is (-1: none)
  int16_t sib;     // next older block with the same first parent (-1: none)
  int16_t jump;    // skew-binary jump ancestor (O(log depth) ancestor queries)
  int16_t plain;   // this block and its first-parent ancestors below it that have one
                   // parent each, counted from here (0: this one has uncles or is genesis):
                   // the frontier walk skips such runs (q_advance)
  int16_t height;
  int8_t miner;    // -1 genesis, 0 attacker, 1..d defenders
  uint8_t np;      // parents
  uint8_t rel;     // attacker block shared (V_REL in the attacker's view)
  uint8_t _pad;
  int32_t work;
  int32_t rew_att, rew_def;  // cumulative rewards of the first-parent chain, units of 1/32
};
static_assert(sizeof(WBlock) == 32, "WBlock layout");

constexpr int32_t NCAND = eth::NCAND, NQ = eth::NQ, NSTACK = eth::NSTACK;
// scratch ints: candidates, keys, two frontiers, share stack, closure (share order)
constexpr int32_t S_CAND = 0, S_KEY = 32, S_QA = 64, S_QB = 96, S_STACK = 128, S_CLOS = 192;
constexpr int32_t S_INTS = 192 + NSTACK;

struct WinMem {
  WBlock* blk;     // [cap_b]
  double* tm;      // [cap_b] append times (Simulator.timestamp)
  int32_t* tips;   // [64]: defender j's preferred block at tips[j] (Honest.state)
  int32_t* scr;    // [S_INTS]
  ReplayMem replay;  // tie_replay scratch
};

__host__ __device__ inline int64_t win_lane_bytes(int32_t cap_b) {
  return eth::align128((int64_t)cap_b * (int64_t)sizeof(WBlock)) +
         eth::align128((int64_t)cap_b * 8) + eth::align128(65 * 4) +
         eth::align128(S_INTS * 4) + eth::align128(REPLAY_BYTES);
}
__host__ __device__ inline WinMem win_mem_at(uint8_t* base, int32_t cap_b) {
  WinMem M;
  int64_t o = 0;
  M.blk = (WBlock*)(base + o);
  o += eth::align128((int64_t)cap_b * (int64_t)sizeof(WBlock));
  M.tm = (double*)(base + o);
  o += eth::align128((int64_t)cap_b * 8);
  M.tips = (int32_t*)(base + o);
  o += eth::align128(65 * 4);
  M.scr = (int32_t*)(base + o);
  o += eth::align128(S_INTS * 4);
  M.replay = ReplayMem::at(base + o);
  return M;
}

// attacker messages reach the defenders (gamma > 0: dmax finite; gamma = 0: never)
__host__ __device__ inline bool arrives(const EthParams& P) { return P.dmax < __builtin_inf(); }

// the window lane runs these configurations (else the event engine does): gym episodes on
// the selfish-mining network, Ethereum proper (not the Nakamoto mode)
__host__ __device__ inline bool win_supported(const EthParams& P) {
  return P.net == 0 && P.mode == 0 && !P.nak && P.d >= 2 && P.d <= 63;
}

struct WinLane {
  double now;
  int32_t c_act, newest;
  uint32_t status;
  int32_t dead;
  int64_t steps;
  // the current window: its defender block (-1: the attacker mined) and miner, the
  // release shared at its interaction (-1: none) and that release's closure size
  int32_t wb, wi, sh, nclos;
  int32_t chain;  // the closure is a first-parent chain (tie_replay applies)
  // ethereum_ssz agent (BetweenActions + Observable)
  int32_t pub, priv, pending, own, foreign;
  int32_t o_pub, o_priv, o_common, o_event;
  // the last common ancestor computed: common_ancestor(ca_a, ca_b) = ca_c (-1: none)
  int32_t ca_a, ca_b, ca_c;

  __host__ __device__ inline void fail(int32_t why) {
    status |= eth::EST_CAPACITY;
    if (!dead) dead = why;
  }
  // serials index the ring directly: append stops the lane before it would wrap
  __host__ __device__ inline WBlock& B(const EthParams& P, const WinMem& M, int32_t s) {
    if ((uint32_t)s > (uint32_t)newest) fail(1);
    return M.blk[s & (P.cap_b - 1)];
  }
  // Simulator.timestamp of block s (its append time)
  __host__ __device__ inline double time_of(const EthParams& P, const WinMem& M, int32_t s) {
    B(P, M, s);  // range check
    return M.tm[s & (P.cap_b - 1)];
  }
  // visibility at quiescence (every message of earlier windows delivered)
  __host__ __device__ static inline bool def_visible(const EthParams& P, const WBlock& b) {
    return b.miner != 0 || (b.rel && arrives(P));
  }

  // Honest.puzzle_payload' (ethereum.ml:234-277) in node `view`'s view: the candidates are
  // the visible children (via the first parent) of the tip's last six ancestors, not in the
  // chain, in generation order then newest first — the children lists' order — ordered by
  // (not own, height) with OCaml's heap sort (Compare.at_most_first, ethereum.ml:269)
  __host__ __device__ inline Payload payload(const EthParams& P, const WinMem& M, int32_t view,
                                             int32_t tip, int32_t filter, int32_t f_own,
                                             int32_t f_foreign) {
    CPR_COST(eth::CC_PAYLOAD);
    int32_t* cand = M.scr + S_CAND;
    int32_t* key = M.scr + S_KEY;
    int32_t ic[19];  // in-chain set: the tip and the parents of tip .. gen 5
    int32_t nua[6];
    int32_t ng = 0, nic = 0;
    ic[nic++] = tip;
    {
      int32_t b = tip;
      for (int32_t gen = 0; gen < 6; ++gen) {
        nua[gen] = -2;
        if (b < 0) continue;
        const WBlock& x = B(P, M, b);
        if (x.np == 0) {
          b = -1;
          continue;
        }
        nua[gen] = x.p[0];
        ng = gen + 1;
        for (int32_t i = 0; i < x.np; ++i) ic[nic++] = x.p[i];
        b = x.p[0];
      }
    }
    int32_t nc = 0;
    for (int32_t g = 0; g < ng && !dead; ++g) {
      for (int32_t s = B(P, M, nua[g]).child; s >= 0 && !dead; s = B(P, M, s).sib) {
        CPR_COST(eth::CC_SCAN);
        const WBlock& c = B(P, M, s);
        bool mine, keep;
        if (view == 0) {  // the attacker sees every block
          mine = c.miner == 0;
          keep = filter == eth::F_MINING ? ((f_own && mine) || (f_foreign && !mine))
                                          : (filter == eth::F_PUBLIC ? (!mine || c.rel) : true);
        } else {
          if (!def_visible(P, c)) continue;
          mine = c.miner == view;
          keep = true;
        }
        if (!keep) continue;
        bool inchain = false;
        for (int32_t i = 0; i < nic; ++i) inchain |= ic[i] == s;
        if (inchain) continue;
        if (nc >= NCAND) {
          fail(3);
          break;
        }
        cand[nc] = s;
        key[nc] = ((mine ? 0 : 1) << 27) | (c.height & 0x7ffffff);
        ++nc;
      }
    }
    eth::EthLane::ocaml_heap_sort(cand, key, nc);
    Payload d;
    const WBlock& t = B(P, M, tip);
    const int32_t nu = nc < 2 ? nc : 2;
    d.p[0] = tip;
    d.p[1] = nu > 0 ? cand[0] : -1;
    d.p[2] = nu > 1 ? cand[1] : -1;
    d.np = 1 + nu;
    d.height = t.height + 1;
    d.work = t.work + 1 + nu;
    return d;
  }

  // skew-binary jump pointers (Myers 1983) over first parents: a block's jump is its
  // parent's jump's jump when the parent's two jumps span equal height gaps, else its
  // parent; jumps depend on the height alone, so ancestor-at-height and first-parent LCA
  // queries take O(log depth) loads
  __host__ __device__ inline int32_t jump_for(const EthParams& P, const WinMem& M,
                                              int32_t parent) {
    const WBlock& pb = B(P, M, parent);
    const WBlock& jb = B(P, M, pb.jump);
    const int32_t jjh = B(P, M, jb.jump).height;
    return (pb.height - jb.height == jb.height - jjh) ? jb.jump : parent;
  }
  // first-parent ancestor of x at height h <= height(x)
  __host__ __device__ inline int32_t ancestor_at(const EthParams& P, const WinMem& M, int32_t x,
                                                 int32_t h) {
    while (!dead) {
      const WBlock& b = B(P, M, x);
      if (b.height <= h || b.np == 0) return x;
      x = B(P, M, b.jump).height >= h ? b.jump : b.p[0];
    }
    return x;
  }

  // first-parent LCA of x and y: level the heights, then descend by jump pointers while
  // the two jumps differ (jumps depend on the height alone, so they stay level)
  __host__ __device__ inline int32_t fp_lca(const EthParams& P, const WinMem& M, int32_t x,
                                            int32_t y) {
    const int32_t hx = B(P, M, x).height, hy = B(P, M, y).height;
    if (hx > hy) x = ancestor_at(P, M, x, hy);
    if (hy > hx) y = ancestor_at(P, M, y, hx);
    while (x != y && !dead) {
      const WBlock& a = B(P, M, x);
      const WBlock& b = B(P, M, y);
      if (a.np == 0 || b.np == 0) break;
      if (a.jump != b.jump) {
        x = a.jump;
        y = b.jump;
      } else {
        x = a.p[0];
        y = b.p[0];
      }
    }
    return x;
  }

  // simulator.ml:122-136, 377-399 (set_rewards, ethereum.ml:173-197: Constant = whitepaper)
  __host__ __device__ inline int32_t append(const EthParams& P, const WinMem& M, int32_t node,
                                            const Payload& d) {
    WBlock& pb = B(P, M, d.p[0]);
    int32_t ra = pb.rew_att, rd = pb.rew_def;
    const int32_t nu = d.np - 1;
    if (node == 0)
      ra += 32 + nu;
    else
      rd += 32 + nu;
    for (int32_t i = 1; i < d.np; ++i) {
      const WBlock& u = B(P, M, d.p[i]);
      const int32_t amt = P.scheme == 0 ? 30 : 4 * (8 - (d.height - u.height));
      if (u.miner == 0)
        ra += amt;
      else if (u.miner > 0)
        rd += amt;
    }
    if (newest + 1 >= P.cap_b) {  // the ring would wrap onto live blocks
      fail(1);
      return 0;
    }
    const int32_t jmp = jump_for(P, M, d.p[0]);
    const int32_t s = ++newest;
    WBlock& b = M.blk[s];
    b.p[0] = (int16_t)d.p[0];
    b.p[1] = (int16_t)(d.np > 1 ? d.p[1] : -1);
    b.p[2] = (int16_t)(d.np > 2 ? d.p[2] : -1);
    b.np = (uint8_t)d.np;
    b.height = (int16_t)d.height;
    b.work = d.work;
    b.miner = (int8_t)node;
    b.rel = 0;
    b.rew_att = ra;
    b.rew_def = rd;
    b.child = -1;
    b.sib = pb.child;  // children lists newest first (dag.ml:32)
    b.jump = (int16_t)jmp;
    b.plain = (int16_t)(d.np == 1 ? pb.plain + 1 : 0);
    pb.child = (int16_t)s;
    M.tm[s] = now;
    return s;
  }

  // Dagtools.common_ancestor (dagtools.ml:102-121) in the attacker's view, which holds
  // every block: ancestors by descending (height, serial) over all parent edges
  __host__ __device__ inline void q_insert(int32_t* q, int32_t* nq, int32_t s, int32_t h) {
    const uint64_t kk = eth::EthLane::ca_key(h, s);
    CPR_COST(eth::CC_MDV);  // (window lane: frontier insertions)
    for (int32_t j = 0; j < *nq; ++j)
      if (q[2 * j + 1] == s) return;
    if (*nq >= NQ / 2) {
      fail(4);
      return;
    }
    int32_t i = *nq;
    while (i > 0 && eth::EthLane::ca_key(q[2 * (i - 1)], q[2 * (i - 1) + 1]) < kk) {
      q[2 * i] = q[2 * (i - 1)];
      q[2 * i + 1] = q[2 * (i - 1) + 1];
      --i;
    }
    q[2 * i] = h;
    q[2 * i + 1] = s;
    ++*nq;
  }
  __host__ __device__ inline int32_t q_next(const EthParams& P, const WinMem& M, int32_t* q,
                                            int32_t* nq) {
    if (*nq == 0) return -1;
    CPR_COST(eth::CC_CA);
    const int32_t s = q[1];
    for (int32_t j = 1; j < *nq; ++j) {
      q[2 * (j - 1)] = q[2 * j];
      q[2 * (j - 1) + 1] = q[2 * j + 1];
    }
    --*nq;
    const WBlock& b = B(P, M, s);
    for (int32_t i = 0; i < b.np; ++i) q_insert(q, nq, b.p[i], B(P, M, b.p[i]).height);
    return s;
  }
  // q_next for the side whose popped block is above the other side's `y` (the walk keeps
  // advancing this side while its popped keys stay above key(y)). When the frontier's top e
  // heads a run of one-parent blocks (WBlock.plain), popping a run block pushes just its
  // first parent, so the walk pops e, its parent, ... for as long as (A) the block popped
  // before stays above key(y) and (B) the next one stays above the frontier's second key
  // k2 (else that one is the top). One jump-pointer descent to the lowest such block
  // replaces those pops and leaves the frontier exactly as they would: that block popped,
  // its parent queued, the rest unchanged. Long private forks otherwise walked the whole
  // fork a block at a time every activation (selfish_release at gamma = 0: ~13 pops per
  // activation, bench configs[2]'s slowest point by 3x)
  __host__ __device__ inline int32_t q_advance(const EthParams& P, const WinMem& M, int32_t* q,
                                               int32_t* nq, int32_t y) {
    if (*nq >= 1) {
      const int32_t e = q[1];
      const WBlock& be = B(P, M, e);
      if (be.plain >= 2) {
        const int32_t he = be.height;
        int32_t lo = he - be.plain + 1;  // the run's last block
        // (A) the block above the landing one is above y: height >= hy, or hy - 1 when the
        // run's block at hy is above y by serial
        const int32_t hy = B(P, M, y).height;
        if (hy > lo) {
          int32_t ha = hy;
          if (hy <= he && ancestor_at(P, M, e, hy) > y) ha = hy - 1;
          lo = ha > lo ? ha : lo;
        }
        // (B) the landing block is above the frontier's second element
        if (*nq >= 2) {
          const int32_t h2 = q[2], s2 = q[3];
          if (h2 >= lo) {
            int32_t hb = h2 + 1;
            if (h2 <= he && ancestor_at(P, M, e, h2) > s2) hb = h2;
            lo = hb > lo ? hb : lo;
          }
        }
        if (lo < he && !dead) {
          CPR_COST(eth::CC_CA);
          const int32_t z = ancestor_at(P, M, e, lo);
          for (int32_t j = 1; j < *nq; ++j) {  // e leaves the frontier
            q[2 * (j - 1)] = q[2 * j];
            q[2 * (j - 1) + 1] = q[2 * j + 1];
          }
          --*nq;
          const int32_t pz = B(P, M, z).p[0];
          q_insert(q, nq, pz, B(P, M, pz).height);
          return z;
        }
      }
    }
    return q_next(P, M, q, nq);
  }
  __host__ __device__ inline int32_t common_ancestor(const EthParams& P, const WinMem& M,
                                                     int32_t a, int32_t b) {
    if (a == b) return a;
    int32_t* qa = M.scr + S_QA;
    int32_t* qb = M.scr + S_QB;
    int32_t na = 0, nb = 0;
    q_insert(qa, &na, a, B(P, M, a).height);
    q_insert(qb, &nb, b, B(P, M, b).height);
    int32_t x = q_next(P, M, qa, &na);
    int32_t y = q_next(P, M, qb, &nb);
    while (x >= 0 && y >= 0 && !dead) {
      if (x == y) return x;
      // both sides on runs of one-parent blocks (each frontier is just the popped block's
      // parent): the walk pops the two first-parent chains alternately, highest key first,
      // and its first common block is their first-parent LCA F. If F lies within both runs
      // that is the answer; otherwise the walk passes both sides at the height L where the
      // first run ends, which one jump-pointer descent per side reaches (q_advance handles a
      // side whose run lies above the other side's block)
      if (na == 1 && nb == 1) {
        const WBlock& bx = B(P, M, x);
        const WBlock& by = B(P, M, y);
        if (bx.plain >= 2 && by.plain >= 2 && qa[1] == bx.p[0] && qb[1] == by.p[0]) {
          const int32_t lx = bx.height - bx.plain + 1, ly = by.height - by.plain + 1;
          const int32_t L = lx > ly ? lx : ly;
          const int32_t f = fp_lca(P, M, x, y);
          if (B(P, M, f).height >= L) return f;
          const int32_t hmin = bx.height < by.height ? bx.height : by.height;
          if (L < hmin && !dead) {
            CPR_COST(eth::CC_CA);
            x = ancestor_at(P, M, x, L);
            y = ancestor_at(P, M, y, L);
            na = nb = 0;
            const int32_t px = B(P, M, x).p[0], py = B(P, M, y).p[0];
            q_insert(qa, &na, px, B(P, M, px).height);
            q_insert(qb, &nb, py, B(P, M, py).height);
            continue;
          }
        }
      }
      const uint64_t kx = eth::EthLane::ca_key(B(P, M, x).height, x);
      const uint64_t ky = eth::EthLane::ca_key(B(P, M, y).height, y);
      if (kx > ky)
        x = q_advance(P, M, qa, &na, y);
      else
        y = q_advance(P, M, qb, &nb, x);
    }
    fail(4);
    return 0;
  }

  // Every uncle of a block c is a child (by first parent) of one of the first-parent
  // ancestors of c's parent (Honest.puzzle_payload'), so all-edge ancestors of a block x
  // are its first-parent chain plus side blocks whose first parent lies on that chain. Two
  // blocks' common ancestors above their first-parent fork F can then only be children of
  // F or siblings of F: the common ancestor has height h(F) or h(F) + 1. So when one side
  // is a block just appended on the other side's previous argument (first parent), the
  // answer can change only through blocks of its uncle closure (uncles, their uncles, ...)
  // at most one level above the previous answer; if all of them are higher, it is the
  // previous answer. That is the common case in long private forks, where the frontier walk
  // below costs the whole fork per activation. Anything else walks.
  __host__ __device__ inline bool uncles_above(const EthParams& P, const WinMem& M, int32_t x,
                                               int32_t hlim) {
    int32_t st[8];
    int32_t sp = 0;
    st[sp++] = x;
    while (sp > 0) {
      const WBlock& b = B(P, M, st[--sp]);
      for (int32_t i = 1; i < b.np; ++i) {
        if (B(P, M, b.p[i]).height <= hlim || sp >= 8) return false;
        st[sp++] = b.p[i];
      }
    }
    return true;
  }
  __host__ __device__ inline int32_t common_ancestor_cached(const EthParams& P, const WinMem& M,
                                                            int32_t a, int32_t b) {
    if (a == ca_a && b == ca_b) return ca_c;
    if (ca_c >= 0 && a != b) {
      const int32_t hl = B(P, M, ca_c).height + 1;
      if (a == ca_a && b == newest && B(P, M, b).p[0] == ca_b && uncles_above(P, M, b, hl)) {
        ca_b = b;
        return ca_c;
      }
      if (b == ca_b && a == newest && B(P, M, a).p[0] == ca_a && uncles_above(P, M, a, hl)) {
        ca_a = a;
        return ca_c;
      }
    }
    // one argument a first-parent ancestor of the other (the attacker's public model on
    // its own released chain, ethereum_ssz.ml:325-362): every ancestor of the lower one is
    // an ancestor of both and it is the highest of them, so it is the answer of the walk.
    // Not cached: the cached pair is the walk's, which the next activation's incremental
    // rule above extends (selfish_release at gamma = 0 alternates the two cases; caching
    // this one cost it the walk over the whole fork at every other activation)
    if (a != b) {
      const bool al = B(P, M, a).height <= B(P, M, b).height;
      const int32_t lo = al ? a : b, hi = al ? b : a;
      if (ancestor_at(P, M, hi, B(P, M, lo).height) == lo) return lo;
    }
    const int32_t c = common_ancestor(P, M, a, b);
    ca_a = a;
    ca_b = b;
    ca_c = c;
    return c;
  }

  // ---------------------------------------------------------------- agent
  __host__ __device__ inline int32_t update_head(const EthParams& P, const WinMem& M,
                                                 int32_t old, int32_t cand) {
    return B(P, M, cand).height > B(P, M, old).height ? cand : old;
  }
  // ethereum_ssz.ml:325-362
  __host__ __device__ inline void prepare(const EthParams& P, const WinMem& M, uint32_t kind,
                                          int32_t x) {
    int32_t p = pub;
    if (pending >= 0) p = update_head(P, M, p, pending);
    int32_t q = priv;
    if (kind == eth::KD_NET) {
      p = update_head(P, M, p, x);
      o_event = 1;
    } else {
      q = x;
      o_event = 0;
    }
    o_pub = p;
    o_priv = q;
    o_common = common_ancestor_cached(P, M, p, q);
  }
  // ethereum_ssz.ml:364-396; orphans only when asked
  __host__ __device__ inline EthObs observe(const EthParams& P, const WinMem& M, bool orphans) {
    const WBlock& c = B(P, M, o_common);
    const WBlock& pr = B(P, M, o_priv);
    const WBlock& pu = B(P, M, o_pub);
    EthObs o;
    o.public_height = pu.height - c.height;
    o.public_work = pu.work - c.work;
    o.private_height = pr.height - c.height;
    o.private_work = pr.work - c.work;
    o.diff_height = o.private_height - o.public_height;
    o.diff_work = o.private_work - o.public_work;
    o.event = o_event;
    o.public_orphans = o.private_orphans_inclusive = o.private_orphans_exclusive = 0;
    if (orphans) {
      o.public_orphans = payload(P, M, 0, o_pub, eth::F_PUBLIC, 0, 0).np - 1;
      o.private_orphans_inclusive = payload(P, M, 0, o_priv, eth::F_MINING, 1, 1).np - 1;
      o.private_orphans_exclusive = payload(P, M, 0, o_priv, eth::F_MINING, 1, 0).np - 1;
    }
    return o;
  }
  // ethereum_ssz.ml:398-429; returns the block to share (-1: none)
  __host__ __device__ inline int32_t apply(const EthParams& P, const WinMem& M, int32_t index) {
    const int32_t action = index >> 2;
    // the private chain's block at height target (its tip if lower): jump pointers
    auto release_upto = [&](int32_t target) {
      CPR_COST(eth::CC_SORT);  // (window lane: release walks)
      return ancestor_at(P, M, o_priv, target);
    };
    int32_t s = -1, np = o_priv;
    switch (action) {
      case eth::A_ADOPT_RELEASE:
        s = o_priv;
        np = o_pub;
        break;
      case eth::A_ADOPT_DISCARD: np = o_pub; break;
      case eth::A_MATCH: s = release_upto(B(P, M, o_pub).height); break;
      case eth::A_OVERRIDE: s = release_upto(B(P, M, o_pub).height + 1); break;
      case eth::A_RELEASE1: s = release_upto(B(P, M, o_common).height + 1); break;
      default: break;
    }
    pub = o_pub;
    priv = np;
    pending = s;
    own = (index >> 1) & 1;
    foreign = index & 1;
    return s;
  }

  // Simulator.handle_action's share (simulator.ml:401-419): the withheld closure of s0 in
  // the reference's recursive order (parents in order), each with its keyed link
  // coordinates (activation count, position). The closure is recorded in share order; it
  // is a chain when each entry's successor is its first parent.
  __host__ __device__ inline void share(const EthParams& P, const WinMem& M, int32_t s0) {
    int32_t* st = M.scr + S_STACK;
    int32_t* clos = M.scr + S_CLOS;
    int32_t sp = 0, off = 0;
    st[sp++] = s0;
    while (sp > 0 && !dead) {
      const int32_t s = st[--sp];
      CPR_COST(eth::CC_SHARE);
      WBlock& b = B(P, M, s);
      if (b.miner != 0 || b.rel) continue;  // received / released: nothing to share
      b.rel = 1;  // its link delays are keyed (c_act, off): off = position in clos
      clos[off++] = s;
      if (sp + b.np > NSTACK) {
        fail(5);
        return;
      }
      for (int32_t i = b.np - 1; i >= 0; --i) st[sp++] = b.p[i];
    }
    nclos = off;
    chain = 1;
    for (int32_t m = 0; m + 1 < off; ++m) chain &= B(P, M, clos[m]).p[0] == clos[m + 1] ? 1 : 0;
  }

  // ---------------------------------------------------------------- the window
  // the visibility time at defender j of the released top: the latest arrival over its
  // closure (a block is visible once its parents are, simulator.ml:424-450); the closure
  // was shared at activation count c_act, position m in share order (keyed link delays)
  template <class St>
  __host__ __device__ inline double release_visible(const EthParams& P, const St& S,
                                                    const WinMem& M, int32_t j) const {
    double v = -__builtin_inf();
    for (int32_t m = 0; m < nclos; ++m) {
      const double a = now + S.link((uint32_t)c_act, (uint32_t)m, (uint32_t)j, P.dmax);
      v = a > v ? a : v;
    }
    return v;
  }

  // the window's deliveries (simulator.ml:481-508, Honest.handler ethereum.ml:284-297):
  // every defender ends on the first-visible block of maximal height among its tip, the
  // defender block b (at now + delta, all but its miner) and the released top sh
  template <class St>
  __host__ __device__ inline void deliver(const EthParams& P, const St& S, const WinMem& M) {
    const bool rel = sh >= 0 && arrives(P);
    const int32_t hs = rel ? B(P, M, sh).height : -1;
    const int32_t hb = wb >= 0 ? B(P, M, wb).height : -1;
    const double tb = now + P.delta;
    uint64_t tie_mask = 0ull;  // defenders whose race tied
    bool tied = false;
    for (int32_t j = 1; j <= P.d; ++j) {
      const int32_t tj = M.tips[j];
      const int32_t ht = B(P, M, tj).height;
      int32_t best = tj, hbest = ht;
      if (wb >= 0 && j != wi && hb > hbest) {
        best = wb;
        hbest = hb;
      }
      if (rel && hs > hbest) {
        best = sh;
      } else if (rel && hs == hbest && best == wb && j != wi) {
        // equal heights at a non-miner defender: first visible wins
        const double v = release_visible(P, S, M, j);
        if (v < tb) best = sh;
        if (v == tb) {
          tied = true;
          tie_mask |= 1ull << (j - 1);
        }
      }
      M.tips[j] = best;
    }
    if (tied) {
      // same instant at some defender: the skew heap's order decides (tie_replay replays
      // the window's events, nakamoto_lane.h)
      status |= ST_TIE;
      bool ok = false;
      uint64_t on_top = 0ull;
      if (chain && nclos <= RMAX) {
        NakParams NP{};
        NP.d = P.d;
        NP.delta = P.delta;
        NP.dmax = P.dmax;
        on_top = tie_replay(NP, S, M.replay, wi, now, 1, nclos, c_act, &ok);
      }
      if (!ok) {
        status |= ST_TIE_UNRESOLVED;
      } else {
        for (int32_t j = 1; j <= P.d; ++j)
          if ((tie_mask >> (j - 1)) & 1ull) M.tips[j] = ((on_top >> (j - 1)) & 1ull) ? sh : wb;
      }
    }
  }

  // the next activation (simulator.ml:465-480 + engine.ml:108-121): clock, miner, draft
  // (Honest.puzzle_payload' or the agent's), append, the attacker's interaction
  template <class St>
  __host__ __device__ inline void activate(const EthParams& P, const St& S, const WinMem& M) {
    int32_t m;
    const double tn = now + S.act((uint32_t)c_act, P.t_att, P.d, P.ev, &m);
    // an activation inside the previous window's deliveries: the closed form does not hold
    double bound = now;  // a zero delay ties the window's own events
    if (wb >= 0) bound = now + P.delta > bound ? now + P.delta : bound;
    if (sh >= 0 && arrives(P)) {
      const double ub = now + (P.dmax - 0.0);
      bound = ub > bound ? ub : bound;
    }
    if (tn <= bound) {
      double last = now;
      if (wb >= 0) last = now + P.delta;
      if (sh >= 0 && arrives(P))
        for (int32_t j = 1; j <= P.d; ++j) {
          const double v = release_visible(P, S, M, j);
          last = v > last ? v : last;
        }
      if (tn <= last) status |= ST_OVERLAP;
    }
    now = tn;
    ++c_act;
    sh = -1;
    nclos = 0;
    uint32_t kind;
    int32_t x;
    if (m == 0) {
      const Payload d = payload(P, M, 0, priv, eth::F_MINING, own, foreign);
      x = append(P, M, 0, d);
      wb = -1;
      wi = 0;
      kind = eth::KD_POW;
    } else {
      const Payload d = payload(P, M, m, M.tips[m], eth::F_ALL, 0, 0);
      x = append(P, M, m, d);
      M.tips[m] = x;
      wb = x;
      wi = m;
      kind = eth::KD_NET;
    }
    prepare(P, M, kind, x);
  }

  // engine.ml:122-170
  template <class St>
  __host__ __device__ inline void gym_reset(const EthParams& P, const St& S, const WinMem& M) {
    now = 0.0;
    c_act = 0;
    newest = 0;
    status = 0u;
    dead = 0;
    steps = 0;
    wb = sh = -1;
    wi = 0;
    nclos = 0;
    chain = 1;
    ca_a = ca_b = ca_c = -1;
    WBlock& r = M.blk[0];
    r.p[0] = r.p[1] = r.p[2] = -1;
    r.np = 0;
    r.height = 0;
    r.work = 0;
    r.miner = -1;
    r.rel = 0;
    r.rew_att = r.rew_def = 0;
    r.child = r.sib = -1;
    r.jump = 0;
    r.plain = 0;
    M.tm[0] = 0.0;
    for (int32_t j = 0; j <= P.d; ++j) M.tips[j] = 0;
    pub = priv = 0;
    pending = -1;
    own = foreign = 1;
    activate(P, S, M);
  }

  // winner over [attacker preference; defenders' tips] (ethereum.ml:159-162)
  __host__ __device__ inline int32_t head(const EthParams& P, const WinMem& M, int32_t att) {
    int32_t h = att;
    int32_t hh = B(P, M, att).height;
    for (int32_t j = 1; j <= P.d; ++j) {
      const int32_t t = M.tips[j];
      const int32_t th = B(P, M, t).height;
      if (th > hh) {
        h = t;
        hh = th;
      }
    }
    return h;
  }

  // engine.ml:176-249: apply, the window's deliveries, the next activation; the head
  template <class St>
  __host__ __device__ inline int32_t gym_step(const EthParams& P, const St& S, const WinMem& M,
                                              int32_t action, bool* done) {
    sh = apply(P, M, action);
    if (sh >= 0) share(P, M, sh);
    ++steps;
    const int32_t att = priv;
    deliver(P, S, M);
    activate(P, S, M);
    const int32_t hd = head(P, M, att);
    const double progress = (double)B(P, M, hd).work;
    *done = dead || !(steps < P.max_steps && progress < P.max_progress && now < P.max_time);
    return hd;
  }
};

}  // namespace ethw
}  // namespace cpr
