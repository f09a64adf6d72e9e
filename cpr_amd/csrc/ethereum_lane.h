// Ethereum (Byzantium + Constant/Discount rewards) with the ethereum_ssz attack space:
// one episode per lane, as an exact per-lane discrete-event engine.
//
// Why an event engine here (and closed-form windows for Nakamoto): Ethereum's fork choice
// reads far more of the DAG than heights — uncle candidates are the visible children of
// the last six ancestors of each node's tip (ethereum.ml:234-277), the attacker's common
// ancestor walks uncle edges (dagtools.ml:102-121) and its observation runs three dry-run
// uncle selections (ethereum_ssz.ml:364-396). Replaying the reference's event semantics
// per lane keeps every one of those reads exact, including same-instant ties, whose order
// the skew heap decides (orderedQueue.ml:17-47).
//
// Per-lane memory (one contiguous region per resident lane):
//   blocks  [cap_b] x 64 B   ring indexed by serial & (cap_b-1); a stale slot (serial
//                            mismatch) marks the episode CPR_ST_CAPACITY
//   vis     [cap_b][n] u8    per node: kind (invisible/received/released/withheld) + got bit
//   heap    [cap_e] x 24 B   skew-heap nodes of the event queue (time, event, block)
//   tips    [n] i32          defenders' preferred blocks (Honest.state)
//   scratch 192 i32          candidate lists, ancestor frontiers, share stack
//
// Reference map: simulator.ml:122-543 (engine), ethereum.ml:89-297 (referee, honest node),
// ethereum_ssz.ml:279-521 (agent, policies), engine.ml:97-249 (gym step), network.ml
// selfish_mining / two_agents (links), distributions.ml (re-specified keyed stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpr_stream.h"
#include "nakamoto_lane.h"

#pragma clang fp contract(off)

namespace cpr {
namespace eth {

constexpr uint32_t EST_CAPACITY = 32u;  // CPR_ST_CAPACITY

enum : uint32_t { EV_CLOCK = 0, EV_DAG = 1, EV_TX = 2, EV_RX = 3, EV_ON = 4, EV_MV = 5, EV_MDV = 6 };
enum : uint32_t { KD_POW = 1, KD_NET = 2 };
enum : uint8_t { V_INV = 0, V_RECV = 1, V_REL = 2, V_WH = 3, V_KIND = 3, V_GOT = 4 };

__host__ __device__ inline uint32_t mkev(uint32_t ty, uint32_t node, uint32_t kind) {
  return ty | (kind << 3) | (node << 5);
}

struct EBlock {
  int32_t serial;
  int32_t p[3];  // parent serials; p[0] = parent, p[1..] = uncles (Nakamoto mode, no
                 // uncles: p[1] = newest child, p[2] = next older sibling)
  int32_t np;
  int32_t height, work;
  int32_t miner;             // -1 = genesis
  int32_t rew_att, rew_def;  // cumulative rewards of the first-parent chain, units of 1/32
  int32_t share_k, share_off;
  double time;  // Simulator.timestamp = append time (the miner sees it first)
  int32_t jump;  // Nakamoto mode: skew-binary jump ancestor (O(log depth) ancestor walks)
  int32_t _pad;
};
static_assert(sizeof(EBlock) == 64, "EBlock layout");

// host studies of the queue's operation sequence (tools/heap_study.cpp) define this
#ifndef CPR_HEAP_HOOK
#define CPR_HEAP_HOOK(op, t)
#endif
// host cost studies (tools/eth_cost_study.cpp) count work items by id (CC_* below)
#ifndef CPR_COST
#define CPR_COST(id)
#endif
enum : int32_t { CC_PUSH = 0, CC_POP = 1, CC_PAYLOAD = 2, CC_SCAN = 3, CC_CA = 4, CC_MDV = 5,
                 CC_EVENT = 6 /* + event type, 7 types */, CC_SHARE = 13, CC_SORT = 14,
                 CC_CAND = 15, CC_N = 16 };

struct HNode {
  double t;
  uint32_t ev;
  int32_t blk;
  int32_t l, r;
};
static_assert(sizeof(HNode) == 24, "HNode layout");

struct EthParams {
  uint64_t t_att;
  int32_t d, n;  // defenders, nodes
  int32_t net;   // 0 selfish mining, 1 two agents, 2 honest clique (all nodes honest),
                 // 3 exponential-delay clique (node 0 attacker; delta = mean link delay)
  int32_t mode;  // 0 gym, 1 loop
  int32_t policy, scheme;
  int32_t cap_b, cap_e;
  double ev, delta, dmax;
  int64_t max_steps, activations;
  double max_progress, max_time;
  // Nakamoto on this engine (exact re-runs of Nakamoto episodes): no
  // uncles, so payloads, rewards (1 per block), work (= height) and the ethereum_ssz agent
  // reduce to nakamoto.ml / nakamoto_ssz.ml; the nakamoto_ssz policy (or table) decides
  int32_t nak, table_dim;
  const uint8_t* table;
  // honest clique (net 2): keyed miner thresholds (n - 1) and uniform link delays
  double lo, hi;
  uint32_t thr[64];
  // fused-episode launches: device counter of episodes handed out beyond the first
  // lanes-many (zeroed before the launch); null = static grid-stride
  unsigned long long* next = nullptr;
};

constexpr int32_t NCAND = 32, NQ = 32, NSTACK = 64;
constexpr int32_t SCR_CAND = 0, SCR_KEY = 32, SCR_QA = 64, SCR_QB = 96, SCR_STACK = 128;
// per node: blocks received (V_GOT) but not yet visible, waiting for a parent
constexpr int32_t SCR_PEND = 192;
constexpr int32_t SCR_INTS = 192 + 72;

struct EthMem {
  EBlock* blk;
  uint8_t* vis;
  HNode* heap;
  int32_t* tips;
  int32_t* scr;
  // per-node outputs (cpr_node_outputs), else null: activations per node, and per block
  // slot the cumulative rewards of every node along the first-parent chain (the
  // reference's per-vertex reward arrays, simulator.ml:377-388), units of 1/32
  int64_t* nact = nullptr;
  int32_t* nrew = nullptr;
};

__host__ __device__ inline int64_t align128(int64_t x) { return (x + 127) / 128 * 128; }

__host__ __device__ inline int64_t eth_lane_bytes(int32_t cap_b, int32_t cap_e, int32_t n) {
  return align128((int64_t)cap_b * 64) + align128((int64_t)cap_b * n) +
         align128((int64_t)cap_e * 24) + align128((int64_t)n * 4) + align128(SCR_INTS * 4);
}

// per-node output region of one lane: activations [n] i64 | rewards [cap_b][n] i32
__host__ __device__ inline int64_t eth_node_bytes(int32_t cap_b, int32_t n) {
  return align128((int64_t)n * 8) + align128((int64_t)cap_b * n * 4);
}
__host__ __device__ inline void eth_node_mem(EthMem& M, uint8_t* base, int32_t n) {
  M.nact = (int64_t*)base;
  M.nrew = (int32_t*)(base + align128((int64_t)n * 8));
}

// bytes of the region after the block ring (visibility, heap, tips, scratch)
__host__ __device__ inline int64_t eth_rest_bytes(int32_t cap_b, int32_t cap_e, int32_t n) {
  return eth_lane_bytes(cap_b, cap_e, n) - align128((int64_t)cap_b * 64);
}
// block ring at blk, the rest at `rest` (e.g. LDS), same layout as eth_mem_at
__host__ __device__ inline EthMem eth_mem_split(uint8_t* blk, uint8_t* rest, int32_t cap_b,
                                                int32_t cap_e, int32_t n) {
  EthMem M;
  int64_t o = 0;
  M.blk = (EBlock*)blk;
  M.vis = rest + o;
  o += align128((int64_t)cap_b * n);
  M.heap = (HNode*)(rest + o);
  o += align128((int64_t)cap_e * 24);
  M.tips = (int32_t*)(rest + o);
  o += align128((int64_t)n * 4);
  M.scr = (int32_t*)(rest + o);
  return M;
}
__host__ __device__ inline EthMem eth_mem_at(uint8_t* base, int32_t cap_b, int32_t cap_e,
                                             int32_t n) {
  EthMem M;
  int64_t o = 0;
  M.blk = (EBlock*)(base + o);
  o += align128((int64_t)cap_b * 64);
  M.vis = base + o;
  o += align128((int64_t)cap_b * n);
  M.heap = (HNode*)(base + o);
  o += align128((int64_t)cap_e * 24);
  M.tips = (int32_t*)(base + o);
  o += align128((int64_t)n * 4);
  M.scr = (int32_t*)(base + o);
  return M;
}

// ---- policies (ethereum_ssz.ml:444-521); action = rank * 4 + own * 2 + foreign
enum : int32_t { A_ADOPT_DISCARD = 0, A_ADOPT_RELEASE = 1, A_OVERRIDE = 2, A_MATCH = 3,
                 A_RELEASE1 = 4, A_WAIT = 5 };

struct EthObs {
  int32_t public_height, public_work, private_height, private_work, diff_height, diff_work,
      public_orphans, private_orphans_inclusive, private_orphans_exclusive, event;
};

__host__ __device__ inline int32_t eth_policy(int32_t policy, const EthObs& o) {
  switch (policy) {
    case 0:  // honest
      return (o.public_work > 0 ? A_ADOPT_RELEASE : A_OVERRIDE) * 4 + 3;
    case 1:    // selfish_release
    case 2: {  // selfish_discard; Byzantium preference `HeaviestChain` -> work
      const int32_t pp = o.private_work, qp = o.public_work;
      int32_t a;
      if (pp < qp)
        a = policy == 1 ? A_ADOPT_RELEASE : A_ADOPT_DISCARD;
      else if (qp == 0)
        a = A_WAIT;
      else
        a = A_OVERRIDE;
      return a * 4 + 2;
    }
    default: {  // 3 fn19, 4 fn19pkel
      const int32_t ph = o.private_height, qh = o.public_height;
      int32_t a;
      if (o.event == 0)
        a = (ph == 2 && qh == 1) ? A_OVERRIDE : A_WAIT;
      else if (ph < qh)
        a = policy == 4 ? A_ADOPT_RELEASE : A_ADOPT_DISCARD;
      else if (ph == qh)
        a = A_MATCH;
      else if (ph == qh + 1)
        a = A_OVERRIDE;
      else
        a = A_RELEASE1;
      return a * 4 + (policy == 4 ? 2 : 3);
    }
  }
}

// table-driven ethereum_ssz policy (include/cpr_hip.h CPR_ETH_POLICY_TABLE): action =
// table[(min(public_height, D-1) * D + min(private_height, D-1)) * 2 + event], 0..23
constexpr int32_t ETH_POLICY_TABLE = 5;
// random actions (loop tasks; cpr_protocols.ml:658-782): CPR_ETH_POLICY_RANDOM, and
// CPR_POLICY_RANDOM for the nakamoto_ssz attacker of the Nakamoto mode
constexpr int32_t ETH_POLICY_RANDOM = 6, NAK_POLICY_RANDOM = 5;
__host__ __device__ inline int32_t eth_table_index(const EthObs& o, int32_t D) {
  auto cl = [](int32_t x, int32_t hi) { return x < 0 ? 0 : (x > hi ? hi : x); };
  return (cl(o.public_height, D - 1) * D + cl(o.private_height, D - 1)) * 2 + o.event;
}
__host__ __device__ inline int32_t eth_policy_t(int32_t policy, const EthObs& o,
                                                const uint8_t* table, int32_t dim) {
  if (policy == ETH_POLICY_TABLE) return (int32_t)table[eth_table_index(o, dim)];
  return eth_policy(policy, o);
}

// the lane's attack policy: ethereum_ssz (ethereum_ssz.ml:444-521) or its table, or in
// Nakamoto mode the
// nakamoto_ssz policy / table (nakamoto_ssz.ml:274-340) mapped onto the same agent
// (Adopt -> Adopt_discard; Override, Match, Wait unchanged; no uncles to choose). Used by
// the gym step and by the attacker's loop-mode handler alike.
__host__ __device__ inline int32_t lane_action(const EthParams& P, const EthObs& o) {
  if (!P.nak) return eth_policy_t(P.policy, o, P.table, P.table_dim);
  const int32_t a = nak_policy(P.policy, o.public_height, o.private_height, o.event, P.table,
                               P.table_dim);
  constexpr int32_t map[4] = {A_ADOPT_DISCARD, A_OVERRIDE, A_MATCH, A_WAIT};
  return map[a & 3] * 4;
}

// uncle filters of Honest.puzzle_payload' callers
enum : int32_t { F_ALL = 0, F_MINING = 1, F_PUBLIC = 2 };

struct Payload {
  int32_t p[3];
  int32_t np;
  int32_t height, work;
};

struct EthLane {
  double now;
  int32_t c_act, newest;
  int32_t act0;  // attacker activations
  double tclk;   // time of the latest activation (the last clock event popped)
  int32_t hroot, hfree, hused;
  uint32_t status;
  int32_t dead;  // capacity exceeded: 1 block ring, 2 event heap, 3 candidates, 4 frontier, 5 stack
                 // 6 queue drained
  // the one outstanding draft (clock -> Dag at the same instant)
  Payload dr;
  int32_t dr_node;
  // ethereum_ssz agent (BetweenActions + Observable)
  int32_t pub, priv, pending, own, foreign;
  int32_t o_pub, o_priv, o_common, o_event;
  int64_t steps;
  int32_t nrand;  // random-policy decisions so far (the keyed draw's index)

  // ------------------------------------------------------------------ storage
  __host__ __device__ inline void fail(int32_t why) {
    status |= EST_CAPACITY;
    if (!dead) dead = why;
  }
  __host__ __device__ inline EBlock& B(const EthParams& P, const EthMem& M, int32_t s) {
    EBlock& b = M.blk[s & (P.cap_b - 1)];
    if (b.serial != s) fail(1);
    return b;
  }
  __host__ __device__ inline uint8_t& V(const EthParams& P, const EthMem& M, int32_t s,
                                        int32_t node) {
    return M.vis[(int64_t)(s & (P.cap_b - 1)) * P.n + node];
  }
  __host__ __device__ inline bool visible(const EthParams& P, const EthMem& M, int32_t s,
                                          int32_t node) {
    return (V(P, M, s, node) & V_KIND) != V_INV;
  }

  // ------------------------------------------------------------------ event queue
  // orderedQueue.ml:17-47 as an in-place skew heap. Events at +inf (messages that never
  // arrive, gamma = 0) are stored too: every insertion swaps children along its path, so
  // they shape the pop order of equal-time events although they never pop in the gym.
  __host__ __device__ inline int32_t halloc(const EthParams& P, const EthMem& M) {
    int32_t i;
    if (hfree >= 0) {
      i = hfree;
      hfree = M.heap[i].l;
    } else if (hused < P.cap_e) {
      i = hused++;
    } else {
      fail(2);
      return -1;
    }
    return i;
  }
  __host__ __device__ inline void push(const EthParams& P, const EthMem& M, double t,
                                       uint32_t ev, int32_t blk) {
    CPR_HEAP_HOOK(0, t);
    int32_t parent = -1, node = hroot;
    for (;;) {
      CPR_COST(CC_PUSH);
      if (node < 0) {
        const int32_t a = halloc(P, M);
        if (a < 0) return;
        HNode& h = M.heap[a];
        h.t = t;
        h.ev = ev;
        h.blk = blk;
        h.l = -1;
        h.r = -1;
        if (parent < 0)
          hroot = a;
        else
          M.heap[parent].l = a;
        return;
      }
      HNode& h = M.heap[node];
      if (t < h.t) {
        const double ot = h.t;
        const uint32_t oe = h.ev;
        const int32_t ob = h.blk;
        h.t = t;
        h.ev = ev;
        h.blk = blk;
        t = ot;
        ev = oe;
        blk = ob;
      } else {
        const int32_t tmp = h.l;
        h.l = h.r;
        h.r = tmp;
      }
      parent = node;
      node = h.l;
    }
  }
  __host__ __device__ inline bool pop(const EthMem& M, double* t, uint32_t* ev, int32_t* blk) {
    if (hroot < 0) return false;
    CPR_HEAP_HOOK(1, M.heap[hroot].t);
    *t = M.heap[hroot].t;
    *ev = M.heap[hroot].ev;
    *blk = M.heap[hroot].blk;
    int32_t parent = -1, side = 0, node = hroot;
    for (;;) {
      CPR_COST(CC_POP);
      const int32_t l = M.heap[node].l, r = M.heap[node].r;
      int32_t repl = -2;
      if (r < 0)
        repl = l;
      else if (l < 0)
        repl = r;
      if (repl != -2) {
        if (parent < 0)
          hroot = repl;
        else if (side == 0)
          M.heap[parent].l = repl;
        else
          M.heap[parent].r = repl;
        M.heap[node].l = hfree;
        hfree = node;
        return true;
      }
      const int32_t c = (M.heap[l].t <= M.heap[r].t) ? l : r;
      M.heap[node].t = M.heap[c].t;
      M.heap[node].ev = M.heap[c].ev;
      M.heap[node].blk = M.heap[c].blk;
      parent = node;
      side = c == l ? 0 : 1;
      node = c;
    }
  }
  __host__ __device__ inline void push_now(const EthParams& P, const EthMem& M, uint32_t ev,
                                           int32_t blk) {
    push(P, M, now, ev, blk);
  }

  // ------------------------------------------------------------------ randomness
  template <class St>
  __host__ __device__ inline int32_t miner_of(const EthParams& P, const St& S, int32_t k) {
    if (P.net == 2) return S.miner_w((uint32_t)k, P.thr, P.n - 1);
    return S.miner((uint32_t)k, P.t_att, P.d);
  }
  template <class St>
  __host__ __device__ inline double act_delay(const EthParams& P, const St& S, int32_t j) {
    return S.clock((uint32_t)j, P.ev);
  }
  template <class St>
  __host__ __device__ inline void schedule_pow(const EthParams& P, const St& S,
                                               const EthMem& M) {
    push(P, M, now + act_delay(P, S, c_act), mkev(EV_CLOCK, 0, KD_POW), -1);
  }

  // ------------------------------------------------------------------ DAG
  // Nakamoto mode (one parent per block): skew-binary jump pointers (Myers 1983). A
  // block's jump is its parent's jump's jump when the parent's two jumps span equal height
  // gaps, else its parent; a jump's height depends on the height alone, so ancestor-at-
  // height and LCA queries take O(log depth) loads instead of the reference's O(depth)
  // walks (dagtools.ml:102-121, ethereum_ssz.ml:407-414). Jumps whose slot in the ring was
  // reused are not followed (the parent is).
  __host__ __device__ inline bool resident(const EthParams& P, int32_t s) const {
    return s >= 0 && newest - s < P.cap_b;
  }
  __host__ __device__ inline int32_t jump_for(const EthParams& P, const EthMem& M,
                                              int32_t parent) {
    const EBlock& pb = B(P, M, parent);
    if (pb.np == 0 || !resident(P, pb.jump)) return parent;
    const EBlock& jb = B(P, M, pb.jump);
    if (jb.np == 0 || !resident(P, jb.jump)) return parent;
    const int32_t jjh = B(P, M, jb.jump).height;
    return (pb.height - jb.height == jb.height - jjh) ? jb.jump : parent;
  }
  // ancestor of x at height h <= height(x)
  __host__ __device__ inline int32_t ancestor_at(const EthParams& P, const EthMem& M,
                                                 int32_t x, int32_t h) {
    while (!dead) {
      const EBlock& b = B(P, M, x);
      if (b.height <= h) return x;
      if (resident(P, b.jump) && B(P, M, b.jump).height >= h)
        x = b.jump;
      else
        x = b.p[0];
    }
    return x;
  }

  // simulator.ml:233-332 (genesis) and 122-136 / 377-399 (append + set_rewards with
  // ethereum.ml:173-197; precursor = first parent)
  __host__ __device__ inline int32_t append(const EthParams& P, const EthMem& M, int32_t node,
                                            const Payload& d) {
    EBlock& pb = B(P, M, d.p[0]);
    int32_t ra = pb.rew_att, rd = pb.rew_def;
    const int32_t nu = d.np - 1;
    if (node == 0)
      ra += 32 + nu;
    else
      rd += 32 + nu;
    for (int32_t i = 1; i < d.np; ++i) {
      EBlock& u = B(P, M, d.p[i]);
      const int32_t amt = P.scheme == 0 ? 30 : 4 * (8 - (d.height - u.height));
      if (u.miner == 0)
        ra += amt;
      else if (u.miner > 0)
        rd += amt;
    }
    const int32_t s = ++newest;
    if (M.nrew) {  // set_rewards per node: the precursor's array plus this block's list
      const int32_t* pr = M.nrew + (int64_t)(d.p[0] & (P.cap_b - 1)) * P.n;
      int32_t* br = M.nrew + (int64_t)(s & (P.cap_b - 1)) * P.n;
      for (int32_t j = 0; j < P.n; ++j) br[j] = pr[j];
      br[node] += 32 + nu;
      for (int32_t i = 1; i < d.np; ++i) {
        const EBlock& u = B(P, M, d.p[i]);
        if (u.miner >= 0) br[u.miner] += P.scheme == 0 ? 30 : 4 * (8 - (d.height - u.height));
      }
    }
    EBlock& b = M.blk[s & (P.cap_b - 1)];
    b.serial = s;
    b.p[0] = d.p[0];
    b.p[1] = d.np > 1 ? d.p[1] : -1;
    b.p[2] = d.np > 2 ? d.p[2] : -1;
    b.np = d.np;
    b.height = d.height;
    b.work = d.work;
    b.miner = node;
    b.rew_att = ra;
    b.rew_def = rd;
    b.share_k = -1;
    b.share_off = 0;
    b.time = now;
    b.jump = P.nak ? jump_for(P, M, d.p[0]) : d.p[0];
    if (P.nak) {  // children list of the parent, newest first (dag.ml:32)
      EBlock& par = B(P, M, d.p[0]);
      b.p[2] = par.p[1];
      par.p[1] = s;
    }
    for (int32_t j = 0; j < P.n; ++j) V(P, M, s, j) = V_INV;
    return s;
  }

  // Honest.puzzle_payload' (ethereum.ml:234-277) in node `view`'s view
  __host__ __device__ inline Payload payload(const EthParams& P, const EthMem& M, int32_t view,
                                             int32_t tip, int32_t filter, int32_t f_own,
                                             int32_t f_foreign) {
    if (P.nak) {  // Nakamoto: Honest.puzzle_payload (nakamoto.ml:77-81), one parent
      const EBlock& t = B(P, M, tip);
      Payload d;
      d.p[0] = tip;
      d.p[1] = d.p[2] = -1;
      d.np = 1;
      d.height = t.height + 1;
      d.work = t.work + 1;
      return d;
    }
    CPR_COST(CC_PAYLOAD);
    int32_t* cand = M.scr + SCR_CAND;
    int32_t* key = M.scr + SCR_KEY;
    int32_t* ic = M.scr + SCR_QA;  // in-chain set (tip + parents of tip..gen5), <= 19
    int32_t nua[6];
    int32_t ng = 0, nic = 0, lowest = -1;
    ic[nic++] = tip;
    {
      int32_t b = tip;
#pragma unroll
      for (int32_t gen = 0; gen < 6; ++gen) {
        nua[gen] = -2;
        if (b >= 0) {
          const EBlock& x = B(P, M, b);
          if (x.np == 0) {
            b = -1;
          } else {
            nua[gen] = x.p[0];
            lowest = x.p[0];
            ng = gen + 1;
            for (int32_t i = 0; i < x.np; ++i) ic[nic++] = x.p[i];
            b = x.p[0];
          }
        }
      }
    }
    // candidates: visible children of nua blocks (via the first parent), not in chain;
    // order: generation ascending, then newest first (children lists are newest first)
    int32_t nc = 0;
    if (ng > 0) {
      for (int32_t s = newest; s > lowest && !dead; --s) {
        CPR_COST(CC_SCAN);
        const uint8_t vk = V(P, M, s, view) & V_KIND;
        if (vk == V_INV) continue;
        const EBlock& c = B(P, M, s);
        if (c.np == 0) continue;
        int32_t g = -1;
#pragma unroll
        for (int32_t i = 0; i < 6; ++i)
          if (nua[i] == c.p[0]) g = i;
        if (g < 0) continue;
        bool inchain = false;
        for (int32_t i = 0; i < nic; ++i) inchain |= ic[i] == s;
        if (inchain) continue;
        const bool mine = vk == V_REL || vk == V_WH;
        bool keep = true;
        if (filter == F_MINING)
          keep = (f_own && mine) || (f_foreign && !mine);
        else if (filter == F_PUBLIC)
          keep = vk == V_REL || vk == V_RECV;
        if (!keep) continue;
        if (nc >= NCAND) {
          fail(3);
          break;
        }
        // stable insertion by generation
        int32_t pos = nc;
        while (pos > 0 && (key[pos - 1] >> 28) > g) {
          cand[pos] = cand[pos - 1];
          key[pos] = key[pos - 1];
          --pos;
        }
        CPR_COST(CC_CAND);
        cand[pos] = s;
        // sort key: not own (bit 27), height (27 bits); generation kept in bits 28+
        key[pos] = (g << 28) | ((mine ? 0 : 1) << 27) | (c.height & 0x7ffffff);
        ++nc;
      }
    }
    for (int32_t i = 0; i < nc; ++i) key[i] &= 0x0fffffff;
    ocaml_heap_sort(cand, key, nc);
    Payload d;
    const EBlock& t = B(P, M, tip);
    const int32_t nu = nc < 2 ? nc : 2;
    d.p[0] = tip;
    d.p[1] = nu > 0 ? cand[0] : -1;
    d.p[2] = nu > 1 ? cand[1] : -1;
    d.np = 1 + nu;
    d.height = t.height + 1;
    d.work = t.work + 1 + nu;
    return d;
  }

  // OCaml stdlib Array.sort (ternary heap sort, not stable) on (key, cand) pairs, keys
  // compared as integers; restated for the device (the tie order is semantics:
  // Compare.at_most_first, compare.ml:66-75, ethereum.ml:269)
  __host__ __device__ static inline void ocaml_heap_sort(int32_t* v, int32_t* k, int32_t l) {
    if (l < 2) return;
    auto maxson = [&](int32_t len, int32_t i) -> int32_t {
      const int32_t i31 = i + i + i + 1;
      int32_t x = i31;
      if (i31 + 2 < len) {
        if (k[i31] < k[i31 + 1]) x = i31 + 1;
        if (k[x] < k[i31 + 2]) x = i31 + 2;
        return x;
      }
      if (i31 + 1 < len && k[i31] < k[i31 + 1]) return i31 + 1;
      if (i31 < len) return i31;
      return -1;
    };
    for (int32_t i = (l + 1) / 3 - 1; i >= 0; --i) {
      // trickle
      const int32_t ek = k[i], ev = v[i];
      int32_t p = i;
      for (;;) {
        const int32_t j = maxson(l, p);
        if (j < 0 || !(k[j] > ek)) break;
        k[p] = k[j];
        v[p] = v[j];
        p = j;
      }
      k[p] = ek;
      v[p] = ev;
    }
    for (int32_t i = l - 1; i >= 2; --i) {
      const int32_t ek = k[i], ev = v[i];
      k[i] = k[0];
      v[i] = v[0];
      // bubble: hole from the root to a leaf
      int32_t p = 0;
      for (;;) {
        const int32_t j = maxson(i, p);
        if (j < 0) break;
        k[p] = k[j];
        v[p] = v[j];
        p = j;
      }
      // trickleup
      for (;;) {
        const int32_t father = (p - 1) / 3;
        if (k[father] < ek) {
          k[p] = k[father];
          v[p] = v[father];
          if (father > 0) {
            p = father;
            continue;
          }
          k[0] = ek;
          v[0] = ev;
          break;
        }
        k[p] = ek;
        v[p] = ev;
        break;
      }
    }
    const int32_t tk = k[0], tv = v[0];
    k[0] = k[1];
    v[0] = v[1];
    k[1] = tk;
    v[1] = tv;
  }

  // Dagtools.common_ancestor (dagtools.ml:102-121) in the attacker's view; ancestors are
  // visited by descending (depth, serial), depth = height + 1 on valid Ethereum DAGs
  __host__ __device__ static inline uint64_t ca_key(int32_t h, int32_t s) {
    return ((uint64_t)(uint32_t)h << 32) | (uint32_t)s;
  }
  // frontier: (height, serial) pairs sorted by descending key, set semantics
  __host__ __device__ inline void q_insert(int32_t* q, int32_t* nq, int32_t s, int32_t h) {
    const uint64_t kk = ca_key(h, s);
    int32_t i = *nq;
    for (int32_t j = 0; j < *nq; ++j)
      if (q[2 * j + 1] == s) return;  // set semantics
    if (*nq >= NQ / 2) {
      fail(4);
      return;
    }
    while (i > 0 && ca_key(q[2 * (i - 1)], q[2 * (i - 1) + 1]) < kk) {
      q[2 * i] = q[2 * (i - 1)];
      q[2 * i + 1] = q[2 * (i - 1) + 1];
      --i;
    }
    q[2 * i] = h;
    q[2 * i + 1] = s;
    ++*nq;
  }
  __host__ __device__ inline int32_t q_next(const EthParams& P, const EthMem& M, int32_t* q,
                                            int32_t* nq) {
    if (*nq == 0) return -1;
    CPR_COST(CC_CA);
    const int32_t s = q[1];
    for (int32_t j = 1; j < *nq; ++j) {
      q[2 * (j - 1)] = q[2 * j];
      q[2 * (j - 1) + 1] = q[2 * j + 1];
    }
    --*nq;
    const EBlock& b = B(P, M, s);
    for (int32_t i = 0; i < b.np; ++i) {
      const int32_t ps = b.p[i];
      if (!visible(P, M, ps, 0)) continue;
      q_insert(q, nq, ps, B(P, M, ps).height);
    }
    return s;
  }
  __host__ __device__ inline int32_t common_ancestor(const EthParams& P, const EthMem& M,
                                                     int32_t a, int32_t b) {
    if (P.nak) {
      // one parent per block: the frontier walk finds the lowest common ancestor of the
      // two tree paths; equal heights first, then jump pairs that still differ (jumps of
      // equal-height blocks have equal heights), else parents
      const int32_t hx = B(P, M, a).height, hy = B(P, M, b).height;
      int32_t x = ancestor_at(P, M, a, hy < hx ? hy : hx);
      int32_t y = ancestor_at(P, M, b, hy < hx ? hy : hx);
      while (x != y && !dead) {
        const EBlock& bx = B(P, M, x);
        const EBlock& by = B(P, M, y);
        if (bx.np == 0 || by.np == 0) {
          fail(4);
          return 0;
        }
        if (bx.jump != by.jump && resident(P, bx.jump) && resident(P, by.jump)) {
          x = bx.jump;
          y = by.jump;
        } else {
          x = bx.p[0];
          y = by.p[0];
        }
      }
      return x;
    }
    int32_t* qa = M.scr + SCR_QA;
    int32_t* qb = M.scr + SCR_QB;
    int32_t na = 0, nb = 0;
    q_insert(qa, &na, a, B(P, M, a).height);
    q_insert(qb, &nb, b, B(P, M, b).height);
    int32_t x = q_next(P, M, qa, &na);
    int32_t y = q_next(P, M, qb, &nb);
    while (x >= 0 && y >= 0 && !dead) {
      if (x == y) return x;
      const uint64_t kx = ca_key(B(P, M, x).height, x), ky = ca_key(B(P, M, y).height, y);
      if (kx > ky)
        x = q_next(P, M, qa, &na);
      else
        y = q_next(P, M, qb, &nb);
    }
    fail(4);
    return 0;
  }

  // ------------------------------------------------------------------ actions
  // Simulator.handle_action share part (simulator.ml:401-419): recursive release of
  // withheld blocks, parents in order; keyed link coordinates (c_act, position)
  __host__ __device__ inline void share(const EthParams& P, const EthMem& M, int32_t node,
                                        int32_t s0) {
    int32_t* st = M.scr + SCR_STACK;
    int32_t sp = 0, off = 0;
    st[sp++] = s0;
    while (sp > 0 && !dead) {
      const int32_t s = st[--sp];
      CPR_COST(CC_SHARE);
      uint8_t& v = V(P, M, s, node);
      if ((v & V_KIND) != V_WH) continue;  // received / released: nothing; invisible: n/a
      v = (uint8_t)((v & ~V_KIND) | V_REL);
      EBlock& b = B(P, M, s);
      b.share_k = c_act;
      b.share_off = off++;
      push_now(P, M, mkev(EV_TX, node, KD_NET), s);
      if (sp + b.np > NSTACK) {
        fail(5);
        return;
      }
      for (int32_t i = b.np - 1; i >= 0; --i) st[sp++] = b.p[i];
    }
  }

  __host__ __device__ inline int32_t update_head(const EthParams& P, const EthMem& M,
                                                 int32_t old, int32_t cand) {
    return B(P, M, cand).height > B(P, M, old).height ? cand : old;
  }

  // ------------------------------------------------------------------ agent
  __host__ __device__ inline void agent_init(int32_t root) {
    pub = priv = root;
    pending = -1;
    own = foreign = 1;
  }
  // ethereum_ssz.ml:325-362
  __host__ __device__ inline void prepare(const EthParams& P, const EthMem& M, uint32_t kind,
                                          int32_t x) {
    int32_t p = pub;
    if (pending >= 0) p = update_head(P, M, p, pending);
    int32_t q = priv;
    if (kind == KD_NET) {
      p = update_head(P, M, p, x);
      o_event = 1;
    } else {
      q = x;
      o_event = 0;
    }
    o_pub = p;
    o_priv = q;
    o_common = common_ancestor(P, M, p, q);
  }
  // ethereum_ssz.ml:364-396; orphans only when asked (the built-in policies never read
  // them)
  __host__ __device__ inline EthObs observe(const EthParams& P, const EthMem& M,
                                            bool orphans) {
    const EBlock& c = B(P, M, o_common);
    const EBlock& pr = B(P, M, o_priv);
    const EBlock& pu = B(P, M, o_pub);
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
      o.public_orphans = payload(P, M, 0, o_pub, F_PUBLIC, 0, 0).np - 1;
      o.private_orphans_inclusive = payload(P, M, 0, o_priv, F_MINING, 1, 1).np - 1;
      o.private_orphans_exclusive = payload(P, M, 0, o_priv, F_MINING, 1, 0).np - 1;
    }
    return o;
  }
  // ethereum_ssz.ml:398-429; returns the block to share (-1: none); index in [0, 24)
  __host__ __device__ inline int32_t apply(const EthParams& P, const EthMem& M, int32_t index) {
    const int32_t action = index >> 2;
    auto release_upto = [&](int32_t target) {
      if (P.nak) return ancestor_at(P, M, o_priv, target < 0 ? 0 : target);
      int32_t b = o_priv;
      while (!dead) {
        const EBlock& x = B(P, M, b);
        if (x.height <= target) break;
        b = x.p[0];
      }
      return b;
    };
    int32_t sh = -1, np = o_priv;
    switch (action) {
      case A_ADOPT_RELEASE:
        sh = o_priv;
        np = o_pub;
        break;
      case A_ADOPT_DISCARD: np = o_pub; break;
      case A_MATCH: sh = release_upto(B(P, M, o_pub).height); break;
      case A_OVERRIDE: sh = release_upto(B(P, M, o_pub).height + 1); break;
      case A_RELEASE1: sh = release_upto(B(P, M, o_common).height + 1); break;
      default: break;
    }
    pub = o_pub;
    priv = np;
    pending = sh;
    own = (index >> 1) & 1;
    foreign = index & 1;
    return sh;
  }

  // ------------------------------------------------------------------ engine
  template <class St>
  __host__ __device__ inline void init(const EthParams& P, const St& S, const EthMem& M) {
    now = 0.0;
    c_act = 0;
    newest = 0;
    act0 = 0;
    tclk = 0.0;
    hroot = -1;
    hfree = -1;
    hused = 0;
    status = 0u;
    dead = 0;
    steps = 0;
    nrand = 0;
    dr_node = -1;
    EBlock& r = M.blk[0];
    r.serial = 0;
    r.p[0] = r.p[1] = r.p[2] = -1;
    r.np = 0;
    r.height = 0;
    r.work = 0;
    r.miner = -1;
    r.rew_att = r.rew_def = 0;
    r.share_k = -1;
    r.share_off = 0;
    r.time = 0.0;
    r.jump = 0;
    for (int32_t j = 0; j < P.n; ++j) {
      V(P, M, 0, j) = V_RECV | V_GOT;
      M.tips[j] = 0;
      M.scr[SCR_PEND + j] = 0;
      if (M.nact) M.nact[j] = 0;
      if (M.nrew) M.nrew[j] = 0;  // genesis rewards, slot 0
    }
    agent_init(0);
    schedule_pow(P, S, M);
  }

  // one popped event that is not the attacker's gym interaction (simulator.ml:421-508)
  template <class St>
  __host__ __device__ inline void handle(const EthParams& P, const St& S, const EthMem& M,
                                         uint32_t ev, int32_t s) {
    const uint32_t ty = ev & 7u, kind = (ev >> 3) & 3u;
    const int32_t node = (int32_t)(ev >> 5);
    CPR_COST(CC_EVENT + (int32_t)ty);
    switch (ty) {
      case EV_MV: {
        uint8_t& v = V(P, M, s, node);
        if ((v & V_KIND) != V_INV) break;
        const EBlock& b = B(P, M, s);
        bool ok = true;
        for (int32_t i = 0; i < b.np; ++i) ok &= visible(P, M, b.p[i], node);
        if (!ok) break;
        if (v & V_GOT) --M.scr[SCR_PEND + node];
        v = (uint8_t)((v & ~V_KIND) | (kind == KD_NET ? V_RECV : V_WH));
        push_now(P, M, mkev(EV_ON, node, kind), s);
        push_now(P, M, mkev(EV_MDV, node, kind), s);
        break;
      }
      case EV_ON: {
        if (node == 0 && P.net != 2) {
          // loop mode: the attacker node's handler (ethereum_ssz.ml:433-441)
          prepare(P, M, kind, s);
          int32_t a;
          if (P.policy == (P.nak ? NAK_POLICY_RANDOM : ETH_POLICY_RANDOM)) {
            constexpr int32_t nmap[4] = {A_ADOPT_DISCARD, A_OVERRIDE, A_MATCH, A_WAIT};
            a = P.nak ? nmap[S.rand_act((uint32_t)nrand++, 4u)] * 4
                      : S.rand_act((uint32_t)nrand++, 24u);
          } else {
            a = lane_action(P, observe(P, M, false));
          }
          const int32_t sh = apply(P, M, a);
          if (sh >= 0) share(P, M, 0, sh);
          break;
        }
        // Honest.handler (ethereum.ml:284-297)
        int32_t& tip = M.tips[node];
        tip = update_head(P, M, tip, s);
        if ((V(P, M, s, node) & V_KIND) == V_WH) share(P, M, node, s);
        break;
      }
      case EV_CLOCK: {
        tclk = now;
        const int32_t m = miner_of(P, S, c_act);
        if (m == 0 && P.net != 2) {
          ++act0;
          dr_node = 0;
          if (P.mode == 1) dr = payload(P, M, 0, priv, F_MINING, own, foreign);
        } else {
          dr_node = m;
          dr = payload(P, M, m, M.tips[m], F_ALL, 0, 0);
        }
        push_now(P, M, mkev(EV_DAG, m, KD_POW), -1);
        if (M.nact) ++M.nact[m];
        ++c_act;
        schedule_pow(P, S, M);
        break;
      }
      case EV_DAG: {
        const int32_t v = append(P, M, node, dr);
        push_now(P, M, mkev(EV_MV, node, KD_POW), v);
        break;
      }
      case EV_TX: {
        const EBlock& b = B(P, M, s);
        for (int32_t dst = 0; dst < P.n; ++dst) {
          if (dst == node) continue;
          double delay;
          if (P.net == 2)  // models.ml:4 uniform propagation delays on every link
            delay = S.link_unif((uint32_t)b.share_k, (uint32_t)b.share_off, (uint32_t)dst, P.lo,
                                P.hi);
          else if (P.net == 3)  // cpr_protocols.ml:481-483 exponential delays on every link
            delay = S.link_exp((uint32_t)b.share_k, (uint32_t)b.share_off, (uint32_t)dst,
                               P.delta);
          else if (P.net == 1)
            delay = 0.0;
          else if (node == 0)
            delay = S.link((uint32_t)b.share_k, (uint32_t)b.share_off, (uint32_t)dst, P.dmax);
          else
            delay = dst == 0 ? 0.0 : P.delta;
          push(P, M, now + delay, mkev(EV_RX, dst, KD_NET), s);
        }
        break;
      }
      case EV_RX: {
        // simulator.ml:488-493: `now < received_at` with received_at = +inf until the
        // first receipt, so a delivery at t = +inf (Simulator.loop draining gamma = 0
        // messages) changes nothing
        if (!(now < __builtin_inf())) break;
        uint8_t& v = V(P, M, s, node);
        if (!(v & V_GOT)) {
          v |= V_GOT;
          if ((v & V_KIND) == V_INV) ++M.scr[SCR_PEND + node];
          push_now(P, M, mkev(EV_MV, node, KD_NET), s);
        }
        break;
      }
      case EV_MDV: {
        // children (newest first) already received at this node become visible; none can
        // be waiting when no received block is invisible here (the scan would find none)
        if (M.scr[SCR_PEND + node] == 0) break;
        if (P.nak) {  // the parent's children list, same order as the scan below
          for (int32_t c = B(P, M, s).p[1]; c > s && !dead; c = B(P, M, c).p[2])
            if (V(P, M, c, node) & V_GOT) push_now(P, M, mkev(EV_MV, node, KD_NET), c);
          break;
        }
        for (int32_t c = newest; c > s && !dead; --c) {
          CPR_COST(CC_MDV);
          if (!(V(P, M, c, node) & V_GOT)) continue;
          const EBlock& cb = B(P, M, c);
          bool child = false;
          for (int32_t i = 0; i < cb.np; ++i) child |= cb.p[i] == s;
          if (child) push_now(P, M, mkev(EV_MV, node, KD_NET), c);
        }
        break;
      }
    }
  }

  // engine.ml:108-121
  template <class St>
  __host__ __device__ inline bool skip_to_interaction(const EthParams& P, const St& S,
                                                      const EthMem& M, uint32_t* kind,
                                                      int32_t* blk) {
    double t;
    uint32_t ev;
    int32_t s;
    while (!dead) {
      if (!pop(M, &t, &ev, &s)) {
        fail(6);
        return false;
      }
      now = t;
      const uint32_t ty = ev & 7u;
      const int32_t node = (int32_t)(ev >> 5);
      if (ty == EV_ON && node == 0) {
        *kind = (ev >> 3) & 3u;
        *blk = s;
        return true;
      }
      if (ty == EV_DAG && node == 0) {
        const Payload d = payload(P, M, 0, priv, F_MINING, own, foreign);
        const int32_t v = append(P, M, 0, d);
        push_now(P, M, mkev(EV_MV, 0, KD_POW), v);
        continue;
      }
      handle(P, S, M, ev, s);
    }
    return false;
  }

  // ---- Nakamoto mode, hybrid re-runs (nak_hybrid.h): the engine is entered and left at
  // quiescent points whose state the closed-form lane (nakamoto_lane.h) holds exactly
  //
  // Quiescent and trivial: the queue holds the next clock event alone (every message of
  // the earlier windows delivered), every defender prefers the same block x, which a
  // defender mined (or genesis), the attacker's private and public blocks are x with no
  // share pending, and no received block waits for a parent. Then the closed-form lane's
  // state is a function of x, the latest activation's time and the counts.
  __host__ __device__ inline bool quiescent_trivial(const EthParams& P, const EthMem& M,
                                                    int32_t* x_out) {
    if (hroot < 0 || dead) return false;
    const HNode& h = M.heap[hroot];
    if (h.l >= 0 || h.r >= 0 || (h.ev & 7u) != EV_CLOCK) return false;
    if (pending >= 0 || priv != pub) return false;
    const int32_t x = priv;
    for (int32_t j = 0; j < P.n; ++j) {
      if (j > 0 && M.tips[j] != x) return false;
      if (M.scr[SCR_PEND + j] != 0) return false;
    }
    if (B(P, M, x).miner == 0) return false;
    *x_out = x;
    return true;
  }
  // the engine at such a point, from the closed-form lane's: block x (serial xs, its
  // height, rewards in 1/32, mining time and miner) is the only block (a root: no parent is
  // ever asked for below it, every later block descends from it), k activations done, the
  // latest at time t, `steps` gym steps counted as gym_step counts them (apply of the
  // current step done); the clock of activation k is scheduled from t as the engine did
  template <class St>
  __host__ __device__ inline void enter_trivial(const EthParams& P, const St& S,
                                                const EthMem& M, int32_t xs, int32_t height,
                                                int32_t ra32, int32_t rd32, double tm,
                                                int32_t miner, int32_t k, double t,
                                                int64_t steps_) {
    now = t;
    tclk = t;
    c_act = k;
    newest = k;
    act0 = 0;
    hroot = -1;
    hfree = -1;
    hused = 0;
    dead = 0;
    steps = steps_;
    nrand = 0;
    dr_node = -1;
    EBlock& r = M.blk[xs & (P.cap_b - 1)];
    r.serial = xs;
    r.p[0] = r.p[1] = r.p[2] = -1;
    r.np = 0;
    r.height = height;
    r.work = height;  // Nakamoto mode: work = height
    r.miner = miner;
    r.rew_att = ra32;
    r.rew_def = rd32;
    r.share_k = -1;
    r.share_off = 0;
    r.time = tm;
    r.jump = xs;
    for (int32_t j = 0; j < P.n; ++j) {
      V(P, M, xs, j) = V_RECV | V_GOT;
      M.tips[j] = xs;
      M.scr[SCR_PEND + j] = 0;
    }
    agent_init(xs);
    schedule_pow(P, S, M);
  }
  // skip_to_interaction that stops (returns 1, *x_out = the block) before popping the clock
  // of an activation >= stop_k at a quiescent trivial point; 0 = the attacker's interaction
  // (*kind, *blk), -1 = none (dead)
  template <class St>
  __host__ __device__ inline int32_t skip_or_stop(const EthParams& P, const St& S,
                                                  const EthMem& M, uint32_t* kind,
                                                  int32_t* blk, int32_t stop_k,
                                                  int32_t* x_out) {
    double t;
    uint32_t ev;
    int32_t s;
    while (!dead) {
      if (c_act >= stop_k && quiescent_trivial(P, M, x_out)) return 1;
      if (!pop(M, &t, &ev, &s)) {
        fail(6);
        return -1;
      }
      now = t;
      const uint32_t ty = ev & 7u;
      const int32_t node = (int32_t)(ev >> 5);
      if (ty == EV_ON && node == 0) {
        *kind = (ev >> 3) & 3u;
        *blk = s;
        return 0;
      }
      if (ty == EV_DAG && node == 0) {
        const Payload d = payload(P, M, 0, priv, F_MINING, own, foreign);
        const int32_t v = append(P, M, 0, d);
        push_now(P, M, mkev(EV_MV, 0, KD_POW), v);
        continue;
      }
      handle(P, S, M, ev, s);
    }
    return -1;
  }

  // winner over [attacker preference; defenders' tips] (ethereum.ml:159-162)
  __host__ __device__ inline int32_t head(const EthParams& P, const EthMem& M, int32_t att) {
    int32_t h = att;
    int32_t hh = B(P, M, att).height;
    for (int32_t j = 1; j < P.n; ++j) {
      const int32_t t = M.tips[j];
      const int32_t th = B(P, M, t).height;
      if (th > hh) {
        h = t;
        hh = th;
      }
    }
    return h;
  }

  // gym: reset (engine.ml:122-170)
  template <class St>
  __host__ __device__ inline void gym_reset(const EthParams& P, const St& S,
                                            const EthMem& M) {
    init(P, S, M);
    uint32_t kind;
    int32_t b;
    if (skip_to_interaction(P, S, M, &kind, &b)) prepare(P, M, kind, b);
  }

  // gym: step (engine.ml:176-249); returns the head, sets *done
  template <class St>
  __host__ __device__ inline int32_t gym_step(const EthParams& P, const St& S,
                                              const EthMem& M, int32_t action, bool* done) {
    const int32_t sh = apply(P, M, action);
    if (sh >= 0) share(P, M, 0, sh);
    ++steps;
    uint32_t kind;
    int32_t b;
    const int32_t att = priv;
    if (skip_to_interaction(P, S, M, &kind, &b)) prepare(P, M, kind, b);
    const int32_t hd = head(P, M, att);
    const double progress = (double)B(P, M, hd).work;
    *done = dead || !(steps < P.max_steps && progress < P.max_progress && now < P.max_time);
    return hd;
  }

  // loop: Simulator.loop ~activations (simulator.ml:519-533), then the head
  template <class St>
  __host__ __device__ inline int32_t loop(const EthParams& P, const St& S, const EthMem& M) {
    init(P, S, M);
    int64_t left = P.activations;
    double t;
    uint32_t ev;
    int32_t s;
    while (!dead && pop(M, &t, &ev, &s)) {
      now = t;
      if ((ev & 7u) == EV_CLOCK) {
        if (left <= 0) continue;
        --left;
      }
      handle(P, S, M, ev, s);
    }
    return head(P, M, P.net == 2 ? M.tips[0] : priv);
  }
};

}  // namespace eth
}  // namespace cpr
