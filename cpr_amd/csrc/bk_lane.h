// B_k (parallel proof of work, bk.ml) with the bk_ssz attack space: one episode per lane,
// as an exact per-lane discrete-event engine.
//
// B_k's honest nodes re-run quorum selection on every event they see (bk.ml:297-310):
// the k smallest own votes, or the leader's smallest own vote plus the earliest-visible
// foreign votes with larger hashes (bk.ml:233-279), ordered by the OCaml heap sort whose
// tie order among equal visibility times is semantics (compare.ml:44-62). Fork choice
// compares heights, confirming-vote counts in the node's view, leader hashes and
// visibility times (bk.ml:217-231). All of that reads per-node visibility and time of
// individual votes, so the lane replays the reference's event semantics itself, with the
// skew-heap tie order of orderedQueue.ml:17-47, like the Ethereum lane.
//
// Per-lane memory (one contiguous region per resident lane):
//   vtx    [cap_v] x 48 B   vertex ring (votes and blocks) indexed by serial & (cap_v-1);
//                           a stale slot (serial mismatch) marks the lane CPR_ST_CAPACITY
//   vis    [cap_v][n] u8    per node: kind (invisible/received/released/withheld) + got bit
//   vt     [cap_v][n] f64   per node: visible_since (simulator.ml:291-294)
//   vc     [cap_v][n] u64   blocks, per node: visible votes on the block by kind (16-bit
//                           received / released / withheld counts), maintained where a
//                           vote's kind changes, so vote counts need no list walk
//   (CPR_BK_AOS = 1, the default: vtx, vn, vh, vis, vt and vc of one slot share one record
//   of 2^rsh bytes — 128 for n <= 3 — so the handlers' accesses to a vertex touch one
//   cache line instead of six; 0: the six arrays above, for A/B runs)
//   quo    [cap_q][k+1] i32 block quorums (tag = block serial, then k vote serials by hash)
//   drafts [cap_d][k+2] i32 outstanding Append drafts (tag, parent, k votes)
//   heap   [cap_e] x 24 B   skew-heap nodes of the event queue
//   tips   [n] i32          defenders' preferred blocks (Honest.state)
//   scratch                 quorum candidates (keys, serials), share stack
//
// Reference map: simulator.ml:122-543 (engine), bk.ml:50-311 (referee, honest node),
// bk_ssz.ml:148-401 (agent, policies), engine.ml:97-249 (gym step), network.ml
// selfish_mining / two_agents (links), keyed stream (cpr_stream.h, TAG_MSG link delays).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpr_stream.h"

// address space of the event-heap slab (LDS) in device code: loads and stores through it
// compile to ds_read / ds_write rather than generic flat accesses
#if defined(__HIP_DEVICE_COMPILE__)
#define CPR_LDS __attribute__((address_space(3)))
#else
#define CPR_LDS
#endif

#pragma clang fp contract(off)

// host cost studies (tools/bk_cost_study.cpp) count work items by id (BC_* below)
#ifndef CPR_BK_COST
#define CPR_BK_COST(id)
#endif

namespace cpr {
namespace bk {

enum : int32_t { BC_PUSH = 0, BC_POP = 1, BC_CONFIRMING = 2, BC_PROPOSE = 3, BC_OBSERVE = 4,
                 BC_APPLY = 5, BC_MDV = 6, BC_EVENT = 7 /* + event type, 7 types */,
                 BC_PROPOSE_CALLS = 14, BC_CONFIRMING_CALLS = 15, BC_N = 16 };

constexpr uint32_t BST_CAPACITY = 32u;  // CPR_ST_CAPACITY

enum : uint32_t { EV_CLOCK = 0, EV_DAG = 1, EV_TX = 2, EV_RX = 3, EV_ON = 4, EV_MV = 5, EV_MDV = 6 };
enum : uint32_t { KD_APP = 0, KD_POW = 1, KD_NET = 2 };
enum : uint8_t { V_INV = 0, V_RECV = 1, V_REL = 2, V_WH = 3, V_KIND = 3, V_GOT = 4 };
enum : int32_t { VF_ALL = 0, VF_MINE = 1, VF_PUBLIC = 2 };

__host__ __device__ inline uint32_t mkev(uint32_t ty, uint32_t node, uint32_t kind) {
  return ty | (kind << 3) | (node << 5);
}

struct BVtx {
  int32_t serial;
  int32_t parent;  // block parent (votes and blocks); -1 = genesis
  int32_t height;
  int32_t vote;    // 1 = Vote, 0 = Block
  int32_t who;     // vote: miner id; block: signer; -1 = genesis
  int32_t pow;     // 30-bit hash bits (votes)
  int32_t rew_att, rew_def;  // rewards of the precursor chain (units of 1)
  int32_t nconf;   // blocks: confirming votes in the global view (Referee.winner)
  int32_t qslot;   // blocks: quorum ring slot
  double time;     // Simulator.timestamp = append time
};
static_assert(sizeof(BVtx) == 48, "BVtx layout");

struct HNode {
  double t;
  uint32_t ev;
  int32_t blk;
  int32_t l, r;
};
static_assert(sizeof(HNode) == 24, "HNode layout");

struct BkParams {
  uint64_t t_att;
  int32_t d, n;   // defenders, nodes
  int32_t net;    // 0 selfish mining, 1 two agents, 2 honest clique (all nodes honest),
                  // 3 exponential-delay clique (node 0 attacker; delta = mean link delay)
  int32_t mode;   // 0 gym, 1 loop
  int32_t policy, scheme, k;
  int32_t cap_v, cap_q, cap_e, cap_d;
  int32_t table_dim;
  double ev, delta, dmax;
  int64_t max_steps, activations;
  double max_progress, max_time;
  const uint8_t* table;  // device pointer (CPR_BK_POLICY_TABLE)
  // honest clique (net 2, models.ml:3-28): keyed miner thresholds (n - 1), U(lo, hi) links
  double lo, hi;
  uint32_t thr[64];
  // fused-episode launches: device counter of episodes handed out beyond the first
  // lanes-many (zeroed before the launch); null = static grid-stride
  unsigned long long* next = nullptr;
};

constexpr int32_t NQS = 128;     // quorum candidates per block and list
constexpr int32_t NSTACK = 1024; // share stack

#ifndef CPR_BK_AOS
#define CPR_BK_AOS 1
#endif
// the per-slot record (CPR_BK_AOS): BVtx | vn (int4) | vh (int32) | vis [n] | vt [n] | vc [n]
constexpr int32_t BK_OFF_VN = 48, BK_OFF_VH = 64, BK_OFF_VIS = 68;
__host__ __device__ inline int32_t bk_off_vt(int32_t n) { return (BK_OFF_VIS + n + 7) & ~7; }
__host__ __device__ inline int32_t bk_off_vc(int32_t n) { return bk_off_vt(n) + 8 * n; }
__host__ __device__ inline int32_t bk_rec_shift(int32_t n) {
  int32_t sh = 6;
  while ((1 << sh) < bk_off_vc(n) + 8 * n) ++sh;
  return sh;
}

struct BkMem {
  // event-heap nodes 0 .. kl-1 live in the workgroup's LDS slab (hl, this lane's part) for
  // the duration of a kernel, the rest in HBM (heap): a window's live events (14-22 at the
  // gym's gamma = .5, tools/bk_cost_study.cpp) stay off the memory hierarchy. Kernels with a
  // slab load nodes 0 .. kl-1 from heap at entry and store them back at exit (bk_heap_*)
  CPR_LDS HNode* hl = nullptr;
  int32_t kl = 0, hs = 1;
  // visibility rows of the newest vw vertices (vw a power of 2, 0 = none) in the same
  // workgroup slab, row-major per lane: byte (slot * n + node) * hs of vl, slot = s & (vw - 1).
  // Writes go to both places (HBM stays complete), reads of a vertex in the window to LDS:
  // the walks (vote lists, MadeDescendantsVisible, the release closure) read recent rows
  CPR_LDS uint8_t* vl = nullptr;
  int32_t vw = 0;
#if CPR_BK_AOS
  uint8_t* rec;     // [cap_v] records of 2^rsh bytes
  int32_t rsh;
#else
  BVtx* vtx;
  // the votes of each block, newest first (the order of the reference's children scans),
  // as two compact per-slot arrays beside the vertices so that a walk reads 4-byte links
  // and visibility bytes, and a vote's 48-byte vertex only when it passes the filter:
  // vh[block] = its newest vote (-1 none), vn[vote] = the next older vote of its block
  int32_t* vh;
  // vote: x = next older vote of its block, y = pow, z = who (the propose scan's fields);
  // block: x = next older child block of its parent, w = its newest child block (-1 none)
  int4* vn;
  uint8_t* vis;
  double* vt;
  uint64_t* vc;
#endif
  int32_t* quo;
  int32_t* drafts;
  HNode* heap;
  int32_t* tips;
  uint64_t* skey;  // [2 * NQS]
  int32_t* sval;   // [2 * NQS]
  int32_t* stack;  // [NSTACK]
  // per-node outputs (cpr_node_outputs), else null: activations per node, and per block
  // quorum slot the cumulative rewards of every node along the block chain (the
  // reference's per-vertex reward arrays, simulator.ml:377-388); genesis = zeros
  int64_t* nact = nullptr;
  int32_t* nrew = nullptr;
};

__host__ __device__ inline int64_t bk_align(int64_t x) { return (x + 127) / 128 * 128; }

__host__ __device__ inline int64_t bk_lane_bytes(const BkParams& P) {
  return
#if CPR_BK_AOS
         bk_align((int64_t)P.cap_v << bk_rec_shift(P.n)) +
#else
         bk_align((int64_t)P.cap_v * (int64_t)sizeof(BVtx)) + bk_align((int64_t)P.cap_v * 4) +
         bk_align((int64_t)P.cap_v * 16) +
         bk_align((int64_t)P.cap_v * P.n) +
         bk_align((int64_t)P.cap_v * P.n * 8) + bk_align((int64_t)P.cap_v * P.n * 8) +
#endif
         bk_align((int64_t)P.cap_q * (P.k + 1) * 4) +
         bk_align((int64_t)P.cap_d * (P.k + 2) * 4) + bk_align((int64_t)P.cap_e * 24) +
         bk_align((int64_t)P.n * 4) + bk_align(2 * NQS * 8) + bk_align(2 * NQS * 4) +
         bk_align(NSTACK * 4);
}

__host__ __device__ inline BkMem bk_mem_at(uint8_t* base, const BkParams& P) {
  BkMem M;
  int64_t o = 0;
#if CPR_BK_AOS
  M.rec = base + o;
  M.rsh = bk_rec_shift(P.n);
  o += bk_align((int64_t)P.cap_v << M.rsh);
#else
  M.vtx = (BVtx*)(base + o);
  o += bk_align((int64_t)P.cap_v * (int64_t)sizeof(BVtx));
  M.vh = (int32_t*)(base + o);
  o += bk_align((int64_t)P.cap_v * 4);
  M.vn = (int4*)(base + o);
  o += bk_align((int64_t)P.cap_v * 16);
  M.vis = base + o;
  o += bk_align((int64_t)P.cap_v * P.n);
  M.vt = (double*)(base + o);
  o += bk_align((int64_t)P.cap_v * P.n * 8);
  M.vc = (uint64_t*)(base + o);
  o += bk_align((int64_t)P.cap_v * P.n * 8);
#endif
  M.quo = (int32_t*)(base + o);
  o += bk_align((int64_t)P.cap_q * (P.k + 1) * 4);
  M.drafts = (int32_t*)(base + o);
  o += bk_align((int64_t)P.cap_d * (P.k + 2) * 4);
  M.heap = (HNode*)(base + o);
  o += bk_align((int64_t)P.cap_e * 24);
  M.tips = (int32_t*)(base + o);
  o += bk_align((int64_t)P.n * 4);
  M.skey = (uint64_t*)(base + o);
  o += bk_align(2 * NQS * 8);
  M.sval = (int32_t*)(base + o);
  o += bk_align(2 * NQS * 4);
  M.stack = (int32_t*)(base + o);
  return M;
}

// raw per-slot fields of vertex serial s (no serial check)
#if CPR_BK_AOS
__host__ __device__ inline uint8_t* bk_rec(const BkParams& P, const BkMem& M, int32_t s) {
  return M.rec + ((int64_t)(s & (P.cap_v - 1)) << M.rsh);
}
__host__ __device__ inline BVtx& bk_vtx(const BkParams& P, const BkMem& M, int32_t s) {
  return *reinterpret_cast<BVtx*>(bk_rec(P, M, s));
}
__host__ __device__ inline int32_t& bk_vh(const BkParams& P, const BkMem& M, int32_t s) {
  return *reinterpret_cast<int32_t*>(bk_rec(P, M, s) + BK_OFF_VH);
}
__host__ __device__ inline int4& bk_vn(const BkParams& P, const BkMem& M, int32_t s) {
  return *reinterpret_cast<int4*>(bk_rec(P, M, s) + BK_OFF_VN);
}
__host__ __device__ inline uint8_t& bk_vis(const BkParams& P, const BkMem& M, int32_t s,
                                           int32_t node) {
  return bk_rec(P, M, s)[BK_OFF_VIS + node];
}
__host__ __device__ inline double& bk_vt(const BkParams& P, const BkMem& M, int32_t s,
                                         int32_t node) {
  return reinterpret_cast<double*>(bk_rec(P, M, s) + bk_off_vt(P.n))[node];
}
__host__ __device__ inline uint64_t& bk_vc(const BkParams& P, const BkMem& M, int32_t s,
                                           int32_t node) {
  return reinterpret_cast<uint64_t*>(bk_rec(P, M, s) + bk_off_vc(P.n))[node];
}
#else
__host__ __device__ inline BVtx& bk_vtx(const BkParams& P, const BkMem& M, int32_t s) {
  return M.vtx[s & (P.cap_v - 1)];
}
__host__ __device__ inline int32_t& bk_vh(const BkParams& P, const BkMem& M, int32_t s) {
  return M.vh[s & (P.cap_v - 1)];
}
__host__ __device__ inline int4& bk_vn(const BkParams& P, const BkMem& M, int32_t s) {
  return M.vn[s & (P.cap_v - 1)];
}
__host__ __device__ inline uint8_t& bk_vis(const BkParams& P, const BkMem& M, int32_t s,
                                           int32_t node) {
  return M.vis[(int64_t)(s & (P.cap_v - 1)) * P.n + node];
}
__host__ __device__ inline double& bk_vt(const BkParams& P, const BkMem& M, int32_t s,
                                         int32_t node) {
  return M.vt[(int64_t)(s & (P.cap_v - 1)) * P.n + node];
}
__host__ __device__ inline uint64_t& bk_vc(const BkParams& P, const BkMem& M, int32_t s,
                                           int32_t node) {
  return M.vc[(int64_t)(s & (P.cap_v - 1)) * P.n + node];
}
#endif

// the LDS heap slab of a kernel (BkMem.hl): this lane's nodes 0 .. kl-1 at
// slab[i * stride + lane]; persistent lanes (rollouts) load the nodes their heap uses at
// entry and store them back at exit, so between kernels the whole heap is in HBM
__host__ __device__ inline void bk_heap_slab(BkMem& M, HNode* slab, int32_t lane,
                                             int32_t stride, int32_t kl) {
  M.hl = (CPR_LDS HNode*)(slab + lane);
  M.hs = stride;
  M.kl = kl;
}
// the visibility window (BkMem.vl) of a kernel: after the heap slab's kl nodes; persistent
// lanes (rollouts) load the window's rows at entry (bk_vis_load)
__host__ __device__ inline void bk_vis_window(BkMem& M, uint8_t* base, int32_t lane, int32_t vw) {
  M.vl = (CPR_LDS uint8_t*)(base + lane);
  M.vw = vw;
}
__host__ __device__ inline void bk_vis_load(const BkMem& M, const BkParams& P, int32_t newest) {
  for (int32_t s = newest - M.vw + 1 < 0 ? 0 : newest - M.vw + 1; s <= newest; ++s)
    for (int32_t j = 0; j < P.n; ++j)
      M.vl[(int64_t)((s & (M.vw - 1)) * P.n + j) * M.hs] = bk_vis(P, M, s, j);
}
__host__ __device__ inline void bk_heap_load(const BkMem& M, int32_t hused) {
  const int32_t n = hused < M.kl ? hused : M.kl;
  for (int32_t i = 0; i < n; ++i) M.hl[(int64_t)i * M.hs] = M.heap[i];
}
__host__ __device__ inline void bk_heap_store(const BkMem& M, int32_t hused) {
  const int32_t n = hused < M.kl ? hused : M.kl;
  for (int32_t i = 0; i < n; ++i) M.heap[i] = M.hl[(int64_t)i * M.hs];
}

// per-node output region of one lane: activations [n] i64 | rewards [cap_q][n] i32
__host__ __device__ inline int64_t bk_node_bytes(const BkParams& P) {
  return bk_align((int64_t)P.n * 8) + bk_align((int64_t)P.cap_q * P.n * 4);
}
__host__ __device__ inline void bk_node_mem(BkMem& M, uint8_t* base, const BkParams& P) {
  M.nact = (int64_t*)base;
  M.nrew = (int32_t*)(base + bk_align((int64_t)P.n * 8));
}

// ---- observation and policies (bk_ssz.ml:21-34, 346-401); Action8 ranks
enum : int32_t { A_ADOPT_PROLONG = 0, A_OVERRIDE_PROLONG = 1, A_MATCH_PROLONG = 2,
                 A_WAIT_PROLONG = 3, A_ADOPT_PROCEED = 4, A_OVERRIDE_PROCEED = 5,
                 A_MATCH_PROCEED = 6, A_WAIT_PROCEED = 7 };

struct BkObs {
  int32_t public_blocks, private_blocks, diff_blocks, public_votes, private_votes_inclusive,
      private_votes_exclusive, lead, event;  // event: 0 Append, 1 ProofOfWork, 2 Network
};

__host__ __device__ inline int32_t bk_table_index(const BkObs& o, int32_t D, int32_t k) {
  auto cl = [](int32_t x, int32_t hi) { return x < 0 ? 0 : (x > hi ? hi : x); };
  const int32_t K1 = k + 1;
  return ((((cl(o.public_blocks, D - 1) * D + cl(o.private_blocks, D - 1)) * K1 +
            cl(o.public_votes, k)) * K1 + cl(o.private_votes_inclusive, k)) * 3) + o.event;
}

__host__ __device__ inline int32_t bk_policy(const BkParams& P, const BkObs& o) {
  const int32_t h = o.public_blocks, a = o.private_blocks;
  switch (P.policy) {
    case 0:  // honest
      return h > a ? A_ADOPT_PROCEED : A_OVERRIDE_PROCEED;
    case 1:  // get-ahead
      return h > a ? A_ADOPT_PROCEED : (h < a ? A_OVERRIDE_PROCEED : A_WAIT_PROCEED);
    case 2:  // minor-delay
      return h > a ? A_ADOPT_PROCEED : (h == 0 ? A_WAIT_PROCEED : A_OVERRIDE_PROCEED);
    case 3: {  // avoid-loss = avoid_loss_alt (bk_ssz.ml:391-401,411-414)
      const int32_t hp = h * P.k + o.public_votes, ap = a * P.k + o.private_votes_inclusive;
      if (h == 0) return A_WAIT_PROCEED;
      if (h == 1 && hp == ap) return A_MATCH_PROCEED;
      if (hp > ap) return A_ADOPT_PROCEED;
      if (hp == ap - 1) return A_OVERRIDE_PROCEED;
      if (h < a - 10) return A_OVERRIDE_PROCEED;
      return A_WAIT_PROCEED;
    }
    default:  // table
      return P.table[bk_table_index(o, P.table_dim, P.k)];
  }
}

// OCaml stdlib Array.sort (ternary heap sort, not stable) on (key, value) pairs with
// 64-bit keys (the ethereum lane has the int32 version; see oracle/src/ocaml_sort.h)
__host__ __device__ inline void ocaml_heap_sort64(int32_t* v, uint64_t* k, int32_t l) {
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
    const uint64_t ek = k[i];
    const int32_t ev = v[i];
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
    const uint64_t ek = k[i];
    const int32_t ev = v[i];
    k[i] = k[0];
    v[i] = v[0];
    int32_t p = 0;
    for (;;) {
      const int32_t j = maxson(i, p);
      if (j < 0) break;
      k[p] = k[j];
      v[p] = v[j];
      p = j;
    }
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
  const uint64_t tk = k[0];
  const int32_t tv = v[0];
  k[0] = k[1];
  v[0] = v[1];
  k[1] = tk;
  v[1] = tv;
}

// visibility times are finite and >= +0.0, so their IEEE bit patterns order like
// OCaml's Float.compare on them
__host__ __device__ inline uint64_t time_key(double t) { return bitsd(t); }

// random actions (loop tasks; cpr_protocols.ml:658-782): CPR_BK_POLICY_RANDOM
constexpr int32_t BK_POLICY_RANDOM = 5;

struct BkLane {
  int32_t nrand;  // random-policy decisions so far (the keyed draw's index)
  double now;
  int32_t c_act, newest, nblk, act0;
  int32_t hroot, hfree, hused, hfree2;
  uint32_t status;
  int32_t dead;  // capacity exceeded: 1 vertex ring, 2 event heap, 3 quorum list, 4 drafts,
                 // 5 share stack, 6 queue drained, 7 quorum ring, 8 zero-time append loop
  int32_t zt;    // appends since the last activation (loop-mode guard, see append_block)
  int32_t dseq;  // Append drafts issued
  // bk_ssz agent (BetweenActions + Observable)
  int32_t pub, priv, pending;
  int32_t o_pub, o_priv, o_common, o_event;
  int64_t steps;

  // ------------------------------------------------------------------ storage
  __host__ __device__ inline void fail(int32_t why) {
    status |= BST_CAPACITY;
    if (!dead) dead = why;
  }
  __host__ __device__ inline BVtx& X(const BkParams& P, const BkMem& M, int32_t s) {
    BVtx& b = bk_vtx(P, M, s);
    if (b.serial != s) fail(1);
    return b;
  }
  __host__ __device__ inline int32_t& VH(const BkParams& P, const BkMem& M, int32_t s) {
    return bk_vh(P, M, s);
  }
  __host__ __device__ inline int32_t& VN(const BkParams& P, const BkMem& M, int32_t s) {
    return bk_vn(P, M, s).x;
  }
  __host__ __device__ inline int4& VR(const BkParams& P, const BkMem& M, int32_t s) {
    return bk_vn(P, M, s);
  }
  __host__ __device__ inline uint8_t& V(const BkParams& P, const BkMem& M, int32_t s,
                                        int32_t node) {
    return bk_vis(P, M, s, node);
  }
  __host__ __device__ inline double& VT(const BkParams& P, const BkMem& M, int32_t s,
                                        int32_t node) {
    return bk_vt(P, M, s, node);
  }
  // visible-vote counts of block b at node (vc): 16-bit fields by kind, V_RECV at bit 0,
  // V_REL at 16, V_WH at 32
  __host__ __device__ inline uint64_t& VC(const BkParams& P, const BkMem& M, int32_t b,
                                          int32_t node) {
    return bk_vc(P, M, b, node);
  }
  __host__ __device__ static inline int32_t vc_field(uint64_t c, uint8_t kind) {
    return (int32_t)((c >> (16 * (kind - 1))) & 0xffffu);
  }
  // counts passing vf: kinds kept by keep(., vf)
  __host__ __device__ static inline int32_t vc_count(uint64_t c, int32_t vf) {
    const int32_t rc = vc_field(c, V_RECV), rl = vc_field(c, V_REL), wh = vc_field(c, V_WH);
    return vf == VF_ALL ? rc + rl + wh : (vf == VF_MINE ? wh + rl : rl + rc);
  }
  __host__ __device__ inline bool visible(const BkParams& P, const BkMem& M, int32_t s,
                                          int32_t node) {
    return (Vg(P, M, s, node) & V_KIND) != V_INV;
  }
  // visibility of vertex s at node: from the LDS window when s is one of the newest vw
  // vertices (every append writes its row into the window slot it takes), else HBM
  __host__ __device__ inline uint8_t Vg(const BkParams& P, const BkMem& M, int32_t s,
                                        int32_t node) const {
    if (s > newest - M.vw) {
      // volatile: a load of its own (not merged with the HBM branch into a flat access)
      return *(const volatile CPR_LDS uint8_t*)&M.vl[(int64_t)((s & (M.vw - 1)) * P.n + node) *
                                                      M.hs];
    }
    return bk_vis(P, M, s, node);
  }
  __host__ __device__ inline void Vs(const BkParams& P, const BkMem& M, int32_t s, int32_t node,
                                     uint8_t v) const {
    bk_vis(P, M, s, node) = v;
    if (s > newest - M.vw) M.vl[(int64_t)((s & (M.vw - 1)) * P.n + node) * M.hs] = v;
  }
  __host__ __device__ inline int32_t* Q(const BkParams& P, const BkMem& M, const BVtx& b) {
    int32_t* q = M.quo + (int64_t)(b.qslot & (P.cap_q - 1)) * (P.k + 1);
    if (q[0] != b.serial) fail(7);
    return q + 1;
  }
  __host__ __device__ static inline bool keep(uint8_t v, int32_t vf) {
    const uint8_t kd = v & V_KIND;
    return vf == VF_ALL || (vf == VF_MINE ? (kd == V_WH || kd == V_REL)
                                          : (kd == V_REL || kd == V_RECV));
  }

  // ------------------------------------------------------------------ event queue
  // orderedQueue.ml:17-47 as an in-place skew heap. Events at +inf (messages that never
  // arrive, gamma = 0) are stored too: every insertion swaps children along its path, so
  // they shape the pop order of equal-time events even though they never pop in a gym
  // episode (B_k is sensitive to that order: which same-instant Append lands first).
  // Nodes are read and written by value through hn_*, each picking the slab (LDS, an
  // address-space-3 pointer: ds_read / ds_write) or the HBM part (global loads) by index,
  // so the compiler never merges the two into one generic (flat) access.
  __host__ __device__ static inline HNode hn_get(const BkMem& M, int32_t i) {
    if (i < M.kl) {
      // volatile: keeps this a load of its own (the compiler would otherwise merge the two
      // branches into one load through a generic pointer)
      const volatile CPR_LDS HNode& v = M.hl[(int64_t)i * M.hs];
      HNode h;
      h.t = v.t;
      h.ev = v.ev;
      h.blk = v.blk;
      h.l = v.l;
      h.r = v.r;
      return h;
    }
    return M.heap[i];
  }
  __host__ __device__ static inline void hn_put(const BkMem& M, int32_t i, const HNode& h) {
    if (i < M.kl)
      M.hl[(int64_t)i * M.hs] = h;
    else
      M.heap[i] = h;
  }
  __host__ __device__ static inline void hn_set_l(const BkMem& M, int32_t i, int32_t v) {
    if (i < M.kl)
      M.hl[(int64_t)i * M.hs].l = v;
    else
      M.heap[i].l = v;
  }
  __host__ __device__ static inline void hn_set_r(const BkMem& M, int32_t i, int32_t v) {
    if (i < M.kl)
      M.hl[(int64_t)i * M.hs].r = v;
    else
      M.heap[i].r = v;
  }
  __host__ __device__ static inline void hn_set_lr(const BkMem& M, int32_t i, int32_t l,
                                                   int32_t r) {
    if (i < M.kl) {
      M.hl[(int64_t)i * M.hs].l = l;
      M.hl[(int64_t)i * M.hs].r = r;
    } else {
      M.heap[i].l = l;
      M.heap[i].r = r;
    }
  }
  __host__ __device__ static inline void hn_set_key(const BkMem& M, int32_t i, double t,
                                                    uint32_t ev, int32_t blk) {
    if (i < M.kl) {
      CPR_LDS HNode& h = M.hl[(int64_t)i * M.hs];
      h.t = t;
      h.ev = ev;
      h.blk = blk;
    } else {
      HNode& h = M.heap[i];
      h.t = t;
      h.ev = ev;
      h.blk = blk;
    }
  }
  // free nodes: slab nodes first (hfree), then HBM nodes (hfree2)
  __host__ __device__ inline int32_t halloc(const BkParams& P, const BkMem& M) {
    int32_t i;
    if (hfree >= 0) {
      i = hfree;
      hfree = hn_get(M, i).l;
    } else if (hused < P.cap_e && (hused < M.kl || hfree2 < 0)) {
      i = hused++;
    } else if (hfree2 >= 0) {
      i = hfree2;
      hfree2 = hn_get(M, i).l;
    } else {
      fail(2);
      return -1;
    }
    return i;
  }
  __host__ __device__ inline void hrelease(const BkMem& M, int32_t node) {
    if (node < M.kl) {
      hn_set_l(M, node, hfree);
      hfree = node;
    } else {
      hn_set_l(M, node, hfree2);
      hfree2 = node;
    }
  }
  __host__ __device__ inline void push(const BkParams& P, const BkMem& M, double t, uint32_t ev,
                                       int32_t blk) {
    int32_t parent = -1, node = hroot;
    for (;;) {
      CPR_BK_COST(BC_PUSH);
      if (node < 0) {
        const int32_t a = halloc(P, M);
        if (a < 0) return;
        HNode h;
        h.t = t;
        h.ev = ev;
        h.blk = blk;
        h.l = -1;
        h.r = -1;
        hn_put(M, a, h);
        if (parent < 0)
          hroot = a;
        else
          hn_set_l(M, parent, a);
        return;
      }
      const HNode h = hn_get(M, node);
      int32_t next;
      if (t < h.t) {  // the new element takes the node, the old one moves down
        hn_set_key(M, node, t, ev, blk);
        t = h.t;
        ev = h.ev;
        blk = h.blk;
        next = h.l;
      } else {  // children swapped, then down the (new) left
        hn_set_lr(M, node, h.r, h.l);
        next = h.r;
      }
      parent = node;
      node = next;
    }
  }
  __host__ __device__ inline bool pop(const BkMem& M, double* t, uint32_t* ev, int32_t* blk) {
    if (hroot < 0) return false;
    HNode cur = hn_get(M, hroot);
    *t = cur.t;
    *ev = cur.ev;
    *blk = cur.blk;
    int32_t parent = -1, side = 0, node = hroot;
    for (;;) {
      CPR_BK_COST(BC_POP);
      const int32_t l = cur.l, r = cur.r;
      int32_t repl = -2;
      if (r < 0)
        repl = l;
      else if (l < 0)
        repl = r;
      if (repl != -2) {
        if (parent < 0)
          hroot = repl;
        else if (side == 0)
          hn_set_l(M, parent, repl);
        else
          hn_set_r(M, parent, repl);
        hrelease(M, node);
        return true;
      }
      const HNode hl_ = hn_get(M, l), hr_ = hn_get(M, r);
      const bool left = hl_.t <= hr_.t;
      cur = left ? hl_ : hr_;
      hn_set_key(M, node, cur.t, cur.ev, cur.blk);
      parent = node;
      side = left ? 0 : 1;
      node = left ? l : r;
    }
  }
  __host__ __device__ inline void push_now(const BkParams& P, const BkMem& M, uint32_t ev,
                                           int32_t blk) {
    push(P, M, now, ev, blk);
  }

  // ------------------------------------------------------------------ randomness
  template <class St>
  __host__ __device__ inline int32_t miner_of(const BkParams& P, const St& S, int32_t j) {
    if (P.net == 2) return S.miner_w((uint32_t)j, P.thr, P.n - 1);
    return S.miner((uint32_t)j, P.t_att, P.d);
  }
  template <class St>
  __host__ __device__ inline void schedule_pow(const BkParams& P, const St& S,
                                               const BkMem& M) {
    push(P, M, now + S.clock((uint32_t)c_act, P.ev), mkev(EV_CLOCK, 0, KD_POW), -1);
  }

  // ------------------------------------------------------------------ DAG
  __host__ __device__ inline void init_vertex(const BkParams& P, const BkMem& M, BVtx& b,
                                              int32_t s) {
    b.serial = s;
    b.nconf = 0;
    b.qslot = -1;
    b.time = now;
    VH(P, M, s) = -1;
    VR(P, M, s).x = -1;
    VR(P, M, s).w = -1;
    for (int32_t j = 0; j < P.n; ++j) Vs(P, M, s, j, V_INV);
  }
  // vote: simulator.ml:122-136 (pow = (bits, serial)), bk.ml:281-286 payload
  template <class St>
  __host__ __device__ inline int32_t append_vote(const BkParams& P, const St& S,
                                                 const BkMem& M, int32_t node, int32_t parent) {
    BVtx& p = X(P, M, parent);
    const int32_t s = ++newest;
    BVtx& b = bk_vtx(P, M, s);
    init_vertex(P, M, b, s);
    b.parent = parent;
    b.height = p.height;
    b.vote = 1;
    b.who = node;
    b.pow = S.pow((uint32_t)s);
    b.rew_att = p.rew_att;  // precursor = the block; votes carry no reward (bk.ml:151-176)
    b.rew_def = p.rew_def;
    p.nconf += 1;
    int4& r = VR(P, M, s);
    r.x = VH(P, M, parent);
    r.y = b.pow;
    r.z = node;
    VH(P, M, parent) = s;
    return s;
  }
  // block from an Append draft (bk.ml:288-295), set_rewards (simulator.ml:377-388)
  __host__ __device__ inline int32_t append_block(const BkParams& P, const BkMem& M,
                                                  int32_t node, int32_t dseq_) {
    const int32_t* dr = M.drafts + (int64_t)(dseq_ & (P.cap_d - 1)) * (P.k + 2);
    if (dr[0] != dseq_) {
      fail(4);
      return 0;
    }
    // guard (not in the reference): in loop mode an attacker policy that keeps adopting
    // re-proposes on the same block at the same instant forever (Simulator.loop has no
    // step bound); stop such a lane after 4096 appends without an activation
    if (P.mode == 1 && ++zt > 4096) {
      fail(8);
      return 0;
    }
    BVtx& p = X(P, M, dr[1]);
    int32_t ra = p.rew_att, rd = p.rew_def;
    const int32_t ph = p.height;
    const int32_t s = ++newest;
    const int32_t qs = nblk++;
    int32_t* q = M.quo + (int64_t)(qs & (P.cap_q - 1)) * (P.k + 1);
    q[0] = s;
    for (int32_t i = 0; i < P.k; ++i) {
      const int32_t v = dr[2 + i];
      q[1 + i] = v;
      if (P.scheme == 0) {  // Constant: 1 per confirmed vote to its miner
        if (X(P, M, v).who == 0)
          ++ra;
        else
          ++rd;
      }
    }
    if (P.scheme != 0) {  // Block: k to the signer
      if (node == 0)
        ra += P.k;
      else
        rd += P.k;
    }
    if (M.nrew) {  // set_rewards per node: the precursor block's array plus this block's
      int32_t* br = M.nrew + (int64_t)(qs & (P.cap_q - 1)) * P.n;
      const int32_t* pr = p.qslot < 0 ? nullptr : M.nrew + (int64_t)(p.qslot & (P.cap_q - 1)) * P.n;
      for (int32_t j = 0; j < P.n; ++j) br[j] = pr ? pr[j] : 0;
      if (P.scheme == 0)
        for (int32_t i = 0; i < P.k; ++i) br[X(P, M, dr[2 + i]).who] += 1;
      else
        br[node] += P.k;
    }
    BVtx& b = bk_vtx(P, M, s);
    init_vertex(P, M, b, s);
    for (int32_t j = 0; j < P.n; ++j) VC(P, M, s, j) = 0;
    b.parent = dr[1];
    {  // newest-first child-block list of the parent
      int4& pr = VR(P, M, dr[1]);
      VR(P, M, s).x = pr.w;
      pr.w = s;
    }
    b.height = ph + 1;
    b.vote = 0;
    b.who = node;
    b.pow = 0;
    b.rew_att = ra;
    b.rew_def = rd;
    b.qslot = qs;
    return s;
  }

  // ------------------------------------------------------------------ honest node views
  // pow hashes (bits, serial) as one ordered key; max_pow = all ones
  __host__ __device__ static inline uint64_t pow_key(const BVtx& v) {
    return ((uint64_t)(uint32_t)v.pow << 32) | (uint32_t)v.serial;
  }
  // Honest.leader_hash_exn (bk.ml:205-215): the block's first quorum vote
  __host__ __device__ inline uint64_t leader_key(const BkParams& P, const BkMem& M, int32_t b) {
    const BVtx& x = X(P, M, b);
    if (x.parent < 0) return ~0ull;
    return pow_key(X(P, M, Q(P, M, x)[0]));
  }
  // confirming votes of block b visible at `node` that pass `vf` (children scan, newest
  // first: only vertices appended after b can be its children)
  // (the count of b's visible votes the children scan would find, from b's counters)
  __host__ __device__ inline int32_t confirming(const BkParams& P, const BkMem& M, int32_t b,
                                                int32_t node, int32_t vf) {
    CPR_BK_COST(BC_CONFIRMING_CALLS);
    return vc_count(VC(P, M, b, node), vf);
  }
  // bk.ml:217-226 (skip_eq; by height; by #votes; by neg leader hash; by neg visible_since)
  __host__ __device__ inline int32_t compare_blocks(const BkParams& P, const BkMem& M,
                                                    int32_t node, int32_t vf, int32_t a,
                                                    int32_t b) {
    if (a == b) return 0;
    const int32_t ha = X(P, M, a).height, hb = X(P, M, b).height;
    if (ha != hb) return ha < hb ? -1 : 1;
    const int32_t ca = confirming(P, M, a, node, vf), cb = confirming(P, M, b, node, vf);
    if (ca != cb) return ca < cb ? -1 : 1;
    const uint64_t la = leader_key(P, M, a), lb = leader_key(P, M, b);
    if (la != lb) return lb < la ? -1 : 1;
    const double ta = VT(P, M, a, node), tb = VT(P, M, b, node);
    return tb < ta ? -1 : (tb > ta ? 1 : 0);
  }
  __host__ __device__ inline int32_t update_head(const BkParams& P, const BkMem& M,
                                                 int32_t node, int32_t vf, int32_t old,
                                                 int32_t cand) {
    return compare_blocks(P, M, node, vf, cand, old) > 0 ? cand : old;
  }

  // Honest.quorum + propose (bk.ml:233-295) at `node`; returns the draft sequence number
  // (written to the draft ring) or -1
  __host__ __device__ inline int32_t propose(const BkParams& P, const BkMem& M, int32_t node,
                                             int32_t vf, int32_t b) {
    uint64_t* mk = M.skey;        // mine: keys / serials, scan order (newest first)
    int32_t* mv = M.sval;
    uint64_t* tk = M.skey + NQS;  // theirs
    int32_t* tv = M.sval + NQS;
    int32_t nmine = 0, ntheirs = 0;
    uint64_t my_hash = ~0ull;
    CPR_BK_COST(BC_PROPOSE_CALLS);
    {
      // the scan's outcome when it would not draft, from b's counters: a node's own votes
      // are exactly those it holds withheld or released (V_WH / V_REL), the others received
      const uint64_t cv = VC(P, M, b, node);
      const int32_t rl = vc_field(cv, V_REL), wh = vc_field(cv, V_WH), rc = vc_field(cv, V_RECV);
      const int32_t nm = rl + (vf != VF_PUBLIC ? wh : 0), nt = vf != VF_MINE ? rc : 0;
      if (nm > NQS || nt > NQS) {  // the scan overflows a candidate list
        fail(3);
        return -1;
      }
      if (dead || nm == 0 || nm + nt < P.k) return -1;  // fast path (bk.ml:254)
    }
    for (int32_t c = VH(P, M, b); c >= 0 && !dead;) {  // b's votes, newest first
      CPR_BK_COST(BC_PROPOSE);
      const int4 r = VR(P, M, c);  // (next, pow, who): pow_key without the vertex
      const int32_t cn = r.x;
      const uint8_t v = Vg(P, M, c, node);
      if ((v & V_KIND) == V_INV || !keep(v, vf)) {
        c = cn;
        continue;
      }
      const uint64_t key = ((uint64_t)(uint32_t)r.y << 32) | (uint32_t)c;
      if (r.z == node) {
        if (nmine >= NQS) {
          fail(3);
          return -1;
        }
        my_hash = key < my_hash ? key : my_hash;
        mk[nmine] = key;
        mv[nmine++] = c;
      } else {
        if (ntheirs >= NQS) {
          fail(3);
          return -1;
        }
        tk[ntheirs] = key;
        tv[ntheirs++] = c;
      }
      c = cn;
    }
    if (dead || nmine == 0 || nmine + ntheirs < P.k) return -1;  // fast path (bk.ml:254)
    const int32_t seq = dseq++;
    int32_t* dr = M.drafts + (int64_t)(seq & (P.cap_d - 1)) * (P.k + 2);
    dr[0] = seq;
    dr[1] = b;
    int32_t* q = dr + 2;
    int32_t nq = 0;
    if (nmine >= P.k) {
      // Compare.first (by compare_pow) k mine: the k smallest hashes (unique keys)
      for (int32_t i = 0; i < nmine; ++i) {
        int32_t rank = 0;
        for (int32_t j = 0; j < nmine; ++j) rank += mk[j] < mk[i] ? 1 : 0;
        if (rank < P.k) q[rank] = mv[i];
      }
      return seq;
    }
    // theirs with hash > my_hash, in children order (the list rebuilt by two prepending
    // folds keeps it), then the k - nmine earliest visible by Array.sort on visible_since
    int32_t n2 = 0;
    for (int32_t i = 0; i < ntheirs; ++i) {
      if (tk[i] > my_hash) {
        tv[n2] = tv[i];
        tk[n2] = time_key(VT(P, M, tv[i], node));
        ++n2;
      }
    }
    if (n2 < P.k - nmine) {
      dseq--;  // no draft after all
      return -1;
    }
    ocaml_heap_sort64(tv, tk, n2);
    // mine @ first (k - nmine) theirs, then List.sort by pow hash (unique keys)
    for (int32_t i = 0; i < nmine; ++i) q[nq++] = mv[i];
    for (int32_t i = 0; i < P.k - nmine; ++i) q[nq++] = tv[i];
    for (int32_t i = 1; i < nq; ++i) {
      const int32_t s = q[i];
      const uint64_t ks = pow_key(X(P, M, s));
      int32_t j = i;
      while (j > 0 && pow_key(X(P, M, q[j - 1])) > ks) {
        q[j] = q[j - 1];
        --j;
      }
      q[j] = s;
    }
    return seq;
  }

  // ------------------------------------------------------------------ actions
  // Simulator.handle_action share part (simulator.ml:401-419): recursive release of
  // withheld vertices, parents in order (block: parent block, then its quorum)
  __host__ __device__ inline void share(const BkParams& P, const BkMem& M, int32_t node,
                                        int32_t s0) {
    int32_t* st = M.stack;
    int32_t sp = 0;
    st[sp++] = s0;
    while (sp > 0 && !dead) {
      const int32_t s = st[--sp];
      const uint8_t v = Vg(P, M, s, node);
      if ((v & V_KIND) != V_WH) continue;  // received / released: nothing
      Vs(P, M, s, node, (uint8_t)((v & ~V_KIND) | V_REL));
      push_now(P, M, mkev(EV_TX, node, KD_NET), s);
      const BVtx& b = X(P, M, s);
      if (b.vote) {  // WH -> REL in the block's counts (X: the block is still in the ring)
        X(P, M, b.parent);
        VC(P, M, b.parent, node) += (1ull << 16) - (1ull << 32);
      }
      if (b.parent < 0) continue;
      const int32_t np = b.vote ? 1 : P.k + 1;
      if (sp + np > NSTACK) {
        fail(5);
        return;
      }
      if (!b.vote) {
        const int32_t* q = Q(P, M, b);
        for (int32_t i = P.k - 1; i >= 0; --i) st[sp++] = q[i];
      }
      st[sp++] = b.parent;
    }
  }

  // ------------------------------------------------------------------ agent (bk_ssz.ml)
  __host__ __device__ inline void agent_init(int32_t root) {
    pub = priv = root;
    pending = -1;
  }
  __host__ __device__ inline int32_t last_block(const BkParams& P, const BkMem& M, int32_t x) {
    const BVtx& b = X(P, M, x);
    return b.vote ? b.parent : x;
  }
  // bk_ssz.ml:196-221; the pending share list is [block; votes of block], whose
  // last_blocks all equal `block`, so folding update_head over it equals one update
  __host__ __device__ inline void prepare(const BkParams& P, const BkMem& M, uint32_t kind,
                                          int32_t x) {
    int32_t p = pub;
    if (pending >= 0) p = update_head(P, M, 0, VF_PUBLIC, p, pending);
    int32_t q = priv;
    if (kind == KD_APP) {
      q = x;
      o_event = 0;
    } else if (kind == KD_POW) {
      o_event = 1;
    } else {
      p = update_head(P, M, 0, VF_PUBLIC, p, last_block(P, M, x));
      o_event = 2;
    }
    o_pub = p;
    o_priv = q;
    // Dagtools.common_ancestor over the vertex DAG; its last_block is the deepest common
    // block of the two block chains
    int32_t a = p, b = q;
    while (a != b && !dead) {
      const int32_t ha = X(P, M, a).height, hb = X(P, M, b).height;
      if (ha >= hb) a = X(P, M, a).parent;
      if (hb >= ha) b = X(P, M, b).parent;
      if (a < 0 || b < 0) {
        fail(1);
        break;
      }
    }
    o_common = a;
  }
  // bk_ssz.ml:225-263
  __host__ __device__ inline BkObs observe(const BkParams& P, const BkMem& M) {
    BkObs o;
    const int32_t ca = X(P, M, o_common).height;
    const int32_t ph = X(P, M, o_priv).height, qh = X(P, M, o_pub).height;
    o.public_blocks = qh - ca;
    o.private_blocks = ph - ca;
    o.diff_blocks = ph - qh;
    o.public_votes = confirming(P, M, o_pub, 0, VF_PUBLIC);
    const uint64_t cv = VC(P, M, o_priv, 0);
    o.private_votes_inclusive = vc_count(cv, VF_ALL);
    o.private_votes_exclusive = vc_count(cv, VF_MINE);
    // `lead` compares the signature of the lowest-hash vote with my_id; votes are never
    // signed (bk.ml:281-286), so it is always false in the reference
    o.lead = 0;
    o.event = o_event;
    return o;
  }
  // bk_ssz.ml:265-331 (share + append through handle_action order: shares, then appends)
  __host__ __device__ inline void apply(const BkParams& P, const BkMem& M, int32_t action) {
    const int32_t kind = action & 3;  // 0 Adopt, 1 Override, 2 Match, 3 Wait
    int32_t np = kind == 0 ? o_pub : o_priv;
    int32_t rel = -1;
    if (kind == 1 || kind == 2) {
      int32_t height = X(P, M, o_pub).height;
      int32_t nvotes = confirming(P, M, o_pub, 0, VF_PUBLIC);
      if (kind == 1) {
        if (nvotes >= P.k) {
          height += 1;
          nvotes = 0;
        } else {
          nvotes += 1;
        }
      }
      int32_t block = o_priv;
      while (!dead && X(P, M, block).height > height) block = X(P, M, block).parent;
      if (nvotes >= P.k) {
        // newest visible child block (the attacker's proposal, if any): the block's
        // newest-first child-block list instead of every vertex appended since
        for (int32_t c = VR(P, M, block).w; c >= 0 && !dead; c = VR(P, M, c).x) {
          if (!visible(P, M, c, 0)) continue;
          block = c;
          nvotes = 0;
          break;
        }
      }
      // votes confirming `block` in children order; Compare.first by visible_since
      uint64_t* vk = M.skey;
      int32_t* vv = M.sval;
      int32_t nv = 0;
      for (int32_t c = VH(P, M, block); c >= 0 && !dead;) {  // block's votes
        CPR_BK_COST(BC_APPLY);
        const int32_t cn = VN(P, M, c);
        if (!visible(P, M, c, 0)) {
          c = cn;
          continue;
        }
        if (nv >= 2 * NQS) {
          fail(3);
          break;
        }
        vk[nv] = time_key(VT(P, M, c, 0));
        vv[nv++] = c;
        c = cn;
      }
      int32_t take = nv;
      if (nv >= nvotes) {
        ocaml_heap_sort64(vv, vk, nv);
        take = nvotes;
      }
      share(P, M, 0, block);
      // share() reuses no scratch, so vv survives
      for (int32_t i = 0; i < take && !dead; ++i) share(P, M, 0, vv[i]);
      rel = block;
    }
    const int32_t d = propose(P, M, 0, action >= 4 ? VF_ALL : VF_MINE, np);
    if (d >= 0) push_now(P, M, mkev(EV_DAG, 0, KD_APP), d);
    pub = o_pub;
    priv = np;
    pending = rel;
  }

  // ------------------------------------------------------------------ engine
  template <class St>
  __host__ __device__ inline void init(const BkParams& P, const St& S, const BkMem& M) {
    now = 0.0;
    nrand = 0;
    c_act = 0;
    newest = 0;
    nblk = 0;
    act0 = 0;
    hroot = -1;
    hfree = -1;
    hfree2 = -1;
    hused = 0;
    status = 0u;
    dead = 0;
    dseq = 0;
    zt = 0;
    steps = 0;
    BVtx& r = bk_vtx(P, M, 0);
    r.serial = 0;
    r.parent = -1;
    r.height = 0;
    r.vote = 0;
    r.who = -1;
    r.pow = 0;
    r.rew_att = r.rew_def = 0;
    r.nconf = 0;
    r.qslot = -1;
    r.time = 0.0;
    VH(P, M, 0) = -1;
    VR(P, M, 0).x = -1;
    VR(P, M, 0).w = -1;
    for (int32_t j = 0; j < P.n; ++j) {
      VC(P, M, 0, j) = 0;
      Vs(P, M, 0, j, V_RECV | V_GOT);
      VT(P, M, 0, j) = 0.0;
      M.tips[j] = 0;
      if (M.nact) M.nact[j] = 0;
    }
    agent_init(0);
    schedule_pow(P, S, M);
  }

  // Honest.handler (bk.ml:297-310) at defender `node` for vertex x
  __host__ __device__ inline void honest(const BkParams& P, const BkMem& M, int32_t node,
                                         int32_t x) {
    const int32_t b = last_block(P, M, x);
    const int32_t d = propose(P, M, node, VF_ALL, b);
    if ((Vg(P, M, x, node) & V_KIND) == V_WH) share(P, M, node, x);
    M.tips[node] = update_head(P, M, node, VF_ALL, M.tips[node], b);
    if (d >= 0) push_now(P, M, mkev(EV_DAG, node, KD_APP), d);
  }

  // one popped event that is not the attacker's gym interaction (simulator.ml:421-508)
  template <class St>
  __host__ __device__ inline void handle(const BkParams& P, const St& S, const BkMem& M,
                                         uint32_t ev, int32_t s) {
    const uint32_t ty = ev & 7u, kind = (ev >> 3) & 3u;
    const int32_t node = (int32_t)(ev >> 5);
    CPR_BK_COST(BC_EVENT + (int32_t)ty);
    switch (ty) {
      case EV_MV: {
        const uint8_t v = Vg(P, M, s, node);
        if ((v & V_KIND) != V_INV) break;
        const BVtx& b = X(P, M, s);
        bool ok = b.parent < 0 || visible(P, M, b.parent, node);
        if (ok && !b.vote) {
          const int32_t* q = Q(P, M, b);
          for (int32_t i = 0; i < P.k && ok; ++i) ok = visible(P, M, q[i], node);
        }
        if (!ok) break;
        const uint8_t nk = kind == KD_NET ? V_RECV : V_WH;
        Vs(P, M, s, node, (uint8_t)((v & ~V_KIND) | nk));
        if (b.vote) {  // X: the counts' block is still in the ring
          X(P, M, b.parent);
          VC(P, M, b.parent, node) += 1ull << (16 * (nk - 1));
        }
        VT(P, M, s, node) = now;
        push_now(P, M, mkev(EV_ON, node, kind), s);
        push_now(P, M, mkev(EV_MDV, node, kind), s);
        break;
      }
      case EV_ON: {
        if (node == 0 && P.net != 2) {
          // loop mode: the attacker node's handler (bk_ssz.ml:334-343)
          prepare(P, M, kind, s);
          apply(P, M, P.policy == BK_POLICY_RANDOM ? S.rand_act((uint32_t)nrand++, 8u)
                                                   : bk_policy(P, observe(P, M)));
          break;
        }
        honest(P, M, node, s);
        break;
      }
      case EV_CLOCK: {
        zt = 0;
        const int32_t m = miner_of(P, S, c_act);
        int32_t parent;
        if (m == 0 && P.net != 2) {
          ++act0;
          parent = priv;  // gym: replaced at the Dag event (engine.ml:112-116)
        } else {
          parent = M.tips[m];
        }
        push_now(P, M, mkev(EV_DAG, m, KD_POW), parent);
        if (M.nact) ++M.nact[m];
        ++c_act;
        schedule_pow(P, S, M);
        break;
      }
      case EV_DAG: {
        const int32_t v = kind == KD_POW ? append_vote(P, S, M, node, s)
                                         : append_block(P, M, node, s);
        push_now(P, M, mkev(EV_MV, node, kind), v);
        break;
      }
      case EV_TX: {
        for (int32_t dst = 0; dst < P.n; ++dst) {
          if (dst == node) continue;
          double delay;
          if (P.net == 2)  // models.ml:4 uniform propagation delays on every link
            delay = S.msg_unif((uint32_t)s, (uint32_t)dst, P.lo, P.hi);
          else if (P.net == 3)  // cpr_protocols.ml:481-483 exponential delays on every link
            delay = S.msg_exp((uint32_t)s, (uint32_t)dst, P.delta);
          else if (P.net == 1)
            delay = 0.0;
          else if (node == 0)
            delay = S.msg((uint32_t)s, (uint32_t)dst, P.dmax);
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
        const uint8_t v = Vg(P, M, s, node);
        if (!(v & V_GOT)) {
          Vs(P, M, s, node, (uint8_t)(v | V_GOT));
          push_now(P, M, mkev(EV_MV, node, KD_NET), s);
        }
        break;
      }
      case EV_MDV: {
        // children (newest first) already received at this node become visible: votes and
        // blocks on block s, or blocks whose quorum holds vote s
        const bool is_vote = X(P, M, s).vote != 0;
        for (int32_t c = newest; c > s && !dead; --c) {
          CPR_BK_COST(BC_MDV);
          if (!(Vg(P, M, c, node) & V_GOT)) continue;
          const BVtx& cb = X(P, M, c);
          bool child = cb.parent == s;
          if (!child && is_vote && !cb.vote) {
            const int32_t* q = Q(P, M, cb);
            for (int32_t i = 0; i < P.k; ++i) child |= q[i] == s;
          }
          if (child) push_now(P, M, mkev(EV_MV, node, KD_NET), c);
        }
        break;
      }
    }
  }

  // engine.ml:108-121
  template <class St>
  __host__ __device__ inline bool skip_to_interaction(const BkParams& P, const St& S,
                                                      const BkMem& M, uint32_t* kind,
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
      const uint32_t kd = (ev >> 3) & 3u;
      if (ty == EV_ON && node == 0) {
        *kind = kd;
        *blk = s;
        return true;
      }
      if (ty == EV_DAG && node == 0 && kd == KD_POW) {
        const int32_t v = append_vote(P, S, M, 0, priv);
        push_now(P, M, mkev(EV_MV, 0, KD_POW), v);
        continue;
      }
      handle(P, S, M, ev, s);
    }
    return false;
  }

  // Referee.winner over [attacker preference; defenders' tips] (bk.ml:134-147): height,
  // then confirming votes in the global view
  __host__ __device__ inline int32_t head(const BkParams& P, const BkMem& M, int32_t att) {
    int32_t h = att;
    int32_t hh = X(P, M, att).height, hc = X(P, M, att).nconf;
    for (int32_t j = 1; j < P.n; ++j) {
      const int32_t t = M.tips[j];
      if (t == h) continue;
      const BVtx& x = X(P, M, t);
      if (x.height > hh || (x.height == hh && x.nconf > hc)) {
        h = t;
        hh = x.height;
        hc = x.nconf;
      }
    }
    return h;
  }

  // gym: reset (engine.ml:122-170)
  template <class St>
  __host__ __device__ inline void gym_reset(const BkParams& P, const St& S, const BkMem& M) {
    init(P, S, M);
    uint32_t kind;
    int32_t b;
    if (skip_to_interaction(P, S, M, &kind, &b)) prepare(P, M, kind, b);
  }

  // gym: step (engine.ml:176-249); returns the head, sets *done
  template <class St>
  __host__ __device__ inline int32_t gym_step(const BkParams& P, const St& S,
                                              const BkMem& M, int32_t action, bool* done) {
    apply(P, M, action);
    ++steps;
    uint32_t kind;
    int32_t b;
    const int32_t att = priv;
    if (skip_to_interaction(P, S, M, &kind, &b)) prepare(P, M, kind, b);
    const int32_t hd = head(P, M, att);
    const double progress = (double)(X(P, M, hd).height * P.k);
    *done = dead || !(steps < P.max_steps && progress < P.max_progress && now < P.max_time);
    return hd;
  }

  // loop: Simulator.loop ~activations (simulator.ml:519-533), then the head
  template <class St>
  __host__ __device__ inline int32_t loop(const BkParams& P, const St& S, const BkMem& M) {
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

}  // namespace bk
}  // namespace cpr
