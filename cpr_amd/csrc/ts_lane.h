// Tailstorm (tailstorm.ml) with the tailstorm_ssz attack space: one episode per lane, as an
// exact per-lane discrete-event engine (same skeleton as bk_lane.h).
//
// Tailstorm's votes form a tree under each summary; summaries are PoW-less, unsigned and
// deterministic, so identical summaries appended by different nodes are deduplicated
// (simulator.ml:139-159). Quorum selection (altruistic / heuristic / optimal,
// tailstorm.ml:271-507) walks vote branches, the attacker's release walks the descendants
// of the common ancestor in (DAG depth, serial) order (tailstorm_ssz.ml:292-314), and the
// head is Compare.first over a heap sort (tailstorm.ml:191-194). The lane keeps per vote
// its summary (last_summary) and parent, so a summary's vote tree is the set of votes whose
// summary field names it, scanned from the vertex ring.
//
// Per-lane memory (one contiguous region per lane):
//   vtx    [cap_v] x 64 B    vertex ring indexed by serial & (cap_v-1)
//   vis    [cap_v][n] u8     per node: kind + got bit;  vt [cap_v][n] f64 visible_since
//   quo    [cap_q][k+1] i32  summary quorums: tag (serial), leaves sorted by
//                            compare_votes_in_block
//   srew   [cap_q][2n] f64   per summary: cumulative rewards per node (set_rewards order),
//                            and its own reward list summed per node (compare_blocks)
//   drafts [cap_d][k+2] i32  outstanding summary drafts (tag, #leaves, leaves)
//   heap   [cap_e] x 24 B    event queue (skew heap, +inf events kept)
//   tips [n] i32, pend [cap_v] i32 (pending released messages), marks [cap_v] u8,
//   shead [cap_v] i32 (per summary: newest child summary), tree scratch [cap_v] each
//
// Tree bookkeeping is incremental: every summary heads a newest-first list of its votes
// (TVtx.thead / TVtx.next) and of its child summaries (shead / TVtx.next), so the tree
// scans (count_post, tree, payload_parent, has_children, MadeVisible children, summary
// dedup) cost the tree's size, not every vertex appended since the summary, and the
// scratch holds a whole ring window: no tree size is capped below the vertex ring.
//
// Reference map: simulator.ml:122-543, tailstorm.ml:86-609, tailstorm_ssz.ml:162-446,
// combinatorics.ml:5-32, engine.ml:97-249.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bk_lane.h"  // HNode, ocaml_heap_sort64, event/kind/visibility enums, time_key
#include "cpr_stream.h"

#pragma clang fp contract(off)

namespace cpr {
namespace ts {

using bk::HNode;
using bk::mkev;
using bk::ocaml_heap_sort64;
using bk::time_key;
constexpr uint32_t EV_CLOCK = bk::EV_CLOCK, EV_DAG = bk::EV_DAG, EV_TX = bk::EV_TX,
                   EV_RX = bk::EV_RX, EV_ON = bk::EV_ON, EV_MV = bk::EV_MV, EV_MDV = bk::EV_MDV;
constexpr uint32_t KD_APP = bk::KD_APP, KD_POW = bk::KD_POW, KD_NET = bk::KD_NET;
constexpr uint8_t V_INV = bk::V_INV, V_RECV = bk::V_RECV, V_REL = bk::V_REL, V_WH = bk::V_WH,
                  V_KIND = bk::V_KIND, V_GOT = bk::V_GOT;

constexpr uint32_t TST_CAPACITY = 32u;   // CPR_ST_CAPACITY
constexpr uint32_t TST_REF_RAISES = 64u; // CPR_ST_REFERENCE_RAISES

// vote filters: all, Honest.appended_by_me, public_visibility, public or in the release set
enum : int32_t { VF_ALL = 0, VF_MINE = 1, VF_PUBLIC = 2, VF_PUBLIC_OR_MARKED = 3 };
// incentive schemes (tailstorm.ml:3,221-227), ids as in cpr_reward_scheme
enum : int32_t { SC_CONSTANT = 0, SC_DISCOUNT = 1, SC_PUNISH = 3, SC_HYBRID = 4 };
enum : int32_t { SEL_ALTRUISTIC = 0, SEL_HEURISTIC = 1, SEL_OPTIMAL = 2 };

struct TVtx {
  int32_t serial;
  int32_t parent;  // vote: its parent; summary: leaves[0] (precursor); genesis -1
  int32_t height;
  int32_t vote;    // 1 Vote, 0 Summary
  int32_t who;     // vote miner; -1 summaries
  int32_t depth;   // vote data depth; 0 summaries
  int32_t pow;     // 30-bit hash bits (votes)
  int32_t ddepth;  // Dag depth (dag.ml:28-35)
  int32_t sum;     // vote: last_summary; summary: itself
  int32_t nconf;   // summary: votes in its tree, global view (Referee.compare_summaries)
  int32_t qslot;   // summary: quorum / reward slot; -1 genesis
  int32_t nq;      // summary: number of leaves
  double time;     // Simulator.timestamp = append time
  int32_t next;    // vote: next older vote of the same tree; summary: next older summary
                   // with the same parent summary (-1 ends either list)
  int32_t thead;   // summary: newest vote of its tree (-1 none)
};
static_assert(sizeof(TVtx) == 64, "TVtx layout");

// optimal quorum: prefixes the search visits before it flags the episode (the oracle's
// TS_BRUTE_FORCE_BUDGET); TsParams.opt_budget, lowered only by the host fuzzer
constexpr int64_t TS_OPT_BUDGET = 100000;

struct TsParams {
  uint64_t t_att;
  int32_t d, n, net, mode;
  int32_t policy, scheme, selection, k;
  int32_t cap_v, cap_q, cap_e, cap_d;
  double ev, delta, dmax;
  int64_t max_steps, activations;
  double max_progress, max_time;
  // honest clique (net 2, models.ml:3-28): keyed miner thresholds (n - 1), U(lo, hi) links
  double lo, hi;
  uint32_t thr[64];
  // table-driven policy (policy == TS_POLICY_TABLE): device table, dimension D
  const uint8_t* table;
  int32_t table_dim;
  // fused-episode launches: device counter of episodes handed out beyond the first
  // lanes-many (zeroed before the launch); null = static grid-stride
  unsigned long long* next = nullptr;
  int64_t opt_budget = TS_OPT_BUDGET;
};

constexpr int32_t NFR = 64;      // common-ancestor frontier (reference walk, tests only)

// the list view of a vertex slot, beside the 64-byte vertices (TsMem.trec): the walks over a
// summary's vote list and child-summary list (tree, count_post, observe, payload_parent,
// has_children, MadeDescendantsVisible) read these 16 bytes and the visibility byte instead
// of a whole vertex. Written once when the vertex is appended (the fields never change).
struct TRec {
  int32_t next;    // TVtx.next
  int32_t depth;   // TVtx.depth (< cap_v <= 4096) | TVtx.who << 16
  int32_t pow;     // TVtx.pow
  int32_t parent;  // TVtx.parent
  __host__ __device__ inline int32_t dep() const { return depth & 0xffff; }
  __host__ __device__ inline int32_t who() const { return depth >> 16; }
};
static_assert(sizeof(TRec) == 16, "TRec layout");

struct TsMem {
  // event-heap nodes 0 .. kl-1 in the workgroup's LDS slab (node-major, stride hs), the
  // rest in HBM (heap); see bk_lane.h BkMem
  CPR_LDS HNode* hl = nullptr;
  int32_t kl = 0, hs = 1;
  // visibility rows of the newest vw vertices in the same slab (see bk_lane.h BkMem.vl)
  CPR_LDS uint8_t* vl = nullptr;
  int32_t vw = 0;
  // list records (TRec) of the newest tw vertices in the same slab, row-major with stride hs
  // (a copy: set_trec writes both, the ring stays complete). configs[3]'s walks read the
  // newest 8 / 16 / 32 vertices in 76-82 / 97-99 / 99.3-99.9 % of their list reads
  // (tools/ts_window_study.cpp)
  CPR_LDS TRec* tl = nullptr;
  int32_t tw = 0;
  TVtx* vtx;
  TRec* trec;
  uint8_t* vis;
  double* vt;
  int32_t* quo;
  double* srew;
  int32_t* drafts;
  HNode* heap;
  int32_t* tips;
  int32_t* pend;
  uint8_t* marks;   // [cap_v]
  int32_t* shead;   // [cap_v] per summary slot: newest child summary
  int32_t* pos;     // [cap_v] per vertex slot: index in cand while a tree is held
  int32_t* cand;    // [cap_v] tree votes, ascending serial
  int32_t* perm;    // [cap_v] indices into cand in BlockSet order (Dag depth, serial)
  int32_t* aux;     // [cap_v] scratch indices
  uint8_t* flag;    // [cap_v]
  uint8_t* flag2;   // [cap_v]
  uint64_t* key;    // [cap_v] sort keys / merge-sort buffer
  int32_t* stack;   // [2 cap_v]
  int32_t* fr;      // [4 * NFR] two frontiers of (ddepth, serial)
  int64_t* nact = nullptr;  // per-node activations (cpr_node_outputs), else null
};

__host__ __device__ inline int64_t ts_align(int64_t x) { return (x + 127) / 128 * 128; }

__host__ __device__ inline int64_t ts_lane_bytes(const TsParams& P) {
  return ts_align((int64_t)P.cap_v * 64) + ts_align((int64_t)P.cap_v * 16) +
         ts_align((int64_t)P.cap_v * P.n) +
         ts_align((int64_t)P.cap_v * P.n * 8) + ts_align((int64_t)P.cap_q * (P.k + 1) * 4) +
         ts_align((int64_t)P.cap_q * 2 * P.n * 8) + ts_align((int64_t)P.cap_d * (P.k + 2) * 4) +
         ts_align((int64_t)P.cap_e * 24) + ts_align((int64_t)P.n * 4) +
         ts_align((int64_t)P.cap_v * 4) + ts_align(P.cap_v) + 5 * ts_align((int64_t)P.cap_v * 4) +
         2 * ts_align(P.cap_v) + ts_align((int64_t)P.cap_v * 8) +
         ts_align((int64_t)P.cap_v * 8) + ts_align(4 * NFR * 4);
}

__host__ __device__ inline TsMem ts_mem_at(uint8_t* base, const TsParams& P) {
  TsMem M;
  int64_t o = 0;
  auto take = [&](int64_t bytes) {
    uint8_t* p = base + o;
    o += ts_align(bytes);
    return p;
  };
  M.vtx = (TVtx*)take((int64_t)P.cap_v * 64);
  M.trec = (TRec*)take((int64_t)P.cap_v * 16);
  M.vis = take((int64_t)P.cap_v * P.n);
  M.vt = (double*)take((int64_t)P.cap_v * P.n * 8);
  M.quo = (int32_t*)take((int64_t)P.cap_q * (P.k + 1) * 4);
  M.srew = (double*)take((int64_t)P.cap_q * 2 * P.n * 8);
  M.drafts = (int32_t*)take((int64_t)P.cap_d * (P.k + 2) * 4);
  M.heap = (HNode*)take((int64_t)P.cap_e * 24);
  M.tips = (int32_t*)take((int64_t)P.n * 4);
  M.pend = (int32_t*)take((int64_t)P.cap_v * 4);
  M.marks = take(P.cap_v);
  M.shead = (int32_t*)take((int64_t)P.cap_v * 4);
  M.pos = (int32_t*)take((int64_t)P.cap_v * 4);
  M.cand = (int32_t*)take((int64_t)P.cap_v * 4);
  M.perm = (int32_t*)take((int64_t)P.cap_v * 4);
  M.aux = (int32_t*)take((int64_t)P.cap_v * 4);
  M.flag = take(P.cap_v);
  M.flag2 = take(P.cap_v);
  M.key = (uint64_t*)take((int64_t)P.cap_v * 8);
  M.stack = (int32_t*)take((int64_t)P.cap_v * 8);
  M.fr = (int32_t*)take(4 * NFR * 4);
  return M;
}

// the LDS heap slab of a kernel (as bk_lane.h bk_heap_*)
__host__ __device__ inline void ts_heap_slab(TsMem& M, HNode* slab, int32_t lane, int32_t stride,
                                             int32_t kl) {
  M.hl = (CPR_LDS HNode*)(slab + lane);
  M.hs = stride;
  M.kl = kl;
}
__host__ __device__ inline void ts_vis_window(TsMem& M, uint8_t* base, int32_t lane, int32_t vw) {
  M.vl = (CPR_LDS uint8_t*)(base + lane);
  M.vw = vw;
}
__host__ __device__ inline void ts_trec_window(TsMem& M, TRec* base, int32_t lane, int32_t tw) {
  M.tl = (CPR_LDS TRec*)(base + lane);
  M.tw = tw;
}
__host__ __device__ inline void ts_vis_load(const TsMem& M, const TsParams& P, int32_t newest) {
  for (int32_t s = newest - M.vw + 1 < 0 ? 0 : newest - M.vw + 1; s <= newest; ++s)
    for (int32_t j = 0; j < P.n; ++j)
      M.vl[(int64_t)((s & (M.vw - 1)) * P.n + j) * M.hs] =
          M.vis[(int64_t)(s & (P.cap_v - 1)) * P.n + j];
}
__host__ __device__ inline void ts_heap_load(const TsMem& M, int32_t hused) {
  const int32_t n = hused < M.kl ? hused : M.kl;
  for (int32_t i = 0; i < n; ++i) M.hl[(int64_t)i * M.hs] = M.heap[i];
}
__host__ __device__ inline void ts_heap_store(const TsMem& M, int32_t hused) {
  const int32_t n = hused < M.kl ? hused : M.kl;
  for (int32_t i = 0; i < n; ++i) M.heap[i] = M.hl[(int64_t)i * M.hs];
}

// ---- observation and policies (tailstorm_ssz.ml:22-38, 365-446); Action8 ranks
struct TsObs {
  int32_t public_blocks, private_blocks, diff_blocks, public_votes, private_votes_inclusive,
      private_votes_exclusive, public_depth, private_depth_inclusive, private_depth_exclusive,
      event;  // 0 Append, 1 ProofOfWork, 2 Network
};

__host__ __device__ inline int32_t ts_policy(int32_t policy, int32_t k, const TsObs& o) {
  const int32_t h = o.public_blocks, a = o.private_blocks;
  const int32_t hp = h * k + o.public_votes, ap = a * k + o.private_votes_inclusive;
  switch (policy) {
    case 0: return h > a ? bk::A_ADOPT_PROCEED : bk::A_OVERRIDE_PROCEED;  // honest
    case 1:  // get-ahead
      return h > a ? bk::A_ADOPT_PROCEED
                   : (h < a ? bk::A_OVERRIDE_PROCEED : bk::A_WAIT_PROCEED);
    case 2:  // minor-delay
      return h > a ? bk::A_ADOPT_PROCEED
                   : (h == 0 ? bk::A_WAIT_PROCEED : bk::A_OVERRIDE_PROCEED);
    case 4:  // avoid-loss-a = avoid_loss
      if (a < h) return bk::A_ADOPT_PROCEED;
      if (h == 0) return bk::A_WAIT_PROCEED;
      if (o.private_votes_inclusive == 0 && a == h + 1) return bk::A_OVERRIDE_PROCEED;
      if (h == a && o.private_votes_inclusive == o.public_votes + 1) return bk::A_OVERRIDE_PROCEED;
      if (a - h > 10) return bk::A_OVERRIDE_PROCEED;
      return bk::A_WAIT_PROCEED;
    case 6:  // long-delay
      if (h > a) return bk::A_ADOPT_PROCEED;
      if (h == 0) return bk::A_WAIT_PROCEED;
      if (h + 10 < a) return bk::A_OVERRIDE_PROCEED;
      if (h * k + o.public_votes + 1 < a * k + o.private_votes_inclusive)
        return bk::A_WAIT_PROCEED;
      return bk::A_OVERRIDE_PROCEED;
    default:  // 3 avoid-loss = avoid_loss_alt, 5 avoid-loss-b = avoid_loss_alt2
      if (h == 0) return bk::A_WAIT_PROCEED;
      if (h == 1 && hp == ap) return policy == 3 ? bk::A_MATCH_PROCEED : bk::A_OVERRIDE_PROCEED;
      if (hp > ap) return bk::A_ADOPT_PROCEED;
      if (hp == ap - 1) return bk::A_OVERRIDE_PROCEED;
      if (h < a - 10) return bk::A_OVERRIDE_PROCEED;
      return bk::A_WAIT_PROCEED;
  }
}

// table-driven tailstorm_ssz policy (include/cpr_hip.h CPR_TS_POLICY_TABLE), the B_k
// layout: table[((((min(pub,D-1)*D + min(priv,D-1))*(k+1) + min(public_votes,k))*(k+1)
// + min(private_votes_inclusive,k))*3 + event], Action8
constexpr int32_t TS_POLICY_TABLE = 7;
// random actions (loop tasks; cpr_protocols.ml:658-782): CPR_TS_POLICY_RANDOM
constexpr int32_t TS_POLICY_RANDOM = 8;
__host__ __device__ inline int32_t ts_table_index(const TsObs& o, int32_t D, int32_t k) {
  auto cl = [](int32_t x, int32_t hi) { return x < 0 ? 0 : (x > hi ? hi : x); };
  const int32_t K1 = k + 1;
  return ((((cl(o.public_blocks, D - 1) * D + cl(o.private_blocks, D - 1)) * K1 +
            cl(o.public_votes, k)) * K1 + cl(o.private_votes_inclusive, k)) * 3) + o.event;
}
__host__ __device__ inline int32_t ts_policy_t(int32_t policy, int32_t k, const TsObs& o,
                                               const uint8_t* table, int32_t dim) {
  if (policy == TS_POLICY_TABLE) return (int32_t)table[ts_table_index(o, dim, k)];
  return ts_policy(policy, k, o);
}
__host__ __device__ inline int32_t ts_policy_p(const TsParams& P, const TsObs& o) {
  return ts_policy_t(P.policy, P.k, o, P.table, P.table_dim);
}

// combinatorics.ml:5-17 in OCaml's 63-bit wrap-around arithmetic; *dz = Division_by_zero
__host__ __device__ inline int64_t ocaml_nck(int64_t n, int64_t k, bool* dz) {
  auto fact = [](int64_t m) {
    int64_t x = 1;
    for (int64_t i = 2; i <= m; ++i) {
      uint64_t u = (uint64_t)x * (uint64_t)i;
      x = ((int64_t)(u << 1)) >> 1;
    }
    return x;
  };
  const int64_t a = fact(n), b = fact(k), c = fact(n - k);
  if (b == 0 || c == 0) {
    *dz = true;
    return 0;
  }
  return (a / b) / c;
}

// host studies only (tools/ts_window_study.cpp): the age (newest serial - s) of every vertex
// record read through X (0), TR (1) and Vg (2)
#ifndef CPR_TS_AGE
#define CPR_TS_AGE(kind, age)
#endif

struct TsLane {
  int32_t nrand;  // random-policy decisions so far (the keyed draw's index)
  double now;
  int32_t c_act, newest, nsum, act0;
  int32_t hroot, hfree, hused, hfree2;
  uint32_t status;
  int32_t dead;  // 1 vertex ring, 2 heap, 3 tree list, 4 drafts, 5 stack, 6 drained, 7 quorum
                 // ring, 8 zero-time loop, 9 pending list, 10 frontier, 11 reference raises,
                 // 12 optimal-quorum brute-force budget
  int32_t zt, dseq;
  int32_t pub, priv, npend;
  int32_t o_pub, o_priv, o_common, o_event;
  int32_t troot;  // summary whose tree cand[] holds
  int32_t tclosed;  // every tree vote's parent is troot or a tree vote (M.key parent links)
  int32_t ca_a, ca_b, ca_s;  // the last common_ancestor call (a, b) and its answer
  int64_t steps;

  // ------------------------------------------------------------------ storage
  __host__ __device__ inline void fail(int32_t why) {
    status |= why == 11 ? TST_REF_RAISES : TST_CAPACITY;
    if (!dead) dead = why;
  }
  __host__ __device__ inline TVtx& X(const TsParams& P, const TsMem& M, int32_t s) {
    CPR_TS_AGE(0, newest - s);
    TVtx& b = M.vtx[s & (P.cap_v - 1)];
    if (b.serial != s) fail(1);
    return b;
  }
  // the list view of vertex s (TRec), from the LDS window when s is among the newest tw.
  // Unchecked: the walks start from a vertex read with X, and every vertex of its lists is
  // newer, so it is in the ring whenever the start is. (No walk reads the record of a vertex
  // between its ++newest and its set_trec, when its window slot still holds s - tw's.)
  __host__ __device__ inline TRec TR(const TsParams& P, const TsMem& M, int32_t s) const {
    CPR_TS_AGE(1, newest - s);
    if (s > newest - M.tw) {
      // one 16-byte LDS read; volatile keeps it a ds_read apart from the ring's global load
      // (else both may be sunk into one generic load of a selected address)
      typedef int32_t v4 __attribute__((ext_vector_type(4)));
      const v4 v = *(const volatile CPR_LDS v4*)&M.tl[(int64_t)(s & (M.tw - 1)) * M.hs];
      TRec r;
      r.next = v.x;
      r.depth = v.y;
      r.pow = v.z;
      r.parent = v.w;
      return r;
    }
    return M.trec[s & (P.cap_v - 1)];
  }
  __host__ __device__ inline void set_trec(const TsParams& P, const TsMem& M, const TVtx& b) {
    TRec r;
    r.next = b.next;
    r.depth = (b.depth & 0xffff) | (int32_t)((uint32_t)b.who << 16);
    r.pow = b.pow;
    r.parent = b.parent;
    M.trec[b.serial & (P.cap_v - 1)] = r;
    if (b.serial > newest - M.tw) M.tl[(int64_t)(b.serial & (M.tw - 1)) * M.hs] = r;
  }
  __host__ __device__ inline uint8_t& V(const TsParams& P, const TsMem& M, int32_t s,
                                        int32_t node) {
    return M.vis[(int64_t)(s & (P.cap_v - 1)) * P.n + node];
  }  // visibility through the LDS window of the newest vw vertices (see bk_lane.h Vg / Vs)
  __host__ __device__ inline uint8_t Vg(const TsParams& P, const TsMem& M, int32_t s,
                                        int32_t node) const {
    CPR_TS_AGE(2, newest - s);
    if (s > newest - M.vw)
      return *(const volatile CPR_LDS uint8_t*)&M.vl[(int64_t)((s & (M.vw - 1)) * P.n + node) *
                                                      M.hs];
    return M.vis[(int64_t)(s & (P.cap_v - 1)) * P.n + node];
  }
  __host__ __device__ inline void Vs(const TsParams& P, const TsMem& M, int32_t s, int32_t node,
                                     uint8_t v) const {
    M.vis[(int64_t)(s & (P.cap_v - 1)) * P.n + node] = v;
    if (s > newest - M.vw) M.vl[(int64_t)((s & (M.vw - 1)) * P.n + node) * M.hs] = v;
  }

  __host__ __device__ inline double& VT(const TsParams& P, const TsMem& M, int32_t s,
                                        int32_t node) {
    return M.vt[(int64_t)(s & (P.cap_v - 1)) * P.n + node];
  }
  __host__ __device__ inline bool visible(const TsParams& P, const TsMem& M, int32_t s,
                                          int32_t node) {
    return (Vg(P, M, s, node) & V_KIND) != V_INV;
  }
  __host__ __device__ inline uint8_t& MK(const TsParams& P, const TsMem& M, int32_t s) {
    return M.marks[s & (P.cap_v - 1)];
  }
  __host__ __device__ inline int32_t* Q(const TsParams& P, const TsMem& M, const TVtx& b) {
    int32_t* q = M.quo + (int64_t)(b.qslot & (P.cap_q - 1)) * (P.k + 1);
    if (q[0] != b.serial) fail(7);
    return q + 1;
  }
  // summary rewards: [0, n) cumulative, [n, 2n) own reward list summed per node
  __host__ __device__ inline double* R(const TsParams& P, const TsMem& M, int32_t qslot) {
    return M.srew + (int64_t)(qslot & (P.cap_q - 1)) * 2 * P.n;
  }
  __host__ __device__ static inline bool keep_kind(uint8_t v, int32_t vf, bool marked) {
    const uint8_t kd = v & V_KIND;
    switch (vf) {
      case VF_MINE: return kd == V_WH || kd == V_REL;
      case VF_PUBLIC: return kd == V_REL || kd == V_RECV;
      case VF_PUBLIC_OR_MARKED: return kd == V_REL || kd == V_RECV || marked;
      default: return true;
    }
  }

  // ------------------------------------------------------------------ event queue
  // orderedQueue.ml:17-47, in place; +inf events are stored (they shape the tie order)
  // Nodes are read and written by value through hn_*, each picking the slab (LDS, an
  // address-space-3 pointer: ds_read / ds_write) or the HBM part (global loads) by index,
  // so the compiler never merges the two into one generic (flat) access.
  __host__ __device__ static inline HNode hn_get(const TsMem& M, int32_t i) {
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
  __host__ __device__ static inline void hn_put(const TsMem& M, int32_t i, const HNode& h) {
    if (i < M.kl)
      M.hl[(int64_t)i * M.hs] = h;
    else
      M.heap[i] = h;
  }
  __host__ __device__ static inline void hn_set_l(const TsMem& M, int32_t i, int32_t v) {
    if (i < M.kl)
      M.hl[(int64_t)i * M.hs].l = v;
    else
      M.heap[i].l = v;
  }
  __host__ __device__ static inline void hn_set_r(const TsMem& M, int32_t i, int32_t v) {
    if (i < M.kl)
      M.hl[(int64_t)i * M.hs].r = v;
    else
      M.heap[i].r = v;
  }
  __host__ __device__ static inline void hn_set_lr(const TsMem& M, int32_t i, int32_t l,
                                                   int32_t r) {
    if (i < M.kl) {
      M.hl[(int64_t)i * M.hs].l = l;
      M.hl[(int64_t)i * M.hs].r = r;
    } else {
      M.heap[i].l = l;
      M.heap[i].r = r;
    }
  }
  __host__ __device__ static inline void hn_set_key(const TsMem& M, int32_t i, double t,
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
  __host__ __device__ inline int32_t halloc(const TsParams& P, const TsMem& M) {
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
  __host__ __device__ inline void hrelease(const TsMem& M, int32_t node) {
    if (node < M.kl) {
      hn_set_l(M, node, hfree);
      hfree = node;
    } else {
      hn_set_l(M, node, hfree2);
      hfree2 = node;
    }
  }
  __host__ __device__ inline void push(const TsParams& P, const TsMem& M, double t, uint32_t ev,
                                       int32_t blk) {
    int32_t parent = -1, node = hroot;
    for (;;) {
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
  __host__ __device__ inline bool pop(const TsMem& M, double* t, uint32_t* ev, int32_t* blk) {
    if (hroot < 0) return false;
    HNode cur = hn_get(M, hroot);
    *t = cur.t;
    *ev = cur.ev;
    *blk = cur.blk;
    int32_t parent = -1, side = 0, node = hroot;
    for (;;) {
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
  __host__ __device__ inline void push_now(const TsParams& P, const TsMem& M, uint32_t ev,
                                           int32_t blk) {
    push(P, M, now, ev, blk);
  }

  // ------------------------------------------------------------------ randomness
  template <class St>
  __host__ __device__ inline int32_t miner_of(const TsParams& P, const St& S, int32_t j) {
    if (P.net == 2) return S.miner_w((uint32_t)j, P.thr, P.n - 1);
    return S.miner((uint32_t)j, P.t_att, P.d);
  }
  template <class St>
  __host__ __device__ inline void schedule_pow(const TsParams& P, const St& S,
                                               const TsMem& M) {
    push(P, M, now + S.clock((uint32_t)c_act, P.ev), mkev(EV_CLOCK, 0, KD_POW), -1);
  }

  // ------------------------------------------------------------------ vote trees
  __host__ __device__ static inline uint64_t pow_key(const TVtx& v) {
    return ((uint64_t)(uint32_t)v.pow << 32) | (uint32_t)v.serial;
  }
  // compare_votes_in_block (tailstorm.ml:124-130): deeper first, then smaller pow
  __host__ __device__ static inline bool vote_before(const TVtx& a, const TVtx& b) {
    if (a.depth != b.depth) return a.depth > b.depth;
    return pow_key(a) < pow_key(b);
  }
  // slot-indexed tree position: valid for s iff pos names a cand entry holding s
  __host__ __device__ inline int32_t& PS(const TsParams& P, const TsMem& M, int32_t s) {
    return M.pos[s & (P.cap_v - 1)];
  }
  __host__ __device__ inline int32_t& SH(const TsParams& P, const TsMem& M, int32_t s) {
    return M.shead[s & (P.cap_v - 1)];
  }
  __host__ __device__ inline bool in_tree(const TsParams& P, const TsMem& M, int32_t n,
                                          int32_t s) {
    const int32_t i = PS(P, M, s);
    return i >= 0 && i < n && M.cand[i] == s;
  }
  // votes of summary b's tree visible at `node` into cand[] (ascending serial): the
  // expansion acc_votes children' (children' b) with children' = children |> filter vf when
  // `restrict` (tailstorm.ml:509-535), else all of confirming_votes b; perm[] = BlockSet
  // order (Dag depth, serial). The candidate set is ancestor-closed down to b (a vote enters
  // only through its parent), so walks from a candidate end at b. pos[] maps back.
  __host__ __device__ inline int32_t tree(const TsParams& P, const TsMem& M, int32_t b,
                                          int32_t node, int32_t vf) {
    int32_t n = 0;
    const int32_t cap = P.cap_v;
    troot = b;
    // one read of each vote: its parent, depth and kind at `node` go to M.key with it
    for (int32_t c = X(P, M, b).thead; c >= 0 && !dead;) {
      const TRec& x = TR(P, M, c);
      const int32_t nx = x.next;
      const uint8_t v = Vg(P, M, c, node);
      if ((v & V_KIND) != V_INV && (vf == VF_ALL || keep_kind(v, vf, false))) {
        if (n >= cap) {
          fail(3);
          return 0;
        }
        const uint8_t kd = v & V_KIND;
        M.key[n] = (uint64_t)(uint32_t)x.dep() | ((uint64_t)(uint32_t)x.parent << 32);
        M.flag[n] = (kd == V_WH || kd == V_REL) ? 1 : 0;  // mine()
        M.cand[n++] = c;
      }
      c = nx;
    }
    if (dead) return 0;
    for (int32_t i = 0, j = n - 1; i < j; ++i, --j) {  // newest-first list -> ascending
      const int32_t t = M.cand[i];
      M.cand[i] = M.cand[j];
      M.cand[j] = t;
      const uint64_t tk = M.key[i];
      M.key[i] = M.key[j];
      M.key[j] = tk;
      const uint8_t tf = M.flag[i];
      M.flag[i] = M.flag[j];
      M.flag[j] = tf;
    }
    int32_t m = 0, maxd = 0;
    tclosed = 1;
    for (int32_t i = 0; i < n; ++i) {
      const int32_t c = M.cand[i];
      const uint64_t ki = M.key[i];
      const int32_t depth = (int32_t)(uint32_t)ki, parent = (int32_t)(ki >> 32);
      const bool own = M.flag[i] != 0;
      const bool pin = parent != b && in_tree(P, M, m, parent);
      if (vf != VF_ALL && parent != b && !pin) continue;
      // the selections' view of the tree vote (M.key[m]): vote depth, position of its
      // parent + 1 (0 = the summary b), and whether `node` withholds or released it
      // (m <= i: entry i is read before entry m is written)
      const int32_t pp = parent == b ? 0 : (pin ? PS(P, M, parent) + 1 : 0);
      if (parent != b && !pin) tclosed = 0;  // parent outside the tree: walk the DAG
      M.key[m] = (uint64_t)(uint32_t)depth | ((uint64_t)(uint32_t)pp << 32) |
                 (own ? (1ull << 63) : 0ull);
      PS(P, M, c) = m;
      M.cand[m++] = c;
      maxd = depth > maxd ? depth : maxd;
    }
    // Dag depth of a tree vote = depth(b) + its vote depth: stable counting sort by vote
    // depth over the serial-ascending cand gives (Dag depth, serial)
    if (maxd + 2 > cap) {
      fail(3);
      return 0;
    }
    int32_t* cnt = M.aux;  // [maxd + 2] <= cap_v
    for (int32_t d = 0; d <= maxd + 1; ++d) cnt[d] = 0;
    for (int32_t i = 0; i < m; ++i) ++cnt[(int32_t)(uint32_t)M.key[i] + 1];
    for (int32_t d = 1; d <= maxd + 1; ++d) cnt[d] += cnt[d - 1];
    for (int32_t i = 0; i < m; ++i) M.perm[cnt[(int32_t)(uint32_t)M.key[i]]++] = i;
    return m;
  }
  // votes of summary b's tree at `node` passing `vf` after expansion (compare_blocks,
  // observe): count and max depth
  __host__ __device__ inline int32_t count_post(const TsParams& P, const TsMem& M, int32_t b,
                                                int32_t node, int32_t vf, int32_t* maxd) {
    int32_t n = 0, d = 0;
    for (int32_t c = X(P, M, b).thead; c >= 0 && !dead;) {
      const TRec& x = TR(P, M, c);
      const uint8_t v = Vg(P, M, c, node);
      if ((v & V_KIND) != V_INV &&
          keep_kind(v, vf, vf == VF_PUBLIC_OR_MARKED && MK(P, M, c))) {
        ++n;
        d = x.dep() > d ? x.dep() : d;
      }
      c = x.next;
    }
    if (maxd) *maxd = d;
    return n;
  }
  __host__ __device__ inline bool mine(const TsParams& P, const TsMem& M, int32_t s,
                                       int32_t node) {
    const uint8_t kd = Vg(P, M, s, node) & V_KIND;
    return kd == V_WH || kd == V_REL;
  }
  // stable bottom-up merge sort of a[0, n) with `before` (strict); tmp holds n entries
  template <class F>
  __host__ __device__ static inline void msort(int32_t* a, int32_t* tmp, int32_t n, F before) {
    int32_t* src = a;
    int32_t* dst = tmp;
    for (int32_t w = 1; w < n; w <<= 1) {
      for (int32_t lo = 0; lo < n; lo += 2 * w) {
        const int32_t mid = lo + w < n ? lo + w : n, hi = lo + 2 * w < n ? lo + 2 * w : n;
        int32_t i = lo, j = mid, o = lo;
        while (i < mid && j < hi) dst[o++] = before(src[j], src[i]) ? src[j++] : src[i++];
        while (i < mid) dst[o++] = src[i++];
        while (j < hi) dst[o++] = src[j++];
      }
      int32_t* t = src;
      src = dst;
      dst = t;
    }
    if (src != a)
      for (int32_t i = 0; i < n; ++i) a[i] = src[i];
  }

  // writes the draft's leaves (sorted by compare_votes_in_block) to q; returns #leaves or 0.
  // The included set is ancestor-closed (a branch enters with all its votes), so a walk up
  // from a candidate counts its fresh votes until the first included one, and a candidate
  // whose vote depth exceeds the deepest included vote by more than `need` cannot fit.
  __host__ __device__ inline int32_t heuristic(const TsParams& P, const TsMem& M, int32_t node,
                                               int32_t n, int32_t* q) {
    // flag = included
    for (int32_t i = 0; i < n; ++i) M.flag[i] = 0;
    int32_t need = P.k, nl = 0, dinc = 0;
    if (tclosed) {
      // on tree()'s view (M.key: depth, parent position, own): the same walks by position
      // instead of by vertex (PS(s) is s's position; the parent chain ends at troot = 0)
      while (need > 0 && !dead) {
        int32_t best = -1, bo = -1, bt = -1;
        for (int32_t pi = 0; pi < n; ++pi) {
          const int32_t i = M.perm[pi];
          if (M.flag[i]) continue;
          if ((int32_t)(uint32_t)M.key[i] - dinc > need) continue;
          int32_t own = 0, tot = 0, p = i + 1;
          while (p != 0) {
            if (M.flag[p - 1]) break;
            if (++tot > need) break;
            const uint64_t kp = M.key[p - 1];
            own += (int32_t)(kp >> 63);
            p = (int32_t)((kp >> 32) & 0x7fffffffu);
          }
          if (tot > need) continue;
          if (own > bo || (own == bo && tot > bt)) {
            best = i;
            bo = own;
            bt = tot;
          }
        }
        if (best < 0) {  // `assert false` in the reference
          fail(11);
          return 0;
        }
        q[nl++] = M.cand[best];
        const int32_t db = (int32_t)(uint32_t)M.key[best];
        dinc = db > dinc ? db : dinc;
        for (int32_t p = best + 1; p != 0;) {
          uint8_t& f = M.flag[p - 1];
          if (f) break;
          f = 1;
          --need;
          p = (int32_t)((M.key[p - 1] >> 32) & 0x7fffffffu);
        }
      }
      return nl;
    }
    while (need > 0 && !dead) {
      int32_t best = -1, bo = -1, bt = -1;
      for (int32_t pi = 0; pi < n; ++pi) {
        const int32_t i = M.perm[pi];
        if (M.flag[i]) continue;
        if (X(P, M, M.cand[i]).depth - dinc > need) continue;
        int32_t own = 0, tot = 0, s = M.cand[i];
        while (s != troot) {
          if (M.flag[PS(P, M, s)]) break;
          if (++tot > need) break;
          own += mine(P, M, s, node) ? 1 : 0;
          s = X(P, M, s).parent;
        }
        if (tot > need) continue;
        if (own > bo || (own == bo && tot > bt)) {
          best = i;
          bo = own;
          bt = tot;
        }
      }
      if (best < 0) {  // `assert false` in the reference
        fail(11);
        return 0;
      }
      q[nl++] = M.cand[best];
      int32_t s = M.cand[best];
      const int32_t db = X(P, M, s).depth;
      dinc = db > dinc ? db : dinc;
      while (s != troot) {
        uint8_t& f = M.flag[PS(P, M, s)];
        if (f) break;
        f = 1;
        --need;
        s = X(P, M, s).parent;
      }
    }
    return nl;
  }
  __host__ __device__ inline int32_t altruistic(const TsParams& P, const TsMem& M, int32_t node,
                                                int32_t n, int32_t* q) {
    // List.sort (stable) of BlockSet.elements by (neg depth, (own 0 | 1, visible_since))
    for (int32_t pi = 0; pi < n; ++pi) M.aux[pi] = M.perm[pi];
    auto before = [&](int32_t a, int32_t b) {  // strict "a sorts before b"
      const TVtx& x = X(P, M, M.cand[a]);
      const TVtx& y = X(P, M, M.cand[b]);
      if (x.depth != y.depth) return x.depth > y.depth;
      const int32_t ox = mine(P, M, x.serial, node) ? 0 : 1, oy = mine(P, M, y.serial, node) ? 0 : 1;
      if (ox != oy) return ox < oy;
      return VT(P, M, x.serial, node) < VT(P, M, y.serial, node);
    };
    msort(M.aux, (int32_t*)M.key, n, before);
    for (int32_t i = 0; i < n; ++i) M.flag[i] = 0;  // acc (ancestor-closed)
    int32_t cnt = 0, nl = 0;
    for (int32_t t = 0; t < n && cnt < P.k && !dead; ++t) {
      const int32_t hd = M.aux[t];
      int32_t nf = 0, s = M.cand[hd];
      while (s != troot && cnt + nf <= P.k) {
        if (M.flag[PS(P, M, s)]) break;
        ++nf;
        s = X(P, M, s).parent;
      }
      if (cnt + nf > P.k || nf < 1) continue;
      for (s = M.cand[hd]; s != troot;) {
        uint8_t& f = M.flag[PS(P, M, s)];
        if (f) break;
        f = 1;
        s = X(P, M, s).parent;
      }
      cnt += nf;
      q[nl++] = M.cand[hd];
    }
    return cnt == P.k ? nl : 0;
  }
  // reward of a draft with these leaves for `node` (reward' folded over my entries)
  __host__ __device__ inline double draft_reward(const TsParams& P, const TsMem& M, int32_t node,
                                                 int32_t n, const int32_t* lv, int32_t nl) {
    for (int32_t i = 0; i < n; ++i) M.flag2[i] = 0;
    const bool punish = P.scheme == SC_PUNISH || P.scheme == SC_HYBRID;
    const bool discount = P.scheme == SC_DISCOUNT || P.scheme == SC_HYBRID;
    const int32_t upto = punish ? 1 : nl;
    for (int32_t t = 0; t < upto; ++t) {
      for (int32_t s = lv[t]; s != troot;) {
        uint8_t& f = M.flag2[PS(P, M, s)];
        if (f) break;
        f = 1;
        s = X(P, M, s).parent;
      }
    }
    const double r = discount ? (double)X(P, M, lv[0]).depth / (double)P.k * 1.0 : 1.0;
    double acc = 0.0;
    for (int32_t i = 0; i < n; ++i)
      if (M.flag2[i] && X(P, M, M.cand[i]).who == node) acc += r;
    return acc;
  }
  __host__ __device__ inline int32_t optimal(const TsParams& P, const TsMem& M, int32_t node,
                                             int32_t n, int32_t* q) {
    bool dz = false;
    const int64_t nck = ocaml_nck(n, P.k, &dz);
    if (dz) {
      fail(11);
      return 0;
    }
    if (nck > 100) return heuristic(P, M, node, n, q);
    if (n < P.k) return 0;
    // a = BlockSet order; pos[cand index] = position in a (M.aux)
    for (int32_t pi = 0; pi < n; ++pi) M.aux[M.perm[pi]] = pi;
    // The reference's subsets in its lexicographic order (iter_n_choose_k), minus the
    // prefixes no completion of which can count (oracle/src/tailstorm.cpp TsView::optimal):
    // the newest vote's vote parent not chosen (Not_connected), or own votes chosen plus
    // min(slots left, own votes after it) worth at most maxdepth / k (discount) or 1 each,
    // summed as the reward sums them, not above the best so far (strict >). Per position:
    // par = its vote parent's position (-1 a summary), own, and own votes after it
    // (M.key as int32 pairs: positions are < cap_v). The search stops after
    // P.opt_budget prefixes (TS_OPT_BUDGET = oracle/src/tailstorm.h TS_BRUTE_FORCE_BUDGET)
    // and flags the episode; both engines count the same prefixes (only those that can
    // still reach k positions), so they flag the same searches at any budget.
    int32_t* par = reinterpret_cast<int32_t*>(M.key);
    int32_t* oaft = par + n;  // own votes at positions > i, [n + 1]
    int32_t maxdepth = 0;
    for (int32_t i = 0; i < n; ++i) {
      const TVtx& x = X(P, M, M.cand[M.perm[i]]);
      par[i] = x.parent != troot ? M.aux[PS(P, M, x.parent)] : -1;
      maxdepth = x.depth > maxdepth ? x.depth : maxdepth;
    }
    oaft[n] = 0;
    for (int32_t i = n - 1; i >= 0; --i)
      oaft[i] = oaft[i + 1] + (X(P, M, M.cand[M.perm[i]]).who == node ? 1 : 0);
    const bool disc = P.scheme == SC_DISCOUNT || P.scheme == SC_HYBRID;
    const double rmax = disc ? (double)maxdepth / (double)P.k * 1.0 : 1.0;
    int32_t* c = M.stack;        // current choice (k <= 64); stack is free here
    int32_t* lv = M.stack + 64;  // leaves of the choice
    // [n]: position chosen in the current prefix (stack holds 2 cap_v ints, n <= cap_v)
    uint8_t* chosen = reinterpret_cast<uint8_t*>(M.stack + 128);
    for (int32_t i = 0; i < n; ++i) chosen[i] = 0;
    double best = -1.0;
    int32_t nbest = 0;
    int64_t visits = 0;
    int32_t j = 0, nxt = 0, ownp = 0;
    for (;;) {
      if (j == P.k) {
        // leaves c (tailstorm.ml:442-481): reach (flag) and leave (flag2) over positions
        for (int32_t i = 0; i < n; ++i) {
          M.flag[i] = 0;
          M.flag2[i] = 1;
        }
        for (int32_t t = 0; t < P.k; ++t) {
          if (par[c[t]] >= 0) M.flag2[par[c[t]]] = 0;
          M.flag[c[t]] = 1;
        }
        int32_t nl = 0;
        for (int32_t i = 0; i < n; ++i)
          if (M.flag[i] && M.flag2[i]) lv[nl++] = M.cand[M.perm[i]];
        for (int32_t i = 1; i < nl; ++i) {  // sort by compare_votes_in_block (unique keys)
          const int32_t v = lv[i];
          int32_t u = i;
          while (u > 0 && vote_before(X(P, M, v), X(P, M, lv[u - 1]))) {
            lv[u] = lv[u - 1];
            --u;
          }
          lv[u] = v;
        }
        const double r = draft_reward(P, M, node, n, lv, nl);
        if (r > best) {
          best = r;
          nbest = nl;
          for (int32_t i = 0; i < nl; ++i) q[i] = lv[i];
        }
        // back to the last choice; the next index there
        --j;
        chosen[c[j]] = 0;
        ownp -= X(P, M, M.cand[M.perm[c[j]]]).who == node ? 1 : 0;
        nxt = c[j] + 1;
        continue;
      }
      int32_t placed = -1;
      for (int32_t i = nxt; i <= n - (P.k - j) && !dead; ++i) {
        if (par[i] >= 0 && !chosen[par[i]]) continue;  // every completion Not_connected
        const int32_t oi = X(P, M, M.cand[M.perm[i]]).who == node ? 1 : 0;
        const int32_t rest = P.k - j - 1 < oaft[i + 1] ? P.k - j - 1 : oaft[i + 1];
        const int32_t cap = ownp + oi + rest;
        if (nbest > 0) {  // cannot beat the best: rmax added cap times
          double bnd = 0.0;
          for (int32_t m = 0; m < cap; ++m) bnd += rmax;
          if (bnd <= best) continue;
        }
        if (++visits > P.opt_budget) {
          fail(12);
          return 0;
        }
        placed = i;
        ownp += oi;
        break;
      }
      if (dead) return 0;
      if (placed >= 0) {
        c[j] = placed;
        chosen[placed] = 1;
        ++j;
        nxt = placed + 1;
        continue;
      }
      if (j == 0) break;
      --j;
      chosen[c[j]] = 0;
      ownp -= X(P, M, M.cand[M.perm[c[j]]]).who == node ? 1 : 0;
      nxt = c[j] + 1;
    }
    if (nbest == 0) fail(11);  // "reward_optim_quorum: no choice"
    return nbest;
  }
  // Honest.next_summary' (tailstorm.ml:530-535): draft seq or -1
  __host__ __device__ inline int32_t next_summary(const TsParams& P, const TsMem& M,
                                                  int32_t node, int32_t b, int32_t vf) {
    // the tree's votes are a subset of b's vote list, whose length is b.nconf (append_vote):
    // fewer than k there and the tree walk cannot find k (every vote of the list is newer
    // than b, so the walk could not meet an overwritten ring slot either)
    if (X(P, M, b).nconf < P.k) return -1;
    const int32_t n = tree(P, M, b, node, vf);
    if (dead || n < P.k) return -1;  // all three selections need k votes
    const int32_t seq = dseq;
    int32_t* dr = M.drafts + (int64_t)(seq & (P.cap_d - 1)) * (P.k + 2);
    int32_t* q = dr + 2;
    int32_t nl;
    if (P.selection == SEL_ALTRUISTIC)
      nl = altruistic(P, M, node, n, q);
    else if (P.selection == SEL_OPTIMAL)
      nl = optimal(P, M, node, n, q);
    else
      nl = heuristic(P, M, node, n, q);
    if (nl <= 0 || dead) return -1;
    if (P.selection != SEL_OPTIMAL || nl != 0) {
      // leaves sorted by compare_votes_in_block (altruistic: by (neg depth, pow), same
      // order since every vote has a pow)
      for (int32_t i = 1; i < nl; ++i) {
        const int32_t v = q[i];
        int32_t j = i;
        while (j > 0 && vote_before(X(P, M, v), X(P, M, q[j - 1]))) {
          q[j] = q[j - 1];
          --j;
        }
        q[j] = v;
      }
    }
    dr[0] = seq;
    dr[1] = nl;
    ++dseq;
    return seq;
  }
  // Honest.puzzle_payload (tailstorm.ml:509-528): parent of the next vote on summary b
  __host__ __device__ inline int32_t payload_parent(const TsParams& P, const TsMem& M,
                                                    int32_t node, int32_t b) {
    int32_t best = b, bd = 0, bp = 0;
    for (int32_t c = X(P, M, b).thead; c >= 0 && !dead;) {
      const TRec& x = TR(P, M, c);
      // vote_before (deeper first, then the smaller (pow, serial))
      if (visible(P, M, c, node) &&
          (best == b || x.dep() > bd ||
           (x.dep() == bd && (((uint64_t)(uint32_t)x.pow << 32) | (uint32_t)c) <
                                 (((uint64_t)(uint32_t)bp << 32) | (uint32_t)best)))) {
        best = c;
        bd = x.dep();
        bp = x.pow;
      }
      c = x.next;
    }
    return best;
  }
  // compare_blocks (tailstorm.ml:539-550) at `node`
  __host__ __device__ inline int32_t compare_blocks(const TsParams& P, const TsMem& M,
                                                    int32_t node, int32_t vf, int32_t a,
                                                    int32_t b) {
    if (a == b) return 0;
    const TVtx& xa = X(P, M, a);
    const TVtx& xb = X(P, M, b);
    if (xa.height != xb.height) return xa.height < xb.height ? -1 : 1;
    const int32_t ca = count_post(P, M, a, node, vf, nullptr);
    const int32_t cb = count_post(P, M, b, node, vf, nullptr);
    if (ca != cb) return ca < cb ? -1 : 1;
    const double ra = xa.qslot < 0 ? 0.0 : R(P, M, xa.qslot)[P.n + node];
    const double rb = xb.qslot < 0 ? 0.0 : R(P, M, xb.qslot)[P.n + node];
    return ra < rb ? -1 : (ra > rb ? 1 : 0);
  }
  __host__ __device__ inline int32_t update_head(const TsParams& P, const TsMem& M, int32_t node,
                                                 int32_t vf, int32_t old, int32_t cand) {
    return compare_blocks(P, M, node, vf, cand, old) > 0 ? cand : old;
  }
  __host__ __device__ inline bool has_children(const TsParams& P, const TsMem& M, int32_t s,
                                               int32_t node) {
    // children of a summary are votes on it: the depth-1 votes of its tree
    for (int32_t c = X(P, M, s).thead; c >= 0 && !dead;) {
      const TRec& x = TR(P, M, c);
      if (x.parent == s && visible(P, M, c, node)) return true;
      c = x.next;
    }
    return false;
  }
  // tailstorm.ml:557-563
  __host__ __device__ inline bool feasible(const TsParams& P, const TsMem& M, int32_t node,
                                           int32_t preferred, int32_t after) {
    const int32_t ext = X(P, M, after).height + 1, cur = X(P, M, preferred).height;
    return cur < ext || (cur == ext && !has_children(P, M, preferred, node));
  }

  // ------------------------------------------------------------------ DAG
  __host__ __device__ inline void init_vertex(const TsParams& P, const TsMem& M, TVtx& b,
                                              int32_t s) {
    b.serial = s;
    b.nconf = 0;
    b.qslot = -1;
    b.nq = 0;
    b.time = now;
    b.next = -1;
    b.thead = -1;
    for (int32_t j = 0; j < P.n; ++j) Vs(P, M, s, j, V_INV);
  }
  template <class St>
  __host__ __device__ inline int32_t append_vote(const TsParams& P, const St& S,
                                                 const TsMem& M, int32_t node, int32_t parent) {
    TVtx& p = X(P, M, parent);
    const int32_t s = ++newest;
    TVtx& b = M.vtx[s & (P.cap_v - 1)];
    init_vertex(P, M, b, s);
    b.parent = parent;
    b.height = p.height;
    b.vote = 1;
    b.who = node;
    b.depth = (p.vote ? p.depth : 0) + 1;
    b.pow = S.pow((uint32_t)s);
    b.ddepth = p.ddepth + 1;
    b.sum = p.vote ? p.sum : parent;
    TVtx& sb = X(P, M, b.sum);
    sb.nconf += 1;
    b.next = sb.thead;  // newest-first vote list of the tree
    sb.thead = s;
    set_trec(P, M, b);
    return s;
  }
  // Dag(node, Append, draft): Simulator.append dedup (simulator.ml:139-159) or a fresh
  // summary with set_rewards (simulator.ml:377-388, tailstorm.ml:204-227). Returns the
  // vertex (existing or new).
  __host__ __device__ inline int32_t append_summary(const TsParams& P, const TsMem& M,
                                                    int32_t dseq_) {
    const int32_t* dr = M.drafts + (int64_t)(dseq_ & (P.cap_d - 1)) * (P.k + 2);
    if (dr[0] != dseq_) {
      fail(4);
      return 0;
    }
    const int32_t nl = dr[1];
    const int32_t* lv = dr + 2;
    const TVtx& l0 = X(P, M, lv[0]);
    const int32_t prev = l0.sum;
    const int32_t height = X(P, M, prev).height + 1;
    // candidates: children of lv[0], newest first; only summaries can equal the draft, and
    // those are child summaries of prev (newest-first list)
    for (int32_t c = SH(P, M, prev); c >= 0 && !dead; c = X(P, M, c).next) {
      const TVtx& y = X(P, M, c);
      if (y.height != height || y.parent != lv[0]) continue;
      const int32_t* yq = Q(P, M, y);
      bool eq = true;
      const int32_t m = y.nq < nl ? y.nq : nl;
      for (int32_t i = 0; i < m && eq; ++i) eq = yq[i] == lv[i];
      if (eq && y.nq != nl) {  // List.for_all2 raises Invalid_argument
        fail(11);
        return c;
      }
      if (eq) return c;  // `Redundant
    }
    if (P.mode == 1 && ++zt > 4096) {  // loop-mode guard, see bk_lane.h
      fail(8);
      return 0;
    }
    const int32_t s = ++newest;
    const int32_t qs = nsum++;
    int32_t* q = M.quo + (int64_t)(qs & (P.cap_q - 1)) * (P.k + 1);
    q[0] = s;
    int32_t dd = 0;
    for (int32_t i = 0; i < nl; ++i) {
      q[1 + i] = lv[i];
      const int32_t d = X(P, M, lv[i]).ddepth;
      dd = d > dd ? d : dd;
    }
    // rewards: cumulative of the precursor (leaf 0 -> ... -> previous summary), then r per
    // vote of the confirmed set (or of leaf 0's branch for punish/hybrid)
    double* rw = R(P, M, qs);
    const TVtx& ps = X(P, M, prev);
    for (int32_t j = 0; j < P.n; ++j) {
      rw[j] = ps.qslot < 0 ? 0.0 : R(P, M, ps.qslot)[j];
      rw[P.n + j] = 0.0;
    }
    const bool punish = P.scheme == SC_PUNISH || P.scheme == SC_HYBRID;
    const bool discount = P.scheme == SC_DISCOUNT || P.scheme == SC_HYBRID;
    const double r = discount ? (double)l0.depth / (double)P.k * 1.0 : 1.0;
    // the confirmed set = union of the leaves' branches; mark to count each vote once
    const int32_t upto = punish ? 1 : nl;
    // (the branches' votes are newer than prev: their list records are in the ring)
    for (int32_t t = 0; t < upto; ++t) {
      int32_t v = lv[t];
      while (v != prev && !dead) {
        MK(P, M, v) = 0;
        v = TR(P, M, v).parent;
      }
    }
    for (int32_t t = 0; t < upto; ++t) {
      int32_t v = lv[t];
      while (v != prev && !dead) {
        uint8_t& mk = MK(P, M, v);
        const TRec& x = TR(P, M, v);
        if (!mk) {
          mk = 1;
          const int32_t w = x.who();
          rw[w] += r;
          rw[P.n + w] += r;
        }
        v = x.parent;
      }
    }
    TVtx& b = M.vtx[s & (P.cap_v - 1)];
    init_vertex(P, M, b, s);
    b.parent = lv[0];
    b.height = height;
    b.vote = 0;
    b.who = -1;
    b.depth = 0;
    b.pow = 0;
    b.ddepth = dd + 1;
    b.sum = s;
    b.qslot = qs;
    b.nq = nl;
    SH(P, M, s) = -1;
    b.next = SH(P, M, prev);  // newest-first child-summary list of prev
    SH(P, M, prev) = s;
    set_trec(P, M, b);
    return s;
  }

  // ------------------------------------------------------------------ actions
  __host__ __device__ inline void share(const TsParams& P, const TsMem& M, int32_t node,
                                        int32_t s0) {
    int32_t* st = M.stack;
    int32_t sp = 0;
    st[sp++] = s0;
    while (sp > 0 && !dead) {
      const int32_t s = st[--sp];
      const uint8_t v = Vg(P, M, s, node);
      if ((v & V_KIND) != V_WH) continue;
      Vs(P, M, s, node, (uint8_t)((v & ~V_KIND) | V_REL));
      push_now(P, M, mkev(EV_TX, node, KD_NET), s);
      const TVtx& b = X(P, M, s);
      if (b.parent < 0) continue;
      const int32_t np = b.vote ? 1 : b.nq;
      if (sp + np > 2 * P.cap_v) {
        fail(5);
        return;
      }
      if (b.vote) {
        st[sp++] = b.parent;
      } else {
        const int32_t* q = Q(P, M, b);
        for (int32_t i = b.nq - 1; i >= 0; --i) st[sp++] = q[i];
      }
    }
  }

  // Dagtools.common_ancestor (dagtools.ml:102-121) in the attacker's view: ancestors by
  // descending (Dag depth, serial), set semantics
  __host__ __device__ static inline uint64_t fr_key(int32_t dd, int32_t s) {
    return ((uint64_t)(uint32_t)dd << 32) | (uint32_t)s;
  }
  __host__ __device__ inline void fr_insert(int32_t* q, int32_t* nq, int32_t s, int32_t dd) {
    const uint64_t kk = fr_key(dd, s);
    for (int32_t j = 0; j < *nq; ++j)
      if (q[2 * j + 1] == s) return;
    if (*nq >= NFR) {
      fail(10);
      return;
    }
    int32_t i = *nq;
    while (i > 0 && fr_key(q[2 * (i - 1)], q[2 * (i - 1) + 1]) < kk) {
      q[2 * i] = q[2 * (i - 1)];
      q[2 * i + 1] = q[2 * (i - 1) + 1];
      --i;
    }
    q[2 * i] = dd;
    q[2 * i + 1] = s;
    ++*nq;
  }
  __host__ __device__ inline int32_t fr_next(const TsParams& P, const TsMem& M, int32_t* q,
                                             int32_t* nq) {
    if (*nq == 0) return -1;
    const int32_t s = q[1];
    for (int32_t j = 1; j < *nq; ++j) {
      q[2 * (j - 1)] = q[2 * j];
      q[2 * (j - 1) + 1] = q[2 * j + 1];
    }
    --*nq;
    const TVtx& b = X(P, M, s);
    if (b.parent >= 0) {
      if (b.vote) {
        fr_insert(q, nq, b.parent, X(P, M, b.parent).ddepth);
      } else {
        const int32_t* lq = Q(P, M, b);
        for (int32_t i = 0; i < b.nq; ++i) fr_insert(q, nq, lq[i], X(P, M, lq[i]).ddepth);
      }
    }
    return s;
  }
  // parent summary of summary x: the tree root of its quorum (tailstorm.ml:124-130)
  __host__ __device__ inline int32_t psum(const TsParams& P, const TsMem& M, int32_t x) {
    return X(P, M, Q(P, M, X(P, M, x))[0]).sum;
  }
  // Dagtools.common_ancestor of two summaries without the frontier walk. The walk returns
  // the intersection's maximal (Dag depth, serial) vertex. A vote lies in exactly one
  // summary tree, and a summary's ancestors are itself, the vote paths from its quorum up
  // to its parent summary, and that summary's ancestors; so the intersection is s* (the
  // summaries' last common summary) with everything below it, plus the votes of tree(s*)
  // on the quorum paths of both chains' children of s*, which all lie deeper than s*.
  // Cost: the summary-chain distance plus those paths, instead of every vertex above the
  // answer (tests/native/ts_vs_oracle.cpp compares it with the oracle's frontier walk).
  __host__ __device__ inline int32_t common_ancestor(const TsParams& P, const TsMem& M,
                                                     int32_t a, int32_t b) {
    // the DAG only grows, so the answer for the same two vertices never changes: the last
    // one is kept (ca_a, ca_b -> ca_s). Every vertex the walk would read lies between the
    // answer and a, b, so reading the answer alone meets an overwritten ring slot exactly
    // when the walk would
    if (a == ca_a && b == ca_b) {
      (void)X(P, M, ca_s);
      return dead ? 0 : ca_s;
    }
    const int32_t r = common_ancestor_sum(P, M, a, b);
    ca_a = a;
    ca_b = b;
    ca_s = r;
    return r;
  }
  __host__ __device__ inline int32_t common_ancestor_sum(const TsParams& P, const TsMem& M,
                                                         int32_t a, int32_t b) {
    int32_t x = a, y = b, cx = -1, cy = -1;
    while (!dead && X(P, M, x).height > X(P, M, y).height) {
      cx = x;
      x = psum(P, M, x);
    }
    while (!dead && X(P, M, y).height > X(P, M, x).height) {
      cy = y;
      y = psum(P, M, y);
    }
    while (!dead && x != y) {
      cx = x;
      x = psum(P, M, x);
      cy = y;
      y = psum(P, M, y);
    }
    if (dead) return 0;
    const int32_t s = x;
    if (cx < 0 || cy < 0) return s;  // one head is s* itself
    const TVtx& bx = X(P, M, cx);
    const TVtx& by = X(P, M, cy);
    const int32_t* qx = Q(P, M, bx);
    const int32_t* qy = Q(P, M, by);
    // marks are scratch shared with reward() and apply(), which leave theirs set: clear the
    // two path sets first (at most 2 k walks of at most k votes)
    for (int32_t i = 0; i < bx.nq && !dead; ++i)
      for (int32_t v = qx[i]; v != s && !dead; v = X(P, M, v).parent) MK(P, M, v) = 0;
    for (int32_t i = 0; i < by.nq && !dead; ++i)
      for (int32_t v = qy[i]; v != s && !dead; v = X(P, M, v).parent) MK(P, M, v) = 0;
    for (int32_t i = 0; i < bx.nq && !dead; ++i)
      for (int32_t v = qx[i]; v != s && !dead && !(MK(P, M, v) & 1u); v = X(P, M, v).parent)
        MK(P, M, v) |= 1u;
    int32_t best = s;
    uint64_t bkey = fr_key(X(P, M, s).ddepth, s);
    for (int32_t i = 0; i < by.nq && !dead; ++i)
      for (int32_t v = qy[i]; v != s && !dead && !(MK(P, M, v) & 2u); v = X(P, M, v).parent) {
        uint8_t& mk = MK(P, M, v);
        if (mk & 1u) {  // shared: its ancestors up to s* are shared and shallower
          const uint64_t kv = fr_key(X(P, M, v).ddepth, v);
          if (kv > bkey) {
            bkey = kv;
            best = v;
          }
          break;
        }
        mk |= 2u;
      }
    return best;
  }

  // the frontier walk as the reference performs it (kept for reference and tests)
  __host__ __device__ inline int32_t common_ancestor_walk(const TsParams& P, const TsMem& M,
                                                          int32_t a, int32_t b) {
    int32_t* qa = M.fr;
    int32_t* qb = M.fr + 2 * NFR;
    int32_t na = 0, nb = 0;
    fr_insert(qa, &na, a, X(P, M, a).ddepth);
    fr_insert(qb, &nb, b, X(P, M, b).ddepth);
    int32_t x = fr_next(P, M, qa, &na);
    int32_t y = fr_next(P, M, qb, &nb);
    while (x >= 0 && y >= 0 && !dead) {
      if (x == y) return x;
      const uint64_t kx = fr_key(X(P, M, x).ddepth, x), ky = fr_key(X(P, M, y).ddepth, y);
      if (kx > ky)
        x = fr_next(P, M, qa, &na);
      else
        y = fr_next(P, M, qb, &nb);
    }
    fail(10);
    return 0;
  }

  // ------------------------------------------------------------------ agent
  // tailstorm_ssz.ml:210-258
  __host__ __device__ inline void prepare(const TsParams& P, const TsMem& M, uint32_t kind,
                                          int32_t x) {
    int32_t p = pub;
    for (int32_t i = 0; i < npend && !dead; ++i)
      p = update_head(P, M, 0, VF_PUBLIC, p, X(P, M, M.pend[i]).sum);
    int32_t q = priv;
    if (kind == KD_APP) {
      q = update_head(P, M, 0, VF_ALL, priv, x);
      o_event = 0;
    } else if (kind == KD_POW) {
      o_event = 1;
    } else {
      p = update_head(P, M, 0, VF_PUBLIC, p, X(P, M, x).sum);
      o_event = 2;
    }
    o_pub = p;
    o_priv = q;
    o_common = common_ancestor(P, M, p, q);
  }
  // tailstorm_ssz.ml:262-290
  __host__ __device__ inline TsObs observe(const TsParams& P, const TsMem& M) {
    TsObs o;
    o.public_votes = count_post(P, M, o_pub, 0, VF_PUBLIC, &o.public_depth);
    // VF_ALL and VF_MINE over the same list in one walk (count_post twice, fused)
    {
      int32_t na = 0, da = 0, nm = 0, dm = 0;
      for (int32_t c = X(P, M, o_priv).thead; c >= 0 && !dead;) {
        const TRec& x = TR(P, M, c);
        const uint8_t kd = Vg(P, M, c, 0) & V_KIND;
        if (kd != V_INV) {
          ++na;
          da = x.dep() > da ? x.dep() : da;
          if (kd == V_WH || kd == V_REL) {
            ++nm;
            dm = x.dep() > dm ? x.dep() : dm;
          }
        }
        c = x.next;
      }
      o.private_votes_inclusive = na;
      o.private_depth_inclusive = da;
      o.private_votes_exclusive = nm;
      o.private_depth_exclusive = dm;
    }
    const int32_t ca = X(P, M, o_common).height;
    const int32_t ph = X(P, M, o_priv).height, qh = X(P, M, o_pub).height;
    o.private_blocks = ph - ca;
    o.public_blocks = qh - ca;
    o.diff_blocks = ph - qh;
    o.event = o_event;
    return o;
  }
  // tailstorm_ssz.ml:292-350
  __host__ __device__ inline void apply(const TsParams& P, const TsMem& M, int32_t action) {
    const int32_t kind = action & 3;  // 0 Adopt, 1 Override, 2 Match, 3 Wait
    npend = 0;
    if (kind == 1 || kind == 2) {
      // withheld descendants of common in view 0, ascending (Dag depth, serial)
      const int32_t c0 = o_common;
      for (int32_t s = c0; s <= newest; ++s) MK(P, M, s) = 0;
      int32_t nw = 0;
      // this scan covers every vertex since the common ancestor: the visibility bytes and
      // list records (a vote has depth >= 1, a summary 0) of several vertices are loaded
      // together, so their latencies overlap, then the vertices are processed in order
      // (a vertex's parent precedes it, so its mark is final when it is read); only a
      // summary's quorum reads the vertex itself
      // four vertices' visibility and list-record fields are loaded together (static
      // indices: they stay in registers), then processed in order
      for (int32_t base = c0; base <= newest && !dead; base += 4) {
        uint8_t vb[4];
        int32_t pb[4], db[4];
#pragma unroll
        for (int32_t q = 0; q < 4; ++q) {
          const int32_t sq = base + q <= newest ? base + q : base;
          vb[q] = Vg(P, M, sq, 0);
          const TRec& r = TR(P, M, sq);
          pb[q] = r.parent;
          db[q] = r.dep();
        }
        bool stop = false;
#pragma unroll
        for (int32_t q = 0; q < 4; ++q) {
          const int32_t s = base + q;
          if (stop || s > newest || dead) {
            stop = true;
            continue;
          }
          const uint8_t v = vb[q];
          if ((v & V_KIND) == V_INV) continue;
          bool d = s == c0;
          if (!d && pb[q] >= 0) {
            if (db[q] > 0) {
              d = pb[q] >= c0 && MK(P, M, pb[q]);
            } else {
              const TVtx& x = X(P, M, s);
              const int32_t* lq = Q(P, M, x);
              for (int32_t i = 0; i < x.nq && !d; ++i) d = lq[i] >= c0 && MK(P, M, lq[i]);
            }
          }
          if (!d) continue;
          MK(P, M, s) = 1;
          if ((v & V_KIND) == V_WH) {
            if (nw >= P.cap_v) {
              fail(9);
              stop = true;
              continue;
            }
            M.pend[nw++] = s;
          }
        }
        if (stop) break;
      }
      // sort by (Dag depth, serial): insertion sort on the (mostly sorted) list
      for (int32_t i = 1; i < nw; ++i) {
        const int32_t v = M.pend[i];
        const uint64_t kv = fr_key(X(P, M, v).ddepth, v);
        int32_t j = i;
        while (j > 0 && fr_key(X(P, M, M.pend[j - 1]).ddepth, M.pend[j - 1]) > kv) {
          M.pend[j] = M.pend[j - 1];
          --j;
        }
        M.pend[j] = v;
      }
      // release search: marks now hold the release set
      for (int32_t s = c0; s <= newest; ++s) MK(P, M, s) = 0;
      // update_head ~vf:public_or_marked o_pub (sum x) for each prefix: the two tree
      // counts compare_blocks reads change by one per marked (withheld, visible) vote, so
      // they are kept per summary (o_pub's, and the latest candidate's) instead of rescanned
      int32_t take = nw, cs = -1, cc = 0, pc = -1;
      for (int32_t i = 0; i < nw && !dead; ++i) {
        const int32_t x = M.pend[i];
        MK(P, M, x) = 1;
        const TVtx& xv = X(P, M, x);
        if (xv.vote) {
          if (xv.sum == cs) ++cc;
          if (pc >= 0 && xv.sum == o_pub) ++pc;
        }
        const int32_t c = xv.sum;
        bool keep_old = true;  // compare_blocks c o_pub <= 0
        if (c != o_pub) {
          const TVtx& xa = X(P, M, c);
          const TVtx& xb = X(P, M, o_pub);
          if (xa.height != xb.height) {
            keep_old = xa.height < xb.height;
          } else {
            if (c != cs) {
              cs = c;
              cc = count_post(P, M, c, 0, VF_PUBLIC_OR_MARKED, nullptr);
            }
            if (pc < 0) pc = count_post(P, M, o_pub, 0, VF_PUBLIC_OR_MARKED, nullptr);
            if (cc != pc) {
              keep_old = cc < pc;
            } else {
              const double ra = xa.qslot < 0 ? 0.0 : R(P, M, xa.qslot)[P.n + 0];
              const double rb = xb.qslot < 0 ? 0.0 : R(P, M, xb.qslot)[P.n + 0];
              keep_old = !(ra > rb);
            }
          }
        }
        if (keep_old) {
          take = kind == 1 ? i + 1 : i;
          break;
        }
      }
      npend = take;
      for (int32_t i = 0; i < npend && !dead; ++i) share(P, M, 0, M.pend[i]);
    }
    const int32_t np = kind == 0 ? o_pub : o_priv;
    // extend: replace the private tip if it has no confirmation, else advance it
    int32_t extend = o_priv;
    if (!has_children(P, M, o_priv, 0)) {
      const TVtx& pr = X(P, M, o_priv);
      if (pr.parent < 0) {  // List.hd [] on the genesis summary
        fail(11);
        return;
      }
      extend = X(P, M, pr.parent).sum;
    }
    const int32_t d = next_summary(P, M, 0, extend, action >= 4 ? VF_ALL : VF_MINE);
    if (d >= 0) push_now(P, M, mkev(EV_DAG, 0, KD_APP), d);
    pub = o_pub;
    priv = np;
  }

  // ------------------------------------------------------------------ engine
  template <class St>
  __host__ __device__ inline void init(const TsParams& P, const St& S, const TsMem& M) {
    now = 0.0;
    nrand = 0;
    c_act = 0;
    newest = 0;
    nsum = 0;
    act0 = 0;
    hroot = -1;
    hfree = -1;
    hfree2 = -1;
    hused = 0;
    status = 0u;
    dead = 0;
    zt = 0;
    dseq = 0;
    npend = 0;
    steps = 0;
    TVtx& r = M.vtx[0];
    r.serial = 0;
    r.parent = -1;
    r.height = 0;
    r.vote = 0;
    r.who = -1;
    r.depth = 0;
    r.pow = 0;
    r.ddepth = 1;  // dag.ml:29: fold max 0 [] + 1
    r.sum = 0;
    r.nconf = 0;
    r.qslot = -1;
    r.nq = 0;
    r.time = 0.0;
    r.next = -1;
    r.thead = -1;
    set_trec(P, M, r);
    SH(P, M, 0) = -1;
    for (int32_t j = 0; j < P.n; ++j) {
      Vs(P, M, 0, j, V_RECV | V_GOT);
      VT(P, M, 0, j) = 0.0;
      M.tips[j] = 0;
      if (M.nact) M.nact[j] = 0;
    }
    pub = priv = 0;
    ca_a = ca_b = ca_s = -1;
    schedule_pow(P, S, M);
  }

  // Honest.handler (tailstorm.ml:565-608) at defender `node` for vertex x
  __host__ __device__ inline void honest(const TsParams& P, const TsMem& M, int32_t node,
                                         int32_t x) {
    if ((Vg(P, M, x, node) & V_KIND) == V_WH) share(P, M, node, x);
    const TVtx& b = X(P, M, x);
    int32_t& tip = M.tips[node];
    if (!b.vote) {
      tip = update_head(P, M, node, VF_ALL, tip, x);
      return;
    }
    const int32_t s = b.sum;
    int32_t d = -1;
    if (feasible(P, M, node, tip, s)) d = next_summary(P, M, node, s, VF_ALL);
    tip = update_head(P, M, node, VF_ALL, tip, s);
    if (d >= 0) push_now(P, M, mkev(EV_DAG, node, KD_APP), d);
  }

  template <class St>
  __host__ __device__ inline void handle(const TsParams& P, const St& S, const TsMem& M,
                                         uint32_t ev, int32_t s) {
    const uint32_t ty = ev & 7u, kind = (ev >> 3) & 3u;
    const int32_t node = (int32_t)(ev >> 5);
    switch (ty) {
      case EV_MV: {
        const uint8_t v = Vg(P, M, s, node);
        if ((v & V_KIND) != V_INV) break;
        const TVtx& b = X(P, M, s);
        bool ok = true;
        if (b.parent >= 0) {
          if (b.vote) {
            ok = visible(P, M, b.parent, node);
          } else {
            const int32_t* q = Q(P, M, b);
            for (int32_t i = 0; i < b.nq && ok; ++i) ok = visible(P, M, q[i], node);
          }
        }
        if (!ok) break;
        Vs(P, M, s, node, (uint8_t)((v & ~V_KIND) | (kind == KD_NET ? V_RECV : V_WH)));
        VT(P, M, s, node) = now;
        push_now(P, M, mkev(EV_ON, node, kind), s);
        push_now(P, M, mkev(EV_MDV, node, kind), s);
        break;
      }
      case EV_ON: {
        if (node == 0 && P.net != 2) {  // loop mode: the attacker's handler (tailstorm_ssz.ml:353-362)
          prepare(P, M, kind, s);
          if (!dead)
            apply(P, M, P.policy == TS_POLICY_RANDOM ? S.rand_act((uint32_t)nrand++, 8u)
                                                     : ts_policy_p(P, observe(P, M)));
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
          parent = payload_parent(P, M, 0, priv);  // gym: replaced at the Dag event
        } else {
          parent = payload_parent(P, M, m, M.tips[m]);
        }
        push_now(P, M, mkev(EV_DAG, m, KD_POW), parent);
        if (M.nact) ++M.nact[m];
        ++c_act;
        schedule_pow(P, S, M);
        break;
      }
      case EV_DAG: {
        const int32_t v = kind == KD_POW ? append_vote(P, S, M, node, s) : append_summary(P, M, s);
        if (!dead) push_now(P, M, mkev(EV_MV, node, kind), v);
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
        if (!(now < __builtin_inf())) break;  // see bk_lane.h
        const uint8_t v = Vg(P, M, s, node);
        if (!(v & V_GOT)) {
          Vs(P, M, s, node, (uint8_t)(v | V_GOT));
          push_now(P, M, mkev(EV_MV, node, KD_NET), s);
        }
        break;
      }
      case EV_MDV: {
        // children (newest first) already received here: votes on s (in the tree s belongs
        // to, or heads), summaries holding s (child summaries of s's tree); two newest-first
        // lists merged by serial
        const TVtx& sb = X(P, M, s);
        const bool sv = sb.vote != 0;
        int32_t cv = sv ? X(P, M, sb.sum).thead : sb.thead;
        int32_t cq = sv ? SH(P, M, sb.sum) : -1;
        while (!dead) {
          while (cv > s && !(TR(P, M, cv).parent == s && (Vg(P, M, cv, node) & V_GOT)))
            cv = TR(P, M, cv).next;
          while (cq > s && !(Vg(P, M, cq, node) & V_GOT)) cq = TR(P, M, cq).next;
          if (cq > s) {  // summary holding s?
            const TVtx& cb = X(P, M, cq);
            bool child = false;
            const int32_t* q = Q(P, M, cb);
            for (int32_t i = 0; i < cb.nq; ++i) child |= q[i] == s;
            if (!child) {
              cq = cb.next;
              continue;
            }
          }
          if (cv <= s && cq <= s) break;
          int32_t c;
          if (cv > cq) {
            c = cv;
            cv = TR(P, M, cv).next;
          } else {
            c = cq;
            cq = TR(P, M, cq).next;
          }
          push_now(P, M, mkev(EV_MV, node, KD_NET), c);
        }
        break;
      }
    }
  }

  template <class St>
  __host__ __device__ inline bool skip_to_interaction(const TsParams& P, const St& S,
                                                      const TsMem& M, uint32_t* kind,
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
        const int32_t v = append_vote(P, S, M, 0, payload_parent(P, M, 0, priv));
        push_now(P, M, mkev(EV_MV, 0, KD_POW), v);
        continue;
      }
      handle(P, S, M, ev, s);
    }
    return false;
  }

  // Referee.winner (tailstorm.ml:191-194): Compare.first (neg compare_summaries) 1 over
  // [attacker preference; defenders' tips], i.e. the first element after Array.sort
  __host__ __device__ inline int32_t head(const TsParams& P, const TsMem& M, int32_t att) {
    int32_t* v = M.stack;  // n <= 65
    uint64_t* k = M.key;
    for (int32_t j = 0; j < P.n; ++j) {
      const int32_t s = j == 0 ? att : M.tips[j];
      const TVtx& x = X(P, M, s);
      v[j] = s;
      k[j] = ~(((uint64_t)(uint32_t)x.height << 32) | (uint32_t)x.nconf);
    }
    ocaml_heap_sort64(v, k, P.n);
    return v[0];
  }

  template <class St>
  __host__ __device__ inline void gym_reset(const TsParams& P, const St& S, const TsMem& M) {
    init(P, S, M);
    uint32_t kind;
    int32_t b;
    if (skip_to_interaction(P, S, M, &kind, &b)) prepare(P, M, kind, b);
  }

  template <class St>
  __host__ __device__ inline int32_t gym_step(const TsParams& P, const St& S,
                                              const TsMem& M, int32_t action, bool* done) {
    apply(P, M, action);
    ++steps;
    uint32_t kind;
    int32_t b;
    const int32_t att = priv;
    if (!dead && skip_to_interaction(P, S, M, &kind, &b)) prepare(P, M, kind, b);
    const int32_t hd = dead ? 0 : head(P, M, att);
    const double progress = (double)(X(P, M, hd).height * P.k);
    *done = dead || !(steps < P.max_steps && progress < P.max_progress && now < P.max_time);
    return hd;
  }

  template <class St>
  __host__ __device__ inline int32_t loop(const TsParams& P, const St& S, const TsMem& M) {
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
    return dead ? 0 : head(P, M, P.net == 2 ? M.tips[0] : priv);
  }
};

}  // namespace ts
}  // namespace cpr
