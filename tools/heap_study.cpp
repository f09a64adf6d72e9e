// Study (not product code): the Ethereum lane's event-queue operation sequence on gym
// episodes, replayed through (a) the reference's skew heap (orderedQueue.ml:17-47) with
// every element explicit, and (b) the same heap with its +inf subtrees held compressed:
// a subtree of +inf elements whose shape is a Braun tree (sizes of the two children
// differ by at most one, left >= right) is one handle carrying its size. Both must pop the
// same elements in the same order; the study counts node visits per step in each.
//
// build: hipcc -O2 -std=c++17 -ffp-contract=off -x hip --offload-arch=gfx950 -I. \
//        tools/heap_study.cpp -o build/heap_study
// usage: build/heap_study [episodes] [gamma] [policy] [alpha]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

static std::vector<std::pair<int, double>>* g_log = nullptr;
#define CPR_HEAP_HOOK(op, t) \
  do {                         \
    if (g_log) g_log->push_back({(op), (t)}); \
  } while (0)
#include "../cpr_amd/csrc/ethereum_lane.h"
#include "../oracle/src/keyed_stream.h"

using namespace cpr;

// ---------------------------------------------------------------- (a) explicit heap
struct Plain {
  struct N {
    double t;
    int id, l, r;
  };
  std::vector<N> n;
  int root = -1;
  long visits = 0, inf_visits = 0;
  void push(double t, int id) {
    int par = -1, node = root;
    for (;;) {
      if (node < 0) {
        n.push_back({t, id, -1, -1});
        const int a = (int)n.size() - 1;
        if (par < 0) root = a; else n[par].l = a;
        return;
      }
      ++visits;
      if (std::isinf(n[node].t)) ++inf_visits;
      N& h = n[node];
      if (t < h.t) {
        std::swap(t, h.t);
        std::swap(id, h.id);
      } else {
        std::swap(h.l, h.r);
      }
      par = node;
      node = h.l;
    }
  }
  bool pop(double* t, int* id) {
    if (root < 0) return false;
    *t = n[root].t;
    *id = n[root].id;
    int par = -1, side = 0, node = root;
    for (;;) {
      ++visits;
      if (std::isinf(n[node].t)) ++inf_visits;
      const int l = n[node].l, r = n[node].r;
      int repl = -2;
      if (r < 0) repl = l; else if (l < 0) repl = r;
      if (repl != -2) {
        if (par < 0) root = repl; else if (side == 0) n[par].l = repl; else n[par].r = repl;
        return true;
      }
      const int c = n[l].t <= n[r].t ? l : r;
      n[node].t = n[c].t;
      n[node].id = n[c].id;
      par = node;
      side = c == l ? 0 : 1;
      node = c;
    }
  }
};

// ---------------------------------------------------------------- (b) compressed heap
// handle h: h >= 0 explicit node; h == -1 empty; h <= -2 Braun tree of +inf, size -h - 1
struct Comp {
  struct N {
    double t;  // +inf: an explicit +inf node (shape only)
    int id, l, r;
  };
  std::vector<N> n;
  std::vector<int> freel;
  long visits = 0;
  int live = 0, max_live = 0;
  int root = -1;
  static int braun(int s) { return -s - 1; }
  static bool is_b(int h) { return h <= -1; }  // empty counts as Braun(0)
  static int bsize(int h) { return -h - 1; }
  int alloc(double t, int id, int l, int r) {
    int i;
    if (!freel.empty()) { i = freel.back(); freel.pop_back(); n[i] = {t, id, l, r}; }
    else { n.push_back({t, id, l, r}); i = (int)n.size() - 1; }
    if (++live > max_live) max_live = live;
    return i;
  }
  void release(int i) { freel.push_back(i); --live; }
  double root_t(int h) const { return h >= 0 ? n[h].t : __builtin_inf(); }
  // explicit +inf node over (l, r): collapses to a Braun handle when the shape is Braun
  int mk_inf(int node, int l, int r) {
    if (is_b(l) && is_b(r)) {
      const int a = bsize(l), b = bsize(r);
      if (a == b || a == b + 1) {
        if (node >= 0) release(node);
        return braun(a + b + 1);
      }
    }
    if (node < 0) node = alloc(__builtin_inf(), -1, l, r);
    else { n[node].t = __builtin_inf(); n[node].l = l; n[node].r = r; }
    return node;
  }
  int ins_inf(int h) {
    if (is_b(h)) return braun(bsize(h) + 1);
    ++visits;
    const int l = n[h].l, r = n[h].r;
    return mk_inf(h, ins_inf(r), l);
  }
  int insert(double t, int id, int h) {
    if (std::isinf(t) && h < 0) return ins_inf(h);
    if (h == -1) return alloc(t, id, -1, -1);
    if (h <= -2) {  // finite element at the root of a Braun +inf tree
      const int s = bsize(h);
      const int a = s / 2, b = (s - 1) / 2;  // ceil((s-1)/2), floor((s-1)/2)
      return alloc(t, id, ins_inf(braun(a) == -1 ? -1 : braun(a)), b ? braun(b) : -1);
    }
    ++visits;
    N& x = n[h];
    if (std::isinf(x.t)) {
      if (std::isinf(t)) return ins_inf(h);
      const int l = x.l, r = x.r;
      n[h].t = t; n[h].id = id; n[h].l = ins_inf(l); n[h].r = r;
      return h;
    }
    if (t < x.t) {
      const double ot = x.t; const int oid = x.id;
      n[h].t = t; n[h].id = id;
      const int nl = insert(ot, oid, n[h].l);
      n[h].l = nl;
    } else {
      const int l = n[h].l;
      const int nl = insert(t, id, n[h].r);
      n[h].l = nl;
      n[h].r = l;
    }
    return h;
  }
  int rem_inf(int h) {  // remove the root element of a +inf tree
    if (h <= -2) {
      const int s = bsize(h);
      if (s == 1) return -1;
      const int a = s / 2, b = (s - 1) / 2;
      if (b == 0) return braun(a);
      return mk_inf(-1, rem_inf(braun(a)), braun(b));
    }
    ++visits;
    const int l = n[h].l, r = n[h].r;
    if (r == -1) { release(h); return l; }
    if (l == -1) { release(h); return r; }
    return mk_inf(h, rem_inf(l), r);
  }
  int remove(int h) {  // h explicit with a finite root
    ++visits;
    const int l = n[h].l, r = n[h].r;
    if (r == -1) { release(h); return l; }
    if (l == -1) { release(h); return r; }
    const double lt = root_t(l), rt = root_t(r);
    if (lt <= rt) {
      if (std::isinf(lt)) return mk_inf(h, rem_inf(l), r);
      n[h].t = n[l].t; n[h].id = n[l].id;
      const int nl = remove(l);
      n[h].l = nl;
    } else {
      n[h].t = n[r].t; n[h].id = n[r].id;
      const int nr = remove(r);
      n[h].r = nr;
    }
    return h;
  }
  void push(double t, int id) { root = insert(t, id, root); }
  bool pop(double* t, int* id) {
    if (root == -1) return false;
    if (root <= -2 || std::isinf(n[root].t)) {
      *t = __builtin_inf(); *id = -1;
      root = rem_inf(root);
      return true;
    }
    *t = n[root].t; *id = n[root].id;
    root = remove(root);
    return true;
  }
};

int main(int argc, char** argv) {
  const int episodes = argc > 1 ? atoi(argv[1]) : 200;
  const double gamma = argc > 2 ? atof(argv[2]) : 0.0;
  const int policy = argc > 3 ? atoi(argv[3]) : 0;
  const double alpha = argc > 4 ? atof(argv[4]) : 0.33;
  const int steps = 2016, d = 2;
  eth::EthParams P{};
  P.t_att = oracle::alpha_threshold(alpha);
  P.d = d; P.n = d + 1; P.net = 0; P.mode = 0; P.nak = 0; P.policy = policy; P.scheme = 0;
  P.cap_b = 1;
  while (P.cap_b < steps + 2) P.cap_b <<= 1;
  P.cap_e = 64 + 512 * P.n + 2 * P.d * steps;
  P.ev = 1.0; P.delta = 1e-9; P.dmax = 0.5 * 1e-9 / gamma;
  P.max_steps = steps; P.activations = steps;
  P.max_progress = __builtin_inf(); P.max_time = __builtin_inf();
  std::vector<uint8_t> mem(eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  long pa = 0, pinf = 0, cv = 0, ops = 0, bad = 0, maxlive = 0, maxsize = 0;
  for (int e = 0; e < episodes; ++e) {
    std::vector<std::pair<int, double>> log;
    g_log = &log;
    const eth::EthMem M = eth::eth_mem_at(mem.data(), P.cap_b, P.cap_e, P.n);
    const Stream S{0x5EED0000u, 0u, (uint32_t)e, 0u};
    eth::EthLane L;
    L.gym_reset(P, S, M);
    for (int s = 0; s < steps; ++s) {
      const eth::EthObs o = L.observe(P, M, false);
      bool done = false;
      L.gym_step(P, S, M, eth::eth_policy(P.policy, o), &done);
      if (done) break;
    }
    g_log = nullptr;
    Plain A;
    Comp B;
    int id = 0, size = 0;
    for (auto& [op, t] : log) {
      ++ops;
      if (op == 0) {
        A.push(t, id); B.push(t, id); ++id; ++size;
        if (size > maxsize) maxsize = size;
      } else {
        double ta, tb; int ia, ib;
        A.pop(&ta, &ia); B.pop(&tb, &ib);
        --size;
        if (ta != t || tb != t || (!std::isinf(t) && ia != ib)) ++bad;
      }
    }
    pa += A.visits; pinf += A.inf_visits; cv += B.visits;
    if (B.max_live > maxlive) maxlive = B.max_live;
  }
  printf("{\"episodes\": %d, \"gamma\": %g, \"policy\": %d, \"ops\": %ld, \"mismatch\": %ld, "
         "\"plain_visits_per_step\": %.1f, \"plain_inf_visits_per_step\": %.1f, "
         "\"compressed_visits_per_step\": %.1f, \"compressed_max_explicit\": %ld, "
         "\"max_heap_size\": %ld}\n",
         episodes, gamma, policy, ops, bad, pa / (double)(episodes * steps),
         pinf / (double)(episodes * steps), cv / (double)(episodes * steps), maxlive, maxsize);
  return bad ? 1 : 0;
}
