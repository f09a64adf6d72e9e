// TEST INFRASTRUCTURE ONLY — CPU oracle, Tailstorm part. See tailstorm.h for the map to
// the reference sources.
#include "tailstorm.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "ocaml_sort.h"

namespace oracle {

static inline bool is_vote(const Block* b) { return b->value.kind == 1; }
static inline bool is_summary(const Block* b) { return b->value.kind == 0; }
static inline int ts_height(const Block* b) { return b->value.height; }
static inline int ts_depth(const Block* b) { return is_vote(b) ? b->value.work : 0; }

// ---------------------------------------------------------------- combinatorics

static int64_t wrap63(__int128 x) {
  // OCaml native ints: 63-bit two's complement
  uint64_t u = (uint64_t)x;
  u <<= 1;
  return ((int64_t)u) >> 1;
}

static int64_t ocaml_factorial(int64_t n) {
  int64_t x = 1;
  for (int64_t i = 2; i <= n; ++i) x = wrap63((__int128)x * i);
  return x;
}

int64_t ocaml_n_choose_k(int64_t n, int64_t k) {
  const int64_t a = ocaml_factorial(n), b = ocaml_factorial(k), c = ocaml_factorial(n - k);
  if (b == 0 || c == 0) throw std::runtime_error("Division_by_zero in Combinatorics.n_choose_k");
  return (a / b) / c;
}

int64_t true_n_choose_k_saturated(int64_t n, int64_t k) {
  if (k < 0 || n < k) return 0;
  if (k > n - k) k = n - k;
  __int128 r = 1;
  for (int64_t i = 1; i <= k; ++i) {
    r = r * (n - k + i) / i;
    if (r > (__int128)INT64_MAX) return INT64_MAX;
  }
  return (int64_t)r;
}

// ---------------------------------------------------------------- referee

// tailstorm.ml:124-130: smaller is better: deeper first, then smaller pow (default min_pow)
int ts_compare_votes_in_block(const Block* a, const Block* b) {
  const int da = ts_depth(a), db = ts_depth(b);
  if (da != db) return db < da ? -1 : 1;  // neg int
  const Pow pa = a->has_pow ? bk_pow(a) : Pow{INT64_MIN, 0};
  const Pow pb = b->has_pow ? bk_pow(b) : Pow{INT64_MIN, 0};
  return pa < pb ? -1 : (pa > pb ? 1 : 0);
}

// acc_votes parents l over the global DAG (referee view)
static BlockSet acc_parents_global(const std::vector<Block*>& l) {
  BlockSet acc;
  std::vector<Block*> st(l.rbegin(), l.rend());
  while (!st.empty()) {
    Block* x = st.back();
    st.pop_back();
    if (!is_vote(x)) continue;
    acc.insert(x);
    for (auto it = x->parents.rbegin(); it != x->parents.rend(); ++it) st.push_back(*it);
  }
  return acc;
}

static Block* last_summary_global(Block* x) {
  while (!is_summary(x)) {
    if (x->parents.size() != 1) throw std::runtime_error("last_summary: votes have one parent");
    x = x->parents[0];
  }
  return x;
}

// tailstorm.ml:156-180
bool ts_validity(const Block* b, int k) {
  if (is_vote(b)) {
    if (b->parents.size() != 1) return false;
    const Block* p = b->parents[0];
    return ts_depth(b) > 0 && b->has_pow && ts_height(b) == ts_height(p) &&
           ts_depth(b) == ts_depth(p) + 1;
  }
  if (b->parents.empty()) return false;
  std::vector<Block*> votes = b->parents;
  // evaluation order of the && chain: height, pow, same_summary, sorted, all votes, unique
  if (!(ts_height(b) > 0)) return false;
  if (b->has_pow) return false;
  {
    Block* parent = last_summary_global(votes[0]);
    for (size_t i = 1; i < votes.size(); ++i)
      if (last_summary_global(votes[i]) != parent) return false;
  }
  for (size_t i = 1; i < votes.size(); ++i)
    if (!(ts_compare_votes_in_block(votes[i - 1], votes[i]) < 0)) return false;
  for (auto* v : votes)
    if (!is_vote(v)) return false;
  if ((int)acc_parents_global(votes).size() != k) return false;
  return ts_height(b) == ts_height(votes[0]) + 1;
}

// tailstorm.ml:204-227: reward' of a summary with parents = first :: _ as all
static std::vector<std::pair<int, double>> reward_list(const std::vector<Block*>& parents,
                                                       bool summary, int scheme, int k,
                                                       const BlockSet& all_votes,
                                                       const BlockSet& first_votes) {
  std::vector<std::pair<int, double>> out;
  if (!summary || parents.empty()) return out;
  const bool discount = scheme == TS_DISCOUNT || scheme == TS_HYBRID;
  const bool punish = scheme == TS_PUNISH || scheme == TS_HYBRID;
  const int depth = ts_depth(parents[0]);
  const double c = 1.;
  const double r = discount ? (double)depth / (double)k * c : c;
  const BlockSet& votes = punish ? first_votes : all_votes;
  for (auto* v : votes) out.push_back({v->value.miner, r});
  return out;
}

void ts_reward(const Block* x, int scheme, int k, std::vector<double>& r) {
  if (!is_summary(x) || x->parents.empty()) return;
  const BlockSet all = acc_parents_global(x->parents);
  const BlockSet first = acc_parents_global({x->parents[0]});
  for (auto& e : reward_list(x->parents, true, scheme, k, all, first)) r[e.first] += e.second;
}

static int global_confirming(Block* b) {
  // acc_votes children (children b) in the global view
  int n = 0;
  std::vector<Block*> st(b->children_app.begin(), b->children_app.end());
  BlockSet seen;
  while (!st.empty()) {
    Block* x = st.back();
    st.pop_back();
    if (!is_vote(x) || seen.count(x)) continue;
    seen.insert(x);
    ++n;
    for (auto* c : x->children_app) st.push_back(c);
  }
  return n;
}

// tailstorm.ml:183-194: Compare.first (neg compare_summaries) 1 l (Array.sort, heap sort)
Block* ts_winner(const std::vector<Block*>& l) {
  for (auto* x : l)
    if (!is_summary(x)) throw std::runtime_error("assert: winner of votes");
  auto cmp = [](Block* a, Block* b) {
    if (a == b) return 0;
    if (ts_height(a) != ts_height(b)) return ts_height(a) < ts_height(b) ? -1 : 1;
    const int ca = global_confirming(a), cb = global_confirming(b);
    return ca < cb ? -1 : (ca > cb ? 1 : 0);
  };
  std::vector<Block*> a = l;
  ocaml_array_sort(a, [&](Block* x, Block* y) { return cmp(y, x); });
  return a[0];
}

// ---------------------------------------------------------------- honest views

std::vector<Block*> TsView::children(const Block* b) const {
  std::vector<Block*> r;
  for (auto it = b->children_app.rbegin(); it != b->children_app.rend(); ++it)
    if (visible(*it)) r.push_back(*it);
  return r;
}

std::vector<Block*> TsView::parents(const Block* b) const {
  std::vector<Block*> r;
  for (auto* p : b->parents)
    if (visible(p)) r.push_back(p);
  return r;
}

Block* TsView::last_summary(Block* x) const {
  while (!is_summary(x)) {
    auto p = parents(x);
    if (p.size() != 1) throw std::runtime_error("last_summary: votes have one parent");
    x = p[0];
  }
  return x;
}

// acc_votes children' (children' b), children' x = children x |> List.filter vf
BlockSet TsView::votes_below(Block* b, const VFilter& vf) const {
  BlockSet acc;
  std::vector<std::vector<Block*>> stack;
  auto kids = [&](Block* x) {
    std::vector<Block*> r;
    for (auto* c : children(x))
      if (!vf || vf(c)) r.push_back(c);
    return r;
  };
  // f acc stack l (tailstorm.ml:134-144); the visit order does not change the set
  std::vector<Block*> work = kids(b);
  while (!work.empty()) {
    Block* x = work.back();
    work.pop_back();
    if (!is_vote(x)) continue;
    if (acc.insert(x).second)
      for (auto* c : kids(x)) work.push_back(c);
  }
  return acc;
}

BlockSet TsView::confirming_votes(Block* b) const {
  if (!is_summary(b)) throw std::runtime_error("assert: confirming_votes of a vote");
  return votes_below(b, nullptr);
}

BlockSet TsView::acc_parents(const std::vector<Block*>& l) const {
  BlockSet acc;
  std::vector<Block*> st(l.begin(), l.end());
  while (!st.empty()) {
    Block* x = st.back();
    st.pop_back();
    if (!is_vote(x)) continue;
    if (acc.insert(x).second)
      for (auto* p : parents(x)) st.push_back(p);
  }
  return acc;
}

// sum of reward' entries for my_id, folded left in list order
double TsView::my_reward_of(const std::vector<Block*>& ps, bool summary) const {
  if (!summary || ps.empty()) return 0.;
  const BlockSet all = acc_parents(ps);
  const BlockSet first = acc_parents({ps[0]});
  double acc = 0.;
  for (auto& e : reward_list(ps, true, scheme, k, all, first))
    if (e.first == view) acc += e.second;
  return acc;
}

// tailstorm.ml:271-313
bool TsView::altruistic(Block* b, const VFilter& vf, std::vector<Block*>* q) const {
  const BlockSet votes = votes_below(b, vf);
  if ((int)votes.size() < k) return false;
  std::vector<Block*> l(votes.begin(), votes.end());
  const int v = view;
  std::stable_sort(l.begin(), l.end(), [this, v](Block* x, Block* y) {
    const int dx = ts_depth(x), dy = ts_depth(y);
    if (dx != dy) return dy < dx;  // neg int
    const int ox = appended_by_me(x) ? 0 : 1, oy = appended_by_me(y) ? 0 : 1;
    if (ox != oy) return ox < oy;
    return float_compare(x->vis[v].time, y->vis[v].time) < 0;
  });
  BlockSet acc;
  int n = 0;
  std::vector<Block*> sel;
  size_t i = 0;
  for (;;) {
    if (n == k) break;
    if (i >= l.size()) return false;
    Block* hd = l[i++];
    BlockSet fresh;
    for (auto* x : acc_parents({hd}))
      if (!acc.count(x)) fresh.insert(x);
    const int nf = (int)fresh.size();
    if (n + nf > k || nf < 1) continue;
    acc.insert(fresh.begin(), fresh.end());
    n += nf;
    sel.push_back(hd);
  }
  std::stable_sort(sel.begin(), sel.end(), [](Block* x, Block* y) {
    const int dx = ts_depth(x), dy = ts_depth(y);
    if (dx != dy) return dy < dx;
    const Pow px = x->has_pow ? bk_pow(x) : bk_max_pow();
    const Pow py = y->has_pow ? bk_pow(y) : bk_max_pow();
    return px < py;
  });
  *q = sel;
  return true;
}

// tailstorm.ml:329-380
bool TsView::heuristic(Block* b, const VFilter& vf, std::vector<Block*>* q) const {
  const BlockSet all_votes = votes_below(b, vf);
  if ((int)all_votes.size() < k) return false;
  BlockSet leaves, votes;
  int n = k;
  auto reward = [&](Block* x, bool all) {
    int i = 0;
    for (auto* y : acc_parents({x}))
      if (!votes.count(y) && (all || appended_by_me(y))) ++i;
    return i;
  };
  while (n > 0) {
    struct C {
      Block* x;
      int own, tot;
    };
    std::vector<C> cs;
    for (auto* x : all_votes) {
      if (votes.count(x)) continue;
      cs.push_back(C{x, reward(x, false), reward(x, true)});
    }
    std::vector<C> fit;
    for (auto& c : cs)
      if (c.tot <= n) fit.push_back(c);
    std::stable_sort(fit.begin(), fit.end(), [](const C& a, const C& b) {
      if (a.own != b.own) return a.own > b.own;
      return a.tot > b.tot;
    });
    if (fit.empty()) throw std::runtime_error("assert false: no branches left");
    Block* x = fit[0].x;
    if (votes.count(x)) throw std::runtime_error("assert: include_ of an included vote");
    leaves.insert(x);
    for (auto* y : acc_parents({x}))
      if (!votes.count(y)) {
        votes.insert(y);
        --n;
      }
    if (n < 0) throw std::runtime_error("assert: !n >= 0");
  }
  std::vector<Block*> l(leaves.begin(), leaves.end());
  std::stable_sort(l.begin(), l.end(), [](Block* x, Block* y) {
    return ts_compare_votes_in_block(x, y) < 0;
  });
  *q = l;
  return true;
}

// tailstorm.ml:418-500 (max_options = 100). The reference visits the k-subsets of the
// candidate votes (BlockSet order) in lexicographic order (iter_n_choose_k), skips the
// ones that are not connected (a vote whose vote parent is not chosen), and keeps the
// first of maximal reward. `brute` = 1 restates that literally. The default enumerates the
// same subsets in the same order but (a) drops a prefix as soon as its newest vote's vote
// parent is not in it — every completion is `Not_connected` — and (b) drops a prefix whose
// best completion cannot reward more than the best so far: own votes chosen plus
// min(slots left, own votes after the prefix's last index), each worth at most the
// largest depth / k (discount) or 1, summed as the reward sums them. A dropped subset is
// either skipped by the reference too or cannot replace its maximum (strict >), so the
// result is the reference's (tests/native/optimal_quorum_bnb.cpp checks it against the
// literal one). The search stops at TS_BRUTE_FORCE_BUDGET prefixes (BudgetExceeded).
// tests (tests/native/optimal_quorum_bnb.cpp): re-derive every pruned search's result by
// the literal enumeration, whose budget they raise
int64_t g_ts_brute_budget = TS_BRUTE_FORCE_BUDGET;
int64_t g_ts_opt_budget = TS_BRUTE_FORCE_BUDGET;
OptimalCheck g_ts_optimal_check;

bool TsView::optimal(Block* b, const VFilter& vf, std::vector<Block*>* q, bool brute) const {
  if (!brute && g_ts_optimal_check.on) {
    std::vector<Block*> q1, q2;
    bool r1 = false, r2 = false, x1 = false, x2 = false;
    g_ts_optimal_check.on = false;
    try {
      r1 = optimal(b, vf, &q1, false);
    } catch (BudgetExceeded&) {
      x1 = true;
    } catch (std::exception& ex) {
      fprintf(stderr, "OPTCHECK: pruned search raised %s (n = %d, k = %d)\n", ex.what(),
              (int)votes_below(b, vf).size(), k);
      g_ts_optimal_check.on = true;
      throw;
    }
    bool e2 = false;
    try {
      r2 = optimal(b, vf, &q2, true);
    } catch (BudgetExceeded&) {
      x2 = true;
    } catch (std::exception& ex) {
      e2 = true;
      fprintf(stderr, "OPTCHECK: literal search raised %s (n = %d, k = %d)\n", ex.what(),
              (int)votes_below(b, vf).size(), k);
    }
    if (e2) ++g_ts_optimal_check.mismatches;
    if (x2) ++g_ts_optimal_check.unverified;
    g_ts_optimal_check.on = true;
    if (!x2) {
      ++g_ts_optimal_check.compared;
      const int64_t nv = (int64_t)votes_below(b, vf).size();
      // (the literal search completed, so n_choose_k did not raise)
      if (nv >= k && ocaml_n_choose_k(nv, k) <= 100 &&
          true_n_choose_k_saturated(nv, k) > TS_BRUTE_FORCE_BUDGET)
        ++g_ts_optimal_check.large;
      if (x1 || r1 != r2 || q1 != q2) ++g_ts_optimal_check.mismatches;
    }
    if (x1) throw BudgetExceeded();
    *q = q1;
    return r1;
  }
  const BlockSet votes = votes_below(b, vf);
  std::vector<Block*> a(votes.begin(), votes.end());
  const int n = (int)a.size();
  if (ocaml_n_choose_k(n, k) > 100) return heuristic(b, vf, q);
  if (n < k) return false;
  if (brute && true_n_choose_k_saturated(n, k) > g_ts_brute_budget) throw BudgetExceeded();
  auto index_of = [&](Block* x) {
    for (int i = 0; i < n; ++i)
      if (a[i] == x) return i;
    throw std::runtime_error("Not_found in BlockMap");
  };
  // vote parent's index (-1: a summary), own flags, own votes after each index
  std::vector<int> par(n, -1), own(n), own_after(n + 1, 0);
  int maxdepth = 0;
  for (int i = 0; i < n; ++i) {
    for (auto* p : parents(a[i]))
      if (is_vote(p)) par[i] = index_of(p);
    own[i] = a[i]->value.miner == view ? 1 : 0;
    maxdepth = std::max(maxdepth, ts_depth(a[i]));
  }
  for (int i = n - 1; i >= 0; --i) own_after[i] = own_after[i + 1] + own[i];
  const bool discount = scheme == TS_DISCOUNT || scheme == TS_HYBRID;
  const double rmax = discount ? (double)maxdepth / (double)k * 1. : 1.;
  std::vector<double> bound(k + 1, 0.);  // bound[m] = rmax added m times
  for (int m = 1; m <= k; ++m) bound[m] = bound[m - 1] + rmax;
  std::vector<char> reach(n), leave(n), chosen(n, 0);
  double opt_reward = -1.;
  bool have = false;
  std::vector<Block*> best;
  std::vector<int> c(k);
  int64_t visits = 0;
  std::function<void(int, int, int)> iter = [&](int s, int j, int ownp) {
    if (j == k) {
      std::fill(reach.begin(), reach.end(), 0);
      std::fill(leave.begin(), leave.end(), 1);
      for (int t = 0; t < k; ++t) {
        const int hd = c[t];
        bool ok = true;
        for (auto* p : parents(a[hd])) {
          if (!is_vote(p)) continue;
          const int ip = index_of(p);
          leave[ip] = 0;
          if (!reach[ip]) {
            ok = false;
            break;
          }
        }
        if (!ok) return;  // `Not_connected
        reach[hd] = 1;
      }
      std::vector<Block*> lv;
      for (int i = 0; i < n; ++i)
        if (reach[i] && leave[i]) lv.push_back(a[i]);
      std::stable_sort(lv.begin(), lv.end(), [](Block* x, Block* y) {
        return ts_compare_votes_in_block(x, y) < 0;
      });
      const double r = my_reward_of(lv, true);
      if (r > opt_reward) {
        opt_reward = r;
        best = lv;
        have = true;
      }
      return;
    }
    // the literal enumeration tries every index (a prefix that cannot reach k positions
    // enumerates nothing); the pruned search, like ts_lane.h TsLane::optimal, only indices
    // from which k - j positions remain, so both count the same visits
    const int last = brute ? n - 1 : n - (k - j);
    for (int i = s; i <= last; ++i) {
      if (!brute) {
        if (par[i] >= 0 && !chosen[par[i]]) continue;  // every completion Not_connected
        const int cap = ownp + own[i] + std::min(k - j - 1, own_after[i + 1]);
        if (have && bound[cap] <= opt_reward) continue;  // cannot beat the best
        if (++visits > g_ts_opt_budget) throw BudgetExceeded();
      }
      c[j] = i;
      chosen[i] = 1;
      iter(i + 1, j + 1, ownp + own[i]);
      chosen[i] = 0;
    }
  };
  iter(0, 0, 0);
  if (!have) throw std::runtime_error("reward_optim_quorum: no choice");
  *q = best;
  return true;
}

bool TsView::quorum(Block* b, const VFilter& vf, std::vector<Block*>* q) const {
  switch (selection) {
    case TS_ALTRUISTIC: return altruistic(b, vf, q);
    case TS_OPTIMAL: return optimal(b, vf, q);
    default: return heuristic(b, vf, q);
  }
}

// tailstorm.ml:509-526
Draft TsView::puzzle_payload(Block* b, const VFilter& vf) const {
  if (!is_summary(b)) throw std::runtime_error("assert: puzzle_payload on a vote");
  const BlockSet vs = votes_below(b, vf);
  std::vector<Block*> l(vs.begin(), vs.end());
  std::stable_sort(l.begin(), l.end(), [](Block* x, Block* y) {
    return ts_compare_votes_in_block(x, y) < 0;
  });
  Block* parent = l.empty() ? b : l[0];
  Draft d;
  d.parents = {parent};
  d.sign = false;
  d.data = NakData{ts_height(b), view, ts_depth(parent) + 1, 1};
  return d;
}

// tailstorm.ml:530-535
bool TsView::next_summary(Block* b, const VFilter& vf, Draft* d) const {
  std::vector<Block*> q;
  if (!quorum(b, vf, &q)) return false;
  d->parents = q;
  d->data = NakData{ts_height(b) + 1, -1, 0, 0};
  d->sign = false;
  return true;
}

// tailstorm.ml:539-550
int TsView::compare_blocks(const VFilter& vf, Block* a, Block* b) const {
  if (a == b) return 0;
  if (ts_height(a) != ts_height(b)) return ts_height(a) < ts_height(b) ? -1 : 1;
  auto count = [&](Block* x) {
    int n = 0;
    for (auto* v : confirming_votes(x))
      if (!vf || vf(v)) ++n;
    return n;
  };
  const int ca = count(a), cb = count(b);
  if (ca != cb) return ca < cb ? -1 : 1;
  const double ra = my_reward_of(parents(a), true), rb = my_reward_of(parents(b), true);
  return float_compare(ra, rb);
}

Block* TsView::update_head(const VFilter& vf, Block* old, Block* consider) const {
  if (!is_summary(consider)) throw std::runtime_error("assert: update_head with a vote");
  return compare_blocks(vf, consider, old) > 0 ? consider : old;
}

// tailstorm.ml:557-563
bool TsView::summary_feasible(Block* preferred, Block* after) const {
  const bool has_conf = !children(preferred).empty();
  const int ext = ts_height(after) + 1, cur = ts_height(preferred);
  return cur < ext || (cur == ext && !has_conf);
}

Draft TsHonest::puzzle_payload() { return V().puzzle_payload(state, nullptr); }

// tailstorm.ml:565-608
Action TsHonest::handler(Kind, Block* x) {
  const TsView v = V();
  Action a;
  if (x->vis[id].kind == WITHHELD) a.share.push_back(x);
  if (is_summary(x)) {
    state = v.update_head(nullptr, state, x);
    return a;
  }
  Block* s = v.last_summary(x);
  if (v.summary_feasible(state, s)) {
    Draft d;
    if (v.next_summary(s, nullptr, &d)) a.append.push_back(d);
  }
  state = v.update_head(nullptr, state, s);
  return a;
}

// ---------------------------------------------------------------- policies / observation

// tailstorm_ssz.ml:365-446; Action8 ranks (ssz_tools.ml:230-263)
int ts_policy(int policy, const TsObs& o, int k) {
  const int h = o.public_blocks, a = o.private_blocks;
  const int hp = h * k + o.public_votes, ap = a * k + o.private_votes_inclusive;
  switch (policy) {
    case TSPOL_HONEST: return h > a ? ADOPT_PROCEED : OVERRIDE_PROCEED;
    case TSPOL_GET_AHEAD:
      return h > a ? ADOPT_PROCEED : (h < a ? OVERRIDE_PROCEED : WAIT_PROCEED);
    case TSPOL_MINOR_DELAY:
      return h > a ? ADOPT_PROCEED : (h == 0 ? WAIT_PROCEED : OVERRIDE_PROCEED);
    case TSPOL_LONG_DELAY:
      if (h > a) return ADOPT_PROCEED;
      if (h == 0) return WAIT_PROCEED;
      if (h + 10 < a) return OVERRIDE_PROCEED;
      if (h * k + o.public_votes + 1 < a * k + o.private_votes_inclusive) return WAIT_PROCEED;
      return OVERRIDE_PROCEED;
    case TSPOL_AVOID_LOSS_A:
      if (a < h) return ADOPT_PROCEED;
      if (h == 0) return WAIT_PROCEED;
      if (o.private_votes_inclusive == 0 && a == h + 1) return OVERRIDE_PROCEED;
      if (h == a && o.private_votes_inclusive == o.public_votes + 1) return OVERRIDE_PROCEED;
      if (a - h > 10) return OVERRIDE_PROCEED;
      return WAIT_PROCEED;
    case TSPOL_AVOID_LOSS:
    case TSPOL_AVOID_LOSS_B:
      if (h == 0) return WAIT_PROCEED;
      if (h == 1 && hp == ap) return policy == TSPOL_AVOID_LOSS ? MATCH_PROCEED : OVERRIDE_PROCEED;
      if (hp > ap) return ADOPT_PROCEED;
      if (hp == ap - 1) return OVERRIDE_PROCEED;
      if (h < a - 10) return OVERRIDE_PROCEED;
      return WAIT_PROCEED;
  }
  throw std::invalid_argument("unknown policy");
}

// NormalizeObs with tailstorm_ssz.ml:41-55 normalizers (fields 3..8 scale k)
void ts_obs_to_floats(const TsObs& o, bool unit, int k, double out[TS_OBS_LEN]) {
  const int v[TS_OBS_LEN] = {o.public_blocks,           o.private_blocks,
                             o.diff_blocks,             o.public_votes,
                             o.private_votes_inclusive, o.private_votes_exclusive,
                             o.public_depth,            o.private_depth_inclusive,
                             o.private_depth_exclusive, o.event};
  for (int i = 0; i < TS_OBS_LEN; ++i) {
    if (i == 9) {
      out[i] = unit ? (double)v[i] / 2. : (double)v[i];
    } else if (!unit) {
      out[i] = (double)v[i];
    } else {
      const double scale = i >= 3 ? (double)k : 1.;
      out[i] = i == 2 ? 0.5 + (1. / M_PI * std::atan((double)v[i] / scale))
                      : 2. / M_PI * std::atan((double)v[i] / scale);
    }
  }
}

TsObs ts_obs_of_floats(const double in[TS_OBS_LEN], bool unit, int k) {
  int v[TS_OBS_LEN];
  for (int i = 0; i < TS_OBS_LEN; ++i) {
    if (i == 9) {
      v[i] = unit ? (int)std::floor(in[i] * 2.) : (int)in[i];
    } else if (!unit) {
      v[i] = (int)in[i];
    } else {
      const double scale = i >= 3 ? (double)k : 1.;
      v[i] = i == 2 ? (int)std::round(std::tan(M_PI * (in[i] - 0.5)) * scale)
                    : (int)std::round(std::tan(M_PI / 2. * in[i]) * scale);
    }
  }
  return TsObs{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9]};
}

// ---------------------------------------------------------------- agent

Draft TsSszAgent::puzzle_payload() const { return V().puzzle_payload(priv, nullptr); }

static VFilter public_vis(int view) {
  return [view](Block* x) {
    return x->vis[view].kind == RELEASED || x->vis[view].kind == RECEIVED;
  };
}

// tailstorm_ssz.ml:210-258
void TsSszAgent::prepare(Kind kd, Block* x) {
  const TsView v = V();
  const VFilter pv = public_vis(my_id);
  Block* p = pub;
  for (auto* m : pending) p = v.update_head(pv, p, v.last_summary(m));
  Block* q = priv;
  switch (kd) {
    case K_APPEND:
      if (!is_summary(x)) throw std::runtime_error("assert: Append of a vote");
      q = v.update_head(nullptr, priv, x);
      o_event = 0;
      break;
    case K_POW: o_event = 1; break;
    case K_NETWORK:
      p = v.update_head(pv, p, is_summary(x) ? x : v.last_summary(x));
      o_event = 2;
      break;
  }
  o_pub = p;
  o_priv = q;
  o_common = common_ancestor(*sim, my_id, p, q);
  if (!o_common) throw std::runtime_error("Option.get: no common ancestor");
}

// tailstorm_ssz.ml:262-290
TsObs TsSszAgent::observe() const {
  const TsView v = V();
  TsObs o{};
  for (auto* x : v.confirming_votes(o_pub))
    if (x->vis[my_id].kind == RELEASED || x->vis[my_id].kind == RECEIVED) {
      o.public_depth = std::max(o.public_depth, ts_depth(x));
      ++o.public_votes;
    }
  for (auto* x : v.confirming_votes(o_priv)) {
    o.private_depth_inclusive = std::max(o.private_depth_inclusive, ts_depth(x));
    ++o.private_votes_inclusive;
    if (v.appended_by_me(x)) {
      o.private_depth_exclusive = std::max(o.private_depth_exclusive, ts_depth(x));
      ++o.private_votes_exclusive;
    }
  }
  const int ca = ts_height(o_common), ph = ts_height(o_priv), qh = ts_height(o_pub);
  o.private_blocks = ph - ca;
  o.public_blocks = qh - ca;
  o.diff_blocks = ph - qh;
  o.event = o_event;
  return o;
}

// tailstorm_ssz.ml:292-350
Action TsSszAgent::apply(int action) {
  if (action < 0 || action >= BK_N_ACTIONS) throw std::invalid_argument("index out of bounds");
  const TsView v = V();
  const int vw = my_id;
  auto release = [&](bool override_) {
    // Dagtools.iterate_descendants ~include_start:true [common]: ascending (depth, serial)
    BlockSet desc;
    std::vector<Block*> st{o_common};
    while (!st.empty()) {
      Block* x = st.back();
      st.pop_back();
      if (!desc.insert(x).second) continue;
      for (auto* c : v.children(x)) st.push_back(c);
    }
    BlockSet now;
    for (Block* x : desc) {
      if (x->vis[vw].kind == RELEASED || x->vis[vw].kind == RECEIVED) continue;
      BlockSet now2 = now;
      now2.insert(x);
      const VFilter vf = [vw, &now2](Block* y) {
        return y->vis[vw].kind == RELEASED || y->vis[vw].kind == RECEIVED || now2.count(y) > 0;
      };
      if (v.update_head(vf, o_pub, v.last_summary(x)) == o_pub) return override_ ? now2 : now;
      now = now2;
    }
    return now;  // override/match not possible; release all
  };
  Action a;
  Block* np = o_priv;
  BlockSet rel;
  switch (action % 4) {
    case 0: np = o_pub; break;
    case 1: rel = release(true); break;
    case 2: rel = release(false); break;
    default: break;
  }
  a.share.assign(rel.begin(), rel.end());
  VFilter vf = nullptr;
  if (action < 4) vf = [this](Block* y) { return V().appended_by_me(y); };
  Block* extend;
  if (v.children(o_priv).empty()) {
    auto ps = v.parents(o_priv);
    if (ps.empty()) throw std::runtime_error("List.hd: summary without parents");
    extend = v.last_summary(ps[0]);
  } else {
    extend = o_priv;
  }
  Draft d;
  if (v.next_summary(extend, vf, &d)) a.append.push_back(d);
  pub = o_pub;
  priv = np;
  pending = a.share;
  return a;
}

Action TsSszAttackerNode::handler(Kind kd, Block* b) {
  agent.prepare(kd, b);
  if (policy == TS_POL_RANDOM) return agent.apply(agent.sim->rng->rand_action(nrand++, 8));
  return agent.apply(ts_policy(policy, agent.observe(), agent.k, table));
}

int ts_policy(int policy, const TsObs& o, int k, const TsTable* t) {
  if (policy != TS_POL_TABLE) return ts_policy(policy, o, k);
  auto cl = [](int x, int hi) { return x < 0 ? 0 : (x > hi ? hi : x); };
  const int D = t->dim, K1 = k + 1;
  return t->actions[((((cl(o.public_blocks, D - 1) * D + cl(o.private_blocks, D - 1)) * K1 +
                       cl(o.public_votes, k)) * K1 + cl(o.private_votes_inclusive, k)) * 3) +
                    o.event];
}

// ---------------------------------------------------------------- gym engine

GymTailstorm::GymTailstorm(const GymParams& p_, int k_, int scheme_, int selection_, int mode,
                           OcamlRandom* oc, uint64_t seed_, uint64_t ep)
    : p(p_), k(k_), scheme(scheme_), selection(selection_), rng_mode(mode), ocaml(oc),
      seed(seed_), episode(ep) {
  std::string e = gym_params_error(p);
  if (!e.empty()) throw std::invalid_argument(e);
  if (k < 1) throw std::invalid_argument("k must be positive");
  net = Network::selfish_mining(p.alpha, p.activation_delay, p.gamma, p.propagation_delay,
                                p.defenders);
}

Kind GymTailstorm::skip_to_interaction(Block** blk) {
  Event ev;
  for (;;) {
    if (!sim->dequeue(&ev)) throw std::runtime_error("simulation should continue forever");
    if (ev.type == EV_ONNODE && ev.node == 0) {
      *blk = ev.blk;
      return ev.kind;
    }
    if (ev.type == EV_DAG && ev.node == 0 && ev.kind == K_POW) {
      Draft d = agent.puzzle_payload();
      Block* v = sim->append(true, 0, d);
      sim->schedule_now(Event{EV_MAKEVIS, 0, K_POW, v, -1});
      continue;
    }
    sim->handle_event(ev);
  }
}

static std::unique_ptr<SimRng> make_ts_rng(int rng_mode, OcamlRandom* oc, uint64_t seed,
                                           uint64_t ep, const Network& net) {
  if (rng_mode == 0)
    return trace_wrap(std::unique_ptr<SimRng>(new OcamlSimRng(oc, net)), net, true);
  auto* r = new KeyedSimRng(seed, ep, net, needs_general_weights(net));
  r->serial_links = true;
  return trace_wrap(std::unique_ptr<SimRng>(r), net, true);
}

static void setup_sim(Sim& s, int k, int scheme) {
  s.proto = 3;
  s.bk_k = k;
  s.bk_scheme = scheme;
}

void GymTailstorm::init() {
  rng = make_ts_rng(rng_mode, ocaml, seed, episode, net);
  sim.reset(new Sim(net, rng.get()));
  setup_sim(*sim, k, scheme);
  std::vector<std::unique_ptr<NodeImpl>> nodes;
  const int n = (int)net.nodes.size();
  for (int i = 0; i < n; i++) {
    if (i == 0) {
      nodes.emplace_back(new DummyNode());
    } else {
      auto* h = new TsHonest();
      h->scheme = scheme;
      h->selection = selection;
      nodes.emplace_back(h);
    }
  }
  sim->init(std::move(nodes));
  Block* root = sim->roots.back();
  static_cast<DummyNode*>(sim->nodes[0].get())->state = root;
  for (int i = 1; i < n; i++) static_cast<TsHonest*>(sim->nodes[i].get())->state = root;
  agent = TsSszAgent();
  agent.sim = sim.get();
  agent.my_id = 0;
  agent.k = k;
  agent.scheme = scheme;
  agent.selection = selection;
  agent.init(root);
  Block* b;
  Kind kd = skip_to_interaction(&b);
  agent.prepare(kd, b);
  episode_steps = 0;
  last_progress = last_chain_time = last_sim_time = last_reward_attacker =
      last_reward_defender = 0.;
}

void GymTailstorm::observe(double obs[TS_OBS_LEN]) const {
  ts_obs_to_floats(agent.observe(), p.unit_obs, k, obs);
}

void GymTailstorm::reset(double obs[TS_OBS_LEN]) {
  init();
  observe(obs);
}

double GymTailstorm::step(int action, double obs[TS_OBS_LEN], bool* done, StepInfo* info) {
  Action act = agent.apply(action);
  sim->handle_action(0, act);
  episode_steps++;
  Block* b;
  Kind kd = skip_to_interaction(&b);
  Block* attacker_pref = agent.priv;
  agent.prepare(kd, b);
  std::vector<Block*> prefs;
  prefs.push_back(attacker_pref);
  for (int i = 1; i < sim->n_nodes; i++) prefs.push_back(sim->nodes[i]->preferred());
  Block* head = ts_winner(prefs);
  const double progress = sim->progress(head);
  *done = !(episode_steps < p.max_steps && progress < p.max_progress && sim->now < p.max_time);
  double ra = 0., rd = 0.;
  for (int i = 0; i < sim->n_nodes; i++) {
    if (i == 0)
      ra += head->rewards[i];
    else
      rd += head->rewards[i];
  }
  const double chain_time = Sim::timestamp(head);
  const double sim_time = sim->now;
  const double reward = ra - last_reward_attacker;
  if (info) {
    info->step_reward_attacker = ra - last_reward_attacker;
    info->step_reward_defender = rd - last_reward_defender;
    info->step_progress = progress - last_progress;
    info->step_chain_time = chain_time - last_chain_time;
    info->step_sim_time = sim_time - last_sim_time;
    info->episode_reward_attacker = ra;
    info->episode_reward_defender = rd;
    info->episode_progress = progress;
    info->episode_chain_time = chain_time;
    info->episode_sim_time = sim_time;
    info->episode_n_steps = episode_steps;
    info->episode_n_activations = sim->c_activations;
    info->head_height = head->value.height;
    info->head_miner = -1;  // summaries have no miner (tailstorm.ml:89-94)
    info->head_work = 0;
  }
  last_chain_time = chain_time;
  last_sim_time = sim_time;
  last_reward_attacker = ra;
  last_reward_defender = rd;
  last_progress = progress;
  observe(obs);
  return reward;
}

void ts_loop_task(const Network& net, int rng_mode, OcamlRandom* r, uint64_t seed,
                  uint64_t episode, int k, int scheme, int selection, int policy,
                  int activations, TsLoopResult* out, const TsTable* table) {
  std::unique_ptr<SimRng> rng = make_ts_rng(rng_mode, r, seed, episode, net);
  Sim sim(net, rng.get());
  setup_sim(sim, k, scheme);
  sim.zt_limit = 4096;
  const int n = (int)net.nodes.size();
  std::vector<std::unique_ptr<NodeImpl>> nodes;
  TsSszAttackerNode* att = nullptr;
  for (int i = 0; i < n; ++i) {
    if (i == 0 && policy >= 0) {
      att = new TsSszAttackerNode();
      att->policy = policy;
      att->table = table;
      nodes.emplace_back(att);
    } else {
      auto* h = new TsHonest();
      h->scheme = scheme;
      h->selection = selection;
      nodes.emplace_back(h);
    }
  }
  sim.init(std::move(nodes));
  Block* root = sim.roots.back();
  for (int i = 0; i < n; ++i) {
    if (i == 0 && att) {
      att->agent.sim = &sim;
      att->agent.my_id = 0;
      att->agent.k = k;
      att->agent.scheme = scheme;
      att->agent.selection = selection;
      att->agent.init(root);
    } else {
      static_cast<TsHonest*>(sim.nodes[i].get())->state = root;
    }
  }
  sim.loop(activations);
  std::vector<Block*> prefs;
  for (auto& nd : sim.nodes) prefs.push_back(nd->preferred());
  Block* h = ts_winner(prefs);
  out->activations.assign(sim.activations.begin(), sim.activations.end());
  out->rewards = h->rewards;
  out->head_time = Sim::timestamp(h);
  out->head_progress = sim.progress(h);
  out->head_height = h->value.height;
  out->n_vertices = (int64_t)sim.dag.size();
}

}  // namespace oracle
