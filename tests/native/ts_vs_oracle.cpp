// TEST INFRASTRUCTURE ONLY. Differential fuzzer for the Tailstorm lane
// (cpr_amd/csrc/ts_lane.h, compiled here for the host) against the CPU oracle's
// restatement (oracle/src/tailstorm.cpp), step by step on the same keyed stream: all ten
// observation fields and the step info after every step; loop-mode tasks on the
// two-agents network compared at the end. Episodes in which the reference raises
// (oracle exception) must be flagged CPR_ST_REFERENCE_RAISES by the lane at the same step.
// Prints one JSON summary line; exit code 1 on any mismatch.
// Usage: ts_vs_oracle [episodes per config] [steps] [k] [selection]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "garbage.h"
#include "../../cpr_amd/csrc/ts_lane.h"
#include "../../oracle/src/tailstorm.h"

using namespace cpr;

static uint32_t mix(uint64_t a, uint64_t b) {
  uint64_t x = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull);
  x ^= x >> 31;
  x *= 0xD6E8FEB86659FD93ull;
  x ^= x >> 32;
  return (uint32_t)x;
}

struct Cfg {
  double alpha, gamma;
  int defenders;
  int policy;  // 0..6 tailstorm_ssz policies, 7 = random actions, 8 = random release-heavy,
               // 9 = a random table (CPR_TS_POLICY_TABLE, loop tasks), 10 = the keyed random
               // attacker (CPR_TS_POLICY_RANDOM, loop tasks)
  int scheme;  // 0 Constant, 1 Discount, 3 Punish, 4 Hybrid
  int steps;
  int two_agents;  // 0 gym, 1 two-agents loop, 2 honest-clique loop (defenders = nodes),
                   // 3 exponential-delay clique loop (attacker + defenders, mean delay prop)
  int k;
  double ev = 1.0;
  double prop = 1.0;
  // engine.ml:209-214's other two done clauses (+inf = off; gym configurations only)
  double max_time = __builtin_inf();
  double max_progress = __builtin_inf();
};

struct Counters {
  long episodes = 0, mismatches = 0, capacity = 0, steps = 0, raises = 0, budget = 0;
};

static int g_sel = 1;

// one random table per k (dim 5): the oracle's TsTable and the lane read the same bytes
static const oracle::TsTable& g_table(int k) {
  static std::vector<oracle::TsTable> tabs(65);
  oracle::TsTable& t = tabs[k];
  if (t.dim == 0) {
    t.dim = 5;
    uint64_t x = 0x7AB1E000u + (uint64_t)k;
    t.actions.resize((size_t)t.dim * t.dim * (k + 1) * (k + 1) * 3);
    for (auto& a : t.actions) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      a = (uint8_t)((x >> 33) % 8);
    }
  }
  return t;
}

static ts::TsParams params_of(const Cfg& cf) {
  ts::TsParams P{};
  P.t_att = oracle::alpha_threshold(cf.alpha);
  P.d = cf.two_agents == 2 ? cf.defenders - 1
        : cf.two_agents == 3 ? cf.defenders
        : cf.two_agents    ? 1
                           : cf.defenders;
  P.n = P.d + 1;
  P.net = cf.two_agents;
  P.mode = cf.two_agents ? 1 : 0;
  if (cf.two_agents == 2) {  // models.ml:3-28 honest clique, as capi.hip validate_bk
    std::vector<double> w;
    for (int i = 0; i < P.n; ++i) w.push_back((double)(i + 1));
    const std::vector<uint32_t> thr = oracle::weight_thresholds(w);
    for (size_t i = 0; i < thr.size(); ++i) P.thr[i] = thr[i];
    P.lo = 0.5;
    P.hi = 1.5;
  }
  P.policy = cf.policy < 7 ? cf.policy
                          : (cf.policy == 9 ? ts::TS_POLICY_TABLE
                                            : (cf.policy == 10 ? ts::TS_POLICY_RANDOM : 0));
  if (cf.policy == 9) {
    P.table = g_table(cf.k).actions.data();
    P.table_dim = g_table(cf.k).dim;
  }
  P.scheme = cf.scheme;
  P.selection = g_sel;
  P.k = cf.k;
  // same sizing rules as capi.hip validate_ts (4096-vertex window)
  const int span = cf.two_agents ? 2 * cf.steps + 2 : cf.steps + 2;
  P.cap_v = 64;
  while (P.cap_v < span + 64 && P.cap_v < 4096) P.cap_v <<= 1;
  P.cap_q = P.cap_v / 2;
  P.cap_e = 256 + 512 * P.n + (cf.gamma == 0.0 && !cf.two_agents ? 2 * P.d * std::min(span, 8192) : 0);
  if (cf.two_agents == 3) P.cap_e = 256 + 512 * P.n;
  P.cap_d = 64;
  P.ev = cf.ev;
  P.delta = 1e-9;
  const double dd = cf.defenders;
  P.dmax = (dd - 1.) / dd * 1e-9 / cf.gamma;
  if (cf.two_agents == 3) {  // as capi.hip validate_bk for CPR_NET_EXP_CLIQUE
    P.delta = cf.prop;
    P.dmax = 0.0;
    P.t_att = oracle::alpha_threshold(1.0 / (double)(cf.defenders + 1));
  }
  P.max_steps = cf.steps;
  P.activations = cf.steps;
  P.max_progress = cf.max_progress;
  P.max_time = cf.max_time;
  P.opt_budget = oracle::g_ts_opt_budget;
  return P;
}

// SLABTEST=1: the lane's event-heap slab (nodes 0..5), visibility window and list-record
// window in host buffers, stride 1, so the host fuzz runs the device kernels' LDS paths too.
// The list-record window starts out filled with garbage (a slot is read only after its
// vertex's set_trec wrote it). TWIN=<rows> sets its size (default 8, 0 = none)
static ts::TsMem with_slab(ts::TsMem M, const ts::TsParams& P) {
  static std::vector<bk::HNode> slab(6);
  static std::vector<uint8_t> win;
  static std::vector<ts::TRec> twin;
  if (!getenv("SLABTEST")) return M;
  win.assign((size_t)8 * P.n, 0);
  ts::ts_heap_slab(M, slab.data(), 0, 1, 6);
  ts::ts_vis_window(M, win.data(), 0, 8);  // and the visibility rows of the newest 8 vertices
  const int tw = getenv("TWIN") ? atoi(getenv("TWIN")) : 8;
  if (tw > 0) {
    twin.assign((size_t)tw, ts::TRec{0x3c3c3c3c, 0x3c3c3c3c, 0x3c3c3c3c, 0x3c3c3c3c});
    ts::ts_trec_window(M, twin.data(), 0, tw);
  }
  return M;
}

static bool run_gym(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C, std::string& why) {
  oracle::GymParams gp;
  gp.alpha = cf.alpha;
  gp.gamma = cf.gamma;
  gp.defenders = cf.defenders;
  gp.max_steps = cf.steps;
  gp.max_progress = cf.max_progress;
  gp.max_time = cf.max_time;
  gp.unit_obs = false;
  oracle::GymTailstorm g(gp, cf.k, cf.scheme, g_sel, 1, nullptr, seed, ep);
  double obs[10];
  const ts::TsParams P = params_of(cf);
  std::vector<uint8_t> mem(ts::ts_lane_bytes(P));
  fill_garbage(mem);
  const ts::TsMem M = with_slab(ts::ts_mem_at(mem.data(), P), P);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  ts::TsLane L;
  bool oracle_raised = false;
  bool oracle_budget = false;
  try {
    g.reset(obs);
  } catch (oracle::BudgetExceeded&) {
    oracle_budget = true;
  } catch (std::exception&) {
    oracle_raised = true;
  }
  L.gym_reset(P, S, M);
  if (oracle_budget) {
    C.budget++;
    if (L.dead != 12) {
      why = "oracle hit the brute-force budget at reset, lane did not";
      C.mismatches++;
      return false;
    }
    return true;
  }
  if (oracle_raised) {
    C.raises++;
    if (!(L.status & ts::TST_REF_RAISES)) {
      why = "oracle raised at reset, lane did not";
      C.mismatches++;
      return false;
    }
    return true;
  }
  char buf[700];
  bool ok = true;
  for (int s = 0;; s++) {
    const oracle::TsObs o = g.observe_int();
    if (L.dead) {
      C.capacity++;
      if (getenv("CAPDBG"))
        fprintf(stderr, "capacity why %d a=%g g=%g pol=%d step %d newest %d hused %d\n", L.dead,
                cf.alpha, cf.gamma, cf.policy, s, L.newest, L.hused);
      return true;
    }
    const ts::TsObs e = L.observe(P, M);
    const int ov[10] = {o.public_blocks, o.private_blocks, o.diff_blocks, o.public_votes,
                        o.private_votes_inclusive, o.private_votes_exclusive, o.public_depth,
                        o.private_depth_inclusive, o.private_depth_exclusive, o.event};
    const int ev[10] = {e.public_blocks, e.private_blocks, e.diff_blocks, e.public_votes,
                        e.private_votes_inclusive, e.private_votes_exclusive, e.public_depth,
                        e.private_depth_inclusive, e.private_depth_exclusive, e.event};
    if (memcmp(ov, ev, sizeof ov) != 0) {
      snprintf(buf, sizeof buf,
               "step %d obs oracle (%d %d %d %d %d %d %d %d %d %d) lane (%d %d %d %d %d %d %d %d %d %d)",
               s, ov[0], ov[1], ov[2], ov[3], ov[4], ov[5], ov[6], ov[7], ov[8], ov[9], ev[0],
               ev[1], ev[2], ev[3], ev[4], ev[5], ev[6], ev[7], ev[8], ev[9]);
      why = buf;
      ok = false;
      break;
    }
    int act;
    if (cf.policy < 7) {
      act = oracle::ts_policy(cf.policy, o, cf.k);
      const int la = ts::ts_policy(P.policy, P.k, e);
      if (la != act) {
        snprintf(buf, sizeof buf, "step %d policy oracle %d lane %d", s, act, la);
        why = buf;
        ok = false;
        break;
      }
    } else {
      const uint32_t r = mix(ep, s);
      act = (int)(r % 8);
      if (cf.policy == 8 && (r >> 8) % 3 != 0) act = 4 + 1 + (int)((r >> 12) % 2);  // Override/Match
    }
    bool done = false;
    oracle::StepInfo info{};
    try {
      g.step(act, obs, &done, &info);
    } catch (oracle::BudgetExceeded&) {
      oracle_budget = true;
    } catch (std::exception&) {
      oracle_raised = true;
    }
    bool ldone = false;
    const int32_t hd = L.gym_step(P, S, M, act, &ldone);
    C.steps++;
    if (oracle_budget) {
      C.budget++;
      if (L.dead != 12) {
        snprintf(buf, sizeof buf, "step %d: oracle hit the budget, lane dead %d", s, L.dead);
        why = buf;
        ok = false;
        break;
      }
      return true;
    }
    if (oracle_raised) {
      C.raises++;
      if (!(L.status & ts::TST_REF_RAISES)) {
        snprintf(buf, sizeof buf, "step %d: oracle raised, lane status %u dead %d", s, L.status,
                 L.dead);
        why = buf;
        ok = false;
      }
      break;
    }
    if (L.status & ts::TST_REF_RAISES) {
      snprintf(buf, sizeof buf, "step %d: lane flags a reference exception, oracle did not", s);
      why = buf;
      ok = false;
      break;
    }
    if (L.dead) {
      C.capacity++;
      if (getenv("CAPDBG"))
        fprintf(stderr, "capacity why %d a=%g g=%g pol=%d step %d newest %d hused %d\n", L.dead,
                cf.alpha, cf.gamma, cf.policy, s, L.newest, L.hused);
      return true;
    }
    const ts::TVtx& hb = L.X(P, M, hd);
    double ra = 0.0, rd = 0.0;
    if (hb.qslot >= 0) {
      const double* rw = L.R(P, M, hb.qslot);
      ra = rw[0];
      for (int j = 1; j < P.n; ++j) rd += rw[j];
    }
    const double prog = (double)(hb.height * cf.k);
    if (ra != info.episode_reward_attacker || rd != info.episode_reward_defender ||
        hb.height != info.head_height || prog != info.episode_progress ||
        hb.time != info.episode_chain_time || L.now != info.episode_sim_time ||
        L.c_act != info.episode_n_activations || ldone != done ||
        L.newest + 1 != (int)g.sim->dag.size()) {
      snprintf(buf, sizeof buf,
               "step %d head lane (ra %.4f rd %.4f h %d tm %.17g t %.17g k %d m %d done %d v %d) "
               "oracle (ra %.4f rd %.4f h %d tm %.17g t %.17g k %ld m %d done %d v %d)",
               s, ra, rd, hb.height, hb.time, L.now, L.c_act, hb.who, (int)ldone, L.newest + 1,
               info.episode_reward_attacker, info.episode_reward_defender, info.head_height,
               info.episode_chain_time, info.episode_sim_time, info.episode_n_activations,
               info.head_miner, (int)done, (int)g.sim->dag.size());
      why = buf;
      ok = false;
      break;
    }
    if (done) break;
  }
  C.episodes++;
  if (!ok) C.mismatches++;
  return ok;
}

static bool run_loop(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C, std::string& why) {
  oracle::TsLoopResult r;
  bool raised = false;
  bool budget = false;
  try {
    oracle::Network net = oracle::Network::two_agents(1.0, cf.alpha);
    if (cf.two_agents == 2) {
      net = oracle::Network{};
      net.flooding = false;
      net.activation_delay = cf.ev;
      net.nodes.resize(cf.defenders);
      for (int i = 0; i < cf.defenders; ++i) {
        net.nodes[i].compute = (double)(i + 1);
        for (int j = 0; j < cf.defenders - 1; ++j)
          net.nodes[i].links.push_back(
              oracle::Link{j >= i ? j + 1 : j, oracle::D_UNIFORM, 0.5, 1.5});
      }
    } else if (cf.two_agents == 3) {  // cpr_protocols.ml:478-485, as oracle_api.cpp loop_net
      const int n = cf.defenders + 1;
      net = oracle::Network{};
      net.flooding = false;
      net.activation_delay = cf.ev;
      net.nodes.resize(n);
      for (int i = 0; i < n; ++i) {
        net.nodes[i].compute = 1. / (double)n;
        for (int j = 0; j < n - 1; ++j)
          net.nodes[i].links.push_back(oracle::Link{j >= i ? j + 1 : j, oracle::D_EXP, cf.prop, 0.0});
      }
    }
    oracle::ts_loop_task(net, 1, nullptr, seed, ep, cf.k, cf.scheme, g_sel,
                         cf.two_agents == 2 ? -1 : (cf.policy == 9 ? oracle::TS_POL_TABLE
                                                           : (cf.policy == 10 ? oracle::TS_POL_RANDOM : cf.policy)),
                         cf.steps, &r, &g_table(cf.k));
  } catch (oracle::BudgetExceeded&) {
    budget = true;
  } catch (std::exception&) {
    raised = true;
  }
  const ts::TsParams P = params_of(cf);
  std::vector<uint8_t> mem(ts::ts_lane_bytes(P));
  fill_garbage(mem);
  const ts::TsMem M = with_slab(ts::ts_mem_at(mem.data(), P), P);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  ts::TsLane L;
  const int32_t hd = L.loop(P, S, M);
  if (budget) {
    C.budget++;
    if (L.dead != 12) {
      why = "loop: oracle hit the budget, lane did not";
      C.mismatches++;
      return false;
    }
    return true;
  }
  if (raised) {
    C.raises++;
    if (!(L.status & ts::TST_REF_RAISES)) {
      why = "loop: oracle raised, lane did not";
      C.mismatches++;
      return false;
    }
    return true;
  }
  if (L.dead) {
    C.capacity++;
    if (getenv("CAPDBG"))
      fprintf(stderr, "loop capacity why %d a=%g pol=%d newest %d hused %d\n", L.dead, cf.alpha,
              cf.policy, L.newest, L.hused);
    return true;
  }
  const ts::TVtx& hb = L.X(P, M, hd);
  const double* rw = L.R(P, M, hb.qslot);
  C.episodes++;
  C.steps += cf.steps;
  bool rw_ok = true;
  int64_t acts = 0;
  for (size_t j = 0; j < r.rewards.size(); ++j) rw_ok = rw_ok && rw[j] == r.rewards[j];
  for (int64_t a : r.activations) acts += a;
  if (!rw_ok || hb.height != r.head_height || hb.time != r.head_time ||
      (cf.two_agents != 2 && L.act0 != r.activations[0]) || L.c_act != acts ||
      L.newest + 1 != r.n_vertices) {
    char buf[400];
    snprintf(buf, sizeof buf,
             "loop lane (ra %.3f rd %.3f h %d tm %.17g a0 %d v %d) oracle (%.3f %.3f %d %.17g %ld %ld)",
             rw[0], rw[1], hb.height, hb.time, L.act0, L.newest + 1, r.rewards[0],
             r.rewards[1], r.head_height, r.head_time, (long)r.activations[0],
             (long)r.n_vertices);
    why = buf;
    C.mismatches++;
    return false;
  }
  return true;
}

int main(int argc, char** argv) {
  const int eps = argc > 1 ? atoi(argv[1]) : 10;
  const int steps = argc > 2 ? atoi(argv[2]) : 300;
  const int k = argc > 3 ? atoi(argv[3]) : 8;
  g_sel = argc > 4 ? atoi(argv[4]) : 1;
  const uint64_t seed = 0x7A110000ull + (uint64_t)k * 16 + (uint64_t)g_sel;
  std::vector<Cfg> cfgs;
  // OPTCHECK=<budget>: every optimal quorum of the oracle is also computed by the
  // reference's literal enumeration (up to <budget> choices) and compared with the pruned
  // search both engines run (oracle/src/tailstorm.cpp TsView::optimal)
  if (const char* oc = getenv("OPTCHECK")) {
    oracle::g_ts_optimal_check.on = true;
    oracle::g_ts_brute_budget = atoll(oc);
  }
  // OPTBUDGET=<visits>: both engines' pruned-search budget lowered to <visits>, so that
  // many searches run out of it: the episodes each engine flags must be the same
  if (const char* ob = getenv("OPTBUDGET")) oracle::g_ts_opt_budget = atoll(ob);
  if (const char* prof = getenv("TSPROF")) {
    // lane only (host profiling, tools: gprof): "policy,episodes" of bench.py configs[3]
    // (two agents, alpha .33, 10^4 activations, discount rewards, selection argv[4])
    int pol = 5, neps = 20;
    if (sscanf(prof, "%d,%d", &pol, &neps) != 2) return 2;
    Cfg cf{0.33, 0.0, 1, pol, 1, 10000, 1, k};
    const ts::TsParams P = params_of(cf);
    std::vector<uint8_t> mem(ts::ts_lane_bytes(P));
    fill_garbage(mem);
    const ts::TsMem M = with_slab(ts::ts_mem_at(mem.data(), P), P);
    long acts = 0;
    for (int e = 0; e < neps; e++) {
      const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)e, 0u};
      ts::TsLane L;
      L.loop(P, S, M);
      acts += L.c_act;
    }
    printf("{\"episodes\": %d, \"activations\": %ld}\n", neps, acts);
    return 0;
  }
  if (const char* one = getenv("TSCASE")) {
    // one exponential-clique case: "defenders,policy,scheme,ev,prop,activations,seed,first,n"
    int d, pol, sch, acts, first, n;
    double ev, prop;
    unsigned long long sd;
    if (sscanf(one, "%d,%d,%d,%lf,%lf,%d,%llu,%d,%d", &d, &pol, &sch, &ev, &prop, &acts, &sd, &first,
               &n) != 9)
      return 2;
    Cfg cf{0, 0, d, pol, sch, acts, 3, k, ev, prop};
    Counters C;
    for (int e = first; e < first + n; e++) {
      std::string why;
      if (!run_loop(cf, sd, e, C, why)) fprintf(stderr, "MISMATCH ep=%d: %s\n", e, why.c_str());
    }
    const auto& oc = oracle::g_ts_optimal_check;
    printf("{\"episodes\": %ld, \"mismatches\": %ld, \"capacity\": %ld, \"raises\": %ld, \"budget\": %ld, \"opt_compared\": %ld, \"opt_large\": %ld, \"opt_mismatches\": %ld, \"opt_unverified\": %ld}\n",
           C.episodes, C.mismatches, C.capacity, C.raises, C.budget, (long)oc.compared, (long)oc.large,
           (long)oc.mismatches, (long)oc.unverified);
    return (C.mismatches || oc.mismatches) ? 1 : 0;
  }
  const double alphas[] = {0.1, 0.25, 0.33, 0.45};
  const double gammas[] = {0.0, 0.5, 0.9};
  for (double a : alphas)
    for (double g : gammas) {
      const int d = std::max(2, (int)std::ceil(1.0 / (1.0 - g)));
      for (int pol : {0, 1, 2, 3, 4, 5, 6, 7, 8})
        cfgs.push_back(Cfg{a, g, d, pol, (pol % 4 == 0) ? 0 : (pol % 4 == 1 ? 1 : (pol % 4 == 2 ? 3 : 4)), steps, 0, k});
    }
  cfgs.push_back(Cfg{0.4, 0.75, 7, 8, 1, steps, 0, k});
  cfgs.push_back(Cfg{0.33, 0.3, 4, 7, 1, steps, 0, k});
  for (double a : alphas)
    for (int pol : {0, 1, 2, 3, 4, 5, 6, 9}) cfgs.push_back(Cfg{a, 0, 1, pol, 1, steps * 2, 1, k});
  // honest cliques: n nodes, compute 1..n, U(0.5, 1.5) links, all four reward schemes
  for (int n : {2, 3, 10})
    for (double ev : {0.5, 2.0, 30.0, 600.0})
      for (int sch : {0, 1, 3, 4}) cfgs.push_back(Cfg{0, 0, n, 0, sch, steps * 2, 2, k, ev});
  // exponential-delay cliques with the attacker as node 0 (configs[3] and its 3-node form)
  for (int d : {1, 2})
    for (double ev : {1.0, 10.0})
      for (int pol : {0, 1, 2, 3, 9}) cfgs.push_back(Cfg{0, 0, d, pol, 1, steps * 2, 3, k, ev, 1.0});
  // gym episodes ended by max_time / max_progress before max_steps (engine.ml:209-214)
  for (int pol : {1, 3, 7})
    for (double g : {0.0, 0.5}) {
      Cfg c{0.33, g, 2, pol, 1, steps, 0, k};
      c.max_time = 0.3 * steps;
      cfgs.push_back(c);
      c.max_time = __builtin_inf();
      c.max_progress = steps / 6;
      cfgs.push_back(c);
    }
  Counters C;
  int shown = 0;
  for (auto& cf : cfgs)
    for (int e = 0; e < eps; e++) {
      std::string why;
      if (getenv("TSDBG"))
        fprintf(stderr, "cfg a=%g g=%g d=%d pol=%d sch=%d two=%d ep=%d\n", cf.alpha, cf.gamma,
                cf.defenders, cf.policy, cf.scheme, cf.two_agents, e);
      const bool ok = cf.two_agents ? run_loop(cf, seed, e, C, why) : run_gym(cf, seed, e, C, why);
      if (!ok && shown < 10) {
        shown++;
        fprintf(stderr, "MISMATCH alpha=%g gamma=%g d=%d pol=%d scheme=%d two=%d ep=%d: %s\n",
                cf.alpha, cf.gamma, cf.defenders, cf.policy, cf.scheme, cf.two_agents, e,
                why.c_str());
      }
    }
  const auto& oc = oracle::g_ts_optimal_check;
  printf("{\"episodes\": %ld, \"steps\": %ld, \"mismatches\": %ld, \"capacity\": %ld, \"raises\": %ld, \"budget\": %ld, \"opt_compared\": %ld, \"opt_large\": %ld, \"opt_mismatches\": %ld, \"opt_unverified\": %ld}\n",
         C.episodes, C.steps, C.mismatches, C.capacity, C.raises, C.budget, (long)oc.compared,
         (long)oc.large, (long)oc.mismatches, (long)oc.unverified);
  return (C.mismatches || oc.mismatches) ? 1 : 0;
}
