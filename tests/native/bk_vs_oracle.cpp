// TEST INFRASTRUCTURE ONLY. Differential fuzzer for the B_k lane
// (cpr_amd/csrc/bk_lane.h, compiled here for the host) against the CPU oracle's
// restatement (oracle/src/bk.cpp), step by step on the same keyed stream: all eight
// observation fields and the step info after every step; loop-mode tasks on the
// two-agents network compared at the end. Prints one JSON summary line; exit code 1 on
// any mismatch. Usage: bk_vs_oracle [episodes per config] [steps] [k]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "garbage.h"
#include "../../cpr_amd/csrc/bk_lane.h"
#include "../../oracle/src/bk.h"

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
  int policy;  // 0..3 bk_ssz policies, 4 = table, 5 = random actions, 6 = random release-heavy
  int scheme;  // 0 Constant, 2 Block
  int steps;
  int two_agents;  // 0 gym, 1 two-agents loop, 2 honest-clique loop (defenders = nodes)
  int k;
  double ev = 1.0;
  // engine.ml:209-214's other two done clauses (+inf = off; gym configurations only)
  double max_time = __builtin_inf();
  double max_progress = __builtin_inf();
};

struct Counters {
  long episodes = 0, mismatches = 0, capacity = 0, steps = 0;
};

static std::vector<uint8_t> g_table;
static int g_dim = 4;

static bk::BkParams params_of(const Cfg& cf) {
  bk::BkParams P{};
  P.t_att = oracle::alpha_threshold(cf.alpha);
  P.d = cf.two_agents == 2 ? cf.defenders - 1 : cf.two_agents ? 1 : cf.defenders;
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
  P.policy = cf.policy < 5 ? cf.policy : 0;
  P.scheme = cf.scheme;
  P.k = cf.k;
  // same sizing rules as capi.hip validate_bk (4096-vertex window)
  const int span = cf.two_agents ? 2 * cf.steps + 2 : cf.steps + 2;
  P.cap_v = 64;
  while (P.cap_v < span + 64 && P.cap_v < 4096) P.cap_v <<= 1;
  P.cap_q = P.cap_v / 2;
  P.cap_e = 256 + 512 * P.n + (cf.gamma == 0.0 && !cf.two_agents ? 2 * P.d * std::min(span, 8192) : 0);
  P.cap_d = 64;
  P.table_dim = g_dim;
  P.table = g_table.data();
  P.ev = cf.ev;
  P.delta = 1e-9;
  const double dd = cf.defenders;
  P.dmax = (dd - 1.) / dd * 1e-9 / cf.gamma;
  P.max_steps = cf.steps;
  P.activations = cf.steps;
  P.max_progress = cf.max_progress;
  P.max_time = cf.max_time;
  return P;
}

// SLABTEST=1: the lane's event-heap slab (nodes 0..5) and visibility window (8 vertices)
// in host buffers, stride 1, so the host fuzz runs the device kernels' LDS paths too
static bk::BkMem with_slab(bk::BkMem M, const bk::BkParams& P) {
  static std::vector<bk::HNode> slab(6);
  static std::vector<uint8_t> win;
  if (!getenv("SLABTEST")) return M;
  win.assign((size_t)8 * P.n, 0);
  bk::bk_heap_slab(M, slab.data(), 0, 1, 6);
  bk::bk_vis_window(M, win.data(), 0, 8);
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
  oracle::GymBk g(gp, cf.k, cf.scheme, 1, nullptr, seed, ep);
  double obs[8];
  g.reset(obs);
  oracle::BkTable tab;
  tab.dim = g_dim;
  tab.k = cf.k;
  tab.actions = g_table;

  const bk::BkParams P = params_of(cf);
  std::vector<uint8_t> mem(bk::bk_lane_bytes(P));
  fill_garbage(mem);
  const bk::BkMem M = with_slab(bk::bk_mem_at(mem.data(), P), P);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  bk::BkLane L;
  L.gym_reset(P, S, M);
  char buf[700];
  bool ok = true;
  for (int s = 0;; s++) {
    const oracle::BkObs o = g.observe_int();
    if (L.dead) {
      C.capacity++;
      if (getenv("CAPDBG"))
        fprintf(stderr, "capacity why %d a=%g g=%g pol=%d step %d newest %d hused %d\n", L.dead,
                cf.alpha, cf.gamma, cf.policy, s, L.newest, L.hused);
      return true;
    }
    const bk::BkObs e = L.observe(P, M);
    const int ov[8] = {o.public_blocks, o.private_blocks, o.diff_blocks, o.public_votes,
                       o.private_votes_inclusive, o.private_votes_exclusive, o.lead, o.event};
    const int ev[8] = {e.public_blocks, e.private_blocks, e.diff_blocks, e.public_votes,
                       e.private_votes_inclusive, e.private_votes_exclusive, e.lead, e.event};
    if (memcmp(ov, ev, sizeof ov) != 0) {
      snprintf(buf, sizeof buf,
               "step %d obs oracle (%d %d %d %d %d %d %d %d) lane (%d %d %d %d %d %d %d %d)", s,
               ov[0], ov[1], ov[2], ov[3], ov[4], ov[5], ov[6], ov[7], ev[0], ev[1], ev[2], ev[3],
               ev[4], ev[5], ev[6], ev[7]);
      why = buf;
      ok = false;
      break;
    }
    int act;
    if (cf.policy < 5) {
      act = oracle::bk_policy(cf.policy, o, cf.k, &tab);
      const int la = bk::bk_policy(P, e);
      if (la != act) {
        snprintf(buf, sizeof buf, "step %d policy oracle %d lane %d", s, act, la);
        why = buf;
        ok = false;
        break;
      }
    } else {
      const uint32_t r = mix(ep, s);
      act = (int)(r % 8);
      if (cf.policy == 6 && (r >> 8) % 3 != 0) act = 4 + 1 + (int)((r >> 12) % 2);  // Override/Match
    }
    bool done = false;
    oracle::StepInfo info{};

    g.step(act, obs, &done, &info);

    bool ldone = false;
    const int32_t hd = L.gym_step(P, S, M, act, &ldone);
    C.steps++;
    if (L.dead) {
      C.capacity++;
      if (getenv("CAPDBG"))
        fprintf(stderr, "capacity why %d a=%g g=%g pol=%d step %d newest %d hused %d\n", L.dead,
                cf.alpha, cf.gamma, cf.policy, s, L.newest, L.hused);
      return true;
    }
    const bk::BVtx& hb = L.X(P, M, hd);
    const double ra = hb.rew_att, rd = hb.rew_def;
    const double prog = (double)(hb.height * cf.k);
    if (ra != info.episode_reward_attacker || rd != info.episode_reward_defender ||
        hb.height != info.head_height || prog != info.episode_progress ||
        hb.time != info.episode_chain_time || L.now != info.episode_sim_time ||
        L.c_act != info.episode_n_activations || hb.who != info.head_miner || ldone != done ||
        L.newest + 1 != (int)g.sim->dag.size()) {
      snprintf(buf, sizeof buf,
               "step %d head lane (ra %.1f rd %.1f h %d tm %.17g t %.17g k %d m %d done %d v %d) "
               "oracle (ra %.1f rd %.1f h %d tm %.17g t %.17g k %ld m %d done %d v %d)",
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

static constexpr int64_t L0_ANY = -1;

static bool run_loop(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C, std::string& why) {
  oracle::BkTable tab;
  tab.dim = g_dim;
  tab.k = cf.k;
  tab.actions = g_table;
  oracle::BkLoopResult r;
  oracle::Network net = oracle::Network::two_agents(1.0, cf.alpha);
  if (cf.two_agents == 2) {
    net = oracle::Network{};
    net.flooding = false;
    net.activation_delay = cf.ev;
    net.nodes.resize(cf.defenders);
    for (int i = 0; i < cf.defenders; ++i) {
      net.nodes[i].compute = (double)(i + 1);
      for (int j = 0; j < cf.defenders - 1; ++j)
        net.nodes[i].links.push_back(oracle::Link{j >= i ? j + 1 : j, oracle::D_UNIFORM, 0.5, 1.5});
    }
  }
  oracle::bk_loop_task(net, 1, nullptr, seed, ep, cf.k, cf.scheme,
                       cf.two_agents == 2 ? -1 : cf.policy, &tab, cf.steps, &r);
  double rd = 0.0;
  int64_t acts = 0;
  for (size_t i = 1; i < r.rewards.size(); ++i) rd += r.rewards[i];
  for (int64_t a : r.activations) acts += a;
  const int64_t a0 = cf.two_agents == 2 ? L0_ANY : r.activations[0];
  const bk::BkParams P = params_of(cf);
  std::vector<uint8_t> mem(bk::bk_lane_bytes(P));
  fill_garbage(mem);
  const bk::BkMem M = with_slab(bk::bk_mem_at(mem.data(), P), P);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  bk::BkLane L;
  const int32_t hd = L.loop(P, S, M);
  if (L.dead) {
    C.capacity++;
    return true;
  }
  const bk::BVtx& hb = L.X(P, M, hd);
  C.episodes++;
  C.steps += cf.steps;
  if (hb.rew_att != r.rewards[0] || hb.rew_def != rd || hb.height != r.head_height ||
      hb.time != r.head_time || (a0 != L0_ANY && L.act0 != a0) ||
      L.c_act != acts || hb.who != r.head_signer ||
      L.newest + 1 != r.n_vertices) {
    char buf[400];
    snprintf(buf, sizeof buf,
             "loop lane (ra %d rd %d h %d tm %.17g a0 %d v %d) oracle (%.1f %.1f %d %.17g %ld %ld)",
             hb.rew_att, hb.rew_def, hb.height, hb.time, L.act0, L.newest + 1, r.rewards[0],
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
  const uint64_t seed = 0xB0B00000ull + (uint64_t)k;
  // a random table policy over (pub, priv, public votes, private votes, event)
  g_table.resize((size_t)g_dim * g_dim * (k + 1) * (k + 1) * 3);
  for (size_t i = 0; i < g_table.size(); ++i) g_table[i] = (uint8_t)(mix(7, i) % 8);
  std::vector<Cfg> cfgs;
  const double alphas[] = {0.1, 0.25, 0.33, 0.45};
  const double gammas[] = {0.0, 0.5, 0.9};
  for (double a : alphas)
    for (double g : gammas) {
      const int d = std::max(2, (int)std::ceil(1.0 / (1.0 - g)));
      for (int pol : {0, 1, 2, 3, 4, 5, 6})
        for (int sch : {0, 2}) cfgs.push_back(Cfg{a, g, d, pol, sch, steps, 0, k});
    }
  cfgs.push_back(Cfg{0.4, 0.75, 7, 6, 0, steps, 0, k});
  cfgs.push_back(Cfg{0.33, 0.3, 4, 5, 0, steps, 0, k});
  for (double a : alphas)
    for (int pol : {0, 1, 2, 3}) cfgs.push_back(Cfg{a, 0, 1, pol, 0, steps * 2, 1, k});
  // honest cliques: n nodes, compute 1..n, U(0.5, 1.5) links, both reward schemes
  for (int n : {2, 3, 10})
    for (double ev : {0.5, 2.0, 30.0, 600.0})
      for (int sch : {0, 2}) cfgs.push_back(Cfg{0, 0, n, 0, sch, steps * 2, 2, k, ev});
  // episodes longer than the 4096-vertex window: the vertex ring, the vote-list links
  // (vh / vn, indexed serial & (cap_v - 1)) and the visibility rows wrap around (the
  // path of round 4's r04o fault investigation)
  cfgs.push_back(Cfg{0.33, 0.5, 2, 1, 0, 6000, 0, k});
  cfgs.push_back(Cfg{0.45, 0.0, 2, 5, 2, 6000, 0, k});
  cfgs.push_back(Cfg{0.40, 0.9, 10, 6, 0, 6000, 0, k});
  // gym episodes ended by max_time / max_progress before max_steps (engine.ml:209-214)
  for (int pol : {1, 3, 5})
    for (double g : {0.0, 0.5}) {
      Cfg c{0.33, g, 2, pol, pol == 3 ? 2 : 0, steps, 0, k};
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
      const bool ok = cf.two_agents ? run_loop(cf, seed, e, C, why) : run_gym(cf, seed, e, C, why);
      if (!ok && shown < 10) {
        shown++;
        fprintf(stderr, "MISMATCH alpha=%g gamma=%g d=%d pol=%d scheme=%d two=%d ep=%d: %s\n",
                cf.alpha, cf.gamma, cf.defenders, cf.policy, cf.scheme, cf.two_agents, e,
                why.c_str());
      }
    }
  printf("{\"episodes\": %ld, \"steps\": %ld, \"mismatches\": %ld, \"capacity\": %ld}\n",
         C.episodes, C.steps, C.mismatches, C.capacity);
  return C.mismatches ? 1 : 0;
}
