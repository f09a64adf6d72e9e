// TEST INFRASTRUCTURE ONLY. Differential fuzzer for the Ethereum lane
// (cpr_amd/csrc/ethereum_lane.h, compiled here for the host) against the CPU oracle's
// restatement (oracle/src/ethereum.cpp), step by step on the same keyed stream: all ten
// observation fields (including the three dry-run uncle selections) and the step info
// after every step; loop-mode tasks on the two-agents network compared at the end; and the
// lane in Nakamoto mode (P.nak) running Simulator.loop tasks on the selfish-mining network
// with a nakamoto_ssz attacker (the withholding sweep's gamma-* tasks, incl. gamma = 0)
// against the oracle's oracle_sm_task; and loop tasks on the exponential-delay clique
// (Ethereum and Nakamoto mode) against the oracle's public entry.
// Prints one JSON summary line; exit code 1 on any mismatch.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "garbage.h"
#include "../../cpr_amd/csrc/ethereum_lane.h"
#include "../../include/cpr_hip.h"
#include "../../oracle/src/ethereum.h"

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
  int policy;  // 0..4 ethereum_ssz policies, 5 = random actions, 6 = random biased to release,
               // 9 = a random table (CPR_ETH_POLICY_TABLE, loop tasks)
  int scheme;
  int steps;
  int two_agents;  // 2: Nakamoto-mode loop task on the selfish-mining network; 3 / 4: loop
                   // task on the exponential-delay clique, Ethereum / Nakamoto mode
  double prop = 1e-9;
};

extern "C" int oracle_sm_task(int rng_mode, void* rng, uint64_t seed, uint64_t episode,
                              double alpha, double gamma, int defenders, double msg_delay,
                              int policy, int activations, int64_t* acts_out,
                              double* rewards_out, double* head_time, double* head_progress,
                              int32_t* head_height, int32_t* head_miner, uint32_t* diag);
extern "C" int oracle_run_episodes(const cpr_config* c, uint64_t first, int64_t n,
                                   cpr_episode_record* out, int threads);

struct Counters {
  long episodes = 0, mismatches = 0, capacity = 0, steps = 0;
};

// a random ethereum_ssz table (dim 6): the oracle's EthTable and the lane read the same bytes
static const oracle::EthTable& g_table() {
  static oracle::EthTable t;
  if (t.dim == 0) {
    t.dim = 6;
    uint64_t x = 0xE7AB1E00u;
    t.actions.resize((size_t)t.dim * t.dim * 2);
    for (auto& a : t.actions) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      a = (uint8_t)((x >> 33) % 24);
    }
  }
  return t;
}

static eth::EthParams params_of(const Cfg& cf) {
  eth::EthParams P{};
  P.t_att = oracle::alpha_threshold(cf.alpha);
  P.d = cf.two_agents == 1 ? 1 : cf.defenders;
  P.n = P.d + 1;
  P.net = cf.two_agents == 1 ? 1 : 0;
  P.mode = cf.two_agents ? 1 : 0;
  P.nak = cf.two_agents == 2 ? 1 : 0;
  P.policy = cf.policy < 5 ? cf.policy : (cf.policy == 9 ? eth::ETH_POLICY_TABLE : 0);
  if (cf.policy == 9) {
    P.table = g_table().actions.data();
    P.table_dim = g_table().dim;
  }
  P.scheme = cf.scheme;
  P.cap_b = 1;
  while (P.cap_b < cf.steps + 2) P.cap_b <<= 1;
  P.cap_e = 64 + 512 * P.n + (cf.gamma == 0.0 ? 2 * P.d * cf.steps : P.d * (cf.steps + 2));
  P.ev = 1.0;
  P.delta = cf.prop;
  const double dd = cf.defenders;
  P.dmax = (dd - 1.) / dd * cf.prop / cf.gamma;
  P.max_steps = cf.steps;
  P.activations = cf.steps;
  P.max_progress = __builtin_inf();
  P.max_time = __builtin_inf();
  if (cf.two_agents >= 3) {
    // capi.hip validate_eth, CPR_NET_EXP_CLIQUE: equal compute, exponential links
    P.d = cf.defenders;
    P.n = P.d + 1;
    P.net = 3;
    P.nak = cf.two_agents == 4 ? 1 : 0;
    P.policy = cf.policy;
    P.t_att = oracle::alpha_threshold(1.0 / (double)P.n);
    P.cap_e = 64 + 512 * P.n + P.d * (cf.steps + 2);  // capi.hip validate_eth
    P.dmax = 0.0;
  }
  return P;
}

static bool run_gym(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C, std::string& why) {
  oracle::GymParams gp;
  gp.alpha = cf.alpha;
  gp.gamma = cf.gamma;
  gp.defenders = cf.defenders;
  gp.max_steps = cf.steps;
  gp.unit_obs = false;
  oracle::GymEthereum g(gp, cf.scheme, 1, nullptr, seed, ep);
  double obs[10];
  g.reset(obs);

  const eth::EthParams P = params_of(cf);
  std::vector<uint8_t> mem(eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  fill_garbage(mem);
  const eth::EthMem M = eth::eth_mem_at(mem.data(), P.cap_b, P.cap_e, P.n);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  eth::EthLane L;
  L.gym_reset(P, S, M);
  char buf[600];
  bool ok = true;
  for (int s = 0;; s++) {
    const oracle::EthObs o = g.observe_int();
    const eth::EthObs e = L.observe(P, M, true);
    const int ov[10] = {o.public_height, o.public_work, o.private_height, o.private_work,
                        o.diff_height, o.diff_work, o.public_orphans,
                        o.private_orphans_inclusive, o.private_orphans_exclusive, o.event};
    const int ev[10] = {e.public_height, e.public_work, e.private_height, e.private_work,
                        e.diff_height, e.diff_work, e.public_orphans,
                        e.private_orphans_inclusive, e.private_orphans_exclusive, e.event};
    if (L.dead) {
      C.capacity++;
      if (getenv("CAPDBG"))
        fprintf(stderr, "capacity why %d a=%g g=%g pol=%d step %d newest %d hused %d\n", L.dead, cf.alpha,
                cf.gamma, cf.policy, s, L.newest, L.hused);
      return true;
    }
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
    if (cf.policy < 5)
      act = oracle::eth_policy(cf.policy, o);
    else {
      const uint32_t r = mix(ep, s);
      act = (int)(r % 24);
      if (cf.policy == 6 && (r >> 8) % 2 == 0) act = (int)(((r >> 12) % 4 == 0 ? 1 : 2 + (r >> 14) % 3) * 4 + (r >> 20) % 4);
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
        fprintf(stderr, "capacity why %d a=%g g=%g pol=%d step %d newest %d hused %d fork %d\n",
                L.dead, cf.alpha, cf.gamma, cf.policy, s, L.newest, L.hused, o.private_height * 1000 + o.public_height);
      return true;
    }
    const eth::EBlock& hb = L.B(P, M, hd);
    const double ra = hb.rew_att / 32.0, rd = hb.rew_def / 32.0;
    if (ra != info.episode_reward_attacker || rd != info.episode_reward_defender ||
        hb.height != info.head_height || hb.work != info.head_work ||
        (double)hb.work != info.episode_progress || hb.time != info.episode_chain_time ||
        L.now != info.episode_sim_time || L.c_act != info.episode_n_activations ||
        hb.miner != info.head_miner || ldone != done) {
      snprintf(buf, sizeof buf,
               "step %d head lane (ra %.5f rd %.5f h %d w %d tm %.17g t %.17g k %d m %d done %d) "
               "oracle (ra %.5f rd %.5f h %d w %d tm %.17g t %.17g k %ld m %d done %d)",
               s, ra, rd, hb.height, hb.work, hb.time, L.now, L.c_act, hb.miner, (int)ldone,
               info.episode_reward_attacker, info.episode_reward_defender, info.head_height,
               info.head_work, info.episode_chain_time, info.episode_sim_time,
               info.episode_n_activations, info.head_miner, (int)done);
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
  oracle::EthLoopResult r;
  oracle::eth_two_agents_task(1, nullptr, seed, ep, cf.alpha, cf.scheme,
                              cf.policy == 9 ? oracle::ETH_POL_TABLE : cf.policy, cf.steps, &r,
                              &g_table());
  const eth::EthParams P = params_of(cf);
  std::vector<uint8_t> mem(eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  fill_garbage(mem);
  const eth::EthMem M = eth::eth_mem_at(mem.data(), P.cap_b, P.cap_e, P.n);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  eth::EthLane L;
  const int32_t hd = L.loop(P, S, M);
  if (L.dead) {
    C.capacity++;
    return true;
  }
  const eth::EBlock& hb = L.B(P, M, hd);
  C.episodes++;
  C.steps += cf.steps;
  if (hb.rew_att / 32.0 != r.rewards[0] || hb.rew_def / 32.0 != r.rewards[1] ||
      hb.height != r.head_height || hb.work != r.head_work || hb.time != r.head_time ||
      L.act0 != r.activations[0] || L.c_act != r.activations[0] + r.activations[1]) {
    char buf[400];
    snprintf(buf, sizeof buf,
             "loop lane (ra %.5f rd %.5f h %d w %d tm %.17g a0 %d) oracle (%.5f %.5f %d %d %.17g %ld)",
             hb.rew_att / 32.0, hb.rew_def / 32.0, hb.height, hb.work, hb.time, L.act0,
             r.rewards[0], r.rewards[1], r.head_height, r.head_work, r.head_time,
             (long)r.activations[0]);
    why = buf;
    C.mismatches++;
    return false;
  }
  return true;
}

static bool run_sm_loop(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C,
                        std::string& why) {
  const int n = cf.defenders + 1;
  std::vector<int64_t> acts(n);
  std::vector<double> rew(n);
  double ht, hp;
  int32_t hh, hm;
  uint32_t diag = 0;
  if (oracle_sm_task(1, nullptr, seed, ep, cf.alpha, cf.gamma, cf.defenders, cf.prop, cf.policy,
                     cf.steps, acts.data(), rew.data(), &ht, &hp, &hh, &hm, &diag) != 0) {
    why = "oracle_sm_task failed";
    C.mismatches++;
    return false;
  }
  double rd = 0.0;
  for (int i = 1; i < n; ++i) rd += rew[i];
  const eth::EthParams P = params_of(cf);
  std::vector<uint8_t> mem(eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  fill_garbage(mem);
  const eth::EthMem M = eth::eth_mem_at(mem.data(), P.cap_b, P.cap_e, P.n);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  eth::EthLane L;
  const int32_t hd = L.loop(P, S, M);
  if (L.dead) {
    C.capacity++;
    return true;
  }
  const eth::EBlock& hb = L.B(P, M, hd);
  C.episodes++;
  C.steps += cf.steps;
  if (hb.rew_att / 32.0 != rew[0] || hb.rew_def / 32.0 != rd || hb.height != hh ||
      hb.time != ht || L.act0 != acts[0]) {
    char buf[400];
    snprintf(buf, sizeof buf,
             "sm loop lane (ra %.5f rd %.5f h %d tm %.17g a0 %d) oracle (%.5f %.5f %d %.17g %ld)",
             hb.rew_att / 32.0, hb.rew_def / 32.0, hb.height, hb.time, L.act0, rew[0], rd, hh,
             ht, (long)acts[0]);
    why = buf;
    C.mismatches++;
    return false;
  }
  return true;
}

// a loop task on the exponential-delay clique (cpr_protocols.ml:478-485) through the oracle's
// public entry (oracle_api.cpp attack_clique_task), compared on the final record
static bool run_exp(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C, std::string& why) {
  cpr_config c{};
  c.protocol = cf.two_agents == 3 ? CPR_PROTO_ETHEREUM : CPR_PROTO_NAKAMOTO;
  c.network = CPR_NET_EXP_CLIQUE;
  c.mode = CPR_MODE_LOOP;
  c.policy = cf.policy;
  c.defenders = cf.defenders;
  c.reward_scheme = cf.scheme;
  c.activation_delay = 1.0;
  c.propagation_delay = cf.prop;
  c.activations = cf.steps;
  c.seed = seed;
  cpr_episode_record r{};
  if (oracle_run_episodes(&c, ep, 1, &r, 1) != 0) {
    why = "oracle_run_episodes failed";
    C.mismatches++;
    return false;
  }
  const eth::EthParams P = params_of(cf);
  std::vector<uint8_t> mem(eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  fill_garbage(mem);
  const eth::EthMem M = eth::eth_mem_at(mem.data(), P.cap_b, P.cap_e, P.n);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  eth::EthLane L;
  const int32_t hd = L.loop(P, S, M);
  if (L.dead) {
    C.capacity++;
    return true;
  }
  const eth::EBlock& hb = L.B(P, M, hd);
  C.episodes++;
  C.steps += cf.steps;
  if (hb.rew_att / 32.0 != r.reward_attacker || hb.rew_def / 32.0 != r.reward_defender ||
      hb.height != r.head_height || hb.time != r.chain_time || L.c_act != r.n_activations ||
      (cf.two_agents == 3 && hb.work != r.head_work)) {
    char buf[400];
    snprintf(buf, sizeof buf,
             "exp clique lane (ra %.5f rd %.5f h %d w %d tm %.17g k %d) oracle (%.5f %.5f %d %d "
             "%.17g %ld)",
             hb.rew_att / 32.0, hb.rew_def / 32.0, hb.height, hb.work, hb.time, L.c_act,
             r.reward_attacker, r.reward_defender, r.head_height, r.head_work, r.chain_time,
             (long)r.n_activations);
    why = buf;
    C.mismatches++;
    return false;
  }
  return true;
}

int main(int argc, char** argv) {
  const int eps = argc > 1 ? atoi(argv[1]) : 20;
  const int steps = argc > 2 ? atoi(argv[2]) : 200;
  const uint64_t seed = 0xE7E70000ull;
  std::vector<Cfg> cfgs;
  const double alphas[] = {0.1, 0.25, 0.35, 0.45};
  const double gammas[] = {0.0, 0.5, 0.9};
  for (double a : alphas)
    for (double g : gammas) {
      const int d = std::max(2, (int)std::ceil(1.0 / (1.0 - g)));
      for (int pol : {0, 1, 2, 3, 4, 5, 6})
        for (int sch : {0, 1}) cfgs.push_back(Cfg{a, g, d, pol, sch, steps, 0});
    }
  cfgs.push_back(Cfg{0.4, 0.75, 7, 6, 1, steps, 0});
  for (double a : alphas)
    for (int pol : {0, 1, 2, 3, 4, 9}) cfgs.push_back(Cfg{a, 0, 1, pol, 1, steps * 4, 1});
  // withholding.ml:29-52 gamma-* tasks (defender message delay 1e-4, and a longer one that
  // makes in-flight overlaps common), nakamoto_ssz policies 0..3
  for (double a : {0.1, 0.25, 0.35, 0.45, 0.5})
    for (double g : {0.0, 0.5, 0.75, 0.9})
      for (int pol : {0, 1, 2, 3})
        for (double prop : {1e-4, 0.05}) {
          const int d = std::max(2, (int)std::ceil(1.0 / (1.0 - g)));
          cfgs.push_back(Cfg{a, g, d, pol, 0, steps * 4, 2, prop});
        }
  // exponential-delay cliques: Ethereum (ethereum_ssz policies, both schemes) and Nakamoto
  // (nakamoto_ssz policies), fast and slow links
  for (int d : {1, 3, 7})
    for (double prop : {0.05, 0.6}) {
      for (int pol : {0, 1, 2, 3, 4})
        for (int sch : {0, 1}) cfgs.push_back(Cfg{0, 0, d, pol, sch, steps * 2, 3, prop});
      for (int pol : {0, 1, 2, 3}) cfgs.push_back(Cfg{0, 0, d, pol, 0, steps * 2, 4, prop});
    }
  Counters C;
  int shown = 0;
  for (auto& cf : cfgs)
    for (int e = 0; e < eps; e++) {
      std::string why;
      const bool ok = cf.two_agents >= 3   ? run_exp(cf, seed, e, C, why)
                      : cf.two_agents == 2 ? run_sm_loop(cf, seed, e, C, why)
                      : cf.two_agents == 1 ? run_loop(cf, seed, e, C, why)
                                           : run_gym(cf, seed, e, C, why);
      if (!ok && shown < 10) {
        shown++;
        fprintf(stderr,
                "MISMATCH alpha=%g gamma=%g d=%d pol=%d scheme=%d net=%d prop=%g ep=%d: %s\n",
                cf.alpha, cf.gamma, cf.defenders, cf.policy, cf.scheme, cf.two_agents, cf.prop,
                e, why.c_str());
      }
    }
  printf("{\"episodes\": %ld, \"steps\": %ld, \"mismatches\": %ld, \"capacity\": %ld}\n",
         C.episodes, C.steps, C.mismatches, C.capacity);
  return C.mismatches ? 1 : 0;
}
