// TEST INFRASTRUCTURE ONLY. Differential fuzzer: the device lane state machine
// (cpr_amd/csrc/nakamoto_lane.h, compiled here for the host) against the CPU oracle's
// faithful event-driven restatement (oracle/src/des.cpp), step by step, on the same keyed
// stream. Prints one JSON summary line; exit code 1 on any unexplained mismatch.
// Build: tests/native/Makefile (hipcc, host code only is executed).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "garbage.h"
#include "../../cpr_amd/csrc/nakamoto_lane.h"
#include "../../oracle/src/des.h"

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
  int policy;  // 0..3, 5 = random actions, 6 = random with bias to match
  int steps;
  int two_agents;  // 1: loop mode on the two-agents network; 2: gym episodes in the flagged
                   // abstract-gamma mode (CPR_NET_ABSTRACT_GAMMA)
};

// host stand-in for the kernel's per-lane memory (ring, spill, replay scratch)
struct HostMem {
  std::vector<double> ring, spill;
  std::vector<uint8_t> replay;
  explicit HostMem(const NakParams& P) : ring(RING), spill(P.cap), replay(REPLAY_BYTES) {
    fill_garbage(ring.data(), ring.size() * sizeof(double));
    fill_garbage(spill.data(), spill.size() * sizeof(double));
    fill_garbage(replay);
  }
  LaneMem lane() {
    LaneMem M;
    M.ring = ring.data();
    M.spill = spill.data();
    M.ring_stride = M.spill_stride = 1;
    M.cap = (int32_t)spill.size();
    M.replay = ReplayMem::at(replay.data());
    return M;
  }
};

extern "C" int oracle_two_agents_task(int, void*, uint64_t, uint64_t, double, int, int, int64_t*,
                                      double*, double*, double*, int32_t*, uint32_t*);

struct Counters {
  long episodes = 0, mismatches = 0, tie_eps = 0, tie_mismatch = 0, overlap_eps = 0,
       lane_tie = 0, unresolved = 0;
  // odd episodes of the two-defender gym configurations run resolve<..., TT = 1> (the
  // closed-form tie rule of the d = 2 summary-only kernels) instead of the heap replay; a
  // tie that rule does not cover (several released blocks) ends the comparison, as the
  // kernel hands such an episode to the exact re-run
  long tt_episodes = 0, tt_ties = 0, tt_unresolved = 0;
};

static bool run_gym(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C, std::string& why) {
  oracle::GymParams gp;
  gp.alpha = cf.alpha;
  gp.gamma = cf.gamma;
  gp.defenders = cf.defenders;
  gp.max_steps = cf.steps;
  gp.unit_obs = false;
  gp.abstract_gamma = cf.two_agents == 2;
  oracle::GymNakamoto g(gp, 1, nullptr, seed, ep);
  double obs[4];
  g.reset(obs);

  NakParams P{};
  P.t_att = oracle::alpha_threshold(cf.alpha);
  P.d = cf.defenders;
  P.ev = 1.0;
  P.delta = 1e-9;
  const double dd = cf.defenders;
  P.dmax = (dd - 1.) / dd * 1e-9 / cf.gamma;
  P.arrive = std::isfinite(P.dmax) ? 1 : 0;
  if (cf.two_agents == 2) {  // as capi.hip validate for CPR_NET_ABSTRACT_GAMMA
    P.delta = 0.0;
    P.dmax = 0.0;
    P.arrive = 1;
    P.abstract_g = 1;
    P.gamma = cf.gamma;
  }
  P.max_steps = cf.steps;
  P.max_progress = __builtin_inf();
  P.max_time = __builtin_inf();
  P.policy = cf.policy < 4 ? cf.policy : 0;
  P.cap = cf.steps + 64;
  HostMem mem(P);
  const LaneMem M = mem.lane();
  Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  NakLane L;
  L.init();
  L.activate(P, S, M);
  bool ok = true;
  char buf[512];
  const bool tt = cf.two_agents == 0 && cf.defenders == 2 && (ep & 1);
  bool tt_stopped = false;
  for (int s = 0;; s++) {
    oracle::NakObs o = g.observe_int();
    int32_t h, a, d, e;
    L.observe(&h, &a, &d, &e);
    if (h != o.public_blocks || a != o.private_blocks || d != o.diff_blocks || e != o.event) {
      snprintf(buf, sizeof buf, "step %d obs lane (%d,%d,%d,%d) oracle (%d,%d,%d,%d)", s, h, a, d, e,
               o.public_blocks, o.private_blocks, o.diff_blocks, o.event);
      why = buf;
      ok = false;
      break;
    }
    int act;
    if (cf.policy < 4)
      act = oracle::nak_policy(cf.policy, o, nullptr);
    else {
      uint32_t r = mix(ep, s);
      act = (int)(r & 3);
      if (cf.policy == 6 && (r >> 8) % 3 == 0) act = 2;
    }
    bool done = false;
    oracle::StepInfo info{};
    g.step(act, obs, &done, &info);
    L.apply(act);
    if (tt) {
      L.resolve<Stream, -1, 1>(P, S, M);
      if (L.status & ST_TIE_UNRESOLVED) {
        tt_stopped = true;
        break;
      }
    } else {
      L.resolve(P, S, M);
    }
    L.activate(P, S, M);
    BRef hd = L.head(P, M);
    const double hd_tm = L.time_of(M, hd);
    if (hd.ra != (int)info.episode_reward_attacker || hd.h - hd.ra != (int)info.episode_reward_defender ||
        hd.h != info.head_height || hd_tm != info.episode_chain_time || L.t != info.episode_sim_time ||
        L.k != info.episode_n_activations || miner_of(P, S, hd.k) != info.head_miner) {
      snprintf(buf, sizeof buf,
               "step %d head lane (ra %d h %d tm %.17g t %.17g k %d miner %d) oracle (ra %g rd %g h %d "
               "tm %.17g t %.17g k %ld miner %d)",
               s, hd.ra, hd.h, hd_tm, L.t, L.k, miner_of(P, S, hd.k), info.episode_reward_attacker,
               info.episode_reward_defender, info.head_height, info.episode_chain_time,
               info.episode_sim_time, info.episode_n_activations, info.head_miner);
      why = buf;
      ok = false;
      break;
    }
    if (done) break;
  }
  uint32_t dg = g.sim->diag;
  C.episodes++;
  if (tt) {
    C.tt_episodes++;
    if (L.status & ST_TIE) C.tt_ties++;
    if (tt_stopped) {
      C.tt_unresolved++;
      return true;
    }
  }
  if (L.status & ST_TIE) C.lane_tie++;
  if (L.status & ST_TIE_UNRESOLVED) C.unresolved++;
  if (dg & oracle::DIAG_TIE) C.tie_eps++;
  if (dg & oracle::DIAG_OVERLAP) C.overlap_eps++;
  if (!ok) {
    if (dg & (oracle::DIAG_TIE | oracle::DIAG_OVERLAP) || (L.status & (ST_TIE | ST_OVERLAP)))
      C.tie_mismatch++;
    else
      C.mismatches++;
  }
  return ok;
}

static bool run_loop(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C, std::string& why) {
  int64_t acts[2];
  double rew[2], ht, hp;
  int32_t hh;
  uint32_t dg;
  oracle_two_agents_task(1, nullptr, seed, ep, cf.alpha, cf.policy, cf.steps, acts, rew, &ht, &hp,
                         &hh, &dg);
  NakParams P{};
  P.t_att = oracle::alpha_threshold(cf.alpha);
  P.d = 1;
  P.ev = 1.0;
  P.arrive = 1;
  P.policy = cf.policy;
  P.max_steps = INT64_MAX;
  P.max_progress = __builtin_inf();
  P.max_time = __builtin_inf();
  P.cap = cf.steps + 64;
  HostMem mem(P);
  const LaneMem M = mem.lane();
  Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  NakLane L;
  L.init();
  for (int i = 0; i < cf.steps; i++) {
    L.activate(P, S, M);
    L.apply(L.policy_action(P));
    L.resolve(P, S, M);
  }
  BRef hd = L.head(P, M);
    const double hd_tm = L.time_of(M, hd);
  C.episodes++;
  if (hd.ra != (int)rew[0] || hd.h - hd.ra != (int)rew[1] || hd.h != hh || hd_tm != ht ||
      L.k != acts[0] + acts[1]) {
    char buf[256];
    snprintf(buf, sizeof buf, "loop lane (ra %d rd %d tm %.17g) oracle (%g %g %.17g)", hd.ra,
             hd.h - hd.ra, hd_tm, rew[0], rew[1], ht);
    why = buf;
    C.mismatches++;
    return false;
  }
  return true;
}

int main(int argc, char** argv) {
  int eps = argc > 1 ? atoi(argv[1]) : 200;
  int steps = argc > 2 ? atoi(argv[2]) : 300;
  uint64_t seed = 0x5eed0000ull;
  std::vector<Cfg> cfgs;
  const double alphas[] = {0.05, 0.25, 0.33, 0.45, 0.5};
  const double gammas[] = {0.0, 0.3, 0.5, 0.75, 0.9};
  for (double a : alphas)
    for (double g : gammas) {
      int d = std::max(2, (int)std::ceil(1.0 / (1.0 - g)));
      for (int pol : {0, 1, 2, 3, 5, 6}) cfgs.push_back(Cfg{a, g, d, pol, steps, 0});
    }
  cfgs.push_back(Cfg{0.33, 0.95, 42, 3, steps, 0});
  cfgs.push_back(Cfg{0.4, 0.5, 5, 6, steps, 0});
  cfgs.push_back(Cfg{0.3, 0.7, 5, 5, steps, 0});
  for (double a : alphas)
    for (int pol : {0, 1, 2, 3}) cfgs.push_back(Cfg{a, 0, 1, pol, steps * 4, 1});
  // flagged abstract-gamma mode: gamma 0 .. 1 incl. the reference-rejected gamma = 1
  for (double a : alphas)
    for (double g : {0.0, 0.5, 0.9, 1.0})
      for (int d : {1, 2, 5})
        for (int pol : {2, 3, 6}) cfgs.push_back(Cfg{a, g, d, pol, steps, 2});
  Counters C;
  int shown = 0;
  for (auto& cf : cfgs)
    for (int e = 0; e < eps; e++) {
      std::string why;
      bool ok = cf.two_agents == 1 ? run_loop(cf, seed, e, C, why) : run_gym(cf, seed, e, C, why);
      if (!ok && shown < 12) {
        shown++;
        fprintf(stderr, "MISMATCH alpha=%g gamma=%g d=%d pol=%d two=%d ep=%d: %s\n", cf.alpha,
                cf.gamma, cf.defenders, cf.policy, cf.two_agents, e, why.c_str());
      }
    }
  printf("{\"episodes\": %ld, \"mismatches\": %ld, \"oracle_tie_episodes\": %ld, "
         "\"lane_tie_episodes\": %ld, \"hazard_mismatches\": %ld, \"overlap_episodes\": %ld, \"unresolved\": %ld, "
         "\"tie_rule_episodes\": %ld, \"tie_rule_ties\": %ld, \"tie_rule_unresolved\": %ld}\n",
         C.episodes, C.mismatches, C.tie_eps, C.lane_tie, C.tie_mismatch, C.overlap_eps, C.unresolved,
         C.tt_episodes, C.tt_ties, C.tt_unresolved);
  return C.mismatches ? 1 : 0;
}
