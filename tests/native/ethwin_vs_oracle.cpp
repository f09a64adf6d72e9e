// TEST INFRASTRUCTURE ONLY. Differential fuzzer for the Ethereum window lane
// (cpr_amd/csrc/eth_window.h, compiled here for the host) against the CPU oracle's event-
// driven restatement (oracle/src/ethereum.cpp GymEthereum), step by step on the same keyed
// stream: all ten observation fields (the three dry-run uncle selections included) before
// every action and the step info after it. An episode the lane flags for the exact re-run
// (W_REDO: overlap, unresolved tie, capacity) stops being compared at that step — the fused
// kernel re-runs it on the event engine — and is counted; the tie-heavy and overlap-heavy
// configurations make sure those paths occur.
// usage: ethwin_vs_oracle [episodes per config] [steps]; one JSON line; exit 1 on mismatch
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../cpr_amd/csrc/eth_window.h"
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
  int policy;  // 0..4 ethereum_ssz policies, 5 random actions, 6 random biased to release
  int scheme;
  int steps;
  double prop;
  // engine.ml:209-214's other two done clauses (+inf = off)
  double max_time = __builtin_inf();
  double max_progress = __builtin_inf();
};

struct Counters {
  long episodes = 0, mismatches = 0, redo = 0, ties = 0, steps = 0, overlaps = 0, ca_pairs = 0;
};

static eth::EthParams params_of(const Cfg& cf) {
  eth::EthParams P{};
  P.t_att = oracle::alpha_threshold(cf.alpha);
  P.d = cf.defenders;
  P.n = P.d + 1;
  P.net = 0;
  P.mode = 0;
  P.nak = 0;
  P.policy = cf.policy < 5 ? cf.policy : 0;
  P.scheme = cf.scheme;
  P.cap_b = 64;
  while (P.cap_b < cf.steps + 2) P.cap_b <<= 1;
  P.ev = 1.0;
  P.delta = cf.prop;
  const double dd = cf.defenders;
  P.dmax = (dd - 1.) / dd * cf.prop / cf.gamma;
  P.max_steps = cf.steps;
  P.max_progress = cf.max_progress;
  P.max_time = cf.max_time;
  return P;
}

static bool run_gym(const Cfg& cf, uint64_t seed, uint64_t ep, Counters& C, std::string& why) {
  oracle::GymParams gp;
  gp.alpha = cf.alpha;
  gp.gamma = cf.gamma;
  gp.defenders = cf.defenders;
  gp.max_steps = cf.steps;
  gp.unit_obs = false;
  gp.propagation_delay = cf.prop;
  gp.max_progress = cf.max_progress;
  gp.max_time = cf.max_time;
  oracle::GymEthereum g(gp, cf.scheme, 1, nullptr, seed, ep);
  double obs[10];
  g.reset(obs);
  const eth::EthParams P = params_of(cf);
  std::vector<uint8_t> mem(ethw::win_lane_bytes(P.cap_b));
  // GARBAGE=<seed>: the lane's region starts out filled with pseudo-random bytes, as the
  // device's pooled memory holds whatever the previous launch left: no output may depend on
  // a byte the lane did not write first
  if (const char* g = getenv("GARBAGE")) {
    uint64_t x = (uint64_t)atoll(g) * 0x9e3779b97f4a7c15ull + ep;
    for (auto& v : mem) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      v = (uint8_t)(x >> 56);
    }
  }
  const ethw::WinMem M = ethw::win_mem_at(mem.data(), P.cap_b);
  const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
  ethw::WinLane L;
  L.gym_reset(P, S, M);
  char buf[700];
  bool ok = true;
  for (int s = 0;; s++) {
    if (L.status & ethw::W_REDO) {
      C.redo++;
      if (L.status & ST_OVERLAP) C.overlaps++;
      return true;
    }
    const oracle::EthObs o = g.observe_int();
    const eth::EthObs e = L.observe(P, M, true);
    const int ov[10] = {o.public_height, o.public_work, o.private_height, o.private_work,
                        o.diff_height, o.diff_work, o.public_orphans,
                        o.private_orphans_inclusive, o.private_orphans_exclusive, o.event};
    const int ev[10] = {e.public_height, e.public_work, e.private_height, e.private_work,
                        e.diff_height, e.diff_work, e.public_orphans,
                        e.private_orphans_inclusive, e.private_orphans_exclusive, e.event};
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
    if (cf.policy < 5) {
      act = oracle::eth_policy(cf.policy, o);
    } else {
      const uint32_t r = mix(ep, s);
      act = (int)(r % 24);
      if (cf.policy == 6 && (r >> 8) % 2 == 0)
        act = (int)(((r >> 12) % 4 == 0 ? 1 : 2 + (r >> 14) % 3) * 4 + (r >> 20) % 4);
    }
    bool done = false;
    oracle::StepInfo info{};
    g.step(act, obs, &done, &info);
    bool ldone = false;
    const int32_t hd = L.gym_step(P, S, M, act, &ldone);
    C.steps++;
    if (L.status & ethw::W_REDO) {
      C.redo++;
      if (L.status & ST_OVERLAP) C.overlaps++;
      return true;
    }
    const ethw::WBlock& hb = L.B(P, M, hd);
    const double ra = hb.rew_att / 32.0, rd = hb.rew_def / 32.0;
    if (ra != info.episode_reward_attacker || rd != info.episode_reward_defender ||
        hb.height != info.head_height || hb.work != info.head_work ||
        (double)hb.work != info.episode_progress || L.time_of(P, M, hd) != info.episode_chain_time ||
        L.now != info.episode_sim_time || L.c_act != info.episode_n_activations ||
        hb.miner != info.head_miner || ldone != done || L.steps != info.episode_n_steps) {
      snprintf(buf, sizeof buf,
               "step %d head lane (ra %.5f rd %.5f h %d w %d tm %.17g t %.17g k %d m %d done %d) "
               "oracle (ra %.5f rd %.5f h %d w %d tm %.17g t %.17g k %ld m %d done %d)",
               s, ra, rd, (int)hb.height, hb.work, L.time_of(P, M, hd), L.now, L.c_act, hb.miner, (int)ldone,
               info.episode_reward_attacker, info.episode_reward_defender, info.head_height,
               info.head_work, info.episode_chain_time, info.episode_sim_time,
               info.episode_n_activations, info.head_miner, (int)done);
      why = buf;
      ok = false;
      break;
    }
    if (done) break;
  }
  // the lane's common-ancestor walk (run jumps included) against a brute-force restatement
  // of Dagtools.common_ancestor (max (height, serial) over the intersection of the two
  // all-edge ancestor sets) for random pairs of this episode's blocks
  if (ok && !(L.status & ethw::W_REDO) && L.newest > 2) {
    std::vector<uint8_t> in_a(L.newest + 1), in_b(L.newest + 1);
    auto anc = [&](int32_t x, std::vector<uint8_t>& in) {
      std::fill(in.begin(), in.end(), 0);
      std::vector<int32_t> st{x};
      while (!st.empty()) {
        const int32_t s = st.back();
        st.pop_back();
        if (s < 0 || in[s]) continue;
        in[s] = 1;
        const ethw::WBlock& b = L.B(P, M, s);
        for (int i = 0; i < b.np; ++i) st.push_back(b.p[i]);
      }
    };
    for (int t = 0; t < 64; ++t) {
      const int32_t a = (int32_t)(mix(ep * 977 + t, 1) % (uint32_t)(L.newest + 1));
      const int32_t b = (int32_t)(mix(ep * 977 + t, 2) % (uint32_t)(L.newest + 1));
      anc(a, in_a);
      anc(b, in_b);
      int32_t best = -1;
      for (int32_t s = 0; s <= L.newest; ++s)
        if (in_a[s] && in_b[s] &&
            (best < 0 || L.B(P, M, s).height > L.B(P, M, best).height ||
             (L.B(P, M, s).height == L.B(P, M, best).height && s > best)))
          best = s;
      const int32_t got = L.common_ancestor(P, M, a, b);
      C.ca_pairs++;
      if (got != best && !L.dead) {
        snprintf(buf, sizeof buf, "common_ancestor(%d, %d) lane %d brute force %d", a, b, got, best);
        why = buf;
        ok = false;
        break;
      }
    }
  }
  C.episodes++;
  if (L.status & ST_TIE) C.ties++;
  if (!ok) C.mismatches++;
  return ok;
}

int main(int argc, char** argv) {
  const int per = argc > 1 ? atoi(argv[1]) : 20;
  const int steps = argc > 2 ? atoi(argv[2]) : 400;
  std::vector<Cfg> cfgs;
  const double alphas[] = {0.1, 0.25, 0.33, 0.4, 0.45, 0.5};
  const double gammas[] = {0.0, 0.3, 0.5, 0.75, 0.9};
  for (int pol = 0; pol <= 6; ++pol)
    for (double a : alphas)
      for (double g : gammas) {
        int d = (int)std::ceil(1.0 / (1.0 - g));
        if (d < 2) d = 2;
        cfgs.push_back({a, g, d, pol, (pol + (int)(a * 100)) % 2, steps, 1e-9});
      }
  // more defenders than the gym's rule, and tie-heavy (tiny delay: same-instant races) and
  // overlap-heavy (long delay: activations inside deliveries) networks
  for (int pol : {3, 5, 6})
    for (double a : {0.33, 0.45}) {
      cfgs.push_back({a, 0.5, 5, pol, 0, steps, 1e-9});
      cfgs.push_back({a, 0.6, 12, pol, 1, steps, 1e-9});
      cfgs.push_back({a, 0.5, 2, pol, 0, steps, 1e-13});
      cfgs.push_back({a, 0.9, 11, pol, 0, steps, 1e-13});
      cfgs.push_back({a, 0.75, 4, pol, 1, steps, 1e-12});
      cfgs.push_back({a, 0.5, 2, pol, 0, steps, 0.05});
      cfgs.push_back({a, 0.9, 11, pol, 1, steps, 0.01});
    }
  // full-length episodes with long private forks (the common-ancestor walk's run jumps,
  // eth_window.h q_advance / common_ancestor: selfish_release at gamma = 0 forks for
  // hundreds of blocks), every policy and both random fuzzers
  for (int pol = 0; pol <= 6; ++pol)
    for (double g : {0.0, 0.5})
      cfgs.push_back({0.45, g, 2, pol, pol % 2, 2016, 1e-9});
  // episodes ended by max_time / max_progress before max_steps (engine.ml:209-214)
  for (int pol : {1, 3, 5})
    for (double a : {0.25, 0.45})
      for (double g : {0.0, 0.5, 0.9}) {
        const int d = g == 0.9 ? 10 : 2;
        Cfg c{a, g, d, pol, pol % 2, steps, 1e-9};
        c.max_time = 0.3 * steps;
        cfgs.push_back(c);
        c.max_time = __builtin_inf();
        c.max_progress = steps / 5;
        cfgs.push_back(c);
        c.max_time = 0.5 * steps;
        c.prop = 0.05;  // overlaps: the re-run path's episodes stop being compared at W_REDO
        cfgs.push_back(c);
      }
  Counters C;
  long shown = 0;
  for (size_t ci = 0; ci < cfgs.size(); ++ci)
    for (int e = 0; e < per; ++e) {
      std::string why;
      if (!run_gym(cfgs[ci], 0x5EED0000ull + ci, (uint64_t)e, C, why) && shown++ < 8)
        fprintf(stderr, "MISMATCH cfg a=%g g=%g d=%d pol=%d scheme=%d prop=%g ep=%d: %s\n",
                cfgs[ci].alpha, cfgs[ci].gamma, cfgs[ci].defenders, cfgs[ci].policy,
                cfgs[ci].scheme, cfgs[ci].prop, e, why.c_str());
    }
  printf("{\"configs\": %zu, \"episodes\": %ld, \"steps\": %ld, \"mismatches\": %ld, "
         "\"redo\": %ld, \"overlaps\": %ld, \"tie_episodes\": %ld, \"ca_pairs\": %ld}\n",
         cfgs.size(), C.episodes, C.steps, C.mismatches, C.redo, C.overlaps, C.ties, C.ca_pairs);
  return C.mismatches ? 1 : 0;
}
