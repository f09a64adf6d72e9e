// TEST INFRASTRUCTURE ONLY. Differential fuzzer for the hybrid exact re-run
// (cpr_amd/csrc/nak_hybrid.h: closed-form lane, event engine around the flagged windows)
// against the whole-episode event engine in Nakamoto mode (ethereum_lane.h, the re-run
// before the hybrid; itself pinned against the oracle by eth_vs_oracle and the GPU parity
// tests), both compiled here for the host, on the same keyed stream: every episode output
// the re-run writes (rewards, height, chain time, head miner, steps, activations, sim time,
// engine status). Propagation delays up to 0.3 activation delays make overlapping windows
// common, so most episodes enter and leave the engine several times.
// usage: hybrid_vs_exact [episodes per config] [steps]; one JSON line; exit 1 on mismatch
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../cpr_amd/csrc/nak_hybrid.h"
#include "../../oracle/src/keyed_stream.h"

using namespace cpr;

struct Cfg {
  double alpha, gamma, prop;
  int policy;  // nakamoto_ssz 0..3, 4 = random table
  int steps;
};

static const std::vector<uint8_t>& g_table() {
  static std::vector<uint8_t> t;
  if (t.empty()) {
    t.resize(8 * 8 * 2);
    uint64_t x = 0x4A4B1D00u;
    for (auto& a : t) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      a = (uint8_t)((x >> 33) % 4);
    }
  }
  return t;
}

int main(int argc, char** argv) {
  const int eps = argc > 1 ? atoi(argv[1]) : 20;
  const int steps = argc > 2 ? atoi(argv[2]) : 400;
  std::vector<Cfg> cfgs;
  for (double a : {0.1, 0.25, 0.35, 0.45, 0.5})
    for (double g : {0.5, 0.75, 0.9})
      for (double prop : {1e-9, 1e-3, 0.05, 0.3})
        for (int pol : {0, 1, 2, 3, 4}) cfgs.push_back(Cfg{a, g, prop, pol, steps});
  long episodes = 0, mism = 0, entered = 0, entries = 0, ended_closed = 0, acts = 0;
  int shown = 0;
  for (const Cfg& cf : cfgs) {
    const int d = std::max(2, (int)std::ceil(1.0 / (1.0 - cf.gamma)));
    const double dd = d;
    NakParams NP{};
    NP.t_att = oracle::alpha_threshold(cf.alpha);
    NP.d = d;
    NP.ev = 1.0;
    NP.delta = cf.prop;
    NP.dmax = (dd - 1.) / dd * cf.prop / cf.gamma;
    NP.arrive = 1;
    NP.max_steps = cf.steps;
    NP.max_progress = __builtin_inf();
    NP.max_time = __builtin_inf();
    NP.policy = cf.policy;
    NP.table = g_table().data();
    NP.table_dim = 8;
    NP.cap = ((cf.steps + 2 + 63) / 64) * 64;
    eth::EthParams EP{};
    EP.t_att = NP.t_att;
    EP.d = d;
    EP.n = d + 1;
    EP.net = 0;
    EP.mode = 0;
    EP.nak = 1;
    EP.policy = cf.policy;
    EP.table = NP.table;
    EP.table_dim = 8;
    EP.scheme = 0;
    EP.cap_b = 64;
    while (EP.cap_b < cf.steps + 2) EP.cap_b <<= 1;
    EP.cap_e = 64 + 512 * EP.n + d * (cf.steps + 2);  // capi.hip validate_eth, finite dmax
    EP.ev = 1.0;
    EP.delta = cf.prop;
    EP.dmax = NP.dmax;
    EP.max_steps = cf.steps;
    EP.max_progress = __builtin_inf();
    EP.max_time = __builtin_inf();
    std::vector<uint8_t> m1(eth::eth_lane_bytes(EP.cap_b, EP.cap_e, EP.n));
    std::vector<uint8_t> m2(eth::eth_lane_bytes(EP.cap_b, EP.cap_e, EP.n));
    std::vector<uint8_t> m3(hybrid_bytes(NP.cap));
    const eth::EthMem M1 = eth::eth_mem_at(m1.data(), EP.cap_b, EP.cap_e, EP.n);
    const eth::EthMem M2 = eth::eth_mem_at(m2.data(), EP.cap_b, EP.cap_e, EP.n);
    const LaneMem LM = hybrid_mem(m3.data(), NP.cap);
    for (int e = 0; e < eps; ++e) {
      const uint64_t seed = 0x5eed1234u, ep = (uint64_t)e * 7919 + (uint64_t)cf.policy;
      const Stream S{(uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)ep, (uint32_t)(ep >> 32)};
      // whole-episode engine (kernels_eth.hip nak_rerun_one)
      eth::EthLane X;
      X.gym_reset(EP, S, M1);
      bool done = X.dead != 0;
      int32_t xh = 0;
      while (!done) xh = X.gym_step(EP, S, M1, eth::lane_action(EP, X.observe(EP, M1, false)), &done);
      const eth::EBlock& xb = X.B(EP, M1, xh);
      // hybrid
      eth::EthLane E;
      NakLane L;
      const HybridResult R = nak_hybrid_episode(NP, EP, S, LM, M2, E, L);
      double ra, rd, tm;
      int32_t h, miner;
      if (R.closed) {
        ra = R.hd.ra;
        rd = R.hd.h - R.hd.ra;
        tm = R.hd.tm;
        h = R.hd.h;
        miner = miner_of(NP, S, R.hd.k);
      } else {
        const eth::EBlock& hb = E.B(EP, M2, R.ehd);
        ra = hb.rew_att / 32.0;
        rd = hb.rew_def / 32.0;
        tm = hb.time;
        h = hb.height;
        miner = hb.miner;
      }
      const uint32_t est = R.entries ? E.status : 0u;
      const bool ok = ra == xb.rew_att / 32.0 && rd == xb.rew_def / 32.0 && tm == xb.time &&
                      h == xb.height && miner == xb.miner && R.steps == X.steps &&
                      R.acts == X.c_act && R.now == X.now && est == X.status;
      ++episodes;
      acts += X.c_act;
      entered += R.entries ? 1 : 0;
      entries += R.entries;
      ended_closed += R.closed;
      if (!ok) {
        ++mism;
        if (shown++ < 10)
          fprintf(stderr,
                  "MISMATCH a=%g g=%g prop=%g pol=%d ep=%d: ra %g/%g rd %g/%g h %d/%d tm %.17g/%.17g "
                  "miner %d/%d steps %ld/%ld acts %d/%d now %.17g/%.17g st %u/%u entries %d closed %d\n",
                  cf.alpha, cf.gamma, cf.prop, cf.policy, e, ra, xb.rew_att / 32.0, rd,
                  xb.rew_def / 32.0, h, xb.height, tm, xb.time, miner, xb.miner,
                  (long)R.steps, (long)X.steps, R.acts, X.c_act, R.now, X.now, est, X.status,
                  R.entries, R.closed);
      }
    }
  }
  printf("{\"episodes\": %ld, \"activations\": %ld, \"mismatches\": %ld, \"entered\": %ld, "
         "\"entries\": %ld, \"ended_closed\": %ld}\n",
         episodes, acts, mism, entered, entries, ended_closed);
  return mism ? 1 : 0;
}
