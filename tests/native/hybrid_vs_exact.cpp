// TEST INFRASTRUCTURE ONLY. Differential fuzzer for the hybrid exact re-run
// (cpr_amd/csrc/nak_hybrid.h: closed-form lane, event engine around the flagged windows)
// against the whole-episode event engine in Nakamoto mode (ethereum_lane.h, the re-run
// before the hybrid; itself pinned against the oracle by eth_vs_oracle and the GPU parity
// tests), both compiled here for the host, on the same keyed stream: every episode output
// the re-run writes (rewards, height, chain time, head miner, steps, activations, sim time,
// engine status). Propagation delays up to 0.3 activation delays make overlapping windows
// common, so most episodes enter and leave the engine several times.
// Each episode runs the hybrid twice: (1) every region in one host buffer, records mode
// (block times kept); (2) the re-run kernel's layout (kernels_eth.hip rerun_episode): the
// closed form's private-chain ring in its own 16-slot buffer (the workgroup's hring), the
// engine's block ring apart from the rest of its lane (eth_mem_split: visibility, heap, tips
// and scratch in a buffer of the kernel's dynamic LDS, 160 KiB - 128, the heap capacity
// reduced to what fits and the episode redone with the whole region in HBM when it
// outgrows that), records mode on even episodes and summary-only (no block times) on odd
// ones. Every buffer carries a canary tail that must survive the episode untouched.
// usage: hybrid_vs_exact [episodes per config] [steps]; one JSON line; exit 1 on mismatch
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "garbage.h"
#include "../../cpr_amd/csrc/nak_hybrid.h"
#include "../../oracle/src/keyed_stream.h"

using namespace cpr;

struct Cfg {
  double alpha, gamma, prop;
  int policy;  // nakamoto_ssz 0..3, 4 = random table
  int steps;
};

// a host buffer of n bytes followed by a canary tail
struct Guarded {
  static constexpr size_t kTail = 256;
  std::vector<uint8_t> v;
  size_t n = 0;
  explicit Guarded(size_t bytes) : v(bytes + kTail, 0), n(bytes) {
    fill_garbage(v.data(), n);  // GARBAGE=<seed>: pooled device memory's leftovers
    arm();
  }
  uint8_t* data() { return v.data(); }
  void arm() { std::fill(v.begin() + (long)n, v.end(), (uint8_t)0xCD); }
  bool intact() const {
    for (size_t i = n; i < v.size(); ++i)
      if (v[i] != 0xCD) return false;
    return true;
  }
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
  long layout_mism = 0, canary_hits = 0, hbm_retries = 0, split_cfgs = 0, reduced_cfgs = 0;
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
    fill_garbage(m1);
    Guarded m2(eth::eth_lane_bytes(EP.cap_b, EP.cap_e, EP.n));
    Guarded m3(hybrid_bytes(NP.cap));
    const eth::EthMem M1 = eth::eth_mem_at(m1.data(), EP.cap_b, EP.cap_e, EP.n);
    const eth::EthMem M2 = eth::eth_mem_at(m2.data(), EP.cap_b, EP.cap_e, EP.n);
    const LaneMem LM = hybrid_mem(m3.data(), NP.cap);
    // the kernel's layout: heap capacity in "LDS" as rerun_episode computes it
    const int64_t lds_bytes = 160 * 1024 - 128;
    const int64_t heap = eth::align128((int64_t)EP.cap_e * 24);
    const int64_t other = eth::eth_rest_bytes(EP.cap_b, EP.cap_e, EP.n) - heap;
    const int64_t room = (lds_bytes - other) / 128 * 128;
    const int32_t lds_cap_e = room >= heap ? EP.cap_e : (room >= 256 * 24 ? (int32_t)(room / 24) : -1);
    Guarded kb(eth::eth_lane_bytes(EP.cap_b, EP.cap_e, EP.n) + hybrid_bytes(NP.cap));
    Guarded klds((size_t)lds_bytes);
    Guarded kring((size_t)RING * 8);
    if (lds_cap_e > 0) ++split_cfgs;
    if (lds_cap_e > 0 && lds_cap_e < EP.cap_e) ++reduced_cfgs;
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
      bool ok = ra == xb.rew_att / 32.0 && rd == xb.rew_def / 32.0 && tm == xb.time &&
                h == xb.height && miner == xb.miner && R.steps == X.steps &&
                R.acts == X.c_act && R.now == X.now && est == X.status;
      // the kernel's layout (rerun_episode): attempt 0 split (heap at lds_cap_e), attempt 1
      // (only after the reduced heap overflowed) the whole region in HBM
      const bool recs = (e & 1) == 0;
      HybridResult K{};
      eth::EthLane KE;
      NakLane KL;
      int attempts = 0;
      for (int attempt = lds_cap_e < 0 ? 1 : 0; attempt < 2; ++attempt) {
        ++attempts;
        eth::EthParams PA = EP;
        if (attempt == 0) PA.cap_e = lds_cap_e;
        const eth::EthMem KM = attempt == 0
                                   ? eth::eth_mem_split(kb.data(), klds.data(), PA.cap_b, PA.cap_e, PA.n)
                                   : eth::eth_mem_at(kb.data(), EP.cap_b, EP.cap_e, EP.n);
        LaneMem KLM = hybrid_mem(kb.data() + eth::eth_lane_bytes(EP.cap_b, EP.cap_e, EP.n), NP.cap);
        KLM.times = recs;
        KLM.ring = (double*)kring.data();
        K = nak_hybrid_episode(NP, PA, S, KLM, KM, KE, KL);
        if (attempt == 0 && K.entries && KE.dead == 2 && PA.cap_e < EP.cap_e) continue;
        break;
      }
      hbm_retries += attempts - 1;
      {
        double kra, krd, ktm;
        int32_t kh;
        if (K.closed) {
          kra = K.hd.ra;
          krd = K.hd.h - K.hd.ra;
          ktm = K.hd.tm;
          kh = K.hd.h;
        } else {
          const eth::EthMem KM = attempts == 2 || lds_cap_e < 0
                                     ? eth::eth_mem_at(kb.data(), EP.cap_b, EP.cap_e, EP.n)
                                     : eth::eth_mem_split(kb.data(), klds.data(), EP.cap_b,
                                                          lds_cap_e, EP.n);
          const eth::EBlock& hb = KE.B(EP, KM, K.ehd);
          kra = hb.rew_att / 32.0;
          krd = hb.rew_def / 32.0;
          ktm = hb.time;
          kh = hb.height;
        }
        const uint32_t kst = K.entries ? KE.status : 0u;
        // summary-only runs keep no block times: the closed form's chain time is not kept
        const bool tm_ok = ktm == xb.time || (!recs && K.closed);
        const bool kok = kra == xb.rew_att / 32.0 && krd == xb.rew_def / 32.0 && tm_ok &&
                         kh == xb.height && K.steps == X.steps && K.acts == X.c_act &&
                         K.now == X.now && kst == X.status;
        if (!kok) {
          ++layout_mism;
          ok = false;
        }
      }
      for (Guarded* g : {&m2, &m3, &kb, &klds, &kring})
        if (!g->intact()) {
          ++canary_hits;
          ok = false;
          g->arm();
        }
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
         "\"entries\": %ld, \"ended_closed\": %ld, \"layout_mismatches\": %ld, "
         "\"canary_hits\": %ld, \"hbm_retries\": %ld, \"split_configs\": %ld, "
         "\"reduced_heap_configs\": %ld}\n",
         episodes, acts, mism, entered, entries, ended_closed, layout_mism, canary_hits,
         hbm_retries, split_cfgs, reduced_cfgs);
  return mism ? 1 : 0;
}
