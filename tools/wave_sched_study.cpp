// Study (not product code): how well wave-coherent dispatch (cpr_amd/csrc/wave_sched.h)
// fills a wave on BASELINE configs[4]'s shape (bk_ssz, k = 8, constant rewards, alpha .33,
// gamma .5, d = 2, 2048-step gym episodes, a random table policy), emulated on the host:
// 64 B_k lanes run the rollout driver of k_bk_rollout (roll_fetch items: the events up to
// the attacker's next interaction, the interaction ending the step), each iteration runs the
// class most lanes hold. Prints items per iteration (lanes doing work out of 64) overall and
// per class, and the class mix.
//
// build: hipcc -O2 -std=c++17 -ffp-contract=off -x hip --offload-arch=gfx950 \
//        tools/wave_sched_study.cpp -o build/wave_sched_study
// usage: build/wave_sched_study [steps per lane] [gamma] [alpha] [k]
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../cpr_amd/csrc/bk_lane.h"
#include "../oracle/src/keyed_stream.h"

using namespace cpr;

enum { C_CLOCK, C_DAG, C_TX, C_RX, C_ON, C_MV, C_MDV, C_ATTACK, C_POW0, C_N };
static const char* kNames[C_N] = {"clock", "dag", "tx", "rx", "on", "mv", "mdv", "attack",
                                  "pow0"};

struct Lane {
  bk::BkLane L;
  std::vector<uint8_t> mem;
  bk::BkMem M;
  Stream S;
  uint64_t ep;
  int cls = -1;
  uint32_t ev = 0;
  int32_t s = 0;
  int32_t att = 0;
  long t = 0;
  bool fresh = false, idle = false;
};

int main(int argc, char** argv) {
  const long n_steps = argc > 1 ? atol(argv[1]) : 4096;
  const double gamma = argc > 2 ? atof(argv[2]) : 0.5;
  const double alpha = argc > 3 ? atof(argv[3]) : 0.33;
  const int k = argc > 4 ? atoi(argv[4]) : 8;
  const int steps = 2048, d = 2, D = 4, W = 64;
  std::vector<uint8_t> table((size_t)D * D * (k + 1) * (k + 1) * 3);
  uint64_t x = 12345;
  for (auto& t : table) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    t = (uint8_t)((x >> 33) % 8);
  }
  bk::BkParams P{};
  P.t_att = oracle::alpha_threshold(alpha);
  P.d = d;
  P.n = d + 1;
  P.net = 0;
  P.mode = 0;
  P.policy = 4;  // CPR_BK_POLICY_TABLE
  P.scheme = 0;
  P.k = k;
  const int span = steps + 2;
  P.cap_v = 64;
  while (P.cap_v < span + 64 && P.cap_v < 4096) P.cap_v <<= 1;
  P.cap_q = P.cap_v / 2;
  P.cap_e = 256 + 512 * P.n + (gamma == 0.0 ? 2 * P.d * span : 0);
  P.cap_d = 64;
  P.table_dim = D;
  P.table = table.data();
  P.ev = 1.0;
  P.delta = 1e-9;
  P.dmax = (d - 1.) / d * 1e-9 / gamma;
  P.max_steps = steps;
  P.max_progress = __builtin_inf();
  P.max_time = __builtin_inf();
  std::vector<Lane> lanes(W);
  for (int i = 0; i < W; ++i) {
    Lane& l = lanes[i];
    l.mem.resize(bk::bk_lane_bytes(P));
    l.M = bk::bk_mem_at(l.mem.data(), P);
    l.ep = (uint64_t)i;
    l.S = Stream{0x5EED0000u, 0u, (uint32_t)l.ep, 0u};
    l.L.gym_reset(P, l.S, l.M);
    // at the decision point: the first action
    l.L.apply(P, l.M, bk::bk_policy(P, l.L.observe(P, l.M)));
    ++l.L.steps;
    l.att = l.L.priv;
  }
  long iters = 0, items = 0, per_cls_items[C_N] = {}, per_cls_iters[C_N] = {};
  for (;;) {
    for (Lane& l : lanes) {  // roll_fetch
      if (l.idle || l.cls >= 0) continue;
      double t;
      uint32_t ev;
      int32_t s;
      if (l.L.dead) {
        l.ev = 0xffffffffu;
        l.cls = C_ATTACK;
        continue;
      }
      if (!l.L.pop(l.M, &t, &ev, &s)) {
        l.L.fail(6);
        l.ev = 0xffffffffu;
        l.cls = C_ATTACK;
        continue;
      }
      l.L.now = t;
      l.ev = ev;
      l.s = s;
      const uint32_t ty = ev & 7u;
      if (ty == 4u && (ev >> 5) == 0u)
        l.cls = C_ATTACK;
      else if (ty == bk::EV_DAG && (ev >> 5) == 0u && ((ev >> 3) & 3u) == bk::KD_POW)
        l.cls = C_POW0;
      else
        l.cls = (int)ty;
    }
    int cnt[C_N] = {};
    for (Lane& l : lanes)
      if (l.cls >= 0) cnt[l.cls]++;
    int best = -1, bn = 0;
    for (int c = 0; c < C_N; ++c)
      if (cnt[c] > bn) {
        bn = cnt[c];
        best = c;
      }
    if (best < 0) break;
    ++iters;
    items += bn;
    per_cls_items[best] += bn;
    per_cls_iters[best] += 1;
    for (Lane& l : lanes) {
      if (l.cls != best) continue;
      l.cls = -1;
      if (best == C_POW0) {
        const int32_t v = l.L.append_vote(P, l.S, l.M, 0, l.L.priv);
        l.L.push_now(P, l.M, bk::mkev(bk::EV_MV, 0, bk::KD_POW), v);
        continue;
      }
      if (best != C_ATTACK) {
        l.L.handle(P, l.S, l.M, l.ev, l.s);
        continue;
      }
      if (l.ev != 0xffffffffu) l.L.prepare(P, l.M, (l.ev >> 3) & 3u, l.s);
      if (l.fresh) {
        l.fresh = false;
      } else {
        const int32_t hd = l.L.head(P, l.M, l.att);
        const double progress = (double)(l.L.X(P, l.M, hd).height * P.k);
        const bool done = l.L.dead ||
                          !(l.L.steps < P.max_steps && progress < P.max_progress && l.L.now < P.max_time);
        ++l.t;
        if (done) {
          l.ep += (uint64_t)W;
          l.S = Stream{0x5EED0000u, 0u, (uint32_t)l.ep, 0u};
          l.L.init(P, l.S, l.M);
          l.fresh = true;
          continue;
        }
      }
      if (l.t >= n_steps) {
        l.idle = true;
        continue;
      }
      l.L.apply(P, l.M, bk::bk_policy(P, l.L.observe(P, l.M)));
      ++l.L.steps;
      l.att = l.L.priv;
    }
  }
  printf("{\"lanes\": %d, \"steps_per_lane\": %ld, \"iterations\": %ld, \"items\": %ld, "
         "\"lanes_busy_per_iteration\": %.2f, \"classes\": {",
         W, n_steps, iters, items, (double)items / (double)iters);
  for (int c = 0; c < C_N; ++c)
    printf("%s\"%s\": {\"items\": %ld, \"iterations\": %ld, \"busy\": %.2f}", c ? ", " : "",
           kNames[c], per_cls_items[c], per_cls_iters[c],
           per_cls_iters[c] ? (double)per_cls_items[c] / per_cls_iters[c] : 0.0);
  printf("}}\n");
  return 0;
}
