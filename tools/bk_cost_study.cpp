// Study (not product code): where the B_k lane's work goes on BASELINE configs[4]'s shape
// (bk_ssz, k = 8, constant rewards, alpha .33, gamma .5, d = 2, 2048-step gym episodes,
// a random table policy). The lane header is compiled for the host with CPR_BK_COST
// counting its work items per activation: skew-heap node visits, the children scans of
// confirming / propose / observe / apply / MadeVisible, events by type.
//
// build: hipcc -O2 -std=c++17 -ffp-contract=off -x hip --offload-arch=gfx950 \
//        tools/bk_cost_study.cpp -o build/bk_cost_study
// usage: build/bk_cost_study [episodes] [gamma] [policy: 0..3, 4 = table] [alpha] [k]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

static long g_cost[16];
#define CPR_BK_COST(id) (++g_cost[(id)])
#include "../cpr_amd/csrc/bk_lane.h"
#include "../oracle/src/keyed_stream.h"

using namespace cpr;

int main(int argc, char** argv) {
  const int episodes = argc > 1 ? atoi(argv[1]) : 50;
  const double gamma = argc > 2 ? atof(argv[2]) : 0.5;
  const int policy = argc > 3 ? atoi(argv[3]) : 4;
  const double alpha = argc > 4 ? atof(argv[4]) : 0.33;
  const int k = argc > 5 ? atoi(argv[5]) : 8;
  const int steps = 2048, d = 2;
  const int D = 4;  // table dim as bench.py configs[4]
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
  P.policy = policy;
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
  std::vector<uint8_t> mem(bk::bk_lane_bytes(P));
  long acts = 0, st = 0, cap = 0, hmax = 0, hsum = 0;
  for (int e = 0; e < episodes; ++e) {
    const bk::BkMem M = bk::bk_mem_at(mem.data(), P);
    const Stream S{0x5EED0000u, 0u, (uint32_t)e, 0u};
    bk::BkLane L;
    L.gym_reset(P, S, M);
    bool done = L.dead != 0;
    while (!done) L.gym_step(P, S, M, bk::bk_policy(P, L.observe(P, M)), &done);
    acts += L.c_act;
    st += L.steps;
    cap += (L.status & bk::BST_CAPACITY) ? 1 : 0;
    hsum += L.hused;
    hmax = L.hused > hmax ? L.hused : hmax;
  }
  const double a = (double)acts;
  const char* names[16] = {"push_visits", "pop_visits", "confirming_scan", "propose_scan",
                           "observe_scan", "apply_scan", "mdv_scan", "ev_clock", "ev_dag",
                           "ev_tx", "ev_rx", "ev_on", "ev_mv", "ev_mdv", "propose_calls",
                           "confirming_calls"};
  printf("{\"episodes\": %d, \"gamma\": %g, \"policy\": %d, \"alpha\": %g, \"k\": %d, "
         "\"capacity\": %ld, \"steps_per_activation\": %.3f, \"heap_high_water_mean\": %.1f, "
         "\"heap_high_water_max\": %ld, \"per_activation\": {",
         episodes, gamma, policy, alpha, k, cap, st / a, hsum / (double)episodes, hmax);
  for (int i = 0; i < 16; ++i) printf("%s\"%s\": %.2f", i ? ", " : "", names[i], g_cost[i] / a);
  printf("}}\n");
  return 0;
}
