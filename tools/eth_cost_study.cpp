// Study (not product code): where the Ethereum lane's work goes on the bench's configs[2]
// points (ethereum_ssz fn19 / selfish_release, constant rewards, 2016-step gym episodes).
// The lane header is compiled for the host with CPR_COST counting its work items (heap
// node visits per push / pop, payloads and their candidate scans, common-ancestor frontier
// steps, MadeVisible scans, events by type, share steps); printed per gym step, with the
// heap's high-water mark and node count at episode end.
//
// build: hipcc -O2 -std=c++17 -ffp-contract=off -x hip --offload-arch=gfx950 \
//        tools/eth_cost_study.cpp -o build/eth_cost_study
// usage: build/eth_cost_study [episodes] [gamma] [policy] [alpha]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

static long g_cost[16];
#define CPR_COST(id) (++g_cost[(id)])
#include "../cpr_amd/csrc/eth_window.h"
#include "../oracle/src/keyed_stream.h"

using namespace cpr;

int main(int argc, char** argv) {
  const int episodes = argc > 1 ? atoi(argv[1]) : 100;
  const double gamma = argc > 2 ? atof(argv[2]) : 0.5;
  const int policy = argc > 3 ? atoi(argv[3]) : 3;
  const double alpha = argc > 4 ? atof(argv[4]) : 0.45;
  const int steps = 2016;
  // envs.py:70-76: d = max(2, ceil(1 / (1 - gamma)))
  int d = (int)std::ceil(1.0 / (1.0 - gamma));
  if (d < 2) d = 2;
  eth::EthParams P{};
  P.t_att = oracle::alpha_threshold(alpha);
  P.d = d;
  P.n = d + 1;
  P.net = 0;
  P.mode = 0;
  P.nak = 0;
  P.policy = policy;
  P.scheme = 0;
  P.cap_b = 64;
  while (P.cap_b < steps + 2) P.cap_b <<= 1;
  P.ev = 1.0;
  P.delta = 1e-9;
  P.dmax = (d - 1.0) / d * 1e-9 / gamma;
  const int64_t extra = std::isfinite(P.dmax) ? (int64_t)d * (steps + 2) : 2 * (int64_t)d * (steps + 2);
  P.cap_e = 64 + 512 * P.n + (int32_t)extra;
  P.max_steps = steps;
  P.max_progress = __builtin_inf();
  P.max_time = __builtin_inf();
  std::vector<uint8_t> mem(eth::eth_lane_bytes(P.cap_b, P.cap_e, P.n));
  long acts = 0, hused = 0, cap = 0;
  for (int e = 0; e < episodes; ++e) {
    const eth::EthMem M = eth::eth_mem_at(mem.data(), P.cap_b, P.cap_e, P.n);
    const Stream S{0x5EED0000u, 0u, (uint32_t)e, 0u};
    eth::EthLane L;
    L.gym_reset(P, S, M);
    bool done = L.dead != 0;
    while (!done) {
      const eth::EthObs o = L.observe(P, M, false);
      L.gym_step(P, S, M, eth::eth_policy(P.policy, o), &done);
    }
    acts += L.c_act;
    hused += L.hused;
    cap += (L.status & eth::EST_CAPACITY) ? 1 : 0;
  }
  const double a = (double)acts;
  const char* names[16] = {"push_visits", "pop_visits", "payloads", "payload_scan", "ca_steps",
                           "mdv_scan", "ev_clock", "ev_dag", "ev_tx", "ev_rx", "ev_on",
                           "ev_mv", "ev_mdv", "share_steps", "sort", "candidates"};
  printf("{\"episodes\": %d, \"gamma\": %g, \"d\": %d, \"policy\": %d, \"alpha\": %g, "
         "\"capacity\": %ld, \"heap_nodes_used_mean\": %.1f, \"per_activation\": {",
         episodes, gamma, d, policy, alpha, cap, hused / (double)episodes);
  for (int i = 0; i < 16; ++i)
    printf("%s\"%s\": %.2f", i ? ", " : "", names[i], g_cost[i] / a);
  printf("}");
  // the window lane (eth_window.h) on the same episodes: episodes it hands to the exact
  // re-run and episodes with a replayed tie
  long redo = 0, ties = 0, unres = 0, ovl = 0, wacts = 0;
  for (int i = 0; i < 16; ++i) g_cost[i] = 0;
  std::vector<uint8_t> wmem(ethw::win_lane_bytes(P.cap_b));
  for (int e = 0; e < episodes; ++e) {
    const ethw::WinMem W = ethw::win_mem_at(wmem.data(), P.cap_b);
    const Stream S{0x5EED0000u, 0u, (uint32_t)e, 0u};
    ethw::WinLane L;
    L.gym_reset(P, S, W);
    bool done = L.dead != 0;
    while (!done) {
      const eth::EthObs o = L.observe(P, W, false);
      L.gym_step(P, S, W, eth::eth_policy(P.policy, o), &done);
    }
    redo += (L.status & ethw::W_REDO) ? 1 : 0;
    ties += (L.status & ST_TIE) ? 1 : 0;
    unres += (L.status & ST_TIE_UNRESOLVED) ? 1 : 0;
    ovl += (L.status & ST_OVERLAP) ? 1 : 0;
    wacts += L.c_act;
  }
  printf(", \"window_lane\": {\"redo\": %ld, \"tie\": %ld, \"tie_unresolved\": %ld, "
         "\"overlap\": %ld, \"per_activation\": {\"payloads\": %.2f, \"children_visited\": %.2f, "
         "\"ca_steps\": %.2f, \"frontier_inserts\": %.2f, \"share_steps\": %.2f, "
         "\"release_walk\": %.2f}}}\n", redo, ties, unres, ovl, g_cost[eth::CC_PAYLOAD] / (double)wacts,
         g_cost[eth::CC_SCAN] / (double)wacts, g_cost[eth::CC_CA] / (double)wacts,
         g_cost[eth::CC_MDV] / (double)wacts, g_cost[eth::CC_SHARE] / (double)wacts,
         g_cost[eth::CC_SORT] / (double)wacts);
  return 0;
}
