// Study (not product code): how far back the Tailstorm lane's vertex reads reach on BASELINE
// configs[3]'s shape (two-agents network, k = 8, discount rewards, heuristic quorums,
// get-ahead and avoid-loss withholding, alpha .33, 10^4-activation Simulator.loop tasks).
// The lane header is compiled for the host with CPR_TS_AGE histogramming the age (newest
// serial - s) of every read of a vertex record (X), its list view (TR) and a visibility byte
// (Vg). A workgroup LDS window of the newest W records would serve the reads younger than W.
//
// build: hipcc -O2 -std=c++17 -ffp-contract=off -x hip --offload-arch=gfx950 \
//        tools/ts_window_study.cpp -o build/ts_window_study
// usage: build/ts_window_study [episodes] [policy: 1 get-ahead, 3 avoid-loss] [alpha]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

static long g_age[3][14];  // [kind][bucket]: age 0, 1, 2-3, 4-7, ..., >= 4096
static inline void age_hit(int kind, int age) {
  int b = 0;
  while (b < 13 && (age >> b) > 0) ++b;
  ++g_age[kind][b];
}
#define CPR_TS_AGE(kind, age) age_hit((kind), (age))
#include "../cpr_amd/csrc/ts_lane.h"
#include "../oracle/src/keyed_stream.h"

using namespace cpr;

int main(int argc, char** argv) {
  const int episodes = argc > 1 ? atoi(argv[1]) : 20;
  const int policy = argc > 2 ? atoi(argv[2]) : 1;
  const double alpha = argc > 3 ? atof(argv[3]) : 0.33;
  const int steps = 10000, k = 8;
  // as tests/native/ts_vs_oracle.cpp params_of for the two-agents loop (capi.hip validate_ts)
  ts::TsParams P{};
  P.t_att = oracle::alpha_threshold(alpha);
  P.d = 1;
  P.n = 2;
  P.net = 1;
  P.mode = 1;
  P.policy = policy;
  P.scheme = 1;
  P.selection = 1;
  P.k = k;
  const int span = 2 * steps + 2;
  P.cap_v = 64;
  while (P.cap_v < span + 64 && P.cap_v < 4096) P.cap_v <<= 1;
  P.cap_q = P.cap_v / 2;
  P.cap_e = 256 + 512 * P.n;
  P.cap_d = 64;
  P.ev = 1.0;
  P.delta = 1e-9;
  P.dmax = 0.0;
  P.max_steps = steps;
  P.activations = steps;
  P.max_progress = __builtin_inf();
  P.max_time = __builtin_inf();
  P.opt_budget = ts::TS_OPT_BUDGET;
  std::vector<uint8_t> mem(ts::ts_lane_bytes(P));
  long acts = 0, cap = 0;
  for (int e = 0; e < episodes; ++e) {
    const ts::TsMem M = ts::ts_mem_at(mem.data(), P);
    const Stream S{0x5EED0000u, 0u, (uint32_t)e, 0u};
    ts::TsLane L;
    L.loop(P, S, M);
    acts += L.c_act;
    cap += (L.status & ts::TST_CAPACITY) ? 1 : 0;
  }
  const char* kinds[3] = {"vertex", "list", "visibility"};
  printf("{\"episodes\": %d, \"policy\": %d, \"alpha\": %g, \"activations\": %ld, \"capacity\": %ld",
         episodes, policy, alpha, acts, cap);
  for (int kd = 0; kd < 3; ++kd) {
    long tot = 0;
    for (int b = 0; b < 14; ++b) tot += g_age[kd][b];
    printf(", \"%s\": {\"reads_per_activation\": %.2f, \"within\": {", kinds[kd], tot / (double)acts);
    long cum = 0;
    for (int b = 0; b < 14; ++b) {
      cum += g_age[kd][b];
      const int w = 1 << b;  // ages < w
      if (b >= 3 && b <= 12) printf("%s\"%d\": %.4f", b > 3 ? ", " : "", w, cum / (double)tot);
    }
    printf("}}");
  }
  printf("}\n");
  return 0;
}
