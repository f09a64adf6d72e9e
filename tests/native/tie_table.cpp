// TEST INFRASTRUCTURE ONLY. The closed-form tie rule of the d = 2 summary-only kernels
// (cpr_amd/csrc/nakamoto_lane.h tie_table_d2) against the lane's own heap replay
// (tie_replay, orderedQueue.ml's insertion / removal rules) over every case the rule
// claims: two defenders, one released block tying the fresh defender block at the non-miner
// defender, both miners, the miner's own copy of the release arriving at t, inside
// (t, t + delta), at t + delta or after, for a grid of clock values and delays.
// Prints one JSON line; exit code 1 on any disagreement.
#include <cstdio>
#include <vector>

#include "../../cpr_amd/csrc/nakamoto_lane.h"

using namespace cpr;

// link draws as the replay and the rule read them: delay dj to the non-miner defender, dm
// to the miner (the rule reads the miner's draw only)
struct MockStream {
  double dj, dm;
  int32_t miner;
  __host__ __device__ double link(uint32_t, uint32_t, uint32_t dest, double) const {
    return (int32_t)dest == miner ? dm : dj;
  }
};

int main() {
  std::vector<uint8_t> mem(REPLAY_BYTES);
  const ReplayMem M = ReplayMem::at(mem.data());
  long cases = 0, bad = 0, on_top = 0;
  for (double t : {0.0, 0.5, 1.0, 3.75, 17.0, 1000.123456789, 2047.9, 65535.5})
    for (double delta : {1e-9, 1e-6, 1e-4, 0.05, 1.0}) {
      NakParams P{};
      P.d = 2;
      P.delta = delta;
      P.dmax = delta;
      for (int32_t miner = 1; miner <= 2; ++miner)
        for (int c = 0; c < 4; ++c) {
          const double dm = c == 0 ? 0.0 : c == 1 ? delta * 0.5 : c == 2 ? delta : delta * 1.5;
          const MockStream S{delta, dm, miner};
          bool ok = false;
          const uint64_t want = tie_replay(P, S, M, miner, t, 1, 1, 7, &ok);
          const uint64_t got = tie_table_d2(P, S, miner, t, 7);
          ++cases;
          if (!ok || want != got) {
            ++bad;
            fprintf(stderr, "t %.17g delta %g miner %d case %d: replay %llx (ok %d) rule %llx\n", t,
                    delta, miner, c, (unsigned long long)want, (int)ok, (unsigned long long)got);
          }
          on_top += want != 0;
        }
    }
  printf("{\"cases\": %ld, \"mismatches\": %ld, \"on_top\": %ld}\n", cases, bad, on_top);
  return bad ? 1 : 0;
}
