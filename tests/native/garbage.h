// GARBAGE=<seed> (host fuzzers): a lane's region starts out filled with pseudo-random bytes,
// as the device's pooled memory holds whatever the previous launch left there; an output
// that changes with it reads a byte the lane did not write first
#pragma once
#include <cstdint>
#include <cstdlib>
#include <vector>

inline void fill_garbage(std::vector<uint8_t>& mem) {
  static uint64_t calls = 0;
  const char* g = getenv("GARBAGE");
  if (!g) return;
  uint64_t x = (uint64_t)atoll(g) * 0x9e3779b97f4a7c15ull + ++calls;
  for (auto& v : mem) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    v = (uint8_t)(x >> 56);
  }
}
