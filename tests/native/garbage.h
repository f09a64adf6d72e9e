// GARBAGE=<seed> (host fuzzers): a lane's region starts out filled with pseudo-random bytes,
// as the device's pooled memory holds whatever the previous launch left there; an output
// that changes with it reads a byte the lane did not write first
#pragma once
#include <cstdint>
#include <cstddef>
#include <cstdlib>
#include <vector>

inline void fill_garbage(void* p, size_t bytes) {
  static uint64_t calls = 0;
  const char* g = getenv("GARBAGE");
  if (!g) return;
  uint64_t x = (uint64_t)atoll(g) * 0x9e3779b97f4a7c15ull + ++calls;
  uint8_t* b = (uint8_t*)p;
  for (size_t i = 0; i < bytes; ++i) {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    b[i] = (uint8_t)(x >> 56);
  }
}
inline void fill_garbage(std::vector<uint8_t>& mem) { fill_garbage(mem.data(), mem.size()); }
