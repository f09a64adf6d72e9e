// TEST INFRASTRUCTURE ONLY. The device's cpr_log (cpr_amd/csrc/cpr_stream.h, compiled here
// for the host) against the oracle's line-by-line fdlibm restatement
// (oracle/src/keyed_stream.h), bit for bit: every 53-bit uniform the keyed stream can feed
// it is in [0, 1); sampled uniformly, near 1, near powers of two and tiny values, plus
// the Philox4x32-10 words against the oracle's keyed blocks. Prints one JSON line.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../cpr_amd/csrc/cpr_stream.h"
#include "../../oracle/src/keyed_stream.h"

static uint64_t sm(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 20000000;
  uint64_t st = 12345, bad = 0, checked = 0;
  auto check = [&](double x) {
    const double a = cpr::cpr_log(x), b = oracle::cpr_log(x);
    uint64_t ua, ub;
    memcpy(&ua, &a, 8);
    memcpy(&ub, &b, 8);
    if (ua != ub && !(std::isnan(a) && std::isnan(b))) {
      if (bad < 5) fprintf(stderr, "MISMATCH x=%a device %a oracle %a\n", x, a, b);
      ++bad;
    }
    ++checked;
  };
  for (long i = 0; i < n; ++i) {
    const uint64_t r = sm(st);
    check(cpr::u53((uint32_t)r, (uint32_t)(r >> 32)));
  }
  for (int e = 1; e <= 60; ++e)
    for (int d = -2000; d <= 2000; ++d) {
      check(1.0 - std::ldexp(1.0, -e) + d * std::ldexp(1.0, -53));
      check(std::ldexp(1.0, -e) + d * std::ldexp(1.0, -e - 52));
    }
  for (int e = 1000; e <= 1074; ++e) check(std::ldexp(1.0, -e));
  check(0.0);
  uint64_t pbad = 0;
  for (long i = 0; i < n / 20; ++i) {
    const uint64_t r = sm(st), q = sm(st);
    const cpr::Stream S{(uint32_t)r, (uint32_t)(r >> 32), (uint32_t)q, (uint32_t)(q >> 32)};
    const uint32_t idx = (uint32_t)sm(st), tag = (uint32_t)sm(st);
    const cpr::Words4 w = S.block(idx, tag);
    uint32_t o[4];
    oracle::KeyedStream(r, q).block(idx, tag, o);
    pbad += (w.w0 != o[0]) + (w.w1 != o[1]) + (w.w2 != o[2]) + (w.w3 != o[3]);
  }
  printf("{\"checked\": %lu, \"log_mismatches\": %lu, \"philox_mismatches\": %lu}\n",
         (unsigned long)checked, (unsigned long)bad, (unsigned long)pbad);
  return bad || pbad ? 1 : 0;
}
