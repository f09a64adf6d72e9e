// TEST INFRASTRUCTURE ONLY — CPU oracle side of the "cpr keyed stream v2".
//
// The reference draws every random number from one sequential OCaml `Random` stream
// (distributions.ml:17,24,90,93; simulator.ml:123), which makes results depend on the
// order in which a discrete-event queue happens to pop same-time events. A batched GPU
// engine cannot reproduce that order cheaply, so the build defines a *keyed* stream in
// which every draw is addressed by its semantic coordinates instead of its position:
//
//   key   = (seed_lo, seed_hi)                          Philox4x32-10 (Salmon et al. 2011)
//   act   : ctr = (ep_lo, ep_hi, j, TAG_ACT)   w0,w1 -> miner of activation j
//                                              w2,w3 -> 53-bit u, delay of clock j
//   link  : ctr = (ep_lo, ep_hi, kw, TAG_LINK | off<<12 | dest>>1)  words (2*(dest&1), +1) -> u
//           kw  = activations simulated when the message was shared (c_activations),
//           off = position of the message in that action's recursive share order
//   pow   : ctr = (ep_lo, ep_hi, serial, TAG_POW)  w0 & 0x3FFFFFFF
//   msg   : ctr = (ep_lo, ep_hi, serial, TAG_MSG | dest>>1)  words (2*(dest&1), +1) -> u
//           link delay of message `serial` to `dest`, used where one node shares several
//           times per activation window (B_k: votes, proposals); a node shares a given
//           vertex at most once (simulator.ml:404-415), so (serial, dest) is unique
//
// exponential(ev) = (-1 * ev) * cpr_log(u)   (same expression shape as distributions.ml:24)
// uniform(lo,hi)  = u * (hi - lo) + lo       (distributions.ml:17)
// miner           = 0 if w0 < floor(alpha * 2^32) else 1 + ((w1 * d) >> 32)
//
// cpr_log is the v2 table-driven log (only IEEE +, *, fma and bit moves; v1 used fdlibm's
// e_log.c), so the GPU and the CPU oracle compute bit-identical event times. This file is an independent restatement of
// the same specification the HIP code implements (cpr_amd/csrc/cpr_stream.h); the two
// are cross-checked draw-by-draw in tests/test_gpu_parity.py.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace oracle {

static const uint32_t TAG_ACT = 0u;
static const uint32_t TAG_LINK = 0x10000000u;
static const uint32_t TAG_POW = 0x20000000u;
static const uint32_t TAG_MSG = 0x30000000u;
// random attacker actions (cpr_protocols.ml:658-782 `Random.int A.Action.n`): the i-th
// policy decision of an episode draws word 0 of block (i, TAG_RAND)
static const uint32_t TAG_RAND = 0x50000000u;

struct Philox4x32 {
  static void block(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; r++) {
      uint64_t p0 = (uint64_t)0xD2511F53u * c0;
      uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
      uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
      uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
      uint32_t n0 = hi1 ^ c1 ^ k0;
      uint32_t n1 = lo1;
      uint32_t n2 = hi0 ^ c3 ^ k1;
      uint32_t n3 = lo0;
      c0 = n0; c1 = n1; c2 = n2; c3 = n3;
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
  }
};

static inline double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

static inline double bits_to_double(uint64_t b) {
  double d;
  memcpy(&d, &b, 8);
  return d;
}
static inline uint64_t double_to_bits(double d) {
  uint64_t b;
  memcpy(&b, &d, 8);
  return b;
}

// keyed stream v2 log, restated: x in [0, 1) is 2^e * xr, xr in [sqrt(2)/2, sqrt(2));
// bucket i = (xr < 1) << 7 | top 7 mantissa bits of x selects INV_C ~ 1/c_i and
// T = -log(INV_C) = T_HI + T_LO (keyed_logtab.inc, from tools/gen_logtab.py);
// log x = e ln2 + T + log1p(r), r = fma(xr, INV_C, -1), log1p by its Taylor polynomial
// through r^8, summed as ((e ln2_hi + T_HI) + p) + (e ln2_lo + T_LO).
struct KeyedLogEntry {
  uint64_t inv_c, t_hi, t_lo;
};
static const KeyedLogEntry kKeyedLog[256] = {
#include "keyed_logtab.inc"
};

static inline double cpr_log(double x) {
  if (x == 0.0) return -1.0 / 0.0;
  const double ln2_hi = bits_to_double(0x3fe62e42fee00000ull);
  const double ln2_lo = bits_to_double(0x3dea39ef35793c76ull);
  const uint64_t ux = double_to_bits(x);
  const uint64_t mant = ux & 0x000FFFFFFFFFFFFFull;
  const uint32_t hi = mant >= 0x6A09E667F3BCDull ? 1u : 0u;
  const int32_t e = (int32_t)(ux >> 52) - 1023 + (int32_t)hi;
  const double xr = bits_to_double(((uint64_t)(1023u - hi) << 52) | mant);
  const KeyedLogEntry& E = kKeyedLog[(hi << 7) | (uint32_t)(mant >> 45)];
  const double r = std::fma(xr, bits_to_double(E.inv_c), -1.0);
  const double c[7] = {-0.125, 1.0 / 7.0, -1.0 / 6.0, 0.2, -0.25, 1.0 / 3.0, -0.5};
  double q = c[0];
  for (int k = 1; k < 7; ++k) q = std::fma(r, q, c[k]);
  const double p = std::fma(r * r, q, r);
  const double de = (double)e;
  const double a = std::fma(de, ln2_hi, bits_to_double(E.t_hi));
  const double b = std::fma(de, ln2_lo, bits_to_double(E.t_lo));
  return (a + p) + b;
}

// cumulative compute thresholds of the keyed miner draw for arbitrary weights:
// thr[i] = floor(sum_{j<=i} w_j / sum w * 2^32), i < n - 1 (fp64, clamped like the
// attacker threshold); the device computes the same table on the host (capi.hip)
inline std::vector<uint32_t> weight_thresholds(const std::vector<double>& w) {
  double total = 0.0;
  for (double x : w) total += x;
  std::vector<uint32_t> thr;
  double cum = 0.0;
  for (size_t i = 0; i + 1 < w.size(); ++i) {
    cum += w[i];
    const double t = cum / total * 4294967296.0;
    thr.push_back(t <= 0.0 ? 0u : (t >= 4294967295.0 ? 4294967295u : (uint32_t)t));
  }
  return thr;
}

struct KeyedStream {
  uint32_t key[2];
  uint32_t ep[2];
  KeyedStream(uint64_t seed, uint64_t episode) {
    key[0] = (uint32_t)seed;
    key[1] = (uint32_t)(seed >> 32);
    ep[0] = (uint32_t)episode;
    ep[1] = (uint32_t)(episode >> 32);
  }
  void block(uint32_t idx, uint32_t tag, uint32_t out[4]) const {
    uint32_t ctr[4] = {ep[0], ep[1], idx, tag};
    Philox4x32::block(ctr, key, out);
  }
  // the i-th random attacker action among n (an integer multiply-high, no float)
  int rand_action(uint32_t i, int n) const {
    uint32_t w[4];
    block(i, TAG_RAND, w);
    return (int)(((uint64_t)w[0] * (uint64_t)n) >> 32);
  }
  // miner of activation j among [attacker] + d equal-weight defenders
  int miner(uint32_t j, uint64_t t_att, int d) const {
    uint32_t w[4];
    block(j, TAG_ACT, w);
    if ((uint64_t)w[0] < t_att) return 0;
    return 1 + (int)(((uint64_t)w[1] * (uint64_t)d) >> 32);
  }
  // miner of activation j for arbitrary compute weights (honest cliques): the first node i
  // with w0 < thr[i], thr = weight_thresholds(...) (n - 1 entries; the last node otherwise)
  int miner_w(uint32_t j, const std::vector<uint32_t>& thr) const {
    uint32_t w[4];
    block(j, TAG_ACT, w);
    int i = 0;
    while (i < (int)thr.size() && w[0] >= thr[i]) ++i;
    return i;
  }
  double act_u(uint32_t j) const {
    uint32_t w[4];
    block(j, TAG_ACT, w);
    return u53(w[2], w[3]);
  }
  double link_u(uint32_t kw, uint32_t off, uint32_t dest) const {
    uint32_t w[4];
    block(kw, TAG_LINK | (off << 12) | (dest >> 1), w);
    return (dest & 1) ? u53(w[2], w[3]) : u53(w[0], w[1]);
  }
  double msg_u(uint32_t serial, uint32_t dest) const {
    uint32_t w[4];
    block(serial, TAG_MSG | (dest >> 1), w);
    return (dest & 1) ? u53(w[2], w[3]) : u53(w[0], w[1]);
  }
  uint32_t pow_bits(uint32_t serial) const {
    uint32_t w[4];
    block(serial, TAG_POW, w);
    return w[0] & 0x3FFFFFFFu;
  }
};

static inline uint64_t alpha_threshold(double alpha) {
  // floor(alpha * 2^32), alpha in [0, 1]
  double t = alpha * 4294967296.0;
  if (t <= 0.0) return 0;
  if (t >= 4294967296.0) return 4294967296ull;
  return (uint64_t)t;
}

}  // namespace oracle
