// Keyed random stream v1, device side.
//
// Every draw of the reference (OCaml Random, distributions.ml:17,24,90,93 and
// simulator.ml:123) is re-addressed by semantic coordinates so one GPU lane can produce
// exactly the values the CPU oracle's event-driven simulator consumes, whatever order
// the event queue pops them in:
//   activation j : Philox4x32-10(ctr = (ep_lo, ep_hi, j, 0), key = seed)
//                  w0 -> attacker iff w0 < floor(alpha 2^32); w1 -> defender (w1*d)>>32
//                  w2,w3 -> u53 -> delay = (-1*ev) * cpr_log(u)
//   link (shared at activation count kw, share position off, dest j) :
//                  ctr = (ep, kw, TAG_LINK | off<<12 | j>>1), words 2*(j&1),+1 -> u53
//   message (vertex serial s, dest j; B_k, where a node shares several times per
//   activation window): ctr = (ep, s, TAG_MSG | j>>1), words 2*(j&1),+1 -> u53
// cpr_log = fdlibm e_log.c (IEEE +,-,*,/ only) so device and host agree bit for bit;
// this TU must be compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace cpr {

constexpr uint32_t TAG_ACT = 0u;
constexpr uint32_t TAG_LINK = 0x10000000u;
constexpr uint32_t TAG_POW = 0x20000000u;
constexpr uint32_t TAG_MSG = 0x30000000u;

struct Words4 {
  uint32_t w0, w1, w2, w3;
};

// a ^ b ^ c in one VALU instruction on gfx950 (v_bitop3_b32, truth table 0x96)
__host__ __device__ inline uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

__host__ __device__ inline Words4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2,
                                                uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = xor3((uint32_t)(p1 >> 32), c1, k0);
    const uint32_t n2 = xor3((uint32_t)(p0 >> 32), c3, k1);
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
    // recompute the round keys with SALU adds in every call instead of holding twenty
    // SGPRs across the activation loop (which spills other uniforms to VGPR lanes); only
    // in translation units whose kernels take one seed for the whole grid
    // (CPR_UNIFORM_SEED), since the barrier pins the keys to SGPRs
#if defined(__HIP_DEVICE_COMPILE__) && defined(CPR_UNIFORM_SEED)
    asm volatile("" : "+s"(k0), "+s"(k1));
#endif
  }
  return Words4{c0, c1, c2, c3};
}

// 53-bit uniform in [0, 1)
__host__ __device__ inline double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

__host__ __device__ inline double dbits(uint64_t b) { return __builtin_bit_cast(double, b); }
__host__ __device__ inline uint64_t bitsd(double d) { return __builtin_bit_cast(uint64_t, d); }

// fdlibm __ieee754_log; domain used here: [0, 1)
__host__ __device__ inline double cpr_log(double x) {
  const double ln2_hi = dbits(0x3fe62e42fee00000ull);
  const double ln2_lo = dbits(0x3dea39ef35793c76ull);
  const double two54 = dbits(0x4350000000000000ull);
  const double Lg1 = dbits(0x3FE5555555555593ull), Lg2 = dbits(0x3FD999999997FA04ull);
  const double Lg3 = dbits(0x3FD2492494229359ull), Lg4 = dbits(0x3FCC71C51D8E78AFull);
  const double Lg5 = dbits(0x3FC7466496CB03DEull), Lg6 = dbits(0x3FC39A09D078C69Full);
  const double Lg7 = dbits(0x3FC2F112DF3E5244ull);
#if defined(__HIP_DEVICE_COMPILE__) && !defined(CPR_NO_CONST_BARRIER)
  // materialise the constants at each use instead of keeping ten SGPR pairs live across
  // the activation loop (which spills other uniforms to VGPR lanes)
  double c_[10] = {ln2_hi, ln2_lo, Lg1, Lg2, Lg3, Lg4, Lg5, Lg6, Lg7, two54};
#pragma unroll
  for (int q = 0; q < 10; ++q) asm volatile("" : "+s"(c_[q]));
#define ln2_hi c_[0]
#define ln2_lo c_[1]
#define Lg1 c_[2]
#define Lg2 c_[3]
#define Lg3 c_[4]
#define Lg4 c_[5]
#define Lg5 c_[6]
#define Lg6 c_[7]
#define Lg7 c_[8]
#define two54 c_[9]
#endif
  uint64_t ux = bitsd(x);
  int32_t hx = (int32_t)(ux >> 32);
  const uint32_t lx = (uint32_t)ux;
  int32_t k = 0;
  if (hx < 0x00100000) {
    if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -__builtin_inf();
    if (hx < 0) return __builtin_nan("");
    k -= 54;
    x *= two54;
    ux = bitsd(x);
    hx = (int32_t)(ux >> 32);
  }
  if (hx >= 0x7ff00000) return x + x;
  k += (hx >> 20) - 1023;
  hx &= 0x000fffff;
  int32_t i = (hx + 0x95f64) & 0x100000;
  ux = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (ux & 0xffffffffull);
  x = dbits(ux);
  k += (i >> 20);
  const double f = x - 1.0;
  double dk, R;
  if ((0x000fffff & (2 + hx)) < 3) {  // |f| < 2^-20 (rare)
    if (f == 0.0) {
      if (k == 0) return 0.0;
      dk = (double)k;
      return dk * ln2_hi + dk * ln2_lo;
    }
    R = f * f * (0.5 - 0.33333333333333333 * f);
    if (k == 0) return f - R;
    dk = (double)k;
    return dk * ln2_hi - ((R - dk * ln2_lo) - f);
  }
#if defined(__HIP_DEVICE_COMPILE__)
  // f / (2 + f) as the compiler's own IEEE division expansion minus v_div_scale and
  // v_div_fixup: here f in [sqrt(2)/2 - 1, sqrt(2) - 1) and 2 + f in [1.7, 2.5), so
  // div_scale would return its operands unchanged (vcc = 0, div_fmas = fma) and div_fixup
  // its quotient: the same bits, three instructions fewer
  const double dd2 = 2.0 + f;
  double rr = __builtin_amdgcn_rcp(dd2);
  rr = __builtin_fma(rr, __builtin_fma(-dd2, rr, 1.0), rr);
  rr = __builtin_fma(rr, __builtin_fma(-dd2, rr, 1.0), rr);
  const double qq = f * rr;
  const double s = __builtin_fma(__builtin_fma(-dd2, qq, f), rr, qq);
#else
  const double s = f / (2.0 + f);
#endif
  dk = (double)k;
  const double z = s * s;
  i = hx - 0x6147a;
  const double w = z * z;
  const int32_t j = 0x6b851 - hx;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  i |= j;
  R = t2 + t1;
  // fdlibm's four tails as one select: its k == 0 forms equal the general forms at dk = 0
  // bit for bit (0 * c = +0, y + 0 = y, and fl(y - f) = -fl(f - y) under round to nearest),
  // so lanes of a wave no longer split over four branches (tests/test_oracle_kat.py checks
  // this against the oracle's line-by-line fdlibm)
  const double hfsq = 0.5 * f * f;
  const double lo = dk * ln2_lo;
  const double tail = i > 0 ? hfsq - (s * (hfsq + R) + lo) : s * (f - R) - lo;
  return dk * ln2_hi - (tail - f);
#if defined(__HIP_DEVICE_COMPILE__) && !defined(CPR_NO_CONST_BARRIER)
#undef ln2_hi
#undef ln2_lo
#undef Lg1
#undef Lg2
#undef Lg3
#undef Lg4
#undef Lg5
#undef Lg6
#undef Lg7
#undef two54
#endif
}

struct Stream {
  uint32_t k0, k1;  // seed
  uint32_t e0, e1;  // episode
  __host__ __device__ inline Words4 block(uint32_t idx, uint32_t tag) const {
    return philox4x32_10(e0, e1, idx, tag, k0, k1);
  }
  // uniform for the message shared at activation count kw, position off in that share
  // order, to node dest
  __host__ __device__ inline double link_u(uint32_t kw, uint32_t off, uint32_t dest) const {
    const Words4 w = block(kw, TAG_LINK | (off << 12) | (dest >> 1));
    return (dest & 1u) ? u53(w.w2, w.w3) : u53(w.w0, w.w1);
  }
  __host__ __device__ inline double msg_u(uint32_t serial, uint32_t dest) const {
    const Words4 w = block(serial, TAG_MSG | (dest >> 1));
    return (dest & 1u) ? u53(w.w2, w.w3) : u53(w.w0, w.w1);
  }

  // ---- draws as the lanes consume them (the same interface as TraceStream)
  // miner of activation j among [attacker] + d equal-weight defenders
  __host__ __device__ inline int32_t miner(uint32_t j, uint64_t t_att, int32_t d) const {
    const Words4 w = block(j, TAG_ACT);
    if ((uint64_t)w.w0 < t_att) return 0;
    return 1 + (int32_t)(((uint64_t)w.w1 * (uint64_t)d) >> 32);
  }
  // exponential delay of clock j (distributions.ml:22-29)
  __host__ __device__ inline double clock(uint32_t j, double ev) const {
    const Words4 w = block(j, TAG_ACT);
    return (-1.0 * ev) * cpr_log(u53(w.w2, w.w3));
  }
  // both draws of activation j from one counter block
  __host__ __device__ inline double act(uint32_t j, uint64_t t_att, int32_t d, double ev,
                                        int32_t* miner_out) const {
    const Words4 w = block(j, TAG_ACT);
    *miner_out = (uint64_t)w.w0 < t_att ? 0 : 1 + (int32_t)(((uint64_t)w.w1 * (uint64_t)d) >> 32);
    return (-1.0 * ev) * cpr_log(u53(w.w2, w.w3));
  }
  __host__ __device__ inline int32_t pow(uint32_t serial) const {
    return (int32_t)(block(serial, TAG_POW).w0 & 0x3FFFFFFFu);
  }
  // miner of activation j for arbitrary compute weights (honest cliques): the first node
  // i with w0 < thr[i] (thr: n - 1 cumulative thresholds, see cpr_weight_thresholds)
  __host__ __device__ inline int32_t miner_w(uint32_t j, const uint32_t* thr, int32_t nthr) const {
    const uint32_t w0 = block(j, TAG_ACT).w0;
    int32_t i = 0;
    while (i < nthr && w0 >= thr[i]) ++i;
    return i;
  }
  // U(lo, hi) delay of the message shared at (kw, off) to dest (distributions.ml:16-20)
  __host__ __device__ inline double link_unif(uint32_t kw, uint32_t off, uint32_t dest, double lo,
                                              double hi) const {
    return link_u(kw, off, dest) * (hi - lo) + lo;
  }
  // U(0, dmax) link delays (network.ml:68-76)
  __host__ __device__ inline double link(uint32_t kw, uint32_t off, uint32_t dest,
                                         double dmax) const {
    return link_u(kw, off, dest) * (dmax - 0.0) + 0.0;
  }
  __host__ __device__ inline double msg(uint32_t serial, uint32_t dest, double dmax) const {
    return msg_u(serial, dest) * (dmax - 0.0) + 0.0;
  }
  // U(lo, hi) delay of message `serial` to dest (B_k / Tailstorm on honest cliques)
  __host__ __device__ inline double msg_unif(uint32_t serial, uint32_t dest, double lo,
                                             double hi) const {
    return msg_u(serial, dest) * (hi - lo) + lo;
  }
  // exponential(ev) delay of message `serial` to dest (distributions.ml:22-29; B_k /
  // Tailstorm on exponential-delay cliques)
  __host__ __device__ inline double msg_exp(uint32_t serial, uint32_t dest, double ev) const {
    return (-1.0 * ev) * cpr_log(msg_u(serial, dest));
  }
};

// ---- replay of an exported activation/delay trace (cpr_replay)
//
// The same draws, read from a trace instead of computed: activation j's miner and clock
// delay, the pow hash of vertex serial s, and message delays keyed by the coordinates of
// the keyed stream (trace_link_key / trace_msg_key), sorted ascending per episode. A draw
// the trace does not hold sets `miss` (the record gets CPR_ST_TRACE_MISS) and returns a
// finite placeholder so the lane still terminates.
__host__ __device__ inline uint64_t trace_link_key(uint32_t kw, uint32_t off, uint32_t dest) {
  return ((uint64_t)kw << 32) | ((uint64_t)(off & 0xFFFFFu) << 12) | (uint64_t)(dest & 0xFFFu);
}
__host__ __device__ inline uint64_t trace_msg_key(uint32_t serial, uint32_t dest) {
  return ((uint64_t)serial << 32) | (uint64_t)(dest & 0xFFFu);
}

struct TraceStream {
  const int32_t* act_miner;  // [n_act]
  const double* act_delay;   // [n_act]
  const int32_t* pow_hash;   // [n_pow], by vertex serial
  const uint64_t* key;       // [n_link], ascending
  const double* delay;       // [n_link]
  int32_t n_act, n_pow, n_link;
  mutable uint32_t miss;

  __host__ __device__ inline int32_t miner(uint32_t j, uint64_t, int32_t) const {
    if (j < (uint32_t)n_act) return act_miner[j];
    miss = 1u;
    return 0;
  }
  __host__ __device__ inline double clock(uint32_t j, double) const {
    if (j < (uint32_t)n_act) return act_delay[j];
    miss = 1u;
    return 1.0;
  }
  __host__ __device__ inline double act(uint32_t j, uint64_t, int32_t, double,
                                        int32_t* miner_out) const {
    if (j < (uint32_t)n_act) {
      *miner_out = act_miner[j];
      return act_delay[j];
    }
    miss = 1u;
    *miner_out = 0;
    return 1.0;
  }
  __host__ __device__ inline int32_t miner_w(uint32_t j, const uint32_t*, int32_t) const {
    return miner(j, 0, 0);
  }
  __host__ __device__ inline double link_unif(uint32_t kw, uint32_t off, uint32_t dest, double,
                                              double) const {
    return lookup(trace_link_key(kw, off, dest));
  }
  __host__ __device__ inline int32_t pow(uint32_t serial) const {
    if (serial < (uint32_t)n_pow) return pow_hash[serial];
    miss = 1u;
    return 0;
  }
  __host__ __device__ inline double lookup(uint64_t k) const {
    int32_t lo = 0, hi = n_link;
    while (lo < hi) {
      const int32_t mid = (lo + hi) >> 1;
      if (key[mid] < k)
        lo = mid + 1;
      else
        hi = mid;
    }
    if (lo < n_link && key[lo] == k) return delay[lo];
    miss = 1u;
    return 0.0;
  }
  __host__ __device__ inline double link(uint32_t kw, uint32_t off, uint32_t dest,
                                         double) const {
    return lookup(trace_link_key(kw, off, dest));
  }
  __host__ __device__ inline double msg(uint32_t serial, uint32_t dest, double) const {
    return lookup(trace_msg_key(serial, dest));
  }
  __host__ __device__ inline double msg_unif(uint32_t serial, uint32_t dest, double,
                                             double) const {
    return lookup(trace_msg_key(serial, dest));
  }
  __host__ __device__ inline double msg_exp(uint32_t serial, uint32_t dest, double) const {
    return lookup(trace_msg_key(serial, dest));
  }
};

}  // namespace cpr
