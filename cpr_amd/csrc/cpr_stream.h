// Keyed random stream v2, device side.
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
// cpr_log = the keyed stream v2 table log (IEEE +, *, fma only) so device and host agree
// bit for bit; this TU must be compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>

#pragma clang fp contract(off)

namespace cpr {

constexpr uint32_t TAG_ACT = 0u;
constexpr uint32_t TAG_LINK = 0x10000000u;
constexpr uint32_t TAG_POW = 0x20000000u;
constexpr uint32_t TAG_MSG = 0x30000000u;
// random attacker actions (cpr_protocols.ml:658-782, Random.int A.Action.n): decision i of
// an episode draws word 0 of block (i, TAG_RAND) (oracle/src/keyed_stream.h rand_action)
constexpr uint32_t TAG_RAND = 0x50000000u;

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

// keyed stream v2 log: x in [0, 1) (the stream's 53-bit uniforms).
// x = 2^e * xr with xr in [sqrt(2)/2, sqrt(2)); bucket i of xr (i = hi << 7 | top 7
// mantissa bits) gives INV_C ~ 1/c_i and T = -log(INV_C) as a double-double
// (tools/gen_logtab.py); log x = e ln2 + T + log1p(r), r = fma(xr, INV_C, -1) (|r| <= 2^-7,
// exact where c_i = 1), log1p as its degree-8 Taylor polynomial. Only IEEE +, *, fma and
// exact bit moves, so the oracle's restatement (oracle/src/keyed_stream.h) is bit-identical;
// at most 1-2 ulp from the true log. Replaces v1's fdlibm e_log.c: a quarter of the f64
// work and no division (tools/nak_probe_ab.sh: the log was 23% of k_run_episodes).
struct LogEnt {
  uint64_t inv_c, t_hi, t_lo;
};
#if defined(__HIP_DEVICE_COMPILE__)
__constant__ static const LogEnt kLogTab[256] = {
#include "cpr_logtab.inc"
};
#else
static const LogEnt kLogTab[256] = {
#include "cpr_logtab.inc"
};
#endif

__host__ __device__ inline double cpr_fma(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_fma(a, b, c);
#else
  return std::fma(a, b, c);
#endif
}

// fma(a, b, c) for a uniform constant c (the log polynomial's coefficients): on the device
// always the three-operand v_fma_f64 with c in SGPRs. Left to itself the compiler picks the
// two-address v_fmac_f64, whose addend is its destination, and copies the loop-invariant
// coefficient into a fresh VGPR pair before each one (a v_mov per term in the activation
// loop). Same IEEE fma, so the host and the oracle agree bit for bit.
#ifndef CPR_FMA_ASM
#define CPR_FMA_ASM 1
#endif
__host__ __device__ inline double cpr_fma_c(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__) && CPR_FMA_ASM
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
  return r;
#else
  return std::fma(a, b, c);
#endif
}

// (an LDS copy of the table measured no faster than constant memory: the 6 KB stay in L1)
__host__ __device__ inline double cpr_log(double x) {
  const double ln2_hi = dbits(0x3fe62e42fee00000ull);  // 32 trailing zeros: e * ln2_hi exact
  const double ln2_lo = dbits(0x3dea39ef35793c76ull);
  const uint64_t ux = bitsd(x);
  const uint64_t mant = ux & 0x000FFFFFFFFFFFFFull;
  const uint32_t hi = mant >= 0x6A09E667F3BCDull ? 1u : 0u;  // xr >= sqrt(2): halve it
  const int32_t e = (int32_t)(ux >> 52) - 1023 + (int32_t)hi;
  const double xr = dbits(((uint64_t)(1023u - hi) << 52) | mant);
  const LogEnt E = kLogTab[(hi << 7) | (uint32_t)(mant >> 45)];
  const double r = cpr_fma(xr, dbits(E.inv_c), -1.0);
  double q = -0.125;
  q = cpr_fma_c(r, q, 1.0 / 7.0);
  q = cpr_fma_c(r, q, -1.0 / 6.0);
  q = cpr_fma_c(r, q, 0.2);
  q = cpr_fma_c(r, q, -0.25);
  q = cpr_fma_c(r, q, 1.0 / 3.0);
  q = cpr_fma_c(r, q, -0.5);
  const double p = cpr_fma(r * r, q, r);
  const double de = (double)e;
  const double a = cpr_fma(de, ln2_hi, dbits(E.t_hi));
  const double b = cpr_fma(de, ln2_lo, dbits(E.t_lo));
  const double y = (a + p) + b;
  return x == 0.0 ? -__builtin_inf() : y;  // x = 0: exponential draw +inf
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
  // activation j's miner and its clock uniform as the 53-bit integer U (u53 = U * 2^-53),
  // without the log: for lanes that read the clock only in rare windows (NakLane LZ)
  __host__ __device__ inline uint64_t act_u(uint32_t j, uint64_t t_att, int32_t d,
                                            int32_t* miner_out) const {
    const Words4 w = block(j, TAG_ACT);
    *miner_out = (uint64_t)w.w0 < t_att ? 0 : 1 + (int32_t)(((uint64_t)w.w1 * (uint64_t)d) >> 32);
    return ((uint64_t)(w.w2 >> 5) << 26) | (uint64_t)(w.w3 >> 6);
  }
  __host__ __device__ inline int32_t pow(uint32_t serial) const {
    return (int32_t)(block(serial, TAG_POW).w0 & 0x3FFFFFFFu);
  }
  // the i-th random attacker action among n (integer multiply-high)
  __host__ __device__ inline int32_t rand_act(uint32_t i, uint32_t n) const {
    return (int32_t)(((uint64_t)block(i, TAG_RAND).w0 * (uint64_t)n) >> 32);
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
  // exponential(ev) delay of the message shared at (kw, off) to dest (distributions.ml:
  // 22-29; Nakamoto / Ethereum on exponential-delay cliques)
  __host__ __device__ inline double link_exp(uint32_t kw, uint32_t off, uint32_t dest,
                                             double ev) const {
    return (-1.0 * ev) * cpr_log(link_u(kw, off, dest));
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
  __host__ __device__ inline double link_exp(uint32_t kw, uint32_t off, uint32_t dest,
                                             double) const {
    return lookup(trace_link_key(kw, off, dest));
  }
  // traces hold no policy draws (a random attacker cannot be replayed from one)
  __host__ __device__ inline int32_t rand_act(uint32_t, uint32_t) const {
    miss = 1u;
    return 0;
  }
};

}  // namespace cpr
