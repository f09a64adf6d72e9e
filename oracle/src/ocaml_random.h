// TEST INFRASTRUCTURE ONLY — part of the CPU oracle. Never linked into libcpr_hip.
//
// Replica of the OCaml 4.12.1 standard-library `Random` module, the only source of
// randomness in the reference simulator (pinned OCaml version:
// /root/reference/.github/workflows/main.yml:19-30). The OCaml stdlib is a third-party
// dependency absent from /root/reference; its published algorithm is restated here:
//   * state: 55 30-bit words + index (lagged Fibonacci),
//   * full_init: MD5 chaining over the decimal seed string,
//   * bits / int / float exactly as in stdlib/random.ml of 4.12.
// Pinned by the reference's own recorded outputs: data/withholding.tsv:2-27 (the 28
// two-agents Nakamoto rows reproduce bit-exactly, see tests/test_oracle_kat.py).
// Consumers in the reference: distributions.ml:17,24,90,93 and simulator.ml:123.
#pragma once
#include <cstdint>
#include <cstring>
#include <string>

namespace oracle {

// ---- MD5 (RFC 1321), used only by OCaml's Random.full_init (Digest.string) ----
struct Md5 {
  static void digest(const uint8_t* msg, size_t len, uint8_t out[16]) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
        0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
        0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
        0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
        0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
        0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
        0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
        0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
        0xeb86d391};
    static const int R[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t h0 = 0x67452301, h1 = 0xefcdab89, h2 = 0x98badcfe, h3 = 0x10325476;
    size_t padded = ((len + 8) / 64 + 1) * 64;
    std::string buf(padded, '\0');
    memcpy(&buf[0], msg, len);
    buf[len] = (char)0x80;
    uint64_t bitlen = (uint64_t)len * 8;
    for (int i = 0; i < 8; i++) buf[padded - 8 + i] = (char)((bitlen >> (8 * i)) & 0xff);
    for (size_t off = 0; off < padded; off += 64) {
      uint32_t w[16];
      for (int i = 0; i < 16; i++) {
        const uint8_t* p = (const uint8_t*)&buf[off + 4 * i];
        w[i] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
               ((uint32_t)p[3] << 24);
      }
      uint32_t a = h0, b = h1, c = h2, d = h3;
      for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) % 16; }
        else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) % 16; }
        else { f = c ^ (b | ~d); g = (7 * i) % 16; }
        uint32_t tmp = d;
        d = c;
        c = b;
        uint32_t x = a + f + K[i] + w[g];
        b = b + ((x << R[i]) | (x >> (32 - R[i])));
        a = tmp;
      }
      h0 += a; h1 += b; h2 += c; h3 += d;
    }
    uint32_t hs[4] = {h0, h1, h2, h3};
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)((hs[i] >> (8 * j)) & 0xff);
  }
};

// ---- OCaml 4.12 Random.State ----
struct OcamlRandom {
  int32_t st[55];
  int idx;

  OcamlRandom() { full_init_one(27182818); }  // = Random.State.default (unseeded)
  explicit OcamlRandom(long seed) { full_init_one(seed); }

  // Random.full_init [| seed |]  (stdlib/random.ml, 4.12)
  void full_init_one(long seed) {
    for (int i = 0; i < 55; i++) st[i] = i;
    std::string accu = "x";
    const int l = 1;
    const int n = 54 + (55 > l ? 55 : l);
    for (int i = 0; i <= n; i++) {
      int j = i % 55;
      std::string in = accu + std::to_string(seed);
      uint8_t d[16];
      Md5::digest((const uint8_t*)in.data(), in.size(), d);
      accu.assign((const char*)d, 16);
      int32_t ex = (int32_t)((uint32_t)d[0] | ((uint32_t)d[1] << 8) | ((uint32_t)d[2] << 16) |
                             ((uint32_t)d[3] << 24));
      st[j] = (st[j] ^ ex) & 0x3FFFFFFF;
    }
    idx = 0;
  }

  // Random.bits: 30 random bits
  int32_t bits() {
    idx = (idx + 1) % 55;
    int32_t cur = st[idx];
    int32_t nv = st[(idx + 24) % 55] + (cur ^ ((cur >> 25) & 0x1F));
    nv &= 0x3FFFFFFF;
    st[idx] = nv;
    return nv;
  }

  // Random.int n, 0 < n < 2^30 (rejection sampling, stdlib intaux)
  int int_(int n) {
    for (;;) {
      int32_t r = bits();
      int32_t v = r % n;
      if (r - v > 0x3FFFFFFF - n + 1) continue;
      return v;
    }
  }

  // Random.float b: ((r1 / 2^30 + r2) / 2^30) * b, r1 drawn first
  double float_(double b) {
    const double scale = 1073741824.0;
    double r1 = (double)bits();
    double r2 = (double)bits();
    return ((r1 / scale + r2) / scale) * b;
  }
};

}  // namespace oracle
