// Probe (round 6): issue cost of the instructions the headline kernel's Philox4x32-10 block
// is made of, next to a plain add. Each lane runs 8 independent chains of one operation
// (enough independent work per wave that dependency latency hides behind the other chains
// and the other waves), 8 waves per SIMD over every CU; the result of each chain is stored
// so that nothing is dead. Wave instructions per second per SIMD against one per cycle-pair
// (the 78.64 T lane-op/s VALU peak the bench prices at: 1.229e12 wave instructions/s over
// 1,024 SIMDs) tells which operations issue at full rate and which take several slots.
// Output: one JSON line per operation.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#ifndef CHAINS
#define CHAINS 8
#endif
constexpr int kChains = CHAINS;
constexpr int kIters = 4096;

enum Op { OP_ADD = 0, OP_MULHI = 2, OP_MAD64 = 3, OP_PHILOX_ROUND = 4 };

template <int OP>
__global__ __launch_bounds__(256) void k_rate(uint32_t* out, uint32_t seed) {
  uint32_t x[kChains], y[kChains];
  for (int c = 0; c < kChains; ++c) {
    x[c] = seed ^ (threadIdx.x * 2654435761u) ^ (c * 0x9e3779b9u) ^ blockIdx.x;
    y[c] = x[c] * 0x85ebca6bu + 1u;
  }
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (OP == OP_ADD) {
        x[c] = x[c] + y[c];  // with the xor below: no closed form the compiler could fold
        y[c] = y[c] ^ x[c];
      } else if (OP == OP_MULHI) {
        x[c] = __umulhi(x[c], 0xD2511F53u) + y[c];
      } else if (OP == OP_MAD64) {
        const uint64_t p = (uint64_t)x[c] * 0xCD9E8D57u;
        x[c] = (uint32_t)p ^ (uint32_t)(p >> 32);
      } else {
        // one Philox4x32 round on (x, y) as two words: both products and the key xors
        const uint64_t p = (uint64_t)x[c] * 0xD2511F53u;
        const uint64_t q = (uint64_t)y[c] * 0xCD9E8D57u;
        x[c] = (uint32_t)(q >> 32) ^ (uint32_t)p ^ (uint32_t)i;
        y[c] = (uint32_t)(p >> 32) ^ (uint32_t)q ^ 0x9e3779b9u;
      }
    }
  }
  uint32_t acc = 0;
  for (int c = 0; c < kChains; ++c) acc ^= x[c] ^ y[c];
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
static void run(const char* name, int instr_per_step, uint32_t* out, int blocks) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);  // warm
  (void)hipEventRecord(a, 0);
  hipLaunchKernelGGL(k_rate<OP>, dim3(blocks), dim3(256), 0, 0, out, 2u);
  (void)hipEventRecord(b, 0);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  const double waves = (double)blocks * 4.0;
  const double winstr = waves * kIters * kChains * instr_per_step;
  const double rate = winstr / (ms * 1e-3);
  printf("{\"op\": \"%s\", \"ms\": %.3f, \"wave_instr_per_s\": %.4e, \"frac_of_1.229e12\": %.3f}\n",
         name, ms, rate, rate / 1.229e12);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int blocks = cus * 8;  // 8 waves per SIMD (256-thread blocks: 4 waves, one per SIMD)
  uint32_t* out = nullptr;
  if (hipMalloc(&out, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
  // VALU instructions per chain step as the compiler emits them (the loops' disassembly:
  // add + xor 2; mulhi 2 (v_mul_hi_u32 + v_add); mad64 2 (v_mad_u64_u32 + v_xor); the Philox
  // round 6 (2 v_mad_u64_u32 + 4 v_xor))
  run<OP_ADD>("v_add_u32 + v_xor", 2, out, blocks);
  run<OP_MULHI>("v_mul_hi_u32 + v_add", 2, out, blocks);
  run<OP_MAD64>("v_mad_u64_u32 + v_xor", 2, out, blocks);
  run<OP_PHILOX_ROUND>("philox round: 2 v_mad_u64_u32 + 4 v_xor", 6, out, blocks);
  (void)hipFree(out);
  return 0;
}
