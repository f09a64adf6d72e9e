// Probe (round 6, the r5ac/r5ad fault study): what the runtime and the CU do when a
// kernel's static LDS plus the dynamic LDS a launch asks for exceed the CU's 160 KiB.
// k_nak_exact_rerun asks for up to kRerunLdsMax = 160 KiB - 256 of dynamic LDS beside its
// static hybrid ring (128 B). The rejected round-5 "wave-wide hybrid" variant added static
// LDS for 64 staged draws and lane 0's engine result (well over 256 B). This program
// launches one-wave kernels with static LDS of 128 B and of 2 KiB, each with dynamic LDS of
// 160 KiB - 256, writes a pattern over all of it and reads it back. No address anywhere
// derives from LDS contents, so a short LDS allocation shows as mismatches, never as a
// fault. Output: one JSON line per case.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int STATIC_WORDS>
__global__ __launch_bounds__(64) void k_probe(uint32_t* out, int64_t dyn_bytes) {
  extern __shared__ __attribute__((aligned(128))) uint32_t dyn[];
  __shared__ uint32_t st[STATIC_WORDS];
  const int64_t nw = dyn_bytes / 4;
  for (int64_t i = threadIdx.x; i < nw; i += 64) dyn[i] = (uint32_t)i ^ 0x5a5a5a5au;
  for (int i = threadIdx.x; i < STATIC_WORDS; i += 64) st[i] = (uint32_t)i ^ 0xa5a5a5a5u;
  __syncthreads();
  uint32_t bad = 0, first_bad = 0xffffffffu, bad_st = 0;
  for (int64_t i = threadIdx.x; i < nw; i += 64)
    if (dyn[i] != ((uint32_t)i ^ 0x5a5a5a5au)) {
      ++bad;
      if ((uint32_t)i < first_bad) first_bad = (uint32_t)i;
    }
  for (int i = threadIdx.x; i < STATIC_WORDS; i += 64)
    if (st[i] != ((uint32_t)i ^ 0xa5a5a5a5u)) ++bad_st;
  atomicAdd(&out[0], bad);
  atomicMin(&out[1], first_bad);
  atomicAdd(&out[2], bad_st);
}

template <int SW>
static void run_case(uint32_t* d_out, int64_t dyn) {
  uint32_t h[3] = {0u, 0xffffffffu, 0u};
  hipMemcpy(d_out, h, sizeof(h), hipMemcpyHostToDevice);
  hipFuncAttributes fa{};
  hipFuncGetAttributes(&fa, (const void*)k_probe<SW>);
  const hipError_t ea = hipFuncSetAttribute((const void*)k_probe<SW>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)dyn);
  (void)hipGetLastError();
  hipLaunchKernelGGL(k_probe<SW>, dim3(1), dim3(64), (size_t)dyn, 0, d_out, dyn);
  const hipError_t el = hipGetLastError();
  const hipError_t es = hipDeviceSynchronize();
  hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
  printf("{\"static_bytes\": %zu, \"dynamic_bytes\": %lld, \"total\": %lld, "
         "\"set_attribute\": \"%s\", \"launch\": \"%s\", \"sync\": \"%s\", "
         "\"dyn_words_bad\": %u, \"first_bad_word\": %d, \"static_words_bad\": %u}\n",
         fa.sharedSizeBytes, (long long)dyn, (long long)(dyn + (int64_t)fa.sharedSizeBytes),
         hipGetErrorString(ea), hipGetErrorString(el), hipGetErrorString(es), h[0],
         h[1] == 0xffffffffu ? -1 : (int)h[1], h[2]);
  fflush(stdout);
}

int main() {
  int lds_max = 0, lds_blk = 0;
  hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0);
  hipDeviceGetAttribute(&lds_blk, hipDeviceAttributeMaxSharedMemoryPerBlock, 0);
  printf("{\"lds_per_cu\": %d, \"lds_per_block\": %d}\n", lds_max, lds_blk);
  uint32_t* d_out = nullptr;
  if (hipMalloc(&d_out, 16) != hipSuccess) return 1;
  const int64_t dyn = 160 * 1024 - 256;  // kRerunLdsMax
  run_case<32>(d_out, dyn);    // the shipped kernel's static 128 B
  run_case<512>(d_out, dyn);   // 2 KiB static: the variant's order of magnitude
  run_case<512>(d_out, 160 * 1024 - 2048);  // the same, dynamic sized from the static use
  hipFree(d_out);
  return 0;
}
