// FETCH_SIZE calibration for the MSM accumulate's access pattern: every lane
// gathers one 64-B affine point (4 x 16-B loads, as load_aff<Fq>) from a 1 GiB table, at a random
// row (k_gather) or at its own row (k_stream, the coalesced case the guide calibrates: FETCH_SIZE
// = 1/2 of the bytes).  Known byte counts: rows * 64 B read, rows * 4 B written per launch.
// Run under rocprofv3 --pmc FETCH_SIZE (and WRITE_SIZE) and compare.  Prints one JSON line each.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr uint32_t LOG_ROWS = 24;  // 2^24 rows x 64 B = 1 GiB table (past the 256 MiB Infinity Cache)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

template <bool RANDOM>
__global__ __launch_bounds__(256) void k_fetch(const uint4* __restrict__ table, uint32_t* __restrict__ out,
                                              uint32_t seed) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint32_t row = RANDOM ? (mix(t ^ seed) & ((1u << LOG_ROWS) - 1)) : t;
  const uint4* p = table + (size_t)row * 4;
  const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
  out[t] = a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
}

template <bool RANDOM>
static int run(const char* name, const uint4* table, uint32_t* out) {
  const uint32_t rows = 1u << LOG_ROWS;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_fetch<RANDOM>, dim3(rows / 256), dim3(256), 0, 0, table, out, 0x9e3779b9u * (r + 1));
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  printf("{\"kernel\": \"%s\", \"launches\": 5, \"read_bytes_per_launch\": %llu, \"write_bytes_per_launch\": %llu, "
         "\"best_ms\": %.4f, \"read_GBps\": %.1f}\n",
         name, (unsigned long long)rows * 64, (unsigned long long)rows * 4, best, rows * 64.0 / (best * 1e-3) / 1e9);
  return 0;
}

int main() {
  uint4* table;
  uint32_t* out;
  CHK(hipMalloc(&table, (size_t(1) << LOG_ROWS) * 64));
  CHK(hipMalloc(&out, (size_t(1) << LOG_ROWS) * 4));
  CHK(hipMemset(table, 0x5a, (size_t(1) << LOG_ROWS) * 64));
  CHK(hipDeviceSynchronize());
  if (run<false>("k_fetch<stream>", table, out)) return 1;
  if (run<true>("k_fetch<gather>", table, out)) return 1;
  CHK(hipFree(table));
  CHK(hipFree(out));
  return 0;
}
