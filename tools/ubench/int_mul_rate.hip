// Microbenchmark: gfx950 integer multiply issue rates that bound the BN254
// field arithmetic ("the peak for v_mad_u64_u32 must be
// measured").  Each kernel runs independent dependency chains per lane so the
// measured figure is throughput, not latency.  Prints one JSON line per test.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;
constexpr int CHAINS = 16;

// v_mad_u64_u32: acc = a * b + acc (64-bit accumulate)
__global__ void k_mad_u64(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x * 2654435761u + seed, b = blockIdx.x ^ 0x9e3779b9u;
  uint64_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = a + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint64_t r, cc;
      asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"((uint32_t)(acc[c] >> 32)), "v"(b), "v"(acc[c]));
      acc[c] = r;
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_mul_lo_u32
__global__ void k_mul_lo(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x ^ 0x9e3779b9u;
  uint32_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 2654435761u + seed + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint32_t r;
      asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(r) : "v"(acc[c]), "v"(b));
      acc[c] = r;
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_mul_hi_u32
__global__ void k_mul_hi(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x ^ 0x9e3779b9u;
  uint32_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 2654435761u + seed + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint32_t r;
      asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(r) : "v"(acc[c]), "v"(b));
      acc[c] = r ^ 1;
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_add_co_u32 (carry chain building block)
__global__ void k_add_co(uint64_t* out, uint32_t seed) {
  uint32_t b = blockIdx.x ^ 0x9e3779b9u;
  uint32_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 2654435761u + seed + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint32_t r;
      asm volatile("v_add_co_u32 %0, vcc, %1, %2" : "=v"(r) : "v"(acc[c]), "v"(b) : "vcc");
      acc[c] = r;
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 64-bit shift / shift-add and 32-bit bit ops used around every column of the FIPS multiply
__global__ void k_lshr_b64(uint64_t* out, uint32_t seed) {
  uint64_t acc[CHAINS];
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = ((uint64_t)(threadIdx.x + seed + c) << 33) | 0x12345u;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint64_t r;
      asm volatile("v_lshrrev_b64 %0, 1, %1" : "=v"(r) : "v"(acc[c]));
      acc[c] = r;
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_lshl_add_u64(uint64_t* out, uint32_t seed) {
  uint64_t acc[CHAINS];
  const uint64_t b = 0x9e3779b97f4a7c15ull ^ blockIdx.x;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x + seed + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      uint64_t r;
      asm volatile("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(acc[c]), "v"(b));
      acc[c] = r;
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s ^= acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
#define K32(NAME, ASM)                                                                  \
  __global__ void NAME(uint64_t* out, uint32_t seed) {                                  \
    uint32_t b = blockIdx.x ^ 0x9e3779b9u, acc[CHAINS];                                 \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x * 2654435761u + seed + c; \
    for (int i = 0; i < ITERS; ++i) {                                                   \
      _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) {                              \
        uint32_t r;                                                                     \
        asm volatile(ASM : "=v"(r) : "v"(acc[c]), "v"(b));                              \
        acc[c] = r;                                                                     \
      }                                                                                 \
    }                                                                                   \
    uint64_t s = 0;                                                                     \
    _Pragma("unroll") for (int c = 0; c < CHAINS; ++c) s ^= acc[c];                     \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                     \
  }
K32(k_alignbit, "v_alignbit_b32 %0, %1, %2, 29")
K32(k_add3, "v_add3_u32 %0, %1, %2, %1")
K32(k_and, "v_and_b32 %0, %1, %2")
K32(k_lshr_b32, "v_lshrrev_b32 %0, 29, %1")

// f64 fma for comparison
__global__ void k_fma_f64(uint64_t* out, uint32_t seed) {
  double acc[CHAINS];
  double b = 1.0000001 + blockIdx.x * 1e-9;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) acc[c] = threadIdx.x + seed + c;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      double r;
      asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(acc[c]), "v"(b), "v"(acc[c]));
      acc[c] = r;
    }
  }
  double s = 0;
#pragma unroll
  for (int c = 0; c < CHAINS; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}


// Plain-C 8x32-bit CIOS Montgomery multiply (BN254 Fq), "no final carry"
// variant (p[7] < 2^31): gives the compiler-generated baseline rate.
__device__ __constant__ uint32_t P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                         0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
constexpr uint32_t PINV = 3834012553u;  // -p^-1 mod 2^32
__device__ __forceinline__ void mont_mul(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t A = (uint64_t)a[0] * b[i] + t[0];
    uint32_t m = (uint32_t)A * PINV;
    uint64_t C = (uint64_t)m * P[0] + (uint32_t)A;
#pragma unroll
    for (int j = 1; j < 8; ++j) {
      A = (uint64_t)a[j] * b[i] + t[j] + (A >> 32);
      C = (uint64_t)m * P[j] + (uint32_t)A + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[7] = (uint32_t)((A >> 32) + (C >> 32));
  }
  // conditional subtract
  uint32_t s[8]; uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) { uint64_t d = (uint64_t)t[j] - P[j] - br; s[j] = (uint32_t)d; br = (d >> 63); }
  bool ge = (br == 0);
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = ge ? s[j] : t[j];
}
constexpr int MITERS = 256;
__global__ void k_mont(uint64_t* out, uint32_t seed) {
  uint32_t x[8], y[8], z[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { x[j] = (threadIdx.x * 2654435761u + seed) ^ (j * 0x1234567u); y[j] = blockIdx.x * 77777u + j; z[j] = x[j] ^ 0x55555555u; }
  x[7] &= 0x0fffffffu; y[7] &= 0x0fffffffu; z[7] &= 0x0fffffffu;
  for (int i = 0; i < MITERS; ++i) {
    mont_mul(x, x, y);
    mont_mul(z, z, y);
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) s ^= x[j] ^ z[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
static int run_mont(uint64_t* d, int blocks, int threads) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_mont, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mont, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double ops = (double)blocks * threads * MITERS * 2;
  printf("{\"op\": \"fp_mont_mul_cios_c\", \"blocks\": %d, \"ms\": %.4f, \"G_mul_per_s\": %.2f}\n", blocks, best, ops / (best * 1e-3) / 1e9);
  return 0;
}

// 9 x 29-bit limb FIPS (product-scanning) Montgomery multiply, R = 2^261.
// Column sums never exceed 2^63, so each partial product is ONE v_mad_u64_u32.
__device__ __constant__ uint32_t P29[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                                           0x2db40c0u, 0xa6e141u, 0xe5c2634u, 0x30644eu};
constexpr uint32_t PINV29 = 0x1c3a4e99u & ((1u << 29) - 1);  // placeholder, fixed below at runtime check
__device__ __forceinline__ void mont_mul29(uint32_t* r, const uint32_t* a, const uint32_t* b, uint32_t pinv) {
  constexpr uint32_t MASK = (1u << 29) - 1;
  uint32_t m[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) { acc += (uint64_t)a[j] * b[i - j]; acc += (uint64_t)m[j] * P29[i - j]; }
    acc += (uint64_t)a[i] * b[0];
    m[i] = ((uint32_t)acc * pinv) & MASK;
    acc += (uint64_t)m[i] * P29[0];
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; ++i) {
#pragma unroll
    for (int j = i - 8; j < 9; ++j) { acc += (uint64_t)a[j] * b[i - j]; acc += (uint64_t)m[j] * P29[i - j]; }
    r[i - 9] = (uint32_t)acc & MASK;
    acc >>= 29;
  }
  r[8] = (uint32_t)acc;
}
__global__ void k_mont29(uint64_t* out, uint32_t seed, uint32_t pinv) {
  uint32_t x[9], y[9], z[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) { x[j] = ((threadIdx.x * 2654435761u + seed) ^ (j * 0x1234567u)) & 0x1fffffffu; y[j] = (blockIdx.x * 77777u + j) & 0x1fffffffu; z[j] = x[j] ^ 0x5555555u; }
  x[8] &= 0xffffu; y[8] &= 0xffffu; z[8] &= 0xffffu;
  for (int i = 0; i < MITERS; ++i) {
    mont_mul29(x, x, y, pinv);
    mont_mul29(z, z, y, pinv);
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) s ^= x[j] ^ z[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
static int run_mont29(uint64_t* d, int blocks, int threads) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  uint32_t pinv = 0x12345u;
  hipLaunchKernelGGL(k_mont29, dim3(blocks), dim3(threads), 0, 0, d, 1u, pinv);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mont29, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r, pinv);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double ops = (double)blocks * threads * MITERS * 2;
  printf("{\"op\": \"fp_mont_mul_fips29_c\", \"blocks\": %d, \"ms\": %.4f, \"G_mul_per_s\": %.2f}\n", blocks, best, ops / (best * 1e-3) / 1e9);
  return 0;
}

template <typename K>
static int run(const char* name, K kern, uint64_t* d, int blocks, int threads) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d, (uint32_t)r);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double ops = (double)blocks * threads * ITERS * CHAINS;
  hipDeviceProp_t prop; CHK(hipGetDeviceProperties(&prop, 0));
  double per_cu_clk = ops / (best * 1e-3) / prop.multiProcessorCount / (prop.clockRate * 1e3);
  printf("{\"op\": \"%s\", \"ms\": %.4f, \"Gops_per_s\": %.1f, \"lane_ops_per_CU_per_clk_at_maxclk\": %.2f}\n",
         name, best, ops / (best * 1e-3) / 1e9, per_cu_clk);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  printf("{\"device\": \"%s\", \"gcn\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", prop.name, prop.gcnArchName,
         prop.multiProcessorCount, prop.clockRate);
  int blocks = prop.multiProcessorCount * 8, threads = 256;
  uint64_t* d;
  CHK(hipMalloc(&d, (size_t)blocks * threads * 8));
  if (run("v_mad_u64_u32", k_mad_u64, d, blocks, threads)) return 1;
  if (run("v_mul_lo_u32", k_mul_lo, d, blocks, threads)) return 1;
  if (run("v_mul_hi_u32", k_mul_hi, d, blocks, threads)) return 1;
  if (run("v_add_co_u32", k_add_co, d, blocks, threads)) return 1;
  if (run("v_fma_f64", k_fma_f64, d, blocks, threads)) return 1;
  if (run("v_lshrrev_b64", k_lshr_b64, d, blocks, threads)) return 1;
  if (run("v_lshl_add_u64", k_lshl_add_u64, d, blocks, threads)) return 1;
  if (run("v_alignbit_b32", k_alignbit, d, blocks, threads)) return 1;
  if (run("v_add3_u32", k_add3, d, blocks, threads)) return 1;
  if (run("v_and_b32", k_and, d, blocks, threads)) return 1;
  if (run("v_lshrrev_b32", k_lshr_b32, d, blocks, threads)) return 1;
  for (int bm : {1, 2, 4, 8}) { uint64_t* d2; CHK(hipMalloc(&d2, (size_t)prop.multiProcessorCount * bm * 256 * 8)); if (run_mont(d2, prop.multiProcessorCount * bm, 256)) return 1; CHK(hipFree(d2)); }
  for (int bm : {1, 2, 4, 8}) { uint64_t* d2; CHK(hipMalloc(&d2, (size_t)prop.multiProcessorCount * bm * 256 * 8)); if (run_mont29(d2, prop.multiProcessorCount * bm, 256)) return 1; CHK(hipFree(d2)); }
  // summary line consumed by bench.py (profiles/ubench_r0N.json): best v_mad_u64_u32 rate over occupancies;
  // every (workgroups per CU, run) row is printed so the peak can be traced
  double best = 0;
  int best_bm = 0;
  for (int bm : {4, 8, 16}) {
    uint64_t* d2; CHK(hipMalloc(&d2, (size_t)prop.multiProcessorCount * bm * 256 * 8));
    hipEvent_t e0, e1; CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_mad_u64, dim3(prop.multiProcessorCount * bm), dim3(256), 0, 0, d2, 1u);
    CHK(hipDeviceSynchronize());
    for (int r = 0; r < 5; ++r) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_mad_u64, dim3(prop.multiProcessorCount * bm), dim3(256), 0, 0, d2, (uint32_t)r);
      CHK(hipEventRecord(e1)); CHK(hipEventSynchronize(e1));
      float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
      double tops = (double)prop.multiProcessorCount * bm * 256 * ITERS * CHAINS / (ms * 1e-3) / 1e12;
      printf("{\"sweep\": \"v_mad_u64_u32\", \"workgroups_per_cu\": %d, \"run\": %d, \"ms\": %.4f, \"tops\": %.3f}\n", bm,
             r, ms, tops);
      if (tops > best) best = tops, best_bm = bm;
    }
    CHK(hipFree(d2));
  }
  // full-rate issue ceiling: every SIMD issues one wave64 VALU instruction per 4 clocks at the max clock
  const double ceil_tops = (double)prop.multiProcessorCount * 64 * (prop.clockRate * 1e3) / 1e12;
  printf("{\"summary\": true, \"v_mad_u64_u32_tops\": %.3f, \"best_workgroups_per_cu\": %d, \"chains_per_lane\": %d, "
         "\"issue_ceiling_tops\": %.3f}\n", best, best_bm, CHAINS, ceil_tops);
  CHK(hipFree(d));
  return 0;
}
