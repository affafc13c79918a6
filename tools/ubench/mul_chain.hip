// Field-multiply instruction-shape microbenchmark (round 3): is the FIPS-29 Montgomery multiply
// faster with each product column as ONE dependent v_mad_u64_u32 chain seeded by the previous
// column's carry (inline asm: no per-column join, the hazard wait states become s_nop), than as the
// compiler emits it (each column summed from 0 on its own, the carry joined by v_lshl_add_u64)?
//   hipcc --offload-arch=gfx950 -O3 -o mul_chain mul_chain.hip && ./mul_chain
// Both variants compute the same function; the asm one is checked against the C++ one per lane.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

constexpr uint32_t MASK = (1u << 29) - 1;
// BN254 Fq in 29-bit limbs and -q^-1 mod 2^29 (values only shape the work; correctness of the
// reduction is not what is measured, the two variants are compared with each other)
__constant__ uint32_t P29[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                                0x2db40c0u,  0xa6e141u,  0xe5c2634u,  0x30644eu};
constexpr uint32_t PINV = 0x0a2e7ca9u & MASK;
constexpr int MITERS = 256;

__device__ __forceinline__ void mul_c(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      acc += (uint64_t)a[j] * b[i - j];
      acc += (uint64_t)m[j] * P29[i - j];
    }
    acc += (uint64_t)a[i] * b[0];
    m[i] = ((uint32_t)acc * PINV) & MASK;
    acc += (uint64_t)m[i] * P29[0];
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; ++i) {
#pragma unroll
    for (int j = i - 8; j < 9; ++j) {
      acc += (uint64_t)a[j] * b[i - j];
      acc += (uint64_t)m[j] * P29[i - j];
    }
    r[i - 9] = (uint32_t)acc & MASK;
    acc >>= 29;
  }
  r[8] = (uint32_t)acc;
}

// acc = x * y + acc as one instruction the compiler cannot re-associate
__device__ __forceinline__ void mac(uint64_t& acc, uint32_t x, uint32_t y) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(x), "v"(y));
}
__device__ __forceinline__ void macs(uint64_t& acc, uint32_t x, uint32_t ys) {  // y in an SGPR
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(x), "s"(ys));
}

// the same chain from C: after every product the accumulator passes through an EMPTY asm that
// claims to modify it, so the compiler cannot re-associate the column, but it still sees (and
// schedules, and hazard-checks) real v_mad_u64_u32 instructions
__device__ __forceinline__ void macb(uint64_t& acc, uint32_t x, uint32_t y) {
  acc += (uint64_t)x * y;
  asm("" : "+v"(acc));
}
__device__ __forceinline__ void mul_bar(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      macb(acc, a[j], b[i - j]);
      macb(acc, m[j], P29[i - j]);
    }
    macb(acc, a[i], b[0]);
    m[i] = ((uint32_t)acc * PINV) & MASK;
    macb(acc, m[i], P29[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; ++i) {
#pragma unroll
    for (int j = i - 8; j < 9; ++j) {
      macb(acc, a[j], b[i - j]);
      macb(acc, m[j], P29[i - j]);
    }
    r[i - 9] = (uint32_t)acc & MASK;
    acc >>= 29;
  }
  r[8] = (uint32_t)acc;
}

// the barrier only on the carry at each column start (acc >>= 29): one empty asm per column
__device__ __forceinline__ void mul_cbar(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      acc += (uint64_t)a[j] * b[i - j];
      acc += (uint64_t)m[j] * P29[i - j];
    }
    acc += (uint64_t)a[i] * b[0];
    m[i] = ((uint32_t)acc * PINV) & MASK;
    acc += (uint64_t)m[i] * P29[0];
    acc >>= 29;
    asm("" : "+v"(acc));
  }
#pragma unroll
  for (int i = 9; i < 17; ++i) {
#pragma unroll
    for (int j = i - 8; j < 9; ++j) {
      acc += (uint64_t)a[j] * b[i - j];
      acc += (uint64_t)m[j] * P29[i - j];
    }
    r[i - 9] = (uint32_t)acc & MASK;
    acc >>= 29;
    asm("" : "+v"(acc));
  }
  r[8] = (uint32_t)acc;
}

__device__ __forceinline__ void mul_asm(uint32_t* r, const uint32_t* a, const uint32_t* b) {
  uint32_t m[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      mac(acc, a[j], b[i - j]);
      macs(acc, m[j], P29[i - j]);
    }
    mac(acc, a[i], b[0]);
    m[i] = ((uint32_t)acc * PINV) & MASK;
    macs(acc, m[i], P29[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; ++i) {
#pragma unroll
    for (int j = i - 8; j < 9; ++j) {
      mac(acc, a[j], b[i - j]);
      macs(acc, m[j], P29[i - j]);
    }
    r[i - 9] = (uint32_t)acc & MASK;
    acc >>= 29;
  }
  r[8] = (uint32_t)acc;
}

// two interleaved independent products per call (the NTT's radix-4 unit and the XYZZ addition
// have such pairs): one chain each, the scheduler may interleave them to cover the wait states
__device__ __forceinline__ void mul_asm2(uint32_t* r, const uint32_t* a, const uint32_t* b, uint32_t* r2,
                                         const uint32_t* a2, const uint32_t* b2) {
  uint32_t m[9], n[9];
  uint64_t acc = 0, acc2 = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      mac(acc, a[j], b[i - j]);
      mac(acc2, a2[j], b2[i - j]);
      macs(acc, m[j], P29[i - j]);
      macs(acc2, n[j], P29[i - j]);
    }
    mac(acc, a[i], b[0]);
    mac(acc2, a2[i], b2[0]);
    m[i] = ((uint32_t)acc * PINV) & MASK;
    n[i] = ((uint32_t)acc2 * PINV) & MASK;
    macs(acc, m[i], P29[0]);
    macs(acc2, n[i], P29[0]);
    acc >>= 29;
    acc2 >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; ++i) {
#pragma unroll
    for (int j = i - 8; j < 9; ++j) {
      mac(acc, a[j], b[i - j]);
      mac(acc2, a2[j], b2[i - j]);
      macs(acc, m[j], P29[i - j]);
      macs(acc2, n[j], P29[i - j]);
    }
    r[i - 9] = (uint32_t)acc & MASK;
    r2[i - 9] = (uint32_t)acc2 & MASK;
    acc >>= 29;
    acc2 >>= 29;
  }
  r[8] = (uint32_t)acc;
  r2[8] = (uint32_t)acc2;
}

// three interleaved chains: two other mads between dependent ones, no wait states needed
__device__ __forceinline__ void mul_asm3(uint32_t* r0, const uint32_t* a0, const uint32_t* b, uint32_t* r1,
                                         const uint32_t* a1, uint32_t* r2, const uint32_t* a2) {
  uint32_t m0[9], m1[9], m2[9];
  uint64_t c0 = 0, c1 = 0, c2 = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      mac(c0, a0[j], b[i - j]);
      mac(c1, a1[j], b[i - j]);
      mac(c2, a2[j], b[i - j]);
      macs(c0, m0[j], P29[i - j]);
      macs(c1, m1[j], P29[i - j]);
      macs(c2, m2[j], P29[i - j]);
    }
    mac(c0, a0[i], b[0]);
    mac(c1, a1[i], b[0]);
    mac(c2, a2[i], b[0]);
    m0[i] = ((uint32_t)c0 * PINV) & MASK;
    m1[i] = ((uint32_t)c1 * PINV) & MASK;
    m2[i] = ((uint32_t)c2 * PINV) & MASK;
    macs(c0, m0[i], P29[0]);
    macs(c1, m1[i], P29[0]);
    macs(c2, m2[i], P29[0]);
    c0 >>= 29;
    c1 >>= 29;
    c2 >>= 29;
  }
#pragma unroll
  for (int i = 9; i < 17; ++i) {
#pragma unroll
    for (int j = i - 8; j < 9; ++j) {
      mac(c0, a0[j], b[i - j]);
      mac(c1, a1[j], b[i - j]);
      mac(c2, a2[j], b[i - j]);
      macs(c0, m0[j], P29[i - j]);
      macs(c1, m1[j], P29[i - j]);
      macs(c2, m2[j], P29[i - j]);
    }
    r0[i - 9] = (uint32_t)c0 & MASK;
    r1[i - 9] = (uint32_t)c1 & MASK;
    r2[i - 9] = (uint32_t)c2 & MASK;
    c0 >>= 29;
    c1 >>= 29;
    c2 >>= 29;
  }
  r0[8] = (uint32_t)c0;
  r1[8] = (uint32_t)c1;
  r2[8] = (uint32_t)c2;
}

template <int V>
__global__ void k_mul(uint64_t* out, uint32_t seed) {
  uint32_t x[9], y[9], z[9], w[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    x[j] = ((threadIdx.x * 2654435761u + seed) ^ (j * 0x1234567u)) & MASK;
    y[j] = (blockIdx.x * 77777u + j) & MASK;
    z[j] = x[j] ^ 0x5555555u;
    w[j] = x[j] ^ 0xaaaaaaau;
  }
  x[8] &= 0xffffu;
  y[8] &= 0xffffu;
  z[8] &= 0xffffu;
  w[8] &= 0xffffu;
  for (int i = 0; i < MITERS; ++i) {  // three products per iteration in every variant
    if (V == 0) {
      mul_c(x, x, y);
      mul_c(z, z, y);
      mul_c(w, w, y);
    } else if (V == 1) {
      mul_asm(x, x, y);
      mul_asm(z, z, y);
      mul_asm(w, w, y);
    } else if (V == 2) {
      mul_asm2(x, x, y, z, z, y);
      mul_asm(w, w, y);
    } else if (V == 4) {
      mul_bar(x, x, y);
      mul_bar(z, z, y);
      mul_bar(w, w, y);
    } else if (V == 5) {
      mul_cbar(x, x, y);
      mul_cbar(z, z, y);
      mul_cbar(w, w, y);
    } else {
      mul_asm3(x, x, y, z, z, w, w);
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) s = s * 0x100000001b3ull ^ x[j] ^ ((uint64_t)z[j] << 32) ^ ((uint64_t)w[j] << 16);
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int V>
static int run(const char* name, uint64_t* d, int blocks, int threads, double* best_out) {
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k_mul<V>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_mul<V>, dim3(blocks), dim3(threads), 0, 0, d, 1u);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double g = (double)blocks * threads * MITERS * 3 / (best * 1e-3) / 1e9;
  printf("{\"op\": \"%s\", \"blocks\": %d, \"ms\": %.4f, \"G_mul_per_s\": %.2f}\n", name, blocks, best, g);
  *best_out = g;
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint64_t *d0, *d1;
  const size_t n = (size_t)cus * 16 * 256;
  CHK(hipMalloc(&d0, n * 8));
  CHK(hipMalloc(&d1, n * 8));
  for (int bm : {2, 4, 8, 16}) {
    double g;
    if (run<0>("fips29_c", d0, cus * bm, 256, &g)) return 1;
    if (run<1>("fips29_asm_chain", d1, cus * bm, 256, &g)) return 1;
    uint64_t *h0 = new uint64_t[(size_t)cus * bm * 256], *h1 = new uint64_t[(size_t)cus * bm * 256];
    CHK(hipMemcpy(h0, d0, (size_t)cus * bm * 256 * 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(h1, d1, (size_t)cus * bm * 256 * 8, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < (size_t)cus * bm * 256; ++i) bad += h0[i] != h1[i];
    if (run<2>("fips29_asm_chain_x2", d1, cus * bm, 256, &g)) return 1;
    CHK(hipMemcpy(h1, d1, (size_t)cus * bm * 256 * 8, hipMemcpyDeviceToHost));
    size_t bad2 = 0;
    for (size_t i = 0; i < (size_t)cus * bm * 256; ++i) bad2 += h0[i] != h1[i];
    if (run<3>("fips29_asm_chain_x3", d1, cus * bm, 256, &g)) return 1;
    CHK(hipMemcpy(h1, d1, (size_t)cus * bm * 256 * 8, hipMemcpyDeviceToHost));
    size_t bad3 = 0;
    for (size_t i = 0; i < (size_t)cus * bm * 256; ++i) bad3 += h0[i] != h1[i];
    if (run<4>("fips29_c_barrier_chain", d1, cus * bm, 256, &g)) return 1;
    CHK(hipMemcpy(h1, d1, (size_t)cus * bm * 256 * 8, hipMemcpyDeviceToHost));
    size_t bad4 = 0;
    for (size_t i = 0; i < (size_t)cus * bm * 256; ++i) bad4 += h0[i] != h1[i];
    if (run<5>("fips29_c_carry_barrier", d1, cus * bm, 256, &g)) return 1;
    CHK(hipMemcpy(h1, d1, (size_t)cus * bm * 256 * 8, hipMemcpyDeviceToHost));
    size_t bad5 = 0;
    for (size_t i = 0; i < (size_t)cus * bm * 256; ++i) bad5 += h0[i] != h1[i];
    printf("{\"check\": \"asm == c\", \"blocks\": %d, \"mismatch_chain\": %zu, \"mismatch_x2\": %zu, "
           "\"mismatch_x3\": %zu, \"mismatch_barrier\": %zu, \"mismatch_carry_barrier\": %zu}\n", cus * bm, bad, bad2,
           bad3, bad4, bad5);
    delete[] h0;
    delete[] h1;
  }
  return 0;
}
