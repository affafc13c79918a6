// Bucket-accumulation variants (round 4): the G1 mixed-addition loop of
// k_accumulate<Fq> (msm_kernels.hpp accumulate) against variants that cut VALU instructions per
// addition, on an H-MSM-shaped workload (2^19 buckets x ~208 entries in tasks of <= 32, random
// gathers from a 2^23 x 13-row table), each variant checked against the baseline's task sums.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../zk-p2p-onramp_amd/csrc -o acc_bench acc_bench.hip
//   ./acc_bench [buckets_log2=19] [entries_per_bucket=208] [reps=5]
// Variants (template flags):
//   PF   the next entry's point gathered one addition ahead (double-buffered raw words)
//   LIMB 1: the table stored as 9 x 29-bit limbs per coordinate (72 B per point, no unpack) with the
//        negated points in a second table (the sign picks the table: no negation on the device);
//        2: packed 64-B points with the negated table (no unpack saving, no negation)
//   WPE  waves per SIMD the register allocation targets (1: unbounded, 4: <= 128 VGPRs)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "msm_kernels.hpp"

using namespace zkp;

#define CHK(x)                                                                        \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);   \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

using FA = Fe<FqAccCfg>;
constexpr int TPB = 256;

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// random affine "points" (field elements < m, not on the curve: the addition's common path does
// not care, and every variant must give the same sums), packed (16 words) and as limbs (18 words,
// plus the negated y in the second table)
__global__ void k_fill(uint32_t* packed, uint32_t* packed_neg, uint32_t* limbs, uint32_t* limbs_neg, size_t n) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  Aff<FA> p;
  for (int c = 0; c < 2; ++c) {
    uint32_t w[8];
    for (int k = 0; k < 8; ++k) w[k] = (uint32_t)mix64(i * 16 + c * 8 + k + 1);
    w[7] &= 0x0fffffffu;  // < 2^252 < m
    FA x = unpack<FqAccCfg>(w);
    (c == 0 ? p.x : p.y) = x;
  }
  store_aff(packed, i, p);
  for (int l = 0; l < NL; ++l) {
    limbs[i * 18 + l] = p.x.v[l];
    limbs[i * 18 + 9 + l] = p.y.v[l];
  }
  const FA ny = sub(fe_zero<FqAccCfg>(), p.y);
  store_aff(packed_neg, i, Aff<FA>{p.x, ny});
  for (int l = 0; l < NL; ++l) {
    limbs_neg[i * 18 + l] = p.x.v[l];
    limbs_neg[i * 18 + 9 + l] = ny.v[l];
  }
}

__global__ void k_vals(uint32_t* vals, size_t n, uint32_t ntab) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const uint64_t r = mix64(i * 7919 + 17);
  vals[i] = (uint32_t)(r % ntab) | ((uint32_t)(r >> 40) & 1u) << 31;
}

template <int LIMB>
__device__ __forceinline__ void load_raw(const uint32_t* __restrict__ tab, const uint32_t* __restrict__ tabn,
                                         uint32_t v, uint32_t (&w)[18]) {
  if (LIMB == 1) {
    const uint32_t* p = ((v >> 31) ? tabn : tab) + (size_t)(v & 0x7fffffffu) * 18;
    const uint2* q = reinterpret_cast<const uint2*>(p);  // 72-B rows: 8-byte aligned
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const uint2 t = q[k];
      w[2 * k] = t.x;
      w[2 * k + 1] = t.y;
    }
  } else {
    const uint4* q = reinterpret_cast<const uint4*>((LIMB == 2 && (v >> 31) ? tabn : tab) + (size_t)(v & 0x7fffffffu) * 16);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 t = q[k];
      w[4 * k] = t.x, w[4 * k + 1] = t.y, w[4 * k + 2] = t.z, w[4 * k + 3] = t.w;
    }
  }
}

template <int LIMB>
__device__ __forceinline__ Aff<FA> to_aff(const uint32_t (&w)[18]) {
  Aff<FA> p;
  if (LIMB == 1) {
#pragma unroll
    for (int l = 0; l < NL; ++l) p.x.v[l] = w[l], p.y.v[l] = w[9 + l];
  } else {
    uint32_t a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = w[k], b[k] = w[8 + k];
    p.x = unpack<FqAccCfg>(a);
    p.y = unpack<FqAccCfg>(b);
  }
  return p;
}

// one task per thread (tasks never straddle a bucket; every bucket of the same length here)
template <bool PF, int LIMB, int WPE>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(WPE))) void k_acc(const uint32_t* __restrict__ tab, const uint32_t* __restrict__ tabn,
                                             const uint32_t* __restrict__ vals, uint32_t ntask, uint32_t S,
                                             uint32_t per_bucket, uint32_t* __restrict__ out) {
  const uint32_t t = blockIdx.x * TPB + threadIdx.x;
  if (t >= ntask) return;
  const uint32_t tpb = (per_bucket + S - 1) / S, b = t / tpb, k = t - b * tpb;
  const uint32_t s0 = b * per_bucket + k * S, s1 = msmk::umin(b * per_bucket + per_bucket, s0 + S);
  Xyzz<FA> acc = xyzz_inf<FA>();
  uint32_t j = s0;
  if (s1 - s0 >= 2) {
    uint32_t w0[18], w1[18];
    const uint32_t v0 = vals[s0], v1 = vals[s0 + 1];
    load_raw<LIMB>(tab, tabn, v0, w0);
    load_raw<LIMB>(tab, tabn, v1, w1);
    acc = xyzz_from_aff_pair(to_aff<LIMB>(w0), (LIMB == 0) && (v0 >> 31), to_aff<LIMB>(w1), (LIMB == 0) && (v1 >> 31));
    j = s0 + 2;
  }
  if (PF) {
    uint32_t w[18] = {};
    uint32_t vn = j < s1 ? vals[j] : 0u;
    bool neg = false;
    if (j < s1) {
      load_raw<LIMB>(tab, tabn, vn, w);
      neg = (vn >> 31) != 0;
      vn = j + 1 < s1 ? vals[j + 1] : 0u;
    }
    for (; j < s1; ++j) {
      const Aff<FA> q = to_aff<LIMB>(w);
      const bool ng = neg;
      if (j + 1 < s1) {  // the next point's gather before this addition's arithmetic
        load_raw<LIMB>(tab, tabn, vn, w);
        neg = (vn >> 31) != 0;
        vn = j + 2 < s1 ? vals[j + 2] : 0u;
      }
      xyzz_add_aff(acc, q, (LIMB == 0) && ng);
    }
  } else {
    uint32_t vn = j < s1 ? vals[j] : 0u;
    for (; j < s1; ++j) {
      const uint32_t v = vn;
      if (j + 1 < s1) vn = vals[j + 1];
      uint32_t w[18];
      load_raw<LIMB>(tab, tabn, v, w);
      xyzz_add_aff(acc, to_aff<LIMB>(w), (LIMB == 0) && (v >> 31));
    }
  }
  store_xyzz(out, t, acc);
}

// the product kernel body itself (msm_kernels.hpp) on the same data, with bucket bounds
__global__ __launch_bounds__(TPB) void k_acc_product(const uint32_t* __restrict__ tab,
                                                     const uint32_t* __restrict__ vals,
                                                     const uint32_t* __restrict__ start,
                                                     const uint32_t* __restrict__ end,
                                                     const uint32_t* __restrict__ off, uint32_t nb, uint32_t S,
                                                     uint32_t* __restrict__ out) {
  msmk::accumulate<Fq>(blockIdx.x * TPB + threadIdx.x, tab, vals, start, end, off, nb, S, nullptr, out);
}

int main(int argc, char** argv) {
  const int lgb = argc > 1 ? atoi(argv[1]) : 19;
  const uint32_t per = argc > 2 ? (uint32_t)atoi(argv[2]) : 208;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const uint32_t S = 32, nb = 1u << lgb;
  const size_t ntab = (size_t)13 << 23;  // the H table: 2^23 points x 13 rows
  const size_t entries = (size_t)nb * per;
  const uint32_t tpb = (per + S - 1) / S, ntask = nb * tpb;
  uint32_t *packed, *packedn, *limbs, *limbsn, *vals, *start, *end, *off, *out[5];
  CHK(hipMalloc(&packed, ntab * 64));
  CHK(hipMalloc(&packedn, ntab * 64));
  CHK(hipMalloc(&limbs, ntab * 72));
  CHK(hipMalloc(&limbsn, ntab * 72));
  CHK(hipMalloc(&vals, entries * 4));
  for (auto& o : out) CHK(hipMalloc(&o, (size_t)ntask * 128));
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((ntab + TPB - 1) / TPB)), dim3(TPB), 0, 0, packed, packedn, limbs, limbsn, ntab);
  hipLaunchKernelGGL(k_vals, dim3((unsigned)((entries + TPB - 1) / TPB)), dim3(TPB), 0, 0, vals, entries, (uint32_t)ntab);
  {
    std::vector<uint32_t> hs(nb + 1), he(nb + 1), ho(nb + 1);
    for (uint32_t b = 0; b < nb; ++b) hs[b] = b * per, he[b] = b * per + per, ho[b] = b * tpb;
    hs[nb] = he[nb] = (uint32_t)entries;
    ho[nb] = ntask;
    CHK(hipMalloc(&start, (nb + 1) * 4));
    CHK(hipMalloc(&end, (nb + 1) * 4));
    CHK(hipMalloc(&off, (nb + 1) * 4));
    CHK(hipMemcpy(start, hs.data(), (nb + 1) * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(end, he.data(), (nb + 1) * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(off, ho.data(), (nb + 1) * 4, hipMemcpyHostToDevice));
  }
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  const dim3 grid((ntask + TPB - 1) / TPB);
  auto run = [&](const char* name, auto launch, int slot) {
    for (int w = 0; w < 2; ++w) launch(slot);
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps; ++r) {
      CHK(hipEventRecord(e0));
      launch(slot);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    const double adds = (double)entries - nb;  // the pair addition of a task counts as one
    printf("{\"variant\": \"%s\", \"ms_best\": %.4f, \"ms_avg\": %.4f, \"ns_per_add\": %.4f, \"frac_mad_peak\": %.4f}\n",
           name, best, sum / reps, best * 1e6 / adds, adds * 1496 / (best * 1e-3) / 37.18e12);
  };
  run("product msmk::accumulate", [&](int s) {
    hipLaunchKernelGGL(k_acc_product, grid, dim3(TPB), 0, 0, packed, vals, start, end, off, nb, S, out[s]);
  }, 0);
#define VAR(name, PFv, LIMBv, WPEv, slot)                                                                  \
  run(name, [&](int s) {                                                                                   \
    hipLaunchKernelGGL((k_acc<PFv, LIMBv, WPEv>), grid, dim3(TPB), 0, 0,                                   \
                       LIMBv == 1 ? limbs : packed, LIMBv == 1 ? limbsn : (LIMBv == 2 ? packedn : packed),    \
                       vals, ntask, S, per, out[s]);                                                       \
  }, slot)
  VAR("baseline (packed, select)", false, 0, 1, 1);
  VAR("NEG (packed, negated table)", false, 2, 1, 2);
  VAR("PF+NEG", true, 2, 1, 3);
  VAR("LIMB (72 B limbs, negated table)", false, 1, 1, 4);
  VAR("baseline, 4 waves", false, 0, 4, 1);
  VAR("NEG, 4 waves", false, 2, 4, 2);
  VAR("PF, 4 waves", true, 0, 4, 3);
  VAR("PF+NEG, 4 waves", true, 2, 4, 4);
  CHK(hipDeviceSynchronize());
  std::vector<uint32_t> ref((size_t)ntask * 32), got(ref.size());
  CHK(hipMemcpy(ref.data(), out[0], ref.size() * 4, hipMemcpyDeviceToHost));
  for (int s = 1; s < 5; ++s) {
    CHK(hipMemcpy(got.data(), out[s], got.size() * 4, hipMemcpyDeviceToHost));
    // every stored coordinate (8 LE words, < 2m) equal mod m: a == b or |a - b| == m
    static const uint32_t M[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                  0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
    auto eqm = [&](const uint32_t* a, const uint32_t* b) {
      bool same = true;
      for (int k = 0; k < 8; ++k) same &= a[k] == b[k];
      if (same) return true;
      for (int dir = 0; dir < 2; ++dir) {  // a - b == m or b - a == m
        const uint32_t* x = dir ? b : a;
        const uint32_t* y = dir ? a : b;
        uint64_t br = 0;
        bool ok = true;
        for (int k = 0; k < 8; ++k) {
          const uint64_t d = (uint64_t)x[k] - y[k] - br;
          ok &= (uint32_t)d == M[k];
          br = (d >> 63) & 1;
        }
        if (ok && !br) return true;
      }
      return false;
    };
    size_t bad = 0;
    for (size_t i = 0; i < ref.size(); i += 8) bad += !eqm(&ref[i], &got[i]);
    printf("{\"check_variant\": %d, \"coordinates_differing_mod_m\": %zu}\n", s, bad);
  }
  return 0;
}
