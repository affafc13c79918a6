// Batch-affine bucket accumulation measured against the XYZZ accumulate.
//
// Workload: the H MSM's bucket layout -- 2^19 buckets x 208 entries (109 M entries), each entry a
// random row of a 13 x 2^23-row G1 table (7 GB: random 64-B gathers) with a random sign bit.  The
// table holds REAL curve points (2^20 distinct multiples of the generator, repeated over the rows;
// some rows at infinity), and pairs with equal, negated and infinite operands are injected, so every
// exceptional path runs and the bucket sums of the two methods must agree exactly.
//
//   baseline   msmk::accumulate<Fq> (the product kernel) on the 208-entry buckets, 48-entry tasks
//              (5 partials per bucket, as the prover's H plan)
//   affine     k_pairs: level 0 of a pairwise tree -- every two consecutive entries of a bucket added
//              in AFFINE coordinates, lambda = (y1 - y0) / (x1 - x0), the inversions of B additions per
//              lane shared by Montgomery's trick (prefix products in lane-interleaved, coalesced scratch;
//              forward pass over the x's, one Fermat inversion per lane, backward pass), then the same
//              accumulate kernel over the 104 pair sums per bucket in 21-entry tasks (again 5 partials
//              per bucket, so the merges after it are unchanged)
// Both produce per-task XYZZ partials; a check kernel folds each bucket's partials and compares the two
// bucket sums projectively (X1 ZZ2 == X2 ZZ1, Y1 ZZZ2 == Y2 ZZZ1).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../zk-p2p-onramp_amd/csrc -o affine_bench affine_bench.hip
//   ./affine_bench [reps=5] [B list, e.g. 64,128,256,512] [rows the entries draw from]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "msm_kernels.hpp"

using namespace zkp;

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

using FA = Fe<FqAccCfg>;
constexpr int TPB = 256;
constexpr uint32_t IDX = 0x7fffffffu;
constexpr uint32_t NPTS_LOG = 20;           // distinct curve points
constexpr size_t NROWS = (size_t)13 << 23;  // the H table: 2^23 points x 13 rows
constexpr uint32_t INF_ROW = 5;             // rows r with r % 2^22 == 5 are the point at infinity

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// point i = s_i G for a random odd 64-bit s_i (double-and-add in XYZZ, one inversion to affine)
__global__ void k_gen_points(uint32_t* pts, uint32_t n) {
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  Fq one = fe_zero<FqCfg>(), two = fe_zero<FqCfg>();
  one.v[0] = 1;
  two.v[0] = 2;
  const Aff<Fq> g{to_mont(one), to_mont(two)};
  const uint64_t s = mix64(0x9E3779B97F4A7C15ull * (i + 1)) | 1ull;
  Xyzz<Fq> acc = xyzz_inf<Fq>();
  for (int b = 63; b >= 0; --b) {
    acc = xyzz_dbl(acc);
    if ((s >> b) & 1ull) xyzz_add_aff(acc, g);
  }
  Aff<Fq> a = xyzz_to_aff(acc);
  a.x = canon(a.x);
  a.y = canon(a.y);
  store_aff(pts, i, a);
}

__global__ void k_fill_table(const uint32_t* __restrict__ pts, uint32_t* __restrict__ tab, size_t nrows) {
  const size_t r = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (r >= nrows) return;
  const uint4* s = reinterpret_cast<const uint4*>(pts + (r & ((1u << NPTS_LOG) - 1)) * 16);
  uint4* d = reinterpret_cast<uint4*>(tab + r * 16);
  const bool inf = (r & ((1u << 22) - 1)) == INF_ROW;
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = inf ? make_uint4(0, 0, 0, 0) : s[k];
}

// random entries; pairs (2p, 2p+1) get equal (p % 2^16 == 0), negated (== 1) and infinite (== 2)
// operands now and then
__global__ void k_vals(uint32_t* vals, size_t npairs, uint32_t nrows) {
  const size_t p = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (p >= npairs) return;
  const uint64_t r0 = mix64(p * 7919 + 17), r1 = mix64(p * 7919 + 18);
  uint32_t a = (uint32_t)(r0 % nrows) | (((uint32_t)(r0 >> 40) & 1u) << 31);
  uint32_t b = (uint32_t)(r1 % nrows) | (((uint32_t)(r1 >> 40) & 1u) << 31);
  const uint32_t k = (uint32_t)(p & 0xffffu);
  if (k == 0) b = a;
  if (k == 1) b = a ^ 0x80000000u;
  if (k == 2) a = INF_ROW | (a & 0x80000000u);
  if (k == 3) a = b = INF_ROW;
  vals[2 * p] = a;
  vals[2 * p + 1] = b;
}

__global__ void k_iota(uint32_t* v, size_t n) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

// the denominator x1 - x0 of pair (P0, P1) for Montgomery's trick; exceptional pairs (an operand at
// infinity, x0 == x1) take 1 and are flagged
__device__ __forceinline__ FA pair_den(const uint32_t* __restrict__ tab, uint2 v, const FA& x0, const FA& x1,
                                       bool& flag) {
  FA d = sub(x1, x0);
  flag = false;
  if (lo_zero(x0) || lo_zero(x1) || maybe_zero(d)) {
    const Aff<FA> p0 = load_aff<FA>(tab, v.x & IDX), p1 = load_aff<FA>(tab, v.y & IDX);
    flag = aff_is_inf(p0) || aff_is_inf(p1) || is_zero(d);
  }
  if (flag) d = fe_one<FqAccCfg>();
  return d;
}

// level 0 of the affine tree: lane l adds the pairs p = l + k L (k < B, p < np): consecutive lanes take
// consecutive pairs at every step (coalesced entry reads, scratch and output)
template <int WPE>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(WPE))) void k_pairs(
    const uint32_t* __restrict__ tab, const uint32_t* __restrict__ vals, uint32_t np, uint32_t L, uint32_t B,
    uint32_t* __restrict__ scratch, uint32_t* __restrict__ out) {
  const uint32_t l = blockIdx.x * TPB + threadIdx.x;
  if (l >= L) return;
  const uint2* vp = reinterpret_cast<const uint2*>(vals);
  FA acc = fe_one<FqAccCfg>();
  uint32_t kn = 0;
  for (uint32_t k = 0; k < B; ++k) {
    const uint32_t p = l + k * L;
    if (p >= np) break;
    const uint2 v = vp[p];
    const FA x0 = load_fe<FqAccCfg>(tab + (size_t)(v.x & IDX) * 16);
    const FA x1 = load_fe<FqAccCfg>(tab + (size_t)(v.y & IDX) * 16);
    store_fe(scratch + ((size_t)k * L + l) * 8, acc);  // prefix product of the pairs before k
    bool flag;
    acc = mul(acc, pair_den(tab, v, x0, x1, flag));
    kn = k + 1;
  }
  FA I = inv(acc);  // 1 / (product of all kn denominators)
  for (int k = (int)kn - 1; k >= 0; --k) {
    const uint32_t p = l + (uint32_t)k * L;
    const uint2 v = vp[p];
    Aff<FA> p0 = load_aff<FA>(tab, v.x & IDX), p1 = load_aff<FA>(tab, v.y & IDX);
    bool flag;
    const FA d = pair_den(tab, v, p0.x, p1.x, flag);
    const FA pre = load_fe<FqAccCfg>(scratch + ((size_t)k * L + l) * 8);
    FA ik, In;
    mul_2(I, pre, I, d, ik, In);  // 1 / d_k, and 1 / (product of the denominators before k)
    I = In;
    if (v.x >> 31) p0.y = sub(fe_zero<FqAccCfg>(), p0.y);
    if (v.y >> 31) p1.y = sub(fe_zero<FqAccCfg>(), p1.y);
    Aff<FA> r;
    if (!flag) {
      const FA lam = mul(lsub(p1.y, p0.y), ik);
      r.x = sub(sub(sqr(lam), p0.x), p1.x);
      r.y = sub(mul(lam, lsub(p0.x, r.x)), p0.y);
    } else {
      const bool i0 = aff_is_inf(p0), i1 = aff_is_inf(p1);
      if (i0) {
        r = p1;
      } else if (i1) {
        r = p0;
      } else if (is_zero(sub(p1.y, p0.y))) {
        r = xyzz_to_aff(xyzz_dbl_aff(p0));
      } else {
        r.x = fe_zero<FqAccCfg>();
        r.y = fe_zero<FqAccCfg>();
      }
    }
    store_aff(out, p, r);
  }
}

__global__ __launch_bounds__(TPB) void k_acc(const uint32_t* __restrict__ pts, const uint32_t* __restrict__ vals,
                                             const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                                             const uint32_t* __restrict__ off, uint32_t nb, uint32_t S,
                                             uint32_t* __restrict__ out) {
  msmk::accumulate<Fq>(blockIdx.x * TPB + threadIdx.x, pts, vals, start, end, off, nb, S, nullptr, out);
}

// bucket b: fold the partials of both methods and compare projectively; bad[b] = 1 on a mismatch
__global__ void k_check(const uint32_t* __restrict__ pa, uint32_t ta, const uint32_t* __restrict__ pb, uint32_t tb,
                        uint32_t nb, uint32_t* __restrict__ bad) {
  const uint32_t b = blockIdx.x * TPB + threadIdx.x;
  if (b >= nb) return;
  Xyzz<Fq> a = xyzz_inf<Fq>(), c = xyzz_inf<Fq>();
  for (uint32_t t = 0; t < ta; ++t) xyzz_add(a, load_xyzz<Fq>(pa, (size_t)b * ta + t));
  for (uint32_t t = 0; t < tb; ++t) xyzz_add(c, load_xyzz<Fq>(pb, (size_t)b * tb + t));
  bool ok;
  if (xyzz_is_inf(a) || xyzz_is_inf(c)) {
    ok = xyzz_is_inf(a) && xyzz_is_inf(c);
  } else {
    a.x = canon8(a.x);
    c.x = canon8(c.x);
    ok = is_zero(sub(mul(a.x, c.zz), mul(c.x, a.zz))) && is_zero(sub(mul(a.y, c.zzz), mul(c.y, a.zzz)));
  }
  bad[b] = ok ? 0u : 1u;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  // rows the entries draw from (default the whole 13 x 2^23-row table; a small value keeps the gathers in
  // the caches and the TLB: isolates the memory latency of the gathers)
  const uint32_t nrows_used = argc > 3 ? (uint32_t)strtoul(argv[3], nullptr, 0) : (uint32_t)NROWS;
  std::vector<uint32_t> Bs;
  {
    const char* s = argc > 2 ? argv[2] : "64,128,256,512";
    while (*s) {
      Bs.push_back((uint32_t)strtoul(s, (char**)&s, 10));
      if (*s == ',') ++s;
    }
  }
  const uint32_t nb = 1u << 19, per = 208, SA = 48, per2 = per / 2, SB = 21;
  const size_t entries = (size_t)nb * per, np = entries / 2;
  const uint32_t tpa = (per + SA - 1) / SA, tpb2 = (per2 + SB - 1) / SB;
  uint32_t *pts, *tab, *vals, *iota, *scratch, *pairs, *partA, *partB, *bad;
  uint32_t *startA, *endA, *offA, *startB, *endB, *offB;
  CHK(hipMalloc(&pts, ((size_t)1 << NPTS_LOG) * 64));
  CHK(hipMalloc(&tab, NROWS * 64));
  CHK(hipMalloc(&vals, entries * 4));
  CHK(hipMalloc(&iota, np * 4));
  CHK(hipMalloc(&scratch, np * 32));  // B x L >= np prefix products, 32 B each (L = ceil(np / B))
  CHK(hipMalloc(&pairs, np * 64));
  CHK(hipMalloc(&partA, (size_t)nb * tpa * 128));
  CHK(hipMalloc(&partB, (size_t)nb * tpb2 * 128));
  CHK(hipMalloc(&bad, (size_t)nb * 4));
  hipLaunchKernelGGL(k_gen_points, dim3((1u << NPTS_LOG) / TPB), dim3(TPB), 0, 0, pts, 1u << NPTS_LOG);
  hipLaunchKernelGGL(k_fill_table, dim3((unsigned)((NROWS + TPB - 1) / TPB)), dim3(TPB), 0, 0, pts, tab, NROWS);
  hipLaunchKernelGGL(k_vals, dim3((unsigned)((np + TPB - 1) / TPB)), dim3(TPB), 0, 0, vals, np, nrows_used);
  hipLaunchKernelGGL(k_iota, dim3((unsigned)((np + TPB - 1) / TPB)), dim3(TPB), 0, 0, iota, np);
  auto bounds = [&](uint32_t pb, uint32_t S, uint32_t*& st, uint32_t*& en, uint32_t*& of) {
    const uint32_t tp = (pb + S - 1) / S;
    std::vector<uint32_t> hs(nb + 1), he(nb + 1), ho(nb + 1);
    for (uint32_t b = 0; b < nb; ++b) hs[b] = b * pb, he[b] = b * pb + pb, ho[b] = b * tp;
    hs[nb] = he[nb] = nb * pb;
    ho[nb] = nb * tp;
    CHK(hipMalloc(&st, (nb + 1) * 4));
    CHK(hipMalloc(&en, (nb + 1) * 4));
    CHK(hipMalloc(&of, (nb + 1) * 4));
    CHK(hipMemcpy(st, hs.data(), (nb + 1) * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(en, he.data(), (nb + 1) * 4, hipMemcpyHostToDevice));
    CHK(hipMemcpy(of, ho.data(), (nb + 1) * 4, hipMemcpyHostToDevice));
  };
  bounds(per, SA, startA, endA, offA);
  bounds(per2, SB, startB, endB, offB);
  CHK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto timeit = [&](auto launch, float& best, float& avg) {
    launch();
    CHK(hipDeviceSynchronize());
    best = 1e30f;
    float sum = 0;
    for (int r = 0; r < reps; ++r) {
      CHK(hipEventRecord(e0));
      launch();
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      float ms;
      CHK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    avg = sum / reps;
  };
  const double adds = (double)entries - nb;  // additions to reduce every bucket to one sum
  float ab, aa;
  const uint32_t ntA = nb * tpa, ntB = nb * tpb2;
  timeit([&] {
    hipLaunchKernelGGL(k_acc, dim3((ntA + TPB - 1) / TPB), dim3(TPB), 0, 0, tab, vals, startA, endA, offA, nb, SA, partA);
  }, ab, aa);
  printf("{\"variant\": \"baseline XYZZ accumulate, 208 entries per bucket, tasks of %u\", \"ms_best\": %.4f, "
         "\"ms_avg\": %.4f, \"task_adds\": %.0f}\n", SA, ab, aa, (double)entries - ntA);
  for (uint32_t B : Bs) {
    const uint32_t L = (uint32_t)((np + B - 1) / B);
    float pb_, pa_, cb, ca;
    timeit([&] {
      hipLaunchKernelGGL(k_pairs<1>, dim3((L + TPB - 1) / TPB), dim3(TPB), 0, 0, tab, vals, (uint32_t)np, L, B, scratch,
                         pairs);
    }, pb_, pa_);
    timeit([&] {
      hipLaunchKernelGGL(k_acc, dim3((ntB + TPB - 1) / TPB), dim3(TPB), 0, 0, pairs, iota, startB, endB, offB, nb, SB,
                         partB);
    }, cb, ca);
    hipLaunchKernelGGL(k_check, dim3(nb / TPB), dim3(TPB), 0, 0, partA, tpa, partB, tpb2, nb, bad);
    std::vector<uint32_t> hb(nb);
    CHK(hipMemcpy(hb.data(), bad, (size_t)nb * 4, hipMemcpyDeviceToHost));
    size_t nbad = 0;
    for (uint32_t x : hb) nbad += x;
    printf("{\"variant\": \"affine pairs B=%u (%u lanes) + XYZZ accumulate of the 104 pair sums, tasks of %u\", "
           "\"pairs_ms_best\": %.4f, \"pairs_ms_avg\": %.4f, \"acc_ms_best\": %.4f, \"acc_ms_avg\": %.4f, "
           "\"total_ms_best\": %.4f, \"vs_baseline\": %.4f, \"buckets_differing\": %zu, \"buckets\": %u}\n",
           B, L, SB, pb_, pa_, cb, ca, pb_ + cb, (pb_ + cb) / ab, nbad, nb);
  }
  (void)adds;
  return 0;
}
