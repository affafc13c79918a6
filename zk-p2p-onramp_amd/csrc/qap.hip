// QAP kernels (see qap.hpp).
#include "qap.hpp"

#include "field.hpp"
#include "hip_check.hpp"

namespace zkp {

namespace {

constexpr int TPB = 256;
inline unsigned grid_for(size_t n) { return (unsigned)((n + TPB - 1) / TPB); }

__global__ __launch_bounds__(TPB) void k_convert_fq_zkey(uint32_t* __restrict__ data, size_t n) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  Fq x = load_fe<FqCfg>(data + i * 8);
  // Montgomery(2^256) -> Montgomery(2^261): x * 2^266 / 2^261; infinity (0) stays 0
  x = mul(x, fe_const<FqCfg>(Conv::FQ_ZKEY_TO_DEV));
  store_fe(data + i * 8, x);
}

__global__ __launch_bounds__(TPB) void k_convert_coefs(uint32_t* __restrict__ vals, size_t n) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  Fr x = load_fe<FrCfg>(vals + i * 8);
  x = mul(x, fe_const<FrCfg>(Conv::FR_COEF_TO_DEV));
  store_fe(vals + i * 8, x);
}

__device__ __forceinline__ Fr row_dot(const uint32_t* __restrict__ rowptr, const uint32_t* __restrict__ col,
                                      const uint32_t* __restrict__ val, const uint32_t* __restrict__ w, uint32_t r) {
  Fr acc = fe_zero<FrCfg>();
  const uint32_t e1 = rowptr[r + 1];
  for (uint32_t e = rowptr[r]; e < e1; ++e) {
    // val = coef*2^522, w standard: mont(val, w) = coef*w*2^261 = Montgomery(coef*w)
    acc = add(acc, mul(load_fe<FrCfg>(val + (size_t)e * 8), load_fe<FrCfg>(w + (size_t)col[e] * 8)));
  }
  return acc;
}

__global__ __launch_bounds__(TPB) void k_build_abc(const uint32_t* __restrict__ rpa, const uint32_t* __restrict__ cla,
                                                   const uint32_t* __restrict__ vla, const uint32_t* __restrict__ rpb,
                                                   const uint32_t* __restrict__ clb, const uint32_t* __restrict__ vlb,
                                                   const uint32_t* __restrict__ w, uint32_t n, uint32_t* __restrict__ a,
                                                   uint32_t* __restrict__ b, uint32_t* __restrict__ c) {
  const uint32_t r = blockIdx.x * TPB + threadIdx.x;
  if (r >= n) return;
  Fr av = row_dot(rpa, cla, vla, w, r);
  Fr bv = row_dot(rpb, clb, vlb, w, r);
  store_fe(a + (size_t)r * 8, av);
  store_fe(b + (size_t)r * 8, bv);
  store_fe(c + (size_t)r * 8, mul(av, bv));
}

__global__ __launch_bounds__(TPB) void k_join_abc(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b,
                                                  const uint32_t* __restrict__ c, uint32_t n,
                                                  uint32_t* __restrict__ p) {
  const uint32_t j = blockIdx.x * TPB + threadIdx.x;
  if (j >= n) return;
  // coset evaluations from the NTT are < 3m (Shoup stage products): a - c as a + 4m - c
  Fr x = sub4(mul(load_fe<FrCfg>(a + (size_t)j * 8), load_fe<FrCfg>(b + (size_t)j * 8)),
              load_fe<FrCfg>(c + (size_t)j * 8));
  store_fe(p + (size_t)j * 8, from_mont(x));
}

__global__ __launch_bounds__(TPB) void k_fr_to_dev(uint32_t* __restrict__ d, size_t n) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  store_fe(d + i * 8, to_mont(load_fe<FrCfg>(d + i * 8)));
}

__global__ __launch_bounds__(TPB) void k_fr_from_dev(uint32_t* __restrict__ d, size_t n) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  store_fe(d + i * 8, from_mont(load_fe<FrCfg>(d + i * 8)));
}

__global__ __launch_bounds__(TPB) void k_fq_from_dev(uint32_t* __restrict__ d, size_t n) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  store_fe(d + i * 8, from_mont(load_fe<FqCfg>(d + i * 8)));
}

// one thread per signal: its block's meta, its rank among the block's large / small lanes
// (wtns_pack.hpp wt_decode_one); the 32-B stores are coalesced, the payload reads mostly so
__global__ __launch_bounds__(TPB) void k_witness_unpack(const uint32_t* __restrict__ stage, uint32_t i0, uint32_t n,
                                                        uint32_t* __restrict__ out) {
  const uint32_t i = i0 + blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const uint32_t g = i / WT_BLOCK, lane = i % WT_BLOCK;
  const uint32_t* region = stage + (size_t)(g / WT_CHUNK_BLOCKS) * wt_chunk_words();
  const uint32_t* mb = region + WT_META_PER_BLOCK * (size_t)(g % WT_CHUNK_BLOCKS);
  const uint64_t smallm = (uint64_t)mb[0] | ((uint64_t)mb[1] << 32), bitm = (uint64_t)mb[2] | ((uint64_t)mb[3] << 32),
                 bitv = (uint64_t)mb[4] | ((uint64_t)mb[5] << 32), large = ~(smallm | bitm);
  const uint64_t below = lane ? ~0ull >> (64 - lane) : 0ull;
  const uint32_t* blk = region + WT_META_WORDS + mb[6];
  uint4* o = reinterpret_cast<uint4*>(out + (size_t)i * 8);
  if ((large >> lane) & 1u) {
    const uint4* q = reinterpret_cast<const uint4*>(blk + 8 * __popcll(large & below));  // 16-B aligned
    o[0] = q[0];
    o[1] = q[1];
  } else {
    const uint32_t x = ((bitm >> lane) & 1u) ? (uint32_t)(bitv >> lane) & 1u
                                             : blk[8 * __popcll(large) + __popcll(smallm & below)];
    o[0] = make_uint4(x, 0u, 0u, 0u);
    o[1] = make_uint4(0u, 0u, 0u, 0u);
  }
}

}  // namespace

void launch_witness_unpack(const uint32_t* stage, uint32_t i0, uint32_t i1, uint32_t* out, hipStream_t st) {
  if (i1 <= i0) return;
  hipLaunchKernelGGL(k_witness_unpack, dim3(grid_for(i1 - i0)), dim3(TPB), 0, st, stage, i0, i1, out);
  HIPX(hipGetLastError());
}

void launch_convert_fq_zkey(uint32_t* data, size_t nelems, hipStream_t st) {
  if (!nelems) return;
  hipLaunchKernelGGL(k_convert_fq_zkey, dim3(grid_for(nelems)), dim3(TPB), 0, st, data, nelems);
  HIPX(hipGetLastError());
}

void launch_convert_coefs(uint32_t* vals, size_t n, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_convert_coefs, dim3(grid_for(n)), dim3(TPB), 0, st, vals, n);
  HIPX(hipGetLastError());
}

void launch_build_abc(const uint32_t* rpa, const uint32_t* cla, const uint32_t* vla, const uint32_t* rpb,
                      const uint32_t* clb, const uint32_t* vlb, const uint32_t* w, uint32_t n, uint32_t* a,
                      uint32_t* b, uint32_t* c, hipStream_t st) {
  hipLaunchKernelGGL(k_build_abc, dim3(grid_for(n)), dim3(TPB), 0, st, rpa, cla, vla, rpb, clb, vlb, w, n, a, b, c);
  HIPX(hipGetLastError());
}

void launch_join_abc(const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t n, uint32_t* p,
                     hipStream_t st) {
  hipLaunchKernelGGL(k_join_abc, dim3(grid_for(n)), dim3(TPB), 0, st, a, b, c, n, p);
  HIPX(hipGetLastError());
}

void launch_fr_to_dev(uint32_t* d, size_t n, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_fr_to_dev, dim3(grid_for(n)), dim3(TPB), 0, st, d, n);
  HIPX(hipGetLastError());
}

void launch_fr_from_dev(uint32_t* d, size_t n, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_fr_from_dev, dim3(grid_for(n)), dim3(TPB), 0, st, d, n);
  HIPX(hipGetLastError());
}

void launch_fq_from_dev(uint32_t* d, size_t n, hipStream_t st) {
  if (!n) return;
  hipLaunchKernelGGL(k_fq_from_dev, dim3(grid_for(n)), dim3(TPB), 0, st, d, n);
  HIPX(hipGetLastError());
}

}  // namespace zkp
