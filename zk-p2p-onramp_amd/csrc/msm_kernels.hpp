// Per-thread bodies of the MSM kernels (__host__ __device__ so that
// tools/hosttest/msm_emu.cpp can replay the exact pipeline on the CPU).
#pragma once
#include "curve.hpp"

namespace zkp {
namespace msmk {

ZDEV uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

ZDEV bool scalar_geq_r(const uint32_t (&s)[9]) {
#pragma unroll
  for (int i = 7; i >= 0; --i) {
    if (s[i] != FrCfg::MOD_W[i]) return s[i] > FrCfg::MOD_W[i];
  }
  return true;
}

ZDEV void scalar_sub_r(uint32_t (&s)[9]) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t d = (uint64_t)s[i] - FrCfg::MOD_W[i] - br;
    s[i] = (uint32_t)d;
    br = (d >> 63) & 1;
  }
}

// load scalar i as 9 words (word 8 = 0), reduced below r
ZDEV void load_scalar(const uint32_t* __restrict__ scalars, uint32_t i, uint32_t (&s)[9]) {
  const uint4* q = reinterpret_cast<const uint4*>(scalars + (size_t)i * 8);
  uint4 a = q[0], b = q[1];
  s[0] = a.x, s[1] = a.y, s[2] = a.z, s[3] = a.w, s[4] = b.x, s[5] = b.y, s[6] = b.z, s[7] = b.w, s[8] = 0u;
  while (scalar_geq_r(s)) scalar_sub_r(s);
}

// signed c-bit digit of window w (windows visited in order, carry threaded through):
// returns |d| (0 for a zero digit); neg = (d < 0)
ZDEV uint32_t digit_mag(const uint32_t (&s)[9], int w, int c, uint32_t& carry, bool& neg) {
  const uint32_t half = 1u << (c - 1), full = 1u << c;
  const int bit = w * c, j = bit >> 5, sh = bit & 31;
  const uint64_t v = (uint64_t)s[j] | ((uint64_t)s[j + 1] << 32);  // sh + c <= 31 + 24 < 64
  const uint32_t raw = ((uint32_t)(v >> sh) & (full - 1)) + carry;
  if (raw > half) {
    carry = 1;
    neg = true;
    return full - raw;  // 0 when raw == 2^c: pure carry
  }
  carry = 0;
  neg = false;
  return raw;
}

// entry of window w of scalar i: bucket key = group*2^(c-1) + |d|-1 with group = w / T,
// base index (t*n + i) | sign with t = w % T (row t of the table holds 2^(c t) P_i)
ZDEV bool digit_entry(const uint32_t (&s)[9], int w, int c, int T, uint32_t n, uint32_t i, uint32_t& carry,
                      uint32_t& key, uint32_t& val) {
  bool neg;
  const uint32_t mag = digit_mag(s, w, c, carry, neg);
  const uint32_t g = (uint32_t)w / (uint32_t)T, t = (uint32_t)w - g * (uint32_t)T;
  key = (g << (c - 1)) + mag - 1;
  val = (t * n + i) | (neg ? 0x80000000u : 0u);
  return mag != 0;
}

// row t of base i from row t-1: 2^dbl * P, dbl = the window width c (affine; infinity stays
// all-zero)
template <class F>
ZDEV void extend_row(uint32_t i, uint32_t* __restrict__ table, uint32_t n, int dbl, int t) {
  if (i >= n) return;
  const Aff<F> p = load_aff<F>(table, (size_t)(t - 1) * n + i);
  Aff<F> a = p;
  if (!aff_is_inf(p)) {
    Xyzz<F> q = xyzz_dbl_aff(p);
    for (int k = 1; k < dbl; ++k) q = xyzz_dbl(q);
    a = xyzz_to_aff(q);
  }
  store_aff(table, (size_t)t * n + i, a);
}

// largest b in [0, nb) with off[b] <= t   (off[0] = 0 <= t < off[nb])
ZDEV uint32_t seg_search(const uint32_t* __restrict__ off, uint32_t nb, uint32_t t) {
  uint32_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= t)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// entries of task t: [s0, s1) of bucket b
ZDEV uint32_t task_len(uint32_t t, const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                       const uint32_t* __restrict__ off, uint32_t nb, uint32_t S) {
  const uint32_t b = seg_search(off, nb, t);
  const uint32_t s0 = start[b] + (t - off[b]) * S;
  return umin(end[b], s0 + S) - s0;
}

// the field the accumulation computes in: G1 with product columns as asm mad chains (consts.hpp
// FqAccCfg: same values and storage, the 4-wave accumulation hides their wait states), G2 as is
template <class F>
struct AccField {
  using type = F;
};
template <>
struct AccField<Fq> {
  using type = Fe<FqAccCfg>;
};

// the field of the merge and reduction kernels (full XYZZ additions, latency-bound chains): the
// accumulation's chained columns and lockstep product pairs (profiles/merge_chain_r03.txt)
template <class F>
struct MergeField {
  using type = typename AccField<F>::type;
};

// thread i runs task perm[i] (tasks ordered by length, longest first: the lanes of a wave run
// equally long chains) or task i (perm == nullptr)
template <class FS>
ZDEV void accumulate(uint32_t i, const uint32_t* __restrict__ points, const uint32_t* __restrict__ vals,
                     const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                     const uint32_t* __restrict__ off, uint32_t nb, uint32_t S, const uint32_t* __restrict__ perm,
                     uint32_t* __restrict__ out) {
  using F = typename AccField<FS>::type;
  if (i >= off[nb]) return;
  const uint32_t t = perm ? perm[i] : i;
  const uint32_t b = seg_search(off, nb, t);
  const uint32_t s0 = start[b] + (t - off[b]) * S;
  const uint32_t s1 = umin(end[b], s0 + S);
  Xyzz<F> acc = xyzz_inf<F>();
  uint32_t j = s0;
  if (s1 - s0 >= 2) {  // the first two entries as an affine + affine addition
    const uint32_t v0 = vals[s0], v1 = vals[s0 + 1];
    acc = xyzz_from_aff_pair(load_aff<F>(points, v0 & 0x7fffffffu), (v0 >> 31) != 0,
                             load_aff<F>(points, v1 & 0x7fffffffu), (v1 >> 31) != 0);
    j = s0 + 2;
  }
  // the next entry's index is loaded one addition ahead: each iteration then waits on one
  // memory latency (its base gather) instead of two dependent ones (index, then base)
  uint32_t vn = j < s1 ? vals[j] : 0u;
  for (; j < s1; ++j) {
    const uint32_t v = vn;
    if (j + 1 < s1) vn = vals[j + 1];
    xyzz_add_aff(acc, load_aff<F>(points, v & 0x7fffffffu), (v >> 31) != 0);
  }
  store_xyzz(out, t, acc);
}

// ---- bucket merge: only "heavy" buckets (more than 2*S2 partials) take merge levels.
// The partials of bucket b live at [off[b], off[b] + c) of a ping-pong pair of buffers:
// after k merge levels applied to it, in buffer k&1 (0 = accumulate output) with
// c = count after k levels.  A level turns c > 2*S2 partials into ceil(c / S2), written
// at the same base off[b] of the other buffer; light buckets are never touched.

// partial count of a bucket with c0 task partials after `levels` merge levels, and the
// number of levels that actually applied to it
ZDEV uint32_t merged_count(uint32_t c0, uint32_t S2, int levels, int& applied) {
  uint32_t c = c0;
  applied = 0;
  for (int l = 0; l < levels && c > 2 * S2; ++l) {
    c = (c + S2 - 1) / S2;
    ++applied;
  }
  return c;
}

// merge tasks of level `lvl` (0-based): cnt[b] = ceil(c/S2) if bucket b is still heavy, else 0
ZDEV void heavy_counts(uint32_t b, const uint32_t* __restrict__ off, uint32_t nb, uint32_t S2, int lvl,
                       uint32_t* __restrict__ cnt) {
  if (b > nb) return;
  if (b == nb) {
    cnt[b] = 0;
    return;
  }
  int applied;
  const uint32_t c = merged_count(off[b + 1] - off[b], S2, lvl, applied);
  cnt[b] = (applied == lvl && c > 2 * S2) ? (c + S2 - 1) / S2 : 0u;
}

// merge task t of level lvl: sums <= S2 consecutive partials of one heavy bucket
template <class FS>
ZDEV void merge_heavy(uint32_t t, const uint32_t* __restrict__ src, const uint32_t* __restrict__ off,
                      const uint32_t* __restrict__ hoff, uint32_t nb, uint32_t S2, int lvl,
                      uint32_t* __restrict__ dst) {
  using F = typename MergeField<FS>::type;
  if (t >= hoff[nb]) return;
  const uint32_t b = seg_search(hoff, nb, t);
  const uint32_t j = t - hoff[b];
  int applied;
  const uint32_t c = merged_count(off[b + 1] - off[b], S2, lvl, applied);
  const uint32_t s0 = off[b] + j * S2;
  const uint32_t s1 = off[b] + umin(c, (j + 1) * S2);
  Xyzz<F> acc = load_xyzz<F>(src, s0);
  for (uint32_t k = s0 + 1; k < s1; ++k) xyzz_add(acc, load_xyzz<F>(src, k));
  store_xyzz(dst, off[b] + j, acc);
}

// one thread per bucket: fold its (<= 2*S2) remaining partials into buckets[b] (infinity if none)
template <class FS>
ZDEV void merge_final(uint32_t b, const uint32_t* __restrict__ part0, const uint32_t* __restrict__ part1,
                      const uint32_t* __restrict__ off, uint32_t nb, uint32_t S2, int levels,
                      uint32_t* __restrict__ buckets) {
  using F = typename MergeField<FS>::type;
  if (b >= nb) return;
  int applied;
  const uint32_t c = merged_count(off[b + 1] - off[b], S2, levels, applied);
  const uint32_t* in = (applied & 1) ? part1 : part0;
  Xyzz<F> acc = xyzz_inf<F>();
  for (uint32_t j = off[b]; j < off[b] + c; ++j) xyzz_add(acc, load_xyzz<F>(in, j));
  store_xyzz(buckets, b, acc);
}

// ---- bucket reduction:  sum_k (k+1) B_k over the 2^(c-1) buckets of a group, as
//   sum_p T_p + M * sum_b 2^b Q_b   with  S_p = sum_j B_(pM+j),  T_p = sum_j (j+1) B_(pM+j)
//   (segments of M buckets) and Q_b = sum of S_p over the p with bit b set.
// Every piece is a plain sum (no doublings inside the tree), so the latency is a few
// short add chains instead of one long running sum; the host applies the 2^b / M weights.

// segment p of group g (one thread): S_p, T_p by running sums over M buckets
template <class FS>
ZDEV void reduce_segments(uint32_t id, const uint32_t* __restrict__ buckets, uint32_t G, uint32_t half, uint32_t M,
                          uint32_t* __restrict__ s_out, uint32_t* __restrict__ t_out) {
  using F = typename MergeField<FS>::type;
  const uint32_t P = half / M;
  if (id >= G * P) return;
  const uint32_t g = id / P, p = id - g * P;
  Xyzz<F> R = xyzz_inf<F>(), T = xyzz_inf<F>();
  for (int j = (int)M - 1; j >= 0; --j) {
    xyzz_add(R, load_xyzz<F>(buckets, (size_t)g * half + (size_t)p * M + (uint32_t)j));
    xyzz_add(T, R);
  }
  store_xyzz(s_out, id, R);
  store_xyzz(t_out, id, T);
}

// elements per first-level output of the subset sums (n1 outputs per sum)
ZDEV uint32_t subset_n1(uint32_t lgP, uint32_t fan) {
  const uint32_t P = 1u << lgP;
  return (P + 2 * fan - 1) / (2 * fan);
}

// first level of the K = lgP + 1 subset sums of group g: sum b < lgP over the P/2 values
// S_p with bit b of p set (fan consecutive per thread), sum lgP over all P values T_p
// (2*fan per thread).  out[(g*K + b)*n1 + j]
template <class FS>
ZDEV void subset_first(uint32_t id, const uint32_t* __restrict__ s_in, const uint32_t* __restrict__ t_in,
                       uint32_t G, uint32_t lgP, uint32_t fan, uint32_t* __restrict__ out) {
  using F = typename MergeField<FS>::type;
  const uint32_t P = 1u << lgP, K = lgP + 1, n1 = subset_n1(lgP, fan);
  if (id >= G * K * n1) return;
  const uint32_t seg = id / n1, j = id - seg * n1, g = seg / K, b = seg - g * K;
  Xyzz<F> acc = xyzz_inf<F>();
  if (b < lgP) {
    const uint32_t lo = (1u << b) - 1;
    for (uint32_t i = j * fan; i < umin((j + 1) * fan, P / 2); ++i) {
      const uint32_t p = ((i >> b) << (b + 1)) | (1u << b) | (i & lo);
      xyzz_add(acc, load_xyzz<F>(s_in, (size_t)g * P + p));
    }
  } else {
    for (uint32_t i = j * 2 * fan; i < umin((j + 1) * 2 * fan, P); ++i)
      xyzz_add(acc, load_xyzz<F>(t_in, (size_t)g * P + i));
  }
  store_xyzz(out, id, acc);
}

// ---- subset sums by workgroup LDS trees: a workgroup of TREE_TPB
// threads sums 2 * TREE_TPB consecutive values of one sum -- two loads and one addition per
// thread, then log2(TREE_TPB) halving levels through LDS -- so the sequential chain of a sum
// over P/2 values is ~1 + 8 additions per launch and ceil(log_512(P/2)) launches, instead of
// fan-in-L chains over ceil(log_L(P/2)) dependent launches (the finish is latency-bound: every
// sequential full addition costs ~5 us on a lightly loaded SIMD).
constexpr int TREE_TPB = 256;
constexpr uint32_t TREE_CHAIN_FAN = 4;  // fan-in of the chain level below the trees (large subset sums)
template <class F>
struct XyzzLimbs;  // 32-bit words of one XYZZ point in the 9-limb compute form
template <>
struct XyzzLimbs<Fq> {
  static constexpr int N = 4 * NL;
};
template <>
struct XyzzLimbs<Fq2> {
  static constexpr int N = 8 * NL;
};
// LDS slot layout: word k of slot s at lds[k * (TREE_TPB / 2) + s] (consecutive slots in
// consecutive banks)
ZDEV void tree_put(uint32_t* lds, int& k, int slot, const Fq& x) {
#pragma unroll
  for (int l = 0; l < NL; ++l) lds[(k + l) * (TREE_TPB / 2) + slot] = x.v[l];
  k += NL;
}
ZDEV void tree_put(uint32_t* lds, int& k, int slot, const Fq2& x) {
  tree_put(lds, k, slot, x.c0);
  tree_put(lds, k, slot, x.c1);
}
ZDEV void tree_get(const uint32_t* lds, int& k, int slot, Fq& x) {
#pragma unroll
  for (int l = 0; l < NL; ++l) x.v[l] = lds[(k + l) * (TREE_TPB / 2) + slot];
  k += NL;
}
ZDEV void tree_get(const uint32_t* lds, int& k, int slot, Fq2& x) {
  tree_get(lds, k, slot, x.c0);
  tree_get(lds, k, slot, x.c1);
}
// the workgroup's sum of every thread's v (valid in thread 0); lds: XyzzLimbs<F>::N * TREE_TPB / 2
// words.  The lazily reduced accumulator x is a valid addition operand as it is (mul operand).
template <class F>
__device__ __forceinline__ Xyzz<F> wg_tree_sum(Xyzz<F> v, uint32_t* lds) {
  const int t = (int)threadIdx.x;
  for (int sh = TREE_TPB / 2; sh >= 1; sh >>= 1) {
    if (t >= sh && t < 2 * sh) {
      int k = 0;
      tree_put(lds, k, t - sh, v.x);
      tree_put(lds, k, t - sh, v.y);
      tree_put(lds, k, t - sh, v.zz);
      tree_put(lds, k, t - sh, v.zzz);
    }
    __syncthreads();
    if (t < sh) {
      Xyzz<F> q;
      int k = 0;
      tree_get(lds, k, t, q.x);
      tree_get(lds, k, t, q.y);
      tree_get(lds, k, t, q.zz);
      tree_get(lds, k, t, q.zzz);
      xyzz_add(v, q);
    }
    __syncthreads();
  }
  return v;
}

// first tree level of the K = lgP + 1 subset sums of group g (seg = g * K + b): chunk `chunk`
// (2 * TREE_TPB values) of sum b -> out[seg * nch + chunk]
template <class F>
__device__ __forceinline__ void subset_tree_first(const uint32_t* __restrict__ s_in, const uint32_t* __restrict__ t_in,
                                                  uint32_t lgP, uint32_t nch, uint32_t seg, uint32_t chunk,
                                                  uint32_t* lds, uint32_t* __restrict__ out) {
  const uint32_t P = 1u << lgP, K = lgP + 1, g = seg / K, b = seg - g * K;
  const uint32_t cnt = b < lgP ? P / 2 : P;
  Xyzz<F> v = xyzz_inf<F>();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t i = chunk * 2 * TREE_TPB + (uint32_t)h * TREE_TPB + threadIdx.x;
    if (i < cnt) {
      if (b < lgP) {
        const uint32_t p = ((i >> b) << (b + 1)) | (1u << b) | (i & ((1u << b) - 1));
        xyzz_add(v, load_xyzz<F>(s_in, (size_t)g * P + p));
      } else {
        xyzz_add(v, load_xyzz<F>(t_in, (size_t)g * P + i));
      }
    }
  }
  v = wg_tree_sum(v, lds);
  if (threadIdx.x == 0) store_xyzz(out, (size_t)seg * nch + chunk, v);
}

// next tree level: segment seg of n_in values -> chunk sums out[seg * n_out + chunk]
template <class F>
__device__ __forceinline__ void subset_tree_next(const uint32_t* __restrict__ in, uint32_t n_in, uint32_t n_out,
                                                 uint32_t seg, uint32_t chunk, uint32_t* lds,
                                                 uint32_t* __restrict__ out) {
  Xyzz<F> v = xyzz_inf<F>();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t i = chunk * 2 * TREE_TPB + (uint32_t)h * TREE_TPB + threadIdx.x;
    if (i < n_in) xyzz_add(v, load_xyzz<F>(in, (size_t)seg * n_in + i));
  }
  v = wg_tree_sum(v, lds);
  if (threadIdx.x == 0) store_xyzz(out, (size_t)seg * n_out + chunk, v);
}

}  // namespace msmk
}  // namespace zkp
