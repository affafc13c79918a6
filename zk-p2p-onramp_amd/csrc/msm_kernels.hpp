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

ZDEV void digits(uint32_t i, const uint32_t* __restrict__ scalars, uint32_t n, int c, int W,
                uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  if (i >= n) return;
  const uint4* q = reinterpret_cast<const uint4*>(scalars + (size_t)i * 8);
  uint4 a = q[0], b = q[1];
  uint32_t s[9] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, 0u};
  while (scalar_geq_r(s)) scalar_sub_r(s);  // snarkjs scalars are < r; others reduce (k*P == (k mod r)*P)
  const uint32_t half = 1u << (c - 1), full = 1u << c, invalid = (uint32_t)W * half;
  uint32_t carry = 0;
  for (int w = 0; w < W; ++w) {
    const int bit = w * c, j = bit >> 5, sh = bit & 31;
    const uint64_t v = (uint64_t)s[j] | ((uint64_t)s[j + 1] << 32);
    uint32_t raw = (uint32_t)(v >> sh) & (full - 1);
    raw += carry;
    uint32_t key, val = i;
    if (raw > half) {
      carry = 1;
      const uint32_t mag = full - raw;  // digit = raw - 2^c <= 0 (0 when raw == 2^c: pure carry)
      key = mag == 0 ? invalid : (uint32_t)w * half + mag - 1;
      val |= 0x80000000u;
    } else {
      carry = 0;
      key = raw == 0 ? invalid : (uint32_t)w * half + raw - 1;
    }
    keys[(size_t)w * n + i] = key;
    vals[(size_t)w * n + i] = val;
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
// returns the key window*2^(c-1) + |d|-1, or `invalid` for a zero digit; neg = (d < 0)
ZDEV uint32_t digit_key(const uint32_t (&s)[9], int w, int c, uint32_t& carry, bool& neg, uint32_t invalid) {
  const uint32_t half = 1u << (c - 1), full = 1u << c;
  const int bit = w * c, j = bit >> 5, sh = bit & 31;
  const uint64_t v = (uint64_t)s[j] | ((uint64_t)s[j + 1] << 32);
  const uint32_t raw = ((uint32_t)(v >> sh) & (full - 1)) + carry;
  if (raw > half) {
    carry = 1;
    neg = true;
    const uint32_t mag = full - raw;  // 0 when raw == 2^c: pure carry
    return mag == 0 ? invalid : (uint32_t)w * half + mag - 1;
  }
  carry = 0;
  neg = false;
  return raw == 0 ? invalid : (uint32_t)w * half + raw - 1;
}

ZDEV void bounds(uint32_t i, const uint32_t* __restrict__ keys, uint32_t total, uint32_t* __restrict__ start,
                uint32_t* __restrict__ end) {
  if (i >= total) return;
  const uint32_t k = keys[i];
  if (i == 0 || keys[i - 1] != k) start[k] = i;
  if (i == total - 1 || keys[i + 1] != k) end[k] = i + 1;
}

// cnt[b] = ceil((end[b]-start[b]) / S) for b < nb, cnt[nb] = 0
ZDEV void task_counts(uint32_t b, const uint32_t* __restrict__ start, const uint32_t* __restrict__ end, uint32_t nb,
                     uint32_t S, uint32_t* __restrict__ cnt) {
  if (b > nb) return;
  cnt[b] = b == nb ? 0u : (end[b] - start[b] + S - 1) / S;
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

template <class F>
ZDEV void accumulate(uint32_t t, const uint32_t* __restrict__ points, const uint32_t* __restrict__ vals,
                     const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                     const uint32_t* __restrict__ off, uint32_t nb, uint32_t S, uint32_t* __restrict__ out) {
  if (t >= off[nb]) return;
  const uint32_t b = seg_search(off, nb, t);
  const uint32_t s0 = start[b] + (t - off[b]) * S;
  const uint32_t s1 = umin(end[b], s0 + S);
  Xyzz<F> acc = xyzz_inf<F>();
  for (uint32_t j = s0; j < s1; ++j) {
    const uint32_t v = vals[j];
    Aff<F> p = load_aff<F>(points, v & 0x7fffffffu);
    if (v >> 31) p.y = sub(f_zero<F>(), p.y);
    xyzz_add_aff(acc, p);
  }
  store_xyzz(out, t, acc);
}

// ---- bucket merge: only "heavy" buckets (more than S2 partials) take merge levels.
// The partials of bucket b live at [off[b], off[b] + c) of a ping-pong pair of buffers:
// after k merge levels applied to it, in buffer k&1 (0 = accumulate output) with
// c = count after k levels.  A level turns c > S2 partials into ceil(c / S2), written
// at the same base off[b] of the other buffer; light buckets are never touched.

// partial count of a bucket with c0 task partials after `levels` merge levels, and the
// number of levels that actually applied to it
ZDEV uint32_t merged_count(uint32_t c0, uint32_t S2, int levels, int& applied) {
  uint32_t c = c0;
  applied = 0;
  for (int l = 0; l < levels && c > S2; ++l) {
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
  cnt[b] = (applied == lvl && c > S2) ? (c + S2 - 1) / S2 : 0u;
}

// merge task t of level lvl: sums <= S2 consecutive partials of one heavy bucket
template <class F>
ZDEV void merge_heavy(uint32_t t, const uint32_t* __restrict__ src, const uint32_t* __restrict__ off,
                      const uint32_t* __restrict__ hoff, uint32_t nb, uint32_t S2, int lvl,
                      uint32_t* __restrict__ dst) {
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

// one thread per bucket: fold its (<= S2) remaining partials into buckets[b] (infinity if none)
template <class F>
ZDEV void merge_final(uint32_t b, const uint32_t* __restrict__ part0, const uint32_t* __restrict__ part1,
                      const uint32_t* __restrict__ off, uint32_t nb, uint32_t S2, int levels,
                      uint32_t* __restrict__ buckets) {
  if (b >= nb) return;
  int applied;
  const uint32_t c = merged_count(off[b + 1] - off[b], S2, levels, applied);
  const uint32_t* in = (applied & 1) ? part1 : part0;
  Xyzz<F> acc = xyzz_inf<F>();
  for (uint32_t j = off[b]; j < off[b] + c; ++j) xyzz_add(acc, load_xyzz<F>(in, j));
  store_xyzz(buckets, b, acc);
}

// level 1 of the bucket reduction: node g of window w covers buckets [gL, gL+L):
//   S = sum B_k,  T = sum (j+1) B_(gL+j)
template <class F>
ZDEV void reduce_first(uint32_t id, const uint32_t* __restrict__ buckets, uint32_t nwin, uint32_t half, uint32_t L,
                       uint32_t* __restrict__ s_out, uint32_t* __restrict__ t_out) {
  const uint32_t nodes = (half + L - 1) / L;
  if (id >= nwin * nodes) return;
  const uint32_t w = id / nodes, g = id - w * nodes;
  Xyzz<F> R = xyzz_inf<F>(), T = xyzz_inf<F>();
  for (int j = (int)L - 1; j >= 0; --j) {
    const uint32_t k = g * L + (uint32_t)j;
    if (k < half) xyzz_add(R, load_xyzz<F>(buckets, (size_t)w * half + k));
    xyzz_add(T, R);
  }
  store_xyzz(s_out, id, R);
  store_xyzz(t_out, id, T);
}

// level l>1: node h of window w has children [hL, hL+L) of width 2^lg_width buckets:
//   S' = sum S_j,  T' = sum T_j + 2^lg_width * sum j S_j
template <class F>
ZDEV void reduce_level(uint32_t id, const uint32_t* __restrict__ s_in, const uint32_t* __restrict__ t_in,
                       uint32_t nwin, uint32_t n_in, uint32_t L, int lg_width, uint32_t* __restrict__ s_out,
                       uint32_t* __restrict__ t_out) {
  const uint32_t nodes = (n_in + L - 1) / L;
  if (id >= nwin * nodes) return;
  const uint32_t w = id / nodes, h = id - w * nodes;
  Xyzz<F> R = xyzz_inf<F>(), U = xyzz_inf<F>(), Tsum = xyzz_inf<F>();
  for (int j = (int)L - 1; j >= 1; --j) {
    const uint32_t k = h * L + (uint32_t)j;
    if (k < n_in) {
      xyzz_add(R, load_xyzz<F>(s_in, (size_t)w * n_in + k));
      xyzz_add(Tsum, load_xyzz<F>(t_in, (size_t)w * n_in + k));
    }
    xyzz_add(U, R);
  }
  {
    const uint32_t k = h * L;
    xyzz_add(R, load_xyzz<F>(s_in, (size_t)w * n_in + k));
    xyzz_add(Tsum, load_xyzz<F>(t_in, (size_t)w * n_in + k));
  }
  for (int i = 0; i < lg_width; ++i) U = xyzz_dbl(U);
  xyzz_add(Tsum, U);
  store_xyzz(s_out, id, R);
  store_xyzz(t_out, id, Tsum);
}

}  // namespace msmk
}  // namespace zkp
