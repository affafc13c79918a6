// BN254 prime-field arithmetic for gfx950 (CDNA4) — device side.
//
// Representation (DESIGN.md "Field arithmetic"):
//   * compute form: 9 limbs x 29 bits in uint32_t, Montgomery radix R' = 2^261,
//     values kept REDUNDANT in [0, 2m) — never a final subtraction inside mul.
//   * storage form (HBM): 8 x 32-bit little-endian words, value < 2^256.
//
// Why 29-bit limbs: gfx950 issues v_mad_u64_u32 (32x32+64 -> 64) at close to the
// full VALU rate (tools/ubench: measured), while every carry out of a 32-bit limb
// costs extra adds/movs.  With 29-bit limbs a product-scanning (FIPS) Montgomery
// multiply accumulates each column of up to 18 partial products in ONE 64-bit
// register pair without overflow (18 * 2^58 < 2^63), so each partial product is
// exactly one v_mad_u64_u32 and carries are resolved once per column (shift).
// Measured 171 G mul/s (vs 98 G mul/s for compiler CIOS on 8x32-bit limbs).
//
// Restates the arithmetic of ffjavascript/wasmcurves (f1m/frm Montgomery
// multiply) in a different radix: results are converted back to
// the snarkjs byte conventions at the boundary, so they are bit-identical.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "consts.hpp"

namespace zkp {

constexpr int NL = 9;
constexpr int LB = 29;
constexpr uint32_t LMASK = (1u << LB) - 1;

template <class C>
struct Fe {
  uint32_t v[NL];
};

using Fq = Fe<FqCfg>;
using Fr = Fe<FrCfg>;

#define ZDEV __host__ __device__ __forceinline__

// acc += x * y.  CH (C::CHAIN, device code): every product column stays ONE dependent chain seeded
// by the previous column's carry.  Left to itself the compiler re-associates each column into a sum
// from 0 plus a 64-bit join of the carry (v_lshl_add_u64 per column).  After each product the
// accumulator passes through an EMPTY asm statement that claims to modify it, so the column cannot be
// re-associated while the compiler still sees, schedules and hazard-checks real v_mad_u64_u32
// instructions (it interleaves independent products' chains to cover the wait states between
// dependent 64-bit mads).  tools/ubench/mul_chain.hip, profiles/mul_chain_r03.txt.  mac_k takes a
// constant.  Host code is always plain C.
template <bool CH>
ZDEV void mac(uint64_t& acc, uint32_t x, uint32_t y) {
  acc += (uint64_t)x * y;
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (CH) asm("" : "+v"(acc));
#endif
}
template <bool CH>
ZDEV void mac_k(uint64_t& acc, uint32_t x, uint32_t k) {
  acc += (uint64_t)x * k;
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (CH) asm("" : "+v"(acc));
#endif
}

template <class C>
ZDEV Fe<C> fe_zero() {
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = 0;
  return r;
}

template <class C>
ZDEV Fe<C> fe_const(const uint32_t (&k)[NL]) {
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = k[i];
  return r;
}

template <class C>
ZDEV Fe<C> fe_one() { return fe_const<C>(C::ONE); }

// Montgomery product a*b/2^261 mod m (FIPS / product scanning).
// Inputs: limbs 0..7 < 2^30, value < 8m.  Output: normalised limbs, value < 2m.
template <class C>
ZDEV Fe<C> mul(const Fe<C>& a, const Fe<C>& b) {
  uint32_t m[NL];
  Fe<C> r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      mac<C::CHAIN>(acc, a.v[j], b.v[i - j]);
      mac_k<C::CHAIN>(acc, m[j], C::MOD[i - j]);
    }
    mac<C::CHAIN>(acc, a.v[i], b.v[0]);
    m[i] = ((uint32_t)acc * C::INV) & LMASK;
    mac_k<C::CHAIN>(acc, m[i], C::MOD[0]);
    acc >>= LB;
  }
#pragma unroll
  for (int i = NL; i < 2 * NL - 1; ++i) {
#pragma unroll
    for (int j = i - NL + 1; j < NL; ++j) {
      mac<C::CHAIN>(acc, a.v[j], b.v[i - j]);
      mac_k<C::CHAIN>(acc, m[j], C::MOD[i - j]);
    }
    r.v[i - NL] = (uint32_t)acc & LMASK;
    acc >>= LB;
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// Product by a CONSTANT with a precomputed quotient (Shoup): a w mod m for w < m given as plain
// limbs and wq = floor(w 2^261 / m) (both normalised, 9 limbs).  q = floor(a wq / 2^261) from the
// product columns 7..17 only (the dropped columns 0..6 sum to < 2^237, so q is the exact floor or
// one less), then a w - q m = (a w + q (2^261 - m)) mod 2^261 from the low columns 0..8.  Since
// a w / m - a wq / 2^261 < a / 2^261 <= 1, the result is in [0, 3m).  a: limbs < 2^31 (a raw sum
// or borrow-form difference is fine), value < 2^261.  A Montgomery-form a stays in Montgomery
// form (w is plain).  143 v_mad_u64_u32 and no per-column quotient digits, against 162 mads plus
// 9 v_mul_lo_u32 for mul(); NTT roots, twiddles and the coset key are all constants.
template <class C>
ZDEV Fe<C> mul_shoup(const Fe<C>& a, const Fe<C>& w, const Fe<C>& wq) {
  uint32_t q[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int c = 7; c < 2 * NL - 1; ++c) {
#pragma unroll
    for (int i = (c - NL + 1 > 0 ? c - NL + 1 : 0); i <= (c < NL - 1 ? c : NL - 1); ++i) mac<C::CHAIN>(acc, a.v[i], wq.v[c - i]);
    if (c >= NL) q[c - NL] = (uint32_t)acc & LMASK;
    acc >>= LB;
  }
  q[NL - 1] = (uint32_t)acc;  // columns 9..16 give q's limbs 0..7, the carry out its top limb (q < 2^261)
  Fe<C> r;
  acc = 0;
#pragma unroll
  for (int c = 0; c < NL; ++c) {
#pragma unroll
    for (int i = 0; i <= c; ++i) {
      mac<C::CHAIN>(acc, a.v[i], w.v[c - i]);
      mac_k<C::CHAIN>(acc, q[i], C::NM[c - i]);
    }
    r.v[c] = (uint32_t)acc & LMASK;
    acc >>= LB;
  }
  return r;
}

// two independent Shoup products a w, c v in lockstep (column chains interleaved, as mul_pair)
template <class C>
ZDEV void mul_shoup_pair(const Fe<C>& a, const Fe<C>& w, const Fe<C>& wq, const Fe<C>& c, const Fe<C>& v,
                         const Fe<C>& vq, Fe<C>& r, Fe<C>& s) {
  uint32_t q[NL], p[NL];
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int k = 7; k < 2 * NL - 1; ++k) {
#pragma unroll
    for (int i = (k - NL + 1 > 0 ? k - NL + 1 : 0); i <= (k < NL - 1 ? k : NL - 1); ++i) {
      mac<C::CHAIN>(x, a.v[i], wq.v[k - i]);
      mac<C::CHAIN>(y, c.v[i], vq.v[k - i]);
    }
    if (k >= NL) {
      q[k - NL] = (uint32_t)x & LMASK;
      p[k - NL] = (uint32_t)y & LMASK;
    }
    x >>= LB;
    y >>= LB;
  }
  q[NL - 1] = (uint32_t)x;
  p[NL - 1] = (uint32_t)y;
  x = 0;
  y = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
#pragma unroll
    for (int i = 0; i <= k; ++i) {
      mac<C::CHAIN>(x, a.v[i], w.v[k - i]);
      mac<C::CHAIN>(y, c.v[i], v.v[k - i]);
      mac_k<C::CHAIN>(x, q[i], C::NM[k - i]);
      mac_k<C::CHAIN>(y, p[i], C::NM[k - i]);
    }
    r.v[k] = (uint32_t)x & LMASK;
    s.v[k] = (uint32_t)y & LMASK;
    x >>= LB;
    y >>= LB;
  }
}

// Shoup quotient of a constant from its canonical Montgomery form wm = w 2^261 mod m (< m):
// w 2^261 = wq m + wm, so wq = floor(w 2^261 / m) = -wm m^-1 mod 2^261 (a low-half product).
template <class C>
ZDEV Fe<C> shoup_quot(const Fe<C>& wm) {
  uint32_t p[NL];
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < NL; ++c) {
#pragma unroll
    for (int i = 0; i <= c; ++i) acc += (uint64_t)wm.v[i] * C::MINV261[c - i];
    p[c] = (uint32_t)acc & LMASK;
    acc >>= LB;
  }
  Fe<C> r;  // 2^261 - p  (mod 2^261)
  uint32_t carry = 1;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint32_t t = (LMASK - p[i]) + carry;
    r.v[i] = t & LMASK;
    carry = t >> LB;
  }
  return r;
}

// Montgomery product of a SUM of two products, (a*b + c*d)/2^261 mod m, with ONE
// reduction ("lazy reduction"): the a*b, c*d and m*MOD partial products of a column
// accumulate together.  All four operands normalised (limbs < 2^29; column sums
// <= 27 * 2^58 < 2^63) and a*b + c*d < m*2^261 (~169 m^2) for an output < 2m.  Used for
// Y3 = R (Q - X3) - Y1 PPP as R*(Q - X3) + Y1*(2m - PPP): one reduction and no
// subtraction instead of two multiplies and a subtraction (~230 instructions saved).
template <class C>
ZDEV Fe<C> mul2(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c, const Fe<C>& d) {
  uint32_t m[NL];
  Fe<C> r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      mac<C::CHAIN>(acc, a.v[j], b.v[i - j]);
      mac<C::CHAIN>(acc, c.v[j], d.v[i - j]);
      mac_k<C::CHAIN>(acc, m[j], C::MOD[i - j]);
    }
    mac<C::CHAIN>(acc, a.v[i], b.v[0]);
    mac<C::CHAIN>(acc, c.v[i], d.v[0]);
    m[i] = ((uint32_t)acc * C::INV) & LMASK;
    mac_k<C::CHAIN>(acc, m[i], C::MOD[0]);
    acc >>= LB;
  }
#pragma unroll
  for (int i = NL; i < 2 * NL - 1; ++i) {
#pragma unroll
    for (int j = i - NL + 1; j < NL; ++j) {
      mac<C::CHAIN>(acc, a.v[j], b.v[i - j]);
      mac<C::CHAIN>(acc, c.v[j], d.v[i - j]);
      mac_k<C::CHAIN>(acc, m[j], C::MOD[i - j]);
    }
    r.v[i - NL] = (uint32_t)acc & LMASK;
    acc >>= LB;
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// Squaring: cross products computed once against a doubled operand.
template <class C>
ZDEV Fe<C> sqr(const Fe<C>& a) {
  uint32_t m[NL], d[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) d[i] = a.v[i] << 1;
  Fe<C> r;
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
#pragma unroll
    for (int j = 0; j < (i + 1) / 2; ++j) mac<C::CHAIN>(acc, d[j], a.v[i - j]);
    if ((i & 1) == 0) mac<C::CHAIN>(acc, a.v[i / 2], a.v[i / 2]);
#pragma unroll
    for (int j = 0; j < i; ++j) mac_k<C::CHAIN>(acc, m[j], C::MOD[i - j]);
    m[i] = ((uint32_t)acc * C::INV) & LMASK;
    mac_k<C::CHAIN>(acc, m[i], C::MOD[0]);
    acc >>= LB;
  }
#pragma unroll
  for (int i = NL; i < 2 * NL - 1; ++i) {
#pragma unroll
    for (int j = i - NL + 1; j < (i + 1) / 2; ++j) mac<C::CHAIN>(acc, d[j], a.v[i - j]);
    if ((i & 1) == 0) mac<C::CHAIN>(acc, a.v[i / 2], a.v[i / 2]);
#pragma unroll
    for (int j = i - NL + 1; j < NL; ++j) mac_k<C::CHAIN>(acc, m[j], C::MOD[i - j]);
    r.v[i - NL] = (uint32_t)acc & LMASK;
    acc >>= LB;
  }
  r.v[NL - 1] = (uint32_t)acc;
  return r;
}

// Two independent Montgomery products / squares in lockstep (the chained columns of both
// interleave, so a dependent mad of one chain follows an independent mad of the other instead of
// a wait state).  Same arithmetic as mul() / sqr() on each pair.
template <class C>
ZDEV void mul_pair(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c, const Fe<C>& d, Fe<C>& r, Fe<C>& s) {
  uint32_t m[NL], n[NL];
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
      mac<C::CHAIN>(x, a.v[j], b.v[i - j]);
      mac<C::CHAIN>(y, c.v[j], d.v[i - j]);
      mac_k<C::CHAIN>(x, m[j], C::MOD[i - j]);
      mac_k<C::CHAIN>(y, n[j], C::MOD[i - j]);
    }
    mac<C::CHAIN>(x, a.v[i], b.v[0]);
    mac<C::CHAIN>(y, c.v[i], d.v[0]);
    m[i] = ((uint32_t)x * C::INV) & LMASK;
    n[i] = ((uint32_t)y * C::INV) & LMASK;
    mac_k<C::CHAIN>(x, m[i], C::MOD[0]);
    mac_k<C::CHAIN>(y, n[i], C::MOD[0]);
    x >>= LB;
    y >>= LB;
  }
#pragma unroll
  for (int i = NL; i < 2 * NL - 1; ++i) {
#pragma unroll
    for (int j = i - NL + 1; j < NL; ++j) {
      mac<C::CHAIN>(x, a.v[j], b.v[i - j]);
      mac<C::CHAIN>(y, c.v[j], d.v[i - j]);
      mac_k<C::CHAIN>(x, m[j], C::MOD[i - j]);
      mac_k<C::CHAIN>(y, n[j], C::MOD[i - j]);
    }
    r.v[i - NL] = (uint32_t)x & LMASK;
    s.v[i - NL] = (uint32_t)y & LMASK;
    x >>= LB;
    y >>= LB;
  }
  r.v[NL - 1] = (uint32_t)x;
  s.v[NL - 1] = (uint32_t)y;
}

// Two lazily reduced sums of N products, r = sum_k a[k] b[k], s = sum_k c[k] d[k], in lockstep with
// chained columns when CH: the Fq2 products of the G2 arithmetic (c0 and c1 of a product).  Operand
// conditions as mul2; N = 4: columns hold <= 36 + 9 partial products < 2^58 (< 2^63.5), the sum
// < ~169 m^2.
template <class C, bool CH, int N>
ZDEV void sop_pair(const Fe<C>* const (&a)[N], const Fe<C>* const (&b)[N], const Fe<C>* const (&c)[N],
                   const Fe<C>* const (&d)[N], Fe<C>& r, Fe<C>& s) {
  uint32_t m[NL], n[NL];
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
#pragma unroll
    for (int j = 0; j < i; ++j) {
#pragma unroll
      for (int k = 0; k < N; ++k) {
        mac<CH>(x, a[k]->v[j], b[k]->v[i - j]);
        mac<CH>(y, c[k]->v[j], d[k]->v[i - j]);
      }
      mac_k<CH>(x, m[j], C::MOD[i - j]);
      mac_k<CH>(y, n[j], C::MOD[i - j]);
    }
#pragma unroll
    for (int k = 0; k < N; ++k) {
      mac<CH>(x, a[k]->v[i], b[k]->v[0]);
      mac<CH>(y, c[k]->v[i], d[k]->v[0]);
    }
    m[i] = ((uint32_t)x * C::INV) & LMASK;
    n[i] = ((uint32_t)y * C::INV) & LMASK;
    mac_k<CH>(x, m[i], C::MOD[0]);
    mac_k<CH>(y, n[i], C::MOD[0]);
    x >>= LB;
    y >>= LB;
  }
#pragma unroll
  for (int i = NL; i < 2 * NL - 1; ++i) {
#pragma unroll
    for (int j = i - NL + 1; j < NL; ++j) {
#pragma unroll
      for (int k = 0; k < N; ++k) {
        mac<CH>(x, a[k]->v[j], b[k]->v[i - j]);
        mac<CH>(y, c[k]->v[j], d[k]->v[i - j]);
      }
      mac_k<CH>(x, m[j], C::MOD[i - j]);
      mac_k<CH>(y, n[j], C::MOD[i - j]);
    }
    r.v[i - NL] = (uint32_t)x & LMASK;
    s.v[i - NL] = (uint32_t)y & LMASK;
    x >>= LB;
    y >>= LB;
  }
  r.v[NL - 1] = (uint32_t)x;
  s.v[NL - 1] = (uint32_t)y;
}

template <class C>
ZDEV void sqr_pair(const Fe<C>& a, const Fe<C>& c, Fe<C>& r, Fe<C>& s) {
  uint32_t m[NL], n[NL], da[NL], dc[NL];
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    da[i] = a.v[i] << 1;
    dc[i] = c.v[i] << 1;
  }
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
#pragma unroll
    for (int j = 0; j < (i + 1) / 2; ++j) {
      mac<C::CHAIN>(x, da[j], a.v[i - j]);
      mac<C::CHAIN>(y, dc[j], c.v[i - j]);
    }
    if ((i & 1) == 0) {
      mac<C::CHAIN>(x, a.v[i / 2], a.v[i / 2]);
      mac<C::CHAIN>(y, c.v[i / 2], c.v[i / 2]);
    }
#pragma unroll
    for (int j = 0; j < i; ++j) {
      mac_k<C::CHAIN>(x, m[j], C::MOD[i - j]);
      mac_k<C::CHAIN>(y, n[j], C::MOD[i - j]);
    }
    m[i] = ((uint32_t)x * C::INV) & LMASK;
    n[i] = ((uint32_t)y * C::INV) & LMASK;
    mac_k<C::CHAIN>(x, m[i], C::MOD[0]);
    mac_k<C::CHAIN>(y, n[i], C::MOD[0]);
    x >>= LB;
    y >>= LB;
  }
#pragma unroll
  for (int i = NL; i < 2 * NL - 1; ++i) {
#pragma unroll
    for (int j = i - NL + 1; j < (i + 1) / 2; ++j) {
      mac<C::CHAIN>(x, da[j], a.v[i - j]);
      mac<C::CHAIN>(y, dc[j], c.v[i - j]);
    }
    if ((i & 1) == 0) {
      mac<C::CHAIN>(x, a.v[i / 2], a.v[i / 2]);
      mac<C::CHAIN>(y, c.v[i / 2], c.v[i / 2]);
    }
#pragma unroll
    for (int j = i - NL + 1; j < NL; ++j) {
      mac_k<C::CHAIN>(x, m[j], C::MOD[i - j]);
      mac_k<C::CHAIN>(y, n[j], C::MOD[i - j]);
    }
    r.v[i - NL] = (uint32_t)x & LMASK;
    s.v[i - NL] = (uint32_t)y & LMASK;
    x >>= LB;
    y >>= LB;
  }
  r.v[NL - 1] = (uint32_t)x;
  s.v[NL - 1] = (uint32_t)y;
}

// carry-propagate limbs 0..7 into 29-bit digits (limb values must be >= 0 and < 2^31)
template <class C>
ZDEV void normalize(Fe<C>& a) {
#pragma unroll
  for (int i = 0; i < NL - 1; ++i) {
    a.v[i + 1] += a.v[i] >> LB;
    a.v[i] &= LMASK;
  }
}

// a - M if a >= M else a   (a normalised; M normalised limbs)
template <class C>
ZDEV Fe<C> cond_sub(const Fe<C>& a, const uint32_t (&M)[NL]) {
  Fe<C> d;
  int32_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    int32_t t = (int32_t)a.v[i] - (int32_t)M[i] + carry;
    d.v[i] = (uint32_t)t & LMASK;
    carry = t >> LB;
  }
  // top limb: keep full (non-masked) value when no borrow
  const bool ge = carry >= 0;
  Fe<C> r;
#pragma unroll
  for (int i = 0; i < NL; ++i) r.v[i] = ge ? d.v[i] : a.v[i];
  return r;
}

// Quotient-estimate reduction: s (limbs 0..7 in [0, 2^32 - 2^10), unnormalised; value
// v in [0, 2^261)) -> v - q m, normalised, value < 1.2m, in ONE carry pass.  q comes from the
// top limb alone, q = floor(s8 * floor(2^264/m) / 2^32) <= v/m (all limbs >= 0), and
// v/m - q < 1 + 2^-3 + (low limbs) / m, so 0 <= v - q m < 1.2m.  v - q m = (v + q (2^261 - m))
// mod 2^261: per limb one v_mad_u64_u32 (q * NM[i] + s[i] + carry < 2^39), a mask and a shift,
// instead of a carry pass plus one or two borrow-chain conditional subtractions with selects
// (34 vs 65-105 instructions).  A top limb that went "negative" (uint32 wrap of a wide-borrow
// form whose true top, after the lower carries, is >= 0) has a value < 2^235 < m: q = 0.
template <class C>
ZDEV Fe<C> qreduce(const Fe<C>& s) {
  const int32_t top = (int32_t)s.v[NL - 1];
  const uint32_t q = top > 0 ? (uint32_t)(((uint64_t)(uint32_t)top * C::QK) >> 32) : 0u;
  Fe<C> r;
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    const uint64_t acc = (uint64_t)q * C::NM[i] + (uint64_t)(s.v[i] + carry);
    r.v[i] = (uint32_t)acc & LMASK;
    carry = (uint32_t)(acc >> LB);
  }
  return r;
}

// s (limbs < 2^31, value < 4m) -> < 2m: qreduce for Fr (C::QRED: the NTT, 3 waves/SIMD, 5 % faster
// per transform), carry pass + one conditional subtraction for Fq, whose XYZZ kernels are
// register-bound (qreduce's 64-bit temporaries: 124 -> 135 VGPRs in k_accumulate, 4 -> 3 waves).
template <class C>
ZDEV Fe<C> reduce2(Fe<C> s) {
  if constexpr (C::QRED) {
    return qreduce(s);
  } else {
    normalize(s);
    return cond_sub(s, C::MOD2);
  }
}

// a + b, inputs < 2m (normalised) -> output < 2m
template <class C>
ZDEV Fe<C> add(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + b.v[i];
  return reduce2(s);
}

// a - b, inputs < 2m -> output < 2m   (computes a + 2m - b)
template <class C>
ZDEV Fe<C> sub(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD2_BORROW[i] - b.v[i];
  return reduce2(s);
}

// a - b for a normalised a < 4m and b <= 4m (computes a + 4m - b): output < 2m (Fr: qreduce < 1.2m).
// The NTT with Shoup root products (outputs < 3m) subtracts with it.
template <class C>
ZDEV Fe<C> sub4(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD4_BORROW[i] - b.v[i];
  if constexpr (C::QRED) {
    return qreduce(s);
  } else {
    normalize(s);
    return cond_sub(cond_sub(s, C::MOD4), C::MOD2);
  }
}

// ---- lazy subtractions: results that only ever feed a multiplication skip the final
// conditional subtraction (and, for one mul operand, even the carry normalisation):
// mul() accepts values < 8m, and one operand with limbs < 2^31 when the other is
// normalised (column sums stay < 9*2^60 + 9*2^58 + 2^35 < 2^64).  ~46 resp. ~70 VALU
// instructions saved per use (an XYZZ mixed add has ~3000).

// a - b + 2m, normalised, value < 4m: an operand of mul() / sqr() only
template <class C>
ZDEV Fe<C> lsub(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD2_BORROW[i] - b.v[i];
  normalize(s);
  return s;
}

// a - b + 4m, NOT normalised (every limb in [0, 2^31), value < 6m): ONE operand of
// mul() whose other operand is normalised; never sqr(), add(), sub(), is_zero(), storage
template <class C>
ZDEV Fe<C> rsub(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD4_BORROW[i] - b.v[i];
  return s;
}

// a - b - 2c for a, b, c < 2m (normalised), result < 2m: one limb pass against 6m in the
// wide borrow form (low limbs + 2^31, so three subtrahends never borrow), one carry
// normalisation (value in (0, 8m)), then conditional subtractions of 4m and 2m.  The
// X3 = R^2 - PPP - 2Q of every XYZZ add in one go (~150 instead of ~250 instructions).
template <class C>
ZDEV Fe<C> sub_2x(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD6_WIDE[i] - b.v[i] - (c.v[i] << 1);
  if constexpr (C::QRED) {
    return qreduce(s);
  } else {
    normalize(s);
    return cond_sub(cond_sub(s, C::MOD4), C::MOD2);
  }
}

// ---- lazily reduced accumulator x (G1 XYZZ additions): X3 = R^2 - PPP - 2Q stays in (0, 8m)
// without its two conditional subtractions (~90 instructions per addition).  Every consumer takes
// an x < 8m: mul()/sqr() operands (the output stays < 2m up to operands of ~11m: a*b/2^261 + m
// < 2m for a*b < 169 m^2), lsub8() for the differences, canon8() before storage.

// a - b - 2c + 6m for a, b, c < 2m (normalised): normalised, value in (0, 8m)
template <class C>
ZDEV Fe<C> sub_2x8(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD6_WIDE[i] - b.v[i] - (c.v[i] << 1);
  normalize(s);
  return s;
}

// a - b + 8m for a < 2m, b < 8m (normalised): normalised, value < 10m -- a mul / sqr operand
template <class C>
ZDEV Fe<C> lsub8(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD8_BORROW[i] - b.v[i];
  normalize(s);
  return s;
}

// x < 8m (normalised) -> < 2m
template <class C>
ZDEV Fe<C> canon8(const Fe<C>& a) { return cond_sub(cond_sub(a, C::MOD4), C::MOD2); }

// a - b + 4m (b < 4m) and a - b + 6m (b < 6m), normalised: mul / sqr operands
template <class C>
ZDEV Fe<C> lsub4(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD4_BORROW[i] - b.v[i];
  normalize(s);
  return s;
}
template <class C>
ZDEV Fe<C> lsub6(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD6_BORROW[i] - b.v[i];
  normalize(s);
  return s;
}
// 2a, limbs shifted (raw: limbs < 2^30 for a normalised a): ONE operand of mul()
template <class C>
ZDEV Fe<C> shl1_raw(const Fe<C>& a) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] << 1;
  return s;
}

// ---- lazy radix-4 sums (NTT): a first-stage sum x + y of two normalised values < 2m is kept
// raw (limbs < 2^30, value < 4m, no carry pass and no conditional subtraction); the second
// stage consumes two such sums:

// a + b for raw sums a, b < 4m: normalised and reduced from < 8m to < 2m
template <class C>
ZDEV Fe<C> add_raw_reduce(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + b.v[i];
  if constexpr (C::QRED) {
    return qreduce(s);
  } else {
    normalize(s);
    return cond_sub(cond_sub(s, C::MOD4), C::MOD2);
  }
}

// a - b + 6m for raw sums a, b < 4m (wide borrow form: every limb stays >= 0), normalised,
// value < 10m: an operand of mul() against a normalised value < 2m only (product < 20 m^2)
template <class C>
ZDEV Fe<C> sub_raw6(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD6_WIDE[i] - b.v[i];
  normalize(s);
  return s;
}

// a - b + 8m for raw sums a, b < 6m of two normalised values each (limbs < 2^30), WITHOUT a carry
// pass: the 8m borrow form whose low limbs are raised by 2^30 (consts MOD8_B30) keeps every limb
// >= 0 and < 2^30 + 2^30 + 2^29 = 2.5 * 2^30, value < 14m.  An operand of mul_shoup (column sums
// <= 9 (2.5 + 0.5) 2^59 < 2^63.8), of mul() against a normalised value, or of qreduce (limbs
// < 2^32 - 2^10) -- never a second raw operand (the NTT's radix-4 unit, round 5: 24 instructions
// fewer than sub_raw6 per use).  The top limb: b's is at most 2 x (3m - 1)'s (0x12259d6), and 8m's
// raised form keeps 0x1832270 there, so it stays >= 0 for every a (round 6, ADVICE r5: the 6m form's
// 0x12259d4 wrapped below zero for a ~ 0 against b ~ 6m; tools/hosttest r4lazy covers that quad)
template <class C>
ZDEV Fe<C> sub_raw6n(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + C::MOD8_B30[i] - b.v[i];
  return s;
}

template <class C>
ZDEV Fe<C> add_raw(const Fe<C>& a, const Fe<C>& b) {
  Fe<C> s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = a.v[i] + b.v[i];
  return s;
}

template <class C>
ZDEV Fe<C> dbl(const Fe<C>& a) { return add(a, a); }

template <class C>
ZDEV Fe<C> neg(const Fe<C>& a) { return sub(fe_zero<C>(), a); }

// canonical representative in [0, m) of a value < 2m
template <class C>
ZDEV Fe<C> canon(const Fe<C>& a) { return cond_sub(a, C::MOD); }

template <class C>
ZDEV bool is_zero_raw(const Fe<C>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) o |= a.v[i];
  return o == 0;
}

// value (< 2m) congruent to 0 mod m
template <class C>
ZDEV bool is_zero(const Fe<C>& a) {
  uint32_t o = 0, q = 0;
#pragma unroll
  for (int i = 0; i < NL; ++i) {
    o |= a.v[i];
    q |= a.v[i] ^ C::MOD[i];
  }
  return o == 0 || q == 0;
}

template <class C>
ZDEV bool eq(const Fe<C>& a, const Fe<C>& b) { return is_zero(sub(a, b)); }

// ---------------------------------------------------------------- storage conversions

// 8 x 32-bit words (value < 2^256) -> 9 x 29-bit limbs
template <class C>
ZDEV Fe<C> unpack(const uint32_t (&w)[8]) {
  Fe<C> r;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int bit = LB * k, j = bit >> 5, s = bit & 31;
    uint32_t lo = w[j] >> s;
    uint32_t hi = (j + 1 < 8 && s != 0) ? (w[j + 1] << (32 - s)) : 0u;
    r.v[k] = (k == NL - 1) ? (lo | hi) : ((lo | hi) & LMASK);
  }
  return r;
}

// 9 x 29-bit normalised limbs (value < 2^256) -> 8 x 32-bit words
template <class C>
ZDEV void pack(const Fe<C>& a, uint32_t (&w)[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int bit = 32 * j, k = bit / LB, s = bit - LB * k;  // word starts s bits into limb k
    uint32_t x = a.v[k] >> s;
    if (k + 1 < NL) x |= a.v[k + 1] << (LB - s);
    if (k + 2 < NL && 2 * LB - s < 32) x |= a.v[k + 2] << (2 * LB - s);
    w[j] = x;
  }
}

template <class C>
ZDEV Fe<C> load_fe(const uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return unpack<C>(w);
}

template <class C>
ZDEV void store_fe(uint32_t* p, const Fe<C>& x) {
  uint32_t w[8];
  pack(x, w);
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

// standard integer (< 2^256) -> Montgomery(R') compute form
template <class C>
ZDEV Fe<C> to_mont(const Fe<C>& a) { return mul(a, fe_const<C>(C::R2)); }

// Montgomery(R') -> canonical standard integer (< m)
template <class C>
ZDEV Fe<C> from_mont(const Fe<C>& a) {
  Fe<C> one = fe_zero<C>();
  one.v[0] = 1;
  return canon(mul(a, one));
}

// a^(m-2) = a^-1 (Fermat), Montgomery form in and out; 0 -> 0.  Square-and-multiply
// over the fixed exponent: ~254 S + ~130 M.  Load-time only (base-table precompute).
template <class C>
ZDEV Fe<C> inv(const Fe<C>& a) {
  Fe<C> r = fe_one<C>();
  for (int wi = 7; wi >= 0; --wi) {
    const uint32_t e = C::MOD_W[wi] - (wi == 0 ? 2u : 0u);
    for (int b = 31; b >= 0; --b) {
      r = sqr(r);
      if ((e >> b) & 1u) r = mul(r, a);
    }
  }
  return r;
}

// ---------------------------------------------------------------- Fq2 = Fq[u]/(u^2+1)

struct Fq2 {
  Fq c0, c1;
};

// 4m - a, normalised, for a normalised a <= 4m (Fq2 components are < 4m: rsub's)
ZDEV Fq neg4(const Fq& a) {
  Fq s;
#pragma unroll
  for (int i = 0; i < NL; ++i) s.v[i] = FqCfg::MOD4_BORROW[i] - a.v[i];
  normalize(s);
  return s;
}

// (a0 + a1 u)(b0 + b1 u) = (a0 b0 - a1 b1) + (a0 b1 + a1 b0) u as two lazily reduced sums
// of products (2 x 162 + 2 x 81 mads, like Karatsuba's 3 x 162, but no Karatsuba adds and
// subtractions: ~650 instead of ~1100 instructions).  Components normalised, < 4m.
// The two components' sums of products run in lockstep with chained columns (sop_pair): the 2-wave
// G2 kernels gain with paired chains (profiles/g2_chain_r03.txt).
ZDEV Fq2 mul(const Fq2& a, const Fq2& b) {
  Fq2 r;
  const Fq nb1 = neg4(b.c1);
  const Fq* x0[2] = {&a.c0, &a.c1};
  const Fq* y0[2] = {&b.c0, &nb1};
  const Fq* y1[2] = {&b.c1, &b.c0};
  sop_pair<FqCfg, true, 2>(x0, y0, x0, y1, r.c0, r.c1);
  return r;
}

// a*b + c*d in Fq2 with two lazily reduced four-product sums
ZDEV Fq2 mul2(const Fq2& a, const Fq2& b, const Fq2& c, const Fq2& d) {
  Fq2 r;
  const Fq nb1 = neg4(b.c1), nd1 = neg4(d.c1);
  const Fq* x[4] = {&a.c0, &a.c1, &c.c0, &c.c1};
  const Fq* y0[4] = {&b.c0, &nb1, &d.c0, &nd1};
  const Fq* y1[4] = {&b.c1, &b.c0, &d.c1, &d.c0};
  sop_pair<FqCfg, true, 4>(x, y0, x, y1, r.c0, r.c1);
  return r;
}

ZDEV Fq2 sqr(const Fq2& a) {
  // (a0 + a1 u)^2 = (a0+a1)(a0-a1) + 2 a0 a1 u
  Fq2 r;
  r.c0 = mul(add(a.c0, a.c1), sub(a.c0, a.c1));
  Fq t = mul(a.c0, a.c1);
  r.c1 = add(t, t);
  return r;
}

// ---- lazily reduced G2 accumulator forms (curve.hpp acc_*): every component normalised, value
// bounds as noted; the products stay < 2m as long as each Fq sum of products of a Fq2 mul/mul2
// (neg4 on the second operand's c1, which must be <= 4m) stays below ~169 m^2.
// a - b + 2m per component for a, b < 2m: < 4m, no conditional subtraction
ZDEV Fq2 lsub2_lazy(const Fq2& a, const Fq2& b) { return Fq2{lsub(a.c0, b.c0), lsub(a.c1, b.c1)}; }
// a - b + 4m per component for a < 2m, b < 4m: < 6m
ZDEV Fq2 lsub4_lazy(const Fq2& a, const Fq2& b) { return Fq2{lsub4(a.c0, b.c0), lsub4(a.c1, b.c1)}; }
// a^2 for components < 6m: (a0 + a1)(a0 - a1 + 6m) [raw sum x normalised, < 144 m^2] and
// (2 a0) a1 [raw x normalised, < 72 m^2] -- no additions reduced, no doubling of the product
ZDEV Fq2 sqr_lazy(const Fq2& a) {
  const Fq s = add_raw(a.c0, a.c1), d = lsub6(a.c0, a.c1), t = shl1_raw(a.c0);
  const Fq* x0[1] = {&s};
  const Fq* y0[1] = {&d};
  const Fq* x1[1] = {&t};
  const Fq* y1[1] = {&a.c1};
  Fq2 r;
  sop_pair<FqCfg, true, 1>(x0, y0, x1, y1, r.c0, r.c1);
  return r;
}
// R^2 - PPP - 2Q per component (each < 2m) -> < 4m: one conditional subtraction instead of two.
// (Not qreduce: its single 27-deep dependent chain per component measured 6 % slower in the
// G2 accumulation, which runs at two waves per SIMD and cannot hide the latency.)
ZDEV Fq2 sub_2x4(const Fq2& a, const Fq2& b, const Fq2& c) {
  return Fq2{cond_sub(sub_2x8(a.c0, b.c0, c.c0), FqCfg::MOD4), cond_sub(sub_2x8(a.c1, b.c1, c.c1), FqCfg::MOD4)};
}
// components < 4m -> < 2m
ZDEV Fq2 canon4(const Fq2& a) { return Fq2{cond_sub(a.c0, FqCfg::MOD2), cond_sub(a.c1, FqCfg::MOD2)}; }

ZDEV Fq2 add(const Fq2& a, const Fq2& b) { return Fq2{add(a.c0, b.c0), add(a.c1, b.c1)}; }
// Fq2 lazy forms: Karatsuba mul() adds the components of each operand, so a raw
// (unnormalised) operand is not allowed; a normalised < 4m one is (sums < 6m after add's
// conditional subtraction, products < 24 m^2 < m R').  sqr() subtracts components, so
// its operand stays canonical: lsub = sub.
ZDEV Fq2 sub_2x(const Fq2& a, const Fq2& b, const Fq2& c) {
  return Fq2{sub_2x(a.c0, b.c0, c.c0), sub_2x(a.c1, b.c1, c.c1)};
}
ZDEV Fq2 lsub(const Fq2& a, const Fq2& b) { return Fq2{sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
ZDEV Fq2 rsub(const Fq2& a, const Fq2& b) { return Fq2{lsub(a.c0, b.c0), lsub(a.c1, b.c1)}; }
ZDEV Fq2 sub(const Fq2& a, const Fq2& b) { return Fq2{sub(a.c0, b.c0), sub(a.c1, b.c1)}; }
ZDEV Fq2 dbl(const Fq2& a) { return add(a, a); }
ZDEV bool is_zero(const Fq2& a) { return is_zero(a.c0) && is_zero(a.c1); }
ZDEV bool is_zero_raw(const Fq2& a) { return is_zero_raw(a.c0) && is_zero_raw(a.c1); }
// (c0 + c1 u)^-1 = (c0 - c1 u) / (c0^2 + c1^2)
ZDEV Fq2 inv(const Fq2& a) {
  const Fq t = inv(add(sqr(a.c0), sqr(a.c1)));
  return Fq2{mul(a.c0, t), mul(sub(fe_zero<FqCfg>(), a.c1), t)};
}

}  // namespace zkp
