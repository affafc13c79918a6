// BN254 G1 / G2 group arithmetic for gfx950 — device side.
//
// Buckets and partial sums use XYZZ coordinates (x = X/ZZ, y = Y/ZZZ,
// ZZ^3 = ZZZ^2): a mixed add (XYZZ + affine) is 8M + 2S and needs no inversion
// (hyperelliptic.org EFD "madd-2008-s"; full add "add-2008-s", doubling
// "dbl-2008-s-1", affine doubling "mdbl-2008-s-1").  Infinity is ZZ == ZZZ == 0
// held exactly (never produced by arithmetic on non-degenerate inputs).  Affine
// infinity is (0, 0), which is off-curve, matching the zkey encoding of the
// point at infinity as all-zero bytes.
//
// Every edge case (P == Q -> doubling, P == -Q -> infinity) is handled, so MSM
// results are exact for any inputs (restating ffjavascript g1m/g2m add, A11).
#pragma once
#include "field.hpp"

namespace zkp {

template <class F>
struct Aff {
  F x, y;
};

template <class F>
struct Xyzz {
  F x, y, zz, zzz;
};

// zero / one of a base field (any Fe<C>: Fq, or Fq as the accumulation computes it) or of Fq2
template <class F>
struct FConst;
template <class C>
struct FConst<Fe<C>> {
  static ZDEV Fe<C> zero() { return fe_zero<C>(); }
  static ZDEV Fe<C> one() { return fe_one<C>(); }
};
template <>
struct FConst<Fq2> {
  static ZDEV Fq2 zero() { return Fq2{fe_zero<FqCfg>(), fe_zero<FqCfg>()}; }
  static ZDEV Fq2 one() { return Fq2{fe_one<FqCfg>(), fe_zero<FqCfg>()}; }
};
template <class F>
ZDEV F f_zero() { return FConst<F>::zero(); }
template <class F>
ZDEV F f_one() { return FConst<F>::one(); }

// Accumulator-coordinate forms: the XYZZ additions keep x and the differences lazily reduced.
//  G1: x < 8m (field.hpp sub_2x8: no conditional subtraction), differences with x via lsub8
//      (< 10m), the d = 4m - PPP operand of the Y3 sum of products unnormalised (rsub: one
//      mul2 operand may have limbs < 2^31, its partner normalised).
//  G2: x < 4m (one conditional subtraction per component instead of two), P, R < 6m / 4m
//      without conditional subtractions, squares of such values by sqr_lazy; the Y3 sum of
//      products puts the < 6m factor first (Fq2 mul2 negates the SECOND factor's c1, which must
//      stay <= 4m).  Bounds: field.hpp, host-tested (tools/hosttest).
template <class C>
ZDEV Fe<C> acc_x3(const Fe<C>& rr, const Fe<C>& ppp, const Fe<C>& q) { return sub_2x8(rr, ppp, q); }
ZDEV Fq2 acc_x3(const Fq2& rr, const Fq2& ppp, const Fq2& q) { return sub_2x4(rr, ppp, q); }
template <class C>
ZDEV Fe<C> acc_xsub(const Fe<C>& a, const Fe<C>& x) { return lsub8(a, x); }  // a - x for an accumulator x
ZDEV Fq2 acc_xsub(const Fq2& a, const Fq2& x) { return lsub4_lazy(a, x); }
template <class C>
ZDEV Fe<C> acc_sub(const Fe<C>& a, const Fe<C>& b) { return lsub(a, b); }  // a - b, both < 2m
ZDEV Fq2 acc_sub(const Fq2& a, const Fq2& b) { return lsub2_lazy(a, b); }
template <class C>
ZDEV Fe<C> acc_sqr(const Fe<C>& a) { return sqr(a); }  // a < 11m
ZDEV Fq2 acc_sqr(const Fq2& a) { return sqr_lazy(a); }  // components < 6m
template <class C>
ZDEV Fe<C> acc_negd(const Fe<C>& a) { return rsub(fe_zero<C>(), a); }
ZDEV Fq2 acc_negd(const Fq2& a) { return lsub2_lazy(Fq2{fe_zero<FqCfg>(), fe_zero<FqCfg>()}, a); }
// Y3 = R T + Y D (T = Q - X3, D = -PPP)
template <class C>
ZDEV Fe<C> acc_y3(const Fe<C>& r, const Fe<C>& t, const Fe<C>& y, const Fe<C>& d) { return mul2(r, t, y, d); }
ZDEV Fq2 acc_y3(const Fq2& r, const Fq2& t, const Fq2& y, const Fq2& d) { return mul2(t, r, d, y); }
template <class C>
ZDEV Fe<C> acc_xcanon(const Fe<C>& x) { return canon8(x); }
ZDEV Fq2 acc_xcanon(const Fq2& x) { return canon4(x); }

// independent products of the mixed addition in lockstep: a chained field config (C::CHAIN) runs
// each pair with interleaved column chains (field.hpp mul_pair / sqr_pair); otherwise, and for Fq2,
// plain products (a lockstep triple measured no better, profiles/mul_pairs_r03.txt)
template <class F>
ZDEV void mul_2(const F& a, const F& b, const F& c, const F& d, F& r, F& s) {
  r = mul(a, b);
  s = mul(c, d);
}
template <class C>
ZDEV void mul_2(const Fe<C>& a, const Fe<C>& b, const Fe<C>& c, const Fe<C>& d, Fe<C>& r, Fe<C>& s) {
  if constexpr (C::CHAIN) {
    mul_pair(a, b, c, d, r, s);
  } else {
    r = mul(a, b);
    s = mul(c, d);
  }
}
template <class F>
ZDEV void acc_sqr_2(const F& a, const F& c, F& r, F& s) {
  r = acc_sqr(a);
  s = acc_sqr(c);
}
template <class C>
ZDEV void acc_sqr_2(const Fe<C>& a, const Fe<C>& c, Fe<C>& r, Fe<C>& s) {
  if constexpr (C::CHAIN) {
    sqr_pair(a, c, r, s);
  } else {
    r = acc_sqr(a);
    s = acc_sqr(c);
  }
}

template <class F>
ZDEV Xyzz<F> xyzz_inf() {
  Xyzz<F> r;
  r.x = f_one<F>();
  r.y = f_one<F>();
  r.zz = f_zero<F>();
  r.zzz = f_zero<F>();
  return r;
}

template <class F>
ZDEV bool xyzz_is_inf(const Xyzz<F>& p) { return is_zero_raw(p.zz); }

// one-limb screens of the exact zero tests: lo_zero(a) is necessary for a == 0 (raw), maybe_zero(a)
// for a normalised a < 2m to be 0 or m (is_zero)
template <class C>
ZDEV bool lo_zero(const Fe<C>& a) { return a.v[0] == 0; }
ZDEV bool lo_zero(const Fq2& a) { return a.c0.v[0] == 0 && a.c1.v[0] == 0; }
template <class C>
ZDEV bool maybe_zero(const Fe<C>& a) { return a.v[0] == 0 || a.v[0] == C::MOD[0]; }
ZDEV bool maybe_zero(const Fq2& a) { return maybe_zero(a.c0) && maybe_zero(a.c1); }

template <class F>
ZDEV bool aff_is_inf(const Aff<F>& p) { return is_zero_raw(p.x) && is_zero_raw(p.y); }

template <class F>
ZDEV Aff<F> aff_neg(const Aff<F>& p) {
  Aff<F> r;
  r.x = p.x;
  r.y = sub(f_zero<F>(), p.y);
  return r;
}

// 2 * (x, y), affine input (mdbl-2008-s-1)
template <class F>
ZDEV Xyzz<F> xyzz_dbl_aff(const Aff<F>& p) {
  F U = dbl(p.y);
  F V = sqr(U);
  F W = mul(U, V);
  F S = mul(p.x, V);
  F X2 = sqr(p.x);
  F M = add(dbl(X2), X2);
  Xyzz<F> r;
  r.x = sub_2x(sqr(M), f_zero<F>(), S);
  r.y = mul2(M, lsub(S, r.x), W, lsub(f_zero<F>(), p.y));  // M (S - X3) - W Y
  r.zz = V;
  r.zzz = W;
  return r;
}

// 2 * P (dbl-2008-s-1, a = 0); p.x may be a lazily reduced accumulator x (acc_xcanon first:
// the doubling formulas take canonical coordinates)
template <class F>
ZDEV Xyzz<F> xyzz_dbl(const Xyzz<F>& p_in) {
  if (xyzz_is_inf(p_in)) return p_in;
  Xyzz<F> p = p_in;
  p.x = acc_xcanon(p.x);
  F U = dbl(p.y);
  F V = sqr(U);
  F W = mul(U, V);
  F S = mul(p.x, V);
  F X2 = sqr(p.x);
  F M = add(dbl(X2), X2);
  Xyzz<F> r;
  r.x = sub_2x(sqr(M), f_zero<F>(), S);
  r.y = mul2(M, lsub(S, r.x), W, lsub(f_zero<F>(), p.y));  // M (S - X3) - W Y
  r.zz = mul(V, p.zz);
  r.zzz = mul(W, p.zzz);
  return r;
}

// acc += (neg ? -q : q) (q affine, may be infinity)  — madd-2008-s.  The common path
// uses lazy subtractions (P, R: lsub; Q - X3 and -y: rsub) where the value only feeds
// a multiplication; zero tests run on PP = P^2 and RR = R^2, which are < 2m.
template <class F>
ZDEV void xyzz_add_aff(Xyzz<F>& acc, const Aff<F>& q, bool neg = false) {
  // the exceptional cases (a base at infinity, an empty accumulator, P = +-Q below) are screened
  // by their low limb first: the exact tests run only where it allows them, never on the common path
  if (lo_zero(q.x) && lo_zero(q.y)) {
    if (aff_is_inf(q)) return;
  }
  if (lo_zero(acc.zz)) {
    if (xyzz_is_inf(acc)) {
      acc.x = q.x;
      acc.y = neg ? sub(f_zero<F>(), q.y) : q.y;
      acc.zz = f_one<F>();
      acc.zzz = f_one<F>();
      return;
    }
  }
  const F qy = neg ? rsub(f_zero<F>(), q.y) : q.y;  // mul operand only
  F U2, S2;
  mul_2(q.x, acc.zz, qy, acc.zzz, U2, S2);
  F P = acc_xsub(U2, acc.x);
  F R = acc_sub(S2, acc.y);
  F PP, RR;
  acc_sqr_2(P, R, PP, RR);
  if (maybe_zero(PP)) {
    if (is_zero(PP)) {
      if (is_zero(RR)) {
        Aff<F> qs = q;
        if (neg) qs.y = sub(f_zero<F>(), q.y);
        acc = xyzz_dbl_aff(qs);
      } else {
        acc = xyzz_inf<F>();
      }
      return;
    }
  }
  F PPP, Q, ZZ3, ZZZ3;
  mul_2(P, PP, acc.x, PP, PPP, Q);
  const F X3 = acc_x3(RR, PPP, Q);
  const F Y3 = acc_y3(R, acc_xsub(Q, X3), acc.y, acc_negd(PPP));  // R (Q - X3) - Y1 PPP
  mul_2(acc.zz, PP, acc.zzz, PPP, ZZ3, ZZZ3);
  acc.x = X3;
  acc.zz = ZZ3;
  acc.zzz = ZZZ3;
  acc.y = Y3;
}

// (np ? -p : p) + (nq ? -q : q), both affine: the first addition of a bucket task.  With
// ZZ1 = ZZZ1 = 1 the mixed add loses its four products by ZZ/ZZZ (U2 = x2, S2 = y2,
// ZZ3 = PP, ZZZ3 = PPP): 4M + 2S instead of 8M + 2S.  Infinity inputs take the generic path.
template <class F>
ZDEV Xyzz<F> xyzz_from_aff_pair(const Aff<F>& p, bool np, const Aff<F>& q, bool nq) {
  Xyzz<F> acc = xyzz_inf<F>();
  if (aff_is_inf(p) || aff_is_inf(q)) {
    xyzz_add_aff(acc, p, np);
    xyzz_add_aff(acc, q, nq);
    return acc;
  }
  const F py = np ? sub(f_zero<F>(), p.y) : p.y;
  const F qy = nq ? sub(f_zero<F>(), q.y) : q.y;
  F P = acc_sub(q.x, p.x);
  F R = acc_sub(qy, py);
  F PP = acc_sqr(P);
  F RR = acc_sqr(R);
  if (is_zero(PP)) {
    if (is_zero(RR)) return xyzz_dbl_aff(Aff<F>{p.x, py});
    return acc;  // p == -q
  }
  F PPP = mul(P, PP);
  F Q = mul(p.x, PP);
  acc.x = acc_x3(RR, PPP, Q);
  acc.y = acc_y3(R, acc_xsub(Q, acc.x), py, acc_negd(PPP));  // R (Q - X3) - Y1 PPP
  acc.zz = PP;
  acc.zzz = PPP;
  return acc;
}

// acc += q (both XYZZ) — add-2008-s, with the same lazy subtractions as xyzz_add_aff
template <class F>
ZDEV void xyzz_add(Xyzz<F>& acc, const Xyzz<F>& q) {
  if (xyzz_is_inf(q)) return;
  if (xyzz_is_inf(acc)) {
    acc = q;
    return;
  }
  F U1, U2, S1, S2;
  mul_2(acc.x, q.zz, q.x, acc.zz, U1, U2);
  mul_2(acc.y, q.zzz, q.y, acc.zzz, S1, S2);
  F P = acc_sub(U2, U1);
  F R = acc_sub(S2, S1);
  F PP, RR;
  acc_sqr_2(P, R, PP, RR);
  if (is_zero(PP)) {
    if (is_zero(RR))
      acc = xyzz_dbl(acc);
    else
      acc = xyzz_inf<F>();
    return;
  }
  F PPP, Q;
  mul_2(P, PP, U1, PP, PPP, Q);
  F X3 = acc_x3(RR, PPP, Q);
  F Y3 = acc_y3(R, acc_xsub(Q, X3), S1, acc_negd(PPP));  // R (Q - X3) - S1 PPP
  F ZZ, ZZZ;
  mul_2(acc.zz, q.zz, acc.zzz, q.zzz, ZZ, ZZZ);
  mul_2(ZZ, PP, ZZZ, PPP, acc.zz, acc.zzz);
  acc.x = X3;
  acc.y = Y3;
}

template <class F>
ZDEV Xyzz<F> xyzz_neg(const Xyzz<F>& p) {
  Xyzz<F> r = p;
  r.y = sub(f_zero<F>(), p.y);
  return r;
}

// XYZZ -> affine (x = X/ZZ, y = Y/ZZZ) with one inversion of ZZ*ZZZ; infinity -> (0, 0)
template <class F>
ZDEV Aff<F> xyzz_to_aff(const Xyzz<F>& p) {
  Aff<F> a;
  if (xyzz_is_inf(p)) {
    a.x = f_zero<F>();
    a.y = f_zero<F>();
    return a;
  }
  const F I = inv(mul(p.zz, p.zzz));
  a.x = mul(p.x, mul(p.zzz, I));
  a.y = mul(p.y, mul(p.zz, I));
  return a;
}

// ---------------------------------------------------------------- storage (HBM) layouts
// G1 affine: 16 words (x, y), each 8 LE words.  G2 affine: 32 words (x.c0, x.c1, y.c0, y.c1).
// XYZZ: 4 coordinates in the same order.

template <class C>
ZDEV void load_f(const uint32_t* p, Fe<C>& x) { x = load_fe<C>(p); }
ZDEV void load_f(const uint32_t* p, Fq2& x) {
  x.c0 = load_fe<FqCfg>(p);
  x.c1 = load_fe<FqCfg>(p + 8);
}
template <class C>
ZDEV void store_f(uint32_t* p, const Fe<C>& x) { store_fe(p, x); }
ZDEV void store_f(uint32_t* p, const Fq2& x) {
  store_fe(p, x.c0);
  store_fe(p + 8, x.c1);
}

template <class F>
struct FWords;
template <class C>
struct FWords<Fe<C>> {
  static constexpr int W = 8;
};
template <>
struct FWords<Fq2> {
  static constexpr int W = 16;
};

template <class F>
ZDEV Aff<F> load_aff(const uint32_t* base, size_t idx) {
  constexpr int W = FWords<F>::W;
  const uint32_t* p = base + idx * (2 * W);
  Aff<F> r;
  load_f(p, r.x);
  load_f(p + W, r.y);
  return r;
}

template <class F>
ZDEV void store_aff(uint32_t* base, size_t idx, const Aff<F>& a) {
  constexpr int W = FWords<F>::W;
  uint32_t* p = base + idx * (2 * W);
  store_f(p, a.x);
  store_f(p + W, a.y);
}

template <class F>
ZDEV Xyzz<F> load_xyzz(const uint32_t* base, size_t idx) {
  constexpr int W = FWords<F>::W;
  const uint32_t* p = base + idx * (4 * W);
  Xyzz<F> r;
  load_f(p, r.x);
  load_f(p + W, r.y);
  load_f(p + 2 * W, r.zz);
  load_f(p + 3 * W, r.zzz);
  return r;
}

template <class F>
ZDEV void store_xyzz(uint32_t* base, size_t idx, const Xyzz<F>& a) {
  constexpr int W = FWords<F>::W;
  uint32_t* p = base + idx * (4 * W);
  store_f(p, acc_xcanon(a.x));  // a G1 accumulator x may be < 8m
  store_f(p + W, a.y);
  store_f(p + 2 * W, a.zz);
  store_f(p + 3 * W, a.zzz);
}

}  // namespace zkp
