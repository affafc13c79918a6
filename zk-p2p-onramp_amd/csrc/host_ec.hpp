// Host-side BN254 arithmetic used by the prover for the O(1) tail of a proof:
// folding MSM window sums (Horner), r/s blinding, affine conversion and the
// final proof assembly (snarkjs groth16_prove "blinding + assembly", SURVEY.md
// §8a row A10).  4 x 64-bit limbs, Montgomery radix 2^256 (as wasmcurves).
// Not on the throughput path: a proof needs a few hundred group operations here.
#pragma once
#include <cstdint>
#include <cstring>
#include <string>

namespace zkp {
namespace host {

using u64 = uint64_t;
using u128 = unsigned __int128;

struct U256 {
  u64 w[4];
};

inline bool u256_geq(const U256& a, const U256& b) {
  for (int i = 3; i >= 0; --i)
    if (a.w[i] != b.w[i]) return a.w[i] > b.w[i];
  return true;
}

inline u64 u256_sub(U256& a, const U256& b) {  // a -= b, returns borrow
  u64 br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 d = (u128)a.w[i] - b.w[i] - br;
    a.w[i] = (u64)d;
    br = (u64)(d >> 127);
  }
  return br;
}

inline u64 u256_add(U256& a, const U256& b) {
  u64 c = 0;
  for (int i = 0; i < 4; ++i) {
    u128 s = (u128)a.w[i] + b.w[i] + c;
    a.w[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  return c;
}

inline bool u256_is_zero(const U256& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0; }

struct FieldDesc {
  U256 mod;
  u64 inv;  // -mod^-1 mod 2^64
  U256 r2;  // 2^512 mod m
};

extern const FieldDesc FQ_DESC;
extern const FieldDesc FR_DESC;

template <const FieldDesc& D>
struct Fp {
  U256 v;  // Montgomery form, canonical (< m)

  static Fp zero() { return Fp{{{0, 0, 0, 0}}}; }
  static Fp raw(const U256& x) { return Fp{x}; }
  static Fp mont_mul(const U256& a, const U256& b) {
    u64 t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
      u64 c = 0;
      for (int j = 0; j < 4; ++j) {
        u128 s = (u128)a.w[j] * b.w[i] + t[j] + c;
        t[j] = (u64)s;
        c = (u64)(s >> 64);
      }
      u128 s = (u128)t[4] + c;
      t[4] = (u64)s;
      t[5] = (u64)(s >> 64);
      u64 m = t[0] * D.inv;
      u128 s0 = (u128)m * D.mod.w[0] + t[0];
      c = (u64)(s0 >> 64);
      for (int j = 1; j < 4; ++j) {
        u128 s1 = (u128)m * D.mod.w[j] + t[j] + c;
        t[j - 1] = (u64)s1;
        c = (u64)(s1 >> 64);
      }
      u128 s2 = (u128)t[4] + c;
      t[3] = (u64)s2;
      t[4] = t[5] + (u64)(s2 >> 64);
    }
    Fp r{{{t[0], t[1], t[2], t[3]}}};
    if (t[4] || u256_geq(r.v, D.mod)) u256_sub(r.v, D.mod);
    return r;
  }
  static Fp from_std(const U256& x) {  // x < m
    return mont_mul(x, D.r2);
  }
  static Fp one() {
    U256 o{{1, 0, 0, 0}};
    return from_std(o);
  }
  U256 to_std() const {
    U256 o{{1, 0, 0, 0}};
    return mont_mul(v, o).v;
  }
  Fp operator*(const Fp& b) const { return mont_mul(v, b.v); }
  Fp operator+(const Fp& b) const {
    Fp r = *this;
    u64 c = u256_add(r.v, b.v);
    if (c || u256_geq(r.v, D.mod)) u256_sub(r.v, D.mod);
    return r;
  }
  Fp operator-(const Fp& b) const {
    Fp r = *this;
    if (u256_sub(r.v, b.v)) u256_add(r.v, D.mod);
    return r;
  }
  Fp neg() const { return zero() - *this; }
  Fp sqr() const { return *this * *this; }
  bool is_zero() const { return u256_is_zero(v); }
  bool operator==(const Fp& b) const { return std::memcmp(v.w, b.v.w, 32) == 0; }
  Fp pow(const U256& e) const {
    Fp r = one(), b = *this;
    for (int i = 0; i < 256; ++i) {
      if ((e.w[i >> 6] >> (i & 63)) & 1) r = r * b;
      b = b.sqr();
    }
    return r;
  }
  Fp inv() const {  // Fermat; 0 -> 0
    U256 e = D.mod;
    U256 two{{2, 0, 0, 0}};
    u256_sub(e, two);
    return pow(e);
  }
};

using Fq = Fp<FQ_DESC>;
using Fr = Fp<FR_DESC>;

struct Fq2 {
  Fq c0, c1;
  static Fq2 zero() { return Fq2{Fq::zero(), Fq::zero()}; }
  static Fq2 one() { return Fq2{Fq::one(), Fq::zero()}; }
  Fq2 operator+(const Fq2& b) const { return Fq2{c0 + b.c0, c1 + b.c1}; }
  Fq2 operator-(const Fq2& b) const { return Fq2{c0 - b.c0, c1 - b.c1}; }
  Fq2 operator*(const Fq2& b) const {
    Fq t0 = c0 * b.c0, t1 = c1 * b.c1;
    return Fq2{t0 - t1, (c0 + c1) * (b.c0 + b.c1) - t0 - t1};
  }
  Fq2 sqr() const { return *this * *this; }
  Fq2 neg() const { return Fq2{c0.neg(), c1.neg()}; }
  bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  bool operator==(const Fq2& b) const { return c0 == b.c0 && c1 == b.c1; }
  Fq2 inv() const {
    Fq t = (c0.sqr() + c1.sqr()).inv();
    return Fq2{c0 * t, (c1 * t).neg()};
  }
};

// Jacobian point (x = X/Z^2, y = Y/Z^3), Z == 0 is infinity.
template <class F>
struct Jac {
  F X, Y, Z;
  static Jac inf() { return Jac{F::one(), F::one(), F::zero()}; }
  bool is_inf() const { return Z.is_zero(); }
};

template <class F>
struct Affine {
  F x, y;
  bool inf;
};

template <class F>
Jac<F> jac_dbl(const Jac<F>& p) {
  if (p.is_inf() || p.Y.is_zero()) return Jac<F>::inf();
  F A = p.X.sqr(), B = p.Y.sqr(), C = B.sqr();
  F t = (p.X + B).sqr() - A - C;
  F D = t + t;
  F E = A + A + A;
  F Fv = E.sqr();
  Jac<F> r;
  r.X = Fv - D - D;
  F C8 = C + C;
  C8 = C8 + C8;
  C8 = C8 + C8;
  r.Y = E * (D - r.X) - C8;
  F yz = p.Y * p.Z;
  r.Z = yz + yz;
  return r;
}

template <class F>
Jac<F> jac_add(const Jac<F>& p, const Jac<F>& q) {
  if (p.is_inf()) return q;
  if (q.is_inf()) return p;
  F Z1Z1 = p.Z.sqr(), Z2Z2 = q.Z.sqr();
  F U1 = p.X * Z2Z2, U2 = q.X * Z1Z1;
  F S1 = p.Y * q.Z * Z2Z2, S2 = q.Y * p.Z * Z1Z1;
  if (U1 == U2) {
    if (S1 == S2) return jac_dbl(p);
    return Jac<F>::inf();
  }
  F H = U2 - U1;
  F I = (H + H).sqr();
  F J = H * I;
  F rr = S2 - S1;
  rr = rr + rr;
  F V = U1 * I;
  Jac<F> r;
  r.X = rr.sqr() - J - V - V;
  F sj = S1 * J;
  r.Y = rr * (V - r.X) - sj - sj;
  r.Z = ((p.Z + q.Z).sqr() - Z1Z1 - Z2Z2) * H;
  return r;
}

template <class F>
Jac<F> jac_from_aff(const Affine<F>& a) {
  if (a.inf) return Jac<F>::inf();
  return Jac<F>{a.x, a.y, F::one()};
}

template <class F>
Affine<F> jac_to_aff(const Jac<F>& p) {
  if (p.is_inf()) return Affine<F>{F::zero(), F::zero(), true};
  F zi = p.Z.inv();
  F zi2 = zi.sqr();
  return Affine<F>{p.X * zi2, p.Y * zi2 * zi, false};
}

// k * P for a 256-bit standard-form scalar k (LE words)
template <class F>
Jac<F> jac_mul(const Jac<F>& p, const U256& k) {
  Jac<F> acc = Jac<F>::inf();
  for (int i = 255; i >= 0; --i) {
    acc = jac_dbl(acc);
    if ((k.w[i >> 6] >> (i & 63)) & 1) acc = jac_add(acc, p);
  }
  return acc;
}

// XYZZ (device partial-sum format) -> Jacobian: X' = X*ZZ, Y' = Y*ZZ*ZZZ... using
// x = X/ZZ, y = Y/ZZZ: take Z = ZZZ/ZZ, then X_j = x Z^2, Y_j = y Z^3.
template <class F>
Jac<F> jac_from_xyzz(const F& X, const F& Y, const F& ZZ, const F& ZZZ) {
  if (ZZ.is_zero()) return Jac<F>::inf();
  // Z = ZZZ * ZZ^-1 would need an inversion; instead use Z = ZZZ*ZZ:
  //   x = X/ZZ = (X*ZZ*ZZZ^2)/(ZZ*ZZZ)^2,  y = Y/ZZZ = (Y*ZZ^3*ZZZ^2)/(ZZ*ZZZ)^3
  F Z = ZZ * ZZZ;
  F ZZZ2 = ZZZ.sqr();
  Jac<F> r;
  r.X = X * ZZ * ZZZ2;
  r.Y = Y * ZZ.sqr() * ZZ * ZZZ2;
  r.Z = Z;
  return r;
}

// ---- byte / device-layout conversions
U256 u256_from_le(const uint8_t* p);
void u256_to_le(const U256& x, uint8_t* p);
// device layout: 8 LE 32-bit words holding x*2^261 mod m (value < 2m)
Fq fq_from_dev(const uint32_t* w);
Fr fr_from_dev(const uint32_t* w);
std::string u256_to_dec(const U256& x);

}  // namespace host
}  // namespace zkp
