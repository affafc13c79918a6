// Host-side BN254 optimal-ate pairing and Groth16 verification (see host_pairing.hpp).
#include "host_pairing.hpp"

#include <vector>

namespace zkp {
namespace host {

namespace {

// ---------------------------------------------------------------- Fq2 helpers
Fq2 f2_muls(const Fq2& a, const Fq& k) { return Fq2{a.c0 * k, a.c1 * k}; }
Fq2 f2_conj(const Fq2& a) { return Fq2{a.c0, a.c1.neg()}; }
Fq2 f2_mul_xi(const Fq2& a) {  // (a0 + a1 u)(9 + u) = (9 a0 - a1) + (a0 + 9 a1) u
  auto nine = [](const Fq& x) {
    Fq x2 = x + x, x4 = x2 + x2, x8 = x4 + x4;
    return x8 + x;
  };
  return Fq2{nine(a.c0) - a.c1, a.c0 + nine(a.c1)};
}
Fq2 f2_pow(Fq2 b, const U256& e) {
  Fq2 r = Fq2::one();
  for (int i = 0; i < 256; ++i) {
    if ((e.w[i >> 6] >> (i & 63)) & 1) r = r * b;
    b = b.sqr();
  }
  return r;
}
Fq fq_small(uint64_t v) { return Fq::from_std(U256{{v, 0, 0, 0}}); }

// ---------------------------------------------------------------- Fq6
Fq6 f6_add(const Fq6& a, const Fq6& b) { return Fq6{a.c0 + b.c0, a.c1 + b.c1, a.c2 + b.c2}; }
Fq6 f6_sub(const Fq6& a, const Fq6& b) { return Fq6{a.c0 - b.c0, a.c1 - b.c1, a.c2 - b.c2}; }
Fq6 f6_neg(const Fq6& a) { return Fq6{a.c0.neg(), a.c1.neg(), a.c2.neg()}; }
Fq6 f6_zero() { return Fq6{Fq2::zero(), Fq2::zero(), Fq2::zero()}; }
Fq6 f6_mul(const Fq6& a, const Fq6& b) {
  const Fq2 t0 = a.c0 * b.c0, t1 = a.c1 * b.c1, t2 = a.c2 * b.c2;
  const Fq2 c0 = t0 + f2_mul_xi((a.c1 + a.c2) * (b.c1 + b.c2) - t1 - t2);
  const Fq2 c1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1 + f2_mul_xi(t2);
  const Fq2 c2 = (a.c0 + a.c2) * (b.c0 + b.c2) - t0 - t2 + t1;
  return Fq6{c0, c1, c2};
}
Fq6 f6_mul_v(const Fq6& a) { return Fq6{f2_mul_xi(a.c2), a.c0, a.c1}; }  // (a0 + a1 v + a2 v^2) v
Fq6 f6_muls(const Fq6& a, const Fq& k) { return Fq6{f2_muls(a.c0, k), f2_muls(a.c1, k), f2_muls(a.c2, k)}; }
// (a0 + a1 v + a2 v^2)(b0 + b1 v)
Fq6 f6_mul_01(const Fq6& a, const Fq2& b0, const Fq2& b1) {
  return Fq6{a.c0 * b0 + f2_mul_xi(a.c2 * b1), a.c0 * b1 + a.c1 * b0, a.c1 * b1 + a.c2 * b0};
}
Fq6 f6_inv(const Fq6& a) {
  const Fq2 c0 = a.c0.sqr() - f2_mul_xi(a.c1 * a.c2);
  const Fq2 c1 = f2_mul_xi(a.c2.sqr()) - a.c0 * a.c1;
  const Fq2 c2 = a.c1.sqr() - a.c0 * a.c2;
  const Fq2 t = a.c0 * c0 + f2_mul_xi(a.c2 * c1 + a.c1 * c2);
  const Fq2 ti = t.inv();
  return Fq6{c0 * ti, c1 * ti, c2 * ti};
}

// ---------------------------------------------------------------- Fq12
Fq12 f12_conj(const Fq12& a) { return Fq12{a.c0, f6_neg(a.c1)}; }
Fq12 f12_sqr(const Fq12& a) { return fq12_mul(a, a); }
Fq12 f12_inv(const Fq12& a) {
  const Fq6 t = f6_inv(f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1))));
  return Fq12{f6_mul(a.c0, t), f6_neg(f6_mul(a.c1, t))};
}

// Frobenius x -> x^p: the coefficient of w^i (basis 1, w, w^2 = v, w^3, w^4 = v^2, w^5) becomes
// conj(coefficient) * xi^(i (p - 1) / 6)
struct FrobConsts {
  Fq2 g[6];
  Fq2 b2;  // 3 / (9 + u), the twist's b
  Fq2 gx, gy;  // xi^((p-1)/3), xi^((p-1)/2): the G2 Frobenius pi(x, y) = (conj(x) gx, conj(y) gy)
  FrobConsts() {
    const Fq2 xi{fq_small(9), fq_small(1)};
    U256 e = FQ_DESC.mod, one{{1, 0, 0, 0}};
    u256_sub(e, one);  // p - 1, divisible by 6
    U256 e6 = e, e3 = e, e2 = e;
    auto div_small = [](U256& x, uint64_t d) {
      u128 rem = 0;
      for (int i = 3; i >= 0; --i) {
        const u128 cur = (rem << 64) | x.w[i];
        x.w[i] = (u64)(cur / d);
        rem = cur % d;
      }
    };
    div_small(e6, 6);
    div_small(e3, 3);
    div_small(e2, 2);
    g[0] = Fq2::one();
    g[1] = f2_pow(xi, e6);
    for (int i = 2; i < 6; ++i) g[i] = g[i - 1] * g[1];
    b2 = Fq2{fq_small(3), Fq::zero()} * xi.inv();
    gx = f2_pow(xi, e3);
    gy = f2_pow(xi, e2);
  }
};
const FrobConsts& fc() {
  static const FrobConsts c;
  return c;
}
Fq12 f12_frob(const Fq12& a) {
  const Fq2* g = fc().g;
  return Fq12{Fq6{f2_conj(a.c0.c0), f2_conj(a.c0.c1) * g[2], f2_conj(a.c0.c2) * g[4]},
              Fq6{f2_conj(a.c1.c0) * g[1], f2_conj(a.c1.c1) * g[3], f2_conj(a.c1.c2) * g[5]}};
}
Fq12 f12_frob_k(Fq12 a, int k) {
  for (int i = 0; i < k; ++i) a = f12_frob(a);
  return a;
}
// a^x, x = u = 4965661367192848881 (the BN parameter)
Fq12 f12_pow_u(const Fq12& a) {
  const uint64_t u = 4965661367192848881ull;
  Fq12 r = fq12_one();
  for (int i = 63; i >= 0; --i) {
    r = f12_sqr(r);
    if ((u >> i) & 1) r = fq12_mul(r, a);
  }
  return r;
}

// f * l for a line l = (yP, 0, 0) + (B0, B1, 0) w  (yP in Fq)
Fq12 f12_mul_line(const Fq12& f, const Fq& yp, const Fq2& b0, const Fq2& b1) {
  const Fq6 t0 = f6_muls(f.c0, yp);         // f0 L0
  const Fq6 t1 = f6_mul_01(f.c1, b0, b1);   // f1 L1
  const Fq6 c1 = f6_add(f6_mul_01(f.c0, b0, b1), f6_muls(f.c1, yp));
  return Fq12{f6_add(t0, f6_mul_v(t1)), c1};
}

}  // namespace

Fq12 fq12_one() { return Fq12{Fq6{Fq2::one(), Fq2::zero(), Fq2::zero()}, f6_zero()}; }

Fq12 fq12_mul(const Fq12& a, const Fq12& b) {
  const Fq6 t0 = f6_mul(a.c0, b.c0), t1 = f6_mul(a.c1, b.c1);
  return Fq12{f6_add(t0, f6_mul_v(t1)), f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), f6_add(t0, t1))};
}

bool fq12_is_one(const Fq12& a) {
  const Fq12 o = fq12_one();
  return a.c0.c0 == o.c0.c0 && a.c0.c1.is_zero() && a.c0.c2.is_zero() && a.c1.c0.is_zero() && a.c1.c1.is_zero() &&
         a.c1.c2.is_zero();
}

// Miller loop of every pair at once: the line of pair i through T_i (slope lam, evaluated at P_i,
// untwisted): yP - lam xP w + (lam xT - yT) w^3  (w^3 = v w)
Fq12 miller_loop_multi(const Affine<Fq>* ps, const Affine<Fq2>* qs, int n) {
  const uint64_t ate_lo = 0x9d797039be763ba8ull;  // 6u + 2 = 29793968203157093288 = 2^64 + ate_lo (65 bits)
  std::vector<int> idx;
  for (int i = 0; i < n; ++i)
    if (!ps[i].inf && !qs[i].inf) idx.push_back(i);
  const int m = (int)idx.size();
  Fq12 f = fq12_one();
  if (m == 0) return f;
  std::vector<Fq2> tx(m), ty(m), den(m), pre(m);
  for (int k = 0; k < m; ++k) tx[k] = qs[idx[k]].x, ty[k] = qs[idx[k]].y;
  // den[k] <- 1 / den[k] for every k with one inversion (Montgomery's trick)
  auto batch_inv = [&](std::vector<Fq2>& d) {
    Fq2 acc = Fq2::one();
    for (int k = 0; k < m; ++k) pre[k] = acc, acc = acc * d[k];
    Fq2 inv = acc.inv();
    for (int k = m - 1; k >= 0; --k) {
      const Fq2 dk = d[k];
      d[k] = inv * pre[k];
      inv = inv * dk;
    }
  };
  const Fq three = fq_small(3);
  auto dbl_step = [&] {
    for (int k = 0; k < m; ++k) den[k] = ty[k] + ty[k];
    batch_inv(den);
    for (int k = 0; k < m; ++k) {
      const Fq2 l = f2_muls(tx[k].sqr(), three) * den[k];
      const Affine<Fq>& p = ps[idx[k]];
      f = f12_mul_line(f, p.y, f2_muls(l, p.x).neg(), l * tx[k] - ty[k]);
      const Fq2 x3 = l.sqr() - tx[k] - tx[k];
      ty[k] = l * (tx[k] - x3) - ty[k];
      tx[k] = x3;
    }
  };
  auto add_step = [&](const std::vector<Affine<Fq2>>& q) {
    for (int k = 0; k < m; ++k) den[k] = q[k].x - tx[k];
    batch_inv(den);
    for (int k = 0; k < m; ++k) {
      const Fq2 l = (q[k].y - ty[k]) * den[k];
      const Affine<Fq>& p = ps[idx[k]];
      f = f12_mul_line(f, p.y, f2_muls(l, p.x).neg(), l * tx[k] - ty[k]);
      const Fq2 x3 = l.sqr() - tx[k] - q[k].x;
      ty[k] = l * (tx[k] - x3) - ty[k];
      tx[k] = x3;
    }
  };
  std::vector<Affine<Fq2>> q0(m), q1(m), q2(m);
  for (int k = 0; k < m; ++k) q0[k] = qs[idx[k]];
  for (int bit = 63; bit >= 0; --bit) {  // bits 63..0 of 6u + 2 (bit 64, the top, is the start T = Q)
    f = f12_sqr(f);
    dbl_step();
    if ((ate_lo >> bit) & 1) add_step(q0);
  }
  // T = (6u + 2) Q; the correction lines through pi(Q) and -pi^2(Q)
  const FrobConsts& c = fc();
  for (int k = 0; k < m; ++k) {
    const Affine<Fq2>& q = q0[k];
    q1[k] = Affine<Fq2>{f2_conj(q.x) * c.gx, f2_conj(q.y) * c.gy, false};
    const Affine<Fq2>& r = q1[k];
    q2[k] = Affine<Fq2>{f2_conj(r.x) * c.gx, (f2_conj(r.y) * c.gy).neg(), false};
  }
  add_step(q1);
  add_step(q2);
  return f;
}

// easy part f^((p^6 - 1)(p^2 + 1)); hard part as ffjavascript (Fuentes-Castaneda et al., "Faster
// hashing to G2"): the reduced pairing raised to 2u (6u^2 + 3u + 1), the value snarkjs reports
Fq12 final_exponentiation(const Fq12& f) {
  Fq12 r = fq12_mul(f12_conj(f), f12_inv(f));
  r = fq12_mul(f12_frob_k(r, 2), r);
  // r is now unitary: its inverse is its conjugate
  const Fq12 y0 = f12_conj(f12_pow_u(r));
  const Fq12 y1 = f12_sqr(y0);
  const Fq12 y2 = f12_sqr(y1);
  Fq12 y3 = fq12_mul(y2, y1);
  const Fq12 y4 = f12_conj(f12_pow_u(y3));
  const Fq12 y5 = f12_sqr(y4);
  Fq12 y6 = f12_conj(f12_pow_u(y5));
  y3 = f12_conj(y3);
  y6 = f12_conj(y6);
  const Fq12 y7 = fq12_mul(y6, y4);
  Fq12 y8 = fq12_mul(y7, y3);
  const Fq12 y9 = fq12_mul(y8, y1);
  const Fq12 y10 = fq12_mul(y8, y4);
  const Fq12 y11 = fq12_mul(y10, r);
  const Fq12 y13 = fq12_mul(f12_frob_k(y9, 1), y11);
  y8 = f12_frob_k(y8, 2);
  const Fq12 y14 = fq12_mul(y8, y13);
  const Fq12 y15 = f12_frob_k(fq12_mul(f12_conj(r), y9), 3);
  return fq12_mul(y15, y14);
}

Fq12 pairing(const Affine<Fq>& p, const Affine<Fq2>& q) { return final_exponentiation(miller_loop_multi(&p, &q, 1)); }

bool g1_on_curve(const Affine<Fq>& p) {
  if (p.inf) return true;
  return p.y.sqr() == p.x.sqr() * p.x + fq_small(3);
}

bool g2_on_curve(const Affine<Fq2>& p) {
  if (p.inf) return true;
  return p.y.sqr() == p.x.sqr() * p.x + fc().b2;
}

bool g2_in_subgroup(const Affine<Fq2>& p) {
  if (p.inf) return true;
  return jac_mul(jac_from_aff(p), FR_DESC.mod).is_inf();
}

bool groth16_verify(const VerifyingKey& vk, const U256* pub, const Affine<Fq>& a, const Affine<Fq2>& b,
                    const Affine<Fq>& c) {
  for (int i = 0; i < vk.n_public; ++i)
    if (u256_geq(pub[i], FR_DESC.mod)) return false;  // Verifier.sol:347 "verifier-gte-snark-scalar-field"
  if (!g1_on_curve(a) || !g1_on_curve(c) || !g2_on_curve(b) || !g2_in_subgroup(b)) return false;
  // vk_x = IC[0] + sum in_i IC[i+1]: Straus with 4-bit windows (shared doublings)
  const int np = vk.n_public;
  std::vector<Jac<Fq>> tab((size_t)np * 16);
  for (int i = 0; i < np; ++i) {
    Jac<Fq>* t = &tab[(size_t)i * 16];
    t[0] = Jac<Fq>::inf();
    t[1] = jac_from_aff(vk.ic[i + 1]);
    for (int d = 2; d < 16; ++d) t[d] = jac_add(t[d - 1], t[1]);
  }
  Jac<Fq> acc = Jac<Fq>::inf();
  for (int win = 63; win >= 0; --win) {
    for (int s = 0; s < 4; ++s) acc = jac_dbl(acc);
    for (int i = 0; i < np; ++i) {
      const unsigned d = (unsigned)(pub[i].w[win >> 4] >> ((win & 15) * 4)) & 15u;
      if (d) acc = jac_add(acc, tab[(size_t)i * 16 + d]);
    }
  }
  acc = jac_add(acc, jac_from_aff(vk.ic[0]));
  const Affine<Fq> vkx = jac_to_aff(acc);
  Affine<Fq> na = a;
  if (!na.inf) na.y = na.y.neg();
  const Affine<Fq> ps[4] = {na, vk.alpha1, vkx, c};
  const Affine<Fq2> qs[4] = {b, vk.beta2, vk.gamma2, vk.delta2};
  return fq12_is_one(final_exponentiation(miller_loop_multi(ps, qs, 4)));
}

}  // namespace host
}  // namespace zkp
