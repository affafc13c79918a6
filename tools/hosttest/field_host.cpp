// Host-side check of the device field/curve code (field.hpp, curve.hpp are
// __host__ __device__): reads ops from stdin, prints results, compared by
// tools/hosttest/check_field.py against the Python oracle.
#include <cstdio>
#include <cstring>
#include <string>
#include "../../zk-p2p-onramp_amd/csrc/curve.hpp"
using namespace zkp;

static void rd(uint32_t w[8]) { for (int i = 0; i < 8; ++i) if (scanf("%x", &w[i]) != 1) exit(1); }
static void pr(const uint32_t w[8]) { for (int i = 0; i < 8; ++i) printf("%08x ", w[i]); }
template <class C> static Fe<C> rdf() { uint32_t w[8]; rd(w); return unpack<C>(w); }
template <class C> static void prf(const Fe<C>& x) { uint32_t w[8]; pack(x, w); pr(w); }
// 9 hex 29-bit limbs (values up to 2^261, e.g. a Shoup quotient)
template <class C> static Fe<C> rdl() { Fe<C> x; for (int i = 0; i < NL; ++i) if (scanf("%x", &x.v[i]) != 1) exit(1); return x; }

int main() {
  char op[32];
  while (scanf("%31s", op) == 1) {
    std::string o(op);
    if (o == "mulq") { Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(); prf(mul(a, b)); }
    else if (o == "sqrq") { Fq a = rdf<FqCfg>(); prf(sqr(a)); }
    else if (o == "addq") { Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(); prf(add(a, b)); }
    else if (o == "subq") { Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(); prf(sub(a, b)); }
    else if (o == "lsubmulq") { Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(), c = rdf<FqCfg>(); prf(mul(lsub(a, b), c)); }
    else if (o == "lsubsqrq") { Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(); prf(sqr(lsub(a, b))); }
    else if (o == "rsubmulq") { Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(), c = rdf<FqCfg>(); prf(mul(c, rsub(a, b))); }
    else if (o == "rsubmulr") { Fr a = rdf<FrCfg>(), b = rdf<FrCfg>(), c = rdf<FrCfg>(); prf(mul(rsub(a, b), c)); }
    else if (o == "sub2xq") { Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(), c = rdf<FqCfg>(); prf(sub_2x(a, b, c)); }
    else if (o == "sub2xr") { Fr a = rdf<FrCfg>(), b = rdf<FrCfg>(), c = rdf<FrCfg>(); prf(sub_2x(a, b, c)); }
    else if (o == "mul2q") { Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(), c = rdf<FqCfg>(), d = rdf<FqCfg>(); prf(mul2(a, b, c, d)); }
    else if (o == "mul2f2") {  // Fq2: (a0+a1 u)(b0+b1 u) + (c0+c1 u)(d0+d1 u); prints c0 then c1
      Fq2 a{rdf<FqCfg>(), rdf<FqCfg>()}, b{rdf<FqCfg>(), rdf<FqCfg>()}, c{rdf<FqCfg>(), rdf<FqCfg>()}, d{rdf<FqCfg>(), rdf<FqCfg>()};
      Fq2 r = mul2(a, b, c, d); prf(r.c0); printf("\n"); prf(r.c1);
    }
    else if (o == "mulf2") {  // Fq2 (a0+a1 u)(b0+b1 u); prints c0 then c1
      Fq2 a{rdf<FqCfg>(), rdf<FqCfg>()}, b{rdf<FqCfg>(), rdf<FqCfg>()};
      Fq2 r = mul(a, b); prf(r.c0); printf("\n"); prf(r.c1);
    }
    else if (o == "r4r") {  // NTT lazy radix-4 stage pair: raw sums x0+x2, x1+x3; prints s02+s13, (s02-s13) w
      Fr x0 = rdf<FrCfg>(), x1 = rdf<FrCfg>(), x2 = rdf<FrCfg>(), x3 = rdf<FrCfg>(), w = rdf<FrCfg>();
      const Fr s02 = add_raw(x0, x2), s13 = add_raw(x1, x3);
      prf(add_raw_reduce(s02, s13)); printf("\n"); prf(mul(sub_raw6(s02, s13), w));
    }
    else if (o == "r4lazy") {  // round-5 NTT unit forms (ntt.hip r4_unit): x0..x3 < 3m normalised,
      // w plain root (words) with its Shoup quotient wq (limbs), tw a table value < 2m (words)
      Fr x0 = rdf<FrCfg>(), x1 = rdf<FrCfg>(), x2 = rdf<FrCfg>(), x3 = rdf<FrCfg>(), w = rdf<FrCfg>();
      Fr wq = rdl<FrCfg>(), tw = rdf<FrCfg>();
      const Fr s02 = add_raw(x0, x2), s13 = add_raw(x1, x3);
      prf(mul_shoup(sub_raw6n(s02, s13), w, wq)); printf("\n");   // full unit: y1 (< 3m)
      prf(qreduce(sub_raw6n(s02, s13))); printf("\n");            // stored last pair: p1 (< 1.2m)
      prf(mul(add_raw(s02, s13), tw)); printf("\n");              // raw last pair p0 x twiddle (< 2m)
      prf(mul(sub_raw6n(s02, s13), tw)); printf("\n");            // raw p1 x twiddle
      prf(mul(add_raw(x0, x2), tw)); printf("\n");                // raw p2 (d02 + d13, each < 3m)
      prf(mul(rsub(x0, x2), tw)); printf("\n");                   // raw p3 / odd stage x - y + 4m
      // last pair (Hh == 1): d02 = x0 - x2 by the root w^0, only reduced; d13 a Shoup product
      const Fr d02 = qreduce(rsub(x0, x2)), d13 = mul_shoup(rsub(x1, x3), w, wq);
      prf(d02); printf("\n");                                       // < 1.2m
      prf(add(d02, d13)); printf("\n");                             // stored p2
      prf(sub4(d02, d13)); printf("\n");                            // stored p3 (stage_sub)
      prf(mul(add_raw(d02, d13), tw)); printf("\n");               // raw p2 x twiddle
      prf(mul(rsub(d02, d13), tw)); printf("\n");                   // raw p3 x twiddle
      // odd b's first radix-2 stage (span 2^(b-1)): x0 + x1 and (x0 - x1) w
      prf(add(x0, x1)); printf("\n");
      prf(mul_shoup(rsub(x0, x1), w, wq)); printf("\n");
      // raw last-round outputs into the Shoup twiddle / coset-key products (round 5 tables)
      prf(mul_shoup(add_raw(s02, s13), w, wq)); printf("\n");
      prf(mul_shoup(add_raw(x0, x2), w, wq)); printf("\n");
      prf(mul_shoup(add_raw(d02, d13), w, wq)); printf("\n");
      prf(mul_shoup(rsub(d02, d13), w, wq));
    }
    else if (o == "shoupr") {  // a (limbs), w (words, plain), wq (limbs): a w mod r in [0, 3r)
      Fr a = rdl<FrCfg>(), w = rdf<FrCfg>(), wq = rdl<FrCfg>();
      prf(mul_shoup(a, w, wq));
    }
    else if (o == "shoupq") {  // canonical Montgomery wm (words): Shoup quotient as 9 hex limbs
      Fr wm = rdf<FrCfg>();
      Fr q = shoup_quot(wm);
      for (int i = 0; i < NL; ++i) printf("%08x ", q.v[i]);
    }
    else if (o == "sub4r") { Fr a = rdf<FrCfg>(), b = rdf<FrCfg>(); prf(sub4(a, b)); }
    else if (o == "x8q") {  // lazily reduced accumulator x = a - b - 2c (< 8m) and its consumers
      Fq a = rdf<FqCfg>(), b = rdf<FqCfg>(), c = rdf<FqCfg>(), d = rdf<FqCfg>();
      const Fq x = sub_2x8(a, b, c);
      prf(canon8(x)); printf("\n"); prf(mul(x, d)); printf("\n"); prf(sqr(lsub8(d, x))); printf("\n");
      prf(mul2(d, lsub8(d, x), a, rsub(fe_zero<FqCfg>(), b)));
    }
    else if (o == "sqrlazyf2") {  // G2 lazy square, components < 6m (tested < 2^256)
      Fq2 a{rdf<FqCfg>(), rdf<FqCfg>()};
      Fq2 r = sqr_lazy(a); prf(r.c0); printf("\n"); prf(r.c1);
    }
    else if (o == "sub2x4f2") {  // G2 lazy X3 (< 4m per component)
      Fq2 a{rdf<FqCfg>(), rdf<FqCfg>()}, b{rdf<FqCfg>(), rdf<FqCfg>()}, c{rdf<FqCfg>(), rdf<FqCfg>()};
      Fq2 r = sub_2x4(a, b, c); prf(r.c0); printf("\n"); prf(r.c1);
    }
    else if (o == "y3f2") {  // G2 Y3 sum of products t r + d y with t < 6m, r < 4m, d <= 2m, y < 2m
      Fq2 t{rdf<FqCfg>(), rdf<FqCfg>()}, r{rdf<FqCfg>(), rdf<FqCfg>()}, d{rdf<FqCfg>(), rdf<FqCfg>()},
          y{rdf<FqCfg>(), rdf<FqCfg>()};
      Fq2 v = acc_y3(r, t, y, d); prf(v.c0); printf("\n"); prf(v.c1);
    }
    else if (o == "addr") { Fr a = rdf<FrCfg>(), b = rdf<FrCfg>(); prf(add(a, b)); }
    else if (o == "subr") { Fr a = rdf<FrCfg>(), b = rdf<FrCfg>(); prf(sub(a, b)); }
    else if (o == "qredq") { Fq a = rdf<FqCfg>(); prf(qreduce(a)); }
    else if (o == "mulr") { Fr a = rdf<FrCfg>(), b = rdf<FrCfg>(); prf(mul(a, b)); }
    else if (o == "canonq") { Fq a = rdf<FqCfg>(); prf(canon(a)); }
    else if (o == "iszq") { Fq a = rdf<FqCfg>(); printf("%d", (int)is_zero(a)); }
    else if (o == "conv") { Fq a = rdf<FqCfg>(); prf(mul(a, fe_const<FqCfg>(Conv::FQ_ZKEY_TO_DEV))); }
    else if (o == "g1add") {  // acc(affine) + q(affine) via xyzz, output xyzz packed
      Aff<Fq> p{rdf<FqCfg>(), rdf<FqCfg>()}, q{rdf<FqCfg>(), rdf<FqCfg>()};
      Xyzz<Fq> acc = xyzz_inf<Fq>();
      xyzz_add_aff(acc, p);
      xyzz_add_aff(acc, q);
      prf(acc_xcanon(acc.x)); prf(acc.y); prf(acc.zz); prf(acc.zzz);
    } else if (o == "g1addx") {  // xyzz + xyzz
      Aff<Fq> p{rdf<FqCfg>(), rdf<FqCfg>()}, q{rdf<FqCfg>(), rdf<FqCfg>()};
      Xyzz<Fq> a = xyzz_inf<Fq>(), b = xyzz_inf<Fq>();
      xyzz_add_aff(a, p); xyzz_add_aff(b, q);
      b = xyzz_dbl(b);
      xyzz_add(a, b);
      prf(acc_xcanon(a.x)); prf(a.y); prf(a.zz); prf(a.zzz);
    }
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
