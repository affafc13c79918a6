// Multithreaded CPU restatement of snarkjs 0.4.22 groth16_prove — TEST
// INFRASTRUCTURE ONLY (see oracle/__init__.py).  Used (a) as the checker for
// large-size GPU parity (full Venmo-shaped proofs are too big for the Python
// oracle) and (b) as bench.py's cpu_baseline ("port": the reference's own CPU
// prover, snarkjs/ffjavascript/rapidsnark, is absent offline — SURVEY.md §8c C1).
//
// Independent of the product code: own 4 x 64-bit Montgomery arithmetic
// (R = 2^256, as wasmcurves), Jacobian points, radix-2 NTT, per-window Pippenger.
// Algorithm restated from SURVEY.md §8a rows A1-A10:
//   buildABC1 -> for X in {A,B,C}: ifft, batchApplyKey(1, Fr.w[k+1]), fft ->
//   joinABC (A*B - C, from Montgomery) -> 4 G1 + 1 G2 multiExp -> blinding.
// Build: make -C oracle   (g++ only; no GPU code).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

typedef unsigned __int128 u128;
typedef uint64_t u64;

struct Mod {
  u64 m[4];
  u64 inv;   // -m^-1 mod 2^64
  u64 r2[4]; // 2^512 mod m
};
// p (Verifier.sol:52), r (Verifier.sol:341)
const Mod MP = {{0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
                0x87d20782e4866389ull,
                {0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull, 0x47ab1eff0a417ff6ull, 0x06d89f71cab8351full}};
const Mod MR = {{0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
                0xc2e1f593efffffffull,
                {0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull, 0x8c49833d53bb8085ull, 0x0216d0b17f4e44a5ull}};

template <const Mod& M>
struct F {
  u64 v[4];
  static F zero() { return F{{0, 0, 0, 0}}; }
  static bool geq(const u64* a, const u64* b) {
    for (int i = 3; i >= 0; --i)
      if (a[i] != b[i]) return a[i] > b[i];
    return true;
  }
  static void subm(u64* a, const u64* b) {
    u64 br = 0;
    for (int i = 0; i < 4; ++i) {
      u128 d = (u128)a[i] - b[i] - br;
      a[i] = (u64)d;
      br = (u64)(d >> 64) & 1;
    }
  }
  friend F operator*(const F& a, const F& b) {
    u64 t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) {
      u64 c = 0;
      for (int j = 0; j < 4; ++j) {
        u128 s = (u128)a.v[j] * b.v[i] + t[j] + c;
        t[j] = (u64)s;
        c = (u64)(s >> 64);
      }
      u128 s = (u128)t[4] + c;
      t[4] = (u64)s;
      t[5] = (u64)(s >> 64);
      const u64 m = t[0] * M.inv;
      u128 s0 = (u128)m * M.m[0] + t[0];
      c = (u64)(s0 >> 64);
      for (int j = 1; j < 4; ++j) {
        u128 s1 = (u128)m * M.m[j] + t[j] + c;
        t[j - 1] = (u64)s1;
        c = (u64)(s1 >> 64);
      }
      u128 s2 = (u128)t[4] + c;
      t[3] = (u64)s2;
      t[4] = t[5] + (u64)(s2 >> 64);
    }
    F r{{t[0], t[1], t[2], t[3]}};
    if (t[4] || geq(r.v, M.m)) subm(r.v, M.m);
    return r;
  }
  friend F operator+(const F& a, const F& b) {
    F r;
    u64 c = 0;
    for (int i = 0; i < 4; ++i) {
      u128 s = (u128)a.v[i] + b.v[i] + c;
      r.v[i] = (u64)s;
      c = (u64)(s >> 64);
    }
    if (c || geq(r.v, M.m)) subm(r.v, M.m);
    return r;
  }
  friend F operator-(const F& a, const F& b) {
    F r;
    u64 br = 0;
    for (int i = 0; i < 4; ++i) {
      u128 d = (u128)a.v[i] - b.v[i] - br;
      r.v[i] = (u64)d;
      br = (u64)(d >> 64) & 1;
    }
    if (br) {
      u64 c = 0;
      for (int i = 0; i < 4; ++i) {
        u128 s = (u128)r.v[i] + M.m[i] + c;
        r.v[i] = (u64)s;
        c = (u64)(s >> 64);
      }
    }
    return r;
  }
  bool is_zero() const { return (v[0] | v[1] | v[2] | v[3]) == 0; }
  bool operator==(const F& b) const { return std::memcmp(v, b.v, 32) == 0; }
  static F from_raw(const uint8_t* p) {
    F r;
    std::memcpy(r.v, p, 32);
    return r;
  }
  static F from_std(const F& x) { return x * F{{M.r2[0], M.r2[1], M.r2[2], M.r2[3]}}; }
  F to_std() const { return *this * F{{1, 0, 0, 0}}; }
  static F one() { return from_std(F{{1, 0, 0, 0}}); }
  F pow(const u64* e) const {
    F r = one(), b = *this;
    for (int i = 0; i < 256; ++i) {
      if ((e[i >> 6] >> (i & 63)) & 1) r = r * b;
      b = b * b;
    }
    return r;
  }
  F inv() const {
    u64 e[4] = {M.m[0] - 2, M.m[1], M.m[2], M.m[3]};
    return pow(e);
  }
};
using Fq = F<MP>;
using Fr = F<MR>;

struct Fq2 {
  Fq a, b;
  friend Fq2 operator+(const Fq2& x, const Fq2& y) { return {x.a + y.a, x.b + y.b}; }
  friend Fq2 operator-(const Fq2& x, const Fq2& y) { return {x.a - y.a, x.b - y.b}; }
  friend Fq2 operator*(const Fq2& x, const Fq2& y) {
    Fq t0 = x.a * y.a, t1 = x.b * y.b;
    return {t0 - t1, (x.a + x.b) * (y.a + y.b) - t0 - t1};
  }
  bool is_zero() const { return a.is_zero() && b.is_zero(); }
  bool operator==(const Fq2& y) const { return a == y.a && b == y.b; }
  static Fq2 zero() { return {Fq::zero(), Fq::zero()}; }
  static Fq2 one() { return {Fq::one(), Fq::zero()}; }
  Fq2 inv() const {
    Fq t = (a * a + b * b).inv();
    return {a * t, Fq::zero() - b * t};
  }
};

template <class E>
E ezero();
template <>
Fq ezero<Fq>() { return Fq::zero(); }
template <>
Fq2 ezero<Fq2>() { return Fq2::zero(); }
template <class E>
E eone();
template <>
Fq eone<Fq>() { return Fq::one(); }
template <>
Fq2 eone<Fq2>() { return Fq2::one(); }

// Jacobian points, Z == 0 infinity
template <class E>
struct J {
  E x, y, z;
};
template <class E>
J<E> jinf() { return {eone<E>(), eone<E>(), ezero<E>()}; }

template <class E>
J<E> jdbl(const J<E>& p) {
  if (p.z.is_zero() || p.y.is_zero()) return jinf<E>();
  E A = p.x * p.x, B = p.y * p.y, C = B * B;
  E D = (p.x + B) * (p.x + B) - A - C;
  D = D + D;
  E Ee = A + A + A, Ff = Ee * Ee;
  J<E> r;
  r.x = Ff - D - D;
  E C8 = C + C;
  C8 = C8 + C8;
  C8 = C8 + C8;
  r.y = Ee * (D - r.x) - C8;
  E yz = p.y * p.z;
  r.z = yz + yz;
  return r;
}

template <class E>
J<E> jadd(const J<E>& p, const J<E>& q) {
  if (p.z.is_zero()) return q;
  if (q.z.is_zero()) return p;
  E z1z1 = p.z * p.z, z2z2 = q.z * q.z;
  E u1 = p.x * z2z2, u2 = q.x * z1z1;
  E s1 = p.y * q.z * z2z2, s2 = q.y * p.z * z1z1;
  if (u1 == u2) return s1 == s2 ? jdbl(p) : jinf<E>();
  E h = u2 - u1, i = (h + h) * (h + h), jj = h * i;
  E rr = s2 - s1;
  rr = rr + rr;
  E vv = u1 * i;
  J<E> r;
  r.x = rr * rr - jj - vv - vv;
  E sj = s1 * jj;
  r.y = rr * (vv - r.x) - sj - sj;
  r.z = ((p.z + q.z) * (p.z + q.z) - z1z1 - z2z2) * h;
  return r;
}

// mixed add with affine (x, y) (madd-2007-bl)
template <class E>
J<E> jadd_aff(const J<E>& p, const E& x2, const E& y2) {
  if (p.z.is_zero()) return {x2, y2, eone<E>()};
  E z1z1 = p.z * p.z;
  E u2 = x2 * z1z1, s2 = y2 * p.z * z1z1;
  if (u2 == p.x) return s2 == p.y ? jdbl(p) : jinf<E>();
  E h = u2 - p.x, hh = h * h, i = hh + hh;
  i = i + i;
  E jj = h * i, rr = s2 - p.y;
  rr = rr + rr;
  E vv = p.x * i;
  J<E> r;
  r.x = rr * rr - jj - vv - vv;
  E yj = p.y * jj;
  r.y = rr * (vv - r.x) - yj - yj;
  r.z = (p.z + h) * (p.z + h) - z1z1 - hh;
  return r;
}

template <class E>
J<E> jmul(J<E> p, const Fr& k_std) {
  J<E> acc = jinf<E>();
  for (int i = 255; i >= 0; --i) {
    acc = jdbl(acc);
    if ((k_std.v[i >> 6] >> (i & 63)) & 1) acc = jadd(acc, p);
  }
  return acc;
}

template <class E>
void jaff(const J<E>& p, E& x, E& y, bool& inf) {
  inf = p.z.is_zero();
  if (inf) {
    x = ezero<E>(), y = ezero<E>();
    return;
  }
  E zi = p.z.inv(), zi2 = zi * zi;
  x = p.x * zi2;
  y = p.y * zi2 * zi;
}

template <class Fn>
void par(int threads, size_t n, Fn&& fn) {
  threads = std::max(1, std::min<int>(threads, (int)std::max<size_t>(1, n / 64)));
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) th.emplace_back([&, t] { fn(n * t / threads, n * (t + 1) / threads, t); });
  for (auto& x : th) x.join();
}

// ---------------- MSM: per-window Pippenger, windows spread over threads
template <class E>
J<E> msm(const uint8_t* pts, const uint8_t* sc, size_t n, int threads) {
  constexpr size_t PW = sizeof(E) * 2;  // bytes per affine point (64 / 128)
  int c = 4;
  while (c < 16 && (size_t(1) << (c + 3)) < n) ++c;
  const int W = (256 + c - 1) / c;
  std::vector<J<E>> win(W, jinf<E>());
  std::atomic<int> next{0};
  std::vector<std::thread> th;
  for (int t = 0; t < std::max(1, threads); ++t) {
    th.emplace_back([&] {
      std::vector<J<E>> b(size_t(1) << c);
      for (;;) {
        const int w = next.fetch_add(1);
        if (w >= W) break;
        std::fill(b.begin(), b.end(), jinf<E>());
        for (size_t i = 0; i < n; ++i) {
          u64 s[5];
          std::memcpy(s, sc + 32 * i, 32);
          s[4] = 0;
          const int bit = w * c, word = bit >> 6, sh = bit & 63;
          u64 d = s[word] >> sh;
          if (sh + c > 64) d |= s[word + 1] << (64 - sh);
          d &= (u64(1) << c) - 1;
          if (!d) continue;
          E x, y;
          std::memcpy(&x, pts + PW * i, sizeof(E));
          std::memcpy(&y, pts + PW * i + sizeof(E), sizeof(E));
          if (x.is_zero() && y.is_zero()) continue;
          b[d] = jadd_aff(b[d], x, y);
        }
        J<E> run = jinf<E>(), acc = jinf<E>();
        for (size_t k = b.size() - 1; k >= 1; --k) {
          run = jadd(run, b[k]);
          acc = jadd(acc, run);
        }
        win[w] = acc;
      }
    });
  }
  for (auto& x : th) x.join();
  J<E> r = win[W - 1];
  for (int w = W - 2; w >= 0; --w) {
    for (int i = 0; i < c; ++i) r = jdbl(r);
    r = jadd(r, win[w]);
  }
  return r;
}

// ---------------- NTT (radix-2 DIT, natural in/out), ffjavascript roots
Fr fr_u64(u64 x) { return Fr::from_std(Fr{{x, 0, 0, 0}}); }

Fr root(int k) {
  // Fr.w[28] = 5^((r-1)/2^28)
  Fr w = fr_u64(5);
  u64 t[4] = {MR.m[0], MR.m[1], MR.m[2], MR.m[3]};
  // (r-1) >> 28
  t[0] -= 1;
  for (int i = 0; i < 4; ++i) t[i] = (t[i] >> 28) | (i < 3 ? t[i + 1] << 36 : 0);
  w = w.pow(t);
  for (int i = 28; i > k; --i) w = w * w;
  return w;
}

void ntt(std::vector<Fr>& a, const Fr& w, int threads) {
  const size_t n = a.size();
  for (size_t i = 1, j = 0; i < n; ++i) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j |= bit;
    if (i < j) std::swap(a[i], a[j]);
  }
  for (size_t m = 1; m < n; m <<= 1) {
    // twiddles w^(n/(2m) * j), j < m
    std::vector<Fr> tw(m);
    Fr wm = w;
    for (size_t s = n / (2 * m); s > 1; s >>= 1) wm = wm * wm;
    tw[0] = Fr::one();
    for (size_t j = 1; j < m; ++j) tw[j] = tw[j - 1] * wm;
    par(threads, n / 2, [&](size_t lo, size_t hi, int) {
      for (size_t q = lo; q < hi; ++q) {
        const size_t grp = q / m, j = q % m, k = grp * 2 * m + j;
        Fr u = a[k], v = a[k + m] * tw[j];
        a[k] = u + v;
        a[k + m] = u - v;
      }
    });
  }
}

uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

struct Sec {
  const uint8_t* p = nullptr;
  u64 n = 0;
};
void sections(const uint8_t* buf, size_t len, Sec* s) {
  size_t pos = 12;
  const uint32_t ns = rd32(buf + 8);
  for (uint32_t i = 0; i < ns; ++i) {
    const uint32_t id = rd32(buf + pos);
    u64 l;
    std::memcpy(&l, buf + pos + 4, 8);
    pos += 12;
    if (id < 16) s[id] = Sec{buf + pos, l};
    pos += l;
    if (pos > len) throw std::runtime_error("truncated");
  }
}

template <class E>
void put_aff(const J<E>& p, uint8_t* out) {
  E x, y;
  bool inf;
  jaff(p, x, y, inf);
  if (inf) {
    std::memset(out, 0, 2 * sizeof(E));
    return;
  }
  if constexpr (sizeof(E) == 32) {
    Fq a = x.to_std(), b = y.to_std();
    std::memcpy(out, a.v, 32);
    std::memcpy(out + 32, b.v, 32);
  } else {
    Fq v[4] = {x.a.to_std(), x.b.to_std(), y.a.to_std(), y.b.to_std()};
    for (int i = 0; i < 4; ++i) std::memcpy(out + 32 * i, v[i].v, 32);
  }
}

}  // namespace

extern "C" {

// MSM over zkey-layout affine points / 32-byte LE scalars -> standard affine (zeros = infinity)
int g16cpu_msm_g1(const uint8_t* pts, const uint8_t* sc, size_t n, int threads, uint8_t* out64) {
  put_aff(msm<Fq>(pts, sc, n, threads), out64);
  return 0;
}
int g16cpu_msm_g2(const uint8_t* pts, const uint8_t* sc, size_t n, int threads, uint8_t* out128) {
  put_aff(msm<Fq2>(pts, sc, n, threads), out128);
  return 0;
}

// Standalone Fr NTT of n = 2^k standard-form LE values (< r), natural order in and out, the
// transforms of snarkjs groth16_prove (the loop in g16cpu_prove below):
// mode 0 Fr.fft (w = Fr.w[k]), 1 Fr.ifft (w^-1, times 1/n), 2 the coset extension
// ifft -> batchApplyKey(1, Fr.w[k+1]) -> fft.  in and out may alias.
int g16cpu_ntt(const uint8_t* in, size_t n, int mode, int threads, uint8_t* out) {
  if (n == 0 || (n & (n - 1)) || n > (size_t(1) << 27) || mode < 0 || mode > 2) return 1;
  int lg = 0;
  while ((size_t(1) << lg) < n) ++lg;
  std::vector<Fr> a(n);
  par(threads, n, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; ++i) a[i] = Fr::from_std(Fr::from_raw(in + 32 * i));
  });
  const Fr wr = root(lg), winv = wr.inv(), ninv = fr_u64(n).inv();
  if (mode == 0) {
    ntt(a, wr, threads);
  } else {
    ntt(a, winv, threads);
    if (mode == 1) {
      par(threads, n, [&](size_t lo, size_t hi, int) {
        for (size_t i = lo; i < hi; ++i) a[i] = a[i] * ninv;
      });
    } else {
      // key ninv * g^i, g = Fr.w[k+1]: each thread starts its run at g^lo
      const Fr g = root(lg + 1);
      par(threads, n, [&](size_t lo, size_t hi, int) {
        u64 e[4] = {lo, 0, 0, 0};
        Fr cur = g.pow(e) * ninv;
        for (size_t i = lo; i < hi; ++i) {
          a[i] = a[i] * cur;
          cur = cur * g;
        }
      });
      ntt(a, wr, threads);
    }
  }
  par(threads, n, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; ++i) {
      Fr v = a[i].to_std();
      std::memcpy(out + 32 * i, v.v, 32);
    }
  });
  return 0;
}

// Full Groth16 proof.  out: A (64) | B (128) | C (64) standard-form LE.  ms[0..4]:
// buildABC, NTT+join, MSM G1, MSM G2, total.
int g16cpu_prove(const uint8_t* zk, size_t zlen, const uint8_t* wt, size_t wlen, const uint8_t* r32,
                 const uint8_t* s32, int threads, uint8_t* out, double* ms) {
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  Sec z[16], w[16];
  sections(zk, zlen, z);
  sections(wt, wlen, w);
  const uint8_t* h = z[2].p;
  const uint32_t nv = rd32(h + 72), np = rd32(h + 76), n = rd32(h + 80);
  const uint8_t* hp = h + 84;
  const uint8_t* wv = w[2].p;
  int lg = 0;
  while ((1u << lg) < n) ++lg;
  // buildABC1 (rows partitioned over threads via a CSR-by-row index)
  const uint32_t ncoef = rd32(z[4].p);
  const uint8_t* cf = z[4].p + 4;
  std::vector<uint32_t> cnt(n + 1, 0);
  for (uint32_t i = 0; i < ncoef; ++i) cnt[rd32(cf + 44 * i + 4) + 1]++;
  for (uint32_t r = 0; r < n; ++r) cnt[r + 1] += cnt[r];
  std::vector<uint32_t> order(ncoef), fill(cnt.begin(), cnt.end() - 1);
  for (uint32_t i = 0; i < ncoef; ++i) order[fill[rd32(cf + 44 * i + 4)]++] = i;
  std::vector<Fr> A(n, Fr::zero()), B(n, Fr::zero()), C(n);
  par(threads, n, [&](size_t lo, size_t hi, int) {
    for (size_t r = lo; r < hi; ++r) {
      for (uint32_t e = cnt[r]; e < cnt[r + 1]; ++e) {
        const uint8_t* c = cf + 44 * (size_t)order[e];
        // raw coef bytes (coef*R^2) times raw witness (standard) = Montgomery(coef*w)
        Fr prod = Fr::from_raw(c + 12) * Fr::from_raw(wv + 32 * (size_t)rd32(c + 8));
        if (rd32(c) == 0)
          A[r] = A[r] + prod;
        else
          B[r] = B[r] + prod;
      }
      C[r] = A[r] * B[r];
    }
  });
  auto t1 = clk::now();
  const Fr wr = root(lg), g = root(lg + 1), winv = wr.inv(), ninv = fr_u64(n).inv();
  std::vector<Fr> gp(n);
  gp[0] = ninv;
  for (uint32_t i = 1; i < n; ++i) gp[i] = gp[i - 1] * g;
  for (auto* X : {&A, &B, &C}) {
    ntt(*X, winv, threads);  // n * ifft
    par(threads, n, [&](size_t lo, size_t hi, int) {
      for (size_t i = lo; i < hi; ++i) (*X)[i] = (*X)[i] * gp[i];
    });
    ntt(*X, wr, threads);
  }
  std::vector<uint8_t> hs((size_t)n * 32);
  par(threads, n, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; ++i) {
      Fr v = (A[i] * B[i] - C[i]).to_std();
      std::memcpy(&hs[32 * i], v.v, 32);
    }
  });
  A.clear(), B.clear(), C.clear();
  auto t2 = clk::now();
  J<Fq> pa = msm<Fq>(z[5].p, wv, nv, threads);
  J<Fq> pb1 = msm<Fq>(z[6].p, wv, nv, threads);
  J<Fq> pc = msm<Fq>(z[8].p, wv + 32 * (size_t)(np + 1), nv - np - 1, threads);
  J<Fq> ph = msm<Fq>(z[9].p, hs.data(), n, threads);
  auto t3 = clk::now();
  J<Fq2> pb = msm<Fq2>(z[7].p, wv, nv, threads);
  auto t4 = clk::now();
  auto g1 = [&](const uint8_t* p) {
    Fq x = Fq::from_raw(p), y = Fq::from_raw(p + 32);
    return (x.is_zero() && y.is_zero()) ? jinf<Fq>() : J<Fq>{x, y, Fq::one()};
  };
  auto g2 = [&](const uint8_t* p) {
    Fq2 x{Fq::from_raw(p), Fq::from_raw(p + 32)}, y{Fq::from_raw(p + 64), Fq::from_raw(p + 96)};
    return (x.is_zero() && y.is_zero()) ? jinf<Fq2>() : J<Fq2>{x, y, Fq2::one()};
  };
  Fr r = Fr::from_raw(r32), s = Fr::from_raw(s32);  // standard form, < r
  J<Fq> alpha1 = g1(hp), beta1 = g1(hp + 64), delta1 = g1(hp + 384);
  J<Fq2> beta2 = g2(hp + 128), delta2 = g2(hp + 448);
  J<Fq> Ap = jadd(jadd(pa, alpha1), jmul(delta1, r));
  J<Fq2> Bp = jadd(jadd(pb, beta2), jmul(delta2, s));
  J<Fq> B1 = jadd(jadd(pb1, beta1), jmul(delta1, s));
  Fr rs = (Fr::from_std(r) * Fr::from_std(s));
  Fr nrs = (Fr::zero() - rs).to_std();
  J<Fq> Cp = jadd(pc, ph);
  Cp = jadd(Cp, jmul(Ap, s));
  Cp = jadd(Cp, jmul(B1, r));
  Cp = jadd(Cp, jmul(delta1, nrs));
  put_aff(Ap, out);
  put_aff(Bp, out + 64);
  put_aff(Cp, out + 192);
  auto t5 = clk::now();
  if (ms) {
    auto d = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    ms[0] = d(t0, t1), ms[1] = d(t1, t2), ms[2] = d(t2, t3), ms[3] = d(t3, t4), ms[4] = d(t0, t5);
  }
  return 0;
}

}  // extern "C"
