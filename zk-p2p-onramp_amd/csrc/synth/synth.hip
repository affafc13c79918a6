// libzkp_synth.so — synthetic Venmo-shaped circuits, witnesses and INSECURE
// known-tau zkeys in snarkjs binary format (include/zkp_synth.h).  TOOLING for
// benchmarks and large-size tests; not part of the proving path.
//
// Bit-for-bit mirror of oracle/circuit.py (gen_program / gen_witness) and
// oracle/setup.py (setup, zkey_coefs); the fixed-base scalar multiplications
// (27.6 M G1 + 6.4 M G2 points for the Venmo shape) run on the GPU with a
// 4-bit windowed table, everything else on host threads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/zkp_synth.h"
#include "../curve.hpp"
#include "../hip_check.hpp"
#include "../host_ec.hpp"

using namespace zkp;
using host::U256;
using HFr = host::Fr;
using HFq = host::Fq;
using HFq2 = host::Fq2;

namespace {

thread_local std::string g_err;

// ------------------------------------------------------------------ RNG (oracle/circuit.py SplitMix64)
struct Rng {
  uint64_t s;
  Rng(uint64_t seed, uint64_t stream) : s(seed + stream * 0x632BE59BD9B4E019ull) {}
  uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t k) { return next() % k; }
  U256 fr() {
    for (;;) {
      U256 v;
      for (int i = 0; i < 4; ++i) v.w[i] = next();
      v.w[3] &= (uint64_t(1) << 62) - 1;
      if (!host::u256_geq(v, host::FR_DESC.mod)) return v;
    }
  }
};

const U256 U_ZERO{{0, 0, 0, 0}};
const U256 U_ONE{{1, 0, 0, 0}};
const U256 U_TWO{{2, 0, 0, 0}};
U256 r_minus_1() {
  U256 v = host::FR_DESC.mod;
  host::u256_sub(v, U_ONE);
  return v;
}

HFr fr_of(const U256& x) { return HFr::from_std(x); }

struct Term {
  uint32_t sig;
  U256 coef;  // standard form, nonzero
};
struct Lc {
  Term t[3];
  int n = 0;
};

// oracle/circuit.py _lc: merge equal signals (sum mod r), drop zeros, sort by signal
Lc make_lc(std::initializer_list<std::pair<uint32_t, U256>> pairs) {
  Lc out;
  std::pair<uint32_t, HFr> acc[3];
  int na = 0;
  for (auto& p : pairs) {
    int k = 0;
    while (k < na && acc[k].first != p.first) ++k;
    if (k == na) acc[na++] = {p.first, fr_of(p.second)};
    else acc[k].second = acc[k].second + fr_of(p.second);
  }
  std::sort(acc, acc + na, [](const auto& a, const auto& b) { return a.first < b.first; });
  for (int k = 0; k < na; ++k)
    if (!acc[k].second.is_zero()) out.t[out.n++] = Term{acc[k].first, acc[k].second.to_std()};
  return out;
}

struct Step {
  uint8_t kind;  // 0 AND, 1 XOR, 2 MUL
  uint32_t a, b, c;
  uint32_t coef;  // index into mulcoef (kind 2)
};

}  // namespace

struct zkp_synth_circuit {
  uint32_t n_vars, n_cons, n_pub, n_in, domain, log_domain;
  std::vector<Step> prog;
  std::vector<std::array<U256, 4>> mulcoef;
  std::vector<uint32_t> boolbits;  // bit signal of each booleanity constraint

  uint32_t n_def() const { return (uint32_t)prog.size(); }

  void constraint(uint32_t c, Lc& A, Lc& B, Lc& C) const {
    if (c < n_def()) {
      const Step& st = prog[c];
      const uint32_t v = 1 + n_pub + n_in + c;
      if (st.kind == 0) {
        A = make_lc({{st.a, U_ONE}});
        B = make_lc({{st.b, U_ONE}});
        C = make_lc({{v, U_ONE}});
      } else if (st.kind == 1) {
        A = make_lc({{st.a, U_TWO}});
        B = make_lc({{st.b, U_ONE}});
        C = make_lc({{st.a, U_ONE}, {st.b, U_ONE}, {v, r_minus_1()}});
      } else {
        const auto& k = mulcoef[st.coef];
        A = make_lc({{st.a, k[0]}, {st.b, k[1]}});
        B = make_lc({{st.c, k[2]}, {0u, k[3]}});
        C = make_lc({{v, U_ONE}});
      }
    } else {
      const uint32_t b = boolbits[c - n_def()];
      A = make_lc({{b, U_ONE}});
      B = make_lc({{b, U_ONE}, {0u, r_minus_1()}});
      C = Lc{};
    }
  }
};

namespace {

// ------------------------------------------------------------------ fixed-base GPU kernel

constexpr int FB_WIN = 4;
constexpr int FB_NWIN = 64;  // 256 bits
constexpr int FB_TBL = FB_NWIN * ((1 << FB_WIN) - 1);

template <class C>
__device__ Fe<C> inv_fermat(const Fe<C>& a) {
  // a^(m-2), m-2 from the 8-word modulus
  uint32_t e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = C::MOD_W[i];
  e[0] -= 2;  // low word of m is >= 2 for both moduli
  Fe<C> r = fe_one<C>();
  bool started = false;
  for (int i = 255; i >= 0; --i) {
    if (started) r = sqr(r);
    if ((e[i >> 5] >> (i & 31)) & 1) {
      r = started ? mul(r, a) : a;
      started = true;
    }
  }
  return r;
}

__device__ Fq f_inv(const Fq& a) { return inv_fermat(a); }
__device__ Fq2 f_inv(const Fq2& a) {
  Fq t = inv_fermat(add(sqr(a.c0), sqr(a.c1)));
  return Fq2{mul(a.c0, t), sub(fe_zero<FqCfg>(), mul(a.c1, t))};
}

// device value x*2^261 -> zkey layout x*2^256 (canonical) words
__device__ void store_zkey_fq(uint32_t* out, const Fq& x, const Fq& k256) { store_fe(out, canon(mul(x, k256))); }
__device__ void store_zkey_f(uint32_t* out, const Fq& x, const Fq& k) { store_zkey_fq(out, x, k); }
__device__ void store_zkey_f(uint32_t* out, const Fq2& x, const Fq& k) {
  store_zkey_fq(out, x.c0, k);
  store_zkey_fq(out + 8, x.c1, k);
}

template <class F>
__global__ __launch_bounds__(256) void k_fixed_base(const uint32_t* __restrict__ scalars, size_t n,
                                                    const uint32_t* __restrict__ table,
                                                    const uint32_t* __restrict__ k256w,
                                                    uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  constexpr int FW = FWords<F>::W;
  const uint32_t* s = scalars + i * 8;
  Xyzz<F> acc = xyzz_inf<F>();
  for (int w = 0; w < FB_NWIN; ++w) {
    const uint32_t d = (s[w >> 3] >> ((w & 7) * 4)) & 15u;
    if (d) xyzz_add_aff(acc, load_aff<F>(table, (size_t)w * 15 + d - 1));
  }
  uint32_t* o = out + i * 2 * FW;  // affine (x, y)
  if (xyzz_is_inf(acc)) {
    for (int k = 0; k < 2 * FW; ++k) o[k] = 0;
    return;
  }
  const Fq k256 = load_fe<FqCfg>(k256w);
  F t = f_inv(mul(acc.zz, acc.zzz));
  F x = mul(mul(acc.x, acc.zzz), t);
  F y = mul(mul(acc.y, acc.zz), t);
  store_zkey_f(o, x, k256);
  store_zkey_f(o + FW, y, k256);
}

// host: standard integer x (raw U256 of a value < p) -> device-layout words (x*2^261 mod p)
void fq_std_to_dev(const HFq& v, uint32_t* w) {
  static const HFq two261 = HFq::from_std(U256{{0, 0, 0, uint64_t(1) << 58}}) * HFq::from_std(U256{{1u << 11, 0, 0, 0}});
  U256 raw = (v * two261).to_std();
  for (int i = 0; i < 4; ++i) {
    w[2 * i] = (uint32_t)raw.w[i];
    w[2 * i + 1] = (uint32_t)(raw.w[i] >> 32);
  }
}

template <class HF>
void put_dev(const HF& v, uint32_t* w);
template <>
void put_dev<HFq>(const HFq& v, uint32_t* w) {
  fq_std_to_dev(v, w);
}
template <>
void put_dev<HFq2>(const HFq2& v, uint32_t* w) {
  fq_std_to_dev(v.c0, w);
  fq_std_to_dev(v.c1, w + 8);
}

template <class HF>
std::vector<uint32_t> make_table(const host::Affine<HF>& g) {
  constexpr int FW = sizeof(HF) == sizeof(HFq) ? 8 : 16;
  std::vector<uint32_t> t((size_t)FB_TBL * 2 * FW);
  host::Jac<HF> base = host::jac_from_aff(g);
  for (int w = 0; w < FB_NWIN; ++w) {
    host::Jac<HF> cur = base;
    for (int d = 1; d < 16; ++d) {
      auto a = host::jac_to_aff(cur);
      put_dev(a.x, &t[((size_t)w * 15 + d - 1) * 2 * FW]);
      put_dev(a.y, &t[((size_t)w * 15 + d - 1) * 2 * FW + FW]);
      cur = host::jac_add(cur, base);
    }
    for (int k = 0; k < FB_WIN; ++k) base = host::jac_dbl(base);
  }
  return t;
}

host::Affine<HFq> g1_gen() {
  return host::Affine<HFq>{HFq::from_std(U_ONE), HFq::from_std(U_TWO), false};
}

U256 u256_dec(const char* s) {
  U256 v = U_ZERO;
  for (; *s; ++s) {
    U256 t = v;  // v = v*10 + d
    U256 acc = U_ZERO;
    for (int k = 0; k < 10; ++k) host::u256_add(acc, t);
    U256 d{{(uint64_t)(*s - '0'), 0, 0, 0}};
    host::u256_add(acc, d);
    v = acc;
  }
  return v;
}

host::Affine<HFq2> g2_gen() {
  // contracts/Verifier.sol:33-36 (x = c0 + c1 u, y likewise)
  HFq2 x{HFq::from_std(u256_dec("10857046999023057135944570762232829481370756359578518086990519993285655852781")),
         HFq::from_std(u256_dec("11559732032986387107991004021392285783925812861821192530917403151452391805634"))};
  HFq2 y{HFq::from_std(u256_dec("8495653923123431417604973247489272438418190587263600148770280649306958101930")),
         HFq::from_std(u256_dec("4082367875863433681332203403145435568316851327593401208105741076214120093531"))};
  return host::Affine<HFq2>{x, y, false};
}

// run k_fixed_base over n scalars (standard-form U256) into zkey-layout bytes
template <class F, class HF>
void fixed_base(int device, const U256* scalars, size_t n, uint8_t* out, const host::Affine<HF>& gen) {
  constexpr int FW = sizeof(HF) == sizeof(HFq) ? 8 : 16;
  if (n == 0) return;
  HIPX(hipSetDevice(device));
  hipStream_t st;
  HIPX(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<uint32_t> tbl = make_table(gen);
  uint32_t k256w[8];
  {  // 2^256 mod p as a plain integer in device words
    U256 k = HFq::one().v;  // raw of value 1 = 2^256 mod p
    for (int i = 0; i < 4; ++i) {
      k256w[2 * i] = (uint32_t)k.w[i];
      k256w[2 * i + 1] = (uint32_t)(k.w[i] >> 32);
    }
  }
  const size_t CH = size_t(1) << 22;
  uint32_t *dt = nullptr, *dk = nullptr, *ds = nullptr, *dout = nullptr;
  HIPX(hipMalloc(&dt, tbl.size() * 4));
  HIPX(hipMalloc(&dk, 32));
  HIPX(hipMalloc(&ds, std::min(n, CH) * 32));
  HIPX(hipMalloc(&dout, std::min(n, CH) * 2 * FW * 4));
  HIPX(hipMemcpyAsync(dt, tbl.data(), tbl.size() * 4, hipMemcpyHostToDevice, st));
  HIPX(hipMemcpyAsync(dk, k256w, 32, hipMemcpyHostToDevice, st));
  for (size_t off = 0; off < n; off += CH) {
    const size_t m = std::min(CH, n - off);
    HIPX(hipMemcpyAsync(ds, scalars + off, m * 32, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_fixed_base<F>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, ds, m, dt, dk, dout);
    HIPX(hipGetLastError());
    HIPX(hipMemcpyAsync(out + off * 2 * FW * 4, dout, m * 2 * FW * 4, hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));
  }
  for (void* p : {(void*)dt, (void*)dk, (void*)ds, (void*)dout}) (void)hipFree(p);
  HIPX(hipStreamDestroy(st));
}

// ------------------------------------------------------------------ host helpers

template <class Fn>
void parallel_for(size_t n, int threads, Fn&& fn) {
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  threads = (int)std::min<size_t>((size_t)threads, std::max<size_t>(1, n / 4096));
  if (threads <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    const size_t a = n * t / threads, b = n * (t + 1) / threads;
    th.emplace_back([&fn, a, b] { fn(a, b); });
  }
  for (auto& x : th) x.join();
}

HFr fr_pow_u64(HFr b, uint64_t e) {
  HFr r = HFr::one();
  while (e) {
    if (e & 1) r = r * b;
    b = b.sqr();
    e >>= 1;
  }
  return r;
}

HFr root_w(int k) {  // Fr.w[k]: nqr^((r-1)/2^28) squared 28-k times
  static const U256 w28 = u256_dec("19103219067921713944291392827692070036145651957329286315305642004821462161904");
  HFr w = HFr::from_std(w28);
  for (int i = 28; i > k; --i) w = w.sqr();
  return w;
}

// out[i] = z * pts[i] / (tau - pts[i]) with pts[i] = first * step^i  (i < n)
void lagrange_like(const HFr& tau, const HFr& first, const HFr& step, const HFr& z, size_t n, std::vector<HFr>& out,
                   int threads) {
  out.resize(n);
  parallel_for(n, threads, [&](size_t a, size_t b) {
    if (a >= b) return;
    HFr p = first * fr_pow_u64(step, a);
    std::vector<HFr> pts(b - a), den(b - a), pref(b - a);
    HFr acc = HFr::one();
    for (size_t i = a; i < b; ++i) {
      pts[i - a] = p;
      den[i - a] = tau - p;
      if (den[i - a].is_zero()) throw std::runtime_error("tau in domain");
      pref[i - a] = acc;
      acc = acc * den[i - a];
      p = p * step;
    }
    HFr inv = acc.inv();
    for (size_t i = b; i-- > a;) {
      HFr di = inv * pref[i - a];
      inv = inv * den[i - a];
      out[i] = z * pts[i - a] * di;
    }
  });
}

void put_u32(std::vector<uint8_t>& v, uint32_t x) {
  for (int i = 0; i < 4; ++i) v.push_back((uint8_t)(x >> (8 * i)));
}
void put_u64(uint8_t* p, uint64_t x) {
  for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(x >> (8 * i));
}
void put_le(uint8_t* p, const U256& x) { host::u256_to_le(x, p); }

void put_g1_raw(uint8_t* p, const host::Affine<HFq>& a) {
  if (a.inf) {
    std::memset(p, 0, 64);
    return;
  }
  put_le(p, a.x.v);
  put_le(p + 32, a.y.v);
}
void put_g2_raw(uint8_t* p, const host::Affine<HFq2>& a) {
  if (a.inf) {
    std::memset(p, 0, 128);
    return;
  }
  put_le(p, a.x.c0.v);
  put_le(p + 32, a.x.c1.v);
  put_le(p + 64, a.y.c0.v);
  put_le(p + 96, a.y.c1.v);
}

template <class Fn>
int guarded(Fn&& fn) {
  try {
    g_err.clear();
    fn();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return 1;
  } catch (...) {
    g_err = "unknown error";
    return 1;
  }
}

}  // namespace

extern "C" {

const char* zkp_synth_last_error(void) { return g_err.c_str(); }

int zkp_synth_circuit_new(uint32_t n_vars, uint32_t n_cons, uint32_t n_pub, uint64_t seed, uint32_t in_permille,
                          zkp_synth_circuit** out) {
  return zkp_synth_circuit_new_mix(n_vars, n_cons, n_pub, seed, in_permille, 70, out);
}

int zkp_synth_circuit_new_mix(uint32_t n_vars, uint32_t n_cons, uint32_t n_pub, uint64_t seed, uint32_t in_permille,
                              uint32_t bool_percent, zkp_synth_circuit** out) {
  return guarded([&] {
    if (bool_percent > 100) throw std::runtime_error("bool_percent must be <= 100");
    auto* c = new zkp_synth_circuit();
    try {
      c->n_vars = n_vars;
      c->n_cons = n_cons;
      c->n_pub = n_pub;
      if (n_vars < n_pub + 1) throw std::runtime_error("n_vars < n_pub + 1");
      const uint32_t n_priv = n_vars - 1 - n_pub;
      c->n_in = std::max<uint32_t>(2, (uint32_t)((uint64_t)n_priv * in_permille / 1000));
      if (n_priv < c->n_in) throw std::runtime_error("too few private signals");
      Rng rng(seed, 3);
      std::vector<uint32_t> bits;
      bits.reserve(n_vars);
      for (uint32_t k = 0; k < c->n_in; ++k) bits.push_back(1 + n_pub + k);
      for (uint32_t v = 1 + n_pub + c->n_in; v < n_vars; ++v) {
        const uint64_t x = rng.below(100);
        Step st{};
        if (x < bool_percent) {
          st.a = bits[rng.below(bits.size())];
          st.b = bits[rng.below(bits.size())];
          st.kind = x < bool_percent / 2 ? 0 : 1;
          bits.push_back(v);
        } else {
          st.kind = 2;
          st.a = (uint32_t)rng.below(v);
          st.b = (uint32_t)rng.below(v);
          st.c = (uint32_t)rng.below(v);
          std::array<U256, 4> k;
          for (auto& e : k) e = rng.fr();
          st.coef = (uint32_t)c->mulcoef.size();
          c->mulcoef.push_back(k);
        }
        c->prog.push_back(st);
      }
      if (c->prog.size() > n_cons) throw std::runtime_error("n_constraints too small for n_vars");
      uint32_t i = 0;
      while (c->prog.size() + c->boolbits.size() < n_cons) {
        const uint32_t b = i < c->n_in ? bits[i] : bits[rng.below(bits.size())];
        ++i;
        c->boolbits.push_back(b);
      }
      uint64_t n = 1;
      c->log_domain = 0;
      while (n < (uint64_t)n_cons + n_pub + 1) {
        n *= 2;
        ++c->log_domain;
      }
      if (c->log_domain > 27) throw std::runtime_error("domain too large");
      c->domain = (uint32_t)n;
    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}

void zkp_synth_circuit_free(zkp_synth_circuit* c) { delete c; }

uint32_t zkp_synth_domain_size(const zkp_synth_circuit* c) { return c ? c->domain : 0; }

int zkp_synth_witness(const zkp_synth_circuit* c, uint64_t wseed, uint8_t* out, size_t cap, size_t* len) {
  return guarded([&] {
    const size_t need = 12 + 12 + 4 + 32 + 4 + 12 + (size_t)c->n_vars * 32;
    if (len) *len = need;
    if (!out) return;
    if (cap < need) throw std::runtime_error("buffer too small");
    Rng rng(wseed, 4);
    std::vector<HFr> w;
    w.reserve(c->n_vars);
    w.push_back(HFr::one());
    for (uint32_t i = 0; i < c->n_pub; ++i) w.push_back(fr_of(U256{{rng.next(), 0, 0, 0}}));
    for (uint32_t i = 0; i < c->n_in; ++i) w.push_back(fr_of(U256{{rng.next() & 1, 0, 0, 0}}));
    for (const Step& st : c->prog) {
      if (st.kind == 0) {
        w.push_back(w[st.a] * w[st.b]);
      } else if (st.kind == 1) {
        HFr ab = w[st.a] * w[st.b];
        w.push_back(w[st.a] + w[st.b] - ab - ab);
      } else {
        const auto& k = c->mulcoef[st.coef];
        w.push_back((fr_of(k[0]) * w[st.a] + fr_of(k[1]) * w[st.b]) * (fr_of(k[2]) * w[st.c] + fr_of(k[3])));
      }
    }
    // wtns v2: magic, version, nSections=2; sec1 {n8, q, nWitness}; sec2 values
    uint8_t* p = out;
    std::memcpy(p, "wtns", 4);
    p[4] = 2, p[5] = p[6] = p[7] = 0;
    p[8] = 2, p[9] = p[10] = p[11] = 0;
    p += 12;
    p[0] = 1, p[1] = p[2] = p[3] = 0;
    put_u64(p + 4, 40);
    p += 12;
    p[0] = 32, p[1] = p[2] = p[3] = 0;
    put_le(p + 4, host::FR_DESC.mod);
    for (int i = 0; i < 4; ++i) p[36 + i] = (uint8_t)(c->n_vars >> (8 * i));
    p += 40;
    p[0] = 2, p[1] = p[2] = p[3] = 0;
    put_u64(p + 4, (uint64_t)c->n_vars * 32);
    p += 12;
    for (uint32_t i = 0; i < c->n_vars; ++i) put_le(p + (size_t)i * 32, w[i].to_std());
  });
}

void zkp_synth_scalars(uint64_t seed, uint64_t stream, size_t n, uint8_t* out) {
  Rng rng(seed, stream);
  for (size_t i = 0; i < n; ++i) put_le(out + 32 * i, rng.fr());
}

int zkp_synth_points_g1(int device, const uint8_t* scalars, size_t n, uint8_t* out) {
  return guarded([&] { fixed_base<Fq, HFq>(device, reinterpret_cast<const U256*>(scalars), n, out, g1_gen()); });
}

int zkp_synth_points_g2(int device, const uint8_t* scalars, size_t n, uint8_t* out) {
  return guarded([&] { fixed_base<Fq2, HFq2>(device, reinterpret_cast<const U256*>(scalars), n, out, g2_gen()); });
}

void zkp_synth_free(uint8_t* buf) { delete[] buf; }

int zkp_synth_zkey(const zkp_synth_circuit* c, uint64_t setup_seed, int device, int threads, uint8_t** out,
                   size_t* len) {
  return zkp_synth_zkey_ex(c, setup_seed, 0, device, threads, out, len);
}

int zkp_synth_zkey_ex(const zkp_synth_circuit* c, uint64_t setup_seed, int unit_gamma_delta, int device, int threads,
                      uint8_t** out, size_t* len) {
  return guarded([&] {
    // toxic waste: stream 7, five nonzero fr() (oracle/setup.py toxic_from_seed); unit_gamma_delta:
    // gamma = delta = 1, the key `zkey new` writes from a ptau of the same tau, alpha, beta
    Rng rng(setup_seed, 7);
    U256 tox[5];
    for (auto& v : tox) {
      do v = rng.fr();
      while (host::u256_is_zero(v));
    }
    const HFr tau = fr_of(tox[0]), alpha = fr_of(tox[1]), beta = fr_of(tox[2]),
              gamma = unit_gamma_delta ? HFr::one() : fr_of(tox[3]), delta = unit_gamma_delta ? HFr::one() : fr_of(tox[4]);
    const size_t n = c->domain;
    const uint32_t nv = c->n_vars, np = c->n_pub;
    // L_c(tau) = (tau^n - 1)/n * w^c / (tau - w^c)
    const HFr w = root_w((int)c->log_domain);
    const HFr nfr = fr_of(U256{{(uint64_t)n, 0, 0, 0}});
    const HFr zl = (fr_pow_u64(tau, n) - HFr::one()) * nfr.inv();
    std::vector<HFr> L;
    lagrange_like(tau, HFr::one(), w, zl, n, L, threads);
    // A_i, B_i, C_i (single pass over constraints)
    std::vector<HFr> A(nv, HFr::zero()), B(nv, HFr::zero()), C(nv, HFr::zero());
    Lc la, lb, lcc;
    for (uint32_t k = 0; k < c->n_cons; ++k) {
      c->constraint(k, la, lb, lcc);
      const HFr& l = L[k];
      for (int t = 0; t < la.n; ++t) A[la.t[t].sig] = A[la.t[t].sig] + fr_of(la.t[t].coef) * l;
      for (int t = 0; t < lb.n; ++t) B[lb.t[t].sig] = B[lb.t[t].sig] + fr_of(lb.t[t].coef) * l;
      for (int t = 0; t < lcc.n; ++t) C[lcc.t[t].sig] = C[lcc.t[t].sig] + fr_of(lcc.t[t].coef) * l;
    }
    for (uint32_t i = 0; i <= np; ++i) A[i] = A[i] + L[c->n_cons + i];
    // H: delta^-1 L^(2n)_(2j+1)(tau), points g w^j, g = Fr.w[log n + 1]
    const HFr g = root_w((int)c->log_domain + 1);
    const HFr n2 = fr_of(U256{{(uint64_t)(2 * n), 0, 0, 0}});
    const HFr zh = (fr_pow_u64(tau, 2 * n) - HFr::one()) * n2.inv();
    std::vector<HFr> H;
    lagrange_like(tau, g, w, zh, n, H, threads);
    const HFr ginv = gamma.inv(), dinv = delta.inv();
    // scalar arrays (standard form) for every point section
    const size_t ncp = nv - np - 1;
    std::vector<U256> sa(nv), sb(nv), sic(np + 1), sc(ncp), sh(n);
    parallel_for(nv, threads, [&](size_t a, size_t b) {
      for (size_t i = a; i < b; ++i) {
        sa[i] = A[i].to_std();
        sb[i] = B[i].to_std();
        const HFr lin = beta * A[i] + alpha * B[i] + C[i];
        if (i <= np)
          sic[i] = (lin * ginv).to_std();
        else
          sc[i - np - 1] = (lin * dinv).to_std();
      }
    });
    parallel_for(n, threads, [&](size_t a, size_t b) {
      for (size_t j = a; j < b; ++j) sh[j] = (H[j] * dinv).to_std();
    });
    L.clear(), L.shrink_to_fit(), H.clear(), H.shrink_to_fit();
    // coefficient section
    uint64_t ncoef = 0;
    for (uint32_t k = 0; k < c->n_cons; ++k) {
      c->constraint(k, la, lb, lcc);
      ncoef += la.n + lb.n;
    }
    ncoef += np + 1;
    // layout
    const uint64_t len2 = 4 + 32 + 4 + 32 + 12 + 64 * 3 + 128 * 3;
    const uint64_t lens[11] = {0, 4, len2, (uint64_t)(np + 1) * 64, 4 + ncoef * 44, (uint64_t)nv * 64,
                               (uint64_t)nv * 64, (uint64_t)nv * 128, (uint64_t)ncp * 64, (uint64_t)n * 64, 68};
    uint64_t total = 12;
    uint64_t off[11];
    for (int s = 1; s <= 10; ++s) {
      off[s] = total + 12;
      total += 12 + lens[s];
    }
    uint8_t* buf = new uint8_t[total];
    try {
      std::memcpy(buf, "zkey", 4);
      uint32_t hdr[2] = {1, 10};
      std::memcpy(buf + 4, hdr, 8);
      for (int s = 1; s <= 10; ++s) {
        uint32_t id = (uint32_t)s;
        std::memcpy(buf + off[s] - 12, &id, 4);
        put_u64(buf + off[s] - 8, lens[s]);
      }
      uint32_t one = 1;
      std::memcpy(buf + off[1], &one, 4);
      // sec2 header
      uint8_t* p = buf + off[2];
      uint32_t n8 = 32;
      std::memcpy(p, &n8, 4);
      put_le(p + 4, host::FQ_DESC.mod);
      std::memcpy(p + 36, &n8, 4);
      put_le(p + 40, host::FR_DESC.mod);
      uint32_t hv[3] = {nv, np, (uint32_t)n};
      std::memcpy(p + 72, hv, 12);
      p += 84;
      const auto G1 = g1_gen();
      const auto G2 = g2_gen();
      auto g1mul = [&](const HFr& k) { return host::jac_to_aff(host::jac_mul(host::jac_from_aff(G1), k.to_std())); };
      auto g2mul = [&](const HFr& k) { return host::jac_to_aff(host::jac_mul(host::jac_from_aff(G2), k.to_std())); };
      put_g1_raw(p, g1mul(alpha));
      put_g1_raw(p + 64, g1mul(beta));
      put_g2_raw(p + 128, g2mul(beta));
      put_g2_raw(p + 256, g2mul(gamma));
      put_g1_raw(p + 384, g1mul(delta));
      put_g2_raw(p + 448, g2mul(delta));
      // sec4 coefficients: value stored as coef * 2^512 mod r
      p = buf + off[4];
      std::memcpy(p, &ncoef, 4);
      p += 4;
      auto put_coef = [&](uint32_t m, uint32_t k, const Term& t) {
        uint32_t h3[3] = {m, k, t.sig};
        std::memcpy(p, h3, 12);
        put_le(p + 12, HFr::from_std(HFr::from_std(t.coef).v).v);
        p += 44;
      };
      for (uint32_t k = 0; k < c->n_cons; ++k) {
        c->constraint(k, la, lb, lcc);
        for (int t = 0; t < la.n; ++t) put_coef(0, k, la.t[t]);
        for (int t = 0; t < lb.n; ++t) put_coef(1, k, lb.t[t]);
      }
      for (uint32_t i = 0; i <= np; ++i) put_coef(0, c->n_cons + i, Term{i, U_ONE});
      // points on the GPU
      fixed_base<Fq, HFq>(device, sic.data(), sic.size(), buf + off[3], G1);
      fixed_base<Fq, HFq>(device, sa.data(), sa.size(), buf + off[5], G1);
      fixed_base<Fq, HFq>(device, sb.data(), sb.size(), buf + off[6], G1);
      fixed_base<Fq2, HFq2>(device, sb.data(), sb.size(), buf + off[7], G2);
      fixed_base<Fq, HFq>(device, sc.data(), sc.size(), buf + off[8], G1);
      fixed_base<Fq, HFq>(device, sh.data(), sh.size(), buf + off[9], G1);
      std::memset(buf + off[10], 0, 68);
    } catch (...) {
      delete[] buf;
      throw;
    }
    *out = buf;
    *len = total;
  });
}

int zkp_synth_r1cs(const zkp_synth_circuit* c, uint8_t** out, size_t* len) {
  return guarded([&] {
    // circom .r1cs v1 (oracle/binfile.py write_r1cs): 1 header, 2 constraints, 3 wire labels; every
    // public signal a public input
    Lc l[3];
    uint64_t len2 = 0;
    for (uint32_t k = 0; k < c->n_cons; ++k) {
      c->constraint(k, l[0], l[1], l[2]);
      for (auto& x : l) len2 += 4 + 36 * (uint64_t)x.n;
    }
    const uint64_t lens[4] = {0, 4 + 32 + 16 + 8 + 4, len2, (uint64_t)c->n_vars * 8};
    const uint64_t total = 12 + 3 * 12 + lens[1] + lens[2] + lens[3];
    uint8_t* buf = new uint8_t[total];
    uint8_t* p = buf;
    std::memcpy(p, "r1cs", 4);
    const uint32_t hv[2] = {1, 3};
    std::memcpy(p + 4, hv, 8);
    p += 12;
    for (uint32_t sid = 1; sid <= 3; ++sid) {
      std::memcpy(p, &sid, 4);
      put_u64(p + 4, lens[sid]);
      p += 12;
      if (sid == 1) {
        const uint32_t n8 = 32;
        std::memcpy(p, &n8, 4);
        put_le(p + 4, host::FR_DESC.mod);
        const uint32_t w4[4] = {c->n_vars, 0, c->n_pub, c->n_vars - 1 - c->n_pub};
        std::memcpy(p + 36, w4, 16);
        put_u64(p + 52, c->n_vars);
        std::memcpy(p + 60, &c->n_cons, 4);
        p += lens[1];
      } else if (sid == 2) {
        for (uint32_t k = 0; k < c->n_cons; ++k) {
          c->constraint(k, l[0], l[1], l[2]);
          for (auto& x : l) {
            const uint32_t cnt = (uint32_t)x.n;
            std::memcpy(p, &cnt, 4);
            p += 4;
            for (int t = 0; t < x.n; ++t, p += 36) {
              std::memcpy(p, &x.t[t].sig, 4);
              put_le(p + 4, x.t[t].coef);
            }
          }
        }
      } else {
        for (uint32_t i = 0; i < c->n_vars; ++i, p += 8) put_u64(p, i);
      }
    }
    *out = buf;
    *len = total;
  });
}

int zkp_synth_ptau(uint32_t power, uint64_t setup_seed, int device, int threads, uint8_t** out, size_t* len) {
  return guarded([&] {
    // a prepared (phase-2-ready) ptau of known tau, alpha, beta (stream 7 as zkp_synth_zkey), the
    // layout of oracle/binfile.py write_ptau: 1 header, 2 tauG1 (2^(power+1) - 1), 3 tauG2 (2^power),
    // 4 alphaTauG1, 5 betaTauG1 (2^power each), 6 betaG2, 7 no contributions, 12..15 the Lagrange
    // forms (lTauG1, lTauG2, lAlphaTauG1, lBetaTauG1) of every level p = 0..power.  INSECURE tooling.
    if (power < 1 || power > 27) throw std::runtime_error("ptau power must be within 1..27");
    Rng rng(setup_seed, 7);
    U256 tox[3];
    for (auto& v : tox) {
      do v = rng.fr();
      while (host::u256_is_zero(v));
    }
    const HFr tau = fr_of(tox[0]), alpha = fr_of(tox[1]), beta = fr_of(tox[2]);
    const uint64_t N = uint64_t(1) << power, NL = (N << 1) - 1;
    const uint64_t lens[16] = {0, 4 + 32 + 8, NL * 64, N * 128, N * 64, N * 64, 128, 4, 0, 0, 0, 0,
                               NL * 64, NL * 128, NL * 64, NL * 64};
    const int ids[11] = {1, 2, 3, 4, 5, 6, 7, 12, 13, 14, 15};
    uint64_t off[16] = {}, total = 12;
    for (int id : ids) {
      off[id] = total + 12;
      total += 12 + lens[id];
    }
    uint8_t* buf = new uint8_t[total];
    try {
      std::memcpy(buf, "ptau", 4);
      const uint32_t hv[2] = {1, 11};
      std::memcpy(buf + 4, hv, 8);
      for (int id : ids) {
        const uint32_t u = (uint32_t)id;
        std::memcpy(buf + off[id] - 12, &u, 4);
        put_u64(buf + off[id] - 8, lens[id]);
      }
      const uint32_t n8 = 32;
      std::memcpy(buf + off[1], &n8, 4);
      put_le(buf + off[1] + 4, host::FQ_DESC.mod);
      std::memcpy(buf + off[1] + 36, &power, 4);
      std::memcpy(buf + off[1] + 40, &power, 4);
      std::memset(buf + off[7], 0, 4);
      const auto G1 = g1_gen();
      const auto G2 = g2_gen();
      put_g2_raw(buf + off[6], host::jac_to_aff(host::jac_mul(host::jac_from_aff(G2), beta.to_std())));
      // the points are stored in Montgomery form like the zkey sections (fixed_base writes that)
      std::vector<U256> sc;
      auto powers = [&](uint64_t n, const HFr& k) {  // k tau^i, i < n
        sc.resize(n);
        parallel_for(n, threads, [&](size_t a, size_t b) {
          HFr x = k * fr_pow_u64(tau, a);
          for (size_t i = a; i < b; ++i, x = x * tau) sc[i] = x.to_std();
        });
      };
      powers(NL, HFr::one());
      fixed_base<Fq, HFq>(device, sc.data(), NL, buf + off[2], G1);
      powers(N, HFr::one());
      fixed_base<Fq2, HFq2>(device, sc.data(), N, buf + off[3], G2);
      powers(N, alpha);
      fixed_base<Fq, HFq>(device, sc.data(), N, buf + off[4], G1);
      powers(N, beta);
      fixed_base<Fq, HFq>(device, sc.data(), N, buf + off[5], G1);
      // Lagrange forms: level p = 2^p points at 2^p - 1: L^(2^p)_i(tau) = (tau^m - 1)/m * w^i/(tau - w^i)
      std::vector<U256> sl(NL), sa(NL), sb(NL);
      for (uint32_t lvl = 0; lvl <= power; ++lvl) {
        const size_t m = size_t(1) << lvl;
        std::vector<HFr> L;
        const HFr mfr = fr_of(U256{{(uint64_t)m, 0, 0, 0}});
        lagrange_like(tau, HFr::one(), root_w((int)lvl), (fr_pow_u64(tau, m) - HFr::one()) * mfr.inv(), m, L, threads);
        parallel_for(m, threads, [&](size_t a, size_t b) {
          for (size_t i = a; i < b; ++i) {
            sl[m - 1 + i] = L[i].to_std();
            sa[m - 1 + i] = (alpha * L[i]).to_std();
            sb[m - 1 + i] = (beta * L[i]).to_std();
          }
        });
      }
      fixed_base<Fq, HFq>(device, sl.data(), NL, buf + off[12], G1);
      fixed_base<Fq2, HFq2>(device, sl.data(), NL, buf + off[13], G2);
      fixed_base<Fq, HFq>(device, sa.data(), NL, buf + off[14], G1);
      fixed_base<Fq, HFq>(device, sb.data(), NL, buf + off[15], G1);
    } catch (...) {
      delete[] buf;
      throw;
    }
    *out = buf;
    *len = total;
  });
}

}  // extern "C"
