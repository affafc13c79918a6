// Phase-2 MPC record of a zkey (see mpc.hpp; restatement checked against oracle/mpc.py).
#include "mpc.hpp"

#include <algorithm>
#include <cstring>
#include <thread>

#include "prover.hpp"

namespace zkp {

using host::Affine;
using host::Jac;
using host::U256;
using HFq = host::Fq;
using HFq2 = host::Fq2;
using HFr = host::Fr;

// ---------------------------------------------------------------- Blake2b-512 (RFC 7693)
namespace {
constexpr uint64_t B2_IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                               0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                               0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
constexpr uint8_t B2_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};
inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
}  // namespace

Blake2b::Blake2b() {
  for (int i = 0; i < 8; ++i) h_[i] = B2_IV[i];
  h_[0] ^= 0x01010000ull ^ 64ull;  // no key, 64-byte digest
}

void Blake2b::compress(bool last) {
  uint64_t m[16], v[16];
  for (int i = 0; i < 16; ++i) {
    uint64_t x = 0;
    for (int b = 7; b >= 0; --b) x = (x << 8) | buf_[8 * i + b];
    m[i] = x;
  }
  for (int i = 0; i < 8; ++i) v[i] = h_[i], v[i + 8] = B2_IV[i];
  v[12] ^= t_[0];
  v[13] ^= t_[1];
  if (last) v[14] = ~v[14];
  auto g = [&](int a, int b, int c, int d, uint64_t x, uint64_t y) {
    v[a] = v[a] + v[b] + x;
    v[d] = rotr64(v[d] ^ v[a], 32);
    v[c] = v[c] + v[d];
    v[b] = rotr64(v[b] ^ v[c], 24);
    v[a] = v[a] + v[b] + y;
    v[d] = rotr64(v[d] ^ v[a], 16);
    v[c] = v[c] + v[d];
    v[b] = rotr64(v[b] ^ v[c], 63);
  };
  for (int r = 0; r < 12; ++r) {
    const uint8_t* s = B2_SIGMA[r];
    g(0, 4, 8, 12, m[s[0]], m[s[1]]);
    g(1, 5, 9, 13, m[s[2]], m[s[3]]);
    g(2, 6, 10, 14, m[s[4]], m[s[5]]);
    g(3, 7, 11, 15, m[s[6]], m[s[7]]);
    g(0, 5, 10, 15, m[s[8]], m[s[9]]);
    g(1, 6, 11, 12, m[s[10]], m[s[11]]);
    g(2, 7, 8, 13, m[s[12]], m[s[13]]);
    g(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
  for (int i = 0; i < 8; ++i) h_[i] ^= v[i] ^ v[i + 8];
}

void Blake2b::update(const void* data, size_t len) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  while (len > 0) {
    if (n_ == 128) {  // the buffered block is not the last one: compress it
      t_[0] += 128;
      if (t_[0] < 128) ++t_[1];
      compress(false);
      n_ = 0;
    }
    const size_t k = std::min(len, (size_t)128 - n_);
    std::memcpy(buf_ + n_, p, k);
    n_ += k, p += k, len -= k;
  }
}

void Blake2b::final(uint8_t out[64]) {
  t_[0] += n_;
  if (t_[0] < n_) ++t_[1];
  std::memset(buf_ + n_, 0, 128 - n_);
  compress(true);
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(h_[i] >> (8 * b));
}

// ---------------------------------------------------------------- ChaCha word stream
ChaChaRng::ChaChaRng(const uint32_t seed[8]) {
  const uint32_t c[4] = {0x61707865, 0x3320646E, 0x79622D32, 0x6B206574};
  for (int i = 0; i < 4; ++i) st[i] = c[i];
  for (int i = 0; i < 8; ++i) st[4 + i] = seed[i];
  for (int i = 12; i < 16; ++i) st[i] = 0;
}

uint32_t ChaChaRng::next_u32() {
  if (idx == 16) {
    auto qr = [](uint32_t* x, int a, int b, int c, int d) {
      x[a] += x[b], x[d] = rotl32(x[d] ^ x[a], 16);
      x[c] += x[d], x[b] = rotl32(x[b] ^ x[c], 12);
      x[a] += x[b], x[d] = rotl32(x[d] ^ x[a], 8);
      x[c] += x[d], x[b] = rotl32(x[b] ^ x[c], 7);
    };
    std::memcpy(buf, st, sizeof st);
    for (int r = 0; r < 10; ++r) {
      qr(buf, 0, 4, 8, 12), qr(buf, 1, 5, 9, 13), qr(buf, 2, 6, 10, 14), qr(buf, 3, 7, 11, 15);
      qr(buf, 0, 5, 10, 15), qr(buf, 1, 6, 11, 12), qr(buf, 2, 7, 8, 13), qr(buf, 3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) buf[i] += st[i];
    idx = 0;
    for (int w = 12; w < 16; ++w)
      if (++st[w] != 0) break;
  }
  return buf[idx++];
}

uint64_t ChaChaRng::next_u64() {
  const uint64_t hi = next_u32();
  return hi << 32 | next_u32();
}

void seed_from_hash(const uint8_t* h, uint32_t seed[8]) {
  for (int i = 0; i < 8; ++i)
    seed[i] = (uint32_t)h[4 * i] << 24 | (uint32_t)h[4 * i + 1] << 16 | (uint32_t)h[4 * i + 2] << 8 | h[4 * i + 3];
}

namespace {

// ---------------------------------------------------------------- field / curve draws
U256 draw254(ChaChaRng& rng, const U256& mod) {  // ffjavascript F.fromRng: 4 x u64, 254 bits, < mod
  U256 v;
  do {
    for (int i = 0; i < 4; ++i) v.w[i] = rng.next_u64();
    v.w[3] &= (uint64_t(1) << 62) - 1;
  } while (host::u256_geq(v, mod));
  return v;
}
HFq fq_from_rng(ChaChaRng& rng) { return HFq::raw(draw254(rng, host::FQ_DESC.mod)); }  // Montgomery reading
HFr fr_from_rng(ChaChaRng& rng) { return HFr::raw(draw254(rng, host::FR_DESC.mod)); }

U256 half_p() {  // (p - 1) / 2
  U256 h = host::FQ_DESC.mod;
  for (int i = 0; i < 4; ++i) h.w[i] = (h.w[i] >> 1) | (i < 3 ? h.w[i + 1] << 63 : 0);
  return h;
}
bool fq_negative(const HFq& y) {
  const U256 v = y.to_std(), h = half_p();
  return !host::u256_geq(h, v);  // v > (p - 1) / 2
}
bool fq2_negative(const HFq2& y) { return y.c1.is_zero() ? fq_negative(y.c0) : fq_negative(y.c1); }

U256 exp_of(uint64_t add, int shift_right) {  // (p + add) >> shift_right (add may be "negative" via wrap)
  U256 e = host::FQ_DESC.mod, a{{add, 0, 0, 0}};
  host::u256_add(e, a);
  for (int s = 0; s < shift_right; ++s)
    for (int i = 0; i < 4; ++i) e.w[i] = (e.w[i] >> 1) | (i < 3 ? e.w[i + 1] << 63 : 0);
  return e;
}

bool fq_sqrt(const HFq& a, HFq& out) {  // p = 3 mod 4
  const HFq s = a.pow(exp_of(1, 2));  // (p + 1) / 4
  if (!(s.sqr() == a)) return false;
  out = s;
  return true;
}

HFq2 f2_pow(HFq2 b, const U256& e) {
  HFq2 r = HFq2::one();
  for (int i = 0; i < 256; ++i) {
    if ((e.w[i >> 6] >> (i & 63)) & 1) r = r * b;
    b = b.sqr();
  }
  return r;
}

bool fq2_sqrt(const HFq2& a, HFq2& out) {  // "Square root computation over even extension fields", p = 3 mod 4
  if (a.is_zero()) {
    out = a;
    return true;
  }
  U256 e34 = host::FQ_DESC.mod;  // (p - 3) / 4
  {
    U256 three{{3, 0, 0, 0}};
    host::u256_sub(e34, three);
    for (int s = 0; s < 2; ++s)
      for (int i = 0; i < 4; ++i) e34.w[i] = (e34.w[i] >> 1) | (i < 3 ? e34.w[i + 1] << 63 : 0);
  }
  const HFq2 a1 = f2_pow(a, e34);
  const HFq2 alpha = a1.sqr() * a;
  const HFq2 a0 = f2_pow(alpha, host::FQ_DESC.mod) * alpha;
  const HFq2 minus_one{HFq::one().neg(), HFq::zero()};
  if (a0 == minus_one) return false;
  const HFq2 x0 = a1 * a;
  HFq2 x;
  if (alpha == minus_one) {
    x = HFq2{HFq::zero(), HFq::one()} * x0;
  } else {
    U256 e12 = host::FQ_DESC.mod;  // (p - 1) / 2
    U256 one{{1, 0, 0, 0}};
    host::u256_sub(e12, one);
    for (int i = 0; i < 4; ++i) e12.w[i] = (e12.w[i] >> 1) | (i < 3 ? e12.w[i + 1] << 63 : 0);
    x = f2_pow(HFq2::one() + alpha, e12) * x0;
  }
  if (!(x.sqr() == a)) return false;
  out = x;
  return true;
}

HFq fq_small(uint64_t v) { return HFq::from_std(U256{{v, 0, 0, 0}}); }

Affine<HFq> g1_from_rng(ChaChaRng& rng) {
  HFq x, y;
  bool greatest;
  for (;;) {
    x = fq_from_rng(rng);
    greatest = rng.next_bool();
    if (fq_sqrt(x.sqr() * x + fq_small(3), y)) break;
  }
  if (greatest != fq_negative(y)) y = y.neg();
  return Affine<HFq>{x, y, false};
}

Affine<HFq2> g2_from_rng(ChaChaRng& rng) {
  static const HFq2 b2 = HFq2{fq_small(3), HFq::zero()} * HFq2{fq_small(9), fq_small(1)}.inv();
  HFq2 x, y;
  bool greatest;
  for (;;) {
    x.c0 = fq_from_rng(rng);
    x.c1 = fq_from_rng(rng);
    greatest = rng.next_bool();
    if (fq2_sqrt(x.sqr() * x + b2, y)) break;
  }
  if (greatest != fq2_negative(y)) y = y.neg();
  // times the twist's cofactor 2p - r (not reduced mod r: the point is not yet in G2)
  U256 cof = host::FQ_DESC.mod;
  host::u256_add(cof, host::FQ_DESC.mod);
  host::u256_sub(cof, host::FR_DESC.mod);
  return host::jac_to_aff(host::jac_mul(host::jac_from_aff(Affine<HFq2>{x, y, false}), cof));
}

Affine<HFq2> hash_to_g2(const uint8_t transcript[64]) {
  uint32_t seed[8];
  seed_from_hash(transcript, seed);
  ChaChaRng rng(seed);
  return g2_from_rng(rng);
}

// ---------------------------------------------------------------- encodings
void put_be(const HFq& x, uint8_t* o) {  // standard form, 32 bytes big-endian
  const U256 v = x.to_std();
  for (int i = 0; i < 32; ++i) o[31 - i] = (uint8_t)(v.w[i >> 3] >> (8 * (i & 7)));
}
void g1_u(const Affine<HFq>& p, uint8_t o[64]) {
  std::memset(o, 0, 64);
  if (p.inf) {
    o[0] = 0x40;
    return;
  }
  put_be(p.x, o);
  put_be(p.y, o + 32);
}
void g2_u(const Affine<HFq2>& p, uint8_t o[128]) {
  std::memset(o, 0, 128);
  if (p.inf) {
    o[0] = 0x40;
    return;
  }
  put_be(p.x.c1, o);
  put_be(p.x.c0, o + 32);
  put_be(p.y.c1, o + 64);
  put_be(p.y.c0, o + 96);
}
// LEM (zkey layout: Montgomery, little-endian; all-zero = infinity)
HFq fq_lem(const uint8_t* p) {
  const U256 v = host::u256_from_le(p);
  if (host::u256_geq(v, host::FQ_DESC.mod)) throw ZkpError(ZKP_ERR_FORMAT, "zkey: coordinate out of range");
  return HFq::raw(v);
}
bool zero_bytes(const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (p[i]) return false;
  return true;
}
Affine<HFq> g1_lem(const uint8_t* p) {
  if (zero_bytes(p, 64)) return Affine<HFq>{HFq::zero(), HFq::zero(), true};
  return Affine<HFq>{fq_lem(p), fq_lem(p + 32), false};
}
Affine<HFq2> g2_lem(const uint8_t* p) {
  if (zero_bytes(p, 128)) return Affine<HFq2>{HFq2::zero(), HFq2::zero(), true};
  return Affine<HFq2>{HFq2{fq_lem(p), fq_lem(p + 32)}, HFq2{fq_lem(p + 64), fq_lem(p + 96)}, false};
}
void put_lem(std::vector<uint8_t>& o, const HFq& x) {
  uint8_t b[32];
  host::u256_to_le(x.v, b);
  o.insert(o.end(), b, b + 32);
}
void put_g1_lem(std::vector<uint8_t>& o, const Affine<HFq>& p) {
  if (p.inf) {
    o.insert(o.end(), 64, 0);
    return;
  }
  put_lem(o, p.x), put_lem(o, p.y);
}
void put_g2_lem(std::vector<uint8_t>& o, const Affine<HFq2>& p) {
  if (p.inf) {
    o.insert(o.end(), 128, 0);
    return;
  }
  put_lem(o, p.x.c0), put_lem(o, p.x.c1), put_lem(o, p.y.c0), put_lem(o, p.y.c1);
}
void put32(std::vector<uint8_t>& o, uint32_t v) {
  for (int i = 0; i < 4; ++i) o.push_back((uint8_t)(v >> (8 * i)));
}
uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
void u32be(Blake2b& h, uint32_t v) {
  const uint8_t b[4] = {(uint8_t)(v >> 24), (uint8_t)(v >> 16), (uint8_t)(v >> 8), (uint8_t)v};
  h.update(b, 4);
}

void hash_g1(Blake2b& h, const Affine<HFq>& p) {
  uint8_t b[64];
  g1_u(p, b);
  h.update(b, 64);
}
void hash_g2(Blake2b& h, const Affine<HFq2>& p) {
  uint8_t b[128];
  g2_u(p, b);
  h.update(b, 128);
}
void hash_pubkey(Blake2b& h, const MpcContribution& c) {
  hash_g1(h, c.delta_after);
  hash_g1(h, c.g1_s);
  hash_g1(h, c.g1_sx);
  hash_g2(h, c.g2_spx);
  h.update(c.transcript, 64);
}

Affine<HFq> g1_times(const Affine<HFq>& p, const U256& k) {
  return host::jac_to_aff(host::jac_mul(host::jac_from_aff(p), k));
}
Affine<HFq2> g2_times(const Affine<HFq2>& p, const U256& k) {
  return host::jac_to_aff(host::jac_mul(host::jac_from_aff(p), k));
}

// the "uncompressed" encoding of `count` zkey-layout points into the hash: converted by a few
// threads per block (a Venmo key holds ~34 M points), hashed in order
template <int PW>  // bytes per point: 64 (G1) or 128 (G2)
void hash_points(Blake2b& h, const uint8_t* lem, size_t count) {
  constexpr size_t BLOCK = size_t(1) << 16;
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<uint8_t> u(BLOCK * PW);
  for (size_t at = 0; at < count; at += BLOCK) {
    const size_t m = std::min(BLOCK, count - at);
    auto work = [&](size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        const uint8_t* s = lem + (at + i) * PW;
        if (PW == 64)
          g1_u(g1_lem(s), u.data() + i * PW);
        else
          g2_u(g2_lem(s), u.data() + i * PW);
      }
    };
    if (m < 4096 || nt == 1) {
      work(0, m);
    } else {
      std::vector<std::thread> th;
      for (unsigned t = 0; t < nt; ++t) th.emplace_back(work, m * t / nt, m * (t + 1) / nt);
      for (auto& t : th) t.join();
    }
    h.update(u.data(), m * PW);
  }
}

// P - Q for affine points (one inversion per call; the H hashing batches them)
void sub_batch(const uint8_t* tau_g1, size_t n, size_t lo, size_t hi, uint8_t* out_u) {
  const size_t m = hi - lo;
  std::vector<Affine<HFq>> P(m), Q(m);
  std::vector<HFq> den(m), pre(m);
  for (size_t j = 0; j < m; ++j) {
    P[j] = g1_lem(tau_g1 + (n + lo + j) * 64);
    Q[j] = g1_lem(tau_g1 + (lo + j) * 64);
    const bool plain = !P[j].inf && !Q[j].inf && !(P[j].x == Q[j].x);
    den[j] = plain ? Q[j].x - P[j].x : HFq::one();
  }
  HFq acc = HFq::one();
  for (size_t j = 0; j < m; ++j) pre[j] = acc, acc = acc * den[j];
  HFq inv = acc.inv();
  for (size_t j = m; j-- > 0;) {
    const HFq d = den[j];
    den[j] = inv * pre[j];
    inv = inv * d;
  }
  for (size_t j = 0; j < m; ++j) {
    Affine<HFq> r;
    const Affine<HFq>& p = P[j];
    const Affine<HFq> nq{Q[j].x, Q[j].y.neg(), Q[j].inf};
    if (p.inf) {
      r = nq;
    } else if (nq.inf) {
      r = p;
    } else if (p.x == nq.x) {  // P = +-Q: through the general Jacobian formulas
      r = host::jac_to_aff(host::jac_add(host::jac_from_aff(p), host::jac_from_aff(nq)));
    } else {
      const HFq lam = (nq.y - p.y) * den[j];
      const HFq x3 = lam.sqr() - p.x - nq.x;
      r = Affine<HFq>{x3, lam * (p.x - x3) - p.y, false};
    }
    g1_u(r, out_u + j * 64);
  }
}

}  // namespace

MpcParams read_mpc(const uint8_t* sec, size_t len) {
  MpcParams m;
  if (len < 68) throw ZkpError(ZKP_ERR_FORMAT, "zkey: section 10 (MPC params) is truncated");
  std::memcpy(m.cs_hash, sec, 64);
  const uint32_t n = rd32(sec + 64);
  size_t o = 68;
  for (uint32_t i = 0; i < n; ++i) {
    if (len - o < 384 + 8) throw ZkpError(ZKP_ERR_FORMAT, "zkey: section 10 contribution is truncated");
    MpcContribution c;
    c.delta_after = g1_lem(sec + o);
    c.g1_s = g1_lem(sec + o + 64);
    c.g1_sx = g1_lem(sec + o + 128);
    c.g2_spx = g2_lem(sec + o + 192);
    std::memcpy(c.transcript, sec + o + 320, 64);
    o += 384;
    c.type = rd32(sec + o);
    const uint32_t plen = rd32(sec + o + 4);
    o += 8;
    if (len - o < plen) throw ZkpError(ZKP_ERR_FORMAT, "zkey: section 10 parameters are truncated");
    c.params.assign(sec + o, sec + o + plen);
    o += plen;
    m.contributions.push_back(std::move(c));
  }
  if (o != len) throw ZkpError(ZKP_ERR_FORMAT, "zkey: section 10 has trailing bytes");
  return m;
}

std::vector<uint8_t> write_mpc(const MpcParams& m) {
  std::vector<uint8_t> o(m.cs_hash, m.cs_hash + 64);
  put32(o, (uint32_t)m.contributions.size());
  for (const MpcContribution& c : m.contributions) {
    put_g1_lem(o, c.delta_after);
    put_g1_lem(o, c.g1_s);
    put_g1_lem(o, c.g1_sx);
    put_g2_lem(o, c.g2_spx);
    o.insert(o.end(), c.transcript, c.transcript + 64);
    put32(o, c.type);
    put32(o, (uint32_t)c.params.size());
    o.insert(o.end(), c.params.begin(), c.params.end());
  }
  return o;
}

// The name bytes snarkjs writes: name.substring(0, 64) counts UTF-16 code units, then UTF-8.  A
// supplementary character (4 UTF-8 bytes) is two units; one cut in half leaves a lone high
// surrogate, which TextEncoder writes as U+FFFD.  Bytes that are not UTF-8 are copied as one unit.
static std::string mpc_name_utf8(const std::string& name) {
  std::string out;
  size_t units = 0, i = 0;
  while (i < name.size() && units < 64) {
    const uint8_t b = (uint8_t)name[i];
    const size_t len = b < 0x80 ? 1 : (b >> 5) == 6 ? 2 : (b >> 4) == 14 ? 3 : (b >> 3) == 30 ? 4 : 1;
    if (i + len > name.size()) {
      out.push_back(name[i++]);
      ++units;
      continue;
    }
    if (len == 4 && units == 63) {  // only the high surrogate fits
      out += "\xEF\xBF\xBD";
      break;
    }
    out.append(name, i, len);
    units += len == 4 ? 2 : 1;
    i += len;
  }
  return out;
}

void mpc_contribute(MpcParams& m, ChaChaRng& rng, const Affine<HFq>& delta1_before, uint32_t type,
                    const std::string& name, const uint8_t* beacon, size_t beacon_len, uint32_t num_iterations_exp,
                    uint8_t k32[32]) {
  Blake2b th;
  th.update(m.cs_hash, 64);
  for (const MpcContribution& c : m.contributions) hash_pubkey(th, c);
  const HFr kf = fr_from_rng(rng);
  if (kf.is_zero()) throw ZkpError(ZKP_ERR_INTERNAL, "contribution: zero secret drawn");
  const U256 k = kf.to_std();
  MpcContribution c;
  c.g1_s = g1_from_rng(rng);
  c.g1_sx = g1_times(c.g1_s, k);
  hash_g1(th, c.g1_s);
  hash_g1(th, c.g1_sx);
  th.final(c.transcript);
  c.g2_spx = g2_times(hash_to_g2(c.transcript), k);
  c.delta_after = g1_times(delta1_before, k);
  c.type = type;
  if (!name.empty()) {
    const std::string nm = mpc_name_utf8(name);
    c.params.push_back(1);
    c.params.push_back((uint8_t)nm.size());
    c.params.insert(c.params.end(), nm.begin(), nm.end());
  }
  if (type == 1) {
    if (beacon_len > 255 || num_iterations_exp > 255) throw ZkpError(ZKP_ERR_INVALID_ARG, "beacon: parameter too long");
    c.params.push_back(2);  // numIterationsExp: the id, then its one value byte (no length byte)
    c.params.push_back((uint8_t)num_iterations_exp);
    c.params.push_back(3);
    c.params.push_back((uint8_t)beacon_len);
    c.params.insert(c.params.end(), beacon, beacon + beacon_len);
  }
  m.contributions.push_back(std::move(c));
  host::u256_to_le(k, k32);
}

void mpc_cs_hash_new(const uint8_t* zkey, size_t len, const uint8_t* tau_g1, size_t tau_g1_points, uint8_t out[64]) {
  const ZkeyParsed z = parse_zkey(zkey, len, false);
  const ZkeyHeader& hd = z.hdr;
  const size_t n = hd.domain_size;
  const Section* s = z.bf.sec;
  if (!s[3].ptr || s[3].len != ((uint64_t)hd.n_public + 1) * 64) throw ZkpError(ZKP_ERR_FORMAT, "zkey: no IC section");
  Blake2b h;
  hash_g1(h, hd.alpha1);
  hash_g1(h, hd.beta1);
  hash_g2(h, hd.beta2);
  hash_g2(h, hd.gamma2);
  hash_g1(h, hd.delta1);
  hash_g2(h, hd.delta2);
  u32be(h, hd.n_public + 1);
  hash_points<64>(h, s[3].ptr, (size_t)hd.n_public + 1);
  // H: (tau^(n+i) - tau^i) G1 by chunks of min(n - 1, 2^14) points (the recalled snarkjs loop)
  constexpr size_t CH = size_t(1) << 14;
  u32be(h, (uint32_t)(n - 1));
  std::vector<uint8_t> hu(CH * 64);
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  for (size_t i = 0; i + 1 < n; i += CH) {
    const size_t m = std::min(n - 1, CH);
    if (n + i + m > tau_g1_points) throw ZkpError(ZKP_ERR_FORMAT, "ptau: too few tauG1 points for the circuit hash");
    if (m < 2048 || nt == 1) {
      sub_batch(tau_g1, n, i, i + m, hu.data());
    } else {
      std::vector<std::thread> th;
      for (unsigned t = 0; t < nt; ++t)
        th.emplace_back(sub_batch, tau_g1, n, i + m * t / nt, i + m * (t + 1) / nt, hu.data() + (m * t / nt) * 64);
      for (auto& t : th) t.join();
    }
    h.update(hu.data(), m * 64);
  }
  const size_t nc = (size_t)hd.n_vars - hd.n_public - 1;
  u32be(h, (uint32_t)nc);
  hash_points<64>(h, s[8].ptr, nc);
  u32be(h, hd.n_vars);
  hash_points<64>(h, s[5].ptr, hd.n_vars);
  u32be(h, hd.n_vars);
  hash_points<64>(h, s[6].ptr, hd.n_vars);
  u32be(h, hd.n_vars);
  hash_points<128>(h, s[7].ptr, hd.n_vars);
  h.final(out);
}

void binfile_replace_section(std::vector<uint8_t>& file, uint32_t id, const std::vector<uint8_t>& payload) {
  if (file.size() < 12) throw ZkpError(ZKP_ERR_FORMAT, "binfile: truncated");
  const uint32_t nsec = rd32(file.data() + 8);
  std::vector<uint8_t> out(file.begin(), file.begin() + 12);
  size_t o = 12;
  bool done = false;
  for (uint32_t i = 0; i < nsec; ++i) {
    if (file.size() - o < 12) throw ZkpError(ZKP_ERR_FORMAT, "binfile: truncated section header");
    const uint32_t sid = rd32(file.data() + o);
    uint64_t ln = 0;
    for (int b = 7; b >= 0; --b) ln = (ln << 8) | file[o + 4 + b];
    if (file.size() - o - 12 < ln) throw ZkpError(ZKP_ERR_FORMAT, "binfile: truncated section");
    const uint8_t* p = file.data() + o + 12;
    const std::vector<uint8_t>* src = nullptr;
    if (sid == id && !done) src = &payload, done = true;
    const uint64_t nl = src ? src->size() : ln;
    put32(out, sid);
    for (int b = 0; b < 8; ++b) out.push_back((uint8_t)(nl >> (8 * b)));
    if (src)
      out.insert(out.end(), src->begin(), src->end());
    else
      out.insert(out.end(), p, p + ln);
    o += 12 + ln;
  }
  if (!done) {
    put32(out, id);
    const uint64_t nl = payload.size();
    for (int b = 0; b < 8; ++b) out.push_back((uint8_t)(nl >> (8 * b)));
    out.insert(out.end(), payload.begin(), payload.end());
    out[8] = (uint8_t)(nsec + 1), out[9] = (uint8_t)((nsec + 1) >> 8), out[10] = (uint8_t)((nsec + 1) >> 16),
    out[11] = (uint8_t)((nsec + 1) >> 24);
  }
  file.swap(out);
}

}  // namespace zkp
