// Setup acceleration, phase 2 start: `snarkjs zkey new <circuit.r1cs>
// <pot.ptau> <circuit_0000.zkey>` (reference dizkus-scripts/3_gen_chunk_zkey.sh:18; part of the
// 782 s / 3 h key generation, zkp-mooc-hackathon-submission.md:98-99) on the GPU.
//
// From the Lagrange forms of the powers of tau (ptau sections 12-15, level k = log2 domain) every
// key point is a sparse linear combination of ptau points with the circuit's coefficients:
//   A_i  = sum_c A[c][i] L_c(tau) G1          (plus the input rows A[nc + i][i] = 1, i <= nPublic)
//   B1_i = sum_c B[c][i] L_c(tau) G1,  B2_i = the same over G2
//   IC_i (i <= nPublic, gamma = 1) / L_i (i > nPublic, delta = 1)
//        = sum_c (A[c][i] beta L_c(tau) + B[c][i] alpha L_c(tau) + C[c][i] L_c(tau)) G1
//   H_j  = L^(2n)_(2j+1)(tau) G1 -- copied from level k + 1 (delta = 1)
// Each point's terms are cut into tasks of <= LIN_TASK terms; a task is one multi-scalar sum by
// Shamir's trick (one shared doubling chain over the scalars' bits, one mixed addition per set
// bit, on the prover's field/curve code), its partials summed per point, then affine and back to
// the zkey encoding.  The header points: alpha1 = alphaTauG1[0], beta1 = betaTauG1[0], beta2 =
// betaG2, gamma2 = delta2 = G2, delta1 = G1.  Section 10 is the empty contribution list with the
// circuit hash (csHash, mpc.cpp / oracle/mpc.py: Blake2b-512 over the key's points and the ptau's
// tauG1 powers), which `zkey verify` recomputes from the r1cs and ptau.
// ptau / r1cs layouts: oracle/binfile.py write_ptau / write_r1cs (recalled, unpinned offline).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "curve.hpp"
#include "hip_check.hpp"
#include "host_ec.hpp"
#include "mpc.hpp"
#include "prover.hpp"
#include "qap.hpp"

namespace zkp {

namespace {

constexpr int TPB = 256;
constexpr uint32_t LIN_TASK = 16;  // terms per Shamir task

struct Words8 {
  uint32_t w[8];
};

// task k = terms [tlo[k], tlo[k+1]): sum_t s_t * P[idx_t] by one shared double-and-add chain
template <class F>
__global__ __launch_bounds__(TPB) void k_lin_tasks(const uint32_t* __restrict__ bases, const uint32_t* __restrict__ tidx,
                                                   const uint32_t* __restrict__ tscal, const uint32_t* __restrict__ tlo,
                                                   uint32_t ntasks, uint32_t* __restrict__ partial) {
  const uint32_t k = blockIdx.x * TPB + threadIdx.x;
  if (k >= ntasks) return;
  const uint32_t lo = tlo[k], hi = tlo[k + 1];
  int top = -1;
  for (uint32_t t = lo; t < hi; ++t)
    for (int w = 7; w >= 0; --w) {
      const uint32_t x = tscal[(size_t)t * 8 + w];
      if (x) {
        top = std::max(top, w * 32 + 31 - __builtin_clz(x));
        break;
      }
    }
  Xyzz<F> acc = xyzz_inf<F>();
  for (int b = top; b >= 0; --b) {
    acc = xyzz_dbl(acc);
    for (uint32_t t = lo; t < hi; ++t)
      if ((tscal[(size_t)t * 8 + (b >> 5)] >> (b & 31)) & 1u) xyzz_add_aff(acc, load_aff<F>(bases, tidx[t]));
  }
  store_xyzz(partial, k, acc);
}

// point r = the sum of its tasks' partials, affine, in the zkey encoding (Montgomery 2^256,
// canonical; infinity = zero words), written at out + r * (point words)
template <class F>
__global__ __launch_bounds__(TPB) void k_lin_rows(const uint32_t* __restrict__ partial,
                                                  const uint32_t* __restrict__ rowtask, uint32_t nrows, Words8 to_zkey,
                                                  uint32_t* __restrict__ out) {
  const uint32_t r = blockIdx.x * TPB + threadIdx.x;
  if (r >= nrows) return;
  Xyzz<F> acc = xyzz_inf<F>();
  for (uint32_t k = rowtask[r]; k < rowtask[r + 1]; ++k) xyzz_add(acc, load_xyzz<F>(partial, k));
  constexpr int W = FWords<F>::W;
  if (xyzz_is_inf(acc)) {
    for (int j = 0; j < 2 * W; ++j) out[(size_t)r * 2 * W + j] = 0;
    return;
  }
  Aff<F> a = xyzz_to_aff(acc);
  const Fq conv = unpack<FqCfg>(to_zkey.w);  // mont(x_dev, 2^256 mod p) = x 2^256 mod p
  auto cvt = [&](F& x) {
    if constexpr (W == 8) {
      x = canon(mul(x, conv));
    } else {
      x.c0 = canon(mul(x.c0, conv));
      x.c1 = canon(mul(x.c1, conv));
    }
  };
  cvt(a.x);
  cvt(a.y);
  store_aff(out, r, a);
}

struct Term {
  uint32_t row, point;
  host::U256 s;  // standard form, < r
};

template <class T>
static void put(std::vector<uint8_t>& o, const T& v) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
  o.insert(o.end(), p, p + sizeof(T));
}
static void put_bytes(std::vector<uint8_t>& o, const void* p, size_t n) {
  const uint8_t* b = static_cast<const uint8_t*>(p);
  o.insert(o.end(), b, b + n);
}
static void put_u256(std::vector<uint8_t>& o, const host::U256& v) { put_bytes(o, v.w, 32); }
static host::U256 u256_le(const uint8_t* p) {
  host::U256 v;
  std::memcpy(v.w, p, 32);
  return v;
}
static host::U256 reduce_r(host::U256 v) {
  while (host::u256_geq(v, host::FR_DESC.mod)) host::u256_sub(v, host::FR_DESC.mod);
  return v;
}

// the points of one key section: sum over each row's terms, on the GPU; returns rows x pw bytes
template <class F>
static std::vector<uint8_t> lincomb(int device, hipStream_t st, const uint32_t* d_bases, std::vector<Term> terms,
                                    uint32_t nrows) {
  constexpr size_t PB = 2 * FWords<F>::W * 4;  // bytes per affine point (64 / 128)
  std::vector<uint8_t> out(nrows * PB, 0);
  if (!nrows) return out;
  std::stable_sort(terms.begin(), terms.end(), [](const Term& a, const Term& b) { return a.row < b.row; });
  std::vector<uint32_t> tidx(terms.size()), tscal(terms.size() * 8), tlo, rowtask(nrows + 1, 0);
  for (size_t t = 0; t < terms.size(); ++t) {
    tidx[t] = terms[t].point;
    for (int i = 0; i < 4; ++i) {
      tscal[t * 8 + 2 * i] = (uint32_t)terms[t].s.w[i];
      tscal[t * 8 + 2 * i + 1] = (uint32_t)(terms[t].s.w[i] >> 32);
    }
  }
  // tasks: runs of <= LIN_TASK terms inside one row
  size_t t = 0;
  for (uint32_t r = 0; r < nrows; ++r) {
    rowtask[r] = (uint32_t)tlo.size();
    while (t < terms.size() && terms[t].row == r) {
      tlo.push_back((uint32_t)t);
      size_t e = t;
      while (e < terms.size() && terms[e].row == r && e - t < LIN_TASK) ++e;
      t = e;
    }
  }
  rowtask[nrows] = (uint32_t)tlo.size();
  const uint32_t ntasks = (uint32_t)tlo.size();
  tlo.push_back((uint32_t)terms.size());
  HIPX(hipSetDevice(device));
  uint32_t *d_idx = nullptr, *d_scal = nullptr, *d_tlo = nullptr, *d_rowtask = nullptr, *d_part = nullptr,
           *d_out = nullptr;
  auto release = [&] {
    for (void* p : {(void*)d_idx, (void*)d_scal, (void*)d_tlo, (void*)d_rowtask, (void*)d_part, (void*)d_out})
      if (p) (void)hipFree(p);
  };
  try {
    HIPX(hipMalloc(&d_idx, std::max<size_t>(tidx.size(), 1) * 4));
    HIPX(hipMalloc(&d_scal, std::max<size_t>(tscal.size(), 1) * 4));
    HIPX(hipMalloc(&d_tlo, tlo.size() * 4));
    HIPX(hipMalloc(&d_rowtask, rowtask.size() * 4));
    HIPX(hipMalloc(&d_part, std::max<size_t>(ntasks, 1) * 4 * FWords<F>::W * 4));
    HIPX(hipMalloc(&d_out, out.size()));
    if (!tidx.empty()) {
      HIPX(hipMemcpyAsync(d_idx, tidx.data(), tidx.size() * 4, hipMemcpyHostToDevice, st));
      HIPX(hipMemcpyAsync(d_scal, tscal.data(), tscal.size() * 4, hipMemcpyHostToDevice, st));
    }
    HIPX(hipMemcpyAsync(d_tlo, tlo.data(), tlo.size() * 4, hipMemcpyHostToDevice, st));
    HIPX(hipMemcpyAsync(d_rowtask, rowtask.data(), rowtask.size() * 4, hipMemcpyHostToDevice, st));
    if (ntasks)
      hipLaunchKernelGGL(k_lin_tasks<F>, dim3((ntasks + TPB - 1) / TPB), dim3(TPB), 0, st, d_bases, d_idx, d_scal,
                         d_tlo, ntasks, d_part);
    Words8 tz;
    const host::U256 one = host::Fq::one().v;  // Montgomery one = 2^256 mod p
    for (int i = 0; i < 4; ++i) tz.w[2 * i] = (uint32_t)one.w[i], tz.w[2 * i + 1] = (uint32_t)(one.w[i] >> 32);
    hipLaunchKernelGGL(k_lin_rows<F>, dim3((nrows + TPB - 1) / TPB), dim3(TPB), 0, st, d_part, d_rowtask, nrows, tz,
                       d_out);
    HIPX(hipGetLastError());
    HIPX(hipMemcpyAsync(out.data(), d_out, out.size(), hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));
  } catch (...) {
    release();
    throw;
  }
  release();
  return out;
}

// a zkey-encoded point array (affine, Montgomery 2^256) uploaded in the device layout
static uint32_t* upload_points(const uint8_t* src, size_t count, size_t pw, hipStream_t st) {
  uint32_t* d = nullptr;
  HIPX(hipMalloc(&d, std::max<size_t>(count * pw, 4)));
  if (count) {
    HIPX(hipMemcpyAsync(d, src, count * pw, hipMemcpyHostToDevice, st));
    launch_convert_fq_zkey(d, count * pw / 32, st);
  }
  return d;
}

}  // namespace

std::vector<uint8_t> zkey_new(int device, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* ptau, size_t ptau_len) {
  // ---- r1cs
  BinFile rb = parse_binfile(r1cs, r1cs_len, "r1cs", 1);
  if (!rb.sec[1].ptr || !rb.sec[2].ptr) throw ZkpError(ZKP_ERR_FORMAT, "r1cs: missing header or constraints");
  const uint8_t* h = rb.sec[1].ptr;
  if (rb.sec[1].len < 4 + 32 + 16 + 8 + 4) throw ZkpError(ZKP_ERR_FORMAT, "r1cs: short header");
  uint32_t n8, n_vars, n_out, n_pub_in, n_prv, n_cons;
  std::memcpy(&n8, h, 4);
  if (n8 != 32) throw ZkpError(ZKP_ERR_FORMAT, "r1cs: field size is not 32 bytes");
  if (std::memcmp(u256_le(h + 4).w, host::FR_DESC.mod.w, 32) != 0)
    throw ZkpError(ZKP_ERR_CURVE, "r1cs: prime is not the bn128 scalar field");
  std::memcpy(&n_vars, h + 36, 4);
  std::memcpy(&n_out, h + 40, 4);
  std::memcpy(&n_pub_in, h + 44, 4);
  std::memcpy(&n_prv, h + 48, 4);
  std::memcpy(&n_cons, h + 60, 4);
  const uint32_t n_pub = n_out + n_pub_in;
  if (n_pub + 1 > n_vars) throw ZkpError(ZKP_ERR_FORMAT, "r1cs: more public signals than wires");
  struct Lin {
    uint32_t s;
    host::U256 v;
  };
  std::vector<std::vector<Lin>> lc[3];
  for (auto& m : lc) m.resize(n_cons);
  {
    const uint8_t* p = rb.sec[2].ptr;
    const uint8_t* e = p + rb.sec[2].len;
    for (uint32_t c = 0; c < n_cons; ++c)
      for (int m = 0; m < 3; ++m) {
        if (p + 4 > e) throw ZkpError(ZKP_ERR_FORMAT, "r1cs: truncated constraints");
        uint32_t k;
        std::memcpy(&k, p, 4);
        p += 4;
        if ((size_t)(e - p) < (size_t)k * 36) throw ZkpError(ZKP_ERR_FORMAT, "r1cs: truncated constraints");
        lc[m][c].resize(k);
        for (uint32_t j = 0; j < k; ++j, p += 36) {
          std::memcpy(&lc[m][c][j].s, p, 4);
          if (lc[m][c][j].s >= n_vars) throw ZkpError(ZKP_ERR_FORMAT, "r1cs: wire index out of range");
          lc[m][c][j].v = reduce_r(u256_le(p + 4));
        }
      }
  }
  // ---- domain and ptau
  uint32_t k = 0;
  while ((uint64_t(1) << k) < (uint64_t)n_cons + n_pub + 1) ++k;
  const uint32_t n = 1u << k;
  BinFile pb = parse_binfile(ptau, ptau_len, "ptau", 1);
  for (int id : {1, 2, 4, 5, 6, 12, 13, 14, 15})
    if (!pb.sec[id].ptr) throw ZkpError(ZKP_ERR_FORMAT, "ptau: missing section " + std::to_string(id));
  uint32_t pn8, power;
  std::memcpy(&pn8, pb.sec[1].ptr, 4);
  if (pn8 != 32 || pb.sec[1].len < 4 + 32 + 8) throw ZkpError(ZKP_ERR_FORMAT, "ptau: bad header");
  if (std::memcmp(u256_le(pb.sec[1].ptr + 4).w, host::FQ_DESC.mod.w, 32) != 0)
    throw ZkpError(ZKP_ERR_CURVE, "ptau: curve is not bn128");
  std::memcpy(&power, pb.sec[1].ptr + 36, 4);
  if (k + 1 > power)
    throw ZkpError(ZKP_ERR_INVALID_ARG, "circuit too big for this power of tau ceremony: domain 2^" +
                                            std::to_string(k) + " needs power >= " + std::to_string(k + 1));
  const uint64_t nlag = (uint64_t(2) << power) - 1;
  if (pb.sec[12].len != nlag * 64 || pb.sec[14].len != nlag * 64 || pb.sec[15].len != nlag * 64 ||
      pb.sec[13].len != nlag * 128 || pb.sec[4].len < 64 || pb.sec[5].len < 64 || pb.sec[6].len != 128)
    throw ZkpError(ZKP_ERR_FORMAT, "ptau: section sizes do not match its power");
  const size_t lvl_k = ((size_t)1 << k) - 1, lvl_k1 = ((size_t)2 << k) - 1;  // first point of a level
  // ---- terms (rows = signals)
  std::vector<Term> ta, tb, tl;
  ta.reserve((size_t)n_cons * 2 + n_pub + 1);
  for (uint32_t c = 0; c < n_cons; ++c) {
    for (auto& x : lc[0][c]) {
      ta.push_back({x.s, c, x.v});
      tl.push_back({x.s, 2 * n + c, x.v});  // beta L_c
    }
    for (auto& x : lc[1][c]) {
      tb.push_back({x.s, c, x.v});
      tl.push_back({x.s, n + c, x.v});  // alpha L_c
    }
    for (auto& x : lc[2][c]) tl.push_back({x.s, c, x.v});
  }
  const host::U256 one_std{{1, 0, 0, 0}};
  for (uint32_t i = 0; i <= n_pub; ++i) {  // input rows A[nc + i][i] = 1
    ta.push_back({i, n_cons + i, one_std});
    tl.push_back({i, 2 * n + n_cons + i, one_std});
  }
  // ---- the GPU sections
  HIPX(hipSetDevice(device));
  hipStream_t st;
  HIPX(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t *g1b = nullptr, *g2b = nullptr;
  std::vector<uint8_t> sa, sb1, sb2, sl;
  try {
    // G1 bases: [lTauG1 | lAlphaTauG1 | lBetaTauG1] of level k; G2: lTauG2 of level k
    std::vector<uint8_t> cat((size_t)3 * n * 64);
    std::memcpy(cat.data(), pb.sec[12].ptr + lvl_k * 64, (size_t)n * 64);
    std::memcpy(cat.data() + (size_t)n * 64, pb.sec[14].ptr + lvl_k * 64, (size_t)n * 64);
    std::memcpy(cat.data() + (size_t)2 * n * 64, pb.sec[15].ptr + lvl_k * 64, (size_t)n * 64);
    g1b = upload_points(cat.data(), (size_t)3 * n, 64, st);
    g2b = upload_points(pb.sec[13].ptr + lvl_k * 128, n, 128, st);
    sa = lincomb<Fq>(device, st, g1b, std::move(ta), n_vars);
    sb1 = lincomb<Fq>(device, st, g1b, tb, n_vars);
    sb2 = lincomb<Fq2>(device, st, g2b, std::move(tb), n_vars);
    sl = lincomb<Fq>(device, st, g1b, std::move(tl), n_vars);
  } catch (...) {
    if (g1b) (void)hipFree(g1b);
    if (g2b) (void)hipFree(g2b);
    (void)hipStreamDestroy(st);
    throw;
  }
  HIPX(hipFree(g1b));
  HIPX(hipFree(g2b));
  HIPX(hipStreamDestroy(st));
  // ---- assemble the zkey (sections 1..10 in order)
  auto lem_fq = [](const host::U256& v, std::vector<uint8_t>& o) { put_u256(o, host::Fq::from_std(v).v); };
  auto u256 = [](const char* dec) {  // decimal -> U256 (generator constants)
    host::U256 v{{0, 0, 0, 0}};
    for (const char* c = dec; *c; ++c) {
      host::u128 carry = (host::u128)(*c - '0');
      for (int i = 0; i < 4; ++i) {
        host::u128 t = (host::u128)v.w[i] * 10 + carry;
        v.w[i] = (host::u64)t;
        carry = t >> 64;
      }
    }
    return v;
  };
  std::vector<uint8_t> g1gen, g2gen;
  lem_fq(host::U256{{1, 0, 0, 0}}, g1gen);
  lem_fq(host::U256{{2, 0, 0, 0}}, g1gen);
  for (const char* d : {"10857046999023057135944570762232829481370756359578518086990519993285655852781",
                        "11559732032986387107991004021392285783925812861821192530917403151452391805634",
                        "8495653923123431417604973247489272438418190587263600148770280649306958101930",
                        "4082367875863433681332203403145435568316851327593401208105741076214120093531"})
    lem_fq(u256(d), g2gen);  // G2 generator (x.c0, x.c1, y.c0, y.c1): Verifier.sol:33-36
  std::vector<std::pair<uint32_t, std::vector<uint8_t>>> secs;
  {
    std::vector<uint8_t> s1;
    put(s1, (uint32_t)1);
    secs.push_back({1, std::move(s1)});
  }
  {
    std::vector<uint8_t> s2;
    put(s2, (uint32_t)32);
    put_u256(s2, host::FQ_DESC.mod);
    put(s2, (uint32_t)32);
    put_u256(s2, host::FR_DESC.mod);
    put(s2, n_vars);
    put(s2, n_pub);
    put(s2, n);
    put_bytes(s2, pb.sec[4].ptr, 64);   // alpha1 = alphaTauG1[0]
    put_bytes(s2, pb.sec[5].ptr, 64);   // beta1 = betaTauG1[0]
    put_bytes(s2, pb.sec[6].ptr, 128);  // beta2
    put_bytes(s2, g2gen.data(), 128);   // gamma2
    put_bytes(s2, g1gen.data(), 64);    // delta1
    put_bytes(s2, g2gen.data(), 128);   // delta2
    secs.push_back({2, std::move(s2)});
  }
  secs.push_back({3, std::vector<uint8_t>(sl.begin(), sl.begin() + (size_t)(n_pub + 1) * 64)});
  {
    // coefficients X = coef * 2^512 mod r (snarkjs: a Montgomery multiply by X gives coef * w)
    auto r2 = [](const host::U256& v) { return host::Fr::from_std(host::Fr::from_std(v).v).v; };
    std::vector<uint8_t> s4;
    uint32_t cnt = 0;
    for (uint32_t c = 0; c < n_cons; ++c) cnt += (uint32_t)(lc[0][c].size() + lc[1][c].size());
    cnt += n_pub + 1;
    put(s4, cnt);
    for (uint32_t c = 0; c < n_cons; ++c)
      for (uint32_t m = 0; m < 2; ++m)
        for (auto& x : lc[m][c]) {
          put(s4, m);
          put(s4, c);
          put(s4, x.s);
          put_u256(s4, r2(x.v));
        }
    for (uint32_t i = 0; i <= n_pub; ++i) {
      put(s4, (uint32_t)0);
      put(s4, n_cons + i);
      put(s4, i);
      put_u256(s4, r2(one_std));
    }
    secs.push_back({4, std::move(s4)});
  }
  secs.push_back({5, std::move(sa)});
  secs.push_back({6, std::move(sb1)});
  secs.push_back({7, std::move(sb2)});
  secs.push_back({8, std::vector<uint8_t>(sl.begin() + (size_t)(n_pub + 1) * 64, sl.end())});
  {
    std::vector<uint8_t> s9((size_t)n * 64);
    for (uint32_t j = 0; j < n; ++j) std::memcpy(s9.data() + (size_t)j * 64, pb.sec[12].ptr + (lvl_k1 + 2 * j + 1) * 64, 64);
    secs.push_back({9, std::move(s9)});
  }
  {
    std::vector<uint8_t> s10(64, 0);
    put(s10, (uint32_t)0);
    secs.push_back({10, std::move(s10)});
  }
  std::vector<uint8_t> out;
  size_t total = 12;
  for (auto& s : secs) total += 12 + s.second.size();
  out.reserve(total);
  put_bytes(out, "zkey", 4);
  put(out, (uint32_t)1);
  put(out, (uint32_t)secs.size());
  for (auto& s : secs) {
    put(out, s.first);
    put(out, (uint64_t)s.second.size());
    put_bytes(out, s.second.data(), s.second.size());
  }
  // section 10 (the last, 68 bytes): the circuit hash over the new key's points and the ptau's
  // tauG1 powers, as `snarkjs zkey new` writes it (mpc.cpp; `zkey verify` compares it)
  mpc_cs_hash_new(out.data(), out.size(), pb.sec[2].ptr, (size_t)(pb.sec[2].len / 64), out.data() + out.size() - 68);
  return out;
}

}  // namespace zkp
