// Setup acceleration: the group arithmetic of a Groth16 phase-2
// contribution, `snarkjs zkey contribute` / `zkey beacon` (reference
// dizkus-scripts/3_gen_chunk_zkey.sh:27,36 and circuit/server-scripts/
// generate_chunked_keys_phase2_groth16.sh:62; 782 s / 3 h published,
// zkp-mooc-hackathon-submission.md:98-99).  A contribution with secret k replaces
// delta by k*delta: delta1, delta2 (section 2) are multiplied by k, and every point of
// the L section (8, C bases) and of the H section (9) -- both carry delta^-1 -- by k^-1.
// That is ~15 M fixed-scalar multiplications for the Venmo key, all here, one thread
// per point (left-to-right double-and-add over the common scalar: warp-uniform
// branches), on the same field/curve code as the prover.  The contribution record in
// section 10 (transcript hash, proof of knowledge) is copied unchanged: its byte
// format belongs to snarkjs and is not reproduced.
#include <cstring>
#include <vector>

#include "curve.hpp"
#include "hip_check.hpp"
#include "host_ec.hpp"
#include "prover.hpp"
#include "qap.hpp"

namespace zkp {

namespace {

constexpr int TPB = 256;

struct Scalar8 {
  uint32_t w[8];  // standard form, LE
};

// p <- k * p for zkey-layout affine points (Montgomery 2^256 LE; all-zero = infinity), in
// place: convert in, double-and-add over k's bits, back to affine, convert out
template <class F>
__global__ __launch_bounds__(TPB) void k_scale_points(uint32_t* __restrict__ pts, size_t n, Scalar8 k,
                                                      Scalar8 to_zkey) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  constexpr int W = FWords<F>::W;
  uint32_t* p = pts + i * 2 * W;
  bool inf = true;
  for (int j = 0; j < 2 * W; ++j) inf &= p[j] == 0;
  if (inf) return;
  const Fq conv_in = fe_const<FqCfg>(Conv::FQ_ZKEY_TO_DEV);
  Aff<F> a = load_aff<F>(pts, i);
  auto cvt = [&](F& x, const Fq& c) {
    if constexpr (W == 8) {
      x = mul(x, c);
    } else {
      x.c0 = mul(x.c0, c);
      x.c1 = mul(x.c1, c);
    }
  };
  cvt(a.x, conv_in);
  cvt(a.y, conv_in);
  Xyzz<F> acc = xyzz_inf<F>();
  int top = 255;
  while (top >= 0 && !((k.w[top >> 5] >> (top & 31)) & 1u)) --top;
  for (int b = top; b >= 0; --b) {
    acc = xyzz_dbl(acc);
    if ((k.w[b >> 5] >> (b & 31)) & 1u) xyzz_add_aff(acc, a);
  }
  Aff<F> r = xyzz_to_aff(acc);
  uint32_t tz[8];
  for (int j = 0; j < 8; ++j) tz[j] = to_zkey.w[j];
  const Fq conv_out = unpack<FqCfg>(tz);  // mont(x_dev, 2^256 mod p) = x * 2^256 mod p
  auto out = [&](F& x) {
    if constexpr (W == 8) {
      x = canon(mul(x, conv_out));
    } else {
      x.c0 = canon(mul(x.c0, conv_out));
      x.c1 = canon(mul(x.c1, conv_out));
    }
  };
  if (xyzz_is_inf(acc)) {  // k*P = infinity (k = 0 mod r)
    for (int j = 0; j < 2 * W; ++j) p[j] = 0;
    return;
  }
  out(r.x);
  out(r.y);
  store_aff(pts, i, r);
}

Scalar8 to_scalar8(const host::U256& v) {
  Scalar8 s;
  for (int i = 0; i < 4; ++i) {
    s.w[2 * i] = (uint32_t)v.w[i];
    s.w[2 * i + 1] = (uint32_t)(v.w[i] >> 32);
  }
  return s;
}

// multiply `count` zkey-layout points at `src` (G1 or G2) by k on `device`, into dst
void scale_section(int device, bool g2, const uint8_t* src, uint8_t* dst, size_t count, const host::U256& k) {
  if (!count) return;
  HIPX(hipSetDevice(device));
  const size_t pb = g2 ? 128 : 64;
  const size_t CH = size_t(1) << 22;  // points per launch: bounded launches, bounded buffer
  uint32_t* d = nullptr;
  HIPX(hipMalloc(&d, std::min(count, CH) * pb));
  hipStream_t st;
  HIPX(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const Scalar8 ks = to_scalar8(k);
  const Scalar8 tz = to_scalar8(host::Fq::one().v);  // Montgomery one = 2^256 mod p
  try {
    for (size_t at = 0; at < count; at += CH) {
      const size_t m = std::min(CH, count - at);
      HIPX(hipMemcpyAsync(d, src + at * pb, m * pb, hipMemcpyHostToDevice, st));
      const unsigned grid = (unsigned)((m + TPB - 1) / TPB);
      if (g2)
        hipLaunchKernelGGL(k_scale_points<Fq2>, dim3(grid), dim3(TPB), 0, st, d, m, ks, tz);
      else
        hipLaunchKernelGGL(k_scale_points<Fq>, dim3(grid), dim3(TPB), 0, st, d, m, ks, tz);
      HIPX(hipGetLastError());
      HIPX(hipMemcpyAsync(dst + at * pb, d, m * pb, hipMemcpyDeviceToHost, st));
      HIPX(hipStreamSynchronize(st));
    }
  } catch (...) {
    (void)hipFree(d);
    (void)hipStreamDestroy(st);
    throw;
  }
  HIPX(hipFree(d));
  HIPX(hipStreamDestroy(st));
}

}  // namespace

std::vector<uint8_t> zkey_apply_delta(int device, const uint8_t* zkey, size_t len, const uint8_t* k32) {
  BinFile bf = parse_binfile(zkey, len, "zkey", 1);
  for (int id : {1, 2, 8, 9})
    if (!bf.sec[id].ptr) throw ZkpError(ZKP_ERR_FORMAT, "zkey: missing section " + std::to_string(id));
  uint32_t proto;
  std::memcpy(&proto, bf.sec[1].ptr, 4);
  if (proto != 1) throw ZkpError(ZKP_ERR_PROTOCOL, "zkey file is not groth16");
  host::U256 k = host::u256_from_le(k32);
  while (host::u256_geq(k, host::FR_DESC.mod)) host::u256_sub(k, host::FR_DESC.mod);
  if (host::u256_is_zero(k)) throw ZkpError(ZKP_ERR_INVALID_ARG, "contribution scalar must be nonzero mod r");
  const host::U256 kinv = host::Fr::from_std(k).inv().to_std();
  std::vector<uint8_t> out(zkey, zkey + len);
  auto off = [&](const Section& s) { return (size_t)(s.ptr - zkey); };
  // section 2: n8q q n8r r nVars nPublic domainSize alpha1 beta1 beta2 gamma2 delta1 delta2
  const size_t hdr = off(bf.sec[2]) + 4 + 32 + 4 + 32 + 12;
  if (bf.sec[2].len < 4 + 32 + 4 + 32 + 12 + 64 * 3 + 128 * 3) throw ZkpError(ZKP_ERR_FORMAT, "zkey: short header");
  const size_t d1 = hdr + 64 + 64 + 128 + 128, d2 = d1 + 64;
  scale_section(device, false, zkey + d1, out.data() + d1, 1, k);
  scale_section(device, true, zkey + d2, out.data() + d2, 1, k);
  if (bf.sec[8].len % 64 || bf.sec[9].len % 64) throw ZkpError(ZKP_ERR_FORMAT, "zkey: bad L/H section size");
  scale_section(device, false, bf.sec[8].ptr, out.data() + off(bf.sec[8]), bf.sec[8].len / 64, kinv);
  scale_section(device, false, bf.sec[9].ptr, out.data() + off(bf.sec[9]), bf.sec[9].len / 64, kinv);
  return out;
}

}  // namespace zkp
