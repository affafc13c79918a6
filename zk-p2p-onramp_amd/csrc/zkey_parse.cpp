// Host-side parsing of snarkjs binfiles: the .wtns and .zkey readers of
// snarkjs@0.4.22 groth16_prove (rows A1-A3), restated with bounds checks on every length field.
// Host-only C++ (no device code), so the CPU suite builds it with AddressSanitizer and
// UndefinedBehaviorSanitizer and feeds it corrupted files (tools/hosttest/parse_fuzz.cpp).
#include <cstring>
#include <string>

#include "prover.hpp"

namespace zkp {

using host::Affine;
using host::U256;
using HFq = host::Fq;
using HFq2 = host::Fq2;

BinFile parse_binfile(const uint8_t* buf, size_t len, const char* magic, uint32_t max_version) {
  if (!buf || len < 12 || std::memcmp(buf, magic, 4) != 0)
    throw ZkpError(ZKP_ERR_FORMAT, std::string(magic) + ": Invalid File format");
  BinFile bf;
  uint32_t nsec;
  std::memcpy(&bf.version, buf + 4, 4);
  std::memcpy(&nsec, buf + 8, 4);
  if (bf.version > max_version) throw ZkpError(ZKP_ERR_FORMAT, std::string(magic) + ": Version not supported");
  size_t pos = 12;
  for (uint32_t i = 0; i < nsec; ++i) {
    if (pos + 12 > len) throw ZkpError(ZKP_ERR_FORMAT, std::string(magic) + ": truncated section header");
    uint32_t id;
    uint64_t sl;
    std::memcpy(&id, buf + pos, 4);
    std::memcpy(&sl, buf + pos + 4, 8);
    pos += 12;
    if (sl > len - pos) throw ZkpError(ZKP_ERR_FORMAT, std::string(magic) + ": truncated section " + std::to_string(id));
    if (id < 16 && !bf.sec[id].ptr) bf.sec[id] = Section{buf + pos, sl};
    pos += sl;
  }
  return bf;
}

static uint32_t rd32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

static const uint8_t R_LE[32] = {0x01, 0x00, 0x00, 0xf0, 0x93, 0xf5, 0xe1, 0x43, 0x91, 0x70, 0xb9, 0x79, 0x48, 0xe8, 0x33, 0x28,
                                 0x5d, 0x58, 0x81, 0x81, 0xb6, 0x45, 0x50, 0xb8, 0x29, 0xa0, 0x31, 0xe1, 0x72, 0x4e, 0x64, 0x30};
static const uint8_t P_LE[32] = {0x47, 0xfd, 0x7c, 0xd8, 0x16, 0x8c, 0x20, 0x3c, 0x8d, 0xca, 0x71, 0x68, 0x91, 0x6a, 0x81, 0x97,
                                 0x5d, 0x58, 0x81, 0x81, 0xb6, 0x45, 0x50, 0xb8, 0x29, 0xa0, 0x31, 0xe1, 0x72, 0x4e, 0x64, 0x30};

WtnsView parse_wtns(const uint8_t* buf, size_t len) {
  BinFile bf = parse_binfile(buf, len, "wtns", 2);
  const Section& s1 = bf.sec[1];
  const Section& s2 = bf.sec[2];
  if (!s1.ptr || !s2.ptr || s1.len < 4) throw ZkpError(ZKP_ERR_FORMAT, "wtns: missing header or witness section");
  const uint32_t n8 = rd32(s1.ptr);
  if (s1.len < 8 + (uint64_t)n8) throw ZkpError(ZKP_ERR_FORMAT, "wtns: bad header section");
  if (n8 != 32 || std::memcmp(s1.ptr + 4, R_LE, 32) != 0)
    throw ZkpError(ZKP_ERR_CURVE, "Curve of the witness does not match the curve of the proving key");
  WtnsView v;
  v.n_witness = rd32(s1.ptr + 4 + n8);
  if (s2.len != (uint64_t)v.n_witness * 32) throw ZkpError(ZKP_ERR_FORMAT, "wtns: Invalid witness section size");
  v.values = s2.ptr;
  return v;
}

static HFq fq_from_zkey(const uint8_t* p) {
  U256 v = host::u256_from_le(p);
  if (host::u256_geq(v, host::FQ_DESC.mod)) throw ZkpError(ZKP_ERR_FORMAT, "zkey: point coordinate out of range");
  return HFq::raw(v);  // zkey stores Montgomery(2^256) = host representation
}

static Affine<HFq> g1_from_zkey(const uint8_t* p) {
  Affine<HFq> a{fq_from_zkey(p), fq_from_zkey(p + 32), false};
  a.inf = a.x.is_zero() && a.y.is_zero();
  return a;
}

static Affine<HFq2> g2_from_zkey(const uint8_t* p) {
  Affine<HFq2> a{HFq2{fq_from_zkey(p), fq_from_zkey(p + 32)}, HFq2{fq_from_zkey(p + 64), fq_from_zkey(p + 96)}, false};
  a.inf = a.x.is_zero() && a.y.is_zero();
  return a;
}

ZkeyParsed parse_zkey(const uint8_t* buf, size_t len, bool with_coefs) {
  ZkeyParsed z;
  z.bf = parse_binfile(buf, len, "zkey", 1);
  const Section& s1 = z.bf.sec[1];
  if (!s1.ptr || s1.len < 4) throw ZkpError(ZKP_ERR_FORMAT, "zkey: missing header section");
  if (rd32(s1.ptr) != 1) throw ZkpError(ZKP_ERR_PROTOCOL, "zkey file is not groth16");
  const Section& s2 = z.bf.sec[2];
  if (!s2.ptr) throw ZkpError(ZKP_ERR_FORMAT, "zkey: missing groth16 header section");
  const uint8_t* p = s2.ptr;
  const uint8_t* end = s2.ptr + s2.len;
  auto need = [&](size_t n) {
    if ((size_t)(end - p) < n) throw ZkpError(ZKP_ERR_FORMAT, "zkey: truncated groth16 header");
  };
  need(4);
  uint32_t n8q = rd32(p);
  p += 4;
  need(n8q + 4);
  if (n8q != 32 || std::memcmp(p, P_LE, 32) != 0) throw ZkpError(ZKP_ERR_CURVE, "zkey: curve not supported (need bn128)");
  p += n8q;
  uint32_t n8r = rd32(p);
  p += 4;
  need(n8r + 12);
  if (n8r != 32 || std::memcmp(p, R_LE, 32) != 0) throw ZkpError(ZKP_ERR_CURVE, "zkey: curve not supported (need bn128)");
  p += n8r;
  ZkeyHeader& h = z.hdr;
  h.n_vars = rd32(p);
  h.n_public = rd32(p + 4);
  h.domain_size = rd32(p + 8);
  p += 12;
  need(64 * 3 + 128 * 3);
  h.alpha1 = g1_from_zkey(p);
  h.beta1 = g1_from_zkey(p + 64);
  h.beta2 = g2_from_zkey(p + 128);
  h.gamma2 = g2_from_zkey(p + 256);
  h.delta1 = g1_from_zkey(p + 384);
  h.delta2 = g2_from_zkey(p + 448);
  if (h.domain_size == 0 || (h.domain_size & (h.domain_size - 1)))
    throw ZkpError(ZKP_ERR_FORMAT, "zkey: domain size is not a power of two");
  while ((1u << h.log_domain) < h.domain_size) ++h.log_domain;
  if (h.log_domain > 27) throw ZkpError(ZKP_ERR_FORMAT, "zkey: domain larger than 2^27 not supported");
  if (h.n_vars < h.n_public + 1) throw ZkpError(ZKP_ERR_FORMAT, "zkey: nVars < nPublic + 1");
  auto chk = [&](int id, uint64_t want) {
    if (!z.bf.sec[id].ptr || z.bf.sec[id].len != want)
      throw ZkpError(ZKP_ERR_FORMAT, "zkey: section " + std::to_string(id) + " has an invalid size");
  };
  chk(5, (uint64_t)h.n_vars * 64);
  chk(6, (uint64_t)h.n_vars * 64);
  chk(7, (uint64_t)h.n_vars * 128);
  chk(8, (uint64_t)(h.n_vars - h.n_public - 1) * 64);
  chk(9, (uint64_t)h.domain_size * 64);
  const Section& s3 = z.bf.sec[3];  // IC (the verification key's public-input points)
  if (s3.ptr && s3.len == ((uint64_t)h.n_public + 1) * 64)
    for (uint32_t i = 0; i <= h.n_public; ++i) h.ic.push_back(g1_from_zkey(s3.ptr + (size_t)i * 64));
  const Section& s4 = z.bf.sec[4];
  if (!s4.ptr || s4.len < 4) throw ZkpError(ZKP_ERR_FORMAT, "zkey: missing coefficients section");
  h.n_coef = rd32(s4.ptr);
  if (s4.len != 4 + (uint64_t)h.n_coef * 44) throw ZkpError(ZKP_ERR_FORMAT, "zkey: coefficients section has an invalid size");
  if (!with_coefs) return z;
  // CSR by (matrix, constraint) with a stable counting sort
  for (int m = 0; m < 2; ++m) z.csr[m].rowptr.assign((size_t)h.domain_size + 1, 0);
  const uint8_t* c = s4.ptr + 4;
  for (uint32_t i = 0; i < h.n_coef; ++i, c += 44) {
    const uint32_t m = rd32(c), row = rd32(c + 4), sig = rd32(c + 8);
    if (m > 1 || row >= h.domain_size || sig >= h.n_vars)
      throw ZkpError(ZKP_ERR_FORMAT, "zkey: coefficient entry out of range");
    z.csr[m].rowptr[row + 1]++;
  }
  for (int m = 0; m < 2; ++m) {
    auto& rp = z.csr[m].rowptr;
    for (size_t r = 0; r < h.domain_size; ++r) rp[r + 1] += rp[r];
    z.csr[m].col.resize(rp.back());
    z.csr[m].val.resize((size_t)rp.back() * 8);
  }
  std::vector<uint32_t> fill[2] = {std::vector<uint32_t>(z.csr[0].rowptr.begin(), z.csr[0].rowptr.end() - 1),
                                   std::vector<uint32_t>(z.csr[1].rowptr.begin(), z.csr[1].rowptr.end() - 1)};
  c = s4.ptr + 4;
  for (uint32_t i = 0; i < h.n_coef; ++i, c += 44) {
    const uint32_t m = rd32(c), row = rd32(c + 4), sig = rd32(c + 8);
    const uint32_t at = fill[m][row]++;
    z.csr[m].col[at] = sig;
    std::memcpy(&z.csr[m].val[(size_t)at * 8], c + 12, 32);
  }
  return z;
}

}  // namespace zkp
