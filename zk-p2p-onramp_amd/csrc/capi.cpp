// C ABI of libzkp_amd.so (include/zkp_amd.h).  Every entry point catches all C++
// exceptions and turns them into a zkp_status plus a thread-local message.
#include <stdexcept>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <fstream>
#include <new>
#include <string>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../../include/zkp_amd.h"
#include "beacon.hpp"
#include "hip_check.hpp"
#include "host_ec.hpp"
#include "host_pairing.hpp"
#include "mpc.hpp"
#include "prover.hpp"
#include "zkey_io.hpp"

static_assert(sizeof(zkp_partial) == 392, "zkp_partial is exchanged as 392 raw bytes");

struct zkp_prover {
  zkp::Prover* impl;
};

namespace {

thread_local std::string g_err;

zkp_status fail(zkp_status s, const std::string& m) {
  g_err = m;
  return s;
}

template <class Fn>
zkp_status guard(Fn&& fn) {
  try {
    g_err.clear();
    fn();
    return ZKP_OK;
  } catch (const zkp::ZkpError& e) {
    return fail(e.status, e.what());
  } catch (const zkp::HipError& e) {
    if (e.code == hipErrorOutOfMemory) return fail(ZKP_ERR_OUT_OF_MEMORY, e.what());
    return fail(ZKP_ERR_DEVICE, e.what());
  } catch (const std::bad_alloc&) {
    return fail(ZKP_ERR_OUT_OF_MEMORY, "host out of memory");
  } catch (const std::invalid_argument& e) {
    return fail(ZKP_ERR_INVALID_ARG, e.what());
  } catch (const std::exception& e) {
    return fail(ZKP_ERR_INTERNAL, e.what());
  } catch (...) {
    return fail(ZKP_ERR_INTERNAL, "unknown error");
  }
}

std::vector<uint8_t> read_file(const char* path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) throw zkp::ZkpError(ZKP_ERR_IO, std::string("cannot open ") + path);
  const std::streamsize n = f.tellg();
  f.seekg(0);
  std::vector<uint8_t> buf((size_t)n);
  if (n && !f.read(reinterpret_cast<char*>(buf.data()), n))
    throw zkp::ZkpError(ZKP_ERR_IO, std::string("cannot read ") + path);
  return buf;
}

// A witness file mapped read-only: the prover's transfer threads read the page cache directly (the
// page faults spread over them) instead of one thread copying 205 MB into a zero-filled buffer
// first.  Regular files only; anything else (a pipe, a device, a procfs node) and a file that cannot
// be mapped is read into a buffer (read_file).  A mapped file must not be truncated by another writer
// while the call runs (the read of a page past the new end would raise SIGBUS): include/zkp_amd.h
// states this for zkp_prove_files.
class MappedFile {
 public:
  explicit MappedFile(const char* path) {
    const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) throw zkp::ZkpError(ZKP_ERR_IO, std::string("cannot open ") + path);
    struct stat st {};
    if (::fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0) {
      void* m = ::mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m != MAP_FAILED) {
        map_ = m;
        len_ = (size_t)st.st_size;
      }
    }
    ::close(fd);
    if (!map_) copy_ = read_file(path);
  }
  ~MappedFile() {
    if (map_) ::munmap(map_, len_);
  }
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
  const uint8_t* data() const { return map_ ? static_cast<const uint8_t*>(map_) : copy_.data(); }
  size_t size() const { return map_ ? len_ : copy_.size(); }

 private:
  void* map_ = nullptr;
  size_t len_ = 0;
  std::vector<uint8_t> copy_;
};

std::string dec(const uint8_t* le32) { return zkp::host::u256_to_dec(zkp::host::u256_from_le(le32)); }

// JSON.stringify(obj, null, 1) of snarkjs' proof object (key order pi_a, pi_b, pi_c, protocol, curve)
std::string proof_json(const zkp_proof* p) {
  std::string s = "{\n \"pi_a\": [\n  \"" + dec(p->pi_a[0]) + "\",\n  \"" + dec(p->pi_a[1]) + "\",\n  \"1\"\n ],\n";
  s += " \"pi_b\": [\n  [\n   \"" + dec(p->pi_b[0][0]) + "\",\n   \"" + dec(p->pi_b[0][1]) + "\"\n  ],\n  [\n   \"" +
       dec(p->pi_b[1][0]) + "\",\n   \"" + dec(p->pi_b[1][1]) + "\"\n  ],\n  [\n   \"1\",\n   \"0\"\n  ]\n ],\n";
  s += " \"pi_c\": [\n  \"" + dec(p->pi_c[0]) + "\",\n  \"" + dec(p->pi_c[1]) + "\",\n  \"1\"\n ],\n";
  s += " \"protocol\": \"groth16\",\n \"curve\": \"bn128\"\n}";
  return s;
}

std::string public_json(const zkp_proof* p) {
  const uint32_t n = std::min(p->n_public, p->public_capacity);
  if (n == 0 || !p->public_signals) return "[]";
  std::string s = "[\n";
  for (uint32_t i = 0; i < n; ++i) {
    s += " \"" + dec(p->public_signals + 32 * i) + "\"";
    s += (i + 1 < n) ? ",\n" : "\n";
  }
  s += "]";
  return s;
}

// "0x" + 64 hex digits of a 32-byte LE integer, quoted (snarkjs p256)
std::string p256(const uint8_t* le32) {
  static const char* hx = "0123456789abcdef";
  std::string s = "\"0x";
  for (int i = 31; i >= 0; --i) {
    s += hx[le32[i] >> 4];
    s += hx[le32[i] & 15];
  }
  return s + "\"";
}

// snarkjs 0.4.22 `zkey export soliditycalldata` (G2 pairs in EIP-197 [c1, c0] order)
std::string calldata(const zkp_proof* p) {
  std::string s = "[" + p256(p->pi_a[0]) + ", " + p256(p->pi_a[1]) + "],";
  s += "[[" + p256(p->pi_b[0][1]) + ", " + p256(p->pi_b[0][0]) + "],[" + p256(p->pi_b[1][1]) + ", " +
       p256(p->pi_b[1][0]) + "]],";
  s += "[" + p256(p->pi_c[0]) + ", " + p256(p->pi_c[1]) + "],[";
  const uint32_t n = std::min(p->n_public, p->public_capacity);
  for (uint32_t i = 0; i < n && p->public_signals; ++i) {
    if (i) s += ",";
    s += p256(p->public_signals + 32 * i);
  }
  return s + "]";
}

zkp_status emit(const std::string& s, char* buf, size_t cap, size_t* needed) {
  if (needed) *needed = s.size() + 1;
  if (buf && cap >= s.size() + 1) {
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return ZKP_OK;
  }
  if (buf) return fail(ZKP_ERR_INVALID_ARG, "buffer too small");
  return ZKP_OK;
}

void write_file(const char* path, const std::string& s) {
  std::ofstream f(path, std::ios::binary);
  if (!f || !f.write(s.data(), (std::streamsize)s.size())) throw zkp::ZkpError(ZKP_ERR_IO, std::string("cannot write ") + path);
}

std::vector<int> dev_list(const int* devices, int ndev) {
  std::vector<int> v;
  if (devices)
    for (int i = 0; i < ndev; ++i) v.push_back(devices[i]);
  return v;
}

}  // namespace

extern "C" {

zkp_status zkp_prover_load_mem(const uint8_t* zkey, size_t len, const int* devices, int ndev, zkp_prover** out) {
  if (!zkey || !out || ndev < 0) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  return guard([&] {
    auto* h = new zkp_prover{nullptr};
    try {
      h->impl = new zkp::Prover(zkey, len, dev_list(devices, ndev));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

zkp_status zkp_prover_load_file(const char* path, const int* devices, int ndev, zkp_prover** out) {
  if (!path || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  std::vector<uint8_t> buf;
  zkp_status s = guard([&] { buf = zkp::read_zkey_source(path); });
  if (s != ZKP_OK) return s;
  return zkp_prover_load_mem(buf.data(), buf.size(), devices, ndev, out);
}

zkp_status zkp_prover_load_chunks(const char* const* paths, int n, const int* devices, int ndev, zkp_prover** out) {
  if (!paths || n < 1 || !out) return fail(ZKP_ERR_INVALID_ARG, "bad argument");
  std::vector<uint8_t> buf;
  zkp_status s = guard([&] { buf = zkp::read_zkey_chunks(std::vector<std::string>(paths, paths + n)); });
  if (s != ZKP_OK) return s;
  return zkp_prover_load_mem(buf.data(), buf.size(), devices, ndev, out);
}

static zkp_status hand_out(std::vector<uint8_t>&& v, uint8_t** out, size_t* len) {
  *out = static_cast<uint8_t*>(std::malloc(std::max<size_t>(v.size(), 1)));
  if (!*out) return fail(ZKP_ERR_OUT_OF_MEMORY, "host out of memory");
  std::memcpy(*out, v.data(), v.size());
  *len = v.size();
  return ZKP_OK;
}

zkp_status zkp_zkey_read(const char* path, uint8_t** out, size_t* len) {
  if (!path || !out || !len) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  std::vector<uint8_t> buf;
  zkp_status s = guard([&] { buf = zkp::read_zkey_source(path); });
  return s != ZKP_OK ? s : hand_out(std::move(buf), out, len);
}

zkp_status zkp_zkey_read_chunks(const char* const* paths, int n, uint8_t** out, size_t* len) {
  if (!paths || n < 1 || !out || !len) return fail(ZKP_ERR_INVALID_ARG, "bad argument");
  std::vector<uint8_t> buf;
  zkp_status s = guard([&] { buf = zkp::read_zkey_chunks(std::vector<std::string>(paths, paths + n)); });
  return s != ZKP_OK ? s : hand_out(std::move(buf), out, len);
}

void zkp_buffer_free(uint8_t* p) { std::free(p); }

zkp_status zkp_zkey_contribute(int device, const uint8_t* zkey, size_t len, const uint8_t* k32, uint8_t** out,
                               size_t* out_len) {
  if (!zkey || !k32 || !out || !out_len) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  std::vector<uint8_t> buf;
  zkp_status s = guard([&] { buf = zkp::zkey_apply_delta(device, zkey, len, k32); });
  return s != ZKP_OK ? s : hand_out(std::move(buf), out, out_len);
}

zkp_status zkp_beacon_secret(const uint8_t* beacon, size_t len, uint32_t num_iterations_exp, uint8_t* k32) {
  if ((!beacon && len) || !k32) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { zkp::beacon_secret(beacon, len, num_iterations_exp, k32); });
}

}  // extern "C"

namespace {
// one phase-2 contribution drawn from rng: the record appended to section 10 (mpc.cpp), then the
// group arithmetic on the GPU (delta -> k delta, L and H -> k^-1) and the new section 10
std::vector<uint8_t> contribute_mpc(int device, const uint8_t* zkey, size_t len, zkp::ChaChaRng& rng, uint32_t type,
                                    const char* name, const uint8_t* beacon, size_t beacon_len, uint32_t e) {
  const zkp::ZkeyParsed z = zkp::parse_zkey(zkey, len, false);
  const zkp::Section& s10 = z.bf.sec[10];
  if (!s10.ptr) throw zkp::ZkpError(ZKP_ERR_FORMAT, "zkey: missing section 10 (MPC parameters)");
  zkp::MpcParams m = zkp::read_mpc(s10.ptr, s10.len);
  uint8_t k[32];
  zkp::mpc_contribute(m, rng, z.hdr.delta1, type, name ? std::string(name) : std::string(), beacon, beacon_len, e, k);
  std::vector<uint8_t> buf = zkp::zkey_apply_delta(device, zkey, len, k);
  zkp::binfile_replace_section(buf, 10, zkp::write_mpc(m));
  return buf;
}
}  // namespace
extern "C" {

zkp_status zkp_zkey_beacon_named(int device, const uint8_t* zkey, size_t len, const uint8_t* beacon, size_t beacon_len,
                                 uint32_t num_iterations_exp, const char* name, uint8_t** out, size_t* out_len) {
  if (!zkey || (!beacon && beacon_len) || !out || !out_len) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  std::vector<uint8_t> buf;
  zkp_status s = guard([&] {
    uint8_t h[32];
    zkp::beacon_hash(beacon, beacon_len, num_iterations_exp, h);
    uint32_t seed[8];
    zkp::seed_from_hash(h, seed);
    zkp::ChaChaRng rng(seed);
    buf = contribute_mpc(device, zkey, len, rng, 1, name, beacon, beacon_len, num_iterations_exp);
  });
  return s != ZKP_OK ? s : hand_out(std::move(buf), out, out_len);
}

zkp_status zkp_zkey_beacon(int device, const uint8_t* zkey, size_t len, const uint8_t* beacon, size_t beacon_len,
                           uint32_t num_iterations_exp, uint8_t** out, size_t* out_len) {
  return zkp_zkey_beacon_named(device, zkey, len, beacon, beacon_len, num_iterations_exp, nullptr, out, out_len);
}

zkp_status zkp_zkey_contribute_entropy(int device, const uint8_t* zkey, size_t len, const uint8_t* rand64,
                                       const char* entropy, const char* name, uint8_t** out, size_t* out_len) {
  if (!zkey || !entropy || !out || !out_len) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  std::vector<uint8_t> buf;
  zkp_status s = guard([&] {
    uint8_t rnd[64];
    if (rand64) {
      std::memcpy(rnd, rand64, 64);
    } else {  // snarkjs misc.getRandomRng: 64 bytes from the OS CSPRNG
      std::ifstream f("/dev/urandom", std::ios::binary);
      if (!f.read(reinterpret_cast<char*>(rnd), 64)) throw zkp::ZkpError(ZKP_ERR_IO, "cannot read /dev/urandom");
    }
    zkp::Blake2b hh;
    hh.update(rnd, 64);
    hh.update(entropy, std::strlen(entropy));
    uint8_t d[64];
    hh.final(d);
    uint32_t seed[8];
    zkp::seed_from_hash(d, seed);
    zkp::ChaChaRng rng(seed);
    buf = contribute_mpc(device, zkey, len, rng, 0, name, nullptr, 0, 0);
  });
  return s != ZKP_OK ? s : hand_out(std::move(buf), out, out_len);
}

zkp_status zkp_blake2b512(const uint8_t* data, size_t len, uint8_t* out64) {
  if ((!data && len) || !out64) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] {
    zkp::Blake2b h;
    h.update(data, len);
    h.final(out64);
  });
}

zkp_status zkp_zkey_new(int device, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* ptau, size_t ptau_len,
                        uint8_t** out, size_t* out_len) {
  if (!r1cs || !ptau || !out || !out_len) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  std::vector<uint8_t> buf;
  zkp_status s = guard([&] { buf = zkp::zkey_new(device, r1cs, r1cs_len, ptau, ptau_len); });
  return s != ZKP_OK ? s : hand_out(std::move(buf), out, out_len);
}

zkp_status zkp_prover_load_part(const uint8_t* zkey, size_t len, int device, int part, int nparts,
                                zkp_prover** out) {
  if (!zkey || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  return guard([&] {
    auto* h = new zkp_prover{nullptr};
    try {
      h->impl = new zkp::Prover(zkey, len, std::vector<int>{device}, part, nparts);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

zkp_status zkp_prove_partial(zkp_prover* p, const uint8_t* wtns, size_t len, zkp_partial* out) {
  if (!p || !wtns || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->prove_partial(wtns, len, out); });
}

zkp_status zkp_prove_partial_staged(zkp_prover* p, int slot, zkp_partial* out) {
  if (!p || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->prove_partial_staged(slot, out); });
}

zkp_status zkp_quotient_part_staged(zkp_prover* p, int slot, int mask, void* const* dst) {
  if (!p || !dst) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->quotient_part_staged(slot, mask, dst); });
}

zkp_status zkp_prove_partial_ext_staged(zkp_prover* p, int slot, const void* const* abc, zkp_partial* out) {
  if (!p || !abc || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->prove_partial_ext_staged(slot, abc, out); });
}

zkp_status zkp_proof_combine(const uint8_t* zkey, size_t len, const zkp_partial* parts, int nparts,
                             const uint8_t* wtns, size_t wlen, const uint8_t* r32, const uint8_t* s32,
                             zkp_proof* out) {
  if (!zkey || !parts || !wtns || !out || nparts < 1) return fail(ZKP_ERR_INVALID_ARG, "bad argument");
  return guard([&] { zkp::proof_combine(zkey, len, parts, nparts, wtns, wlen, r32, s32, out); });
}

zkp_status zkp_prover_info(const zkp_prover* p, uint32_t* n_vars, uint32_t* n_public, uint32_t* domain_size) {
  if (!p) return fail(ZKP_ERR_INVALID_ARG, "null prover");
  const auto& h = p->impl->header();
  if (n_vars) *n_vars = h.n_vars;
  if (n_public) *n_public = h.n_public;
  if (domain_size) *domain_size = h.domain_size;
  return ZKP_OK;
}

zkp_status zkp_prove(zkp_prover* p, const uint8_t* wtns, size_t len, const uint8_t* r32, const uint8_t* s32,
                     zkp_proof* out) {
  if (!p || !wtns || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->prove(wtns, len, r32, s32, out); });
}

zkp_status zkp_prove_batch(zkp_prover* p, const uint8_t* const* wtns, const size_t* lens, int n,
                           const uint8_t* const* r32s, const uint8_t* const* s32s, zkp_proof* outs) {
  return zkp_prove_batch_status(p, wtns, lens, n, r32s, s32s, outs, nullptr);
}

zkp_status zkp_prove_batch_status(zkp_prover* p, const uint8_t* const* wtns, const size_t* lens, int n,
                                  const uint8_t* const* r32s, const uint8_t* const* s32s, zkp_proof* outs,
                                  zkp_status* statuses) {
  if (!p || (n > 0 && (!wtns || !lens || !outs)) || n < 0) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  zkp_status first = ZKP_OK;
  std::string msg;
  zkp_status s = guard([&] { first = p->impl->prove_batch(wtns, lens, n, r32s, s32s, outs, statuses, &msg); });
  if (s != ZKP_OK) return s;
  return first == ZKP_OK ? ZKP_OK : fail(first, msg);
}

zkp_status zkp_prove_files(zkp_prover* p, const char* wtns_path, const char* proof_path, const char* public_path) {
  if (!p || !wtns_path || !proof_path || !public_path) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] {
    const MappedFile w(wtns_path);
    const uint32_t npub = p->impl->header().n_public;
    std::vector<uint8_t> pub((size_t)npub * 32 + 32);
    zkp_proof pr{};
    pr.public_capacity = npub;
    pr.public_signals = pub.data();
    p->impl->prove(w.data(), w.size(), nullptr, nullptr, &pr);
    write_file(proof_path, proof_json(&pr));
    write_file(public_path, public_json(&pr));
  });
}

zkp_status zkp_proof_json(const zkp_proof* proof, char* buf, size_t cap, size_t* needed) {
  if (!proof) return fail(ZKP_ERR_INVALID_ARG, "null proof");
  return emit(proof_json(proof), buf, cap, needed);
}

zkp_status zkp_public_json(const zkp_proof* proof, char* buf, size_t cap, size_t* needed) {
  if (!proof) return fail(ZKP_ERR_INVALID_ARG, "null proof");
  return emit(public_json(proof), buf, cap, needed);
}

zkp_status zkp_proof_calldata(const zkp_proof* proof, char* buf, size_t cap, size_t* needed) {
  if (!proof) return fail(ZKP_ERR_INVALID_ARG, "null proof");
  return emit(calldata(proof), buf, cap, needed);
}

zkp_status zkp_prover_timings(const zkp_prover* p, float* ms, int n) {
  if (!p || !ms) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  p->impl->timings(ms, n);
  return ZKP_OK;
}

void zkp_prover_free(zkp_prover* p) {
  if (!p) return;
  delete p->impl;
  delete p;
}

zkp_status zkp_prover_set_verify(zkp_prover* p, int on) {
  if (!p || !p->impl) return fail(ZKP_ERR_INVALID_ARG, "null prover");
  return guard([&] { p->impl->set_verify(on == 0 ? 0 : (on == 2 ? 2 : 1)); });
}

zkp_status zkp_prover_get_verify(const zkp_prover* p, int* mode) {
  if (!p || !p->impl || !mode) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  *mode = p->impl->verify_mode();
  return ZKP_OK;
}

}  // extern "C"

namespace {
using zkp::host::Affine;
using HFq = zkp::host::Fq;
using HFq2 = zkp::host::Fq2;
HFq fq_std(const uint8_t* b) {
  const zkp::host::U256 v = zkp::host::u256_from_le(b);
  if (zkp::host::u256_geq(v, zkp::host::FQ_DESC.mod)) throw zkp::ZkpError(ZKP_ERR_INVALID_ARG, "coordinate >= p");
  return HFq::from_std(v);
}
bool all_zero(const uint8_t* b, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (b[i]) return false;
  return true;
}
Affine<HFq> g1_std(const uint8_t* b) {
  if (all_zero(b, 64)) return Affine<HFq>{HFq::zero(), HFq::zero(), true};
  return Affine<HFq>{fq_std(b), fq_std(b + 32), false};
}
Affine<HFq2> g2_std(const uint8_t* b) {
  if (all_zero(b, 128)) return Affine<HFq2>{HFq2::zero(), HFq2::zero(), true};
  return Affine<HFq2>{HFq2{fq_std(b), fq_std(b + 32)}, HFq2{fq_std(b + 64), fq_std(b + 96)}, false};
}
}  // namespace
extern "C" {

zkp_status zkp_proof_verify(const uint8_t* zkey, size_t len, const zkp_proof* proof, int* valid) {
  if (!zkey || !proof || !valid) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] {
    *valid = 0;
    const zkp::ZkeyParsed z = zkp::parse_zkey(zkey, len, false);
    const zkp::ZkeyHeader& h = z.hdr;
    if (h.ic.size() != (size_t)h.n_public + 1) throw zkp::ZkpError(ZKP_ERR_FORMAT, "zkey: no IC section");
    if (proof->n_public != h.n_public || proof->public_capacity < h.n_public || (h.n_public && !proof->public_signals))
      throw zkp::ZkpError(ZKP_ERR_INVALID_ARG, "proof: public signals do not match the key's nPublic");
    zkp::host::VerifyingKey vk;
    vk.alpha1 = h.alpha1, vk.beta2 = h.beta2, vk.gamma2 = h.gamma2, vk.delta2 = h.delta2;
    vk.ic = h.ic.data();
    vk.n_public = (int)h.n_public;
    std::vector<zkp::host::U256> pub(h.n_public);
    for (uint32_t i = 0; i < h.n_public; ++i) pub[i] = zkp::host::u256_from_le(proof->public_signals + 32 * (size_t)i);
    const Affine<HFq> a = g1_std(proof->pi_a[0]), c = g1_std(proof->pi_c[0]);
    const Affine<HFq2> b = g2_std(proof->pi_b[0][0]);
    *valid = zkp::host::groth16_verify(vk, pub.data(), a, b, c) ? 1 : 0;
  });
}

zkp_status zkp_pairing(const uint8_t* g1, const uint8_t* g2, uint8_t* out384) {
  if (!g1 || !g2 || !out384) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] {
    const Affine<HFq> p = g1_std(g1);
    const Affine<HFq2> q = g2_std(g2);
    if (!zkp::host::g1_on_curve(p) || !zkp::host::g2_on_curve(q))
      throw zkp::ZkpError(ZKP_ERR_INVALID_ARG, "pairing: point not on the curve");
    const zkp::host::Fq12 f = zkp::host::pairing(p, q);
    const HFq2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
    for (int i = 0; i < 6; ++i) {
      zkp::host::u256_to_le(c[i]->c0.to_std(), out384 + 64 * i);
      zkp::host::u256_to_le(c[i]->c1.to_std(), out384 + 64 * i + 32);
    }
  });
}

const char* zkp_last_error(void) { return g_err.c_str(); }

const char* zkp_version(void) { return "zkp_amd 0.1 gfx950"; }

zkp_status zkp_msm_g1(int device, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out64,
                      int* is_inf) {
  if ((n && (!points || !scalars)) || !out64 || !is_inf) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { zkp::msm_points(device, zkp::Curve::G1, points, scalars, n, out64, is_inf); });
}

zkp_status zkp_msm_g2(int device, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out128,
                      int* is_inf) {
  if ((n && (!points || !scalars)) || !out128 || !is_inf) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { zkp::msm_points(device, zkp::Curve::G2, points, scalars, n, out128, is_inf); });
}

zkp_status zkp_msm(int device, int g2, const uint8_t* points, const uint8_t* scalars, size_t n, int window_bits,
                   int table_depth, uint8_t* out, int* is_inf) {
  if ((n && (!points || !scalars)) || !out || !is_inf) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  if (window_bits < 0 || (window_bits > 0 && window_bits < 8) || window_bits > 24 || table_depth < 0)
    return fail(ZKP_ERR_INVALID_ARG, "MSM window bits must be 0 (automatic) or within 8..24, table_depth >= 0");
  return guard([&] {
    zkp::msm_points(device, g2 ? zkp::Curve::G2 : zkp::Curve::G1, points, scalars, n, out, is_inf, window_bits,
                    table_depth);
  });
}

zkp_status zkp_prover_msm_config(const zkp_prover* p, double* out, int n) {
  if (!p || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->msm_config(out, n); });
}

zkp_status zkp_ntt_fr(int device, uint8_t* data, size_t n, int mode) {
  if (!data || mode < 0 || mode > 2) return fail(ZKP_ERR_INVALID_ARG, "bad argument");
  return guard([&] { zkp::ntt_fr(device, data, n, mode); });
}

zkp_status zkp_quotient(zkp_prover* p, const uint8_t* wtns, size_t len, uint8_t* out) {
  if (!p || !wtns || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->quotient(wtns, len, out); });
}

zkp_status zkp_witness_stage(zkp_prover* p, int dev_index, int slot, const uint8_t* wtns, size_t len) {
  if (!p || !wtns) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->stage(dev_index, slot, wtns, len); });
}

zkp_status zkp_prove_staged(zkp_prover* p, int dev_index, int slot, const uint8_t* r32, const uint8_t* s32,
                            zkp_proof* out) {
  if (!p || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->prove_staged(dev_index, slot, r32, s32, out); });
}

zkp_status zkp_prover_instrument(zkp_prover* p, int on) {
  if (!p) return fail(ZKP_ERR_INVALID_ARG, "null prover");
  return guard([&] { p->impl->set_instrument(on != 0); });
}

zkp_status zkp_prover_kernel_stats(const zkp_prover* p, double* out, int n) {
  if (!p || !out) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { p->impl->kernel_stats(out, n); });
}

zkp_status zkp_prover_launch_stats(const zkp_prover* p, double* out, int max_records, int* n_records) {
  if (!p || !n_records || (max_records > 0 && !out)) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] { *n_records = p->impl->launch_records(out, max_records); });
}

zkp_status zkp_bench_msm_ex(int device, int g2, const uint8_t* points, const uint8_t* scalars, size_t n, int warmup,
                            int iters, double* stats, int nstats, uint8_t* out, int* is_inf) {
  if (!points || !scalars || !stats || nstats < 0) return fail(ZKP_ERR_INVALID_ARG, "null argument");
  return guard([&] {
    zkp::MsmBench b = zkp::bench_msm(device, g2 ? zkp::Curve::G2 : zkp::Curve::G1, points, scalars, n, warmup,
                                     iters, out, is_inf);
    const double v[8] = {b.ms_per_msm, b.ms_accumulate, (double)b.mixed_adds, (double)b.tasks,
                         (double)b.c, (double)b.windows, (double)b.table_ms, (double)b.depth};
    for (int i = 0; i < nstats && i < 8; ++i) stats[i] = v[i];
  });
}

zkp_status zkp_bench_msm(int device, int g2, const uint8_t* points, const uint8_t* scalars, size_t n, int warmup,
                         int iters, double* stats, uint8_t* out, int* is_inf) {
  return zkp_bench_msm_ex(device, g2, points, scalars, n, warmup, iters, stats, 6, out, is_inf);
}

zkp_status zkp_bench_plan(int device, const uint8_t* scalars, size_t n, int window_bits, int dense, int warmup,
                          int iters, double* ms) {
  if (!scalars || !ms || window_bits < 0 || window_bits == 1 || window_bits > 24)
    return fail(ZKP_ERR_INVALID_ARG, "bad argument");
  return guard([&] { *ms = zkp::bench_plan(device, scalars, n, window_bits, dense, warmup, iters); });
}

zkp_status zkp_bench_ntt(int device, int log_n, int warmup, int iters, double* ms) {
  if (!ms || log_n < 1 || log_n > 27) return fail(ZKP_ERR_INVALID_ARG, "bad argument");
  return guard([&] { *ms = zkp::bench_ntt(device, log_n, 1, warmup, iters); });
}

zkp_status zkp_bench_ntt_batch(int device, int log_n, int count, int warmup, int iters, double* ms) {
  if (!ms || log_n < 1 || log_n > 27 || count < 1 || count > 3) return fail(ZKP_ERR_INVALID_ARG, "bad argument");
  return guard([&] { *ms = zkp::bench_ntt(device, log_n, count, warmup, iters); });
}

}  // extern "C"
