// Groth16 prover core (device-resident zkey, per-device pipelines, batch scheduler).
//
// Restates snarkjs 0.4.22 groth16_prove MI355X-first:
//  * load: parse + validate the zkey once, upload the five point sections and
//    the A/B coefficient matrix (as CSR) to HBM of every device; they stay
//    resident for the life of the handle (the reference re-reads 3.5 GB per proof).
//  * prove: only the witness crosses PCIe; buildABC -> 3 x coset NTT -> joinABC
//    -> 4 G1 MSMs on one stream while the G2 MSM runs on a second stream;
//    the O(1) tail (window Horner, r/s blinding, affine) runs on the host.
//  * batch: one host worker thread per device pulls witnesses from a shared
//    queue (replicas, no collectives: SURVEY.md §8e E1(1)).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/zkp_amd.h"
#include "host_ec.hpp"
#include "msm.hpp"
#include "ntt.hpp"

namespace zkp {

struct ZkpError : std::runtime_error {
  zkp_status status;
  ZkpError(zkp_status s, const std::string& m) : std::runtime_error(m), status(s) {}
};

struct Section {
  const uint8_t* ptr = nullptr;
  uint64_t len = 0;
};

// Parsed view of a snarkjs binfile (no copies; points into the caller's buffer)
struct BinFile {
  uint32_t version = 0;
  Section sec[16];
};
BinFile parse_binfile(const uint8_t* buf, size_t len, const char* magic, uint32_t max_version);

struct ZkeyHeader {
  uint32_t n_vars = 0, n_public = 0, domain_size = 0, log_domain = 0;
  uint32_t n_coef = 0;
  host::Affine<host::Fq> alpha1, beta1, delta1;
  host::Affine<host::Fq2> beta2, gamma2, delta2;
  std::vector<host::Affine<host::Fq>> ic;  // section 3 (nPublic + 1 points; empty if the key has none)
};

struct WtnsView {
  uint32_t n_witness = 0;
  const uint8_t* values = nullptr;  // n_witness x 32 bytes, standard form LE
};
WtnsView parse_wtns(const uint8_t* buf, size_t len);

struct Csr {
  std::vector<uint32_t> rowptr, col, val;  // val: 8 words per entry (raw zkey bytes)
};
// a groth16 zkey: sections, header (validated: curve, sizes of sections 4-9, power-of-two
// domain <= 2^27) and, with_coefs, the A/B coefficients as CSR by (matrix, constraint)
struct ZkeyParsed {
  BinFile bf;
  ZkeyHeader hdr;
  Csr csr[2];
};
ZkeyParsed parse_zkey(const uint8_t* buf, size_t len, bool with_coefs = true);

class DevicePipeline;

class Prover {
 public:
  // part / nparts > 1: hold only point slice `part` (one device) -> prove_partial only
  Prover(const uint8_t* zkey, size_t len, const std::vector<int>& devices, int part = 0, int nparts = 1);
  ~Prover();
  const ZkeyHeader& header() const { return hdr_; }
  // r32/s32 nullable (CSPRNG).  Thread-safe.
  void prove(const uint8_t* wtns, size_t len, const uint8_t* r32, const uint8_t* s32, zkp_proof* out);
  // every proof is attempted; statuses (nullable) receives each proof's status; returns the
  // first failing status (ZKP_OK if none) with its message in *first_error
  zkp_status prove_batch(const uint8_t* const* wtns, const size_t* lens, int n, const uint8_t* const* r32s,
                         const uint8_t* const* s32s, zkp_proof* outs, zkp_status* statuses, std::string* first_error);
  void quotient(const uint8_t* wtns, size_t len, uint8_t* out);
  void timings(float* ms, int n) const;
  // HBM-resident witnesses (benchmarks time the proof without the PCIe copy)
  void stage(int dev, int slot, const uint8_t* wtns, size_t len);
  void prove_staged(int dev, int slot, const uint8_t* r32, const uint8_t* s32, zkp_proof* out);
  // per-kernel HIP-event statistics of the bucket-accumulate kernels
  void set_instrument(bool on);
  void kernel_stats(double* out, int n) const;
  // per-launch records {kind, mixed adds, ms, workgroups} (zkp_prover_launch_stats); returns the number held
  int launch_records(double* out, int max_records) const;
  int device_count() const { return ndevices_; }  // entries of the `devices` list
  int pipelines_per_device() const { return inflight_; }
  // point-range split of one proof: this slice's MSM partial sums
  void prove_partial(const uint8_t* wtns, size_t len, zkp_partial* out);
  void prove_partial_staged(int slot, zkp_partial* out);
  // distributed quotient of a split proof (zkp_quotient_part_staged / zkp_prove_partial_ext_staged)
  void quotient_part_staged(int slot, int mask, void* const* dst);
  void prove_partial_ext_staged(int slot, const void* const* abc, zkp_partial* out);
  int part() const { return part_; }
  int nparts() const { return nparts_; }
  // MSM configuration of device 0: [0] witness c, [1] witness depth, [2] witness groups,
  // [3] H c, [4] H depth, [5] H groups, [6] base-table bytes per device, [7..9] the second witness
  // configuration's c, depth, groups (0 when the prover keeps one)
  void msm_config(double* out, int n) const;
  // verify-before-return (the reference verifies every proof after proving,
  // dizkus-scripts/5_gen_proof.sh:14-21): every proof of zkp_prove / zkp_prove_batch /
  // zkp_prove_staged is checked by the host pairing (host_pairing.cpp) against the zkey's
  // verification key; a proof that fails is an error (ZKP_ERR_INTERNAL), never returned.
  // Modes: 0 off, 1 every proof, 2 (the default) zkp_prove_batch only -- there the host pairing runs
  // on the worker thread while the next proof computes (measured free), while on a single proof it
  // adds its ~2.6 ms to the latency.  Environment ZKP_VERIFY=0/1/2 at load overrides the default.
  void set_verify(int mode) { verify_.store(mode); }
  int verify_mode() const { return verify_.load(); }
  bool verify() const { return verify_.load() == 1; }        // single-proof paths
  bool verify_batch() const { return verify_.load() != 0; }  // zkp_prove_batch[_status]

 private:
  void require_full() const;
  DevicePipeline& pick_device();
  ZkeyHeader hdr_;
  int part_ = 0, nparts_ = 1;
  int inflight_ = 1, ndevices_ = 0;
  // inflight_ consecutive pipelines per entry of the device list (ZKP_INFLIGHT)
  std::vector<std::unique_ptr<DevicePipeline>> devs_;
  DevicePipeline& staged_pipeline(int dev_index) const;
  void retire_device(const DevicePipeline& failed);
  std::vector<std::vector<std::vector<uint8_t>>> staged_pub_;  // [dev][slot] -> first (nPub+1)*32 witness bytes
  mutable std::mutex smu_;
  std::atomic<unsigned> rr_{0};
  mutable std::mutex tmu_;
  float last_ms_[11] = {};  // [8]: verify-before-return (host ms), [9]: witness transfer MB, [10]: witness MSM configuration
  std::atomic<int> verify_{2};
  // test hook ZKP_TEST_CORRUPT_H: 1 = every proof's piH + G1 generator (a silent device error),
  // 2 = only the odd-indexed proofs of a batch (the batch must refuse those and prove the rest)
  int corrupt_h_ = 0;
  // throws ZkpError(ZKP_ERR_INTERNAL) unless the assembled proof verifies; returns the host ms spent
  float verify_or_throw(const WtnsView& w, const zkp_proof* out) const;
  friend class DevicePipeline;
};

// sum the partials of one split (host only: parses the zkey header, no device) and
// assemble the proof exactly as Prover::prove would
void proof_combine(const uint8_t* zkey, size_t len, const zkp_partial* parts, int nparts, const uint8_t* wtns,
                   size_t wlen, const uint8_t* r32, const uint8_t* s32, zkp_proof* out);

// phase-2 contribution math on the GPU (setup.hip): delta -> k*delta
std::vector<uint8_t> zkey_apply_delta(int device, const uint8_t* zkey, size_t len, const uint8_t* k32);
// `snarkjs zkey new`: the phase-2 starting key (gamma = delta = 1) of a circom .r1cs from a
// prepared .ptau (sections 12-15), the point sections built on `device` (zkey_new.hip)
std::vector<uint8_t> zkey_new(int device, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* ptau, size_t ptau_len);

// kernel-level helpers (C-ABI zkp_msm_g1/g2, zkp_ntt_fr)
// c / depth: window bits and base-table depth (0 = automatic, as the prover)
void msm_points(int device, Curve curve, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out,
                int* is_inf, int c = 0, int depth = 0);
void ntt_fr(int device, uint8_t* data, size_t n, int mode);
// device-resident kernel benchmarks (HIP events on the engine stream)
struct MsmBench {
  float ms_per_msm = 0;         // whole MSM pipeline
  float ms_accumulate = 0;      // bucket-accumulate kernel, per launch
  uint64_t mixed_adds = 0;      // per launch
  uint64_t tasks = 0;           // per launch
  int c = 0, windows = 0;
  int depth = 0;        // base-table rows T (T = windows: every window's 2^(c t) P precomputed)
  float table_ms = 0;   // building those tables (outside the timed MSMs: fixed bases, built at load)
};
MsmBench bench_msm(int device, Curve curve, const uint8_t* points, const uint8_t* scalars, size_t n, int warmup,
                   int iters, uint8_t* out, int* is_inf);
// ms per coset_extend_batch (iNTT + coset key + NTT) of count vectors of 2^log_n Fr elements
float bench_ntt(int device, int log_n, int count, int warmup, int iters);
// ms per MsmPlan::build (digits + bucket grouping + task offsets) of n scalars, window bits c (0 = auto),
// dense (every digit an entry: the H plan) or compacted
float bench_plan(int device, const uint8_t* scalars, size_t n, int c, int dense, int warmup, int iters);

}  // namespace zkp
