// Fr NTT engine for the QAP quotient on gfx950.
//
// Replaces ffjavascript Fr.ifft / Fr.batchApplyKey / Fr.fft as used by snarkjs
// groth16_prove: for each of A, B, C
//   evaluations on <w> (natural order)  --iNTT-->  coefficients
//   --x g^i-->  --NTT-->  evaluations on the coset g<w> (natural order)
// with w = Fr.w[log2 n] and g = Fr.w[log2 n + 1] (ffjavascript convention).
//
// Multi-pass "four-step" structure: a pass splits the current block of size m = 2^lm
// into 2^b rows x n2 columns, runs 2^b-point DFTs in LDS over the strided row index
// for a tile of consecutive columns (radix-2 stages on LDS-resident 9-limb values,
// the stage roots staged in LDS), and multiplies by the inter-pass twiddle
// w_m^(col*row), read from a per-(block size, direction) table indexed by the
// element's position in the block (coalesced like the data; one multiply, no
// exponent arithmetic).  The inverse runs these passes DIF-style (natural in ->
// digit-reversed out); the forward runs the TRANSPOSED passes in reverse order
// (digit-reversed in -> natural out), so no permutation pass is ever needed.  In
// coset_extend the innermost inverse pass, the coset key g^f(pos)/n (a table in
// digit-reversed position order) and the innermost forward pass are ONE kernel: the
// tile never leaves LDS between them.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

namespace zkp {

class NttEngine {
 public:
  NttEngine(int log_n, hipStream_t stream);
  ~NttEngine();
  NttEngine(const NttEngine&) = delete;
  NttEngine& operator=(const NttEngine&) = delete;

  int log_n() const { return log_n_; }
  // data: n Fr elements, device layout (Montgomery R' = 2^261, 8 LE words each)
  // natural-order evaluations on <w>  ->  natural-order evaluations on g<w>
  void coset_extend(uint32_t* data);
  // the same for count (1..3) vectors of n elements each, every pass one launch over all of them
  // (the quotient's A, B, C)
  void coset_extend_batch(uint32_t* const* data, int count);
  // plain transforms (natural in, natural out), for tests
  void forward(uint32_t* data);  // A_j = sum a_i w^(ij)
  void inverse(uint32_t* data);  // a_i = n^-1 sum A_j w^(-ij)
  hipStream_t stream() const { return stream_; }
  size_t table_bytes() const { return table_bytes_; }

 private:
  // passes [first, last) of the DIF sequence (dir 1 = inverse root), resp. of the
  // transposed DIT sequence in reverse order
  void dif_passes(uint32_t* const* data, int count, bool inv, int first, int last);
  void dit_passes(uint32_t* const* data, int count, bool inv, int first, int last);
  void launch_pass(uint32_t* const* data, int count, int mode, int p, bool inv);
  void scale(uint32_t* data, int mode);  // 0: x g^f(pos)/n   1: x 1/n (digit-reversed layout ok)
  void digit_reverse(uint32_t* data, bool to_natural);
  int log_n_;
  hipStream_t stream_;
  std::vector<int> bits_;  // pass radix bits (DIF order)
  std::vector<int> lms_;   // block size log of each DIF pass
  int h_ = 0;              // split of the twiddle exponent tables
  // device tables (dev layout): [0] forward root, [1] inverse root
  uint32_t* tw_lo_[2] = {nullptr, nullptr};
  uint32_t* tw_hi_[2] = {nullptr, nullptr};
  std::vector<uint32_t*> tw_pass_[2];      // per DIF pass p: w_(2^lm)^(col*row) by position in block (null: none)
  uint32_t* loc_[2] = {nullptr, nullptr};  // local roots w_1024^e, e < 512
  uint32_t* rtab_[2][9] = {};              // [dir][b]: staged stage roots of a b-bit pass (Shoup form)
  uint32_t* coset_lo_ = nullptr;           // g^e / n, e < 2^h
  uint32_t* coset_hi_ = nullptr;           // g^(e 2^h)
  uint32_t* coset_pos_ = nullptr;          // g^f(pos) / n by digit-reversed position
  uint32_t* ninv_ = nullptr;               // 1/n (dev form)
  uint32_t* scratch_ = nullptr;            // for digit_reverse (tests only)
  size_t table_bytes_ = 0;
};

}  // namespace zkp
