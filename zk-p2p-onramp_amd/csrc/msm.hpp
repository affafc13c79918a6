// Pippenger multi-scalar multiplication over BN254 G1 / G2 on gfx950.
//
// Replaces ffjavascript ``G1.multiExpAffine`` / ``G2.multiExpAffine``
// (g1m/g2m_multiexpAffine_chunk) as called five times by
// snarkjs ``groth16_prove``.  Result is bit-identical as a group element; the
// algorithm is a GPU re-design, not a translation:
//
//  1. digits    : one thread per scalar writes W signed c-bit digits as
//                 (key = window*2^(c-1) + |d|-1, val = point | sign<<31).
//  2. sort      : radix sort of the (key, val) pairs -> points grouped by bucket.
//  3. bounds    : bucket [start, end) ranges from the sorted keys.
//  4. accumulate: the sorted list is cut into tasks of <= S entries that never
//                 straddle a bucket, so every thread does the same bounded work
//                 whatever the scalar distribution (0/1-heavy witnesses put
//                 most points into a single bucket).  Mixed XYZZ additions.
//  5. merge     : buckets with more than S2 task partials ("heavy": the 0/1-rich
//                 witness buckets) are folded by segmented merge levels that skip
//                 every light bucket; then one thread per bucket sums what is left.
//  6. reduce    : per window, sum_k (k+1) B_k by an L-ary tree of running sums.
//  7. windows   : W window sums go to the host, which folds them by Horner.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace zkp {

struct MsmParams {
  int c = 16;        // window bits
  int windows = 16;  // ceil(255 / c)
  int S = 32;        // max points per accumulate task
  int S2 = 32;       // fan-in of a merge level
  int L = 8;         // fan-in of a bucket-reduction level
  static MsmParams for_size(size_t n) {
    MsmParams p;
    int lg = 0;
    while ((size_t(1) << lg) < n) ++lg;
    // bucket count 2^(c-1) per window ~ n/16..n/32 keeps buckets ~16-32 deep
    p.c = lg - 3 < 8 ? 8 : (lg - 3 > 16 ? 16 : lg - 3);
    p.windows = (255 + p.c - 1) / p.c;
    return p;
  }
};

// words per coordinate element: G1 -> Fq (8 words), G2 -> Fq2 (16 words)
enum class Curve { G1 = 1, G2 = 2 };

class MsmEngine {
 public:
  MsmEngine(Curve curve, size_t max_n, hipStream_t stream);
  ~MsmEngine();
  MsmEngine(const MsmEngine&) = delete;
  MsmEngine& operator=(const MsmEngine&) = delete;

  // points: device, affine, device layout (Montgomery R'=2^261, 8 LE words per Fq).
  // scalars: device, 8 LE 32-bit words per scalar (standard form, any value < 2^256).
  // Enqueues the whole pipeline on the engine's stream; the W window sums (XYZZ,
  // device layout, window_words() words) land in d_out (device).  Nothing is
  // synchronised: the caller orders/awaits the stream.
  void run(const uint32_t* points, const uint32_t* scalars, size_t n, uint32_t* d_out);
  size_t window_words() const { return (size_t)prm_.windows * 4 * fwords_; }

  // Kernel instrumentation (HIP events on this engine's stream).  When enabled,
  // every run() brackets the bucket-accumulate kernel with events and copies the
  // number of nonzero digits (= mixed additions) to pinned memory.  collect()
  // must be called after the stream is synchronised.
  struct Stats {
    double accumulate_ms = 0;  // summed over launches
    uint64_t launches = 0;
    uint64_t mixed_adds = 0;   // nonzero (point, window) digits processed
    uint64_t tasks = 0;
  };
  void set_instrument(bool on) { instrument_ = on; }
  void collect(Stats& s);
  const MsmParams& params() const { return prm_; }
  Curve curve() const { return curve_; }
  hipStream_t stream() const { return stream_; }
  size_t max_n() const { return max_n_; }

 private:
  Curve curve_;
  size_t max_n_;
  hipStream_t stream_;
  MsmParams prm_;
  size_t nbuckets_ = 0;     // windows * 2^(c-1)
  size_t max_entries_ = 0;  // max_n * windows
  size_t max_tasks_ = 0;
  int merge_levels_ = 0;
  // device buffers
  uint32_t *keys_ = nullptr, *vals_ = nullptr, *keys_sorted_ = nullptr, *vals_sorted_ = nullptr;
  uint32_t *bstart_ = nullptr, *bend_ = nullptr, *cnt_ = nullptr, *off_a_ = nullptr, *off_b_ = nullptr;
  uint32_t *part_a_ = nullptr, *part_b_ = nullptr, *buckets_ = nullptr;
  uint32_t *bcnt_ = nullptr, *boff_ = nullptr;  // compacted digit emission: per (window, block) counts/offsets
  uint32_t* h_valid_ = nullptr;                 // pinned: number of nonzero digits of the current run
  uint32_t last_valid_ = 0;
  uint32_t *lvl_s_[2] = {nullptr, nullptr}, *lvl_t_[2] = {nullptr, nullptr};
  void* sort_tmp_ = nullptr;
  size_t sort_tmp_bytes_ = 0;
  void* scan_tmp_ = nullptr;
  size_t scan_tmp_bytes_ = 0;
  int fwords_;  // words per field element (8 or 16)
  // instrumentation
  static constexpr int MAX_PENDING = 16;
  bool instrument_ = false;
  int pending_ = 0;
  hipEvent_t ev_[MAX_PENDING][2];
  uint32_t* h_counts_ = nullptr;  // pinned: [invalid-bucket start, end, tasks] per pending run
  uint32_t h_total_[MAX_PENDING] = {};
};

}  // namespace zkp
