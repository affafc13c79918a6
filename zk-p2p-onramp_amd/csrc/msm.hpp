// Pippenger multi-scalar multiplication over BN254 G1 / G2 on gfx950.
//
// Replaces ffjavascript ``G1.multiExpAffine`` / ``G2.multiExpAffine``
// (g1m/g2m_multiexpAffine_chunk) as called five times by
// snarkjs ``groth16_prove``.  Result is bit-identical as a group element; the
// algorithm is a GPU re-design, not a translation.  Three objects:
//
//  MsmBases  (per point set, built once at zkey load, resident in HBM)
//     depth T rows of the affine bases: row t = 2^(c*t) * P_i.  With T = W
//     (the default: 288 GB of HBM pays for it) every window of a scalar lands
//     in ONE shared set of 2^(c-1) buckets, so the per-window bucket reduction
//     and the host Horner fold disappear; with T < W the W windows fall into
//     G = ceil(W/T) bucket groups, folded by Horner with shift c*T.
//
//  MsmPlan   (per scalar vector, per proof; shared by every MSM over the same
//     scalars -- A, B1, C and the G2 MSM B2 all use the witness)
//     1. digits : the nonzero signed c-bit digits as (key = group*2^(c-1) + |d|-1,
//                 val = (t*n + i) | sign<<31), computed from the scalars inside
//     2. sort   : the hand-written three-pass LDS-staged bucket sort (hsort_kernels.hpp)
//     3. bounds : bucket [start, end) ranges, accumulate-task offsets (tasks of
//                 <= S entries never straddle a bucket), the task order by length and
//                 the offsets of the heavy-bucket merge levels.
//
//  MsmEngine (per curve and stream: partial sums, buckets, reduction tree)
//     4. accumulate: one thread per task, mixed XYZZ additions of gathered bases;
//                 every thread does the same bounded work whatever the scalar
//                 distribution (0/1-heavy witnesses put most points in one bucket).
//     5. merge  : buckets with more than 2*S2 task partials are folded by segmented
//                 merge levels that skip the light buckets; one thread per bucket
//                 sums what is left.
//     6. reduce : per group, sum_k (k+1) B_k = sum_p T_p + M sum_b 2^b Q_b from
//                 segment running sums (S_p, T_p over M buckets) and bit-subset
//                 sums Q_b = sum_{p: bit b} S_p, all plain L-ary tree sums.
//     7. out    : G x K points (XYZZ, device layout); the host applies the 2^b, M
//                 and group (2^(c T g)) weights by Horner (msm_fold).
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace zkp {

struct MsmParams {
  int c = 16;        // window bits
  int windows = 16;  // W = ceil(255 / c)   (254-bit scalars + the signed-digit carry)
  int depth = 16;    // T: precomputed rows per base
  int groups = 1;    // G = ceil(W / T) bucket groups
  int S = 32;        // max entries per accumulate task
  int S2 = 4;        // fan-in of a heavy-bucket merge level (short chains: latency-bound)
  int M = 4;         // buckets per reduction segment (running sums)
  // c_override / depth_override: 0 = automatic.  Window bits must lie in [MIN_C, MAX_C]: W <= 32
  // windows keep a scalar block's digits in one LDS stage of the bucket sort, and the bucket key
  // (group and bucket bits, <= 27) splits into its three passes (hsort_kernels.hpp).
  static constexpr int MIN_C = 8, MAX_C = 24;
  static MsmParams make(size_t n, int c_override = 0, int depth_override = 0) {
    MsmParams p;
    int lg = 0;
    while ((size_t(1) << lg) < n) ++lg;
    // one bucket set of 2^(c-1) buckets against n*W entries: c = lg - 4 keeps every bucket ~8*W
    // entries deep and the bucket reduction (2^c full adds) small; 20 bits caps the automatic choice
    p.c = c_override > 0 ? c_override : (lg - 4 < MIN_C ? MIN_C : (lg - 4 > 20 ? 20 : lg - 4));
    if (p.c < MIN_C || p.c > MAX_C)
      throw std::invalid_argument("MSM window bits must be within " + std::to_string(MIN_C) + ".." +
                                  std::to_string(MAX_C) + " (got " + std::to_string(p.c) + ")");
    p.windows = (255 + p.c - 1) / p.c;
    p.depth = depth_override > 0 ? (depth_override < p.windows ? depth_override : p.windows) : p.windows;
    p.groups = (p.windows + p.depth - 1) / p.depth;
    if (p.M > (1 << (p.c - 1))) p.M = 1 << (p.c - 1);
    return p;
  }
  // reduction output: per group, lgP subset sums Q_b and sum_p T_p (P = 2^(c-1) / M segments)
  int lg_m() const { int l = 0; while ((1 << l) < M) ++l; return l; }
  int lgP() const { return c - 1 - lg_m(); }
  int K() const { return lgP() + 1; }
  size_t half() const { return size_t(1) << (c - 1); }
  size_t buckets() const { return (size_t)groups * half(); }
};

// Window bits for a DENSE plan (hand-written bucket sort) near c.  The top window of a 254-bit
// scalar holds only 254 - (W - 1) c digit bits: for c = 18, 19, 21 (2, 7, 2 bits) all n of its
// digits fall into a handful of buckets, i.e. into one or a few sub-bins of the sort's pass C,
// which gives every sub-bin ONE workgroup -- measured 1.3 ms for that kernel alone at 2^20
// points and c = 18 (0.05 ms at c = 20), +13 ms per Venmo proof at c = 21
// (273c6e8:tools/gpu/experiments/r2_hsort_c*.sh).  Keep c whose top window spans >= 12 bits (>= 128
// sub-bins), trying c+1, c-1, c+2, ... within [8, 20]; below 2^17 points one workgroup per
// sub-bin copes (n entries at most), so c stays.
inline int dense_window_bits(int c, size_t n) {
  auto top = [](int cc) { return 254 - ((255 + cc - 1) / cc - 1) * cc; };
  if (n < (size_t(1) << 17) || top(c) >= 12) return c;
  for (int d = 1; d <= 6; ++d) {
    if (c + d <= 20 && top(c + d) >= 12) return c + d;
    if (c - d >= 8 && top(c - d) >= 12) return c - d;
  }
  return c;
}

// words per coordinate element: G1 -> Fq (8 words), G2 -> Fq2 (16 words)
enum class Curve { G1 = 1, G2 = 2 };

inline int curve_fwords(Curve c) { return c == Curve::G1 ? 8 : 16; }

// Precomputed base table: rows() x n affine points (device layout, Montgomery R'=2^261).
class MsmBases {
 public:
  MsmBases(Curve curve, size_t n, int c, int depth);
  ~MsmBases();
  MsmBases(const MsmBases&) = delete;
  MsmBases& operator=(const MsmBases&) = delete;
  // row 0 (n points): the caller fills it (device layout), then extend() derives rows 1..T-1
  uint32_t* row0() { return d_; }
  void extend(hipStream_t st);
  const uint32_t* data() const { return d_; }
  size_t n() const { return n_; }
  int c() const { return c_; }
  int depth() const { return depth_; }
  Curve curve() const { return curve_; }
  size_t bytes() const { return bytes_; }
  static size_t bytes_for(Curve curve, size_t n, int depth) {
    return (size_t)depth * (n ? n : 1) * 8 * curve_fwords(curve);
  }

 private:
  Curve curve_;
  size_t n_;
  int c_, depth_;
  size_t bytes_ = 0;
  uint32_t* d_ = nullptr;
};

class MsmPlan {
  struct Init {};  // the delegated-to constructor: members only, so a failing allocation in the
                   // delegating one runs the destructor (no device memory leaks on out-of-memory)
  MsmPlan(Init, size_t max_n, const MsmParams& prm, hipStream_t stream);

 public:
  MsmPlan(size_t max_n, const MsmParams& prm, hipStream_t stream);
  ~MsmPlan();
  MsmPlan(const MsmPlan&) = delete;
  MsmPlan& operator=(const MsmPlan&) = delete;
  // scalars: device, 8 LE 32-bit words each (standard form, any value < 2^256: reduced below r
  // when loaded, msm_kernels.hpp load_scalar, so W = ceil(255 / c) windows always hold the carry).
  // Enqueues on the plan's stream, never blocks the host (the exact entry count stays on the
  // device: entries_dev()); records ready() at the end.
  void build(const uint32_t* scalars, size_t n);
  // dense (uniform scalars, e.g. the H MSM's: nearly every digit is nonzero and the buckets evenly
  // filled): pass C of the sort takes one workgroup per sub-bin; otherwise (the 0/1-heavy witness:
  // whole waves of entries in one bucket) wave-aggregated LDS claims and a tiled pass C
  void set_dense(bool d) { dense_ = d; }
  bool dense() const { return dense_; }
  const MsmParams& params() const { return prm_; }
  hipEvent_t ready() const { return ready_; }
  hipStream_t stream() const { return stream_; }
  size_t n() const { return n_; }
  size_t max_n() const { return max_n_; }
  // entries the accumulate grid is sized for: the bound n * W (the exact count stays on the device)
  uint32_t entries() const { return total_; }
  // device word holding the exact nonzero-digit count once ready() (nullptr for an empty plan)
  const uint32_t* entries_dev() const { return hs_built_ ? hs_binbase_ + hs_nbins_ : nullptr; }
  int merge_levels() const { return merge_levels_; }

  // device results (read-only once ready())
  const uint32_t* vals() const { return vals_sorted_; }
  const uint32_t* bstart() const { return bstart_; }
  const uint32_t* bend() const { return bend_; }
  const uint32_t* task_off() const { return off_task_; }
  const uint32_t* perm() const { return perm_; }  // task order (by length)
  const uint32_t* level_off(int lv) const { return off_lvl_[lv]; }
  size_t max_tasks_now() const { return max_tasks_now_; }
  size_t max_tasks() const { return max_tasks_; }

 private:
  MsmParams prm_;
  size_t max_n_, n_ = 0;
  hipStream_t stream_;
  hipEvent_t ready_ = nullptr;
  size_t nbuckets_ = 0, max_entries_ = 0, max_tasks_ = 0, max_tasks_now_ = 0;
  int merge_levels_ = 0;
  uint32_t total_ = 0;
  uint32_t *vals_sorted_ = nullptr;              // base|sign words in bucket order (the accumulation's input)
  uint32_t *bstart_ = nullptr, *bend_ = nullptr, *cnt_ = nullptr, *off_task_ = nullptr;
  std::vector<uint32_t*> off_lvl_;                // merge level l's offsets: lvl_all_ + l * (buckets + 1)
  uint32_t *lvl_all_ = nullptr, *lvl_tsum_ = nullptr;
  bool dense_ = false;
  // the three-pass LDS-staged bucket sort (hsort_kernels.hpp)
  bool hs_built_ = false;
  uint32_t hs_max_tiles3_ = 0;
  uint32_t *hs_toff3_ = nullptr, *hs_hist3_ = nullptr, *hs_off3_ = nullptr;
  int hs_b2_ = 0, hs_b3_ = 0, hs_k_ = 1;  // hs_k_: scalars per thread in pass A
  uint32_t hs_nbins_ = 0, hs_nblk_ = 0, hs_max_tiles_ = 0;
  uint32_t *hs_hist_ = nullptr, *hs_blkoff_ = nullptr, *hs_binbase_ = nullptr;
  uint32_t *hs_toff_ = nullptr, *hs_hist2_ = nullptr, *hs_off2_ = nullptr, *hs_subbase_ = nullptr;
  void *hs_ent_a_ = nullptr, *hs_ent_b_ = nullptr;  // 8-byte (key, base|sign) entries
  // accumulate-task order by length (longest first)
  uint32_t *perm_ = nullptr, *tl_hist_ = nullptr, *tl_off_ = nullptr;
  uint32_t* tsum_ = nullptr;                    // tile sums of the look-back-free scans
};

class MsmEngine {
  struct Init {};  // as MsmPlan::Init
  MsmEngine(Init, Curve curve, const MsmParams& prm, size_t max_n, hipStream_t stream);

 public:
  MsmEngine(Curve curve, const MsmParams& prm, size_t max_n, hipStream_t stream);
  ~MsmEngine();
  MsmEngine(const MsmEngine&) = delete;
  MsmEngine& operator=(const MsmEngine&) = delete;

  // sum_i s_i * P_i for the plan's scalars over the bases (bases.n() == plan.n(),
  // same c and depth).  Waits for plan.ready() on the engine's stream, enqueues
  // everything there; the G group sums (XYZZ, device layout, window_words() words)
  // land in d_out (device).  Nothing is synchronised.
  void run(const MsmPlan& plan, const MsmBases& bases, uint32_t* d_out);
  // the same in two phases: accumulate() on the engine's stream (bucket-task partial sums),
  // finish() (merges + reduction + output) on stream `st` (0 = the engine's), which the
  // caller must order after accumulate(), e.g. by an event; lets a stream run the next
  // MSM's accumulation while another finishes this one
  void accumulate(const MsmPlan& plan, const MsmBases& bases);
  void finish(const MsmPlan& plan, uint32_t* d_out, hipStream_t st = nullptr);
  size_t window_words() const { return window_words_for(curve_, prm_); }
  static size_t window_words_for(Curve c, const MsmParams& p) { return (size_t)p.groups * p.K() * 4 * curve_fwords(c); }

  // Kernel instrumentation (HIP events on this engine's stream).  When enabled,
  // every run() brackets the bucket-accumulate kernel with events; collect()
  // must be called after the stream is synchronised.
  struct Launch {
    float ms;       // HIP events on the engine's stream around the launch
    uint32_t adds;  // nonzero digits it accumulated (mixed additions)
    uint32_t blocks;  // workgroups of the launch (matches a kernel trace's grid size / TPB)
  };
  struct Stats {
    double accumulate_ms = 0;  // summed over launches
    uint64_t launches = 0;
    uint64_t mixed_adds = 0;   // nonzero (point, window) digits processed
    uint64_t tasks = 0;
    std::vector<Launch> per_launch;  // every collected launch, in order
  };
  void set_instrument(bool on) { instrument_ = on; }
  void collect(Stats& s);
  const MsmParams& params() const { return prm_; }
  Curve curve() const { return curve_; }
  hipStream_t stream() const { return stream_; }

 private:
  Curve curve_;
  MsmParams prm_;
  size_t max_n_;
  hipStream_t stream_;
  size_t nbuckets_ = 0, max_tasks_ = 0;
  int fwords_;
  uint32_t *part_a_ = nullptr, *part_b_ = nullptr, *buckets_ = nullptr;
  uint32_t *seg_s_ = nullptr, *seg_t_ = nullptr, *sub_[2] = {nullptr, nullptr};
  static constexpr int MAX_PENDING = 16;
  bool instrument_ = false;
  int pending_ = 0;
  hipEvent_t ev_[MAX_PENDING][2] = {};
  uint32_t* h_counts_ = nullptr;  // pinned: tasks per pending run, then entries per pending run
  uint32_t h_total_[MAX_PENDING] = {};
  bool h_total_dev_[MAX_PENDING] = {};
  uint32_t h_blocks_[MAX_PENDING] = {};  // entries copied from the device (h_counts_[MAX_PENDING + i])
};

// merge levels needed for n points with the given params (worst case: one bucket of
// a group receives a digit of every window of the group)
inline int msm_merge_levels(size_t max_n, const MsmParams& prm) {
  size_t m = ((max_n ? max_n : 1) * (size_t)prm.depth + prm.S - 1) / prm.S;
  int levels = 0;
  while (m > 2 * (size_t)prm.S2) {
    m = (m + prm.S2 - 1) / prm.S2;
    ++levels;
  }
  return levels;
}

}  // namespace zkp
