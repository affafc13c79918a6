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
//     1. digits : compacted emission of the nonzero signed c-bit digits as
//                 (key = group*2^(c-1) + |d|-1, val = (t*n + i) | sign<<31),
//                 window-major, point order within a window.
//     2. sort   : stable radix sort on the c-1 bucket bits (groups stay grouped).
//     3. bounds : bucket [start, end) ranges, accumulate-task offsets (tasks of
//                 <= S entries never straddle a bucket) and the offsets of the
//                 heavy-bucket merge levels.
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
  int L = 8;         // fan-in of a subset-sum tree level
  int nb1 = 255;     // windows 0..nb1-1 are c bits wide, the rest c-1 (>= windows: all c bits)
  // c_override / depth_override: 0 = automatic.  balanced (only with depth == windows, one bucket
  // group): the W windows split the 255 digit bits as nb1 x c + (W - nb1) x (c - 1), so the top window
  // is not a narrow one whose n digits pile into its few low buckets (c = 20: 8 x 20 + 5 x 19 bits
  // instead of 12 x 20 + 15; the (c-1)-bit windows use the lower half of the shared buckets)
  static MsmParams make(size_t n, int c_override = 0, int depth_override = 0, bool balanced = false) {
    MsmParams p;
    int lg = 0;
    while ((size_t(1) << lg) < n) ++lg;
    // one bucket set of 2^(c-1) buckets against n*W entries: c = lg - 3 keeps every
    // bucket ~16*W entries deep and the bucket reduction (2^c full adds) < 2% of the
    // accumulation; 20 bits caps the sort at three 8-bit passes.
    p.c = c_override > 0 ? c_override : (lg - 4 < 8 ? 8 : (lg - 4 > 20 ? 20 : lg - 4));
    if (p.c < 2) p.c = 2;
    if (p.c > 24) p.c = 24;
    p.windows = (255 + p.c - 1) / p.c;
    p.depth = depth_override > 0 ? (depth_override < p.windows ? depth_override : p.windows) : p.windows;
    p.groups = (p.windows + p.depth - 1) / p.depth;
    if (p.M > (1 << (p.c - 1))) p.M = 1 << (p.c - 1);
    if (balanced && p.groups == 1 && p.c >= 3) {
      const int nb = 255 - p.windows * (p.c - 1);
      p.nb1 = nb < 0 ? 0 : (nb > p.windows ? p.windows : nb);
    }
    return p;
  }
  bool balanced() const { return nb1 < windows; }
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
// (tools/gpu/experiments/r2_hsort_c*.sh).  Keep c whose top window spans >= 12 bits (>= 128
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
  MsmBases(Curve curve, size_t n, int c, int depth, int nb1 = 255);
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
  int nb1() const { return nb1_; }
  Curve curve() const { return curve_; }
  size_t bytes() const { return bytes_; }
  static size_t bytes_for(Curve curve, size_t n, int depth) {
    return (size_t)depth * (n ? n : 1) * 8 * curve_fwords(curve);
  }

 private:
  Curve curve_;
  size_t n_;
  int c_, depth_, nb1_;
  size_t bytes_ = 0;
  uint32_t* d_ = nullptr;
};

class MsmPlan {
 public:
  MsmPlan(size_t max_n, const MsmParams& prm, hipStream_t stream);
  ~MsmPlan();
  MsmPlan(const MsmPlan&) = delete;
  MsmPlan& operator=(const MsmPlan&) = delete;
  // scalars: device, 8 LE 32-bit words each (standard form, any value < 2^256: reduced below r
  // when loaded, msm_kernels.hpp load_scalar, so W = ceil(255 / c) windows always hold the carry).
  // Enqueues on the plan's stream and blocks the host once (the task grid needs the
  // number of nonzero digits); records ready() at the end.  Grouping by bucket: a stable
  // rocprim radix sort, or with ZKP_PLAN_SORT=bins a two-level counting sort (msm.hip).
  void build(const uint32_t* scalars, size_t n);
  // dense emission (for uniform scalars, e.g. the H MSM's): every (window, point) digit is an
  // entry, zero digits keyed past the last bucket, so build() never blocks the host and the
  // entry count is the bound n * W (entries() then counts the rare zero digits too)
  void set_dense(bool d) { dense_ = d; }
  bool dense() const { return dense_; }
  const MsmParams& params() const { return prm_; }
  hipEvent_t ready() const { return ready_; }
  hipStream_t stream() const { return stream_; }
  size_t n() const { return n_; }
  size_t max_n() const { return max_n_; }
  // entries the accumulate grid is sized for: the nonzero digits, or for the hand-sorted plans (whose
  // count stays on the device: no host round trip) the bound n * W
  uint32_t entries() const { return total_; }
  // device word holding the exact nonzero-digit count once ready() (hand-sorted plans), else nullptr
  const uint32_t* entries_dev() const { return hs_built_ ? hs_binbase_ + hs_nbins_ : nullptr; }
  int merge_levels() const { return merge_levels_; }

  // device results (read-only once ready())
  const uint32_t* vals() const { return vals_sorted_; }
  const uint32_t* bstart() const { return bstart_; }
  const uint32_t* bend() const { return bend_; }
  const uint32_t* task_off() const { return off_task_; }
  const uint32_t* perm() const { return use_perm_ ? perm_ : nullptr; }  // task order (by length)
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
  uint32_t *keys_ = nullptr, *vals_ = nullptr, *keys_sorted_ = nullptr, *vals_sorted_ = nullptr;
  uint32_t *bstart_ = nullptr, *bend_ = nullptr, *cnt_ = nullptr, *off_task_ = nullptr;
  std::vector<uint32_t*> off_lvl_;                // merge level l's offsets: lvl_all_ + l * (buckets + 1)
  uint32_t *lvl_all_ = nullptr, *lvl_tsum_ = nullptr;
  uint32_t *bcnt_ = nullptr, *boff_ = nullptr;  // per (window, digit block) counts / offsets
  // bucket binning (default grouping): coarse bins x binning blocks counts / offsets
  bool use_bins_ = false;
  bool dense_ = false;
  int dense_bits_ = 0;                          // key bits of the dense sort (sentinel = buckets)
  int fine_bits_ = 0;
  uint32_t nbins_ = 0;
  uint32_t *hist_ = nullptr, *hoff_ = nullptr;
  uint32_t *nch_ = nullptr, *choff_ = nullptr, *hist2_ = nullptr, *hoff2_ = nullptr;
  size_t max_chunks_ = 0;
  uint32_t* h_valid_ = nullptr;                 // pinned: number of nonzero digits
  // dense plans: the hand-written three-pass LDS-staged bucket sort (hsort_kernels.hpp);
  // ZKP_H_SORT=rocprim restores the onesweep radix sort of the sentinel-keyed digits
  bool use_hsort_ = false;
  // compacted (witness) plans sorted by the same passes (ZKP_W_SORT=rocprim: the onesweep sort and
  // a host round trip for the entry count), always with the tiled pass C (skewed buckets); dense
  // plans take the one-workgroup-per-sub-bin pass C unless ZKP_HS_TILED_C=1
  bool use_wsort_ = false, hs_tiled_c_ = false, hs_built_ = false;
  uint32_t hs_max_tiles3_ = 0;
  uint32_t *hs_toff3_ = nullptr, *hs_hist3_ = nullptr, *hs_off3_ = nullptr;
  int hs_b2_ = 0, hs_b3_ = 0, hs_k_ = 1;  // hs_k_: scalars per thread in pass A
  uint32_t hs_nbins_ = 0, hs_nblk_ = 0, hs_max_tiles_ = 0;
  uint32_t *hs_hist_ = nullptr, *hs_blkoff_ = nullptr, *hs_bintot_ = nullptr, *hs_binbase_ = nullptr;
  uint32_t *hs_toff_ = nullptr, *hs_hist2_ = nullptr, *hs_off2_ = nullptr, *hs_subbase_ = nullptr;
  void *hs_ent_a_ = nullptr, *hs_ent_b_ = nullptr;  // 8-byte (key, base|sign) entries
  // accumulate-task order by length (ZKP_TASK_ORDER=bucket: bucket order)
  bool use_perm_ = false;
  uint32_t *perm_ = nullptr, *tl_hist_ = nullptr, *tl_off_ = nullptr;
  uint32_t* tsum_ = nullptr;                    // tile sums of the look-back-free scans
  size_t tsum_len_ = 0;
  void* sort_tmp_ = nullptr;
  size_t sort_tmp_bytes_ = 0;
  void* scan_tmp_ = nullptr;
  size_t scan_tmp_bytes_ = 0;
};

class MsmEngine {
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
  size_t window_words() const { return (size_t)prm_.groups * prm_.K() * 4 * fwords_; }

  // Kernel instrumentation (HIP events on this engine's stream).  When enabled,
  // every run() brackets the bucket-accumulate kernel with events; collect()
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
  hipEvent_t ev_[MAX_PENDING][2];
  uint32_t* h_counts_ = nullptr;  // pinned: tasks per pending run, then entries per pending run
  uint32_t h_total_[MAX_PENDING] = {};
  bool h_total_dev_[MAX_PENDING] = {};  // entries copied from the device (h_counts_[MAX_PENDING + i])
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
