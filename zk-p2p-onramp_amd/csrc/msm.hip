// Pippenger MSM engine for BN254 G1/G2 on gfx950.  See msm.hpp for the pipeline.
#include "msm.hpp"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "curve.hpp"
#include "msm_kernels.hpp"
#include "hip_check.hpp"

namespace zkp {

namespace {

constexpr int TPB = 256;

inline unsigned grid_for(size_t n, int tpb = TPB) { return (unsigned)((n + tpb - 1) / tpb); }

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// row t of the base table from row t-1: 2^c * P, affine.  One launch per row keeps
// every launch short (~T-1 launches of n threads at zkey load).
template <class F>
__global__ __launch_bounds__(TPB) void k_extend_row(uint32_t* __restrict__ table, uint32_t n, int dbl, int t) {
  msmk::extend_row<F>(blockIdx.x * TPB + threadIdx.x, table, n, dbl, t);
}

// G2 (Fq2) accumulation and bucket merges (the wide finish kernels): without a bound the
// compiler takes 256 VGPRs + AGPRs (one wave per SIMD, nothing to hide the mad-chain
// latency); two waves per SIMD (a few spilled dwords; accumulation measured 5.24 -> 4.55 ms
// per 6.4 M-point G2 MSM)
// (G1: no bound, 118 VGPRs and four waves per SIMD; 3 / 5 / 6 waves measured slower, profiles/acc_waves_r03.txt)
template <class F>
struct AccWaves {
  static constexpr int value = FWords<F>::W == 16 ? 2 : 1;
};
template <class F>
struct MergeWaves {
  static constexpr int value = FWords<F>::W == 16 ? 2 : 1;
};
template <class F>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(AccWaves<F>::value))) void k_accumulate(const uint32_t* __restrict__ points,
                                                    const uint32_t* __restrict__ vals,
                                                    const uint32_t* __restrict__ start,
                                                    const uint32_t* __restrict__ end,
                                                    const uint32_t* __restrict__ off, uint32_t nb, uint32_t S,
                                                    const uint32_t* __restrict__ perm, uint32_t* __restrict__ out) {
  msmk::accumulate<F>(blockIdx.x * TPB + threadIdx.x, points, vals, start, end, off, nb, S, perm, out);
}

// accumulate-task order by length, longest first (a counting sort over the S + 1 lengths): the
// lanes of a wave then run chains of equal length -- without it every bucket's short last task
// idles the lanes beside it (~7 % of the uniform-scalar H accumulation at S = 32)
__global__ __launch_bounds__(TPB) void k_tlen_count(const uint32_t* __restrict__ start, const uint32_t* __restrict__ end,
                                                    const uint32_t* __restrict__ off, uint32_t nb, uint32_t S,
                                                    uint32_t* __restrict__ hist) {
  extern __shared__ uint32_t h[];  // S + 1 counters
  for (uint32_t k = threadIdx.x; k <= S; k += TPB) h[k] = 0;
  __syncthreads();
  const uint32_t t = blockIdx.x * TPB + threadIdx.x;
  if (t < off[nb]) atomicAdd(&h[S - msmk::task_len(t, start, end, off, nb, S)], 1u);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k <= S; k += TPB) hist[(size_t)k * gridDim.x + blockIdx.x] = h[k];
}
__global__ __launch_bounds__(TPB) void k_tlen_scatter(const uint32_t* __restrict__ start,
                                                      const uint32_t* __restrict__ end,
                                                      const uint32_t* __restrict__ off, uint32_t nb, uint32_t S,
                                                      const uint32_t* __restrict__ hoff, uint32_t* __restrict__ perm) {
  extern __shared__ uint32_t cur[];  // S + 1 cursors
  for (uint32_t k = threadIdx.x; k <= S; k += TPB) cur[k] = hoff[(size_t)k * gridDim.x + blockIdx.x];
  __syncthreads();
  const uint32_t t = blockIdx.x * TPB + threadIdx.x;
  if (t < off[nb]) perm[atomicAdd(&cur[S - msmk::task_len(t, start, end, off, nb, S)], 1u)] = t;
}
template <class F>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(MergeWaves<F>::value))) void k_merge_heavy(const uint32_t* __restrict__ src,
                                                     const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ hoff, uint32_t nb, uint32_t S2,
                                                     int lvl, uint32_t* __restrict__ dst) {
  msmk::merge_heavy<F>(blockIdx.x * TPB + threadIdx.x, src, off, hoff, nb, S2, lvl, dst);
}
template <class F>
__global__ __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(MergeWaves<F>::value))) void k_merge_final(const uint32_t* __restrict__ part0,
                                                     const uint32_t* __restrict__ part1,
                                                     const uint32_t* __restrict__ off, uint32_t nb, uint32_t S2,
                                                     int levels, uint32_t* __restrict__ buckets) {
  msmk::merge_final<F>(blockIdx.x * TPB + threadIdx.x, part0, part1, off, nb, S2, levels, buckets);
}
template <class F>
__global__ __launch_bounds__(TPB) void k_reduce_segments(const uint32_t* __restrict__ buckets, uint32_t G,
                                                         uint32_t half, uint32_t M, uint32_t* __restrict__ s_out,
                                                         uint32_t* __restrict__ t_out) {
  msmk::reduce_segments<F>(blockIdx.x * TPB + threadIdx.x, buckets, G, half, M, s_out, t_out);
}
template <class F>
__global__ __launch_bounds__(TPB) void k_subset_first(const uint32_t* __restrict__ s_in,
                                                      const uint32_t* __restrict__ t_in, uint32_t G, uint32_t lgP,
                                                      uint32_t fan, uint32_t* __restrict__ out) {
  msmk::subset_first<F>(blockIdx.x * TPB + threadIdx.x, s_in, t_in, G, lgP, fan, out);
}
// (no waves-per-SIMD bound: a latency-bound tree, one wave per SIMD suffices; bounding the G2 variant
// to two waves spills ~290 dwords)
template <class F>
__global__ __launch_bounds__(msmk::TREE_TPB) void k_subset_tree_first(
    const uint32_t* __restrict__ s_in, const uint32_t* __restrict__ t_in, uint32_t lgP, uint32_t nch,
    uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[msmk::XyzzLimbs<F>::N * (msmk::TREE_TPB / 2)];
  msmk::subset_tree_first<F>(s_in, t_in, lgP, nch, blockIdx.y, blockIdx.x, lds, out);
}
template <class F>
__global__ __launch_bounds__(msmk::TREE_TPB) void k_subset_tree_next(
    const uint32_t* __restrict__ in, uint32_t n_in, uint32_t n_out, uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[msmk::XyzzLimbs<F>::N * (msmk::TREE_TPB / 2)];
  msmk::subset_tree_next<F>(in, n_in, n_out, blockIdx.y, blockIdx.x, lds, out);
}
// largest first-level tree grid (workgroups): larger subset sums (the proof's H MSM: 18 sums of 2^16
// values) start with a full-lane fan-in chain level (profiles/subset_tree_r02.txt)
constexpr size_t TREE_FIRST_MAX = 512;

// count (or, with rank != nullptr, claim a slot for) one entry in LDS counter h[b]; lanes of a
// wave that all hit the same counter (the skewed buckets of 0/1 witness values) use one atomic
__device__ __forceinline__ uint32_t lds_claim(uint32_t* h, uint32_t b, bool valid) {
  const uint64_t m = __ballot(valid);
  if (!m) return 0;
  const int leader = __builtin_ctzll(m);
  const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)b, leader);
  const uint64_t same = __ballot(valid && b == b0);
  if (same == m) {
    uint32_t base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(&h[b0], (uint32_t)__popcll(m));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
    return base + lane_rank(m);
  }
  return valid ? atomicAdd(&h[b], 1u) : 0u;
}

#include "hsort_kernels.hpp"

// heavy-merge grid bound per level: heavy c > S2  =>  ceil(c/S2) <= 2c/S2
inline size_t level_bound(size_t bound, int S2) { return 2 * bound / S2 + 1; }

template <class F>
void run_accumulate(const MsmPlan& plan, const MsmBases& bases, uint32_t* part_a, hipStream_t st, hipEvent_t ev0,
                    hipEvent_t ev1) {
  const MsmParams& prm = plan.params();
  const uint32_t nb = (uint32_t)prm.buckets();
  if (ev0) HIPX(hipEventRecord(ev0, st));
  if (plan.entries() > 0)
    hipLaunchKernelGGL(k_accumulate<F>, dim3(grid_for(plan.max_tasks_now())), dim3(TPB), 0, st, bases.data(),
                       plan.vals(), plan.bstart(), plan.bend(), plan.task_off(), nb, (uint32_t)prm.S, plan.perm(),
                       part_a);
  if (ev1) HIPX(hipEventRecord(ev1, st));
  HIPX(hipGetLastError());
}

template <class F>
void run_finish(const MsmPlan& plan, uint32_t* part_a, uint32_t* part_b, uint32_t* buckets, uint32_t* seg_s,
                uint32_t* seg_t, uint32_t* const sub[2], uint32_t* d_out, hipStream_t st) {
  const MsmParams& prm = plan.params();
  const uint32_t nb = (uint32_t)prm.buckets();
  const uint32_t half = (uint32_t)prm.half();
  const uint32_t G = (uint32_t)prm.groups;
  const size_t xyzz_bytes = 16 * (size_t)FWords<F>::W;
  size_t bound = plan.max_tasks_now();
  for (int lv = 0; lv < plan.merge_levels() && plan.entries() > 0; ++lv) {
    bound = level_bound(bound, prm.S2);
    const uint32_t* src = (lv & 1) ? part_b : part_a;
    uint32_t* dst = (lv & 1) ? part_a : part_b;
    hipLaunchKernelGGL(k_merge_heavy<F>, dim3(grid_for(bound)), dim3(TPB), 0, st, src, plan.task_off(),
                       plan.level_off(lv), nb, (uint32_t)prm.S2, lv, dst);
  }
  hipLaunchKernelGGL(k_merge_final<F>, dim3(grid_for(nb)), dim3(TPB), 0, st, part_a, part_b, plan.task_off(), nb,
                     (uint32_t)prm.S2, plan.merge_levels(), buckets);
  // bucket reduction: segments, then the K = lgP + 1 subset sums per group by L-ary tree
  const uint32_t M = (uint32_t)prm.M, lgP = (uint32_t)prm.lgP(), K = (uint32_t)prm.K();
  hipLaunchKernelGGL(k_reduce_segments<F>, dim3(grid_for((size_t)G * (half / M))), dim3(TPB), 0, st, buckets, G, half,
                     M, seg_s, seg_t);
  // workgroup LDS trees: 2 * TREE_TPB values per workgroup and launch level
  int cur = 0;
  constexpr uint32_t CH = 2 * msmk::TREE_TPB;
  uint32_t n = ((1u << lgP) + CH - 1) / CH;
  if ((size_t)G * K * n <= TREE_FIRST_MAX) {  // about one round of workgroups: the tree from the inputs
    hipLaunchKernelGGL(k_subset_tree_first<F>, dim3(n, G * K), dim3(msmk::TREE_TPB), 0, st, seg_s, seg_t, lgP, n,
                       sub[0]);
  } else {  // many inputs (the H MSM: K x 2^16): a full-lane fan-in chain level first (short: the
            // trees above it take the rest), then trees
    const uint32_t cf = msmk::TREE_CHAIN_FAN;
    n = (((1u << lgP) + 2 * cf - 1) / (2 * cf));
    hipLaunchKernelGGL(k_subset_first<F>, dim3(grid_for((size_t)G * K * n)), dim3(TPB), 0, st, seg_s, seg_t, G, lgP,
                       cf, sub[0]);
  }
  while (n > 1) {
    const uint32_t next = (n + CH - 1) / CH;
    hipLaunchKernelGGL(k_subset_tree_next<F>, dim3(next, G * K), dim3(msmk::TREE_TPB), 0, st, sub[cur], n, next,
                       sub[cur ^ 1]);
    cur ^= 1;
    n = next;
  }
  HIPX(hipGetLastError());
  HIPX(hipMemcpyAsync(d_out, sub[cur], (size_t)G * K * xyzz_bytes, hipMemcpyDeviceToDevice, st));
}

}  // namespace

// ------------------------------------------------------------------ MsmBases

MsmBases::MsmBases(Curve curve, size_t n, int c, int depth) : curve_(curve), n_(n), c_(c), depth_(depth) {
  if (depth < 1 || c < 2) throw std::runtime_error("MsmBases: bad parameters");
  if ((size_t)depth * std::max<size_t>(n, 1) >= (size_t(1) << 31))
    throw std::runtime_error("MsmBases: depth * n must stay below 2^31 (31-bit base indices)");
  bytes_ = bytes_for(curve, n, depth);
  HIPX(hipMalloc(&d_, bytes_));
}

MsmBases::~MsmBases() {
  if (d_) (void)hipFree(d_);
}

void MsmBases::extend(hipStream_t st) {
  if (n_ == 0) return;
  for (int t = 1; t < depth_; ++t) {
    if (curve_ == Curve::G1)
      hipLaunchKernelGGL(k_extend_row<Fq>, dim3(grid_for(n_)), dim3(TPB), 0, st, d_, (uint32_t)n_, c_, t);
    else
      hipLaunchKernelGGL(k_extend_row<Fq2>, dim3(grid_for(n_)), dim3(TPB), 0, st, d_, (uint32_t)n_, c_, t);
  }
  HIPX(hipGetLastError());
}

// ------------------------------------------------------------------ MsmPlan

MsmPlan::MsmPlan(Init, size_t max_n, const MsmParams& prm, hipStream_t stream)
    : prm_(prm), max_n_(std::max<size_t>(max_n, 1)), stream_(stream) {}

MsmPlan::MsmPlan(size_t max_n, const MsmParams& prm, hipStream_t stream) : MsmPlan(Init{}, max_n, prm, stream) {
  if (prm_.c < MsmParams::MIN_C || prm_.c > MsmParams::MAX_C || prm_.windows > HS_STAGE / HS_TPB)
    throw std::invalid_argument("MSM: window bits outside the plan's range");
  if (max_n_ * prm_.depth >= (size_t(1) << 31)) throw std::runtime_error("MSM size too large for 31-bit base indices");
  nbuckets_ = prm_.buckets();
  max_entries_ = max_n_ * prm_.windows;
  if (max_entries_ >= 0xffffffffull) throw std::runtime_error("MSM size too large for 32-bit entry indices");
  max_tasks_ = (max_entries_ + prm_.S - 1) / prm_.S + nbuckets_;
  merge_levels_ = msm_merge_levels(max_n_, prm_);
  HIPX(hipMalloc(&vals_sorted_, max_entries_ * 4));
  HIPX(hipMalloc(&bstart_, (nbuckets_ + 1) * 4));
  HIPX(hipMalloc(&bend_, (nbuckets_ + 1) * 4));
  HIPX(hipMalloc(&cnt_, (nbuckets_ + 1) * 4));
  HIPX(hipMalloc(&off_task_, (nbuckets_ + 1) * 4));
  HIPX(hipMalloc(&perm_, max_tasks_ * 4));
  const size_t ntl = (size_t)(prm_.S + 1) * grid_for(max_tasks_);
  HIPX(hipMalloc(&tl_hist_, ntl * 4));
  HIPX(hipMalloc(&tl_off_, ntl * 4));
  off_lvl_.assign(merge_levels_, nullptr);
  if (merge_levels_ > 0) {
    HIPX(hipMalloc(&lvl_all_, (size_t)merge_levels_ * (nbuckets_ + 1) * 4));
    for (int l = 0; l < merge_levels_; ++l) off_lvl_[l] = lvl_all_ + (size_t)l * (nbuckets_ + 1);
    HIPX(hipMalloc(&lvl_tsum_, (size_t)merge_levels_ * scan_tiles_for(nbuckets_ + 1) * 4));
  }
  // bucket-key bits kb = b1 (bin) + b2 (sub-bin) + b3 (bucket in sub-bin): b3 = 5 for the one-
  // workgroup-per-sub-bin pass C (k_hs_fine), up to 9 (tiled pass C) when kb > 23 (c > 20 with
  // several bucket groups); b1, b2 <= 9
  int kb = 1;
  while ((size_t(1) << kb) < nbuckets_) ++kb;
  hs_b3_ = std::max(std::min(kb, HS_B3), kb - HS_MAX_B1 - HS_MAX_B2);
  hs_b2_ = (kb - hs_b3_) / 2;
  const int b1 = kb - hs_b3_ - hs_b2_;
  if (b1 > HS_MAX_B1 || hs_b2_ > HS_MAX_B2 || hs_b3_ > HS_MAX_B2)
    throw std::invalid_argument("MSM: too many buckets for the bucket sort (window bits x bucket groups)");
  hs_nbins_ = (uint32_t)((nbuckets_ + (size_t(1) << (hs_b2_ + hs_b3_)) - 1) >> (hs_b2_ + hs_b3_));
  hs_k_ = std::max(1, std::min(4, HS_STAGE / (HS_TPB * prm_.windows)));
  if (hs_k_ == 3) hs_k_ = 2;
  hs_nblk_ = (uint32_t)((max_n_ + hs_k_ * HS_TPB - 1) / (hs_k_ * HS_TPB));
  hs_max_tiles_ = (uint32_t)((max_entries_ + HS_TILE - 1) / HS_TILE + hs_nbins_);
  const uint32_t nq = hs_nbins_ << hs_b2_;
  hs_max_tiles3_ = (uint32_t)((max_entries_ + HS_TILE - 1) / HS_TILE + nq);
  const size_t nh3 = ((size_t)hs_max_tiles3_ << hs_b3_) + 1;
  HIPX(hipMalloc(&hs_toff3_, ((size_t)nq + 1) * 4));
  HIPX(hipMalloc(&hs_hist3_, nh3 * 4));
  HIPX(hipMalloc(&hs_off3_, nh3 * 4));
  const size_t nh = (size_t)hs_nbins_ * hs_nblk_, nh2 = (size_t)hs_max_tiles_ << hs_b2_;
  HIPX(hipMalloc(&hs_hist_, nh * 4));
  HIPX(hipMalloc(&hs_blkoff_, nh * 4));
  HIPX(hipMalloc(&hs_binbase_, (hs_nbins_ + 1) * 4));
  HIPX(hipMalloc(&hs_toff_, (hs_nbins_ + 1) * 4));
  HIPX(hipMalloc(&hs_hist2_, nh2 * 4));
  HIPX(hipMalloc(&hs_off2_, nh2 * 4));
  HIPX(hipMalloc(&hs_subbase_, ((size_t)nq + 1) * 4));
  HIPX(hipMalloc(&hs_ent_a_, max_entries_ * 8));
  HIPX(hipMalloc(&hs_ent_b_, max_entries_ * 8));
  const size_t scan_n = std::max(std::max(std::max(nbuckets_ + 1, nh3), std::max(nh2, ntl)), nh);
  HIPX(hipMalloc(&tsum_, (scan_tiles_for(scan_n) + 1) * 4));
  HIPX(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
}

MsmPlan::~MsmPlan() {
  if (ready_) (void)hipEventDestroy(ready_);
  for (void* p : {(void*)vals_sorted_, (void*)bstart_, (void*)bend_, (void*)cnt_, (void*)off_task_, (void*)hs_hist_,
                  (void*)hs_blkoff_, (void*)hs_binbase_, (void*)hs_toff_, (void*)hs_hist2_,
                  (void*)hs_off2_, (void*)hs_subbase_, hs_ent_a_, hs_ent_b_, (void*)tsum_, (void*)perm_,
                  (void*)tl_hist_, (void*)tl_off_, (void*)hs_toff3_, (void*)hs_hist3_, (void*)hs_off3_,
                  (void*)lvl_all_, (void*)lvl_tsum_})
    if (p) (void)hipFree(p);
}

void MsmPlan::build(const uint32_t* scalars, size_t n) {
  if (n > max_n_) throw std::runtime_error("MSM: n exceeds plan capacity");
  n_ = n;
  const uint32_t W = (uint32_t)prm_.windows;
  const uint32_t nb = (uint32_t)nbuckets_;
  hipStream_t st = stream_;
  // total_ = n * W bounds the nonzero digits (the accumulate grid: threads past the last task exit),
  // so nothing waits on the host; the exact count stays on the device (entries_dev)
  total_ = (uint32_t)(n * W);
  hs_built_ = false;
  if (total_ == 0) {
    HIPX(hipMemsetAsync(bstart_, 0, (nbuckets_ + 1) * 4, st));
    HIPX(hipMemsetAsync(bend_, 0, (nbuckets_ + 1) * 4, st));
    HIPX(hipMemsetAsync(cnt_, 0, (nbuckets_ + 1) * 4, st));
  } else {
    // the hand-written three-pass LDS-staged bucket sort (hsort_kernels.hpp), zero digits dropped in
    // pass A.  Dense plans (uniform scalars: the H MSM) group their sub-bins with one workgroup each
    // (k_hs_fine); compacted plans (the witness: whole waves of one bin / sub-bin / bucket) take the
    // wave-aggregated LDS claims and the tiled pass C, as do keys with more than 5 bucket bits per
    // sub-bin
    const int k = hs_k_;
    const uint32_t nblk = (uint32_t)((n + k * HS_TPB - 1) / (k * HS_TPB)), nsub = 1u << hs_b2_;
    const int sh1 = hs_b2_ + hs_b3_;
    uint2* ea = static_cast<uint2*>(hs_ent_a_);
    uint2* eb = static_cast<uint2*>(hs_ent_b_);
    // A: digits -> bins
    auto count1 = k == 4 ? k_hs_count1<4> : (k == 2 ? k_hs_count1<2> : k_hs_count1<1>);
    hipLaunchKernelGGL(count1, dim3(nblk), dim3(HS_TPB), 0, st, scalars, (uint32_t)n, prm_.c, (int)W, prm_.depth, sh1,
                       hs_nbins_, hs_hist_);
    scan_nolookback(hs_hist_, hs_blkoff_, (size_t)hs_nbins_ * nblk, tsum_, st);
    hipLaunchKernelGGL(k_hs_binbase, dim3(1), dim3(512), 0, st, hs_blkoff_, hs_hist_, hs_nbins_, nblk, hs_binbase_,
                       hs_toff_);
    auto scatter1 = k == 4 ? k_hs_scatter1<4> : (k == 2 ? k_hs_scatter1<2> : k_hs_scatter1<1>);
    const size_t lds1 = (size_t)k * HS_TPB * W * 8 + (size_t)hs_nbins_ * 8;
    hipLaunchKernelGGL(scatter1, dim3(nblk), dim3(HS_TPB), lds1, st, scalars, (uint32_t)n, prm_.c, (int)W, prm_.depth,
                       sh1, hs_nbins_, hs_blkoff_, ea);
    // B: bins -> sub-bins (tiles past the used ones exit; their counters stay zero)
    const size_t tiles = ((size_t)total_ + HS_TILE - 1) / HS_TILE + hs_nbins_;
    const size_t nh2 = tiles << hs_b2_;
    HIPX(hipMemsetAsync(hs_hist2_, 0, nh2 * 4, st));
    const bool skew = !dense_;
    hipLaunchKernelGGL((skew ? k_hs_count2<true> : k_hs_count2<false>), dim3((unsigned)tiles), dim3(HS_TPB), 0, st, ea,
                       hs_binbase_, hs_toff_, hs_nbins_, hs_b3_, nsub, hs_hist2_);
    scan_nolookback(hs_hist2_, hs_off2_, nh2, tsum_, st);
    const uint32_t nq = hs_nbins_ * nsub;
    hipLaunchKernelGGL(k_hs_subbase, dim3(grid_for(nq + 1)), dim3(HS_TPB), 0, st, hs_off2_, hs_binbase_, hs_toff_,
                       hs_nbins_, nsub, hs_subbase_);
    hipLaunchKernelGGL((skew ? k_hs_scatter2<true, false> : k_hs_scatter2<false, false>), dim3((unsigned)tiles),
                       dim3(HS_TPB), 0, st, ea, hs_binbase_, hs_toff_, hs_nbins_, hs_b3_, nsub, hs_off2_, eb, nullptr);
    // C: sub-bins -> buckets, bounds and task counts
    if (dense_ && hs_b3_ <= HS_B3) {
      hipLaunchKernelGGL(k_hs_fine, dim3(nq), dim3(HS_FINE_TPB), 0, st, eb, hs_subbase_, nq, hs_b3_, nb,
                         (uint32_t)prm_.S, vals_sorted_, bstart_, bend_, cnt_);
    } else {  // tiled: pass B one level down (no workgroup takes more than HS_TILE entries)
      const uint32_t nf = 1u << hs_b3_;
      hipLaunchKernelGGL(k_hs_subtiles, dim3(1), dim3(SC_TPB), 0, st, hs_subbase_, nq, hs_toff3_);
      const size_t tiles3 = ((size_t)total_ + HS_TILE - 1) / HS_TILE + nq, nh3 = tiles3 << hs_b3_;
      HIPX(hipMemsetAsync(hs_hist3_, 0, nh3 * 4, st));
      hipLaunchKernelGGL(k_hs_count2<true>, dim3((unsigned)tiles3), dim3(HS_TPB), 0, st, eb, hs_subbase_, hs_toff3_, nq,
                         0, nf, hs_hist3_);
      scan_nolookback(hs_hist3_, hs_off3_, nh3, tsum_, st);
      hipLaunchKernelGGL((k_hs_scatter2<true, true>), dim3((unsigned)tiles3), dim3(HS_TPB), 0, st, eb, hs_subbase_,
                         hs_toff3_, nq, 0, nf, hs_off3_, nullptr, vals_sorted_);
      hipLaunchKernelGGL(k_hs_bounds3, dim3(grid_for((size_t)nb + 1)), dim3(HS_TPB), 0, st, hs_toff3_, hs_off3_,
                         hs_subbase_, hs_b3_, nb, (uint32_t)prm_.S, bstart_, bend_, cnt_);
    }
    hs_built_ = true;
  }
  // accumulate-task offsets and the heavy-bucket merge levels' offsets (look-back-free scans: they
  // run beside the accumulations of the other streams)
  scan_nolookback(cnt_, off_task_, nbuckets_ + 1, tsum_, st);
  max_tasks_now_ = ((size_t)total_ + prm_.S - 1) / prm_.S + nbuckets_;
  if (total_ > 0) {
    // accumulate-task order by length, longest first
    const unsigned nblk = grid_for(max_tasks_now_);
    const size_t lds = (size_t)(prm_.S + 1) * 4, nh = (size_t)(prm_.S + 1) * nblk;
    hipLaunchKernelGGL(k_tlen_count, dim3(nblk), dim3(TPB), lds, st, bstart_, bend_, off_task_, nb, (uint32_t)prm_.S,
                       tl_hist_);
    scan_nolookback(tl_hist_, tl_off_, nh, tsum_, st);
    hipLaunchKernelGGL(k_tlen_scatter, dim3(nblk), dim3(TPB), lds, st, bstart_, bend_, off_task_, nb,
                       (uint32_t)prm_.S, tl_off_, perm_);
  }
  if (merge_levels_ > 0 && total_ > 0) {
    const uint32_t nt = (uint32_t)scan_tiles_for(nbuckets_ + 1);
    hipLaunchKernelGGL(k_lvl_tiles, dim3(nt), dim3(SC_TPB), 0, st, off_task_, nb, (uint32_t)prm_.S2, merge_levels_,
                       nt, lvl_tsum_);
    hipLaunchKernelGGL(k_lvl_top, dim3(merge_levels_), dim3(SC_TPB), 0, st, lvl_tsum_, nt);
    hipLaunchKernelGGL(k_lvl_apply, dim3(nt), dim3(SC_TPB), 0, st, off_task_, nb, (uint32_t)prm_.S2, merge_levels_,
                       nt, lvl_tsum_, lvl_all_);
  }
  HIPX(hipGetLastError());
  HIPX(hipEventRecord(ready_, st));
}

// ------------------------------------------------------------------ MsmEngine

MsmEngine::MsmEngine(Init, Curve curve, const MsmParams& prm, size_t max_n, hipStream_t stream)
    : curve_(curve), prm_(prm), max_n_(std::max<size_t>(max_n, 1)), stream_(stream) {}

MsmEngine::MsmEngine(Curve curve, const MsmParams& prm, size_t max_n, hipStream_t stream)
    : MsmEngine(Init{}, curve, prm, max_n, stream) {
  fwords_ = curve_fwords(curve);
  const size_t half = prm_.half();
  nbuckets_ = prm_.buckets();
  max_tasks_ = (max_n_ * prm_.windows + prm_.S - 1) / prm_.S + nbuckets_;
  const size_t xyzz_words = 4 * (size_t)fwords_;
  HIPX(hipMalloc(&part_a_, max_tasks_ * xyzz_words * 4));
  HIPX(hipMalloc(&part_b_, max_tasks_ * xyzz_words * 4));
  HIPX(hipMalloc(&buckets_, nbuckets_ * xyzz_words * 4));
  const size_t nseg = (size_t)prm_.groups * (half / prm_.M);
  HIPX(hipMalloc(&seg_s_, nseg * xyzz_words * 4));
  HIPX(hipMalloc(&seg_t_, nseg * xyzz_words * 4));
  const size_t n1 = (size_t)prm_.groups * prm_.K() *
                    std::max(((half / prm_.M) + 2 * msmk::TREE_CHAIN_FAN - 1) / (2 * msmk::TREE_CHAIN_FAN),
                             ((half / prm_.M) + 2 * msmk::TREE_TPB - 1) / (2 * msmk::TREE_TPB));
  for (int i = 0; i < 2; ++i) HIPX(hipMalloc(&sub_[i], n1 * xyzz_words * 4));
  for (auto& e : ev_) {
    HIPX(hipEventCreate(&e[0]));
    HIPX(hipEventCreate(&e[1]));
  }
  HIPX(hipHostMalloc(&h_counts_, 2 * MAX_PENDING * 4, hipHostMallocDefault));
}

MsmEngine::~MsmEngine() {
  for (auto& e : ev_) {
    if (e[0]) (void)hipEventDestroy(e[0]);
    if (e[1]) (void)hipEventDestroy(e[1]);
  }
  if (h_counts_) (void)hipHostFree(h_counts_);
  for (void* p : {(void*)part_a_, (void*)part_b_, (void*)buckets_, (void*)seg_s_, (void*)seg_t_, (void*)sub_[0],
                  (void*)sub_[1]})
    if (p) (void)hipFree(p);
}

void MsmEngine::collect(Stats& s) {
  for (int i = 0; i < pending_; ++i) {
    float ms = 0;
    HIPX(hipEventElapsedTime(&ms, ev_[i][0], ev_[i][1]));
    const uint32_t adds = h_total_dev_[i] ? h_counts_[MAX_PENDING + i] : h_total_[i];
    s.accumulate_ms += ms;
    s.launches += 1;
    s.mixed_adds += adds;
    s.tasks += h_counts_[i];
    s.per_launch.push_back({ms, adds, h_blocks_[i]});
  }
  pending_ = 0;
}

void MsmEngine::accumulate(const MsmPlan& plan, const MsmBases& bases) {
  const MsmParams& p = plan.params();
  if (p.c != prm_.c || p.depth != prm_.depth || p.windows != prm_.windows)
    throw std::runtime_error("MSM: plan and engine parameters differ");
  if (bases.c() != p.c || bases.depth() != p.depth || bases.curve() != curve_)
    throw std::runtime_error("MSM: base table does not match the plan (c, depth, curve)");
  if (bases.n() != plan.n()) throw std::runtime_error("MSM: base table size differs from the scalar count");
  if (plan.n() > max_n_) throw std::runtime_error("MSM: n exceeds engine capacity");
  HIPX(hipStreamWaitEvent(stream_, plan.ready(), 0));
  const int slot = (instrument_ && pending_ < MAX_PENDING && plan.entries() > 0) ? pending_++ : -1;
  hipEvent_t e0 = slot >= 0 ? ev_[slot][0] : nullptr, e1 = slot >= 0 ? ev_[slot][1] : nullptr;
  if (curve_ == Curve::G1)
    run_accumulate<Fq>(plan, bases, part_a_, stream_, e0, e1);
  else
    run_accumulate<Fq2>(plan, bases, part_a_, stream_, e0, e1);
  if (slot >= 0) {
    h_total_[slot] = plan.entries();  // every nonzero digit is one mixed addition
    h_blocks_[slot] = (uint32_t)grid_for(plan.max_tasks_now());
    h_total_dev_[slot] = plan.entries_dev() != nullptr;
    if (h_total_dev_[slot])  // hand-sorted plans: the exact count, not the grid bound n * W
      HIPX(hipMemcpyAsync(&h_counts_[MAX_PENDING + slot], plan.entries_dev(), 4, hipMemcpyDeviceToHost, stream_));
    HIPX(hipMemcpyAsync(&h_counts_[slot], plan.task_off() + plan.params().buckets(), 4, hipMemcpyDeviceToHost,
                        stream_));
  }
}

void MsmEngine::finish(const MsmPlan& plan, uint32_t* d_out, hipStream_t st) {
  if (!st) st = stream_;
  if (curve_ == Curve::G1)
    run_finish<Fq>(plan, part_a_, part_b_, buckets_, seg_s_, seg_t_, sub_, d_out, st);
  else
    run_finish<Fq2>(plan, part_a_, part_b_, buckets_, seg_s_, seg_t_, sub_, d_out, st);
}

void MsmEngine::run(const MsmPlan& plan, const MsmBases& bases, uint32_t* d_out) {
  accumulate(plan, bases);
  finish(plan, d_out, stream_);
}

}  // namespace zkp
