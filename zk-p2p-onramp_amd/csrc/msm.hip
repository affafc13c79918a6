// Pippenger MSM engine for BN254 G1/G2 on gfx950.  See msm.hpp for the pipeline.
#include "msm.hpp"

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "curve.hpp"
#include "msm_kernels.hpp"
#include "hip_check.hpp"

namespace zkp {

namespace {

constexpr int TPB = 256;

inline unsigned grid_for(size_t n, int tpb = TPB) { return (unsigned)((n + tpb - 1) / tpb); }

__global__ __launch_bounds__(TPB) void k_digits(const uint32_t* __restrict__ scalars, uint32_t n, int c, int W,
                                                uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  msmk::digits(blockIdx.x * TPB + threadIdx.x, scalars, n, c, W, keys, vals);
}
constexpr int WAVES = TPB / 64;

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// pass 1 of the compacted digit emission: nonzero digits per (window, block)
__global__ __launch_bounds__(TPB) void k_digit_count(const uint32_t* __restrict__ scalars, uint32_t n, int c, int W,
                                                     uint32_t* __restrict__ bcnt) {
  __shared__ uint32_t cnt[32];
  if (threadIdx.x < 32) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  const bool active = i < n;
  uint32_t s[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (active) msmk::load_scalar(scalars, i, s);
  const uint32_t invalid = 0xffffffffu;
  uint32_t carry = 0;
  bool neg;
  for (int w = 0; w < W; ++w) {
    const uint32_t key = msmk::digit_key(s, w, c, carry, neg, invalid);
    const uint64_t m = __ballot(active && key != invalid);
    if ((threadIdx.x & 63) == 0) atomicAdd(&cnt[w], (uint32_t)__popcll(m));
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)W) bcnt[(size_t)threadIdx.x * gridDim.x + blockIdx.x] = cnt[threadIdx.x];
}

// pass 2: write (key, point | sign) of every nonzero digit at
//   boff[window][block] + (entries of earlier waves of the block) + (earlier lanes of the wave)
// -> window-major, point order within a window (deterministic)
__global__ __launch_bounds__(TPB) void k_digit_write(const uint32_t* __restrict__ scalars, uint32_t n, int c, int W,
                                                     const uint32_t* __restrict__ boff, uint32_t* __restrict__ keys,
                                                     uint32_t* __restrict__ vals) {
  __shared__ uint32_t wcnt[32][WAVES];
  const uint32_t i = blockIdx.x * TPB + threadIdx.x;
  const int wave = threadIdx.x >> 6;
  const bool active = i < n;
  uint32_t s[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (active) msmk::load_scalar(scalars, i, s);
  const uint32_t invalid = 0xffffffffu;
  uint32_t carry = 0;
  bool neg;
  for (int w = 0; w < W; ++w) {
    const uint32_t key = msmk::digit_key(s, w, c, carry, neg, invalid);
    const uint64_t m = __ballot(active && key != invalid);
    if ((threadIdx.x & 63) == 0) wcnt[w][wave] = (uint32_t)__popcll(m);
  }
  __syncthreads();
  carry = 0;
  for (int w = 0; w < W; ++w) {
    const uint32_t key = msmk::digit_key(s, w, c, carry, neg, invalid);
    const bool valid = active && key != invalid;
    const uint64_t m = __ballot(valid);
    if (valid) {
      uint32_t base = boff[(size_t)w * gridDim.x + blockIdx.x];
      for (int v = 0; v < wave; ++v) base += wcnt[w][v];
      const uint32_t pos = base + lane_rank(m);
      keys[pos] = key;
      vals[pos] = i | (neg ? 0x80000000u : 0u);
    }
  }
}

__global__ __launch_bounds__(TPB) void k_bounds(const uint32_t* __restrict__ keys, uint32_t total,
                                                uint32_t* __restrict__ start, uint32_t* __restrict__ end) {
  msmk::bounds(blockIdx.x * TPB + threadIdx.x, keys, total, start, end);
}
__global__ __launch_bounds__(TPB) void k_task_counts(const uint32_t* __restrict__ start,
                                                     const uint32_t* __restrict__ end, uint32_t nb, uint32_t S,
                                                     uint32_t* __restrict__ cnt) {
  msmk::task_counts(blockIdx.x * TPB + threadIdx.x, start, end, nb, S, cnt);
}
__global__ __launch_bounds__(TPB) void k_heavy_counts(const uint32_t* __restrict__ off, uint32_t nb, uint32_t S2,
                                                      int lvl, uint32_t* __restrict__ cnt) {
  msmk::heavy_counts(blockIdx.x * TPB + threadIdx.x, off, nb, S2, lvl, cnt);
}
template <class F>
__global__ __launch_bounds__(TPB) void k_accumulate(const uint32_t* __restrict__ points,
                                                    const uint32_t* __restrict__ vals,
                                                    const uint32_t* __restrict__ start,
                                                    const uint32_t* __restrict__ end,
                                                    const uint32_t* __restrict__ off, uint32_t nb, uint32_t S,
                                                    uint32_t* __restrict__ out) {
  msmk::accumulate<F>(blockIdx.x * TPB + threadIdx.x, points, vals, start, end, off, nb, S, out);
}
template <class F>
__global__ __launch_bounds__(TPB) void k_merge_heavy(const uint32_t* __restrict__ src,
                                                     const uint32_t* __restrict__ off,
                                                     const uint32_t* __restrict__ hoff, uint32_t nb, uint32_t S2,
                                                     int lvl, uint32_t* __restrict__ dst) {
  msmk::merge_heavy<F>(blockIdx.x * TPB + threadIdx.x, src, off, hoff, nb, S2, lvl, dst);
}
template <class F>
__global__ __launch_bounds__(TPB) void k_merge_final(const uint32_t* __restrict__ part0,
                                                     const uint32_t* __restrict__ part1,
                                                     const uint32_t* __restrict__ off, uint32_t nb, uint32_t S2,
                                                     int levels, uint32_t* __restrict__ buckets) {
  msmk::merge_final<F>(blockIdx.x * TPB + threadIdx.x, part0, part1, off, nb, S2, levels, buckets);
}
template <class F>
__global__ __launch_bounds__(TPB) void k_reduce_first(const uint32_t* __restrict__ buckets, uint32_t nwin,
                                                      uint32_t half, uint32_t L, uint32_t* __restrict__ s_out,
                                                      uint32_t* __restrict__ t_out) {
  msmk::reduce_first<F>(blockIdx.x * TPB + threadIdx.x, buckets, nwin, half, L, s_out, t_out);
}
template <class F>
__global__ __launch_bounds__(TPB) void k_reduce_level(const uint32_t* __restrict__ s_in,
                                                      const uint32_t* __restrict__ t_in, uint32_t nwin,
                                                      uint32_t n_in, uint32_t L, int lg_width,
                                                      uint32_t* __restrict__ s_out, uint32_t* __restrict__ t_out) {
  msmk::reduce_level<F>(blockIdx.x * TPB + threadIdx.x, s_in, t_in, nwin, n_in, L, lg_width, s_out, t_out);
}

template <class F>
void launch_accumulate(const uint32_t* points, const uint32_t* vals, const uint32_t* bstart, const uint32_t* bend,
                       const uint32_t* off, uint32_t nb, uint32_t S, uint32_t* out, size_t max_tasks,
                       hipStream_t st) {
  hipLaunchKernelGGL(k_accumulate<F>, dim3(grid_for(max_tasks)), dim3(TPB), 0, st, points, vals, bstart, bend, off,
                     nb, S, out);
}

}  // namespace

MsmEngine::MsmEngine(Curve curve, size_t max_n, hipStream_t stream)
    : curve_(curve), max_n_(std::max<size_t>(max_n, 1)), stream_(stream) {
  if (max_n_ >= (size_t(1) << 31)) throw std::runtime_error("MSM size too large");
  prm_ = MsmParams::for_size(max_n_);
  fwords_ = curve == Curve::G1 ? 8 : 16;
  const size_t half = size_t(1) << (prm_.c - 1);
  nbuckets_ = (size_t)prm_.windows * half;
  max_entries_ = max_n_ * prm_.windows;
  if (max_entries_ >= 0xffffffffull) throw std::runtime_error("MSM size too large for 32-bit entry indices");
  max_tasks_ = (max_entries_ + prm_.S - 1) / prm_.S + nbuckets_;
  {
    size_t m = (max_n_ + prm_.S - 1) / prm_.S;  // worst-case partials of one bucket
    merge_levels_ = 0;
    while (m > (size_t)prm_.S2) {
      m = (m + prm_.S2 - 1) / prm_.S2;
      ++merge_levels_;
    }
  }
  const size_t xyzz_words = 4 * (size_t)fwords_;
  HIPX(hipMalloc(&keys_, max_entries_ * 4));
  HIPX(hipMalloc(&vals_, max_entries_ * 4));
  HIPX(hipMalloc(&keys_sorted_, max_entries_ * 4));
  HIPX(hipMalloc(&vals_sorted_, max_entries_ * 4));
  HIPX(hipMalloc(&bstart_, (nbuckets_ + 1) * 4));
  HIPX(hipMalloc(&bend_, (nbuckets_ + 1) * 4));
  HIPX(hipMalloc(&cnt_, (nbuckets_ + 1) * 4));
  HIPX(hipMalloc(&off_a_, (nbuckets_ + 1) * 4));
  HIPX(hipMalloc(&off_b_, (nbuckets_ + 1) * 4));
  const size_t ncnt = (size_t)prm_.windows * grid_for(max_n_) + 1;  // per (window, digit block) counts
  HIPX(hipMalloc(&bcnt_, ncnt * 4));
  HIPX(hipMalloc(&boff_, ncnt * 4));
  HIPX(hipHostMalloc(&h_valid_, 4, hipHostMallocDefault));
  HIPX(hipMalloc(&part_a_, max_tasks_ * xyzz_words * 4));
  HIPX(hipMalloc(&part_b_, max_tasks_ * xyzz_words * 4));
  HIPX(hipMalloc(&buckets_, nbuckets_ * xyzz_words * 4));
  const size_t lvl1 = (size_t)prm_.windows * ((half + prm_.L - 1) / prm_.L);
  for (int i = 0; i < 2; ++i) {
    HIPX(hipMalloc(&lvl_s_[i], lvl1 * xyzz_words * 4));
    HIPX(hipMalloc(&lvl_t_[i], lvl1 * xyzz_words * 4));
  }
  int end_bit = 1;
  while ((size_t(1) << end_bit) <= nbuckets_) ++end_bit;
  HIPX(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp_bytes_, keys_, keys_sorted_, vals_, vals_sorted_,
                                          (int)max_entries_, 0, end_bit, stream_));
  HIPX(hipMalloc(&sort_tmp_, sort_tmp_bytes_));
  HIPX(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_tmp_bytes_, cnt_, off_a_,
                                        (int)std::max(nbuckets_ + 1, ncnt), stream_));
  HIPX(hipMalloc(&scan_tmp_, scan_tmp_bytes_));
  for (auto& e : ev_) {
    HIPX(hipEventCreate(&e[0]));
    HIPX(hipEventCreate(&e[1]));
  }
  HIPX(hipHostMalloc(&h_counts_, MAX_PENDING * 3 * 4, hipHostMallocDefault));
}

void MsmEngine::collect(Stats& s) {
  for (int i = 0; i < pending_; ++i) {
    float ms = 0;
    HIPX(hipEventElapsedTime(&ms, ev_[i][0], ev_[i][1]));
    s.accumulate_ms += ms;
    s.launches += 1;
    s.mixed_adds += h_total_[i];
    s.tasks += h_counts_[3 * i + 2];
  }
  pending_ = 0;
}

MsmEngine::~MsmEngine() {
  for (auto& e : ev_) {
    (void)hipEventDestroy(e[0]);
    (void)hipEventDestroy(e[1]);
  }
  if (h_counts_) (void)hipHostFree(h_counts_);
  if (h_valid_) (void)hipHostFree(h_valid_);
  for (void* p : {(void*)keys_, (void*)vals_, (void*)keys_sorted_, (void*)vals_sorted_, (void*)bstart_, (void*)bend_,
                  (void*)cnt_, (void*)off_a_, (void*)off_b_, (void*)part_a_, (void*)part_b_, (void*)buckets_,
                  (void*)lvl_s_[0], (void*)lvl_s_[1], (void*)lvl_t_[0], (void*)lvl_t_[1], sort_tmp_, scan_tmp_,
                  (void*)bcnt_, (void*)boff_})
    if (p) (void)hipFree(p);
}

void MsmEngine::run(const uint32_t* points, const uint32_t* scalars, size_t n, uint32_t* d_out) {
  if (n > max_n_) throw std::runtime_error("MSM: n exceeds engine capacity");
  const size_t xyzz_bytes = 16 * (size_t)fwords_;
  const uint32_t W = (uint32_t)prm_.windows;
  const uint32_t half = 1u << (prm_.c - 1);
  const uint32_t nb = (uint32_t)nbuckets_;
  hipStream_t st = stream_;
  if (n == 0) {
    // all windows = infinity
    HIPX(hipMemsetAsync(buckets_, 0, nbuckets_ * xyzz_bytes, st));
  } else {
    // 1. digits, compacted: only nonzero digits, window-major, point order within a window
    const uint32_t nblk = grid_for(n);
    hipLaunchKernelGGL(k_digit_count, dim3(nblk), dim3(TPB), 0, st, scalars, (uint32_t)n, prm_.c, (int)W, bcnt_);
    HIPX(hipMemsetAsync(bcnt_ + (size_t)W * nblk, 0, 4, st));
    size_t stmp0 = scan_tmp_bytes_;
    HIPX(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, stmp0, bcnt_, boff_, (int)((size_t)W * nblk + 1), st));
    hipLaunchKernelGGL(k_digit_write, dim3(nblk), dim3(TPB), 0, st, scalars, (uint32_t)n, prm_.c, (int)W, boff_,
                       keys_, vals_);
    HIPX(hipMemcpyAsync(h_valid_, boff_ + (size_t)W * nblk, 4, hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));  // the sort needs the entry count on the host
    const uint32_t total = *h_valid_;
    last_valid_ = total;
    if (total == 0) {
      HIPX(hipMemsetAsync(buckets_, 0, nbuckets_ * xyzz_bytes, st));
    } else {
      // 2. stable LSD sort on the (c-1) bucket bits only: windows stay grouped, so equal
      //    (window, bucket) keys end up contiguous after 2 radix passes instead of 3
      size_t tmp = sort_tmp_bytes_;
      HIPX(hipcub::DeviceRadixSort::SortPairs(sort_tmp_, tmp, keys_, keys_sorted_, vals_, vals_sorted_, (int)total,
                                              0, prm_.c - 1, st));
    HIPX(hipMemsetAsync(bstart_, 0, (nbuckets_ + 1) * 4, st));
    HIPX(hipMemsetAsync(bend_, 0, (nbuckets_ + 1) * 4, st));
    hipLaunchKernelGGL(k_bounds, dim3(grid_for(total)), dim3(TPB), 0, st, keys_sorted_, total, bstart_, bend_);
    hipLaunchKernelGGL(k_task_counts, dim3(grid_for(nbuckets_ + 1)), dim3(TPB), 0, st, bstart_, bend_, nb,
                       (uint32_t)prm_.S, cnt_);
    size_t stmp = scan_tmp_bytes_;
    HIPX(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, stmp, cnt_, off_a_, (int)(nbuckets_ + 1), st));
    const size_t max_tasks_now = ((size_t)total + prm_.S - 1) / prm_.S + nbuckets_;
    const int slot = (instrument_ && pending_ < MAX_PENDING) ? pending_++ : -1;
    if (slot >= 0) HIPX(hipEventRecord(ev_[slot][0], st));
    if (curve_ == Curve::G1)
      launch_accumulate<Fq>(points, vals_sorted_, bstart_, bend_, off_a_, nb, (uint32_t)prm_.S, part_a_,
                            max_tasks_now, st);
    else
      launch_accumulate<Fq2>(points, vals_sorted_, bstart_, bend_, off_a_, nb, (uint32_t)prm_.S, part_a_,
                             max_tasks_now, st);
    if (slot >= 0) {
      HIPX(hipEventRecord(ev_[slot][1], st));
      h_total_[slot] = total;  // every compacted entry is one mixed addition
      HIPX(hipMemcpyAsync(&h_counts_[3 * slot + 2], &off_a_[nb], 4, hipMemcpyDeviceToHost, st));
    }
    // merge levels for heavy buckets only (part_a <-> part_b at each bucket's own base off_a[b])
    size_t bound = max_tasks_now;
    for (int lv = 0; lv < merge_levels_; ++lv) {
      hipLaunchKernelGGL(k_heavy_counts, dim3(grid_for(nbuckets_ + 1)), dim3(TPB), 0, st, off_a_, nb,
                         (uint32_t)prm_.S2, lv, cnt_);
      stmp = scan_tmp_bytes_;
      HIPX(hipcub::DeviceScan::ExclusiveSum(scan_tmp_, stmp, cnt_, off_b_, (int)(nbuckets_ + 1), st));
      bound = 2 * bound / prm_.S2 + 1;  // heavy c > S2  =>  ceil(c/S2) <= 2c/S2
      const uint32_t* src = (lv & 1) ? part_b_ : part_a_;
      uint32_t* dst = (lv & 1) ? part_a_ : part_b_;
      if (curve_ == Curve::G1)
        hipLaunchKernelGGL(k_merge_heavy<Fq>, dim3(grid_for(bound)), dim3(TPB), 0, st, src, off_a_, off_b_, nb,
                           (uint32_t)prm_.S2, lv, dst);
      else
        hipLaunchKernelGGL(k_merge_heavy<Fq2>, dim3(grid_for(bound)), dim3(TPB), 0, st, src, off_a_, off_b_, nb,
                           (uint32_t)prm_.S2, lv, dst);
    }
    if (curve_ == Curve::G1)
      hipLaunchKernelGGL(k_merge_final<Fq>, dim3(grid_for(nbuckets_)), dim3(TPB), 0, st, part_a_, part_b_, off_a_,
                         nb, (uint32_t)prm_.S2, merge_levels_, buckets_);
    else
      hipLaunchKernelGGL(k_merge_final<Fq2>, dim3(grid_for(nbuckets_)), dim3(TPB), 0, st, part_a_, part_b_, off_a_,
                         nb, (uint32_t)prm_.S2, merge_levels_, buckets_);
    }
  }
  // bucket reduction tree per window
  const uint32_t L = (uint32_t)prm_.L;
  uint32_t nodes = (half + L - 1) / L;
  int cur = 0;
  if (curve_ == Curve::G1)
    hipLaunchKernelGGL(k_reduce_first<Fq>, dim3(grid_for((size_t)W * nodes)), dim3(TPB), 0, st, buckets_, W, half,
                       L, lvl_s_[0], lvl_t_[0]);
  else
    hipLaunchKernelGGL(k_reduce_first<Fq2>, dim3(grid_for((size_t)W * nodes)), dim3(TPB), 0, st, buckets_, W, half,
                       L, lvl_s_[0], lvl_t_[0]);
  int lg_width = 0;
  {
    uint32_t l = L;
    while (l > 1) {
      l >>= 1;
      ++lg_width;
    }
  }
  const int lg_L = lg_width;
  while (nodes > 1) {
    const uint32_t next = (nodes + L - 1) / L;
    if (curve_ == Curve::G1)
      hipLaunchKernelGGL(k_reduce_level<Fq>, dim3(grid_for((size_t)W * next)), dim3(TPB), 0, st, lvl_s_[cur],
                         lvl_t_[cur], W, nodes, L, lg_width, lvl_s_[cur ^ 1], lvl_t_[cur ^ 1]);
    else
      hipLaunchKernelGGL(k_reduce_level<Fq2>, dim3(grid_for((size_t)W * next)), dim3(TPB), 0, st, lvl_s_[cur],
                         lvl_t_[cur], W, nodes, L, lg_width, lvl_s_[cur ^ 1], lvl_t_[cur ^ 1]);
    cur ^= 1;
    nodes = next;
    lg_width += lg_L;
  }
  HIPX(hipGetLastError());
  HIPX(hipMemcpyAsync(d_out, lvl_t_[cur], (size_t)W * xyzz_bytes, hipMemcpyDeviceToDevice, st));
}

}  // namespace zkp
