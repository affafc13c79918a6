// Bucket sort of an MSM plan (the H MSM's uniform quotient scalars and the witness MSMs' 0/1-heavy
// ones), hand-written for gfx950, included by msm.hip.  It groups the nonzero (window, point) digits
// by bucket key for the accumulate tasks.  No workgroup ever waits on another one: every pass is
// reduce-then-scan (a decoupled look-back radix sort, rocprim's onesweep, stalled whenever the blocks
// it waits on shared the CUs with the long accumulation kernels of the other streams:
// profiles/plan_sort_r02.json).
//
// Key bits kb = ceil(log2 buckets) split as b1 (bin) + b2 (sub-bin) + b3 (bucket in sub-bin);
// for the Venmo H plan (2^19 buckets) 7 + 7 + 5; b3 grows past 5 (tiled pass C) only for kb > 23.  Three MSD passes, every scatter staged in LDS
// so that consecutive lanes write consecutive addresses of one destination run:
//   A  k_hs_count1 / scan / k_hs_binbase / k_hs_scatter1
//        digits computed from the scalars (zero digits dropped), grouped by bin: per (bin, block
//        of K * HS_TPB scalars, <= HS_STAGE entries) counts, their bin-major exclusive scan (every
//        (bin, block) run's position), bin bases; a
//        block's entries counted, scanned and placed in LDS, then written as runs (~52 entries
//        per bin for 2^7 bins), entries (key, base|sign) as one 8-byte word
//   B  k_hs_count2 / scan / k_hs_subbase / k_hs_scatter2
//        every bin cut into tiles of HS_TILE entries; per (bin, sub-bin, tile) counts in one flat
//        array laid out bin-major, sub-bin, tile -- its exclusive scan IS every (sub-bin, tile)
//        run's final position; a tile staged whole in LDS (64 KiB) and written as runs of
//        ~HS_TILE / 2^b2 entries
//   C  k_hs_fine: one workgroup per sub-bin (~6.6 K entries): LDS histogram of the b3 bucket bits,
//        bucket bounds + accumulate-task counts, then the bucket-sorted base|sign words built in
//        LDS and written out contiguously (sub-bins above HS_CAP entries -- skewed scalars --
//        scatter straight to global memory instead)
// Order inside a bucket is not fixed (LDS atomics); a bucket sum is the same group element in
// any order, so the MSM result does not change.
// Included by msm.hip inside namespace zkp's anonymous namespace (needs msm_kernels.hpp).
#pragma once

constexpr int HS_TPB = 256;
constexpr int HS_STAGE = 8192;      // pass-A LDS stage (entries of 8 B: 64 KiB)
constexpr int HS_TILE = 8192;       // pass-B tile (64 KiB of LDS)
constexpr int HS_CAP = 8192;        // pass-C sub-bins up to this many entries sort in LDS (32 KiB)
constexpr int HS_FINE_TPB = 512;
constexpr int HS_MAX_B1 = 9, HS_MAX_B2 = 9, HS_B3 = 5;
constexpr int SC_TPB = 1024;        // look-back-free scan
constexpr int SC_TILE = SC_TPB * 4;

// exclusive scan of one value per thread over a workgroup of NT threads (NT % 64 == 0)
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  uint32_t wbase = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const uint32_t s = sh[w];
    wbase += w < wave ? s : 0u;
    tot += s;
  }
  __syncthreads();
  total = tot;
  return wbase + x - v;
}

// exclusive scan in place of cnt[0..m) (m <= PER * NT) held in LDS; returns the total
template <int NT, int PER>
__device__ __forceinline__ uint32_t lds_excl_scan(uint32_t* cnt, uint32_t m, uint32_t* sh) {
  uint32_t v[PER], sum = 0;
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const uint32_t b = threadIdx.x * PER + p;
    v[p] = b < m ? cnt[b] : 0u;
    sum += v[p];
  }
  uint32_t total;
  uint32_t e = block_excl_scan<NT>(sum, sh, total);
#pragma unroll
  for (int p = 0; p < PER; ++p) {
    const uint32_t b = threadIdx.x * PER + p;
    if (b < m) cnt[b] = e;
    e += v[p];
  }
  __syncthreads();
  return total;
}

// ---------------------------------------------------------------- look-back-free device scan
// out[j] = sum of in[< j] for j < n: tile sums, one workgroup scans them, every tile adds its base
__global__ __launch_bounds__(SC_TPB) void k_scan_tiles(const uint32_t* __restrict__ in, uint32_t n,
                                                       uint32_t* __restrict__ tsum) {
  __shared__ uint32_t sh[SC_TPB / 64];
  uint32_t v = 0;
  const size_t base = (size_t)blockIdx.x * SC_TILE + threadIdx.x * 4;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (base + q < n) v += in[base + q];
  uint32_t tot;
  (void)block_excl_scan<SC_TPB>(v, sh, tot);
  if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}
__global__ __launch_bounds__(SC_TPB) void k_scan_top(uint32_t* __restrict__ tsum, uint32_t nt) {
  __shared__ uint32_t sh[SC_TPB / 64];
  uint32_t carry = 0;
  for (uint32_t j0 = 0; j0 < nt; j0 += SC_TPB) {
    const uint32_t j = j0 + threadIdx.x;
    const uint32_t v = j < nt ? tsum[j] : 0u;
    uint32_t tot;
    const uint32_t e = block_excl_scan<SC_TPB>(v, sh, tot);
    if (j < nt) tsum[j] = carry + e;
    carry += tot;
  }
}
__global__ __launch_bounds__(SC_TPB) void k_scan_apply(const uint32_t* __restrict__ in, uint32_t n,
                                                       const uint32_t* __restrict__ tsum, uint32_t* __restrict__ out) {
  __shared__ uint32_t sh[SC_TPB / 64];
  const size_t base = (size_t)blockIdx.x * SC_TILE + threadIdx.x * 4;
  uint32_t v[4], run = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    v[q] = base + q < n ? in[base + q] : 0u;
    run += v[q];
  }
  uint32_t tot;
  uint32_t e = block_excl_scan<SC_TPB>(run, sh, tot) + tsum[blockIdx.x];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (base + q < n) out[base + q] = e;
    e += v[q];
  }
}
inline size_t scan_tiles_for(size_t n) { return (n + SC_TILE - 1) / SC_TILE; }
inline void scan_nolookback(const uint32_t* in, uint32_t* out, size_t n, uint32_t* tsum, hipStream_t st) {
  const unsigned nt = (unsigned)scan_tiles_for(n);
  hipLaunchKernelGGL(k_scan_tiles, dim3(nt), dim3(SC_TPB), 0, st, in, (uint32_t)n, tsum);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SC_TPB), 0, st, tsum, nt);
  hipLaunchKernelGGL(k_scan_apply, dim3(nt), dim3(SC_TPB), 0, st, in, (uint32_t)n, tsum, out);
}

// ---------------------------------------------------------------- heavy-bucket merge levels
// Every merge level's offsets in one go (three launches instead of four per level): level l's
// count of bucket b is a function of its task count alone (msmk::heavy_counts), so the tiles
// scan all levels at once; out[l * (nb + 1) + b] = sum over b' < b of level l's counts.
__device__ __forceinline__ uint32_t lvl_count(uint32_t c0, uint32_t S2, int lvl) {
  int applied;
  const uint32_t c = msmk::merged_count(c0, S2, lvl, applied);
  return (applied == lvl && c > 2 * S2) ? (c + S2 - 1) / S2 : 0u;
}
__global__ __launch_bounds__(SC_TPB) void k_lvl_tiles(const uint32_t* __restrict__ off, uint32_t nb, uint32_t S2,
                                                      int L, uint32_t nt, uint32_t* __restrict__ tsum) {
  __shared__ uint32_t sh[SC_TPB / 64];
  const size_t base = (size_t)blockIdx.x * SC_TILE + threadIdx.x * 4;
  uint32_t c0[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) c0[q] = base + q < nb ? off[base + q + 1] - off[base + q] : 0u;
  for (int l = 0; l < L; ++l) {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) v += lvl_count(c0[q], S2, l);
    uint32_t tot;
    (void)block_excl_scan<SC_TPB>(v, sh, tot);
    if (threadIdx.x == 0) tsum[(size_t)l * nt + blockIdx.x] = tot;
  }
}
__global__ __launch_bounds__(SC_TPB) void k_lvl_top(uint32_t* __restrict__ tsum, uint32_t nt) {
  __shared__ uint32_t sh[SC_TPB / 64];
  uint32_t* t = tsum + (size_t)blockIdx.x * nt;
  uint32_t carry = 0;
  for (uint32_t j0 = 0; j0 < nt; j0 += SC_TPB) {
    const uint32_t j = j0 + threadIdx.x;
    const uint32_t v = j < nt ? t[j] : 0u;
    uint32_t tot;
    const uint32_t e = block_excl_scan<SC_TPB>(v, sh, tot);
    if (j < nt) t[j] = carry + e;
    carry += tot;
  }
}
__global__ __launch_bounds__(SC_TPB) void k_lvl_apply(const uint32_t* __restrict__ off, uint32_t nb, uint32_t S2,
                                                      int L, uint32_t nt, const uint32_t* __restrict__ tsum,
                                                      uint32_t* __restrict__ out) {
  __shared__ uint32_t sh[SC_TPB / 64];
  const size_t base = (size_t)blockIdx.x * SC_TILE + threadIdx.x * 4;
  uint32_t c0[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) c0[q] = base + q < nb ? off[base + q + 1] - off[base + q] : 0u;
  for (int l = 0; l < L; ++l) {
    uint32_t v[4], run = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = lvl_count(c0[q], S2, l);
      run += v[q];
    }
    uint32_t tot;
    uint32_t e = block_excl_scan<SC_TPB>(run, sh, tot) + tsum[(size_t)l * nt + blockIdx.x];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (base + q <= nb) out[(size_t)l * (nb + 1) + base + q] = e;
      e += v[q];
    }
  }
}

// ---------------------------------------------------------------- pass A: digits -> bins
// a workgroup takes K * HS_TPB scalars (K * HS_TPB * W <= HS_STAGE entries), K per thread
template <int K>
__global__ __launch_bounds__(HS_TPB) void k_hs_count1(const uint32_t* __restrict__ scalars, uint32_t n, int c, int W,
                                                      int T, int sh1, uint32_t nbins, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[1 << HS_MAX_B1];
  for (uint32_t b = threadIdx.x; b < nbins; b += HS_TPB) h[b] = 0;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < K; ++q) {
    const uint32_t i = blockIdx.x * (K * HS_TPB) + q * HS_TPB + threadIdx.x;
    if (i >= n) break;
    uint32_t s[9];
    msmk::load_scalar(scalars, i, s);
    uint32_t carry = 0;
    for (int w = 0; w < W; ++w) {
      uint32_t key, val;
      if (msmk::digit_entry(s, w, c, T, n, i, carry, key, val)) atomicAdd(&h[key >> sh1], 1u);
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += HS_TPB) hist[(size_t)b * gridDim.x + blockIdx.x] = h[b];
}

// bin bases and pass-B tile offsets from the exclusive scan of the whole bin-major hist[bin][blk] array
// (nbins <= 512, one workgroup): that scan IS every (bin, block) run's final position (bin base + the
// block's offset inside its bin), so a look-back-free device scan (3 full-width launches) replaces the
// per-bin sequential scan that one workgroup per bin did over ~16 K blocks (0.3 ms on the H plan's
// critical path, round 6):  binbase[b] = entries of bins < b (binbase[nbins] = all), toff[b] = tiles of
// bins < b
__global__ __launch_bounds__(512) void k_hs_binbase(const uint32_t* __restrict__ pos, const uint32_t* __restrict__ hist,
                                                    uint32_t nbins, uint32_t nblk, uint32_t* __restrict__ binbase,
                                                    uint32_t* __restrict__ toff) {
  __shared__ uint32_t sh[512 / 64];
  const size_t last = (size_t)nbins * nblk - 1;
  const uint32_t all = pos[last] + hist[last];
  const uint32_t b = threadIdx.x;
  const uint32_t lo = b < nbins ? pos[(size_t)b * nblk] : all;
  const uint32_t hi = b + 1 < nbins ? pos[(size_t)(b + 1) * nblk] : all;
  const uint32_t v = b < nbins ? hi - lo : 0u;
  uint32_t ttot;
  const uint32_t te = block_excl_scan<512>((v + HS_TILE - 1) / HS_TILE, sh, ttot);
  if (b < nbins) binbase[b] = lo, toff[b] = te;
  if (b == 0) binbase[nbins] = all, toff[nbins] = ttot;
}

// the block's digits counted per bin, scanned, placed in an LDS stage grouped by bin (LDS
// atomics), then the stage written out linearly: consecutive lanes, consecutive addresses of a run
template <int K>
__global__ __launch_bounds__(HS_TPB) void k_hs_scatter1(const uint32_t* __restrict__ scalars, uint32_t n, int c,
                                                        int W, int T, int sh1, uint32_t nbins,
                                                        const uint32_t* __restrict__ pos,
                                                        uint2* __restrict__ ent) {
  constexpr int NB = 1 << HS_MAX_B1;
  // dynamic LDS: the stage (K * HS_TPB * W entries) then cnt / off (nbins each): 54.3 KiB for the
  // H plan (W = 13, K = 2, 2^7 bins) -> three workgroups per CU
  extern __shared__ uint2 stage[];
  uint32_t* cnt = reinterpret_cast<uint32_t*>(stage + K * HS_TPB * W);
  uint32_t* off = cnt + nbins;
  __shared__ uint32_t sh[HS_TPB / 64];
  for (uint32_t b = threadIdx.x; b < nbins; b += HS_TPB) cnt[b] = 0;
  __syncthreads();
  // the block's entries stay in registers between the count and the placement (K * W <= EM * K)
  constexpr int EM = HS_STAGE / HS_TPB / K;
  constexpr uint32_t NONE = 0xffffffffu;
  uint2 e[K][EM];
#pragma unroll
  for (int q = 0; q < K; ++q) {
    const uint32_t i = blockIdx.x * (K * HS_TPB) + q * HS_TPB + threadIdx.x;
    uint32_t s[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const bool act = i < n;
    if (act) msmk::load_scalar(scalars, i, s);
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < EM; ++w) {
      e[q][w] = make_uint2(NONE, 0u);
      if (w < W) {
        uint32_t key, val;
        if (msmk::digit_entry(s, w, c, T, n, i, carry, key, val) && act) {
          e[q][w] = make_uint2(key, val);
          atomicAdd(&cnt[key >> sh1], 1u);
        }
      }
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += HS_TPB) off[b] = cnt[b];
  __syncthreads();
  const uint32_t total = lds_excl_scan<HS_TPB, NB / HS_TPB>(off, nbins, sh);
  for (uint32_t b = threadIdx.x; b < nbins; b += HS_TPB) cnt[b] = off[b];  // cursors
  __syncthreads();
#pragma unroll
  for (int q = 0; q < K; ++q)
#pragma unroll
    for (int w = 0; w < EM; ++w)
      if (e[q][w].x != NONE) stage[atomicAdd(&cnt[e[q][w].x >> sh1], 1u)] = e[q][w];
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nbins; b += HS_TPB)  // the cursors become destination bases
    off[b] = pos[(size_t)b * gridDim.x + blockIdx.x] - off[b];
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < total; j += HS_TPB) {
    const uint2 e = stage[j];
    ent[off[e.x >> sh1] + j] = e;
  }
}

// ---------------------------------------------------------------- pass B: bins -> sub-bins
struct HsTile {
  uint32_t b, t, nt, lo, hi;
};
__device__ __forceinline__ bool hs_tile(const uint32_t* __restrict__ binbase, const uint32_t* __restrict__ toff,
                                        uint32_t nbins, uint32_t id, HsTile& r) {
  if (id >= toff[nbins]) return false;
  r.b = msmk::seg_search(toff, nbins, id);
  r.t = id - toff[r.b];
  r.nt = toff[r.b + 1] - toff[r.b];
  r.lo = binbase[r.b] + r.t * HS_TILE;
  r.hi = msmk::umin(binbase[r.b + 1], r.lo + HS_TILE);
  return true;
}

// hist2[(toff[b] * nsub) + sub * nt_b + t]: entries of tile t of bin b in sub-bin `sub`
// (sub = (key >> b3) & (nsub - 1)).  AGG: wave-aggregated LDS claims (lds_claim), for skewed
// keys where whole waves hit one counter (the witness plan's bucket of every value 1).
// The same kernel is pass C of the tiled variant (tiles of sub-bins, b3 = 0, nsub = buckets per
// sub-bin).
template <bool AGG>
__global__ __launch_bounds__(HS_TPB) void k_hs_count2(const uint2* __restrict__ ent,
                                                      const uint32_t* __restrict__ binbase,
                                                      const uint32_t* __restrict__ toff, uint32_t nbins, int b3,
                                                      uint32_t nsub, uint32_t* __restrict__ hist2) {
  __shared__ uint32_t h[1 << HS_MAX_B2];
  HsTile r;
  if (!hs_tile(binbase, toff, nbins, blockIdx.x, r)) return;
  for (uint32_t s = threadIdx.x; s < nsub; s += HS_TPB) h[s] = 0;
  __syncthreads();
  if (AGG) {
    for (uint32_t j0 = r.lo; j0 < r.hi; j0 += HS_TPB) {  // whole waves iterate (lds_claim ballots)
      const uint32_t j = j0 + threadIdx.x;
      const bool ok = j < r.hi;
      (void)lds_claim(h, ok ? (ent[j].x >> b3) & (nsub - 1) : 0u, ok);
    }
  } else {
    for (uint32_t j = r.lo + threadIdx.x; j < r.hi; j += HS_TPB) atomicAdd(&h[(ent[j].x >> b3) & (nsub - 1)], 1u);
  }
  __syncthreads();
  const size_t base = (size_t)toff[r.b] * nsub + r.t;
  for (uint32_t s = threadIdx.x; s < nsub; s += HS_TPB) hist2[base + (size_t)s * r.nt] = h[s];
}

// subbase[b * nsub + s] = first entry of sub-bin s of bin b; subbase[nbins * nsub] = all entries
__global__ __launch_bounds__(HS_TPB) void k_hs_subbase(const uint32_t* __restrict__ off2,
                                                       const uint32_t* __restrict__ binbase,
                                                       const uint32_t* __restrict__ toff, uint32_t nbins,
                                                       uint32_t nsub, uint32_t* __restrict__ subbase) {
  const uint32_t q = blockIdx.x * HS_TPB + threadIdx.x;
  const uint32_t nq = nbins * nsub;
  if (q > nq) return;
  if (q == nq) {
    subbase[q] = binbase[nbins];
    return;
  }
  const uint32_t b = q / nsub, s = q - b * nsub, nt = toff[b + 1] - toff[b];
  subbase[q] = nt ? off2[(size_t)toff[b] * nsub + (size_t)s * nt] : binbase[b];
}

// AGG as in k_hs_count2; VALS: write only the base|sign words (.y) to vout (pass C of the tiled
// variant: the bucket-ordered vals the accumulation reads), else the whole entries to out
template <bool AGG, bool VALS>
__global__ __launch_bounds__(HS_TPB) void k_hs_scatter2(const uint2* __restrict__ ent,
                                                        const uint32_t* __restrict__ binbase,
                                                        const uint32_t* __restrict__ toff, uint32_t nbins, int b3,
                                                        uint32_t nsub, const uint32_t* __restrict__ off2,
                                                        uint2* __restrict__ out, uint32_t* __restrict__ vout) {
  constexpr int NS = 1 << HS_MAX_B2;
  __shared__ uint32_t cnt[NS], off[NS], cur[NS], gbase[NS];
  __shared__ uint2 stage[HS_TILE];
  __shared__ uint32_t sh[HS_TPB / 64];
  HsTile r;
  if (!hs_tile(binbase, toff, nbins, blockIdx.x, r)) return;
  for (uint32_t s = threadIdx.x; s < nsub; s += HS_TPB) cnt[s] = 0;
  __syncthreads();
  constexpr int PT = HS_TILE / HS_TPB;
  uint2 e[PT];
#pragma unroll
  for (int p = 0; p < PT; ++p) {
    const uint32_t j = r.lo + p * HS_TPB + threadIdx.x;
    e[p] = j < r.hi ? ent[j] : make_uint2(0u, 0u);
  }
#pragma unroll
  for (int p = 0; p < PT; ++p) {
    const bool ok = r.lo + p * HS_TPB + threadIdx.x < r.hi;
    if (AGG)
      (void)lds_claim(cnt, (e[p].x >> b3) & (nsub - 1), ok);
    else if (ok)
      atomicAdd(&cnt[(e[p].x >> b3) & (nsub - 1)], 1u);
  }
  __syncthreads();
  const size_t base = (size_t)toff[r.b] * nsub + r.t;
  for (uint32_t s = threadIdx.x; s < nsub; s += HS_TPB) off[s] = cnt[s];
  __syncthreads();
  (void)lds_excl_scan<HS_TPB, NS / HS_TPB>(off, nsub, sh);
  for (uint32_t s = threadIdx.x; s < nsub; s += HS_TPB) {
    cur[s] = off[s];
    gbase[s] = off2[base + (size_t)s * r.nt] - off[s];
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PT; ++p) {
    const bool ok = r.lo + p * HS_TPB + threadIdx.x < r.hi;
    if (AGG) {
      const uint32_t slot = lds_claim(cur, (e[p].x >> b3) & (nsub - 1), ok);
      if (ok) stage[slot] = e[p];
    } else if (ok) {
      stage[atomicAdd(&cur[(e[p].x >> b3) & (nsub - 1)], 1u)] = e[p];
    }
  }
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < r.hi - r.lo; j += HS_TPB) {
    const uint2 x = stage[j];
    if (VALS)
      vout[gbase[(x.x >> b3) & (nsub - 1)] + j] = x.y;
    else
      out[gbase[(x.x >> b3) & (nsub - 1)] + j] = x;
  }
}

// ---------------------------------------------------------------- pass C, tiled variant
// For plans whose sub-bins can hold millions of entries (the compacted witness plan: every
// witness value 1 is a digit of bucket 0; the H plan's deep low buckets) pass C is pass B again
// one level down: every sub-bin cut into tiles of HS_TILE entries, per (sub-bin, bucket, tile)
// counts (k_hs_count2<true>, b3 = 0) whose flat exclusive scan is every run's final position,
// the tiles staged in LDS and written as bucket runs of base|sign words (k_hs_scatter2<true,
// true>), then the bucket bounds and task counts (k_hs_bounds3).  No workgroup takes more than
// HS_TILE entries whatever the skew.
// toff3[q] = tiles of sub-bins < q (toff3[nq] = all); one workgroup
__global__ __launch_bounds__(SC_TPB) void k_hs_subtiles(const uint32_t* __restrict__ subbase, uint32_t nq,
                                                        uint32_t* __restrict__ toff3) {
  __shared__ uint32_t sh[SC_TPB / 64];
  uint32_t carry = 0;
  for (uint32_t j0 = 0; j0 < nq; j0 += SC_TPB) {
    const uint32_t j = j0 + threadIdx.x;
    const uint32_t v = j < nq ? (subbase[j + 1] - subbase[j] + HS_TILE - 1) / HS_TILE : 0u;
    uint32_t tot;
    const uint32_t e = block_excl_scan<SC_TPB>(v, sh, tot);
    if (j < nq) toff3[j] = carry + e;
    carry += tot;
  }
  if (threadIdx.x == 0) toff3[nq] = carry;
}
// bucket k = (q << b3) + f: [start, end) from the scanned (sub-bin, bucket, tile) counts, task
// counts ceil(len / S), cnt[nb] = 0
__global__ __launch_bounds__(HS_TPB) void k_hs_bounds3(const uint32_t* __restrict__ toff3,
                                                       const uint32_t* __restrict__ off3,
                                                       const uint32_t* __restrict__ subbase, int b3, uint32_t nb,
                                                       uint32_t S, uint32_t* __restrict__ start,
                                                       uint32_t* __restrict__ end, uint32_t* __restrict__ cnt) {
  const uint32_t k = blockIdx.x * HS_TPB + threadIdx.x;
  if (k > nb) return;
  if (k == nb) {
    cnt[nb] = 0;
    return;
  }
  const uint32_t nf = 1u << b3, q = k >> b3, f = k & (nf - 1);
  const uint32_t nt = toff3[q + 1] - toff3[q];
  uint32_t s = subbase[q], e = subbase[q];
  if (nt) {
    const size_t base = (size_t)toff3[q] * nf;
    s = off3[base + (size_t)f * nt];
    e = f + 1 < nf ? off3[base + (size_t)(f + 1) * nt] : subbase[q + 1];
  }
  start[k] = s;
  end[k] = e;
  cnt[k] = (e - s + S - 1) / S;
}

// ---------------------------------------------------------------- pass C: sub-bins -> buckets
// one workgroup per sub-bin q (buckets (q << b3) + f): bucket bounds and accumulate-task counts
// ceil(len / S) (cnt[nb] = 0 by the last sub-bin), then the base|sign words in bucket order
__global__ __launch_bounds__(HS_FINE_TPB) void k_hs_fine(const uint2* __restrict__ ent,
                                                         const uint32_t* __restrict__ subbase, uint32_t nq, int b3,
                                                         uint32_t nb, uint32_t S, uint32_t* __restrict__ vout,
                                                         uint32_t* __restrict__ start, uint32_t* __restrict__ end,
                                                         uint32_t* __restrict__ cnt) {
  __shared__ uint32_t h[1 << HS_B3];
  __shared__ uint32_t sorted[HS_CAP];
  const uint32_t q = blockIdx.x, nf = 1u << b3, fmask = nf - 1;
  const uint32_t lo = subbase[q], hi = subbase[q + 1];
  if (threadIdx.x < nf) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t j = lo + threadIdx.x; j < hi; j += HS_FINE_TPB) atomicAdd(&h[ent[j].x & fmask], 1u);
  __syncthreads();
  if (threadIdx.x < 64) {  // one wave scans the <= 64 bucket counters
    const uint32_t f = threadIdx.x;
    const uint32_t len = f < nf ? h[f] : 0u;
    uint32_t x = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (f >= (uint32_t)d) x += y;
    }
    const uint32_t e = x - len;
    const uint32_t bucket = (q << b3) + f;
    if (f < nf && bucket < nb) {
      start[bucket] = lo + e;
      end[bucket] = lo + e + len;
      cnt[bucket] = (len + S - 1) / S;
    }
    if (f < nf) h[f] = e;
  }
  if (q == nq - 1 && threadIdx.x == 0) cnt[nb] = 0;
  __syncthreads();
  const bool in_lds = hi - lo <= (uint32_t)HS_CAP;
  for (uint32_t j = lo + threadIdx.x; j < hi; j += HS_FINE_TPB) {
    const uint2 x = ent[j];
    const uint32_t slot = atomicAdd(&h[x.x & fmask], 1u);
    if (in_lds)
      sorted[slot] = x.y;
    else
      vout[lo + slot] = x.y;
  }
  if (in_lds) {
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < hi - lo; j += HS_FINE_TPB) vout[lo + j] = sorted[j];
  }
}
