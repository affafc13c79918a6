// Fr NTT engine (see ntt.hpp for the algorithm).
#include "ntt.hpp"

#include <stdexcept>

#include "field.hpp"
#include "hip_check.hpp"
#include "host_ec.hpp"

namespace zkp {

namespace {

constexpr int TPB = 256;  // table kernels
// tile and pass widths measured against 2^11 / 2^12-element tiles (512 / 1024 threads, 7- and 8-bit
// passes): the 2^10 tile is fastest at 2^20 and 2^23 (profiles/ntt_tiles_r04.txt)
constexpr int NTT_TPB = 256;   // threads per pass workgroup (one radix-4 unit per round)
constexpr int LOG_TILE = 10;   // elements per workgroup tile (2^10: 36 KiB of LDS)
constexpr int LOC_LOG = 10;   // local-root table: w_1024^e, e < 512
constexpr int MAX_PASS_BITS = 8;
constexpr int MAX_TW = 1 << (MAX_PASS_BITS - 1);  // stage roots w_(2^b)^j, j < 2^(b-1), b <= 8
// the stage-root products are Shoup products by constants (field.hpp mul_shoup: 143 mads, no per-column
// quotient digits): each root's plain limbs and its quotient floor(w 2^261 / r) are staged in LDS
// (2 x 9 words per root); their outputs are < 3m, so the differences that take them use sub4
constexpr int RW = 2 * NL;  // LDS words per root


__device__ __forceinline__ uint32_t brev(uint32_t x, int b) { return __builtin_bitreverse32(x) >> (32 - b); }

// w_n^E from the two-level table, E < n
__device__ __forceinline__ Fr tw_pow(const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi, uint32_t E,
                                     int h) {
  Fr a = load_fe<FrCfg>(lo + (size_t)(E & ((1u << h) - 1)) * 8);
  Fr b = load_fe<FrCfg>(hi + (size_t)(E >> h) * 8);
  return mul(a, b);
}

// Tile geometry of one pass over blocks of 2^lm elements (2^b rows x n2 = 2^(lm-b)
// columns): a tile holds 2^lbt whole blocks (innermost passes, n2 small) or one block's
// 2^b rows x 2^lc consecutive columns; E = 2^(lbt + b + lc) elements.
struct Tile {
  int lm, b, lc, lbt;
};

// the vectors of one launch (coset_extend_batch: A, B and C of the quotient in one grid): workgroup
// w works on tile w mod 2^lt of vector w >> lt, so a pass over three vectors is one launch of 3x the
// tiles -- 2^20's 1024 tiles per vector over 768 resident workgroups leave a third of a round
// half-idle per launch, 3072 fill four rounds
struct Polys {
  uint32_t* p0;
  uint32_t* p1;
  uint32_t* p2;
  int lt;  // log2 tiles per vector
};

// the stage roots of a b-bit pass, precomputed once per (direction, b) in their LDS layout
// (k_root_table): staging is a copy (no products per root per workgroup)
__device__ __forceinline__ void stage_roots(uint32_t* __restrict__ ltw, const uint32_t* __restrict__ rtab) {
  const uint4* s = reinterpret_cast<const uint4*>(rtab);
  uint4* d = reinterpret_cast<uint4*>(ltw);
  for (int k = threadIdx.x; k < RW * MAX_TW / 4; k += NTT_TPB) d[k] = s[k];
}

// rtab in the LDS layout of stage_roots: ltw[l * MAX_TW + j] = limb l of the plain root w_(2^b)^j,
// ltw[(NL + l) * MAX_TW + j] = limb l of its Shoup quotient, j < 2^(b-1) (the rest zero)
__global__ __launch_bounds__(TPB) void k_root_table(uint32_t* __restrict__ rtab, const uint32_t* __restrict__ loc, int b) {
  const int j = blockIdx.x * TPB + threadIdx.x;
  if (j >= MAX_TW) return;
  Fr w = fe_zero<FrCfg>(), wq = fe_zero<FrCfg>();
  if (j < (1 << (b - 1))) {
    const Fr x = load_fe<FrCfg>(loc + (size_t)(j << (LOC_LOG - b)) * 8);  // canonical Montgomery form
    w = from_mont(x);
    wq = shoup_quot(x);
  }
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    rtab[l * MAX_TW + j] = w.v[l];
    rtab[(NL + l) * MAX_TW + j] = wq.v[l];
  }
}

// LDS data-tile swizzle: element e lives at word e ^ S(e), S(e) = (h ^ 2h ^ 8h) mod 32, h = e >> 5
// (an XOR of bits 5.. into the bank bits 0..4).  ds_read_b32 / ds_write_b32 banks are word mod 32 per
// 32-lane half; unswizzled, the later radix-4 rounds hit 2- and 4-way conflicts and the digit-reversed
// reads of the store phase 8-way ones.  This S makes every access phase of every tile geometry the
// NTT uses (b, lc, lbt for 2^12..2^23) conflict-free (searched by simulating the bank mapping of all
// the phases).  S is linear over GF(2) in the bits of e, so for x whose bits are disjoint from e0's,
// swz(e0 | x) = swz(e0) ^ swz(x): a radix-4 unit swizzles e0 once and XORs wave-uniform row offsets.
__device__ __forceinline__ int swz(int e) {
  const int h = e >> 5;
  return e ^ ((h ^ (h << 1) ^ (h << 3)) & 31);
}

// LDS tile access: lds[limb * E + element].  With a compile-time E (LE > 0: the 1024-element tiles of
// every transform of 2^10 points or more) limb l is a constant byte offset l * 4E of one address
// register (ds_read2st64 pairs), instead of nine address registers and adds per element per round.
template <int LE>
__device__ __forceinline__ Fr lds_get(const uint32_t* __restrict__ lds, int E_rt, int e) {
  const int E = LE ? (1 << LE) : E_rt;
  Fr x;
#pragma unroll
  for (int l = 0; l < NL; ++l) x.v[l] = lds[l * E + e];
  return x;
}
template <int LE>
__device__ __forceinline__ void lds_put(uint32_t* __restrict__ lds, int E_rt, int e, const Fr& x) {
  const int E = LE ? (1 << LE) : E_rt;
#pragma unroll
  for (int l = 0; l < NL; ++l) lds[l * E + e] = x.v[l];
}
// x - y for stage values (Shoup products: < 3m)
__device__ __forceinline__ Fr stage_sub(const Fr& x, const Fr& y) { return sub4(x, y); }
// a * w_ja and c * w_jc as one lockstep pair of Shoup products (field.hpp mul_shoup_pair; with Fr's
// chained columns the two chains fill each other's wait states); outputs < 3m
__device__ __forceinline__ void root_mul_pair(const Fr& a, uint32_t ja, const Fr& c, uint32_t jc,
                                              const uint32_t* __restrict__ ltw, Fr& r, Fr& s) {
  Fr w, wq, v, vq;
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    w.v[l] = ltw[l * MAX_TW + ja];
    wq.v[l] = ltw[(NL + l) * MAX_TW + ja];
    v.v[l] = ltw[l * MAX_TW + jc];
    vq.v[l] = ltw[(NL + l) * MAX_TW + jc];
  }
  mul_shoup_pair(a, w, wq, c, v, vq, r, s);
}
// a * w_j alone (output < 3m)
__device__ __forceinline__ Fr root_mul(const Fr& a, uint32_t j, const uint32_t* __restrict__ ltw) {
  Fr w, wq;
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    w.v[l] = ltw[l * MAX_TW + j];
    wq.v[l] = ltw[(NL + l) * MAX_TW + j];
  }
  return mul_shoup(a, w, wq);
}

// one radix-4 unit (thread work item q) of round t: rows r0 + {0, H/2, H, 3H/2} of stage t
// (span H) and t+1 (span H/2), r0 = grp 2H + i.
// Value bounds (round 5, host-tested: tools/hosttest op r4lazy): every tile value between rounds is
// normalised (limbs < 2^29) and < 3m (Shoup outputs < 3m, qreduce outputs < 1.2m).  The first-stage
// sums stay raw (< 6m, limbs < 2^30); their difference takes the 2^30-raised 6m borrow form without a
// carry pass (sub_raw6n: limbs < 2.5 * 2^30, < 12m), a mul_shoup operand.  RAW: the unit is the last
// one of a DFT whose outputs only feed a Montgomery product (the DIF pass's inter-pass twiddle, the
// coset key between the fused kernel's two DFTs): its four outputs stay unreduced (< 12m, limbs
// < 2.5 * 2^30 -- a mul() operand against the normalised table value), 4 reductions fewer.
template <int LE>
__device__ __forceinline__ void r4_unit(uint32_t* __restrict__ lds, const uint32_t* __restrict__ ltw, int E, int b,
                                        int lc, int t, int q, bool raw) {
  const uint32_t C = 1u << lc;
  const int lhalf = b - 1 - t;
  const uint32_t Hh = 1u << (lhalf - 1);
  const uint32_t col = (uint32_t)q & (C - 1), bq = ((uint32_t)q >> lc) & ((1u << (b - 2)) - 1);
  const uint32_t bl = (uint32_t)q >> (lc + b - 2);
  const uint32_t i = bq & (Hh - 1), grp = bq >> (lhalf - 1);
  const uint32_t r0 = (grp << (lhalf + 1)) | i;
  const int base = (int)(bl << (b + lc)) + (int)col;
  const int st = (int)(Hh << lc);
  // swizzled rows e0 + k st = e0 | k st (disjoint bits): p0 ^ swz(k st)
  const int p0 = swz(base + (int)(r0 << lc)), p1 = p0 ^ swz(st), p2 = p0 ^ swz(2 * st), p3 = p0 ^ swz(3 * st);
  const Fr x0 = lds_get<LE>(lds, E, p0), x1 = lds_get<LE>(lds, E, p1), x2 = lds_get<LE>(lds, E, p2),
           x3 = lds_get<LE>(lds, E, p3);
  // stage t: (x0, x2) with w_(2H)^i, (x1, x3) with w_(2H)^(i + H/2); stage t+1: (s02, s13)
  // and (d02, d13), both with w_H^i.  Roots as exponents of w_(2^b) (stage t: i << t).
  // the unit's independent root products in lockstep pairs (d02 / d13, then y1 / y3 by the same
  // root); inside a round every lane multiplies (w^0 = 1 for i = 0: no divergent j == 0 path).  The
  // last pair of a DFT (Hh == 1, a round-uniform branch; odd b too, dft_stages) has i = 0 for every lane: stage t's
  // first difference takes w^0 = 1 and is only reduced (qreduce: < 1.2m, ~43 instructions instead of
  // half a lockstep Shoup pair)
  const uint32_t j = i << (t + 1);
  Fr d02, d13;
  if (Hh > 1) {
    root_mul_pair(rsub(x0, x2), i << t, rsub(x1, x3), (i + Hh) << t, ltw, d02, d13);
  } else {
    d02 = qreduce(rsub(x0, x2));
    d13 = root_mul(rsub(x1, x3), 1u << t, ltw);
  }
  const Fr s02 = add_raw(x0, x2), s13 = add_raw(x1, x3);  // < 6m, limbs < 2^30
  if (Hh > 1) {
    lds_put<LE>(lds, E, p0, add_raw_reduce(s02, s13));
    Fr y1, y3;
    root_mul_pair(sub_raw6n(s02, s13), j, rsub(d02, d13), j, ltw, y1, y3);
    lds_put<LE>(lds, E, p1, y1);
    lds_put<LE>(lds, E, p3, y3);
    lds_put<LE>(lds, E, p2, add(d02, d13));
  } else if (raw) {  // last pair (span 1, no multiply in stage t+1), outputs into a Montgomery product
    lds_put<LE>(lds, E, p0, add_raw(s02, s13));    // < 12m, limbs < 2^31
    lds_put<LE>(lds, E, p1, sub_raw6n(s02, s13));  // < 12m, limbs < 2.5 * 2^30
    lds_put<LE>(lds, E, p2, add_raw(d02, d13));    // < 6m, limbs < 2^30
    lds_put<LE>(lds, E, p3, rsub(d02, d13));       // < 7m, limbs < 1.5 * 2^30
  } else {  // last pair, outputs stored: one reduction each
    lds_put<LE>(lds, E, p0, add_raw_reduce(s02, s13));
    lds_put<LE>(lds, E, p1, qreduce(sub_raw6n(s02, s13)));
    lds_put<LE>(lds, E, p2, add(d02, d13));
    lds_put<LE>(lds, E, p3, stage_sub(d02, d13));
  }
}

// b radix-2 DIF stages on the LDS tile (rows natural in, bit-reversed out), done two at a
// time as radix-4 groups in registers (half the LDS traffic and barriers of radix-2), an odd b's
// extra stage first.  raw: the outputs feed a Montgomery product only (r4_unit).  Every access
// phase stays bank-conflict-free under swz (simulated for the 2^12..2^23 geometries, both orders)
template <int LE>
__device__ __forceinline__ void dft_stages(uint32_t* __restrict__ lds, const uint32_t* __restrict__ ltw, int E_rt,
                                           int b, int lc, bool raw) {
  const int E = LE ? (1 << LE) : E_rt;
  const uint32_t C = 1u << lc;
  int t = 0;
  if ((b & 1) && b > 1) {
    // odd b: the lone radix-2 stage goes FIRST (span 2^(b-1), roots w_(2^b)^r), so that the radix-4
    // rounds end on a span-2/span-1 pair whose stage-t root is w^0 (r4_unit, Hh == 1): 0.25 products
    // per element fewer than a radix-4 run ending on the root-free span-1 stage.  Two pairs per
    // thread in lockstep; outputs < 1.2m (qreduce) and < 3m (Shoup), normalised
    const uint32_t half = 1u << (b - 1);
    const int stp = swz((int)(half << lc));
    auto pos = [&](int q, uint32_t& r) {
      const uint32_t col = (uint32_t)q & (C - 1);
      r = ((uint32_t)q >> lc) & (half - 1);
      const uint32_t bl = (uint32_t)q >> (lc + b - 1);
      return swz((int)(bl << (b + lc)) + (int)(r << lc) + (int)col);
    };
    for (int q = threadIdx.x; q < (E >> 1); q += 2 * NTT_TPB) {
      uint32_t ra, rc;
      const int a0 = pos(q, ra), a1 = a0 ^ stp;
      const Fr x0 = lds_get<LE>(lds, E, a0), x1 = lds_get<LE>(lds, E, a1);
      if (q + NTT_TPB < (E >> 1)) {
        const int c0 = pos(q + NTT_TPB, rc), c1 = c0 ^ stp;
        const Fr y0 = lds_get<LE>(lds, E, c0), y1 = lds_get<LE>(lds, E, c1);
        Fr u, v;
        root_mul_pair(rsub(x0, x1), ra, rsub(y0, y1), rc, ltw, u, v);
        lds_put<LE>(lds, E, a0, add(x0, x1));
        lds_put<LE>(lds, E, a1, u);
        lds_put<LE>(lds, E, c0, add(y0, y1));
        lds_put<LE>(lds, E, c1, v);
      } else {
        lds_put<LE>(lds, E, a1, root_mul(rsub(x0, x1), ra, ltw));
        lds_put<LE>(lds, E, a0, add(x0, x1));
      }
    }
    __syncthreads();
    t = 1;
  }
  for (; t + 1 < b; t += 2) {
    for (int q = threadIdx.x; q < (E >> 2); q += NTT_TPB) r4_unit<LE>(lds, ltw, E, b, lc, t, q, raw);
    __syncthreads();
  }
  if (t < b) {  // b == 1: the one radix-2 stage (span 1)
    for (int q = threadIdx.x; q < (E >> 1); q += NTT_TPB) {
      const uint32_t col = (uint32_t)q & (C - 1), bq = ((uint32_t)q >> lc) & ((1u << (b - 1)) - 1);
      const uint32_t bl = (uint32_t)q >> (lc + b - 1);
      const int p0 = swz((int)(bl << (b + lc)) + (int)((bq << 1) << lc) + (int)col), p1 = p0 ^ swz((int)C);
      const Fr x = lds_get<LE>(lds, E, p0), y = lds_get<LE>(lds, E, p1);
      if (raw) {  // < 6m and < 7m, into a Montgomery product
        lds_put<LE>(lds, E, p0, add_raw(x, y));
        lds_put<LE>(lds, E, p1, rsub(x, y));
      } else {
        lds_put<LE>(lds, E, p0, add(x, y));
        lds_put<LE>(lds, E, p1, stage_sub(x, y));  // span 1: the root is w_2^0 = 1
      }
    }
    __syncthreads();
  }
}

// element e of tile `tile` -> global index g and position in its block
__device__ __forceinline__ void tile_coords(const Tile& T, uint32_t tile, int e, size_t& g, uint32_t& pos) {
  const uint32_t C = 1u << T.lc, n2 = 1u << (T.lm - T.b);
  const uint32_t col = (uint32_t)e & (C - 1);
  const uint32_t row = ((uint32_t)e >> T.lc) & ((1u << T.b) - 1);
  const uint32_t bl = (uint32_t)e >> (T.lc + T.b);
  size_t block;
  uint32_t col0;
  if (T.lbt > 0) {
    block = ((size_t)tile << T.lbt) + bl;
    col0 = 0;
  } else {
    const uint32_t tpb = n2 >> T.lc;
    block = tile / tpb;
    col0 = (tile - (uint32_t)block * tpb) << T.lc;
  }
  pos = row * n2 + col0 + col;
  g = (block << T.lm) + pos;
}

// LDS index holding output row k1 of element e's (block, column) after dft_stages
__device__ __forceinline__ int brev_src(const Tile& T, int e) {
  const int mask = ((1 << T.b) - 1) << T.lc;
  const uint32_t k1 = ((uint32_t)e >> T.lc) & ((1u << T.b) - 1);
  return (e & ~mask) | (int)(brev(k1, T.b) << T.lc);
}

// Addresses of element e = threadIdx.x + it * NTT_TPB of a full tile.  tile_coords (global index,
// position in its block), the LDS slot swz(e) and the digit-reversed slot swz(brev_src(e)) are all
// linear in e's bit-fields (disjoint bits add, resp. XOR), so each is the part of threadIdx.x --
// computed once per thread (lane_base) -- plus the part of it * NTT_TPB, the same for every lane
// (scalar registers; lane_at): ~2 vector instructions per element and phase instead of ~15 (round 5)
struct Lane {
  size_t g;
  uint32_t pos;
  int sw, sb;  // swz(e), swz(brev_src(e))
};
__device__ __forceinline__ Lane lane_base(const Tile& T, uint32_t tile) {
  Lane L;
  tile_coords(T, tile, (int)threadIdx.x, L.g, L.pos);
  L.sw = swz((int)threadIdx.x);
  L.sb = swz(brev_src(T, (int)threadIdx.x));
  return L;
}
__device__ __forceinline__ Lane lane_at(const Lane& L, const Tile& T, uint32_t tile, int it) {
  size_t gz, gh;
  uint32_t pz, ph;
  tile_coords(T, tile, 0, gz, pz);
  tile_coords(T, tile, it * NTT_TPB, gh, ph);
  Lane r;
  r.g = L.g + (gh - gz);
  r.pos = L.pos + (ph - pz);
  r.sw = L.sw ^ swz(it * NTT_TPB);
  r.sb = L.sb ^ swz(brev_src(T, it * NTT_TPB));
  return r;
}

// MODE 0: DIF pass (DFT, then inter-pass twiddle), 1: DIT pass (twiddle, then DFT),
// 2: the fused innermost pair of coset_extend (lm == b): inverse-root DFT, coset key
//    (table by digit-reversed position), forward-root DFT on one LDS-resident tile.
// tw: w_(2^lm)^(col*row) by position in block (null when n2 == 1).  rootsA / rootsB: the stage
// roots (the k_root_table of this b and direction), B for MODE 2's forward DFT.
template <int MODE, int LE>
__global__ __launch_bounds__(NTT_TPB) void k_ntt(Polys P, Tile T, const uint32_t* __restrict__ tw,
                                             const uint32_t* __restrict__ rootsA, const uint32_t* __restrict__ rootsB,
                                             const uint32_t* __restrict__ coset) {
  __shared__ uint32_t lds[NL << LOG_TILE];  // SoA: lds[limb * E + element]
  __shared__ __attribute__((aligned(16))) uint32_t ltw[RW * MAX_TW];
  const int E = LE ? (1 << LE) : (1 << (T.b + T.lc + T.lbt));  // LE: the tile size known at compile time
  const uint32_t vec = blockIdx.x >> P.lt, tile = blockIdx.x & ((1u << P.lt) - 1);
  uint32_t* __restrict__ data = vec == 0 ? P.p0 : (vec == 1 ? P.p1 : P.p2);
  stage_roots(ltw, rootsA);
  constexpr int VPT = (1 << LOG_TILE) / NTT_TPB;  // elements per thread of a full tile
  Lane L0{};
  if (LE) L0 = lane_base(T, tile);
  if (LE && MODE == 1 && tw) {
    // full tiles: the twiddle products of two elements at a time in lockstep (mul_pair)
#pragma unroll
    for (int it = 0; it < VPT; it += 2) {
      const Lane a = lane_at(L0, T, tile, it), c = lane_at(L0, T, tile, it + 1);
      Fr x0, x1;
      mul_pair(load_fe<FrCfg>(data + a.g * 8), load_fe<FrCfg>(tw + (size_t)a.pos * 8), load_fe<FrCfg>(data + c.g * 8),
               load_fe<FrCfg>(tw + (size_t)c.pos * 8), x0, x1);
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        lds[l * E + a.sw] = x0.v[l];
        lds[l * E + c.sw] = x1.v[l];
      }
    }
  } else if (LE) {
#pragma unroll
    for (int it = 0; it < VPT; ++it) {
      const Lane a = lane_at(L0, T, tile, it);
      const Fr x = load_fe<FrCfg>(data + a.g * 8);
#pragma unroll
      for (int l = 0; l < NL; ++l) lds[l * E + a.sw] = x.v[l];
    }
  } else {
    for (int e = threadIdx.x; e < E; e += NTT_TPB) {
      size_t g;
      uint32_t pos;
      tile_coords(T, tile, e, g, pos);
      Fr x = load_fe<FrCfg>(data + g * 8);
      if (MODE == 1 && tw) x = mul(x, load_fe<FrCfg>(tw + (size_t)pos * 8));
#pragma unroll
      for (int l = 0; l < NL; ++l) lds[l * E + swz(e)] = x.v[l];
    }
  }
  __syncthreads();
  // raw last round: MODE 0's outputs meet the inter-pass twiddle, MODE 2's first DFT the coset key
  dft_stages<LE>(lds, ltw, E, T.b, T.lc, MODE == 2 || (MODE == 0 && tw != nullptr));
  if (MODE == 2) {
    // output row k1 (natural position in the block) sits at LDS row brev(k1): key it with
    // g^f(pos)/n and put it back at row k1 as the forward DFT's input
    // (a fixed trip count keeps v[] in registers: a runtime-indexed array went to scratch; full
    // tiles key two elements at a time in lockstep)
    Fr v[VPT];
    if (LE) {
#pragma unroll
      for (int it = 0; it < VPT; it += 2) {
        const Lane a = lane_at(L0, T, tile, it), c = lane_at(L0, T, tile, it + 1);
        Fr x0, x1;
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          x0.v[l] = lds[l * E + a.sb];
          x1.v[l] = lds[l * E + c.sb];
        }
        mul_pair(x0, load_fe<FrCfg>(coset + a.g * 8), x1, load_fe<FrCfg>(coset + c.g * 8), v[it], v[it + 1]);
      }
    } else {
#pragma unroll
      for (int it = 0; it < VPT; ++it) {
        const int e = (int)threadIdx.x + it * NTT_TPB;
        if (e < E) {
          const int src = swz(brev_src(T, e));
          Fr x;
#pragma unroll
          for (int l = 0; l < NL; ++l) x.v[l] = lds[l * E + src];
          size_t g;
          uint32_t pos;
          tile_coords(T, tile, e, g, pos);
          v[it] = mul(x, load_fe<FrCfg>(coset + g * 8));
        }
      }
    }
    __syncthreads();
    stage_roots(ltw, rootsB);  // the forward roots replace the inverse ones (no reader until the next barrier)
#pragma unroll
    for (int it = 0; it < VPT; ++it) {
      const int e = (int)threadIdx.x + it * NTT_TPB;
      if (e < E) {
        const int sw = LE ? lane_at(L0, T, tile, it).sw : swz(e);
#pragma unroll
        for (int l = 0; l < NL; ++l) lds[l * E + sw] = v[it].v[l];
      }
    }
    __syncthreads();
    dft_stages<LE>(lds, ltw, E, T.b, T.lc, false);
  }
  if (LE && MODE == 0 && tw) {
#pragma unroll
    for (int it = 0; it < VPT; it += 2) {
      const Lane a = lane_at(L0, T, tile, it), c = lane_at(L0, T, tile, it + 1);
      Fr x0, x1;
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        x0.v[l] = lds[l * E + a.sb];
        x1.v[l] = lds[l * E + c.sb];
      }
      Fr y0, y1;
      mul_pair(x0, load_fe<FrCfg>(tw + (size_t)a.pos * 8), x1, load_fe<FrCfg>(tw + (size_t)c.pos * 8), y0, y1);
      store_fe(data + a.g * 8, y0);
      store_fe(data + c.g * 8, y1);
    }
  } else if (LE) {
#pragma unroll
    for (int it = 0; it < VPT; ++it) {
      const Lane a = lane_at(L0, T, tile, it);
      Fr x;
#pragma unroll
      for (int l = 0; l < NL; ++l) x.v[l] = lds[l * E + a.sb];
      if (MODE == 0 && tw) x = mul(x, load_fe<FrCfg>(tw + (size_t)a.pos * 8));
      store_fe(data + a.g * 8, x);
    }
  } else {
    for (int e = threadIdx.x; e < E; e += NTT_TPB) {
      const int src = swz(brev_src(T, e));
      Fr x;
#pragma unroll
      for (int l = 0; l < NL; ++l) x.v[l] = lds[l * E + src];
      size_t g;
      uint32_t pos;
      tile_coords(T, tile, e, g, pos);
      if (MODE == 0 && tw) x = mul(x, load_fe<FrCfg>(tw + (size_t)pos * 8));
      store_fe(data + g * 8, x);
    }
  }
}

// tw[pos] = w_(2^lm)^(col * row), pos = row * n2 + col, from the two-level w_n tables
__global__ __launch_bounds__(TPB) void k_pass_table(uint32_t* __restrict__ out, int k, int lm, int b,
                                                    const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi,
                                                    int h) {
  const size_t pos = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (pos >= (size_t(1) << lm)) return;
  const uint32_t n2 = 1u << (lm - b);
  const uint32_t row = (uint32_t)(pos >> (lm - b)), col = (uint32_t)pos & (n2 - 1);
  const uint32_t ex = (uint32_t)(((uint64_t)row * col) << (k - lm)) & (uint32_t)((uint64_t(1) << k) - 1);
  store_fe(out + pos * 8, tw_pow(lo, hi, ex, h));
}

struct PassBits {
  int n;
  int b[8];
};

// digit-reversed position -> frequency index
__device__ __forceinline__ uint32_t freq_of(uint32_t pos, int k, const PassBits& pb) {
  uint32_t f = 0;
  int consumed = 0, shift = 0;
  for (int i = 0; i < pb.n; ++i) {
    const int b = pb.b[i];
    const uint32_t d = (pos >> (k - consumed - b)) & ((1u << b) - 1);
    f |= d << shift;
    shift += b;
    consumed += b;
  }
  return f;
}

// coset key table: out[pos] = g^f(pos) / n
__global__ __launch_bounds__(TPB) void k_coset_table(uint32_t* __restrict__ out, int k, PassBits pb,
                                                     const uint32_t* __restrict__ c_lo,
                                                     const uint32_t* __restrict__ c_hi, int h) {
  const uint32_t pos = blockIdx.x * TPB + threadIdx.x;
  if (pos >= (1u << k)) return;
  store_fe(out + (size_t)pos * 8, tw_pow(c_lo, c_hi, freq_of(pos, k, pb), h));
}

// x / n (inverse transform of the tests)
__global__ __launch_bounds__(TPB) void k_scale(uint32_t* __restrict__ data, int k, const uint32_t* __restrict__ ninv) {
  const uint32_t pos = blockIdx.x * TPB + threadIdx.x;
  if (pos >= (1u << k)) return;
  store_fe(data + (size_t)pos * 8, mul(load_fe<FrCfg>(data + (size_t)pos * 8), load_fe<FrCfg>(ninv)));
}

__global__ __launch_bounds__(TPB) void k_digit_reverse(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       int k, PassBits pb, int to_natural) {
  const uint32_t pos = blockIdx.x * TPB + threadIdx.x;
  if (pos >= (1u << k)) return;
  const uint32_t f = freq_of(pos, k, pb);
  const uint32_t src = to_natural ? pos : f, dst = to_natural ? f : pos;
  const uint4* s = reinterpret_cast<const uint4*>(in + (size_t)src * 8);
  uint4* d = reinterpret_cast<uint4*>(out + (size_t)dst * 8);
  d[0] = s[0];
  d[1] = s[1];
}

// ---------------- host helpers: table generation
using HFr = host::Fr;

host::U256 words8_to_u256(const uint32_t* w) {
  host::U256 r;
  for (int i = 0; i < 4; ++i) r.w[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  return r;
}

// value x (host Fr) -> device layout words: the standard integer x * 2^261 mod r
void fr_to_dev_words(const HFr& x, uint32_t* out) {
  static const HFr two261 =
      HFr::from_std(host::U256{{0, 0, 0, uint64_t(1) << 58}}) * HFr::from_std(host::U256{{uint64_t(1) << 11, 0, 0, 0}});
  host::U256 raw = (x * two261).to_std();
  for (int i = 0; i < 4; ++i) {
    out[2 * i] = (uint32_t)raw.w[i];
    out[2 * i + 1] = (uint32_t)(raw.w[i] >> 32);
  }
}

HFr fr_pow(const HFr& b, uint64_t e) {
  HFr r = HFr::one(), x = b;
  while (e) {
    if (e & 1) r = r * x;
    x = x.sqr();
    e >>= 1;
  }
  return r;
}

uint32_t* upload_powers(const HFr& base, size_t count, uint64_t step_pow, const HFr& mulk, hipStream_t st) {
  // entries: mulk * base^(i*step_pow)
  std::vector<uint32_t> h(count * 8);
  HFr step = fr_pow(base, step_pow);
  HFr cur = mulk;
  for (size_t i = 0; i < count; ++i) {
    fr_to_dev_words(cur, h.data() + i * 8);
    cur = cur * step;
  }
  uint32_t* d = nullptr;
  HIPX(hipMalloc(&d, h.size() * 4));
  HIPX(hipMemcpyAsync(d, h.data(), h.size() * 4, hipMemcpyHostToDevice, st));
  HIPX(hipStreamSynchronize(st));
  return d;
}

HFr root_of_unity(int lg) {  // Fr.w[lg]
  return HFr::from_std(words8_to_u256(FR_ROOTS_W[lg]));
}

PassBits make_pb(const std::vector<int>& bits) {
  PassBits pb{};
  pb.n = (int)bits.size();
  for (int i = 0; i < pb.n; ++i) pb.b[i] = bits[i];
  return pb;
}

Tile make_tile(int k, int lm, int b) {
  Tile T;
  T.lm = lm;
  T.b = b;
  const int le = std::min(LOG_TILE, k);      // tile elements (log)
  T.lc = std::min(le - b, lm - b);           // columns of one block in the tile
  T.lbt = le - b - T.lc;                     // whole blocks per tile (innermost passes)
  return T;
}

}  // namespace

NttEngine::NttEngine(int log_n, hipStream_t stream) : log_n_(log_n), stream_(stream) {
  if (log_n < 0 || log_n > 27) throw std::runtime_error("NTT size out of range");
  const int k = log_n;
  if (k > 0) {
    const int p = (k + MAX_PASS_BITS - 1) / MAX_PASS_BITS;
    int rem = k;
    for (int i = 0; i < p; ++i) {
      const int b = (rem + (p - i) - 1) / (p - i);
      bits_.push_back(b);
      lms_.push_back(rem);
      rem -= b;
    }
  }
  h_ = (k + 1) / 2;
  const HFr one = HFr::one();
  const HFr w = root_of_unity(k);
  const HFr wi = w.inv();
  const size_t nlo = size_t(1) << h_, nhi = size_t(1) << (k - h_);
  tw_lo_[0] = upload_powers(w, nlo, 1, one, stream_);
  tw_hi_[0] = upload_powers(w, nhi, nlo, one, stream_);
  tw_lo_[1] = upload_powers(wi, nlo, 1, one, stream_);
  tw_hi_[1] = upload_powers(wi, nhi, nlo, one, stream_);
  const HFr w1024 = root_of_unity(LOC_LOG);
  loc_[0] = upload_powers(w1024, size_t(1) << (LOC_LOG - 1), 1, one, stream_);
  loc_[1] = upload_powers(w1024.inv(), size_t(1) << (LOC_LOG - 1), 1, one, stream_);
  // coset key g = Fr.w[k+1] (Fr.shift when k == 28; not reachable: k <= 27)
  const HFr g = root_of_unity(k + 1);
  host::U256 nstd{{uint64_t(1) << k, 0, 0, 0}};
  const HFr ninv = HFr::from_std(nstd).inv();
  coset_lo_ = upload_powers(g, nlo, 1, ninv, stream_);
  coset_hi_ = upload_powers(g, nhi, nlo, one, stream_);
  ninv_ = upload_powers(one, 1, 1, ninv, stream_);
  // stage-root tables per (direction, pass bits) in the kernels' LDS layout (k_root_table)
  for (int dir = 0; dir < 2; ++dir)
    for (int b : bits_)
      if (!rtab_[dir][b]) {
        HIPX(hipMalloc(&rtab_[dir][b], (size_t)RW * MAX_TW * 4));
        hipLaunchKernelGGL(k_root_table, dim3((MAX_TW + TPB - 1) / TPB), dim3(TPB), 0, stream_, rtab_[dir][b],
                           loc_[dir], b);
      }
  // per-pass twiddle tables (one multiply per element instead of lo*hi per element) and
  // the coset key by digit-reversed position: ~3 n x 32 B of HBM
  for (int dir = 0; dir < 2; ++dir) {
    tw_pass_[dir].assign(bits_.size(), nullptr);
    for (size_t p = 0; p < bits_.size(); ++p) {
      const int lm = lms_[p], b = bits_[p];
      if (lm == b) continue;  // innermost pass: n2 = 1, no twiddle
      const size_t cnt = size_t(1) << lm;
      HIPX(hipMalloc(&tw_pass_[dir][p], cnt * 32));
      table_bytes_ += cnt * 32;
      hipLaunchKernelGGL(k_pass_table, dim3((unsigned)((cnt + TPB - 1) / TPB)), dim3(TPB), 0, stream_,
                         tw_pass_[dir][p], k, lm, b, tw_lo_[dir], tw_hi_[dir], h_);
    }
  }
  if (k > 0) {
    const size_t n = size_t(1) << k;
    HIPX(hipMalloc(&coset_pos_, n * 32));
    table_bytes_ += n * 32;
    hipLaunchKernelGGL(k_coset_table, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, stream_, coset_pos_, k,
                       make_pb(bits_), coset_lo_, coset_hi_, h_);
  }
  HIPX(hipGetLastError());
  HIPX(hipStreamSynchronize(stream_));
}

NttEngine::~NttEngine() {
  for (uint32_t* p : {tw_lo_[0], tw_lo_[1], tw_hi_[0], tw_hi_[1], loc_[0], loc_[1], coset_lo_, coset_hi_, ninv_,
                      scratch_, coset_pos_})
    if (p) (void)hipFree(p);
  for (auto& v : tw_pass_)
    for (uint32_t* p : v)
      if (p) (void)hipFree(p);
  for (auto& d : rtab_)
    for (uint32_t* p : d)
      if (p) (void)hipFree(p);
}

// mode 0: DIF pass p, 1: DIT (transposed) pass p, 2: fused innermost pass (inverse then forward);
// over count (1..3) vectors in one grid
void NttEngine::launch_pass(uint32_t* const* data, int count, int mode, int p, bool inv) {
  const int k = log_n_;
  const Tile T = make_tile(k, lms_[p], bits_[p]);
  const int lt = k - (T.b + T.lc + T.lbt);
  const size_t tiles = (size_t)count << lt;
  const Polys P{data[0], count > 1 ? data[1] : data[0], count > 2 ? data[2] : data[0], lt};
  const int d = inv ? 1 : 0;
  const uint32_t *ra = rtab_[d][T.b], *rinv = rtab_[1][T.b], *rfwd = rtab_[0][T.b];
  const uint32_t* none = nullptr;
  // full 1024-element tiles (every transform of 2^10 points or more) take the compile-time tile size
  const bool full = T.b + T.lc + T.lbt == LOG_TILE;
  auto k0 = full ? k_ntt<0, LOG_TILE> : k_ntt<0, 0>;
  auto k1 = full ? k_ntt<1, LOG_TILE> : k_ntt<1, 0>;
  auto k2 = full ? k_ntt<2, LOG_TILE> : k_ntt<2, 0>;
  if (mode == 0)
    hipLaunchKernelGGL(k0, dim3((unsigned)tiles), dim3(NTT_TPB), 0, stream_, P, T, tw_pass_[d][p], ra, none, none);
  else if (mode == 1)
    hipLaunchKernelGGL(k1, dim3((unsigned)tiles), dim3(NTT_TPB), 0, stream_, P, T, tw_pass_[d][p], ra, none, none);
  else
    hipLaunchKernelGGL(k2, dim3((unsigned)tiles), dim3(NTT_TPB), 0, stream_, P, T, none, rinv, rfwd, coset_pos_);
}

void NttEngine::dif_passes(uint32_t* const* data, int count, bool inv, int first, int last) {
  for (int p = first; p < last; ++p) launch_pass(data, count, 0, p, inv);
}

void NttEngine::dit_passes(uint32_t* const* data, int count, bool inv, int first, int last) {
  // transposed passes in reverse order: block sizes grow back from the innermost
  for (int p = last - 1; p >= first; --p) launch_pass(data, count, 1, p, inv);
}

void NttEngine::scale(uint32_t* data, int mode) {
  (void)mode;
  const size_t n = size_t(1) << log_n_;
  hipLaunchKernelGGL(k_scale, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, stream_, data, log_n_, ninv_);
}

void NttEngine::digit_reverse(uint32_t* data, bool to_natural) {
  const size_t n = size_t(1) << log_n_;
  if (!scratch_) HIPX(hipMalloc(&scratch_, n * 32));
  HIPX(hipMemcpyAsync(scratch_, data, n * 32, hipMemcpyDeviceToDevice, stream_));
  hipLaunchKernelGGL(k_digit_reverse, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, stream_, scratch_, data,
                     log_n_, make_pb(bits_), to_natural ? 1 : 0);
}

void NttEngine::coset_extend_batch(uint32_t* const* data, int count) {
  if (count < 1 || count > 3) throw std::invalid_argument("coset_extend_batch: 1..3 vectors");
  if (log_n_ == 0) {
    // n = 1: coefficient = value; evaluation at g is the same constant
    return;
  }
  const int P = (int)bits_.size();
  dif_passes(data, count, true, 0, P - 1);  // inverse, outer passes
  launch_pass(data, count, 2, P - 1, true);  // innermost inverse pass + coset key + innermost forward pass
  dit_passes(data, count, false, 0, P - 1);  // forward, outer passes (transposed, reverse order)
  HIPX(hipGetLastError());
}

void NttEngine::coset_extend(uint32_t* data) { coset_extend_batch(&data, 1); }

void NttEngine::forward(uint32_t* data) {
  if (log_n_ == 0) return;
  dif_passes(&data, 1, false, 0, (int)bits_.size());
  digit_reverse(data, true);
  HIPX(hipGetLastError());
}

void NttEngine::inverse(uint32_t* data) {
  if (log_n_ == 0) return;
  dif_passes(&data, 1, true, 0, (int)bits_.size());
  scale(data, 1);
  digit_reverse(data, true);
  HIPX(hipGetLastError());
}

}  // namespace zkp
