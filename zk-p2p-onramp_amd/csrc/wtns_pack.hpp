// Compact witness transfer, host side (DevicePipeline::upload; decoded by qap.hip k_witness_unpack).
// A witness is n signals of 32 B (canonical little-endian Fr values); most signals of a circom
// witness are bits or small counters, so the host sends, per block of WT_BLOCK = 64 signals, the
// bit values (0 / 1) in the block's metadata only, the values >= 2^32 in full (8 words, in lane
// order) and then the low word of every other value (in lane order), padded to 4 words so every
// block starts 16-B aligned.  Blocks are grouped in chunks of WT_CHUNK_BLOCKS (64K signals), each in
// a worst-case-sized region of its own, so chunks are encoded and sent independently.  A chunk
// region holds the metadata of its blocks (WT_META_PER_BLOCK words each: the 64-bit masks of the
// small lanes, of the bit lanes and of the bit values -- lanes past n count as bits of value 0 and are
// never read -- and the block's payload offset) and then, at word WT_META_WORDS, the payload.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

#include <emmintrin.h>

namespace zkp {

constexpr uint32_t WT_BLOCK = 64, WT_CHUNK_BLOCKS = 1024, WT_META_PER_BLOCK = 7;
constexpr size_t WT_META_WORDS = WT_META_PER_BLOCK * WT_CHUNK_BLOCKS;  // 28 KiB: payload stays 16-B aligned
// every region ends in WT_SLACK spare words (never sent): round 4's first encoder wrote one word past
// an all-large block, which for a chunk's last block was the next chunk's metadata, possibly already
// written by another thread; the encoder now stores only inside each block's payload
constexpr size_t WT_SLACK = 4;
constexpr size_t wt_chunk_words() { return WT_META_WORDS + (size_t)WT_CHUNK_BLOCKS * WT_BLOCK * 8 + WT_SLACK; }
inline uint32_t wt_blocks(uint32_t n) { return (n + WT_BLOCK - 1) / WT_BLOCK; }
inline uint32_t wt_chunks(uint32_t n) { return (wt_blocks(n) + WT_CHUNK_BLOCKS - 1) / WT_CHUNK_BLOCKS; }

// encodes chunk c of the n-signal witness at src into its region (wt_chunk_words() words); returns
// the number of leading words of the region to send.  Every store lands inside the block's own
// payload (no stray writes; the slack words are kept as a guard).  n_large (optional): incremented by
// the chunk's count of values >= 2^32 (the prover picks its witness MSM configuration from it).
inline size_t wt_encode_chunk(const uint8_t* src, uint32_t n, uint32_t c, uint32_t* region,
                              uint32_t* n_large = nullptr) {
  const uint32_t nblk = wt_blocks(n);
  const uint32_t b0 = c * WT_CHUNK_BLOCKS, b1 = nblk < b0 + WT_CHUNK_BLOCKS ? nblk : b0 + WT_CHUNK_BLOCKS;
  uint32_t* meta = region;
  uint32_t* pay = region + WT_META_WORDS;
  uint32_t off = 0, nl = 0;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t i0 = b * WT_BLOCK, m = n - i0 < WT_BLOCK ? n - i0 : WT_BLOCK;
    const uint8_t* v = src + (size_t)i0 * 32;
    // the lane classes from 16-B compares (small: words 1..7 zero; bit: small with word 0 <= 1), then
    // the large values and the small low words each walked over the set bits of their lane mask (no
    // per-lane branch on the class: a 0/1-heavy witness mixes them unpredictably) and written with
    // non-temporal stores: the staging is write-once memory read by the DMA engine, so no cache line
    // is read for ownership first
    const __m128i hi3 = _mm_set_epi32(-1, -1, -1, 0), zero = _mm_setzero_si128();
    const uint64_t valid = m < WT_BLOCK ? (1ull << m) - 1 : ~0ull;
    uint64_t smallm = 0, bitm = ~valid, bitv = 0;
    for (uint32_t l = 0; l < m; ++l) {
      const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(v + 32 * l));
      const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(v + 32 * l + 16));
      const __m128i o = _mm_or_si128(_mm_and_si128(a, hi3), c);
      const uint64_t small = (uint64_t)(_mm_movemask_epi8(_mm_cmpeq_epi32(o, zero)) == 0xFFFF);
      const uint32_t w0 = (uint32_t)_mm_cvtsi128_si32(a);
      const uint64_t bit = small & (uint64_t)(w0 <= 1u);
      smallm |= (small & ~bit) << l;
      bitm |= bit << l;
      bitv |= (bit & w0) << l;
    }
    const uint64_t large = ~(smallm | bitm);
    __m128i* out = reinterpret_cast<__m128i*>(pay + off);  // 16-B aligned: offsets are multiples of 4 words
    uint32_t L = 0;
    for (uint64_t bm = large; bm; bm &= bm - 1, ++L) {
      const uint8_t* x = v + 32 * (uint32_t)__builtin_ctzll(bm);
      _mm_stream_si128(out++, _mm_loadu_si128(reinterpret_cast<const __m128i*>(x)));
      _mm_stream_si128(out++, _mm_loadu_si128(reinterpret_cast<const __m128i*>(x + 16)));
    }
    alignas(16) uint32_t lo[WT_BLOCK + 3];
    uint32_t ns = 0;
    for (uint64_t sm = smallm; sm; sm &= sm - 1) std::memcpy(&lo[ns++], v + 32 * (uint32_t)__builtin_ctzll(sm), 4);
    for (uint32_t k = ns; k < ((ns + 3) & ~3u); ++k) lo[k] = 0;
    for (uint32_t k = 0; k < ns; k += 4) _mm_stream_si128(out++, _mm_load_si128(reinterpret_cast<const __m128i*>(lo + k)));
    uint32_t* mb = meta + WT_META_PER_BLOCK * (size_t)(b - b0);
    mb[0] = (uint32_t)smallm;
    mb[1] = (uint32_t)(smallm >> 32);
    mb[2] = (uint32_t)bitm;
    mb[3] = (uint32_t)(bitm >> 32);
    mb[4] = (uint32_t)bitv;
    mb[5] = (uint32_t)(bitv >> 32);
    mb[6] = off;
    off += (8 * L + ns + 3) & ~3u;
    nl += L;
  }
  if (n_large) *n_large += nl;
  _mm_sfence();  // the non-temporal stores are globally visible before the chunk's DMA is enqueued
  return WT_META_WORDS + off;
}

// the decode of signal i (k_witness_unpack's per-thread step) from the chunk regions at stage, for
// host tests
inline void wt_decode_one(const uint32_t* stage, uint32_t i, uint32_t out[8]) {
  const uint32_t g = i / WT_BLOCK, lane = i % WT_BLOCK;
  const uint32_t* region = stage + (size_t)(g / WT_CHUNK_BLOCKS) * wt_chunk_words();
  const uint32_t* mb = region + WT_META_PER_BLOCK * (size_t)(g % WT_CHUNK_BLOCKS);
  const uint64_t smallm = (uint64_t)mb[0] | ((uint64_t)mb[1] << 32), bitm = (uint64_t)mb[2] | ((uint64_t)mb[3] << 32),
                 bitv = (uint64_t)mb[4] | ((uint64_t)mb[5] << 32), large = ~(smallm | bitm);
  const uint64_t below = lane ? ~0ull >> (64 - lane) : 0ull;
  const uint32_t* blk = region + WT_META_WORDS + mb[6];
  std::memset(out, 0, 32);
  if ((bitm >> lane) & 1u)
    out[0] = (uint32_t)(bitv >> lane) & 1u;
  else if ((smallm >> lane) & 1u)
    out[0] = blk[8 * __builtin_popcountll(large) + __builtin_popcountll(smallm & below)];
  else
    std::memcpy(out, blk + 8 * __builtin_popcountll(large & below), 32);
}

}  // namespace zkp
