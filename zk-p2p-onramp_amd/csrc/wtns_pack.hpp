// Compact witness transfer, host side (DevicePipeline::upload; decoded by qap.hip k_witness_unpack).
// A witness is n signals of 32 B (canonical little-endian Fr values); most signals of a circom
// witness are bits or small counters, so the host sends, per block of WT_BLOCK = 64 signals, the
// values >= 2^32 in full (8 words, in lane order) followed by the low word of every other value (in
// lane order), padded to 4 words so every block starts 16-B aligned.  Blocks are grouped in chunks
// of WT_CHUNK_BLOCKS (64K signals), each in a worst-case-sized region of its own, so chunks are
// encoded and sent (one DMA each) independently.  A chunk region holds the meta of its blocks (3 words
// each: the 64-bit small-lane mask, lanes past n counting as small and never read, and the block's
// payload offset) and then, at word WT_META_WORDS, the payload.
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>

#include <emmintrin.h>

namespace zkp {

constexpr uint32_t WT_BLOCK = 64, WT_CHUNK_BLOCKS = 1024;
constexpr size_t WT_META_WORDS = 3 * WT_CHUNK_BLOCKS;  // 12 KiB: payload stays 16-B aligned
// the branch-free small-word copy of a block with no small lane writes one word past the block's
// payload: for the chunk's last block that is the first word after the worst-case payload, so every
// region ends in WT_SLACK spare words (never sent) instead of in the next chunk's metadata, which
// another thread may already have written
constexpr size_t WT_SLACK = 4;
constexpr size_t wt_chunk_words() { return WT_META_WORDS + (size_t)WT_CHUNK_BLOCKS * WT_BLOCK * 8 + WT_SLACK; }
inline uint32_t wt_blocks(uint32_t n) { return (n + WT_BLOCK - 1) / WT_BLOCK; }
inline uint32_t wt_chunks(uint32_t n) { return (wt_blocks(n) + WT_CHUNK_BLOCKS - 1) / WT_CHUNK_BLOCKS; }

// encodes chunk c of the n-signal witness at src into its region (wt_chunk_words() words); returns
// the number of leading words of the region to send.  The stray writes of the branch-free copies
// stay inside the region: a block's large slots end at most 8 words past its payload when it has a
// small lane (payload <= 8 L + 64 - L, so still within the 512 words of an all-large block), its
// small words at most 1 word past it (the last block's: into WT_SLACK).
inline size_t wt_encode_chunk(const uint8_t* src, uint32_t n, uint32_t c, uint32_t* region) {
  const uint32_t nblk = wt_blocks(n);
  const uint32_t b0 = c * WT_CHUNK_BLOCKS, b1 = nblk < b0 + WT_CHUNK_BLOCKS ? nblk : b0 + WT_CHUNK_BLOCKS;
  uint32_t* meta = region;
  uint32_t* pay = region + WT_META_WORDS;
  uint32_t off = 0;
  for (uint32_t b = b0; b < b1; ++b) {
    const uint32_t i0 = b * WT_BLOCK, m = n - i0 < WT_BLOCK ? n - i0 : WT_BLOCK;
    const uint8_t* v = src + (size_t)i0 * 32;
    // branch-free (a 0/1-heavy witness mixes the kinds unpredictably): the small-lane mask from
    // 16-B compares, then the large values to consecutive 32-B slots (each lane writes its slot, a
    // small lane's is overwritten by the next large one or by the small words), then the low words
    const __m128i hi3 = _mm_set_epi32(-1, -1, -1, 0), zero = _mm_setzero_si128();
    uint64_t mask = m < WT_BLOCK ? ~0ull << m : 0ull;
    for (uint32_t l = 0; l < m; ++l) {
      const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(v + 32 * l));
      const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(v + 32 * l + 16));
      const __m128i o = _mm_or_si128(_mm_and_si128(a, hi3), c);
      mask |= (uint64_t)(_mm_movemask_epi8(_mm_cmpeq_epi32(o, zero)) == 0xFFFF) << l;
    }
    const uint32_t L = WT_BLOCK - (uint32_t)__builtin_popcountll(mask);
    uint32_t* big = pay + off;
    for (uint32_t l = 0; l < m; ++l) {
      _mm_storeu_si128(reinterpret_cast<__m128i*>(big), _mm_loadu_si128(reinterpret_cast<const __m128i*>(v + 32 * l)));
      _mm_storeu_si128(reinterpret_cast<__m128i*>(big + 4),
                       _mm_loadu_si128(reinterpret_cast<const __m128i*>(v + 32 * l + 16)));
      big += 8 * (uint32_t)(~(mask >> l) & 1u);
    }
    uint32_t* small = pay + off + 8 * L;
    uint32_t ns = 0;
    for (uint32_t l = 0; l < m; ++l) {
      uint32_t x;
      std::memcpy(&x, v + 32 * l, 4);
      small[ns] = x;
      ns += (uint32_t)(mask >> l) & 1u;
    }
    uint32_t* mb = meta + 3 * (size_t)(b - b0);
    mb[0] = (uint32_t)mask;
    mb[1] = (uint32_t)(mask >> 32);
    mb[2] = off;
    off += (8 * L + ns + 3) & ~3u;
  }
  return WT_META_WORDS + off;
}

// the decode of signal i (k_witness_unpack's per-thread step) from the chunk regions at stage, for
// host tests
inline void wt_decode_one(const uint32_t* stage, uint32_t i, uint32_t out[8]) {
  const uint32_t g = i / WT_BLOCK, lane = i % WT_BLOCK;
  const uint32_t* region = stage + (size_t)(g / WT_CHUNK_BLOCKS) * wt_chunk_words();
  const uint32_t* mb = region + 3 * (size_t)(g % WT_CHUNK_BLOCKS);
  const uint64_t mask = (uint64_t)mb[0] | ((uint64_t)mb[1] << 32);
  const uint64_t below = lane ? mask & (~0ull >> (64 - lane)) : 0ull;
  const uint32_t ns = (uint32_t)__builtin_popcountll(below), nl = lane - ns,
                 L = WT_BLOCK - (uint32_t)__builtin_popcountll(mask);
  const uint32_t* blk = region + WT_META_WORDS + mb[2];
  std::memset(out, 0, 32);
  if ((mask >> lane) & 1u)
    out[0] = blk[8 * L + ns];
  else
    std::memcpy(out, blk + 8 * nl, 32);
}

}  // namespace zkp
