// Host check + timing of the compact witness encoding (csrc/wtns_pack.hpp): encodes witnesses of
// several value mixes chunk by chunk, decodes every signal as k_witness_unpack does (wt_decode_one)
// and compares with the input; then times the encoder over a Venmo-sized witness with T threads.
// usage: wtns_pack_test [n] [threads]   (prints "ok" lines and one timing line per mix)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../../zk-p2p-onramp_amd/csrc/wtns_pack.hpp"

using namespace zkp;

static void fill(std::vector<uint32_t>& v, uint32_t n, int mix, uint64_t seed) {
  std::mt19937_64 g(seed);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t* x = &v[(size_t)i * 8];
    for (int k = 0; k < 8; ++k) x[k] = 0;
    const uint64_t r = g();
    bool large;
    switch (mix) {
      case 0: large = true; break;               // all uniform
      case 1: large = false; break;              // all small
      case 2: large = (r % 10) >= 7; break;      // 70 % small
      default: large = (i % 6) == 2 || (i % 6) == 3 || ((i / 64) % 7 == 3);  // lane patterns + whole blocks
    }
    if (large) {
      for (int k = 0; k < 8; ++k) x[k] = (uint32_t)g();
      x[7] &= 0x1FFFFFFF;
      if (mix == 3 && i % 6 == 2) x[0] = 0, x[1] = 1, x[2] = x[3] = x[4] = x[5] = x[6] = x[7] = 0;  // 2^32
      if (mix == 3 && i % 6 == 3) x[1] = x[2] = x[3] = x[4] = x[5] = x[6] = 0, x[7] = 0x10000000;  // top word only
    } else {
      x[0] = mix == 3 && i % 6 == 1 ? 0xFFFFFFFFu : (uint32_t)(r >> 3) & ((i & 1) ? 1u : 0xFFFFFFFFu);
    }
  }
}

int main(int argc, char** argv) {
  const uint32_t nbig = argc > 1 ? (uint32_t)atoi(argv[1]) : 6400000;
  const int T = argc > 2 ? atoi(argv[2]) : 4;
  int bad = 0;
  std::mt19937_64 sizes(12345);
  std::vector<uint32_t> ns = {1u, 63u, 64u, 65u, 65536u, 65536u * 2 - 1, 3u * 65536 + 37, 4u * 65536};
  for (int r = 0; r < 4; ++r) ns.push_back(1 + (uint32_t)(sizes() % (5u * 65536)));
  for (uint32_t n : ns) {
    for (int mix = 0; mix < 4; ++mix) {
      std::vector<uint32_t> v((size_t)n * 8), stage((size_t)wt_chunks(n) * wt_chunk_words(), 0xDEADBEEFu);
      fill(v, n, mix, n * 7 + mix);
      // chunks in DESCENDING (mixes 0, 2) or shuffled (mixes 1, 3) order: a stray write past a chunk's
      // region would land in a chunk already encoded (the device path encodes chunks on 16 threads in
      // any order)
      std::vector<uint32_t> order(wt_chunks(n));
      for (uint32_t c = 0; c < order.size(); ++c) order[c] = (uint32_t)order.size() - 1 - c;
      if (mix & 1) std::shuffle(order.begin(), order.end(), sizes);
      for (uint32_t c : order) {
        const size_t w = wt_encode_chunk(reinterpret_cast<const uint8_t*>(v.data()), n, c,
                                         stage.data() + (size_t)c * wt_chunk_words());
        if (w > wt_chunk_words() || (w - WT_META_WORDS) % 4) ++bad, printf("chunk size %zu\n", w);
      }
      for (uint32_t i = 0; i < n; ++i) {
        uint32_t o[8];
        wt_decode_one(stage.data(), i, o);
        for (int k = 0; k < 8; ++k)
          if (o[k] != v[(size_t)i * 8 + k]) {
            if (bad++ < 5) printf("mismatch n %u mix %d signal %u word %d\n", n, mix, i, k);
          }
      }
    }
  }
  printf(bad ? "FAIL %d\n" : "ok roundtrip\n", bad);
  const char* names[] = {"uniform", "small", "70pct-small", "patterns"};
  for (int mix : {0, 2}) {
    const uint32_t n = nbig;
    std::vector<uint32_t> v((size_t)n * 8), stage((size_t)wt_chunks(n) * wt_chunk_words());
    fill(v, n, mix, 99);
    double best = 1e9;
    size_t total = 0;
    for (int rep = 0; rep < 5; ++rep) {
      std::vector<size_t> words(wt_chunks(n));
      auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> th;
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          for (uint32_t c = t; c < wt_chunks(n); c += T)
            words[c] = wt_encode_chunk(reinterpret_cast<const uint8_t*>(v.data()), n, c,
                                       stage.data() + (size_t)c * wt_chunk_words());
        });
      for (auto& x : th) x.join();
      best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      total = 0;
      for (size_t w : words) total += w * 4;
    }
    printf("encode %s n %u threads %d: %.2f ms (%.1f GB/s of witness), %.1f MB to send (%.3f of 32 B/signal)\n",
           names[mix], n, T, best, n * 32.0 / best / 1e6, total / 1e6, total / (n * 32.0));
  }
  return bad ? 1 : 0;
}
