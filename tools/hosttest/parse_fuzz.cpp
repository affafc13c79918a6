// Host parser robustness under AddressSanitizer + UndefinedBehaviorSanitizer (the
// zkey / wtns readers take untrusted files).  Built by tests/test_parser_sanitized.py:
//   hipcc -O1 -g -Xarch_host -fsanitize=address,undefined -Xarch_host -fno-sanitize-recover=all
//         parse_fuzz.cpp zkey_parse.cpp host_ec.cpp zkey_io.cpp -lz   (host code only)
// usage: parse_fuzz <file.zkey> <file.wtns> <seed> <mutations>
// Every input -- the files, every truncation on a grid, seeded byte flips, section-length fields
// overwritten with huge / off-by-one values, garbage behind a gzip magic -- must either parse or
// throw ZkpError; a sanitizer report or any other exception fails (non-zero exit).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>

#include "../../zk-p2p-onramp_amd/csrc/prover.hpp"
#include "../../zk-p2p-onramp_amd/csrc/zkey_io.hpp"

using namespace zkp;

static std::vector<uint8_t> slurp(const char* p) {
  std::ifstream f(p, std::ios::binary);
  return std::vector<uint8_t>(std::istreambuf_iterator<char>(f), {});
}

static long ok = 0, rejected = 0;

template <class F>
static void run(const std::vector<uint8_t>& b, F&& parse) {
  // an exact-size heap copy: any read past the end is an ASan report
  uint8_t* p = b.empty() ? nullptr : (uint8_t*)std::malloc(b.size());
  if (p) std::memcpy(p, b.data(), b.size());
  try {
    parse(p, b.size());
    ++ok;
  } catch (const ZkpError&) {
    ++rejected;
  }
  std::free(p);
}

static void zkey_parse(const uint8_t* p, size_t n) {
  ZkeyParsed z = parse_zkey(p, n, true);
  (void)z;
}
static void wtns_parse(const uint8_t* p, size_t n) {
  WtnsView w = parse_wtns(p, n);
  // touch every witness value the view claims
  volatile uint8_t acc = 0;
  for (size_t i = 0; i < (size_t)w.n_witness * 32; i += 31) acc ^= w.values[i];
}
static void gz_parse(const uint8_t* p, size_t n) {
  std::vector<uint8_t> v(p, p + n);
  std::vector<uint8_t> out = gunzip_if_needed(std::move(v));
  (void)out;
}

template <class F>
static void mutate_all(const std::vector<uint8_t>& base, F&& parse, std::mt19937_64& rng, int nmut) {
  run(base, parse);
  // truncations: every byte of the first 1 KiB, then a grid
  for (size_t t = 0; t < base.size(); t += (t < 1024 ? 1 : base.size() / 257 + 1)) {
    std::vector<uint8_t> b(base.begin(), base.begin() + t);
    run(b, parse);
  }
  // section-length fields (a u64 after each u32 id from offset 12 on) set to extremes
  const uint64_t evil[] = {0, 1, 0xffffffffull, 0xffffffffffffffffull, (uint64_t)base.size(), (uint64_t)base.size() - 11};
  for (size_t off = 16; off + 8 <= std::min<size_t>(base.size(), 4096); off += 4)
    for (uint64_t v : evil) {
      std::vector<uint8_t> b = base;
      std::memcpy(b.data() + off, &v, 8);
      run(b, parse);
    }
  // seeded byte flips (most in the headers, where the lengths and counts live)
  for (int i = 0; i < nmut; ++i) {
    std::vector<uint8_t> b = base;
    const int k = 1 + (int)(rng() % 4);
    for (int j = 0; j < k; ++j) {
      const size_t lim = (rng() & 1) ? std::min<size_t>(b.size(), 2048) : b.size();
      b[rng() % lim] ^= (uint8_t)(1u << (rng() % 8));
    }
    run(b, parse);
  }
}

int main(int argc, char** argv) {
  if (argc < 5) {
    std::fprintf(stderr, "usage: parse_fuzz <zkey> <wtns> <seed> <mutations>\n");
    return 2;
  }
  const std::vector<uint8_t> zk = slurp(argv[1]), wt = slurp(argv[2]);
  if (zk.size() < 16 || wt.size() < 16) return 2;
  std::mt19937_64 rng(std::strtoull(argv[3], nullptr, 10));
  const int nmut = std::atoi(argv[4]);
  mutate_all(zk, zkey_parse, rng, nmut);
  mutate_all(wt, wtns_parse, rng, nmut);
  // gzip reader: a gzip magic followed by garbage / a truncated real stream
  std::vector<uint8_t> g = {0x1f, 0x8b, 0x08, 0x00};
  for (int i = 0; i < 64; ++i) g.push_back((uint8_t)rng());
  mutate_all(g, gz_parse, rng, nmut / 4);
  std::printf("parse_fuzz: %ld parsed, %ld rejected with ZkpError\n", ok, rejected);
  return 0;
}
