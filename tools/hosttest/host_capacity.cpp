// Host-side capacity of the configs[3] batch at N devices: G encoder groups run
// concurrently, one per device of an N-GPU batch, each encoding host witnesses back to back with T
// threads into its own staging region (csrc/wtns_pack.hpp wt_encode_chunk: the exact per-proof host
// work of zkp_prove_batch's upload, minus the DMA enqueues).  Reports witnesses/s over all groups and
// the host-memory traffic it implies, against the proofs/s the GPUs would need (N x the 1-GPU rate).
// No GPU is used: it runs here and on the GPU box's host cores alike.
// usage: host_capacity <n_signals> <groups> <threads_per_group> <seconds> <mix: 70|0> [distinct=2]
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "../../zk-p2p-onramp_amd/csrc/wtns_pack.hpp"

using namespace zkp;

// the bench's synthetic witness mix: bool_pct % of the signals 0/1, the rest uniform < 2^253
static void fill(std::vector<uint32_t>& v, uint32_t n, int bool_pct, uint64_t seed) {
  std::mt19937_64 g(seed);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t* x = &v[(size_t)i * 8];
    const uint64_t r = g();
    if ((int)(r % 100) < bool_pct) {
      for (int k = 0; k < 8; ++k) x[k] = 0;
      x[0] = (uint32_t)(r >> 40) & 1u;
    } else {
      for (int k = 0; k < 8; ++k) x[k] = (uint32_t)g();
      x[7] &= 0x1FFFFFFF;
    }
  }
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: host_capacity <n_signals> <groups> <threads_per_group> <seconds> <bool_pct> [distinct]\n");
    return 2;
  }
  const uint32_t n = (uint32_t)atoi(argv[1]);
  const int G = atoi(argv[2]), T = atoi(argv[3]), bool_pct = atoi(argv[5]);
  const double secs = atof(argv[4]);
  const int D = argc > 6 ? atoi(argv[6]) : 2;
  const uint32_t nch = wt_chunks(n);
  std::vector<std::vector<std::vector<uint32_t>>> wit(G, std::vector<std::vector<uint32_t>>(D));
  std::vector<std::vector<uint32_t>> stage(G);
  for (int g = 0; g < G; ++g) {
    for (int d = 0; d < D; ++d) {
      wit[g][d].resize((size_t)n * 8);
      fill(wit[g][d], n, bool_pct, 1000 * g + d + 1);
    }
    stage[g].assign((size_t)nch * wt_chunk_words(), 0u);
  }
  std::atomic<bool> stop{false};
  std::vector<long> done(G, 0);
  std::vector<double> sent(G, 0.0);
  auto group = [&](int g) {
    // one witness at a time per group, its chunks split over T threads (as DevicePipeline::upload)
    std::vector<size_t> words(nch);
    int d = 0;
    while (!stop.load(std::memory_order_relaxed)) {
      const uint8_t* src = reinterpret_cast<const uint8_t*>(wit[g][d].data());
      std::vector<std::thread> th;
      for (int t = 1; t < T; ++t)
        th.emplace_back([&, t] {
          for (uint32_t c = t; c < nch; c += T) words[c] = wt_encode_chunk(src, n, c, stage[g].data() + (size_t)c * wt_chunk_words());
        });
      for (uint32_t c = 0; c < nch; c += T) words[c] = wt_encode_chunk(src, n, c, stage[g].data() + (size_t)c * wt_chunk_words());
      for (auto& x : th) x.join();
      size_t w = 0;
      for (size_t x : words) w += x;
      sent[g] += w * 4.0;
      ++done[g];
      d = (d + 1) % D;
    }
  };
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> gs;
  for (int g = 0; g < G; ++g) gs.emplace_back(group, g);
  std::this_thread::sleep_for(std::chrono::duration<double>(secs));
  stop = true;
  for (auto& x : gs) x.join();
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  long tot = 0;
  double bytes = 0;
  for (int g = 0; g < G; ++g) tot += done[g], bytes += sent[g];
  const double wps = tot / el;
  printf("{\"n_signals\": %u, \"groups\": %d, \"threads_per_group\": %d, \"bool_pct\": %d, \"seconds\": %.2f, "
         "\"witnesses\": %ld, \"witnesses_per_s\": %.1f, \"host_read_GBps\": %.1f, \"staging_written_GBps\": %.1f, "
         "\"pcie_payload_MB_per_witness\": %.1f}\n",
         n, G, T, bool_pct, el, tot, wps, wps * n * 32.0 / 1e9, bytes / el / 1e9, tot ? bytes / tot / 1e6 : 0.0);
  return 0;
}
