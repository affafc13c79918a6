// CPU replay of the MSM pipeline (msm_kernels.hpp per-thread bodies, same
// parameters as MsmEngine) for debugging without a GPU.
// usage: msm_emu <g1|g2> <file: points(zkey layout)|scalars> <n>   -> prints affine result (hex words)
#include <algorithm>
#include <cstdio>
#include <numeric>
#include <vector>
#include "../../zk-p2p-onramp_amd/csrc/msm_kernels.hpp"
#include "../../zk-p2p-onramp_amd/csrc/msm.hpp"
#include "../../zk-p2p-onramp_amd/csrc/host_ec.hpp"
using namespace zkp;

template <class F, class HF>
static host::Jac<HF> run(std::vector<uint32_t>& pts, std::vector<uint32_t>& sc, uint32_t n) {
  constexpr int FW = FWords<F>::W;
  // convert points to device layout
  for (size_t i = 0; i < pts.size() / 8; ++i) {
    Fq x = load_fe<FqCfg>(&pts[i * 8]);
    x = mul(x, fe_const<FqCfg>(Conv::FQ_ZKEY_TO_DEV));
    store_fe(&pts[i * 8], x);
  }
  MsmParams prm = MsmParams::for_size(std::max<uint32_t>(n, 1));
  const uint32_t W = prm.windows, half = 1u << (prm.c - 1), nb = W * half;
  // compacted digit emission (window-major, point order) as k_digit_count/k_digit_write
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> per(W);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s[9];
    msmk::load_scalar(sc.data(), i, s);
    uint32_t carry = 0;
    bool neg;
    for (uint32_t w = 0; w < W; ++w) {
      uint32_t key = msmk::digit_key(s, (int)w, prm.c, carry, neg, 0xffffffffu);
      if (key != 0xffffffffu) per[w].push_back({key, i | (neg ? 0x80000000u : 0u)});
    }
  }
  std::vector<uint32_t> ks, vs;
  for (auto& v : per)
    for (auto& e : v) ks.push_back(e.first), vs.push_back(e.second);
  // stable sort on the bucket bits only (as the (c-1)-bit radix sort)
  std::vector<uint32_t> idx(ks.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return (ks[a] & (half - 1)) < (ks[b] & (half - 1)); });
  { std::vector<uint32_t> k2(ks.size()), v2(ks.size()); for (size_t i = 0; i < idx.size(); ++i) { k2[i] = ks[idx[i]]; v2[i] = vs[idx[i]]; } ks.swap(k2); vs.swap(v2); }
  const uint32_t total2 = (uint32_t)ks.size();
  std::vector<uint32_t> st(nb + 1, 0), en(nb + 1, 0), cnt(nb + 1), off(nb + 1);
  for (uint32_t i = 0; i < total2; ++i) msmk::bounds(i, ks.data(), total2, st.data(), en.data());
  for (uint32_t b = 0; b <= nb; ++b) msmk::task_counts(b, st.data(), en.data(), nb, prm.S, cnt.data());
  uint32_t acc = 0;
  for (uint32_t b = 0; b <= nb; ++b) { off[b] = acc; acc += cnt[b]; }
  const uint32_t ntask = off[nb];
  std::vector<uint32_t> part((size_t)(ntask + 1) * 4 * FW);
  for (uint32_t t = 0; t < ntask; ++t) msmk::accumulate<F>(t, pts.data(), vs.data(), st.data(), en.data(), off.data(), nb, prm.S, part.data());
  // heavy-bucket merge levels (as MsmEngine::run)
  int levels = 0;
  for (size_t m = (n + prm.S - 1) / prm.S; m > (size_t)prm.S2; m = (m + prm.S2 - 1) / prm.S2) ++levels;
  std::vector<uint32_t> part1(part.size()), hcnt(nb + 1), hoff(nb + 1);
  for (int lv = 0; lv < levels; ++lv) {
    for (uint32_t b = 0; b <= nb; ++b) msmk::heavy_counts(b, off.data(), nb, prm.S2, lv, hcnt.data());
    uint32_t a2 = 0;
    for (uint32_t b = 0; b <= nb; ++b) { hoff[b] = a2; a2 += hcnt[b]; }
    const uint32_t* src = (lv & 1) ? part1.data() : part.data();
    uint32_t* dst = (lv & 1) ? part.data() : part1.data();
    for (uint32_t t = 0; t < hoff[nb]; ++t) msmk::merge_heavy<F>(t, src, off.data(), hoff.data(), nb, prm.S2, lv, dst);
  }
  std::vector<uint32_t> buckets((size_t)nb * 4 * FW);
  for (uint32_t b = 0; b < nb; ++b)
    msmk::merge_final<F>(b, part.data(), part1.data(), off.data(), nb, prm.S2, levels, buckets.data());
  uint32_t nodes = (half + prm.L - 1) / prm.L;
  std::vector<uint32_t> s0((size_t)W * nodes * 4 * FW), t0(s0.size()), s1(s0.size()), t1(s0.size());
  for (uint32_t id = 0; id < W * nodes; ++id) msmk::reduce_first<F>(id, buckets.data(), W, half, prm.L, s0.data(), t0.data());
  int lgw = 3;
  while (nodes > 1) {
    uint32_t next = (nodes + prm.L - 1) / prm.L;
    for (uint32_t id = 0; id < W * next; ++id) msmk::reduce_level<F>(id, s0.data(), t0.data(), W, nodes, prm.L, lgw, s1.data(), t1.data());
    std::swap(s0, s1); std::swap(t0, t1);
    nodes = next; lgw += 3;
  }
  // fold windows on host (same as prover.hip fold_windows)
  auto ld = [&](uint32_t w) {
    const uint32_t* p = t0.data() + (size_t)w * 4 * FW;
    if constexpr (FW == 8)
      return host::jac_from_xyzz(host::fq_from_dev(p), host::fq_from_dev(p + 8), host::fq_from_dev(p + 16), host::fq_from_dev(p + 24));
    else {
      auto f2 = [](const uint32_t* q) { return host::Fq2{host::fq_from_dev(q), host::fq_from_dev(q + 8)}; };
      return host::jac_from_xyzz(f2(p), f2(p + 16), f2(p + 32), f2(p + 48));
    }
  };
  host::Jac<HF> r = ld(W - 1);
  for (int w = (int)W - 2; w >= 0; --w) {
    for (int i = 0; i < prm.c; ++i) r = host::jac_dbl(r);
    r = host::jac_add(r, ld(w));
  }
  return r;
}

int main(int argc, char** argv) {
  bool g2 = std::string(argv[1]) == "g2";
  FILE* f = fopen(argv[2], "rb");
  uint32_t n = atoi(argv[3]);
  size_t pw = g2 ? 32 : 16;
  std::vector<uint32_t> pts(n * pw), sc(n * 8 + 8);
  if (fread(pts.data(), 4, pts.size(), f) != pts.size()) return 1;
  if (fread(sc.data(), 4, n * 8, f) != n * 8) return 1;
  if (!g2) {
    auto a = host::jac_to_aff(run<Fq, host::Fq>(pts, sc, n));
    if (a.inf) { printf("inf\n"); return 0; }
    auto x = a.x.to_std(), y = a.y.to_std();
    printf("%s %s\n", host::u256_to_dec(x).c_str(), host::u256_to_dec(y).c_str());
  } else {
    auto a = host::jac_to_aff(run<Fq2, host::Fq2>(pts, sc, n));
    if (a.inf) { printf("inf\n"); return 0; }
    printf("%s %s %s %s\n", host::u256_to_dec(a.x.c0.to_std()).c_str(), host::u256_to_dec(a.x.c1.to_std()).c_str(),
           host::u256_to_dec(a.y.c0.to_std()).c_str(), host::u256_to_dec(a.y.c1.to_std()).c_str());
  }
  return 0;
}
