// CPU replay of the MSM pipeline (msm_kernels.hpp per-thread bodies, same
// parameters as MsmEngine) for debugging without a GPU.
// usage: msm_emu <g1|g2> <file: points(zkey layout)|scalars> <n> [c] [depth]   -> prints affine result (decimal)
#include <algorithm>
#include <cstdio>
#include <numeric>
#include <vector>
#include "../../zk-p2p-onramp_amd/csrc/msm_kernels.hpp"
#include "../../zk-p2p-onramp_amd/csrc/msm.hpp"
#include "../../zk-p2p-onramp_amd/csrc/host_ec.hpp"
using namespace zkp;

template <class F, class HF>
static host::Jac<HF> run(std::vector<uint32_t>& pts, std::vector<uint32_t>& sc, uint32_t n, int c_ovr, int d_ovr) {
  constexpr int FW = FWords<F>::W;
  // convert points to device layout
  for (size_t i = 0; i < pts.size() / 8; ++i) {
    Fq x = load_fe<FqCfg>(&pts[i * 8]);
    x = mul(x, fe_const<FqCfg>(Conv::FQ_ZKEY_TO_DEV));
    store_fe(&pts[i * 8], x);
  }
  MsmParams prm = MsmParams::make(std::max<uint32_t>(n, 1), c_ovr, d_ovr);
  const uint32_t W = prm.windows, T = prm.depth, G = prm.groups, half = 1u << (prm.c - 1), nb = G * half;
  // base table rows 1..T-1 (as MsmBases::extend)
  std::vector<uint32_t> table((size_t)T * n * 2 * FW);
  std::copy(pts.begin(), pts.begin() + (size_t)n * 2 * FW, table.begin());
  for (uint32_t t = 1; t < T; ++t)
    for (uint32_t i = 0; i < n; ++i) msmk::extend_row<F>(i, table.data(), n, prm.c, (int)t);
  // the nonzero digits (window-major, point order); the device sort groups them by bucket in another order
  std::vector<std::vector<std::pair<uint32_t, uint32_t>>> per(W);
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s[9];
    msmk::load_scalar(sc.data(), i, s);
    uint32_t carry = 0, key, val;
    for (uint32_t w = 0; w < W; ++w)
      if (msmk::digit_entry(s, (int)w, prm.c, (int)T, n, i, carry, key, val)) per[w].push_back({key, val});
  }
  std::vector<uint32_t> ks, vs;
  for (auto& v : per)
    for (auto& e : v) ks.push_back(e.first), vs.push_back(e.second);
  // stable sort on the whole bucket key (group and bucket bits), as the bucket sort groups them
  std::vector<uint32_t> idx(ks.size());
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return ks[a] < ks[b]; });
  { std::vector<uint32_t> k2(ks.size()), v2(ks.size()); for (size_t i = 0; i < idx.size(); ++i) { k2[i] = ks[idx[i]]; v2[i] = vs[idx[i]]; } ks.swap(k2); vs.swap(v2); }
  const uint32_t total2 = (uint32_t)ks.size();
  std::vector<uint32_t> st(nb + 1, 0), en(nb + 1, 0), cnt(nb + 1), off(nb + 1);
  for (uint32_t i = 0; i < total2; ++i) {  // bucket [start, end) and ceil(len / S) tasks (as k_hs_fine / k_hs_bounds3)
    if (i == 0 || ks[i - 1] != ks[i]) st[ks[i]] = i;
    if (i == total2 - 1 || ks[i + 1] != ks[i]) en[ks[i]] = i + 1;
  }
  for (uint32_t b = 0; b <= nb; ++b) cnt[b] = b == nb ? 0u : (en[b] - st[b] + prm.S - 1) / prm.S;
  uint32_t acc = 0;
  for (uint32_t b = 0; b <= nb; ++b) { off[b] = acc; acc += cnt[b]; }
  const uint32_t ntask = off[nb];
  std::vector<uint32_t> part((size_t)(ntask + 1) * 4 * FW);
  for (uint32_t t = 0; t < ntask; ++t) msmk::accumulate<F>(t, table.data(), vs.data(), st.data(), en.data(), off.data(), nb, prm.S, nullptr, part.data());
  // heavy-bucket merge levels (as MsmPlan::build + MsmEngine::run)
  const int levels = msm_merge_levels(std::max<uint32_t>(n, 1), prm);
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
  // reduction (as run_finish): segments, then the K subset sums, each by one subset_first thread whose
  // fan-in covers all its values (the device sums them by LDS trees: the same group elements)
  const uint32_t M = prm.M, lgP = prm.lgP(), K = prm.K(), P = half / M, fan = std::max<uint32_t>(P, 1);
  std::vector<uint32_t> ss((size_t)G * P * 4 * FW), tt(ss.size());
  for (uint32_t id = 0; id < G * P; ++id) msmk::reduce_segments<F>(id, buckets.data(), G, half, M, ss.data(), tt.data());
  const uint32_t nn = msmk::subset_n1(lgP, fan);  // 1
  std::vector<uint32_t> sub((size_t)G * K * nn * 4 * FW);
  for (uint32_t id = 0; id < G * K * nn; ++id) msmk::subset_first<F>(id, ss.data(), tt.data(), G, lgP, fan, sub.data());
  // host fold (same as prover.hip msm_fold)
  auto ld = [&](uint32_t w) {
    const uint32_t* p = sub.data() + (size_t)w * 4 * FW;
    if constexpr (FW == 8)
      return host::jac_from_xyzz(host::fq_from_dev(p), host::fq_from_dev(p + 8), host::fq_from_dev(p + 16), host::fq_from_dev(p + 24));
    else {
      auto f2 = [](const uint32_t* q) { return host::Fq2{host::fq_from_dev(q), host::fq_from_dev(q + 8)}; };
      return host::jac_from_xyzz(f2(p), f2(p + 16), f2(p + 32), f2(p + 48));
    }
  };
  auto group = [&](uint32_t g) {
    host::Jac<HF> a = lgP > 0 ? ld(g * K + lgP - 1) : host::Jac<HF>::inf();
    for (int b = (int)lgP - 2; b >= 0; --b) a = host::jac_add(host::jac_dbl(a), ld(g * K + b));
    for (int i = 0; i < prm.lg_m(); ++i) a = host::jac_dbl(a);
    return host::jac_add(a, ld(g * K + lgP));
  };
  host::Jac<HF> r = group(G - 1);
  for (int g = (int)G - 2; g >= 0; --g) {
    for (int i = 0; i < prm.c * (int)T; ++i) r = host::jac_dbl(r);
    r = host::jac_add(r, group(g));
  }
  return r;
}

int main(int argc, char** argv) {
  bool g2 = std::string(argv[1]) == "g2";
  FILE* f = fopen(argv[2], "rb");
  uint32_t n = atoi(argv[3]);
  const int c_ovr = argc > 4 ? atoi(argv[4]) : 0, d_ovr = argc > 5 ? atoi(argv[5]) : 0;
  size_t pw = g2 ? 32 : 16;
  std::vector<uint32_t> pts(n * pw), sc(n * 8 + 8);
  if (fread(pts.data(), 4, pts.size(), f) != pts.size()) return 1;
  if (fread(sc.data(), 4, n * 8, f) != n * 8) return 1;
  if (!g2) {
    auto a = host::jac_to_aff(run<Fq, host::Fq>(pts, sc, n, c_ovr, d_ovr));
    if (a.inf) { printf("inf\n"); return 0; }
    auto x = a.x.to_std(), y = a.y.to_std();
    printf("%s %s\n", host::u256_to_dec(x).c_str(), host::u256_to_dec(y).c_str());
  } else {
    auto a = host::jac_to_aff(run<Fq2, host::Fq2>(pts, sc, n, c_ovr, d_ovr));
    if (a.inf) { printf("inf\n"); return 0; }
    printf("%s %s %s %s\n", host::u256_to_dec(a.x.c0.to_std()).c_str(), host::u256_to_dec(a.x.c1.to_std()).c_str(),
           host::u256_to_dec(a.y.c0.to_std()).c_str(), host::u256_to_dec(a.y.c1.to_std()).c_str());
  }
  return 0;
}
