// Groth16 prover core (see prover.hpp).
#include "prover.hpp"

#include <functional>

#include <sched.h>
#include <sys/random.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <future>
#include <shared_mutex>
#include <thread>

#include "hip_check.hpp"
#include "host_pairing.hpp"
#include "qap.hpp"

namespace zkp {

using host::Affine;
using host::Jac;
using host::U256;
using HFq = host::Fq;
using HFq2 = host::Fq2;
using HFr = host::Fr;

// parsing (parse_binfile, parse_wtns, parse_zkey): zkey_parse.cpp, host-only (sanitizer-tested)

// ------------------------------------------------------------------ host EC helpers

static HFq2 fq2_from_dev(const uint32_t* w) { return HFq2{host::fq_from_dev(w), host::fq_from_dev(w + 8)}; }

template <class F>
static F f_from_dev(const uint32_t* w);
template <>
HFq f_from_dev<HFq>(const uint32_t* w) {
  return host::fq_from_dev(w);
}
template <>
HFq2 f_from_dev<HFq2>(const uint32_t* w) {
  return fq2_from_dev(w);
}

// fold an MSM engine output (device XYZZ layout, G x K points: per group the lgP subset
// sums Q_b then sum_p T_p) into the MSM value:
//   R_g = sum_p T_p + M * sum_b 2^b Q_b,   result = sum_g 2^(c T g) R_g   (Horner both)
template <class F>
static Jac<F> msm_fold(const uint32_t* win, const MsmParams& p) {
  constexpr int FW = sizeof(F) == sizeof(HFq) ? 8 : 16;
  auto load = [&](size_t k) {
    const uint32_t* q = win + k * 4 * FW;
    return host::jac_from_xyzz(f_from_dev<F>(q), f_from_dev<F>(q + FW), f_from_dev<F>(q + 2 * FW),
                               f_from_dev<F>(q + 3 * FW));
  };
  const int K = p.K(), lgP = p.lgP();
  auto group = [&](int g) {
    Jac<F> acc = lgP > 0 ? load((size_t)g * K + lgP - 1) : Jac<F>::inf();
    for (int b = lgP - 2; b >= 0; --b) acc = host::jac_add(host::jac_dbl(acc), load((size_t)g * K + b));
    for (int i = 0; i < p.lg_m(); ++i) acc = host::jac_dbl(acc);
    return host::jac_add(acc, load((size_t)g * K + lgP));
  };
  Jac<F> r = group(p.groups - 1);
  for (int g = p.groups - 2; g >= 0; --g) {
    for (int i = 0; i < p.c * p.depth; ++i) r = host::jac_dbl(r);
    r = host::jac_add(r, group(g));
  }
  return r;
}

static U256 scalar_or_random(const uint8_t* s32) {
  U256 v;
  if (s32) {
    v = host::u256_from_le(s32);
    while (host::u256_geq(v, host::FR_DESC.mod)) host::u256_sub(v, host::FR_DESC.mod);
    return v;
  }
  for (;;) {
    uint8_t b[32];
    size_t got = 0;
    while (got < 32) {
      ssize_t k = getrandom(b + got, 32 - got, 0);
      if (k <= 0) throw ZkpError(ZKP_ERR_INTERNAL, "getrandom failed");
      got += (size_t)k;
    }
    b[31] &= 0x3f;  // 254 bits
    v = host::u256_from_le(b);
    if (!host::u256_geq(v, host::FR_DESC.mod)) return v;
  }
}

static void put_fq(const HFq& x, uint8_t* out) { host::u256_to_le(x.to_std(), out); }

// ------------------------------------------------------------------ device pipeline

// host cores this process may use: the affinity mask, capped by a cgroup v2 CPU quota (the GPU boxes
// show 256 CPUs to nproc but allow 16)
static int host_cores() {
  static const int n = [] {
    int c = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) c = CPU_COUNT(&set);
    if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long per = 0;
      if (std::fscanf(f, "%31s %ld", q, &per) == 2 && std::strcmp(q, "max") != 0 && per > 0) {
        const long quota = std::atol(q);
        if (quota > 0) c = std::min(c, (int)std::max(1L, (quota + per / 2) / per));
      }
      std::fclose(f);
    }
    return std::max(1, c);
  }();
  return n;
}

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return (v && *v) ? std::atoi(v) : dflt;
}

// MSM tuning options: ONE environment variable read when a prover (or a kernel-level MSM) is built,
// ZKP_MSM = "key=value[,key=value...]" (empty / unset: automatic everything):
//   w=<bits>  h=<bits>    window bits of the witness plan / the H plan and the kernel-level MSMs (8..24)
//   depth=<rows>          base-table rows T per point (1..W; default W, or the largest depth whose
//                         tables fit half of the free HBM)
//   task_w=<n> task_h=<n> entries per bucket-accumulation task of either plan (default 48 / 48)
//   seg=<n>               buckets per bucket-reduction segment (a power of two; default 4)
//   plan=dense|compact    the plan variant of the kernel-level MSMs (zkp_msm_*; default dense)
// A malformed value or an unknown key is a ZKP_ERR_INVALID_ARG: a typo never silently tunes nothing.
//   w2=<bits>             window bits of the second witness plan (default w + 2; full provers only)
//   wsets=1|2             witness-MSM configurations kept resident (default 2: w and w2)
//   wsel=first|second|auto  which one a proof takes (default auto: by the witness's share of values
//                         >= 2^32, DevicePipeline::pick_wset)
struct MsmOptions {
  int w = 0, h = 0, depth = 0, task_w = 0, task_h = 0, seg = 0, w2 = 0, wsets = 2;
  int dense = 1;
  int wsel = 0;  // 0 auto, 1 first, 2 second
};
static MsmOptions msm_options() {
  MsmOptions o;
  const char* e = std::getenv("ZKP_MSM");
  if (!e) return o;
  std::string spec(e);
  size_t at = 0;
  while (at < spec.size()) {
    size_t end = spec.find(',', at);
    if (end == std::string::npos) end = spec.size();
    const std::string item = spec.substr(at, end - at);
    at = end + 1;
    if (item.empty()) continue;
    const size_t eq = item.find('=');
    if (eq == std::string::npos) throw ZkpError(ZKP_ERR_INVALID_ARG, "ZKP_MSM: '" + item + "' is not key=value");
    const std::string key = item.substr(0, eq), val = item.substr(eq + 1);
    if (key == "plan") {
      if (val != "dense" && val != "compact") throw ZkpError(ZKP_ERR_INVALID_ARG, "ZKP_MSM: plan=dense|compact");
      o.dense = val == "dense" ? 1 : 0;
      continue;
    }
    if (key == "wsel") {
      if (val != "first" && val != "second" && val != "auto")
        throw ZkpError(ZKP_ERR_INVALID_ARG, "ZKP_MSM: wsel=first|second|auto");
      o.wsel = val == "first" ? 1 : (val == "second" ? 2 : 0);
      continue;
    }
    char* stop = nullptr;
    const long v = std::strtol(val.c_str(), &stop, 10);
    if (val.empty() || *stop || v <= 0 || v > (1 << 20))
      throw ZkpError(ZKP_ERR_INVALID_ARG, "ZKP_MSM: bad value in '" + item + "'");
    int* dst = key == "w" ? &o.w : key == "h" ? &o.h : key == "depth" ? &o.depth : key == "task_w" ? &o.task_w
             : key == "task_h" ? &o.task_h : key == "seg" ? &o.seg : key == "w2" ? &o.w2
             : key == "wsets" ? &o.wsets : nullptr;
    if (!dst) throw ZkpError(ZKP_ERR_INVALID_ARG, "ZKP_MSM: unknown key '" + key + "'");
    if (key == "seg" && (v & (v - 1))) throw ZkpError(ZKP_ERR_INVALID_ARG, "ZKP_MSM: seg must be a power of two");
    if (key == "wsets" && v > 2) throw ZkpError(ZKP_ERR_INVALID_ARG, "ZKP_MSM: wsets=1|2");
    *dst = (int)v;
  }
  return o;
}

static MsmParams make_params(size_t n, int c, int depth) {
  try {
    return MsmParams::make(n, c, depth);
  } catch (const std::invalid_argument& x) {
    throw ZkpError(ZKP_ERR_INVALID_ARG, x.what());
  }
}

// MSM parameters for a prover: window bits automatic (ZKP_MSM w= / h= override); table depth = W
// (one bucket set) unless the tables would not fit in half of the free HBM, then the largest depth
// that does (ZKP_MSM depth= overrides).
static void choose_msm_params(size_t n_w, size_t n_h, const MsmOptions& o, MsmParams& pw, MsmParams& ph) {
  // measured on the Venmo shape (273c6e8:tools/gpu/experiments/sweep_c2.sh): the witness MSMs (70 % of the
  // digits of a 0/1-heavy witness are single entries) prefer one bit less than lg n - 4, the
  // uniform-scalar H MSM one bit more (fewer windows; the bucket reduction is cheap), moved off the
  // widths whose top window collapses into a few buckets (dense_window_bits)
  auto lg = [](size_t n) {
    int l = 0;
    while ((size_t(1) << l) < n) ++l;
    return l;
  };
  auto clampc = [](int c) { return c < 8 ? 8 : (c > 20 ? 20 : c); };
  const int cw = o.w ? o.w : clampc(lg(n_w) - 5);
  const int ch = o.h ? o.h : dense_window_bits(clampc(lg(n_h) - 3), n_h);
  // H-plan tasks of <= 48 entries (the uniform quotient scalars fill every bucket evenly, ~208 entries at
  // the Venmo shape: 5 task partials per bucket instead of 7, so the latency-bound merge_final at the end
  // of the proof folds fewer): +0.7 % and +0.9 % proofs/s over 32, 7 of 7 alternated rounds on two boxes
  // (profiles/task_size_ab_r05.txt).  Witness-plan tasks of <= 48 too since the G2 accumulation runs first
  // (round 6): +0.6 / +1.0 % over 32 on two boxes, every alternated pair; 96 ties, 128 and 192 lose
  // (profiles/task_w_ab_r06.txt)
  auto tune = [&] {
    pw.S = o.task_w > 0 ? o.task_w : 48;
    ph.S = o.task_h > 0 ? o.task_h : 48;
    for (MsmParams* q : {&pw, &ph})
      if (o.seg > 0 && o.seg <= (1 << (q->c - 1))) q->M = o.seg;
  };
  pw = make_params(n_w, cw, o.depth);
  ph = make_params(n_h, ch, o.depth);
  tune();
  if (o.depth > 0) return;
  size_t free_b = 0, total_b = 0;
  HIPX(hipMemGetInfo(&free_b, &total_b));
  const size_t row_w = n_w * (3 * 64 + 128), row_h = n_h * 64;
  const size_t budget = free_b / 2;
  int depth = std::max(pw.windows, ph.windows);
  while (depth > 1 && (size_t)std::min(depth, pw.windows) * row_w + (size_t)std::min(depth, ph.windows) * row_h > budget)
    --depth;
  pw = make_params(n_w, cw, depth);
  ph = make_params(n_h, ch, depth);
  tune();
}

// upload `count` zkey points (snarkjs LEM layout) into row 0 of a base table at point
// offset `at`, convert to the device Montgomery form, then derive the shifted rows
static void fill_bases(MsmBases& b, const uint8_t* src, size_t count, size_t at, hipStream_t st) {
  const size_t pw = b.curve() == Curve::G1 ? 16 : 32;  // words per point
  if (at) HIPX(hipMemsetAsync(b.row0(), 0, at * pw * 4, st));  // leading infinity points
  if (count) {
    HIPX(hipMemcpyAsync(b.row0() + at * pw, src, count * pw * 4, hipMemcpyHostToDevice, st));
    launch_convert_fq_zkey(b.row0() + at * pw, count * pw / 8, st);
  }
  b.extend(st);
}

// [lo, hi) of slice `part` when n items are cut into nparts contiguous ranges.  With
// ZKP_SPLIT_BALANCE=1 (a split proof with the distributed quotient) and G = nparts > 3, the parts
// that extend a quotient vector (0..2: rank v % G extends vector v) get weight max(1, 11 - G) and
// the others 11: with one coset extension costing r = 1/8 of the proof's MSM work M (S24: ~6.6 of
// ~53 ms), Q + M s_q = M s_o and 3 s_q + (G - 3) s_o = 1 give s_q = (11 - G) / (8 G),
// s_o = 11 / (8 G).  lo = n W_<k / W in integers (zkp_amd.dist.split_range and
// oracle.groth16.split_range compute the same).
static void split_range(size_t n, int part, int nparts, size_t& lo, size_t& hi) {
  const char* e = std::getenv("ZKP_SPLIT_BALANCE");
  if (!(e && std::atoi(e) == 1) || nparts <= 3) {
    lo = n * (size_t)part / (size_t)nparts;
    hi = n * (size_t)(part + 1) / (size_t)nparts;
    return;
  }
  const size_t wq = (size_t)std::max(1, 11 - nparts);
  auto cum = [&](int k) { return wq * (size_t)std::min(k, 3) + (size_t)11 * (size_t)std::max(k - 3, 0); };
  const size_t total = cum(nparts);
  lo = n * cum(part) / total;
  hi = n * cum(part + 1) / total;
}

// A long-lived host thread that runs one job at a time (the per-proof G1 / G2 enqueue jobs of a
// pipeline: no thread creation on the proof's critical path)
class JobThread {
 public:
  JobThread() : th_([this] { loop(); }) {}
  ~JobThread() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void start(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = std::move(f);
      done_ = false;
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return done_; });
  }

 private:
  void loop() {
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
      cv_.wait(lk, [&] { return stop_ || job_; });
      if (!job_) return;  // stop with no job pending
      std::function<void()> f = std::move(job_);
      job_ = nullptr;
      lk.unlock();
      f();  // the jobs catch their own exceptions
      lk.lock();
      done_ = true;
      cv_.notify_all();
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::function<void()> job_;
  bool stop_ = false, done_ = true;
  std::thread th_;  // last: started once the state above exists
};

class DevicePipeline {
 public:
  // part / nparts: this pipeline holds only slice `part` of every point section (the
  // point-range split of one proof over several GPUs); 0 / 1 = all
  // share: another pipeline of the same device and slice whose base tables (the ~38 GB of
  // precomputed points) this one uses instead of building its own (ZKP_INFLIGHT > 1: several
  // proofs in flight per device, each with its own streams, plans, engines and buffers)
  DevicePipeline(int dev, const ZkeyParsed& z, int part = 0, int nparts = 1, const DevicePipeline* share = nullptr)
      : dev_(dev), hdr_(z.hdr) {
    HIPX(hipSetDevice(dev_));
    // s0 carries the critical path (quotient -> H plan -> H MSM): highest priority, so the
    // A/B1/C (s2) and B2 (s1) MSMs fill the CUs it leaves idle instead of delaying it
    int prio_lo = 0, prio_hi = 0;
    HIPX(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIPX(hipStreamCreateWithPriority(&s0_, hipStreamNonBlocking, prio_hi));
    HIPX(hipStreamCreateWithPriority(&s1_, hipStreamNonBlocking, prio_lo));
    HIPX(hipStreamCreateWithPriority(&s2_, hipStreamNonBlocking, prio_lo));
    // s3 runs every MSM's finish (merges + reduction: short latency-bound launches) at high
    // priority, so they slip in between the long accumulations instead of queueing behind them
    HIPX(hipStreamCreateWithPriority(&s3_, hipStreamNonBlocking, prio_hi));
    for (auto& e : ev_) HIPX(hipEventCreate(&e));
    HIPX(hipEventCreateWithFlags(&ev_g2acc_, hipEventDisableTiming));
    const ZkeyHeader& h = hdr_;
    const size_t nd_all = h.domain_size, c0 = (size_t)h.n_public + 1;  // first witness index with a C base
    split_range(h.n_vars, part, nparts, wlo_, whi_);
    split_range(h.domain_size, part, nparts, hlo_, hhi_);
    const size_t nv = whi_ - wlo_, nd = hhi_ - hlo_;
    const MsmOptions opt = msm_options();
    MsmParams pw, ph;
    choose_msm_params(nv, nd, opt, pw, ph);
    wsel_opt_ = opt.wsel;
    // base tables: A, B1, C, B2 indexed by witness signal (C's first nPublic+1 bases are
    // infinity, so one witness plan serves all four), H by domain index
    auto build_wtables = [&](WSet& w) {
      w.ta = std::make_shared<MsmBases>(Curve::G1, nv, w.pw.c, w.pw.depth);
      w.tb1 = std::make_shared<MsmBases>(Curve::G1, nv, w.pw.c, w.pw.depth);
      w.tc = std::make_shared<MsmBases>(Curve::G1, nv, w.pw.c, w.pw.depth);
      w.tb2 = std::make_shared<MsmBases>(Curve::G2, nv, w.pw.c, w.pw.depth);
      fill_bases(*w.ta, z.bf.sec[5].ptr + wlo_ * 64, nv, 0, s0_);
      fill_bases(*w.tb1, z.bf.sec[6].ptr + wlo_ * 64, nv, 0, s0_);
      fill_bases(*w.tb2, z.bf.sec[7].ptr + wlo_ * 128, nv, 0, s0_);
      const size_t cfirst = std::max(wlo_, c0);  // first witness index of the slice with a C base
      const size_t lead = std::min(cfirst, whi_) - wlo_;
      const size_t cnt = whi_ > cfirst ? whi_ - cfirst : 0;
      fill_bases(*w.tc, cnt ? z.bf.sec[8].ptr + (cfirst - c0) * 64 : nullptr, cnt, lead, s0_);
    };
    if (share) {
      if (share->dev_ != dev_ || share->wlo_ != wlo_ || share->whi_ != whi_ || share->hlo_ != hlo_ ||
          share->hhi_ != hhi_)
        throw ZkpError(ZKP_ERR_INTERNAL, "shared base tables of another device or slice");
      nws_ = share->wset2_tables_ ? 2 : 1;
      for (int k = 0; k < nws_; ++k) {
        const WSet& o = share->ws_[k];
        ws_[k].pw = o.pw, ws_[k].ta = o.ta, ws_[k].tb1 = o.tb1, ws_[k].tc = o.tc, ws_[k].tb2 = o.tb2;
      }
      th_ = share->th_;
      // the H plan and engine must read th_ with the parameters it was built with: a sibling's own
      // choose_msm_params can pick another depth when less HBM is free by now
      ph = share->plan_h_->params();
      if (th_->c() != ph.c || th_->depth() != ph.depth)
        throw ZkpError(ZKP_ERR_INTERNAL, "shared H table built with other parameters");
    } else {
      ws_[0].pw = pw;
      build_wtables(ws_[0]);
      th_ = std::make_shared<MsmBases>(Curve::G1, nd, ph.c, ph.depth);
      fill_bases(*th_, z.bf.sec[9].ptr + hlo_ * 64, nd, 0, s0_);
      // the second witness configuration (round 5): c = w + 2 bits, one bucket set,
      // for witnesses whose values are mostly >= 2^32 (all-uniform: c = 20 is ~7 % faster than 18 on the
      // Venmo shape, profiles/wsweep_r04.txt); full provers only, and only where its tables fit in half
      // of the HBM still free (the Venmo key: +26.6 GB)
      const int c2 = opt.w2 ? opt.w2 : std::min(24, pw.c + 2);
      if (nparts == 1 && opt.wsets == 2 && c2 != pw.c) {
        HIPX(hipStreamSynchronize(s0_));
        size_t free_b = 0, total_b = 0;
        HIPX(hipMemGetInfo(&free_b, &total_b));
        const MsmParams p2 = make_params(nv, c2, 0);
        if ((size_t)p2.windows * nv * (3 * 64 + 128) <= free_b / 2) {
          ws_[1].pw = make_params(nv, c2, p2.windows);
          ws_[1].pw.S = opt.task_w > 0 ? opt.task_w : 48;
          if (opt.seg > 0 && opt.seg <= (1 << (ws_[1].pw.c - 1))) ws_[1].pw.M = opt.seg;
          build_wtables(ws_[1]);
          nws_ = 2;
        }
      }
    }
    for (int m = 0; m < 2; ++m) {
      const Csr& c = z.csr[m];
      HIPX(hipMalloc(&rowptr_[m], c.rowptr.size() * 4));
      HIPX(hipMemcpyAsync(rowptr_[m], c.rowptr.data(), c.rowptr.size() * 4, hipMemcpyHostToDevice, s0_));
      HIPX(hipMalloc(&col_[m], std::max<size_t>(c.col.size() * 4, 4)));
      HIPX(hipMalloc(&val_[m], std::max<size_t>(c.val.size() * 4, 32)));
      if (!c.col.empty()) {
        HIPX(hipMemcpyAsync(col_[m], c.col.data(), c.col.size() * 4, hipMemcpyHostToDevice, s0_));
        HIPX(hipMemcpyAsync(val_[m], c.val.data(), c.val.size() * 4, hipMemcpyHostToDevice, s0_));
        launch_convert_coefs(val_[m], c.col.size(), s0_);
      }
    }
    // witness upload slots: each has its own copy stream, so a proof's
    // witness H2D runs outside the compute lock and overlaps the proof in flight, and its own pinned
    // staging buffer and copy threads (upload()); allocated on the slot's first host-witness upload
    // (ensure_upload_slot), so staged-only and split provers hold no pinned staging or copy threads
    for (auto& b : abc_) HIPX(hipMalloc(&b, nd_all * 32));
    HIPX(hipMalloc(&pscal_, nd_all * 32));
    ntt_ = std::make_unique<NttEngine>((int)h.log_domain, s0_);
    // the witness plan feeds A/B1/C on s2 and B2 on s1; they overlap the quotient on s0, which then
    // plans and runs the H MSM.  The witness plan runs on the high-priority finish stream s3 (ahead
    // of its G1 finishes), so its sort passes are not starved by the quotient's NTTs on s0: the
    // witness accumulations start ~5 ms earlier; proof 26.69 -> 26.58 ms (profiles/wplan_r03.txt)
    nv_ = nv;
    build_engines(ws_[0]);
    plan_h_ = std::make_unique<MsmPlan>(nd, ph, s0_);
    // H scalars are uniform (quotient evaluations): dense plan (one workgroup per sub-bin)
    plan_h_->set_dense(true);
    g1h_ = std::make_unique<MsmEngine>(Curve::G1, ph, nd, s0_);
    winh_ = g1h_->window_words();
    // the second witness configuration's plan and engines (~6 GB at the Venmo shape) come later
    // (add_second_wset), after every pipeline of the prover holds its essentials; the group-sum slots
    // are sized for both
    wset2_tables_ = nws_ > 1;
    nws_ = 1;
    wina_ = ws_[0].g1[0]->window_words();
    win2_ = ws_[0].g2->window_words();
    if (wset2_tables_) {
      const MsmParams& p2 = ws_[1].pw;
      wina_ = std::max(wina_, MsmEngine::window_words_for(Curve::G1, p2));
      win2_ = std::max(win2_, MsmEngine::window_words_for(Curve::G2, p2));
    }
    HIPX(hipMalloc(&dwin_, win_total() * 4));
    HIPX(hipHostMalloc(&hwin_, win_total() * 4, hipHostMallocDefault));
    // a full prover's first upload slot exists from load on, so a one-shot prover's first host-witness
    // proof does not pay its ~410 MB of HBM, ~220 MB of pinned memory, streams and copy threads, and an
    // out-of-memory surfaces here rather than at prove time; the second slot stays lazy
    if (nparts == 1) ensure_upload_slot(0);
    HIPX(hipStreamSynchronize(s0_));
  }

  // the second witness configuration's plan and engines, this pipeline's own: with many pipelines on
  // one GPU (ZKP_INFLIGHT, a multi-device rehearsal) HBM can run out here, and the pipeline then keeps
  // the first configuration only (the shared tables stay).  Called by the Prover once every pipeline
  // is built.
  void add_second_wset() {
    if (!wset2_tables_ || nws_ > 1) return;
    HIPX(hipSetDevice(dev_));
    try {
      build_engines(ws_[1]);
      nws_ = 2;
    } catch (const HipError& e) {
      if (e.code != hipErrorOutOfMemory) throw;
      (void)hipGetLastError();
      ws_[1].plan.reset();
      for (auto& g : ws_[1].g1) g.reset();
      ws_[1].g2.reset();
    }
  }

  ~DevicePipeline() {
    (void)hipSetDevice(dev_);
    ntt_.reset();
    for (auto& w : ws_) w = WSet{};
    g1h_.reset();
    plan_h_.reset();
    th_.reset();
    for (void* p : {(void*)rowptr_[0], (void*)rowptr_[1], (void*)col_[0], (void*)col_[1], (void*)val_[0],
                    (void*)val_[1], (void*)up_[0], (void*)up_[1], (void*)abc_[0], (void*)abc_[1], (void*)abc_[2],
                    (void*)pscal_,
                    (void*)dwin_})
      if (p) (void)hipFree(p);
    for (uint32_t* p : slots_)
      if (p) (void)hipFree(p);
    if (hwin_) (void)hipHostFree(hwin_);
    for (auto& e : ev_) (void)hipEventDestroy(e);
    if (ev_g2acc_) (void)hipEventDestroy(ev_g2acc_);
    for (int k = 0; k < NUP; ++k) {
      for (auto& t : copiers_[k]) t.reset();
      if (sup_[k]) (void)hipStreamSynchronize(sup_[k]), (void)hipStreamDestroy(sup_[k]);
      for (int j = 0; j + 1 < NDMA; ++j) {
        if (sdma_[k][j]) (void)hipStreamSynchronize(sdma_[k][j]), (void)hipStreamDestroy(sdma_[k][j]);
        if (evdma_[k][j]) (void)hipEventDestroy(evdma_[k][j]);
      }
      if (uph_[k]) (void)hipHostFree(uph_[k]);
      if (upstage_[k]) (void)hipFree(upstage_[k]);
    }
    (void)hipStreamDestroy(s0_);
    (void)hipStreamDestroy(s1_);
    (void)hipStreamDestroy(s2_);
    (void)hipStreamDestroy(s3_);
  }

  struct MsmOut {
    Jac<HFq> a, b1, c, h;
    Jac<HFq2> b2;
    float ms[6];
    float pcie_mb = 0;  // witness transfer payload (prove() from a host witness)
    int wset = 0;       // the witness configuration the proof took (pick_wset)
  };
  // called with a, b1, c, b2 folded (h not yet) while the H MSM still runs on the device
  using EarlyFn = std::function<void(const MsmOut&)>;

  // ---- witness upload slots.  acquire_upload() blocks until one of the NUP slots is free;
  // upload() copies a witness into it (the calling thread waits for it, the compute streams do
  // not); prove_uploaded() then runs the proof on it under the compute lock.  Two callers (two
  // zkp_prove threads, or the two batch workers of a device) thus overlap one proof's upload with
  // the other's compute.
  int acquire_upload() {
    std::unique_lock<std::mutex> lk(upmu_);
    upcv_.wait(lk, [&] {
      for (bool b : upbusy_)
        if (!b) return true;
      return false;
    });
    for (int k = 0; k < NUP; ++k)
      if (!upbusy_[k]) {
        upbusy_[k] = true;
        return k;
      }
    return 0;  // unreachable
  }
  void release_upload(int k) {
    {
      std::lock_guard<std::mutex> lk(upmu_);
      upbusy_[k] = false;
    }
    upcv_.notify_one();
  }
  struct UploadSlot {  // RAII: one acquired upload slot
    DevicePipeline* d;
    int k;
    explicit UploadSlot(DevicePipeline* dp) : d(dp), k(dp->acquire_upload()) {}
    ~UploadSlot() { d->release_upload(k); }
  };
  // H2D of a witness (pageable host memory, 32 B per signal) into slot k.  PCIe is the limit (a
  // 205 MB witness: ~4.3 ms at ~48 GB/s through pinned memory), so the transfer is COMPACT: NCOPY
  // host threads encode chunks of 64K signals (qap.hpp WT_*: per block of 64, the values >= 2^32 as
  // 32 B, the others as their low word, plus a 12-byte block meta) straight into the slot's pinned
  // buffer and enqueue each chunk's DMA (pinned -> HBM staging, the slot's copy stream) as soon as it
  // is encoded, so encoding and PCIe overlap; one kernel then expands the chunks into the 32-B
  // witness layout.  A 0/1-heavy witness moves ~2.5x fewer bytes; an all-uniform one as many plus the
  // meta.  Returns the wall time (ms).
  // the resources of upload slot k, created on its first use (the caller holds slot k)
  void ensure_upload_slot(int k) {
    if (up_[k]) return;
    const size_t stage_words = std::max<size_t>(wt_chunks(hdr_.n_vars), 1) * wt_chunk_words();
    // (each piece only if missing: a failed first attempt leaves no leak behind the next one)
    if (!upstage_[k]) HIPX(hipMalloc(&upstage_[k], stage_words * 4));
    if (!uph_[k]) HIPX(hipHostMalloc(&uph_[k], stage_words * 4, hipHostMallocDefault));
    if (!sup_[k]) HIPX(hipStreamCreateWithFlags(&sup_[k], hipStreamNonBlocking));
    for (int j = 0; j + 1 < NDMA; ++j) {
      if (!sdma_[k][j]) HIPX(hipStreamCreateWithFlags(&sdma_[k][j], hipStreamNonBlocking));
      if (!evdma_[k][j]) HIPX(hipEventCreateWithFlags(&evdma_[k][j], hipEventDisableTiming));
    }
    for (auto& t : copiers_[k])
      if (!t) t = std::make_unique<JobThread>();
    HIPX(hipMalloc(&up_[k], std::max<size_t>((size_t)hdr_.n_vars * 32, 32)));  // last: marks the slot ready
  }
  float upload(int k, const WtnsView& w, uint64_t* pcie_bytes = nullptr) {
    HIPX(hipSetDevice(dev_));
    const auto t0 = std::chrono::steady_clock::now();
    ensure_upload_slot(k);
    const uint32_t n = hdr_.n_vars;
    const uint32_t nch = wt_chunks(n);
    const size_t chw = wt_chunk_words();
    const uint8_t* src = w.values;
    uint32_t* pin = reinterpret_cast<uint32_t*>(uph_[k]);
    hipStream_t st = sup_[k];
    std::exception_ptr errs[NCOPY];
    std::atomic<uint64_t> sent{0};
    std::atomic<uint32_t> large{0};
    // encode threads: every usable host core for a lone upload (the single-proof latency path), the
    // cores shared out among concurrent uploads (an 8-GPU batch has up to 16 at once: 8 groups of 16
    // threads encode 705 Venmo witnesses/s on a 16-core quota, of 2 threads 1,096/s;
    // profiles/host_capacity_r05.json)
    struct Active {
      Active() { ++uploads_active_; }
      ~Active() { --uploads_active_; }
    } active;
    const int T = std::max(2, std::min(NCOPY, host_cores() / std::max(1, uploads_active_.load())));
    // chunk c's DMA goes to stream c % NDMA: one copy queue serialises the ~100 chunk copies with
    // ~10 us between them (rocprofv3 --memory-copy-trace: 2.7 ms for 62 MB), parallel queues overlap
    // those gaps and each other's transfers
    auto dma_stream = [&](uint32_t c) { return (c % NDMA) == 0 ? st : sdma_[k][c % NDMA - 1]; };
    auto part = [&](int t) {
      try {
        HIPX(hipSetDevice(dev_));
        uint32_t nl = 0;
        for (uint32_t c = (uint32_t)t; c < nch; c += (uint32_t)T) {
          const size_t words = wt_encode_chunk(src, n, c, pin + (size_t)c * chw, &nl);
          HIPX(hipMemcpyAsync(upstage_[k] + (size_t)c * chw, pin + (size_t)c * chw, words * 4, hipMemcpyHostToDevice,
                              dma_stream(c)));
          sent += words * 4;
        }
        large += nl;
      } catch (...) {
        errs[t] = std::current_exception();
      }
    };
    for (int t = 1; t < T; ++t) copiers_[k][t - 1]->start([&, t] { part(t); });
    part(0);
    for (int t = 1; t < T; ++t) copiers_[k][t - 1]->wait();
    for (auto& e : errs)
      if (e) {
        (void)hipStreamSynchronize(st);
        for (int j = 0; j + 1 < NDMA; ++j) (void)hipStreamSynchronize(sdma_[k][j]);
        std::rethrow_exception(e);
      }
    // one expansion after every chunk's DMA has been enqueued (the other copy queues joined by events
    // recorded here, after every encode thread has enqueued its copies)
    for (int j = 0; j + 1 < NDMA; ++j) {
      HIPX(hipEventRecord(evdma_[k][j], sdma_[k][j]));
      HIPX(hipStreamWaitEvent(st, evdma_[k][j], 0));
    }
    launch_witness_unpack(upstage_[k], 0, n, up_[k], st);
    HIPX(hipStreamSynchronize(st));
    if (pcie_bytes) *pcie_bytes = sent.load();
    up_large_[k] = n ? (double)large.load() / n : 0.0;
    return std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  MsmOut prove_uploaded(int k, float h2d_ms, const EarlyFn& early = {}) {
    std::lock_guard<std::mutex> lk(mu_);
    HIPX(hipSetDevice(dev_));
    maybe_inject_fault();
    HIPX(hipEventRecord(ev_[0], s0_));
    HIPX(hipEventRecord(ev_[1], s0_));
    MsmOut o = prove_dev(up_[k], early, pick_wset(up_large_[k]));
    o.ms[0] = h2d_ms;
    return o;
  }
  // test hook (ZKP_TEST_FAIL, read by Prover): this pipeline
  // reports a device failure on its (after+1)-th proof and every later one
  void set_fault_injection(int after) { fail_after_ = after; }
  bool healthy() const { return healthy_.load(); }
  void mark_failed() { healthy_.store(false); }
  int device() const { return dev_; }

  // quotient (rows A4..A8) from a device-resident witness; result scalars in pscal_
  void enqueue_quotient(const uint32_t* d_wit) {
    const ZkeyHeader& h = hdr_;
    launch_build_abc(rowptr_[0], col_[0], val_[0], rowptr_[1], col_[1], val_[1], d_wit, h.domain_size, abc_[0],
                     abc_[1], abc_[2], s0_);
    HIPX(hipEventRecord(ev_[2], s0_));
    // one vector per launch, not coset_extend_batch: the batched passes (3x the workgroups at s0's
    // high priority) finish the quotient ~1.8 ms sooner but crowd out the G2 and witness
    // accumulations that fill the per-vector launches' last-round gaps -- -4 % proofs/s, +0.5 ms
    // latency on one box, 4 alternating rounds (profiles/ntt_batch_ab_r04.txt)
    for (auto* b : abc_) ntt_->coset_extend(b);
    launch_join_abc(abc_[0], abc_[1], abc_[2], h.domain_size, pscal_, s0_);
    HIPX(hipEventRecord(ev_[3], s0_));
  }

  // keep a witness resident in HBM slot `slot` (benchmarks: timing without PCIe)
  // Staging slots are written under stage_mu_ held exclusively, and read (slot lookup AND the whole
  // proof that reads the slot, on this pipeline or a ZKP_INFLIGHT sibling) under stage_mu_ shared:
  // restaging waits for the proofs that read the old witness.  Lock order: stage_mu_, then mu_.
  std::unique_lock<std::shared_mutex> lock_stage() { return std::unique_lock<std::shared_mutex>(stage_mu_); }
  void stage(int slot, const WtnsView& w) {  // caller holds lock_stage()
    std::lock_guard<std::mutex> lk(mu_);
    HIPX(hipSetDevice(dev_));
    if (slot < 0 || slot > 4096) throw ZkpError(ZKP_ERR_INVALID_ARG, "bad staging slot");
    if ((size_t)slot >= slots_.size()) slots_.resize(slot + 1, nullptr);
    if (!slots_[slot]) HIPX(hipMalloc(&slots_[slot], (size_t)hdr_.n_vars * 32));
    if ((size_t)slot >= slot_large_.size()) slot_large_.resize(slot + 1, 0.0);
    HIPX(hipMemcpyAsync(slots_[slot], w.values, (size_t)hdr_.n_vars * 32, hipMemcpyHostToDevice, s0_));
    // the share of values >= 2^32 (pick_wset), counted while the copy runs
    size_t nl = 0;
    for (size_t i = 0; i < hdr_.n_vars; ++i) {
      const uint8_t* v = w.values + 32 * i;
      uint32_t w1;
      uint64_t hi[3];
      std::memcpy(&w1, v + 4, 4);
      std::memcpy(hi, v + 8, 24);
      nl += (w1 | hi[0] | hi[1] | hi[2]) != 0;
    }
    slot_large_[slot] = hdr_.n_vars ? (double)nl / hdr_.n_vars : 0.0;
    HIPX(hipStreamSynchronize(s0_));
  }
  double slot_large(int slot) const {  // caller holds the staging lock (shared)
    return slot >= 0 && (size_t)slot < slot_large_.size() ? slot_large_[slot] : 0.0;
  }
  const uint32_t* slot_ptr(int slot) const {
    if (slot < 0 || (size_t)slot >= slots_.size() || !slots_[slot])
      throw ZkpError(ZKP_ERR_INVALID_ARG, "staging slot is empty");
    return slots_[slot];
  }

  void set_instrument(bool on) {
    std::lock_guard<std::mutex> lk(mu_);
    for (int k = 0; k < nws_; ++k) {
      for (auto& g : ws_[k].g1) g->set_instrument(on);
      ws_[k].g2->set_instrument(on);
    }
    g1h_->set_instrument(on);
    stats_g1_ = MsmEngine::Stats{};
    stats_g2_ = MsmEngine::Stats{};
    launches_.clear();
  }
  void stats(MsmEngine::Stats& g1, MsmEngine::Stats& g2) {
    std::lock_guard<std::mutex> lk(mu_);
    g1 = stats_g1_;
    g2 = stats_g2_;
  }
  // every instrumented accumulate launch since set_instrument(true): {kind, adds, ms}, kind 0..2 the
  // witness MSMs A, B1, C (G1), 3 the H MSM (G1), 4 the witness MSM B2 (G2)
  void launch_records(std::vector<std::array<double, 4>>& out) {
    std::lock_guard<std::mutex> lk(mu_);
    out.insert(out.end(), launches_.begin(), launches_.end());
  }
  void msm_params(MsmParams& pw, MsmParams& ph, MsmParams* pw2 = nullptr) const {
    pw = ws_[0].plan->params();
    ph = plan_h_->params();
    if (pw2) *pw2 = nws_ > 1 ? ws_[1].plan->params() : MsmParams{};
  }
  int witness_sets() const { return nws_; }
  size_t table_bytes() const {
    size_t b = th_->bytes();
    for (int k = 0; k < (wset2_tables_ ? 2 : 1); ++k)  // resident tables, whether or not this pipeline's engines use them
      b += ws_[k].ta->bytes() + ws_[k].tb1->bytes() + ws_[k].tc->bytes() + ws_[k].tb2->bytes();
    return b;
  }
  // the witness configuration a proof takes: the second (wider windows) when the witness's share of
  // values >= 2^32 is above WSET2_LARGE_FRAC (each such value carries a digit in every window; 0/1 and
  // other small values only one or two), unless ZKP_MSM wsel= fixes it
  int pick_wset(double large_frac) const {
    if (nws_ < 2 || wsel_opt_ == 1) return 0;
    if (wsel_opt_ == 2) return 1;
    return large_frac > WSET2_LARGE_FRAC ? 1 : 0;
  }
  static constexpr double WSET2_LARGE_FRAC = 0.55;

  void quotient(const WtnsView& w, uint8_t* out) {
    UploadSlot slot(this);
    upload(slot.k, w);
    std::lock_guard<std::mutex> lk(mu_);
    HIPX(hipSetDevice(dev_));
    enqueue_quotient(up_[slot.k]);
    HIPX(hipMemcpyAsync(out, pscal_, (size_t)hdr_.domain_size * 32, hipMemcpyDeviceToHost, s0_));
    HIPX(hipStreamSynchronize(s0_));
  }

  // Distributed quotient of a split proof, stage 1: buildABC on the
  // witness in `slot`, then the coset extension (rows A5-A7) of the vectors in mask (bit 0
  // A, 1 B, 2 C) only, each copied whole (domain x 32 bytes, device layout: Montgomery
  // 2^261, 8 packed words) to dst[v], device memory on this device.  Returns when done.
  void quotient_part_staged(int slot, int mask, void* const* dst) {
    std::shared_lock<std::shared_mutex> sl(stage_mu_);
    std::lock_guard<std::mutex> lk(mu_);
    HIPX(hipSetDevice(dev_));
    const uint32_t* d = slot_ptr(slot);
    const ZkeyHeader& h = hdr_;
    launch_build_abc(rowptr_[0], col_[0], val_[0], rowptr_[1], col_[1], val_[1], d, h.domain_size, abc_[0], abc_[1],
                     abc_[2], s0_);
    uint32_t* sel[3];
    int cnt = 0;
    for (int v = 0; v < 3; ++v) {
      if (!(mask >> v & 1)) continue;
      if (!dst[v]) throw ZkpError(ZKP_ERR_INVALID_ARG, "quotient part: null destination");
      sel[cnt++] = abc_[v];
    }
    if (cnt) ntt_->coset_extend_batch(sel, cnt);
    for (int v = 0; v < 3; ++v)
      if (mask >> v & 1)
        HIPX(hipMemcpyAsync(dst[v], abc_[v], (size_t)h.domain_size * 32, hipMemcpyDeviceToDevice, s0_));
    HIPX(hipStreamSynchronize(s0_));
  }

  // stage 2: this slice's partial sums with the H scalars joined (row A8) from abc[0..2] =
  // the coset evaluations of A, B, C at this part's domain slice (device memory, ready)
  MsmOut prove_ext_staged(int slot, const void* const* abc) {
    std::shared_lock<std::shared_mutex> sl(stage_mu_);
    std::lock_guard<std::mutex> lk(mu_);
    HIPX(hipSetDevice(dev_));
    const uint32_t* d = slot_ptr(slot);
    for (int v = 0; v < 3; ++v)
      if (!abc[v]) throw ZkpError(ZKP_ERR_INVALID_ARG, "partial prove: null quotient slice");
    HIPX(hipEventRecord(ev_[0], s0_));
    HIPX(hipEventRecord(ev_[1], s0_));
    for (int v = 0; v < 3; ++v) ext_abc_[v] = static_cast<const uint32_t*>(abc[v]);
    try {
      MsmOut o = prove_dev(d);
      for (auto& e : ext_abc_) e = nullptr;
      return o;
    } catch (...) {
      for (auto& e : ext_abc_) e = nullptr;
      throw;
    }
  }

  MsmOut prove(const WtnsView& w, const EarlyFn& early = {}) {
    UploadSlot slot(this);
    uint64_t bytes = 0;
    const float ms = upload(slot.k, w, &bytes);
    MsmOut o = prove_uploaded(slot.k, ms, early);
    o.pcie_mb = (float)(bytes * 1e-6);
    return o;
  }

  MsmOut prove_staged(int slot, const EarlyFn& early = {}) {
    std::shared_lock<std::shared_mutex> sl(stage_mu_);
    return prove_resident(slot_ptr(slot), early, slot_large(slot));
  }
  // shared hold of this (first) pipeline's staging slots for a proof that reads one of them
  std::shared_lock<std::shared_mutex> hold_stage() { return std::shared_lock<std::shared_mutex>(stage_mu_); }

  // a proof of a witness already resident on this GPU: this pipeline's staging slot, or a
  // ZKP_INFLIGHT sibling's (staged witnesses live in the device's first pipeline)
  MsmOut prove_resident(const uint32_t* d_wit, const EarlyFn& early = {}, double large_frac = 0.0) {
    std::lock_guard<std::mutex> lk(mu_);
    HIPX(hipSetDevice(dev_));
    HIPX(hipEventRecord(ev_[0], s0_));
    HIPX(hipEventRecord(ev_[1], s0_));
    return prove_dev(d_wit, early, pick_wset(large_frac));
  }
  // claimed by a staged caller (Prover::prove_staged spreads concurrent callers over the pipelines)
  std::atomic<bool> staged_busy{false};

  // the whole device pipeline on a resident witness (caller holds mu_, ev_[0..1] recorded)
  MsmOut prove_dev(const uint32_t* d_wit, const EarlyFn& early = {}, int wsel = 0) {
    WSet& ws = ws_[wsel < nws_ ? wsel : 0];
    const size_t win2 = ws.g2->window_words();
    // group-sum layout in dwin_ (slots sized for the larger witness configuration): A | B1 | C
    // (engines ws.g1) | H (g1h) | B2 (ws.g2)
    uint32_t* wa = dwin_;
    uint32_t* wh = dwin_ + 3 * wina_;
    uint32_t* wb2 = wh + winh_;
    // s2: witness plan, then the G1 accumulations A, B1, C back to back; s3 finishes each
    // (merges + reduction: latency-bound chains) while s2 accumulates the next;
    // s1: G2 MSM B2 on the same plan; s0: quotient (buildABC, 3 coset NTTs, joinABC),
    // H plan, H MSM.  A starts when the G2 accumulation ends: the G2 finish (a latency-bound chain
    // on the low-priority s1) then runs beside A, B1 and C instead of waiting out the H accumulation
    // and sharing the proof's tail with the H finish (+0.4 %, 7 of 8 alternated pairs:
    // profiles/g2_first_ab_r06.txt).
    // MsmPlan::build blocks its host thread once (the sort needs the nonzero-digit
    // count), so each stream is fed from its own host thread; the G2 thread starts
    // once the witness plan is enqueued (its stream then waits on plan.ready()).
    // ZKP_SERIAL=1 (profiling only) chains the three streams so every kernel runs alone.
    std::exception_ptr err[3];
    std::promise<void> planned;
    std::shared_future<void> planned_f = planned.get_future().share();
    bool planned_set = false;
    const int g2first = serial_ ? 0 : g2first_;
    std::promise<void> g2acc;
    std::shared_future<void> g2acc_f = g2acc.get_future().share();
    bool g2acc_set = false;
    auto g1_job = [&] {
      try {
        HIPX(hipSetDevice(dev_));
        HIPX(hipStreamWaitEvent(s2_, ev_[1], 0));
        HIPX(hipEventRecord(ev_[9], s2_));
        HIPX(hipStreamWaitEvent(ws.plan->stream(), ev_[1], 0));
        ws.plan->build(d_wit + wlo_ * 8, whi_ - wlo_);
        planned.set_value();
        planned_set = true;
        const MsmBases* tabs[3] = {ws.ta.get(), ws.tb1.get(), ws.tc.get()};
        for (int m = 0; m < 3; ++m) {
          if (g2first && m == g2first - 1) {
            g2acc_f.get();
            HIPX(hipStreamWaitEvent(s2_, ev_g2acc_, 0));
          }
          ws.g1[m]->accumulate(*ws.plan, *tabs[m]);
          HIPX(hipEventRecord(ev_[10 + m], s2_));
          HIPX(hipStreamWaitEvent(s3_, ev_[10 + m], 0));
          ws.g1[m]->finish(*ws.plan, wa + m * wina_, s3_);
          if (serial_) {  // profiling: no overlap between the finish and the next accumulation
            HIPX(hipEventRecord(ev_[13], s3_));
            HIPX(hipStreamWaitEvent(s2_, ev_[13], 0));
          }
        }
        HIPX(hipEventRecord(ev_[8], s3_));
      } catch (...) {
        err[0] = std::current_exception();
        if (!planned_set) planned.set_exception(std::current_exception());
      }
    };
    auto g2_job = [&] {
      try {
        planned_f.get();
        HIPX(hipSetDevice(dev_));
        if (serial_) HIPX(hipStreamWaitEvent(s1_, ev_[8], 0));
        HIPX(hipEventRecord(ev_[7], s1_));
        // the finish on s1 too: s3 is in-order, the G1 finishes must not queue behind it (gating the
        // G2 finish on the H plan, on either stream, measured +0.9 ms: profiles/g2_finish_r03.txt)
        ws.g2->accumulate(*ws.plan, *ws.tb2);
        if (g2first) {
          HIPX(hipEventRecord(ev_g2acc_, s1_));
          g2acc.set_value();
          g2acc_set = true;
        }
        ws.g2->finish(*ws.plan, wb2, s1_);
        HIPX(hipEventRecord(ev_[6], s1_));
      } catch (...) {
        err[1] = std::current_exception();
        if (g2first && !g2acc_set) g2acc.set_exception(std::current_exception());
      }
    };
    auto h_job = [&] {
      try {
        if (serial_) HIPX(hipStreamWaitEvent(s0_, ev_[6], 0));
        if (ext_abc_[0]) {  // distributed quotient: only the join of this domain slice
          HIPX(hipEventRecord(ev_[2], s0_));
          launch_join_abc(ext_abc_[0], ext_abc_[1], ext_abc_[2], (uint32_t)(hhi_ - hlo_), pscal_ + hlo_ * 8, s0_);
          HIPX(hipEventRecord(ev_[3], s0_));
        } else {
          enqueue_quotient(d_wit);
        }
        plan_h_->build(pscal_ + hlo_ * 8, hhi_ - hlo_);
        g1h_->run(*plan_h_, *th_, wh);
      } catch (...) {
        err[2] = std::current_exception();
      }
    };
    if (serial_) {
      g1_job();
      if (!err[0]) g2_job();
      if (!err[0] && !err[1]) h_job();
    } else {
      jt_g2_.start(g2_job);
      jt_g1_.start(g1_job);
      h_job();
      jt_g1_.wait();
      jt_g2_.wait();
    }
    for (auto& e : err)
      if (e) {
        (void)hipDeviceSynchronize();  // let every enqueued kernel drain before buffers are reused
        std::rethrow_exception(e);
      }
    HIPX(hipEventRecord(ev_[4], s0_));
    // the witness MSMs' group sums (A | B1 | C, B2) go to the host as soon as their finishes end
    // (s3 holds the G1 finishes; it waits for the G2 finish), so the host folds them and the caller
    // blinds A, B and the r/s part of C (`early`) while the H MSM still runs; only C + H, the
    // affine conversions and the H fold remain after the device is done
    HIPX(hipStreamWaitEvent(s3_, ev_[6], 0));
    HIPX(hipMemcpyAsync(hwin_, dwin_, 3 * wina_ * 4, hipMemcpyDeviceToHost, s3_));
    HIPX(hipMemcpyAsync(hwin_ + 3 * wina_ + winh_, wb2, win2 * 4, hipMemcpyDeviceToHost, s3_));
    HIPX(hipEventRecord(ev_[15], s3_));
    HIPX(hipMemcpyAsync(hwin_ + 3 * wina_, wh, winh_ * 4, hipMemcpyDeviceToHost, s0_));
    HIPX(hipEventRecord(ev_[5], s0_));
    MsmOut o;
    const MsmParams& pa = ws.g1[0]->params();
    const MsmParams& ph = g1h_->params();
    HIPX(hipEventSynchronize(ev_[15]));
    o.a = msm_fold<HFq>(hwin_, pa);
    o.b1 = msm_fold<HFq>(hwin_ + wina_, pa);
    o.c = msm_fold<HFq>(hwin_ + 2 * wina_, pa);
    o.b2 = msm_fold<HFq2>(hwin_ + 3 * wina_ + winh_, pa);
    if (early) {
      try {
        early(o);
      } catch (...) {
        (void)hipStreamSynchronize(s0_);  // the H MSM and its copy still run: drain before rethrowing
        (void)hipStreamSynchronize(s3_);
        throw;
      }
    }
    HIPX(hipStreamSynchronize(s0_));
    HIPX(hipStreamSynchronize(s3_));
    for (int m = 0; m < 3; ++m) collect_kind(*ws.g1[m], m, stats_g1_);
    collect_kind(*g1h_, 3, stats_g1_);
    collect_kind(*ws.g2, 4, stats_g2_);
    o.wset = wsel < nws_ ? wsel : 0;
    o.h = msm_fold<HFq>(hwin_ + 3 * wina_, ph);
    HIPX(hipEventElapsedTime(&o.ms[0], ev_[0], ev_[1]));  // wtns H2D
    HIPX(hipEventElapsedTime(&o.ms[1], ev_[1], ev_[2]));  // buildABC
    HIPX(hipEventElapsedTime(&o.ms[2], ev_[2], ev_[3]));  // NTT + join
    HIPX(hipEventElapsedTime(&o.ms[3], ev_[9], ev_[8]));  // witness plan + G1 MSMs A, B1, C (s2)
    HIPX(hipEventElapsedTime(&o.ms[4], ev_[7], ev_[6]));  // G2 MSM (s1)
    HIPX(hipEventElapsedTime(&o.ms[5], ev_[3], ev_[4]));  // H plan + G1 MSM H (s0)
    return o;
  }

 private:
  int dev_;
  size_t wlo_ = 0, whi_ = 0, hlo_ = 0, hhi_ = 0;  // witness / domain slice held by this pipeline
  bool serial_ = env_int("ZKP_SERIAL", 0) == 1;  // profiling: no stream overlap
  ZkeyHeader hdr_;
  hipStream_t s0_ = nullptr, s1_ = nullptr, s2_ = nullptr, s3_ = nullptr;
  // the G2 accumulation's end on s1: the first G1 witness accumulation (A) waits for it (g2first_ = k:
  // accumulation k - 1 waits; ZKP_G2FIRST=0 lets A, B1, C run beside it from the start)
  hipEvent_t ev_g2acc_ = nullptr;
  int g2first_ = env_int("ZKP_G2FIRST", 1);
  hipEvent_t ev_[16];
  JobThread jt_g1_, jt_g2_;  // host threads feeding s2 (witness plan, G1 MSMs) and s1 (G2 MSM)
  // one witness-MSM configuration (the witness plan serves A, B1, C and B2): window bits, base tables
  // (shared by the pipelines of one device), plan and engines (per pipeline)
  struct WSet {
    MsmParams pw;
    std::shared_ptr<MsmBases> ta, tb1, tc, tb2;
    std::unique_ptr<MsmPlan> plan;
    std::unique_ptr<MsmEngine> g1[3], g2;  // g1: A, B1, C
  };
  WSet ws_[2];
  int nws_ = 1, wsel_opt_ = 0;
  bool wset2_tables_ = false;  // this device holds the second configuration's tables (add_second_wset)
  size_t nv_ = 0;              // witness signals of this pipeline's slice
  void build_engines(WSet& w) {
    w.plan = std::make_unique<MsmPlan>(nv_, w.pw, s3_);
    for (auto& g : w.g1) g = std::make_unique<MsmEngine>(Curve::G1, w.pw, nv_, s2_);
    w.g2 = std::make_unique<MsmEngine>(Curve::G2, w.pw, nv_, s1_);
  }
  std::shared_ptr<MsmBases> th_;  // shared by the pipelines of one device
  uint32_t* rowptr_[2] = {nullptr, nullptr};
  uint32_t* col_[2] = {nullptr, nullptr};
  uint32_t* val_[2] = {nullptr, nullptr};
  static constexpr int NUP = 2;    // witness upload slots (double buffering)
  static constexpr int NCOPY = 16;  // host threads per upload at most (compact encoding into pinned memory, DMA enqueues)
  static inline std::atomic<int> uploads_active_{0};  // uploads in progress in this process (all pipelines)
  uint32_t* up_[NUP] = {nullptr, nullptr};      // the witness slots (32 B per signal)
  uint32_t* upstage_[NUP] = {nullptr, nullptr};  // compact chunk regions (HBM)
  uint8_t* uph_[NUP] = {nullptr, nullptr};       // pinned staging of each slot: compact chunk regions

  hipStream_t sup_[NUP] = {nullptr, nullptr};
  static constexpr int NDMA = 4;  // copy queues per upload slot (sup_ and NDMA - 1 more)
  hipStream_t sdma_[NUP][NDMA > 1 ? NDMA - 1 : 1] = {};
  hipEvent_t evdma_[NUP][NDMA > 1 ? NDMA - 1 : 1] = {};
  std::unique_ptr<JobThread> copiers_[NUP][NCOPY - 1];
  std::mutex upmu_;
  std::condition_variable upcv_;
  bool upbusy_[NUP] = {false, false};
  std::atomic<bool> healthy_{true};
  int fail_after_ = -1, proofs_done_ = 0;
  void maybe_inject_fault() {
    if (fail_after_ >= 0 && proofs_done_++ >= fail_after_) {
      healthy_.store(false);
      throw HipError(hipErrorLaunchFailure, "injected device failure (ZKP_TEST_FAIL)", __FILE__, __LINE__);
    }
  }
  uint32_t* abc_[3] = {nullptr, nullptr, nullptr};
  uint32_t* pscal_ = nullptr;
  const uint32_t* ext_abc_[3] = {nullptr, nullptr, nullptr};  // set only inside prove_ext_staged
  std::unique_ptr<NttEngine> ntt_;
  std::unique_ptr<MsmPlan> plan_h_;
  std::unique_ptr<MsmEngine> g1h_;
  size_t wina_ = 0, winh_ = 0, win2_ = 0;  // group-sum slot sizes (max over the witness configurations)
  size_t win_total() const { return 3 * wina_ + winh_ + win2_; }
  uint32_t* dwin_ = nullptr;
  uint32_t* hwin_ = nullptr;
  std::mutex mu_;
  std::shared_mutex stage_mu_;  // staging slots (see stage())
  std::vector<uint32_t*> slots_;
  std::vector<double> slot_large_;     // per staging slot: share of witness values >= 2^32
  double up_large_[NUP] = {0.0, 0.0};  // per upload slot, of the witness last uploaded
  MsmEngine::Stats stats_g1_, stats_g2_;
  std::vector<std::array<double, 4>> launches_;  // {kind, adds, ms, workgroups} per instrumented launch (capped)
  void collect_kind(MsmEngine& e, int kind, MsmEngine::Stats& agg) {
    MsmEngine::Stats s;
    e.collect(s);
    agg.accumulate_ms += s.accumulate_ms, agg.launches += s.launches, agg.mixed_adds += s.mixed_adds;
    agg.tasks += s.tasks;
    for (const auto& l : s.per_launch)
      if (launches_.size() < 65536) launches_.push_back({(double)kind, (double)l.adds, (double)l.ms, (double)l.blocks});
  }
};

// ------------------------------------------------------------------ Prover

Prover::Prover(const uint8_t* zkey, size_t len, const std::vector<int>& devices, int part, int nparts)
    : part_(part), nparts_(nparts) {
  if (nparts < 1 || part < 0 || part >= nparts) throw ZkpError(ZKP_ERR_INVALID_ARG, "bad part / nparts");
  if (nparts > 1 && devices.size() > 1) throw ZkpError(ZKP_ERR_INVALID_ARG, "a partial prover runs on one device");
  ZkeyParsed z = parse_zkey(zkey, len);
  hdr_ = z.hdr;
  int ndev = 0;
  HIPX(hipGetDeviceCount(&ndev));
  if (ndev <= 0) throw ZkpError(ZKP_ERR_DEVICE, "no HIP device available");
  std::vector<int> devs = devices.empty() ? std::vector<int>{0} : devices;
  // ZKP_INFLIGHT = k > 1: k pipelines per device sharing its base tables, so zkp_prove_batch
  // (one worker per pipeline) and concurrent zkp_prove callers keep k proofs in flight per GPU
  // devs_ holds inflight_ consecutive pipelines per entry of `devices`; the staged entry points'
  // dev_index names an entry of `devices` (its first pipeline).  An ordinal listed twice (a
  // multi-device rehearsal on one GPU) shares the base tables of its first listing.
  inflight_ = std::max(1, std::min(4, env_int("ZKP_INFLIGHT", 1)));
  for (int d : devs)
    if (d < 0 || d >= ndev) throw ZkpError(ZKP_ERR_INVALID_ARG, "device ordinal out of range");
  ndevices_ = (int)devs.size();
  devs_.resize((size_t)ndevices_ * inflight_);
  // the first listing of every ordinal builds its base tables (upload + row derivation, ~2 s
  // for the Venmo key): one host thread per GPU, so an 8-GPU load takes as long as one
  std::vector<int> owner(ndevices_, -1);  // entry whose tables entry e shares (-1: builds its own)
  for (int e = 0; e < ndevices_; ++e)
    for (int f = 0; f < e && owner[e] < 0; ++f)
      if (devs[f] == devs[e] && owner[f] < 0) owner[e] = f;
  {
    std::vector<std::exception_ptr> errs(ndevices_);
    std::vector<std::thread> th;
    for (int e = 0; e < ndevices_; ++e)
      if (owner[e] < 0)
        th.emplace_back([&, e] {
          try {
            devs_[(size_t)e * inflight_] = std::make_unique<DevicePipeline>(devs[e], z, part, nparts);
          } catch (...) {
            errs[e] = std::current_exception();
          }
        });
    for (auto& t : th) t.join();
    for (auto& x : errs)
      if (x) std::rethrow_exception(x);
  }
  for (int e = 0; e < ndevices_; ++e) {
    const DevicePipeline* first = devs_[(size_t)(owner[e] < 0 ? e : owner[e]) * inflight_].get();
    if (owner[e] >= 0) devs_[(size_t)e * inflight_] = std::make_unique<DevicePipeline>(devs[e], z, part, nparts, first);
    for (int k = 1; k < inflight_; ++k)
      devs_[(size_t)e * inflight_ + k] = std::make_unique<DevicePipeline>(devs[e], z, part, nparts, first);
  }
  for (auto& d : devs_) d->add_second_wset();
  // test hooks (never set in production): verify-before-return default, a corrupted H partial
  // (exercises verify-before-return), an injected device failure (exercises the batch re-queue)
  {
    const int v = env_int("ZKP_VERIFY", 2);
    verify_.store(v >= 0 && v <= 2 ? v : 2);
  }
  corrupt_h_ = env_int("ZKP_TEST_CORRUPT_H", 0);
  // ZKP_TEST_FAIL="<pipeline>:<after>": that pipeline reports a device failure from its (after+1)-th proof on
  if (const char* f = std::getenv("ZKP_TEST_FAIL")) {
    int fp = -1, after = 0;
    if (std::sscanf(f, "%d:%d", &fp, &after) == 2 && fp >= 0 && fp < (int)devs_.size())
      devs_[fp]->set_fault_injection(after);
  }
}

// next healthy pipeline in round-robin order (a pipeline that hit a HIP error is skipped)
DevicePipeline& Prover::pick_device() {
  const size_t nd = devs_.size();
  const unsigned start = rr_.fetch_add(1);
  for (size_t i = 0; i < nd; ++i) {
    DevicePipeline& d = *devs_[(start + i) % nd];
    if (d.healthy()) return d;
  }
  throw ZkpError(ZKP_ERR_DEVICE, "every device of this prover has failed");
}

Prover::~Prover() = default;

// a HIP error on one pipeline retires every pipeline of its device: the error may be sticky
// device state that the ZKP_INFLIGHT siblings share
// (a logical device = one entry of the device list and its inflight_ pipelines)
void Prover::retire_device(const DevicePipeline& failed) {
  size_t at = 0;
  while (at < devs_.size() && devs_[at].get() != &failed) ++at;
  const size_t first = at / inflight_ * inflight_;
  for (size_t i = first; i < first + inflight_ && i < devs_.size(); ++i) devs_[i]->mark_failed();
}

// snarkjs groth16_prove's blinding, in two phases: everything but piH
// (assemble_pre: runs while the H MSM is still on the device) and C + piH + the encoding.
struct Blinded {
  Jac<HFq> Cpart;  // piC' + s A + r B1 - (r s) delta1
  Affine<HFq> a;   // A and B are final here: converted to affine before piH exists
  Affine<HFq2> b;
};
static Blinded assemble_pre(const ZkeyHeader& h, const DevicePipeline::MsmOut& m, const uint8_t* r32,
                            const uint8_t* s32) {
  const U256 r = scalar_or_random(r32), s = scalar_or_random(s32);
  const Jac<HFq> alpha1 = host::jac_from_aff(h.alpha1), beta1 = host::jac_from_aff(h.beta1),
                 delta1 = host::jac_from_aff(h.delta1);
  const Jac<HFq2> beta2 = host::jac_from_aff(h.beta2), delta2 = host::jac_from_aff(h.delta2);
  Blinded o;
  // A = piA' + alpha1 + r delta1
  const Jac<HFq> A = host::jac_add(host::jac_add(m.a, alpha1), host::jac_mul(delta1, r));
  // B = piB' + beta2 + s delta2 ; B1 = piB1' + beta1 + s delta1
  const Jac<HFq2> B = host::jac_add(host::jac_add(m.b2, beta2), host::jac_mul(delta2, s));
  Jac<HFq> B1 = host::jac_add(host::jac_add(m.b1, beta1), host::jac_mul(delta1, s));
  // C = piC' + piH + s A + r B1 - (r s) delta1
  HFr rs = HFr::from_std(r) * HFr::from_std(s);
  U256 nrs = rs.neg().to_std();
  Jac<HFq> C = m.c;
  C = host::jac_add(C, host::jac_mul(A, s));
  C = host::jac_add(C, host::jac_mul(B1, r));
  o.Cpart = host::jac_add(C, host::jac_mul(delta1, nrs));
  o.a = host::jac_to_aff(A);
  o.b = host::jac_to_aff(B);
  return o;
}
static void assemble_post(const ZkeyHeader& h, const Blinded& bl, const Jac<HFq>& piH, const WtnsView& w,
                          zkp_proof* out) {
  const Affine<HFq>& a = bl.a;
  const Affine<HFq2>& b = bl.b;
  auto c = host::jac_to_aff(host::jac_add(bl.Cpart, piH));
  put_fq(a.x, out->pi_a[0]);
  put_fq(a.y, out->pi_a[1]);
  put_fq(b.x.c0, out->pi_b[0][0]);
  put_fq(b.x.c1, out->pi_b[0][1]);
  put_fq(b.y.c0, out->pi_b[1][0]);
  put_fq(b.y.c1, out->pi_b[1][1]);
  put_fq(c.x, out->pi_c[0]);
  put_fq(c.y, out->pi_c[1]);
  out->n_public = h.n_public;
  if (out->public_signals && out->public_capacity)
    std::memcpy(out->public_signals, w.values + 32, (size_t)std::min(h.n_public, out->public_capacity) * 32);
}
static void assemble(const ZkeyHeader& h, const DevicePipeline::MsmOut& m, const WtnsView& w, const uint8_t* r32,
                     const uint8_t* s32, zkp_proof* out) {
  assemble_post(h, assemble_pre(h, m, r32, s32), m.h, w, out);
}

// test hook ZKP_TEST_CORRUPT_H: the H MSM result off by one generator, as a silent device error would
static Jac<HFq> maybe_corrupt(const Jac<HFq>& h, bool on) {
  if (!on) return h;
  const Affine<HFq> g{HFq::one(), HFq::one() + HFq::one(), false};  // (1, 2)
  return host::jac_add(h, host::jac_from_aff(g));
}

float Prover::verify_or_throw(const WtnsView& w, const zkp_proof* out) const {
  const auto t0 = std::chrono::steady_clock::now();
  if (hdr_.ic.size() != (size_t)hdr_.n_public + 1)
    throw ZkpError(ZKP_ERR_FORMAT, "verify: the zkey has no IC section (nPublic + 1 points)");
  host::VerifyingKey vk;
  vk.alpha1 = hdr_.alpha1;
  vk.beta2 = hdr_.beta2;
  vk.gamma2 = hdr_.gamma2;
  vk.delta2 = hdr_.delta2;
  vk.ic = hdr_.ic.data();
  vk.n_public = (int)hdr_.n_public;
  std::vector<U256> pub(hdr_.n_public);
  for (uint32_t i = 0; i < hdr_.n_public; ++i) pub[i] = host::u256_from_le(w.values + 32 * (size_t)(i + 1));
  auto fq = [](const uint8_t* b) { return HFq::from_std(host::u256_from_le(b)); };
  const Affine<HFq> a{fq(out->pi_a[0]), fq(out->pi_a[1]), false};
  const Affine<HFq2> b{HFq2{fq(out->pi_b[0][0]), fq(out->pi_b[0][1])}, HFq2{fq(out->pi_b[1][0]), fq(out->pi_b[1][1])},
                       false};
  const Affine<HFq> c{fq(out->pi_c[0]), fq(out->pi_c[1]), false};
  if (!host::groth16_verify(vk, pub.data(), a, b, c))
    throw ZkpError(ZKP_ERR_INTERNAL,
                   "proof failed verify-before-return (pairing check against the zkey's verification key): not "
                   "returned; the device result is suspect");
  return std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

static WtnsView check_wtns(const ZkeyHeader& h, const uint8_t* wtns, size_t len) {
  WtnsView w = parse_wtns(wtns, len);
  if (w.n_witness != h.n_vars)
    throw ZkpError(ZKP_ERR_WITNESS_LENGTH, "Invalid witness length. Circuit: " + std::to_string(h.n_vars) +
                                               ", witness: " + std::to_string(w.n_witness));
  return w;
}

static void jac_to_bytes_g1(const Jac<HFq>& p, uint8_t* out) {
  std::memset(out, 0, 64);
  auto a = host::jac_to_aff(p);
  if (!a.inf) put_fq(a.x, out), put_fq(a.y, out + 32);
}
static void jac_to_bytes_g2(const Jac<HFq2>& p, uint8_t* out) {
  std::memset(out, 0, 128);
  auto a = host::jac_to_aff(p);
  if (!a.inf) put_fq(a.x.c0, out), put_fq(a.x.c1, out + 32), put_fq(a.y.c0, out + 64), put_fq(a.y.c1, out + 96);
}
static bool all_zero(const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (p[i]) return false;
  return true;
}
static HFq fq_from_std_bytes(const uint8_t* p) {
  U256 v = host::u256_from_le(p);
  if (host::u256_geq(v, host::FQ_DESC.mod)) throw ZkpError(ZKP_ERR_INVALID_ARG, "partial: coordinate out of range");
  return HFq::from_std(v);
}
static Jac<HFq> g1_from_bytes(const uint8_t* p) {
  if (all_zero(p, 64)) return Jac<HFq>::inf();
  return host::jac_from_aff(Affine<HFq>{fq_from_std_bytes(p), fq_from_std_bytes(p + 32), false});
}
static Jac<HFq2> g2_from_bytes(const uint8_t* p) {
  if (all_zero(p, 128)) return Jac<HFq2>::inf();
  return host::jac_from_aff(Affine<HFq2>{HFq2{fq_from_std_bytes(p), fq_from_std_bytes(p + 32)},
                                         HFq2{fq_from_std_bytes(p + 64), fq_from_std_bytes(p + 96)}, false});
}
static void msm_out_to_partial(const DevicePipeline::MsmOut& m, int part, int nparts, zkp_partial* out) {
  jac_to_bytes_g1(m.a, out->a);
  jac_to_bytes_g1(m.b1, out->b1);
  jac_to_bytes_g1(m.c, out->c);
  jac_to_bytes_g1(m.h, out->h);
  jac_to_bytes_g2(m.b2, out->b2);
  out->part = (uint32_t)part;
  out->nparts = (uint32_t)nparts;
}

void Prover::require_full() const {
  if (nparts_ != 1)
    throw ZkpError(ZKP_ERR_INVALID_ARG, "this prover holds one point range (part " + std::to_string(part_) + " of " +
                                            std::to_string(nparts_) + "): use zkp_prove_partial + zkp_proof_combine");
}

void Prover::prove_partial(const uint8_t* wtns, size_t len, zkp_partial* out) {
  WtnsView w = check_wtns(hdr_, wtns, len);
  DevicePipeline::MsmOut m = devs_[0]->prove(w);
  msm_out_to_partial(m, part_, nparts_, out);
  std::lock_guard<std::mutex> lk(tmu_);
  for (int i = 0; i < 5; ++i) last_ms_[i] = m.ms[i];
  last_ms_[7] = m.ms[5];
  last_ms_[9] = m.pcie_mb;
  last_ms_[10] = (float)m.wset;
}

void Prover::prove_partial_staged(int slot, zkp_partial* out) {
  DevicePipeline::MsmOut m = devs_[0]->prove_staged(slot);
  msm_out_to_partial(m, part_, nparts_, out);
  std::lock_guard<std::mutex> lk(tmu_);
  for (int i = 0; i < 5; ++i) last_ms_[i] = m.ms[i];
  last_ms_[7] = m.ms[5];
  last_ms_[9] = m.pcie_mb;
  last_ms_[10] = (float)m.wset;
}

void Prover::quotient_part_staged(int slot, int mask, void* const* dst) {
  if (mask < 0 || mask > 7) throw ZkpError(ZKP_ERR_INVALID_ARG, "quotient part: mask must be within 0..7");
  devs_[0]->quotient_part_staged(slot, mask, dst);
}

void Prover::prove_partial_ext_staged(int slot, const void* const* abc, zkp_partial* out) {
  DevicePipeline::MsmOut m = devs_[0]->prove_ext_staged(slot, abc);
  msm_out_to_partial(m, part_, nparts_, out);
  std::lock_guard<std::mutex> lk(tmu_);
  for (int i = 0; i < 5; ++i) last_ms_[i] = m.ms[i];
  last_ms_[7] = m.ms[5];
  last_ms_[9] = m.pcie_mb;
  last_ms_[10] = (float)m.wset;
}

void proof_combine(const uint8_t* zkey, size_t len, const zkp_partial* parts, int nparts, const uint8_t* wtns,
                   size_t wlen, const uint8_t* r32, const uint8_t* s32, zkp_proof* out) {
  if (nparts < 1) throw ZkpError(ZKP_ERR_INVALID_ARG, "no partials");
  ZkeyParsed z = parse_zkey(zkey, len, false);
  WtnsView w = check_wtns(z.hdr, wtns, wlen);
  std::vector<int> seen(nparts, 0);
  DevicePipeline::MsmOut m;
  m.a = m.b1 = m.c = m.h = Jac<HFq>::inf();
  m.b2 = Jac<HFq2>::inf();
  for (int i = 0; i < nparts; ++i) {
    const zkp_partial& p = parts[i];
    if ((int)p.nparts != nparts || p.part >= p.nparts || seen[p.part]++)
      throw ZkpError(ZKP_ERR_INVALID_ARG, "partials must be parts 0..nparts-1 of one split, each exactly once");
    m.a = host::jac_add(m.a, g1_from_bytes(p.a));
    m.b1 = host::jac_add(m.b1, g1_from_bytes(p.b1));
    m.c = host::jac_add(m.c, g1_from_bytes(p.c));
    m.h = host::jac_add(m.h, g1_from_bytes(p.h));
    m.b2 = host::jac_add(m.b2, g2_from_bytes(p.b2));
  }
  assemble(z.hdr, m, w, r32, s32, out);
}

void Prover::prove(const uint8_t* wtns, size_t len, const uint8_t* r32, const uint8_t* s32, zkp_proof* out) {
  require_full();
  auto t0 = std::chrono::steady_clock::now();
  WtnsView w = check_wtns(hdr_, wtns, len);
  DevicePipeline& d = pick_device();
  DevicePipeline::MsmOut m;
  Blinded bl;
  try {
    m = d.prove(w, [&](const DevicePipeline::MsmOut& o) { bl = assemble_pre(hdr_, o, r32, s32); });
  } catch (const HipError&) {
    retire_device(d);
    throw;
  }
  auto t1 = std::chrono::steady_clock::now();
  assemble_post(hdr_, bl, maybe_corrupt(m.h, corrupt_h_ == 1), w, out);
  auto t2 = std::chrono::steady_clock::now();
  const float vms = verify() ? verify_or_throw(w, out) : 0.f;
  std::lock_guard<std::mutex> lk(tmu_);
  for (int i = 0; i < 5; ++i) last_ms_[i] = m.ms[i];
  last_ms_[7] = m.ms[5];
  last_ms_[9] = m.pcie_mb;
  last_ms_[10] = (float)m.wset;
  last_ms_[5] = std::chrono::duration<float, std::milli>(t2 - t1).count();
  last_ms_[6] = std::chrono::duration<float, std::milli>(t2 - t0).count();
  last_ms_[8] = vms;
}

// Batch scheduler: a shared queue of witness indices; two
// worker threads per device pipeline (one uploads the next witness into a free upload slot
// while the other's proof computes), per-proof status, and re-queue on device failure: a
// worker whose device raises a HIP error puts its witness back at the head of the queue
// and retires the device; the other devices finish the batch.  A witness that is itself
// invalid (format, length, curve) fails alone.
zkp_status Prover::prove_batch(const uint8_t* const* wtns, const size_t* lens, int n, const uint8_t* const* r32s,
                               const uint8_t* const* s32s, zkp_proof* outs, zkp_status* statuses,
                               std::string* first_error) {
  require_full();
  std::vector<zkp_status> st(n, ZKP_ERR_INTERNAL);
  std::vector<std::string> msg(n);
  std::mutex qm;
  std::condition_variable qcv;
  std::deque<int> q;
  for (int i = 0; i < n; ++i) q.push_back(i);
  int outstanding = n;
  const size_t nd = devs_.size();
  auto live_devices = [&] {
    size_t k = 0;
    for (auto& d : devs_) k += d->healthy() ? 1 : 0;
    return k;
  };
  auto finish = [&](int i, zkp_status s, const std::string& m) {
    std::lock_guard<std::mutex> lk(qm);
    st[i] = s;
    msg[i] = m;
    --outstanding;
    qcv.notify_all();
  };
  auto worker = [&](size_t di) {
    DevicePipeline& d = *devs_[di];
    for (;;) {
      int i;
      {
        std::unique_lock<std::mutex> lk(qm);
        qcv.wait(lk, [&] { return !q.empty() || outstanding == 0 || !d.healthy(); });
        if (q.empty() || !d.healthy()) return;
        i = q.front();
        q.pop_front();
      }
      WtnsView w;
      try {
        w = check_wtns(hdr_, wtns[i], lens[i]);
      } catch (const ZkpError& e) {
        finish(i, e.status, e.what());
        continue;
      }
      try {
        Blinded bl;
        DevicePipeline::MsmOut m = d.prove(w, [&](const DevicePipeline::MsmOut& o) {
          bl = assemble_pre(hdr_, o, r32s ? r32s[i] : nullptr, s32s ? s32s[i] : nullptr);
        });
        assemble_post(hdr_, bl, maybe_corrupt(m.h, corrupt_h_ == 1 || (corrupt_h_ == 2 && (i & 1))), w, &outs[i]);
        if (verify_batch()) verify_or_throw(w, &outs[i]);  // on the worker thread: overlaps the next proof
        finish(i, ZKP_OK, "");
      } catch (const HipError& e) {
        retire_device(d);  // every pipeline of that device (ZKP_INFLIGHT siblings share its state)
        std::lock_guard<std::mutex> lk(qm);
        if (live_devices() > 0) {
          q.push_front(i);  // re-queue on a healthy device
        } else {            // nothing left to run on: fail this and everything queued
          st[i] = ZKP_ERR_DEVICE;
          msg[i] = e.what();
          --outstanding;
          while (!q.empty()) {
            st[q.front()] = ZKP_ERR_DEVICE;
            msg[q.front()] = std::string("no healthy device left: ") + e.what();
            q.pop_front();
            --outstanding;
          }
        }
        qcv.notify_all();
        return;
      } catch (const ZkpError& e) {
        finish(i, e.status, e.what());
      } catch (const std::bad_alloc&) {
        finish(i, ZKP_ERR_OUT_OF_MEMORY, "host out of memory");
      } catch (const std::exception& e) {
        finish(i, ZKP_ERR_INTERNAL, e.what());
      }
    }
  };
  if (live_devices() == 0) {
    for (int i = 0; i < n; ++i) st[i] = ZKP_ERR_DEVICE, msg[i] = "every device of this prover has failed";
  } else {
    std::vector<std::thread> th;
    for (size_t di = 0; di < nd; ++di)
      for (int k = 0; k < 2; ++k) th.emplace_back(worker, di);
    for (auto& t : th) t.join();
  }
  zkp_status first = ZKP_OK;
  for (int i = 0; i < n; ++i) {
    if (statuses) statuses[i] = st[i];
    if (st[i] != ZKP_OK && first == ZKP_OK) {
      first = st[i];
      if (first_error) *first_error = "proof " + std::to_string(i) + ": " + msg[i];
    }
  }
  return first;
}

void Prover::quotient(const uint8_t* wtns, size_t len, uint8_t* out) {
  WtnsView w = check_wtns(hdr_, wtns, len);
  devs_[0]->quotient(w, out);
}

void Prover::timings(float* ms, int n) const {
  std::lock_guard<std::mutex> lk(tmu_);
  for (int i = 0; i < n && i < 11; ++i) ms[i] = last_ms_[i];
}

DevicePipeline& Prover::staged_pipeline(int dev_index) const {
  if (dev_index < 0 || dev_index >= ndevices_)
    throw ZkpError(ZKP_ERR_INVALID_ARG, "device index " + std::to_string(dev_index) + " out of range (the prover has " +
                                            std::to_string(ndevices_) + " devices)");
  return *devs_[(size_t)dev_index * inflight_];
}

void Prover::stage(int dev, int slot, const uint8_t* wtns, size_t len) {
  DevicePipeline& d = staged_pipeline(dev);
  WtnsView w = check_wtns(hdr_, wtns, len);
  auto ex = d.lock_stage();  // no staged proof of this device reads a slot or its public signals now
  d.stage(slot, w);
  std::lock_guard<std::mutex> lk(smu_);
  if (staged_pub_.size() < (size_t)ndevices_) staged_pub_.resize(ndevices_);
  auto& v = staged_pub_[dev];
  if ((size_t)slot >= v.size()) v.resize(slot + 1);
  v[slot].assign(w.values, w.values + (size_t)(hdr_.n_public + 1) * 32);
}

void Prover::prove_staged(int dev, int slot, const uint8_t* r32, const uint8_t* s32, zkp_proof* out) {
  require_full();
  DevicePipeline& base = staged_pipeline(dev);
  auto staged = base.hold_stage();  // the slot stays valid and unchanged until the proof is done
  const uint32_t* d_wit = base.slot_ptr(slot);
  const double large_frac = base.slot_large(slot);
  // concurrent staged callers on one device take its idle ZKP_INFLIGHT pipelines (the staged
  // witnesses live in the first one; the others read them in place); with none idle the call
  // queues on the first pipeline
  DevicePipeline* d = &base;
  bool claimed = false;
  for (int k = 0; k < inflight_ && !claimed; ++k) {
    DevicePipeline* c = devs_[(size_t)dev * inflight_ + k].get();
    bool idle = false;
    if (c->staged_busy.compare_exchange_strong(idle, true)) d = c, claimed = true;
  }
  struct Release {
    DevicePipeline* d;
    bool on;
    ~Release() {
      if (on) d->staged_busy.store(false);
    }
  } release{d, claimed};
  auto t0 = std::chrono::steady_clock::now();
  Blinded bl;
  DevicePipeline::MsmOut m = d->prove_resident(
      d_wit, [&](const DevicePipeline::MsmOut& o) { bl = assemble_pre(hdr_, o, r32, s32); }, large_frac);
  auto t1 = std::chrono::steady_clock::now();
  WtnsView w;
  {
    std::lock_guard<std::mutex> lk(smu_);
    w.values = staged_pub_[dev][slot].data();
    w.n_witness = hdr_.n_vars;
  }
  assemble_post(hdr_, bl, maybe_corrupt(m.h, corrupt_h_ == 1), w, out);
  auto t2 = std::chrono::steady_clock::now();
  const float vms = verify() ? verify_or_throw(w, out) : 0.f;
  std::lock_guard<std::mutex> lk(tmu_);
  for (int i = 0; i < 5; ++i) last_ms_[i] = m.ms[i];
  last_ms_[7] = m.ms[5];
  last_ms_[9] = m.pcie_mb;
  last_ms_[10] = (float)m.wset;
  last_ms_[5] = std::chrono::duration<float, std::milli>(t2 - t1).count();
  last_ms_[6] = std::chrono::duration<float, std::milli>(t2 - t0).count();
  last_ms_[8] = vms;
}

void Prover::set_instrument(bool on) {
  for (auto& d : devs_) d->set_instrument(on);
}

void Prover::msm_config(double* out, int n) const {
  MsmParams pw, ph, pw2;
  devs_[0]->msm_params(pw, ph, &pw2);
  const bool two = devs_[0]->witness_sets() > 1;
  const double v[10] = {(double)pw.c, (double)pw.depth, (double)pw.groups, (double)ph.c,
                        (double)ph.depth, (double)ph.groups, (double)devs_[0]->table_bytes(),
                        two ? (double)pw2.c : 0.0, two ? (double)pw2.depth : 0.0, two ? (double)pw2.groups : 0.0};
  for (int i = 0; i < n && i < 10; ++i) out[i] = v[i];
}

void Prover::kernel_stats(double* out, int n) const {
  MsmEngine::Stats a{}, b{};
  for (auto& d : devs_) {
    MsmEngine::Stats x, y;
    d->stats(x, y);
    a.accumulate_ms += x.accumulate_ms, a.launches += x.launches, a.mixed_adds += x.mixed_adds, a.tasks += x.tasks;
    b.accumulate_ms += y.accumulate_ms, b.launches += y.launches, b.mixed_adds += y.mixed_adds, b.tasks += y.tasks;
  }
  const double v[8] = {a.accumulate_ms, (double)a.launches, (double)a.mixed_adds, (double)a.tasks,
                       b.accumulate_ms, (double)b.launches, (double)b.mixed_adds, (double)b.tasks};
  for (int i = 0; i < n && i < 8; ++i) out[i] = v[i];
}

int Prover::launch_records(double* out, int max_records) const {
  std::vector<std::array<double, 4>> all;
  for (auto& d : devs_) d->launch_records(all);
  const int n = (int)std::min<size_t>(all.size(), (size_t)std::max(0, max_records));
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < 4; ++j) out[4 * i + j] = all[i][j];
  return (int)all.size();
}

// ------------------------------------------------------------------ kernel-level helpers

// One device-resident MSM set-up for the kernel-level entry points: base table from
// zkey-layout points (row 0 uploaded + converted, rows 1..T-1 derived), a plan and an engine.
struct MsmRig {
  hipStream_t st = nullptr;
  MsmParams prm;
  std::unique_ptr<MsmBases> bases;
  std::unique_ptr<MsmPlan> plan;
  std::unique_ptr<MsmEngine> eng;
  uint32_t *ds = nullptr, *dw = nullptr;
  size_t n;
  Curve curve;
  float table_ms = 0;  // base-table build: row 0 upload + conversion + the derived rows (HIP events)
  MsmRig(int device, Curve cv, const uint8_t* points, const uint8_t* scalars, size_t n_, int c, int depth)
      : n(n_), curve(cv) {
    HIPX(hipSetDevice(device));
    HIPX(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    try {
      // automatic window bits and plan: the prover's H-MSM choice (dense plan, c = lg n - 3 clamped to
      // [8, 20] and moved off a collapsed top window); measured on configs[1] (G1 2^20, uniform
      // scalars, 273c6e8:tools/gpu/experiments/r2_msm_c.sh): 1.84 ms against 2.06 ms for a compacted plan at
      // c = lg n - 4.  ZKP_MSM plan=compact selects the witness plan's variant (tests).
      int lg = 0;
      while ((size_t(1) << lg) < n) ++lg;
      const MsmOptions opt = msm_options();
      const int c_auto = opt.h ? opt.h : dense_window_bits(std::min(20, std::max(8, lg - 3)), n);
      prm = make_params(std::max<size_t>(n, 1), c ? c : c_auto, depth);
      prm.S = opt.task_h > 0 ? opt.task_h : 48;  // the H plan's task size too (choose_msm_params)
      bases = std::make_unique<MsmBases>(curve, n, prm.c, prm.depth);
      hipEvent_t t0, t1;
      HIPX(hipEventCreate(&t0));
      HIPX(hipEventCreate(&t1));
      HIPX(hipEventRecord(t0, st));
      fill_bases(*bases, points, n, 0, st);
      HIPX(hipEventRecord(t1, st));
      HIPX(hipEventSynchronize(t1));
      HIPX(hipEventElapsedTime(&table_ms, t0, t1));
      (void)hipEventDestroy(t0), (void)hipEventDestroy(t1);
      plan = std::make_unique<MsmPlan>(std::max<size_t>(n, 1), prm, st);
      plan->set_dense(opt.dense != 0);
      eng = std::make_unique<MsmEngine>(curve, prm, std::max<size_t>(n, 1), st);
      HIPX(hipMalloc(&ds, std::max<size_t>(n * 32, 32)));
      HIPX(hipMalloc(&dw, eng->window_words() * 4));
      if (n) HIPX(hipMemcpyAsync(ds, scalars, n * 32, hipMemcpyHostToDevice, st));
    } catch (...) {
      release();
      throw;
    }
  }
  void run() {
    plan->build(ds, n);
    eng->run(*plan, *bases, dw);
  }
  // fold the group sums and write the affine result (standard-form LE)
  void result(uint8_t* out, int* is_inf) {
    std::vector<uint32_t> hw(eng->window_words());
    HIPX(hipMemcpyAsync(hw.data(), dw, hw.size() * 4, hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));
    if (curve == Curve::G1) {
      auto a = host::jac_to_aff(msm_fold<HFq>(hw.data(), prm));
      *is_inf = a.inf ? 1 : 0;
      std::memset(out, 0, 64);
      if (!a.inf) {
        put_fq(a.x, out);
        put_fq(a.y, out + 32);
      }
    } else {
      auto a = host::jac_to_aff(msm_fold<HFq2>(hw.data(), prm));
      *is_inf = a.inf ? 1 : 0;
      std::memset(out, 0, 128);
      if (!a.inf) {
        put_fq(a.x.c0, out);
        put_fq(a.x.c1, out + 32);
        put_fq(a.y.c0, out + 64);
        put_fq(a.y.c1, out + 96);
      }
    }
  }
  void release() {
    if (st) (void)hipStreamSynchronize(st);
    eng.reset();
    plan.reset();
    bases.reset();
    for (void* p : {(void*)ds, (void*)dw})
      if (p) (void)hipFree(p);
    ds = dw = nullptr;
    if (st) (void)hipStreamDestroy(st);
    st = nullptr;
  }
  ~MsmRig() { release(); }
};

void msm_points(int device, Curve curve, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out,
                int* is_inf, int c, int depth) {
  MsmRig rig(device, curve, points, scalars, n, c, depth);
  rig.run();
  rig.result(out, is_inf);
}

MsmBench bench_msm(int device, Curve curve, const uint8_t* points, const uint8_t* scalars, size_t n, int warmup,
                   int iters, uint8_t* out, int* is_inf) {
  if (n == 0 || iters <= 0) throw ZkpError(ZKP_ERR_INVALID_ARG, "bench_msm: n and iters must be > 0");
  MsmRig rig(device, curve, points, scalars, n, 0, 0);
  hipEvent_t e0, e1;
  HIPX(hipEventCreate(&e0));
  HIPX(hipEventCreate(&e1));
  MsmBench r;
  try {
    for (int i = 0; i < warmup; ++i) rig.run();
    HIPX(hipStreamSynchronize(rig.st));
    // pass 1: whole-pipeline time (plan + engine), host-blocking once per MSM as in a proof
    HIPX(hipEventRecord(e0, rig.st));
    for (int i = 0; i < iters; ++i) rig.run();
    HIPX(hipEventRecord(e1, rig.st));
    HIPX(hipEventSynchronize(e1));
    float ms = 0;
    HIPX(hipEventElapsedTime(&ms, e0, e1));
    r.ms_per_msm = ms / iters;
    // pass 2: per-launch events around the bucket-accumulate kernel
    rig.eng->set_instrument(true);
    MsmEngine::Stats s;
    for (int i = 0; i < std::min(iters, 8); ++i) rig.run();
    HIPX(hipStreamSynchronize(rig.st));
    rig.eng->collect(s);
    r.ms_accumulate = (float)(s.accumulate_ms / std::max<uint64_t>(1, s.launches));
    r.mixed_adds = s.mixed_adds / std::max<uint64_t>(1, s.launches);
    r.tasks = s.tasks / std::max<uint64_t>(1, s.launches);
    r.c = rig.prm.c;
    r.windows = rig.prm.windows;
    r.depth = rig.prm.depth;
    r.table_ms = rig.table_ms;
    if (out && is_inf) rig.result(out, is_inf);
  } catch (...) {
    (void)hipEventDestroy(e0), (void)hipEventDestroy(e1);
    throw;
  }
  (void)hipEventDestroy(e0), (void)hipEventDestroy(e1);
  return r;
}

float bench_plan(int device, const uint8_t* scalars, size_t n, int c, int dense, int warmup, int iters) {
  if (n == 0 || iters <= 0) throw ZkpError(ZKP_ERR_INVALID_ARG, "bench_plan: n and iters must be > 0");
  HIPX(hipSetDevice(device));
  hipStream_t st;
  HIPX(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t* d = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float ms = 0;
  try {
    HIPX(hipEventCreate(&e0));
    HIPX(hipEventCreate(&e1));
    const MsmParams prm = make_params(n, c, 0);
    MsmPlan plan(n, prm, st);
    plan.set_dense(dense != 0);
    HIPX(hipMalloc(&d, n * 32));
    HIPX(hipMemcpyAsync(d, scalars, n * 32, hipMemcpyHostToDevice, st));
    for (int i = 0; i < warmup; ++i) plan.build(d, n);
    HIPX(hipStreamSynchronize(st));
    HIPX(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) plan.build(d, n);
    HIPX(hipEventRecord(e1, st));
    HIPX(hipEventSynchronize(e1));
    HIPX(hipEventElapsedTime(&ms, e0, e1));
  } catch (...) {
    if (d) (void)hipFree(d);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(st);
    throw;
  }
  HIPX(hipFree(d));
  (void)hipEventDestroy(e0), (void)hipEventDestroy(e1);
  HIPX(hipStreamDestroy(st));
  return ms / iters;
}

float bench_ntt(int device, int log_n, int count, int warmup, int iters) {
  if (iters <= 0) throw ZkpError(ZKP_ERR_INVALID_ARG, "bench_ntt: iters must be > 0");
  if (count < 1 || count > 3) throw ZkpError(ZKP_ERR_INVALID_ARG, "bench_ntt: 1..3 vectors");
  if (log_n < 0 || log_n > 27) throw ZkpError(ZKP_ERR_INVALID_ARG, "bench_ntt: log_n out of range");
  HIPX(hipSetDevice(device));
  hipStream_t st;
  HIPX(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t n = size_t(1) << log_n;
  uint32_t* d = nullptr;
  hipEvent_t e0, e1;
  HIPX(hipEventCreate(&e0));
  HIPX(hipEventCreate(&e1));
  float ms = 0;
  try {
    NttEngine eng(log_n, st);
    HIPX(hipMalloc(&d, n * 32 * count));
    std::vector<uint32_t> seed(n * 8);
    uint64_t x = 0x5A4B5032;
    for (auto& v : seed) {  // uniform-ish Fr-sized values
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      v = (uint32_t)(x >> 32);
    }
    for (size_t i = 0; i < n; ++i) seed[i * 8 + 7] &= 0x0fffffffu;
    uint32_t* vecs[3];
    for (int v = 0; v < count; ++v) {
      vecs[v] = d + (size_t)v * n * 8;
      HIPX(hipMemcpyAsync(vecs[v], seed.data(), n * 32, hipMemcpyHostToDevice, st));
    }
    HIPX(hipStreamSynchronize(st));  // seed is released at the end of the scope
    for (int i = 0; i < warmup; ++i) eng.coset_extend_batch(vecs, count);
    HIPX(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) eng.coset_extend_batch(vecs, count);
    HIPX(hipEventRecord(e1, st));
    HIPX(hipEventSynchronize(e1));
    HIPX(hipEventElapsedTime(&ms, e0, e1));
  } catch (...) {
    if (d) (void)hipFree(d);
    (void)hipEventDestroy(e0), (void)hipEventDestroy(e1), (void)hipStreamDestroy(st);
    throw;
  }
  HIPX(hipFree(d));
  (void)hipEventDestroy(e0), (void)hipEventDestroy(e1);
  HIPX(hipStreamDestroy(st));
  return ms / iters;
}

void ntt_fr(int device, uint8_t* data, size_t n, int mode) {
  if (n == 0 || (n & (n - 1))) throw ZkpError(ZKP_ERR_INVALID_ARG, "NTT size must be a power of two");
  int k = 0;
  while ((size_t(1) << k) < n) ++k;
  HIPX(hipSetDevice(device));
  hipStream_t st;
  HIPX(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t* d = nullptr;
  try {
    NttEngine eng(k, st);
    HIPX(hipMalloc(&d, n * 32));
    HIPX(hipMemcpyAsync(d, data, n * 32, hipMemcpyHostToDevice, st));
    launch_fr_to_dev(d, n, st);
    if (mode == 0)
      eng.forward(d);
    else if (mode == 1)
      eng.inverse(d);
    else
      eng.coset_extend(d);
    launch_fr_from_dev(d, n, st);
    HIPX(hipMemcpyAsync(data, d, n * 32, hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));
  } catch (...) {
    if (d) (void)hipFree(d);
    (void)hipStreamDestroy(st);
    throw;
  }
  HIPX(hipFree(d));
  HIPX(hipStreamDestroy(st));
}

}  // namespace zkp
