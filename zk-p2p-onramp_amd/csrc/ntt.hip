// Fr NTT engine (see ntt.hpp for the algorithm).
#include "ntt.hpp"

#include <stdexcept>

#include "field.hpp"
#include "hip_check.hpp"
#include "host_ec.hpp"

namespace zkp {

namespace {

constexpr int TPB = 256;
constexpr int LOG_TILE = 10;  // elements per workgroup tile (n1 * C = 1024, 36 KiB of LDS)
constexpr int LOC_LOG = 10;   // local-root table: w_1024^e, e < 512
constexpr int MAX_PASS_BITS = 8;

__device__ __forceinline__ uint32_t brev(uint32_t x, int b) { return __builtin_bitreverse32(x) >> (32 - b); }

// w_n^E from the two-level table, E < n
__device__ __forceinline__ Fr tw_pow(const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi, uint32_t E,
                                     int h) {
  Fr a = load_fe<FrCfg>(lo + (size_t)(E & ((1u << h) - 1)) * 8);
  Fr b = load_fe<FrCfg>(hi + (size_t)(E >> h) * 8);
  return mul(a, b);
}

// One pass over blocks of size 2^lm: n1 = 2^b point DFTs over the strided index,
// tile = 2^lc consecutive columns.  dit: twiddle before the DFT, else after.
__global__ __launch_bounds__(TPB) void k_ntt_pass(uint32_t* __restrict__ data, int k, int lm, int b, int lc, int dit,
                                                  const uint32_t* __restrict__ loc,
                                                  const uint32_t* __restrict__ tw_lo,
                                                  const uint32_t* __restrict__ tw_hi, int h) {
  __shared__ uint32_t lds[NL << LOG_TILE];  // SoA: lds[limb * E + element]
  const int E = 1 << (b + lc);
  const int C = 1 << lc;
  const uint32_t n2 = 1u << (lm - b);
  const uint32_t tiles_per_block = n2 >> lc;
  const uint32_t tile = blockIdx.x;
  const uint32_t blk = tile / tiles_per_block;
  const uint32_t col0 = (tile - blk * tiles_per_block) << lc;
  const size_t base = (size_t)blk << lm;
  const int tw_shift = k - lm;  // w_m^e = w_n^(e << (k - lm))

  for (int e = threadIdx.x; e < E; e += TPB) {
    const uint32_t row = (uint32_t)e >> lc, col = (uint32_t)e & (C - 1);
    const size_t g = base + (size_t)row * n2 + col0 + col;
    Fr x = load_fe<FrCfg>(data + g * 8);
    if (dit) {
      const uint32_t ex = (col0 + col) * row;
      if (ex) x = mul(x, tw_pow(tw_lo, tw_hi, ex << tw_shift, h));
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) lds[l * E + e] = x.v[l];
  }
  __syncthreads();
  for (int t = 0; t < b; ++t) {
    const int lhalf = b - 1 - t;
    for (int q = threadIdx.x; q < (E >> 1); q += TPB) {
      const uint32_t col = (uint32_t)q & (C - 1), bq = (uint32_t)q >> lc;
      const uint32_t grp = bq >> lhalf, i = bq & ((1u << lhalf) - 1);
      const uint32_t r0 = (grp << (lhalf + 1)) + i, r1 = r0 + (1u << lhalf);
      const int e0 = (int)((r0 << lc) + col), e1 = (int)((r1 << lc) + col);
      Fr x, y;
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        x.v[l] = lds[l * E + e0];
        y.v[l] = lds[l * E + e1];
      }
      Fr s = add(x, y);
      // x - y only feeds the twiddle multiply when i != 0: raw (unnormalised) subtraction
      Fr d = i ? mul(rsub(x, y), load_fe<FrCfg>(loc + (size_t)(i << (t + LOC_LOG - b)) * 8)) : sub(x, y);
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        lds[l * E + e0] = s.v[l];
        lds[l * E + e1] = d.v[l];
      }
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < E; e += TPB) {
    const uint32_t k1 = (uint32_t)e >> lc, col = (uint32_t)e & (C - 1);
    const int src = (int)((brev(k1, b) << lc) + col);
    Fr x;
#pragma unroll
    for (int l = 0; l < NL; ++l) x.v[l] = lds[l * E + src];
    if (!dit) {
      const uint32_t ex = (col0 + col) * k1;
      if (ex) x = mul(x, tw_pow(tw_lo, tw_hi, ex << tw_shift, h));
    }
    const size_t g = base + (size_t)k1 * n2 + col0 + col;
    store_fe(data + g * 8, x);
  }
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

// mode 0: x * g^f(pos) / n ; mode 1: x / n
__global__ __launch_bounds__(TPB) void k_scale(uint32_t* __restrict__ data, int k, PassBits pb, int mode,
                                               const uint32_t* __restrict__ c_lo, const uint32_t* __restrict__ c_hi,
                                               int h, const uint32_t* __restrict__ ninv) {
  const uint32_t pos = blockIdx.x * TPB + threadIdx.x;
  if (pos >= (1u << k)) return;
  Fr x = load_fe<FrCfg>(data + (size_t)pos * 8);
  if (mode == 0) {
    const uint32_t f = freq_of(pos, k, pb);
    x = mul(x, tw_pow(c_lo, c_hi, f, h));
  } else {
    x = mul(x, load_fe<FrCfg>(ninv));
  }
  store_fe(data + (size_t)pos * 8, x);
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
}

NttEngine::~NttEngine() {
  for (uint32_t* p : {tw_lo_[0], tw_lo_[1], tw_hi_[0], tw_hi_[1], loc_[0], loc_[1], coset_lo_, coset_hi_, ninv_,
                      scratch_})
    if (p) (void)hipFree(p);
}

void NttEngine::dif_passes(uint32_t* data, bool inv) {
  const int k = log_n_;
  int lm = k;
  for (int b : bits_) {
    const int lc = std::min(LOG_TILE - b, lm - b);
    const size_t tiles = (size_t(1) << k) >> (b + lc);
    hipLaunchKernelGGL(k_ntt_pass, dim3((unsigned)tiles), dim3(TPB), 0, stream_, data, k, lm, b, lc, 0,
                       loc_[inv ? 1 : 0], tw_lo_[inv ? 1 : 0], tw_hi_[inv ? 1 : 0], h_);
    lm -= b;
  }
}

void NttEngine::dit_passes(uint32_t* data, bool inv) {
  const int k = log_n_;
  // transposed passes in reverse order: block sizes grow back from the innermost
  std::vector<int> lms;
  int lm = k;
  for (int b : bits_) {
    lms.push_back(lm);
    lm -= b;
  }
  for (int i = (int)bits_.size() - 1; i >= 0; --i) {
    const int b = bits_[i], lmi = lms[i];
    const int lc = std::min(LOG_TILE - b, lmi - b);
    const size_t tiles = (size_t(1) << k) >> (b + lc);
    hipLaunchKernelGGL(k_ntt_pass, dim3((unsigned)tiles), dim3(TPB), 0, stream_, data, k, lmi, b, lc, 1,
                       loc_[inv ? 1 : 0], tw_lo_[inv ? 1 : 0], tw_hi_[inv ? 1 : 0], h_);
  }
}

static PassBits make_pb(const std::vector<int>& bits) {
  PassBits pb{};
  pb.n = (int)bits.size();
  for (int i = 0; i < pb.n; ++i) pb.b[i] = bits[i];
  return pb;
}

void NttEngine::scale(uint32_t* data, int mode) {
  const size_t n = size_t(1) << log_n_;
  hipLaunchKernelGGL(k_scale, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, stream_, data, log_n_,
                     make_pb(bits_), mode, coset_lo_, coset_hi_, h_, ninv_);
}

void NttEngine::digit_reverse(uint32_t* data, bool to_natural) {
  const size_t n = size_t(1) << log_n_;
  if (!scratch_) HIPX(hipMalloc(&scratch_, n * 32));
  HIPX(hipMemcpyAsync(scratch_, data, n * 32, hipMemcpyDeviceToDevice, stream_));
  hipLaunchKernelGGL(k_digit_reverse, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, stream_, scratch_, data,
                     log_n_, make_pb(bits_), to_natural ? 1 : 0);
}

void NttEngine::coset_extend(uint32_t* data) {
  if (log_n_ == 0) {
    // n = 1: coefficient = value; evaluation at g is the same constant
    return;
  }
  dif_passes(data, true);
  scale(data, 0);
  dit_passes(data, false);
  HIPX(hipGetLastError());
}

void NttEngine::forward(uint32_t* data) {
  if (log_n_ == 0) return;
  dif_passes(data, false);
  digit_reverse(data, true);
  HIPX(hipGetLastError());
}

void NttEngine::inverse(uint32_t* data) {
  if (log_n_ == 0) return;
  dif_passes(data, true);
  scale(data, 1);
  digit_reverse(data, true);
  HIPX(hipGetLastError());
}

}  // namespace zkp
