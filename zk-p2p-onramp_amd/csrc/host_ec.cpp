// Host-side BN254 constants and conversions (see host_ec.hpp).
#include "host_ec.hpp"

namespace zkp {
namespace host {

// p = 21888242871839275222246405745257275088696311157297823662689037894645226208583 (Verifier.sol:52)
const FieldDesc FQ_DESC = {
    {{0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull}},
    0x87d20782e4866389ull,
    {{0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull, 0x47ab1eff0a417ff6ull, 0x06d89f71cab8351full}},
};
// r = 21888242871839275222246405745257275088548364400416034343698204186575808495617 (Verifier.sol:341)
const FieldDesc FR_DESC = {
    {{0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull}},
    0xc2e1f593efffffffull,
    {{0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull, 0x8c49833d53bb8085ull, 0x0216d0b17f4e44a5ull}},
};

U256 u256_from_le(const uint8_t* p) {
  U256 r;
  for (int i = 0; i < 4; ++i) {
    u64 v = 0;
    for (int b = 7; b >= 0; --b) v = (v << 8) | p[i * 8 + b];
    r.w[i] = v;
  }
  return r;
}

void u256_to_le(const U256& x, uint8_t* p) {
  for (int i = 0; i < 4; ++i)
    for (int b = 0; b < 8; ++b) p[i * 8 + b] = (uint8_t)(x.w[i] >> (8 * b));
}

static U256 words_to_u256(const uint32_t* w) {
  U256 r;
  for (int i = 0; i < 4; ++i) r.w[i] = (u64)w[2 * i] | ((u64)w[2 * i + 1] << 32);
  return r;
}

template <const FieldDesc& D>
static Fp<D> from_dev_impl(const uint32_t* w) {
  // x_dev = x * 2^261 (value < 2m).  Reduce, then mont_mul by 2^251 gives x * 2^256.
  U256 v = words_to_u256(w);
  while (u256_geq(v, D.mod)) u256_sub(v, D.mod);
  U256 k{{0, 0, 0, u64(1) << 59}};  // 2^251 (< m)
  return Fp<D>::mont_mul(v, k);
}

Fq fq_from_dev(const uint32_t* w) { return from_dev_impl<FQ_DESC>(w); }
Fr fr_from_dev(const uint32_t* w) { return from_dev_impl<FR_DESC>(w); }

std::string u256_to_dec(const U256& x) {
  U256 v = x;
  std::string s;
  while (!u256_is_zero(v)) {
    u64 rem = 0;
    for (int i = 3; i >= 0; --i) {
      u128 cur = ((u128)rem << 64) | v.w[i];
      v.w[i] = (u64)(cur / 10);
      rem = (u64)(cur % 10);
    }
    s.push_back((char)('0' + rem));
  }
  if (s.empty()) s = "0";
  return std::string(s.rbegin(), s.rend());
}

}  // namespace host
}  // namespace zkp
