// `snarkjs zkey beacon` secret derivation (host only; beacon.cpp).
#pragma once
#include <cstddef>
#include <cstdint>

namespace zkp {
// 2^num_iterations_exp chained SHA-256 of the beacon bytes
void beacon_hash(const uint8_t* beacon, size_t len, uint32_t num_iterations_exp, uint8_t out[32]);
// the contribution scalar k (32-byte LE, < r) of `zkey beacon <beacon> <num_iterations_exp>`
void beacon_secret(const uint8_t* beacon, size_t len, uint32_t num_iterations_exp, uint8_t k32[32]);
}  // namespace zkp
