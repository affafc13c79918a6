// Kernels around the NTT: zkey->device layout conversion, buildABC (sparse
// A.w, B.w and C = A*B on the domain) and joinABC (P = A*B - C, out of
// Montgomery form, as 8-word MSM scalars).  snarkjs groth16_prove rows A1, A4,
// A8.
#pragma once
#include "wtns_pack.hpp"
#include <hip/hip_runtime.h>
#include <cstddef>
#include <cstdint>

namespace zkp {

// zkey points (affine, Montgomery 2^256, LE words) -> device layout in place.
// nelems = number of Fq elements (2 per G1 point, 4 per G2 point).
void launch_convert_fq_zkey(uint32_t* data, size_t nelems, hipStream_t st);
// zkey section-4 values X = coef*2^512 mod r -> device c' = coef*2^522 mod r in place
void launch_convert_coefs(uint32_t* vals, size_t n, hipStream_t st);
// CSR SpMV for both matrices + pointwise C: outputs (device layout, Montgomery R')
//   a[c] = sum_{e in row c of A} mont(val_e, w[col_e]),  b likewise,  c[c] = a[c]*b[c]
void launch_build_abc(const uint32_t* rowptr_a, const uint32_t* col_a, const uint32_t* val_a,
                      const uint32_t* rowptr_b, const uint32_t* col_b, const uint32_t* val_b,
                      const uint32_t* witness, uint32_t n, uint32_t* a, uint32_t* b, uint32_t* c, hipStream_t st);
// p[j] = standard-form canonical (a[j]*b[j] - c[j]) as 8 LE words
void launch_join_abc(const uint32_t* a, const uint32_t* b, const uint32_t* c, uint32_t n, uint32_t* p,
                     hipStream_t st);
// Compact witness transfer (wtns_pack.hpp): expands signals [i0, i1) from the chunk regions at stage
// into 8-word values at out (signal i at out + 8 i).
void launch_witness_unpack(const uint32_t* stage, uint32_t i0, uint32_t i1, uint32_t* out, hipStream_t st);
// Fr device layout <-> standard 8-word values (tests)
void launch_fr_to_dev(uint32_t* data, size_t n, hipStream_t st);
void launch_fr_from_dev(uint32_t* data, size_t n, hipStream_t st);
// Fq/G device layout -> standard form (used to return points for tests)
void launch_fq_from_dev(uint32_t* data, size_t n, hipStream_t st);

}  // namespace zkp
