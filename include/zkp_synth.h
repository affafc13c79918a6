/*
 * zkp_synth.h — TOOLING, not the proving path: generators for Venmo-shaped
 * synthetic circuits, witnesses and INSECURE known-tau proving keys in the exact
 * snarkjs binary formats, so that benchmarks and large-size tests can run without
 * the (absent) 3.5 GB Venmo zkey.
 *
 * Bit-for-bit mirror of oracle/circuit.py + oracle/setup.py (tests compare the
 * bytes for small sizes); the large fixed-base scalar multiplications run on the
 * GPU (libzkp_synth.so links the same field/curve code as libzkp_amd.so).
 */
#ifndef ZKP_SYNTH_H
#define ZKP_SYNTH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct zkp_synth_circuit zkp_synth_circuit;

/* 0 on success, nonzero on failure (message via zkp_synth_last_error) */
int zkp_synth_circuit_new(uint32_t n_vars, uint32_t n_constraints, uint32_t n_public, uint64_t seed,
                          uint32_t in_permille, zkp_synth_circuit** out);
/* The same with the witness mix as a knob: a defining step is AND (x < bool_percent/2) or XOR
 * (x < bool_percent), producing a bit, else MUL (a uniform value), for x uniform in [0, 100).
 * zkp_synth_circuit_new = bool_percent 70 (the Venmo-shape assumption);
 * 0 = every defined signal uniform (only the input bits stay 0/1). */
int zkp_synth_circuit_new_mix(uint32_t n_vars, uint32_t n_constraints, uint32_t n_public, uint64_t seed,
                              uint32_t in_permille, uint32_t bool_percent, zkp_synth_circuit** out);
void zkp_synth_circuit_free(zkp_synth_circuit* c);
uint32_t zkp_synth_domain_size(const zkp_synth_circuit* c);

/* .wtns (v2) bytes for witness seed wseed; size = 44 + 12*2 + 32*nVars + ...: query with out=NULL */
int zkp_synth_witness(const zkp_synth_circuit* c, uint64_t wseed, uint8_t* out, size_t cap, size_t* len);

/* Full .zkey (v1 groth16) for setup seed; buffer allocated by the library (free with
 * zkp_synth_free).  threads: host threads for the QAP evaluation (0 = all cores). */
int zkp_synth_zkey(const zkp_synth_circuit* c, uint64_t setup_seed, int device, int threads, uint8_t** out,
                   size_t* len);
/* The same with gamma = delta = 1 when unit_gamma_delta != 0: the key `snarkjs zkey new` writes from a
 * ptau of the same tau, alpha, beta (zkp_synth_ptau; sections 2..9 then equal zkp_zkey_new's). */
int zkp_synth_zkey_ex(const zkp_synth_circuit* c, uint64_t setup_seed, int unit_gamma_delta, int device, int threads,
                      uint8_t** out, size_t* len);
/* circom .r1cs (v1) of the synthetic circuit (the layout of oracle/binfile.py write_r1cs) */
int zkp_synth_r1cs(const zkp_synth_circuit* c, uint8_t** out, size_t* len);
/* A prepared known-tau .ptau (v1, sections 1-7 and the Lagrange sections 12-15 of every level
 * 0..power; oracle/binfile.py write_ptau) with tau, alpha, beta of setup_seed as zkp_synth_zkey: every
 * point on the GPU.  INSECURE (the toxic waste is the seed), for setup benchmarks and tests. */
int zkp_synth_ptau(uint32_t power, uint64_t setup_seed, int device, int threads, uint8_t** out, size_t* len);
void zkp_synth_free(uint8_t* buf);

/* k_i * G (G1: 64-byte / G2: 128-byte zkey-layout affine points) for n 32-byte LE scalars */
int zkp_synth_points_g1(int device, const uint8_t* scalars, size_t n, uint8_t* out);
int zkp_synth_points_g2(int device, const uint8_t* scalars, size_t n, uint8_t* out);

/* n uniform Fr scalars (32-byte LE) from SplitMix64(seed, stream) exactly like the oracle's fr() */
void zkp_synth_scalars(uint64_t seed, uint64_t stream, size_t n, uint8_t* out);

const char* zkp_synth_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* ZKP_SYNTH_H */
