/*
 * zkp_amd.h — C ABI of libzkp_amd.so, the MI355X-native Groth16 prover that is a
 * drop-in for the snarkjs `groth16.prove(zkey, wtns)` hot path of ZKP2P.
 *
 * Reference interface replaced (paths relative to the reference repo):
 *   - CLI  `snarkjs groth16 prove <zkey> <wtns> <proof.json> <public.json>`
 *          dizkus-scripts/5_gen_proof.sh:8, circuit/scripts/generate_proof_groth16.sh:11,
 *          and its rapidsnark twin dizkus-scripts/6_gen_proof_rapidsnark.sh:26,
 *          circuit/server-scripts/generate_proof.sh:5
 *   - JS   `snarkjs.groth16.fullProve(input, wasm, zkey)` -> groth16.prove(zkey, wtns)
 *          app/src/helpers/zkp.ts:94  (snarkjs@0.4.22, package-lock.json:3884-3896)
 * The N-API addon (zk-p2p-onramp_amd/js/) binds exactly these entry points; see
 * INTEGRATION.md for the binding a maintainer adds on the reference side.
 *
 * Conventions: plain pointers and sizes, no exceptions across the ABI, status codes
 * plus a thread-local message (zkp_last_error).  All field values cross the ABI as
 * 32-byte little-endian integers in STANDARD (non-Montgomery) form, exactly the
 * bytes snarkjs writes as decimal strings in proof.json / public.json.
 */
#ifndef ZKP_AMD_H
#define ZKP_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum zkp_status {
  ZKP_OK = 0,
  ZKP_ERR_INVALID_ARG = 1,     /* null pointer / bad size                                   */
  ZKP_ERR_IO = 2,              /* file open/read/write failure                              */
  ZKP_ERR_FORMAT = 3,          /* bad magic, version or section layout (binfileutils)      */
  ZKP_ERR_PROTOCOL = 4,        /* zkey is not groth16   (snarkjs: "zkey file is not groth16") */
  ZKP_ERR_CURVE = 5,           /* field mismatch        (snarkjs: "Curve of the witness does not match the curve of the proving key") */
  ZKP_ERR_WITNESS_LENGTH = 6,  /* nWitness != nVars     (snarkjs: "Invalid witness length") */
  ZKP_ERR_DEVICE = 7,          /* HIP runtime error / no usable MI355X                     */
  ZKP_ERR_OUT_OF_MEMORY = 8,
  ZKP_ERR_INTERNAL = 9
} zkp_status;

/* Opaque prover handle: parsed + validated zkey whose point sections are resident in
 * HBM of every device in the list (uploaded once at load).  Immutable after load;
 * concurrent zkp_prove calls on one handle are safe.  Each device holds k proving
 * pipelines (environment ZKP_INFLIGHT = k, 1..4, default 1) that share one copy of its
 * base tables: up to k proofs run concurrently per device, each pipeline one at a time,
 * and each pipeline has two witness upload slots (a witness H2D overlaps the proof in
 * flight).  zkp_prove round-robins over the healthy pipelines; zkp_prove_batch runs two
 * workers per pipeline. */
typedef struct zkp_prover zkp_prover;

/* One Groth16 proof: affine coordinates, standard-form LE (the pi_a/pi_b/pi_c of
 * proof.json without the projective "1"/["1","0"] tails).  public_signals is a
 * caller-owned buffer of public_capacity * 32 bytes receiving w[1..nPublic]. */
typedef struct zkp_proof {
  uint8_t pi_a[2][32];    /* x, y                              */
  uint8_t pi_b[2][2][32]; /* [x.c0, x.c1], [y.c0, y.c1]        */
  uint8_t pi_c[2][32];    /* x, y                              */
  uint32_t n_public;      /* set by zkp_prove                  */
  uint32_t public_capacity;
  uint8_t* public_signals;
} zkp_proof;

/* MSM partial sums of one point range of one proof (the point-range split of a single
 * proof over several GPUs).  Affine standard-form LE, all-zero =
 * infinity.  392 bytes, no padding: ranks exchange these by an RCCL all-gather. */
typedef struct zkp_partial {
  uint8_t a[64], b1[64], c[64], h[64]; /* G1: sum over the slice of w_i A_i, w_i B1_i, w_i C_i, P_j H_j */
  uint8_t b2[128];                     /* G2: sum over the slice of w_i B2_i                          */
  uint32_t part, nparts;
} zkp_partial;

/* Load a .zkey (snarkjs groth16, version 1) from a path or a memory buffer.
 * devices: HIP device ordinals (NULL/0 -> device 0).  Every device gets a full
 * resident copy (batch mode: proofs are spread over devices by zkp_prove_batch). */
zkp_status zkp_prover_load_file(const char* zkey_path, const int* devices, int ndev, zkp_prover** out);
zkp_status zkp_prover_load_mem(const uint8_t* zkey, size_t len, const int* devices, int ndev, zkp_prover** out);

/* Chunked / compressed proving keys (the app's circuit.zkey{b..k}.gz: reference
 * app/src/helpers/zkp.ts:11-13,51-68).  zkp_prover_load_file and zkp_zkey_read accept a
 * path that exists (gzip detected by magic), else path.gz, else the chunks
 * path{a..z}[.gz] in suffix order.  Chunks are either a byte split of one binfile or
 * per-chunk "zkey" binfiles holding disjoint sections (told apart by content). */
zkp_status zkp_prover_load_chunks(const char* const* paths, int n, const int* devices, int ndev, zkp_prover** out);
/* Host only: the merged, decompressed zkey bytes (free with zkp_buffer_free). */
zkp_status zkp_zkey_read(const char* path, uint8_t** out, size_t* len);
zkp_status zkp_zkey_read_chunks(const char* const* paths, int n, uint8_t** out, size_t* len);
void zkp_buffer_free(uint8_t* p);

/* Setup acceleration, primitive: the group arithmetic of a phase-2 contribution with a given
 * secret k (32-byte LE, nonzero mod r) on `device`: delta1, delta2 x k (section 2), every
 * L (section 8) and H (section 9) point x k^-1.  Section 10 (the contribution record) is
 * copied unchanged, so the result does not pass `zkey verify`: the snarkjs commands are
 * zkp_zkey_contribute_entropy / zkp_zkey_beacon.  *out: the new zkey (zkp_buffer_free). */
zkp_status zkp_zkey_contribute(int device, const uint8_t* zkey, size_t len, const uint8_t* k32, uint8_t** out,
                               size_t* out_len);

/* Setup acceleration: `snarkjs zkey beacon <in.zkey> <out.zkey> <beaconHashHex> <numIterationsExp>
 * [-n=name]` (reference dizkus-scripts/3_gen_chunk_zkey.sh:36).  zkp_beacon_secret (host only)
 * derives the contribution scalar as snarkjs@0.4.22 / ffjavascript do: 2^e chained SHA-256 of the
 * beacon, a ChaCha20 stream seeded with the hash, Fr.fromRng; k32: 32-byte LE.  zkp_zkey_beacon
 * draws the rest of the contribution from the same stream (G1.fromRng, the transcript, hashToG2),
 * applies k on the GPU and appends the type-1 record (deltaAfter, proof of knowledge,
 * transcript, numIterationsExp, beacon hash, name) to section 10, so the key passes `zkey
 * verify` (reference circuit/scripts/generate_keys_phase2_groth16.sh:26).  e <= 63; name may be
 * NULL (not recorded).  Record bytes restated (oracle/mpc.py), parity unpinned. */
zkp_status zkp_beacon_secret(const uint8_t* beacon, size_t len, uint32_t num_iterations_exp, uint8_t* k32);
zkp_status zkp_zkey_beacon(int device, const uint8_t* zkey, size_t len, const uint8_t* beacon, size_t beacon_len,
                           uint32_t num_iterations_exp, uint8_t** out, size_t* out_len);
zkp_status zkp_zkey_beacon_named(int device, const uint8_t* zkey, size_t len, const uint8_t* beacon, size_t beacon_len,
                                 uint32_t num_iterations_exp, const char* name, uint8_t** out, size_t* out_len);

/* Setup acceleration: `snarkjs zkey contribute <in.zkey> <out.zkey> -e=<entropy> [-n=name]`
 * (reference dizkus-scripts/3_gen_chunk_zkey.sh:27): the contribution's rng is ChaCha20 seeded with
 * Blake2b-512(64 random bytes || entropy) (snarkjs misc.getRandomRng); rand64: those 64 bytes
 * (NULL: /dev/urandom; non-NULL only for reproducible tests).  The secret and the type-0 record
 * are drawn as for the beacon; the group arithmetic runs on `device`. */
zkp_status zkp_zkey_contribute_entropy(int device, const uint8_t* zkey, size_t len, const uint8_t* rand64,
                                       const char* entropy, const char* name, uint8_t** out, size_t* out_len);

/* Host only: Blake2b-512 of a buffer (the hash of the MPC transcript and circuit hash; exported so
 * the CPU tests pin it against Python's hashlib). */
zkp_status zkp_blake2b512(const uint8_t* data, size_t len, uint8_t* out64);

/* Setup acceleration: `snarkjs zkey new <circuit.r1cs> <pot.ptau> <circuit_0000.zkey>`
 * (reference dizkus-scripts/3_gen_chunk_zkey.sh:18) on `device`: the phase-2 starting key
 * (gamma = delta = 1) of a circom .r1cs (v1) from a prepared .ptau (v1, Lagrange sections 12-15,
 * power >= log2(domain) + 1).  A/B1/B2/IC/L are sparse sums of ptau Lagrange points with the
 * circuit's coefficients, built on the GPU; H is copied from the odd points of the next level.
 * Section 10 holds no contributions and the circuit hash (csHash: Blake2b-512 over the key's
 * points and the ptau's tauG1 powers, host).  *out: the zkey (zkp_buffer_free). */
zkp_status zkp_zkey_new(int device, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* ptau, size_t ptau_len,
                        uint8_t** out, size_t* out_len);

/* Load only point slice `part` of `nparts` (contiguous ranges of the witness-indexed
 * sections 5-8 and of section 9) onto one device.  Such a prover computes partial sums
 * only (zkp_prove_partial); the quotient is computed in full on every part. */
zkp_status zkp_prover_load_part(const uint8_t* zkey, size_t len, int device, int part, int nparts,
                                zkp_prover** out);

zkp_status zkp_prover_info(const zkp_prover* p, uint32_t* n_vars, uint32_t* n_public, uint32_t* domain_size);

/* Prove one witness (.wtns bytes, version <= 2).  r32 / s32: 32-byte LE blinding
 * scalars (< r); NULL -> drawn from the OS CSPRNG (production).  Non-NULL is for
 * bit-exact tests: A, B, C are then a deterministic function of (zkey, wtns, r, s). */
zkp_status zkp_prove(zkp_prover* p, const uint8_t* wtns, size_t len, const uint8_t* r32, const uint8_t* s32,
                     zkp_proof* out);

/* Prove n witnesses, spread over the prover's devices: a shared queue, two host workers per
 * device (the next witness's H2D overlaps the current proof), every proof attempted.
 * r32s / s32s may be NULL (all random) or arrays of n pointers.  Returns ZKP_OK if every
 * proof succeeded, else the first failing proof's status (message names its index). */
zkp_status zkp_prove_batch(zkp_prover* p, const uint8_t* const* wtns, const size_t* lens, int n,
                           const uint8_t* const* r32s, const uint8_t* const* s32s, zkp_proof* outs);
/* The same with a per-proof status array (n entries; proofs with ZKP_OK are valid).  A
 * device that fails (HIP error) is retired and its witness re-queued to the remaining
 * devices; an invalid witness fails alone. */
zkp_status zkp_prove_batch_status(zkp_prover* p, const uint8_t* const* wtns, const size_t* lens, int n,
                                  const uint8_t* const* r32s, const uint8_t* const* s32s, zkp_proof* outs,
                                  zkp_status* statuses);

/* Partial MSM sums of this prover's slice for one witness (any prover; a full one
 * reports part 0 of 1). */
zkp_status zkp_prove_partial(zkp_prover* p, const uint8_t* wtns, size_t len, zkp_partial* out);
/* Host only (no device): sum the nparts partials of one split, then blind (r32 / s32 as
 * in zkp_prove) and assemble the proof; public signals come from wtns.  The result is
 * bit-identical to zkp_prove on the full key. */
zkp_status zkp_proof_combine(const uint8_t* zkey, size_t len, const zkp_partial* parts, int nparts,
                             const uint8_t* wtns, size_t wlen, const uint8_t* r32, const uint8_t* s32,
                             zkp_proof* out);

/* CLI-equivalent: `groth16 prove <zkey> <wtns> <proof.json> <public.json>` on a
 * loaded prover; writes JSON byte-compatible with snarkjs (JSON.stringify(x,null,1)).
 * A regular witness file is memory-mapped for the transfer: it must not be truncated by another
 * writer during the call (other file kinds are read into a buffer first). */
zkp_status zkp_prove_files(zkp_prover* p, const char* wtns_path, const char* proof_json_path,
                           const char* public_json_path);

/* Format a proof as snarkjs proof.json / public.json text.  Returns the needed size
 * (including NUL) in *needed; writes when cap is large enough. */
zkp_status zkp_proof_json(const zkp_proof* proof, char* buf, size_t cap, size_t* needed);
zkp_status zkp_public_json(const zkp_proof* proof, char* buf, size_t cap, size_t* needed);

/* `snarkjs zkey export soliditycalldata` text of a proof + its public signals
 * (reference circuit/scripts/generate_calldata.sh:3): a, b (G2 pairs in EIP-197
 * [c1, c0] order, as Verifier.sol:184-188 expects), c, inputs as "0x" + 64 hex digits. */
zkp_status zkp_proof_calldata(const zkp_proof* proof, char* buf, size_t cap, size_t* needed);

/* Per-stage device timings (ms) of the last zkp_prove on this handle:
 * [0] wtns H2D, [1] buildABC, [2] NTT/quotient, [3] MSM G1 A,B1,C (own stream, overlaps
 * [1]-[2]), [4] MSM G2 B2 (own stream), [5] host assembly, [6] total wall, [7] MSM G1 H,
 * [8] verify-before-return (host; 0 when off), [9] the witness transfer's PCIe payload in MB
 * (compact encoding; 0 for staged proofs), [10] the witness-MSM configuration
 * the proof took (0: the default window bits, 1: the second, wider ones; zkp_prover_msm_config).
 * n = capacity of ms (entries beyond n are not written). */
zkp_status zkp_prover_timings(const zkp_prover* p, float* ms, int n);

void zkp_prover_free(zkp_prover* p);

/* Verify-before-return (the reference verifies every proof right after proving:
 * dizkus-scripts/5_gen_proof.sh:14-21 `snarkjs groth16 verify`).  A checked proof is verified on
 * the host (optimal-ate pairing, the Verifier.sol:340-358 equation) against the zkey's verification
 * key before it is returned; a proof that fails the check is never returned: the call (or that
 * proof's batch status) reports ZKP_ERR_INTERNAL ("proof failed verify-before-return ...").
 * on = 0: off; 1: every proof of zkp_prove / zkp_prove_batch[_status] / zkp_prove_staged /
 * zkp_prove_files; 2 (the DEFAULT): the proofs of zkp_prove_batch[_status] only -- there the check
 * runs on the worker thread while the next proof computes (no measured throughput cost), while on
 * a single proof it would add a few ms of one host core to the latency.  The environment
 * ZKP_VERIFY=0/1/2 at load overrides the default.  Any other nonzero `on` means 1. */
zkp_status zkp_prover_set_verify(zkp_prover* p, int on);
/* The current verify-before-return mode (0, 1 or 2 as above). */
zkp_status zkp_prover_get_verify(const zkp_prover* p, int* mode);

/* Host only (no device): `snarkjs groth16 verify` of one proof against a zkey's verification key
 * (sections 2 and 3).  *valid = 1 if the proof verifies (public signals from proof->public_signals,
 * each < r), else 0; the status reports only malformed input. */
zkp_status zkp_proof_verify(const uint8_t* zkey, size_t len, const zkp_proof* proof, int* valid);

/* Host only: the BN254 optimal-ate pairing e(P, Q) as snarkjs reports GT elements (ffjavascript's
 * final exponentiation), e.g. vk_alphabeta_12 = e(vk_alpha_1, vk_beta_2) of a verification key.
 * g1: x, y (64 bytes), g2: x.c0, x.c1, y.c0, y.c1 (128 bytes), standard-form LE, all-zero =
 * infinity.  out: 12 x 32 bytes, the Fq12 coefficients in snarkjs' JSON nesting order
 * [[c0.c0, c0.c1, c0.c2], [c1.c0, c1.c1, c1.c2]], each Fq2 as (c0, c1). */
zkp_status zkp_pairing(const uint8_t* g1, const uint8_t* g2, uint8_t* out384);

/* Thread-local message of the last failing call on this thread ("" if none). */
const char* zkp_last_error(void);

/* Library / build identification, e.g. "zkp_amd 0.1 gfx950". */
const char* zkp_version(void);

/* ---- kernel-level entry points (tests and benchmarks; same kernels as zkp_prove) ----
 * points: zkey layout (affine, Montgomery 2^256 LE; infinity = zero bytes),
 * scalars: 32-byte LE standard form.  out: affine standard-form LE (64 / 128 bytes),
 * all-zero + *is_inf = 1 for the point at infinity. */
zkp_status zkp_msm_g1(int device, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out64,
                      int* is_inf);
zkp_status zkp_msm_g2(int device, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out128,
                      int* is_inf);
/* The same MSM with explicit Pippenger parameters (tests / tuning): window_bits c
 * (0 = automatic, else 8..24) and base-table depth T (0 = automatic = all windows in
 * one bucket set; 1 = no precomputed rows, one bucket group per window). */
zkp_status zkp_msm(int device, int g2, const uint8_t* points, const uint8_t* scalars, size_t n, int window_bits,
                   int table_depth, uint8_t* out, int* is_inf);
/* In-place Fr transforms on n = 2^k standard-form LE elements, natural order:
 * mode 0: forward (A_j = sum a_i w^ij), 1: inverse, 2: coset-extend (snarkjs
 * ifft -> batchApplyKey(1, Fr.w[k+1]) -> fft). */
zkp_status zkp_ntt_fr(int device, uint8_t* data, size_t n, int mode);
/* The H-MSM scalars P_j (standard form, n = domain) for (zkey, wtns): rows A4..A8. */
zkp_status zkp_quotient(zkp_prover* p, const uint8_t* wtns, size_t len, uint8_t* out);

/* ---- benchmarking / serving helpers ----
 * Keep a witness resident in HBM (dev_index: index into the `devices` list the prover was
 * loaded with, 0..ndev-1, whatever ZKP_INFLIGHT is; the witness goes to that device's first
 * pipeline; any slot number); zkp_prove_staged then runs the proof without the PCIe copy.
 * Calls for different dev_index values run concurrently; concurrent calls for the same
 * dev_index take that device's idle ZKP_INFLIGHT pipelines (which read the staged witness in
 * place) and queue on its first pipeline when none is idle. */
zkp_status zkp_witness_stage(zkp_prover* p, int dev_index, int slot, const uint8_t* wtns, size_t len);
zkp_status zkp_prove_staged(zkp_prover* p, int dev_index, int slot, const uint8_t* r32, const uint8_t* s32,
                            zkp_proof* out);
zkp_status zkp_prove_partial_staged(zkp_prover* p, int slot, zkp_partial* out);
/* Distributed quotient of a split proof: instead of every part
 * recomputing all three coset extensions, part v % nparts computes vector v (A, B, C) and
 * the parts exchange domain slices (zkp_amd.dist: RCCL send/recv over xGMI).
 * Stage 1: buildABC on the witness staged in `slot`, then the coset extension of the
 * vectors selected by mask (bit 0 A, 1 B, 2 C); vector v is copied whole (domain_size x
 * 32 bytes, opaque device layout) to dst[v], device memory on this prover's device
 * (entries of unselected vectors may be NULL).  Returns when the copies are complete. */
zkp_status zkp_quotient_part_staged(zkp_prover* p, int slot, int mask, void* const* dst);
/* Stage 2: the partial sums of this prover's slice with the H-MSM scalars joined from
 * abc[0..2] = device pointers to the stage-1 values of A, B, C at this part's domain
 * slice [part*n/nparts, (part+1)*n/nparts) (contiguous, complete before the call). */
zkp_status zkp_prove_partial_ext_staged(zkp_prover* p, int slot, const void* const* abc, zkp_partial* out);
/* Bracket every bucket-accumulate kernel launch with HIP events (on its stream).
 * zkp_prover_kernel_stats: [0] G1 accumulate ms (sum), [1] G1 launches, [2] G1 mixed
 * additions, [3] G1 tasks, [4..7] the same for G2.  Enabling resets the counters. */
zkp_status zkp_prover_instrument(zkp_prover* p, int on);
zkp_status zkp_prover_kernel_stats(const zkp_prover* p, double* out, int n);
/* Every instrumented bucket-accumulate launch since zkp_prover_instrument(p, 1), in order: record i =
 * out[4i .. 4i+3] = {kind, mixed additions, ms (HIP events on the launch's stream), workgroups of the
 * launch (to match the dispatch in a kernel trace)}, kind 0 / 1 / 2 =
 * the witness MSMs A / B1 / C (G1), 3 = the H MSM (G1), 4 = the witness MSM B2 (G2).  Writes at most
 * max_records records; *n_records = the number held (up to 65536 per pipeline). */
zkp_status zkp_prover_launch_stats(const zkp_prover* p, double* out, int max_records, int* n_records);
/* MSM configuration chosen at load (device 0): [0] witness-MSM window bits c, [1] its
 * base-table depth T, [2] its bucket groups ceil(W/T), [3..5] the same for the H MSM,
 * [6] bytes of precomputed base tables per device, [7..9] c, T and groups of the second witness-MSM
 * configuration (wider windows, taken by witnesses whose values are mostly >= 2^32; 0 when the
 * prover keeps only one).  n = capacity of out. */
zkp_status zkp_prover_msm_config(const zkp_prover* p, double* out, int n);
/* Device-resident kernel benchmarks.  MSM: stats[0] ms per MSM, [1] ms per
 * accumulate-kernel launch, [2] mixed additions per launch, [3] tasks per launch,
 * [4] window bits c, [5] windows.  out/is_inf receive the result (verification). */
zkp_status zkp_bench_msm(int device, int g2, const uint8_t* points, const uint8_t* scalars, size_t n, int warmup,
                         int iters, double* stats, uint8_t* out, int* is_inf);
/* The same with nstats = capacity of stats, and [6] ms to build the base tables (row 0 upload and
 * conversion + the derived rows 2^(c t) P, t < T: fixed bases, outside the timed MSMs, as the prover
 * builds them at zkey load), [7] the table depth T (rows per point). */
zkp_status zkp_bench_msm_ex(int device, int g2, const uint8_t* points, const uint8_t* scalars, size_t n, int warmup,
                            int iters, double* stats, int nstats, uint8_t* out, int* is_inf);
/* ms per MSM plan build (digits, bucket grouping, task offsets) of n scalars (32-byte LE):
 * window_bits 0 = automatic; dense != 0: every (window, point) digit an entry, grouped by the
 * hand-written LDS-staged bucket sort (the H MSM's plan), else the compacted witness plan */
zkp_status zkp_bench_plan(int device, const uint8_t* scalars, size_t n, int window_bits, int dense, int warmup,
                          int iters, double* ms);
/* ms per coset-extension (iNTT + coset key + NTT) of 2^log_n Fr elements */
zkp_status zkp_bench_ntt(int device, int log_n, int warmup, int iters, double* ms);
/* ms per batched coset-extension of count (1..3) vectors of 2^log_n Fr elements, every pass one
 * launch over all of them: what the prover runs on the quotient's A, B, C */
zkp_status zkp_bench_ntt_batch(int device, int log_n, int count, int warmup, int iters, double* ms);

#ifdef __cplusplus
}
#endif
#endif /* ZKP_AMD_H */
