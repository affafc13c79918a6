// The phase-2 MPC record of a zkey (section 10) -- host only: the circuit hash (csHash) that
// `snarkjs zkey new` writes, the contribution entries that `zkey contribute` / `zkey beacon` append,
// and their primitives (Blake2b-512, ffjavascript's ChaCha word stream and field / curve draws,
// snarkjs' hashToG2, the "uncompressed" point encoding).  Reference call sites:
// dizkus-scripts/3_gen_chunk_zkey.sh:18,27,36 and the gate circuit/scripts/generate_keys_phase2_
// groth16.sh:26 (`zkey verify`).  The algorithms are snarkjs@0.4.22 / ffjavascript 0.2.55's
// (absent offline); the restatement this must equal byte for byte is oracle/mpc.py, whose module
// docstring lists the recalled conventions (parity unpinned: no snarkjs-written zkey exists here).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "host_ec.hpp"

namespace zkp {

// RFC 7693 Blake2b with a 64-byte digest, no key
class Blake2b {
 public:
  Blake2b();
  void update(const void* data, size_t len);
  void final(uint8_t out[64]);

 private:
  void compress(bool last);
  uint64_t h_[8], t_[2] = {0, 0};
  uint8_t buf_[128];
  size_t n_ = 0;
};

// ffjavascript ChaCha: a ChaCha20 word stream, state = constants, seed (words 4..11), counter
// words 12..15 (one 16-word block per refill, counter carried across 12..15)
struct ChaChaRng {
  uint32_t st[16], buf[16];
  int idx = 16;
  explicit ChaChaRng(const uint32_t seed[8]);
  uint32_t next_u32();
  uint64_t next_u64();  // high word first
  bool next_bool() { return (next_u32() & 1u) != 0; }
};
// the seed of a 32+-byte hash: its first 8 big-endian 32-bit words
void seed_from_hash(const uint8_t* h, uint32_t seed[8]);

struct MpcContribution {
  host::Affine<host::Fq> delta_after, g1_s, g1_sx;
  host::Affine<host::Fq2> g2_spx;
  uint8_t transcript[64];
  uint32_t type = 0;           // 0 contribute, 1 beacon
  std::vector<uint8_t> params;  // raw parameter bytes (name / numIterationsExp / beacon hash)
};
struct MpcParams {
  uint8_t cs_hash[64];
  std::vector<MpcContribution> contributions;
};

MpcParams read_mpc(const uint8_t* sec, size_t len);
std::vector<uint8_t> write_mpc(const MpcParams& m);

// Draw one contribution from rng (k = Fr.fromRng, then g1_s = G1.fromRng), append its record
// (deltaAfter = k * delta1_before) and return k as 32-byte LE standard form.  type 1 (beacon)
// records numIterationsExp and the beacon hash; a non-empty name is recorded first.
void mpc_contribute(MpcParams& m, ChaChaRng& rng, const host::Affine<host::Fq>& delta1_before, uint32_t type,
                    const std::string& name, const uint8_t* beacon, size_t beacon_len, uint32_t num_iterations_exp,
                    uint8_t k32[32]);

// csHash of a new key (`zkey new`): over its header points and point sections (key bytes, zkey
// layout) and the H points (tau^(n+i) - tau^i) G1 from the ptau's tauG1 (LEM, >= 2n points)
void mpc_cs_hash_new(const uint8_t* zkey, size_t len, const uint8_t* tau_g1, size_t tau_g1_points, uint8_t out[64]);

// replace (or append) section `id` of a binfile held in `file`
void binfile_replace_section(std::vector<uint8_t>& file, uint32_t id, const std::vector<uint8_t>& payload);

}  // namespace zkp
