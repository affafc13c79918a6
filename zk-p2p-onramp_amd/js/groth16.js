'use strict';
/*
 * Drop-in for snarkjs' `groth16.prove(zkeyFileName, witnessFileName, logger)`
 * (snarkjs@0.4.22, reference package-lock.json:3884-3896; callers
 * app/src/helpers/zkp.ts:94 via fullProve, dizkus-scripts/5_gen_proof.sh:8 via the CLI).
 *
 * Same arguments (a path or a fastfile memory descriptor {type:"mem", data}), same
 * Promise<{proof, publicSignals}> result with decimal strings and snarkjs' key order,
 * same Error messages (from the C ABI).  The zkey is loaded once per process and stays
 * resident in HBM (snarkjs re-reads it on every call): a path zkey is keyed by its path, a
 * memory zkey ({type:"mem"} / Buffer, the fullProve / fastfile path) by the SHA-256 of its
 * bytes, so repeated proofs with the same in-memory key reuse the resident handle.  The hash is
 * computed once per key buffer (a WeakMap on the underlying ArrayBuffer remembers it), not on
 * every call: a GB-scale key would otherwise block the event loop for ~1 s per proof.  There is
 * no CPU fallback: if the native addon or libzkp_amd.so is missing, require() throws.
 */
const crypto = require('crypto');
const fs = require('fs');
const path = require('path');
const addon = require(path.join(__dirname, 'build', 'zkp_napi.node'));

const provers = new Map();     // zkey path -> handle
const memProvers = new Map();  // sha256(zkey bytes) -> handle, most recently used last
const MEM_PROVERS_MAX = 2;     // each holds its key's base tables in HBM (~50 GB for Venmo)
const memKeyHash = new WeakMap();  // ArrayBuffer -> [{off, len, hash}] of key buffers already hashed

function readInput(x) {
  if (x && typeof x === 'object' && x.type === 'mem') return Buffer.from(x.data.buffer ? x.data : Buffer.from(x.data));
  if (Buffer.isBuffer(x)) return x;
  return fs.readFileSync(x);
}

function sampleHash(buf) {
  const h = crypto.createHash('sha256').update(buf.subarray(0, Math.min(4096, buf.length)));
  for (let k = 0; k < 32 && buf.length > 4096; ++k) {
    const at = Math.floor((buf.length - 256) * (k + 1) / 32);
    h.update(buf.subarray(at, at + 256));
  }
  return h.digest('hex');
}

function proverFor(zkey, devices) {
  if (typeof zkey === 'string') {
    let h = provers.get(zkey);
    if (!h) {
      h = addon.loadProver(zkey, devices);
      provers.set(zkey, h);
    }
    return h;
  }
  const src = zkey && typeof zkey === 'object' && zkey.type === 'mem' ? zkey.data : zkey;
  const buf = ArrayBuffer.isView(src) ? Buffer.from(src.buffer, src.byteOffset, src.byteLength) : readInput(zkey);
  // The full SHA-256 of a key buffer is computed once per (ArrayBuffer, offset, length).  Key
  // buffers are meant to be immutable; a buffer re-filled with another key (a file re-read into
  // it, a reused fastfile mem object) is caught by a sampled fingerprint (the first 4 KiB and 32
  // evenly spaced 256-byte windows) checked on every hit: a mismatch re-hashes the whole buffer.
  let seen = ArrayBuffer.isView(src) ? memKeyHash.get(src.buffer) : undefined;
  let hit = seen && seen.find((e) => e.off === src.byteOffset && e.len === src.byteLength);
  if (hit && hit.sample !== sampleHash(buf)) {
    seen.splice(seen.indexOf(hit), 1);
    hit = undefined;
  }
  if (!hit) {
    hit = { off: buf.byteOffset, len: buf.byteLength, hash: crypto.createHash('sha256').update(buf).digest('hex'),
            sample: sampleHash(buf) };
    if (ArrayBuffer.isView(src)) {
      if (!seen) memKeyHash.set(src.buffer, (seen = []));
      seen.push(hit);
    }
  }
  const key = hit.hash + ':' + JSON.stringify(devices || []);
  let h = memProvers.get(key);
  if (h) {
    memProvers.delete(key);  // refresh its LRU position
  } else {
    h = addon.loadProver(buf, devices);
    while (memProvers.size >= MEM_PROVERS_MAX) {  // evict the least recently used key; a proof
      const [k0, h0] = memProvers.entries().next().value;  // still running on it keeps it alive
      memProvers.delete(k0);                               // until it finishes (addon refcount)
      addon.freeProver(h0);
    }
  }
  memProvers.set(key, h);
  return h;
}

function toBuf32(v) {
  if (v === undefined || v === null) return undefined;
  if (Buffer.isBuffer(v)) return v;
  let x = BigInt(v);
  const b = Buffer.alloc(32);
  for (let i = 0; i < 32; ++i) { b[i] = Number(x & 0xffn); x >>= 8n; }
  return b;
}

/**
 * @param zkeyFileName  path | {type:"mem", data}
 * @param witnessFileName path | {type:"mem", data}
 * @param logger        optional snarkjs-style logger ({debug, info})
 * @param opts          {devices?: number[], r?: bigint|string, s?: bigint|string}  (r/s: tests only)
 */
async function prove(zkeyFileName, witnessFileName, logger, opts) {
  opts = opts || {};
  const h = proverFor(zkeyFileName, opts.devices);
  const wtns = readInput(witnessFileName);
  if (logger && logger.debug) logger.debug('zkp_amd: proving on MI355X');
  return toSnarkjs(await addon.prove(h, wtns, toBuf32(opts.r), toBuf32(opts.s)));
}

function toSnarkjs(r) {
  const proof = {
    pi_a: [r.piA[0], r.piA[1], '1'],
    pi_b: [[r.piB[0][0], r.piB[0][1]], [r.piB[1][0], r.piB[1][1]], ['1', '0']],
    pi_c: [r.piC[0], r.piC[1], '1'],
    protocol: 'groth16',
    curve: 'bn128',
  };
  return { proof, publicSignals: r.publicSignals };
}

/**
 * Many onramp proofs in one call (configs[3] batch): the witnesses are spread over the
 * prover's devices (opts.devices) by the native batch scheduler, each device overlapping the
 * next witness's upload with the current proof.  Resolves to one entry per witness:
 * {proof, publicSignals}, or an Error for a witness that failed (the others still prove).
 * @param witnesses  array of path | {type:"mem", data} | Buffer
 * @param opts       {devices?: number[], rs?: (bigint|string)[], ss?: (bigint|string)[]}  (rs/ss: tests only)
 */
async function proveBatch(zkeyFileName, witnesses, logger, opts) {
  opts = opts || {};
  const h = proverFor(zkeyFileName, opts.devices);
  const bufs = witnesses.map(readInput);
  if (logger && logger.debug) logger.debug(`zkp_amd: proving a batch of ${bufs.length} on MI355X`);
  const rs = opts.rs ? opts.rs.map(toBuf32) : undefined;
  const ss = opts.ss ? opts.ss.map(toBuf32) : undefined;
  const res = await addon.proveBatch(h, bufs, rs, ss);
  return res.map((r) => (r instanceof Error ? r : toSnarkjs(r)));
}

// `snarkjs zkey export soliditycalldata` text (snarkjs 0.4.22 groth16ExportSolidityCallData,
// called at reference circuit/scripts/generate_calldata.sh:3): 64-hex-digit "0x" words,
// G2 coordinates in the EIP-197 [c1, c0] order that Verifier.sol:184-188 / :366-369 expects.
function p256(n) {
  let s = BigInt(n).toString(16);
  while (s.length < 64) s = '0' + s;
  return `"0x${s}"`;
}

async function exportSolidityCallData(proof, publicSignals) {
  const inputs = publicSignals.map(p256).join(',');
  return `[${p256(proof.pi_a[0])}, ${p256(proof.pi_a[1])}],` +
    `[[${p256(proof.pi_b[0][1])}, ${p256(proof.pi_b[0][0])}],[${p256(proof.pi_b[1][1])}, ${p256(proof.pi_b[1][0])}]],` +
    `[${p256(proof.pi_c[0])}, ${p256(proof.pi_c[1])}],` +
    `[${inputs}]`;
}

// Argument list of Ramp.onRamp(uint256[2] _a, uint256[2][2] _b, uint256[2] _c, uint256[msgLen] _signals)
// exactly as the app builds it (reference app/src/components/SubmitOrderOnRampForm.tsx:36-55:
// pi_a / pi_c without the projective "1", each pi_b pair reversed to [c1, c0]).
function onRampArgs(proof, publicSignals) {
  return [
    proof.pi_a.slice(0, 2),
    proof.pi_b.slice(0, 2).map((g2point) => g2point.slice().reverse()),
    proof.pi_c.slice(0, 2),
    publicSignals,
  ];
}

/*
 * snarkjs' `zKey.newZKey(r1csName, ptauName, zkeyName, logger)` (the `zkey new` step,
 * reference dizkus-scripts/3_gen_chunk_zkey.sh:18): the phase-2 initial key (gamma = delta = 1)
 * built on the GPU.  r1cs / ptau are paths or {type:"mem"} descriptors; with a zkeyName the key
 * is written there, and the key bytes are returned either way.
 */
async function newZKey(r1csName, ptauName, zkeyName, logger, device) {
  const out = addon.zkeyNew(readInput(r1csName), readInput(ptauName), device || 0);
  if (typeof zkeyName === 'string') fs.writeFileSync(zkeyName, out);
  else if (zkeyName && typeof zkeyName === 'object' && zkeyName.type === 'mem') zkeyName.data = out;
  if (logger && logger.info) logger.info(`zkey new: ${out.length} bytes`);
  return out;
}

/*
 * snarkjs' `zKey.beacon(zkeyNameOld, zkeyNameNew, name, beaconHashStr, numIterationsExp, logger)`
 * (reference dizkus-scripts/3_gen_chunk_zkey.sh:36): delta -> k delta, L/H -> k^-1 on the GPU, with
 * k and the contribution record (section 10: proof of knowledge, transcript, beacon parameters,
 * name) derived from the beacon as snarkjs does (oracle/mpc.py restates it; parity unpinned).
 */
async function beacon(zkeyNameOld, zkeyNameNew, name, beaconHashStr, numIterationsExp, logger, device) {
  const hex = String(beaconHashStr);
  const bytes = /^([0-9a-fA-F]{2})+$/.test(hex) ? Buffer.from(hex, 'hex') : Buffer.alloc(0);
  if (bytes.length === 0) throw new Error('Invalid Beacon Hash. (It must be a valid hexadecimal sequence)');
  const e = Number(numIterationsExp);
  if (!Number.isInteger(e) || e < 10 || e > 63) throw new Error('Invalid numIterationsExp. (Must be between 10 and 63)');
  const out = addon.zkeyBeacon(readInput(zkeyNameOld), bytes, e, device || 0, name ? String(name) : undefined);
  if (typeof zkeyNameNew === 'string') fs.writeFileSync(zkeyNameNew, out);
  else if (zkeyNameNew && typeof zkeyNameNew === 'object' && zkeyNameNew.type === 'mem') zkeyNameNew.data = out;
  if (logger && logger.info) logger.info(`zkey beacon ${name || ''}: ${out.length} bytes`);
  return out;
}

/*
 * snarkjs' `zKey.contribute(zkeyNameOld, zkeyNameNew, name, entropy, logger)` (reference
 * dizkus-scripts/3_gen_chunk_zkey.sh:27, `zkey contribute -e=... -n=...`): the secret and the
 * record drawn from ChaCha20 seeded with Blake2b(64 random bytes || entropy), the group arithmetic
 * on the GPU.
 */
async function contribute(zkeyNameOld, zkeyNameNew, name, entropy, logger, device) {
  if (!entropy) throw new Error('zkey contribute: entropy is required (-e=...)');
  const out = addon.zkeyContribute(readInput(zkeyNameOld), String(entropy), name ? String(name) : undefined,
                                   device || 0);
  if (typeof zkeyNameNew === 'string') fs.writeFileSync(zkeyNameNew, out);
  else if (zkeyNameNew && typeof zkeyNameNew === 'object' && zkeyNameNew.type === 'mem') zkeyNameNew.data = out;
  if (logger && logger.info) logger.info(`zkey contribute ${name || ''}: ${out.length} bytes`);
  return out;
}

function release() {
  for (const h of provers.values()) addon.freeProver(h);
  for (const h of memProvers.values()) addon.freeProver(h);
  provers.clear();
  memProvers.clear();
}

module.exports = {
  groth16: { prove, proveBatch },
  proveBatch,
  zKey: { exportSolidityCallData, newZKey, beacon, contribute },
  newZKey,
  beacon,
  contribute,
  prove,
  exportSolidityCallData,
  onRampArgs,
  release,
  version: addon.version,
};
