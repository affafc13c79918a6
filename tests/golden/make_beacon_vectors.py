"""Generate tests/golden/beacon_vectors.json: ChaCha20 keystream blocks from OpenSSL's
`enc -chacha20` (an independent implementation, pinning oracle/beacon.py's block function
and counter), plus beacon secrets from oracle/beacon.py (regression values, parity unpinned).
Run from the repo root: python tests/golden/make_beacon_vectors.py"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from oracle import beacon  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "beacon_vectors.json")


def openssl_keystream(seed_words, nbytes):
    key = b"".join(w.to_bytes(4, "little") for w in seed_words)  # state words 4..11, little-endian bytes
    iv = bytes(16)  # 32-bit block counter 0 + 96-bit nonce 0 (state words 12..15)
    r = subprocess.run(["openssl", "enc", "-chacha20", "-K", key.hex(), "-iv", iv.hex()], input=bytes(nbytes),
                       capture_output=True, check=True)
    return r.stdout.hex()


def main():
    seeds = [[0] * 8, list(range(8)), [0x01234567, 0x89ABCDEF, 0xDEADBEEF, 0xFFFFFFFF, 0, 1, 0x80000000, 0x7FFFFFFF]]
    chacha = [{"seed": s, "keystream_hex": openssl_keystream(s, 64 * 3)} for s in seeds]
    beacons = []
    for hx, e in [("0102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f20", 10), ("00", 0), ("ff" * 7, 4)]:
        b = bytes.fromhex(hx)
        beacons.append({"beacon_hex": hx, "num_iterations_exp": e, "hash_hex": beacon.beacon_hash(b, e).hex(),
                        "k": str(beacon.beacon_secret(b, e))})
    json.dump({"chacha20_openssl": chacha, "beacon_oracle": beacons}, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
