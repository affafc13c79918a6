#!/usr/bin/env python3
"""Cold start of the prover from the app's chunked, gzip-compressed proving key (SURVEY.md §8f
row 2; reference app/src/helpers/zkp.ts:11-13,51-68 and upload_chunked_keys_to_s3.sh:13-22:
circuit.zkey{b..k}.gz) at Venmo size on one MI355X.  The Venmo-shaped synthetic zkey (3.35 GB,
insecure known-tau) is byte-split into ten chunks b..k, each gzip-compressed, and the load is
timed end to end (read + inflate + merge, parse + H2D + base tables) with the chunks inflated in
parallel (default) and on one thread, beside the plain file and the in-memory key.  Files are in
the page cache (written just before), as on a server that has just downloaded the chunks.
usage: bench_coldstart.py [out.json] [workdir=/tmp/zkp_coldstart]"""
import json
import multiprocessing as mp
import os
import shutil
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zk-p2p-onramp_amd"))
import zkp_amd  # noqa: E402
from zkp_amd import synth  # noqa: E402

SUFFIX = "bcdefghijk"


def _gz(args):
    path, data = args
    c = zlib.compressobj(6, zlib.DEFLATED, 16 + zlib.MAX_WBITS)
    with open(path, "wb") as f:
        f.write(c.compress(data))
        f.write(c.flush())
    return os.path.getsize(path)


def timed(fn):
    t0 = time.time()
    r = fn()
    return r, time.time() - t0


def main(out=None, work="/tmp/zkp_coldstart"):
    os.makedirs(work, exist_ok=True)
    circ = synth.Circuit.venmo(0x5A4B5032)
    zk, t_synth = timed(lambda: circ.zkey(0x5A4B5033))
    raw = zk.bytes() if hasattr(zk, "bytes") else bytes(zk)
    n = len(raw)
    step = (n + len(SUFFIX) - 1) // len(SUFFIX)
    parts = [(os.path.join(work, "circuit.zkey%s.gz" % s), raw[i * step:(i + 1) * step]) for i, s in enumerate(SUFFIX)]
    with mp.Pool(len(parts)) as pool:
        sizes, t_gz = timed(lambda: pool.map(_gz, parts))
    del parts
    plain = os.path.join(work, "circuit_plain.zkey")
    with open(plain, "wb") as f:
        f.write(raw)
    res = {"zkey_bytes": n, "chunks": len(SUFFIX), "gz_bytes": sum(sizes), "synth_s": round(t_synth, 2),
           "compress_s_10proc": round(t_gz, 2)}
    chunk_path = os.path.join(work, "circuit.zkey")
    buf, res["inflate_merge_parallel_s"] = timed(lambda: zkp_amd.read_zkey(chunk_path))
    assert buf == raw, "chunked key does not read back"
    del buf
    p, res["load_chunks_gz_parallel_s"] = timed(lambda: zkp_amd.Prover(chunk_path, devices=[0]))
    p.close()
    p, res["load_plain_file_s"] = timed(lambda: zkp_amd.Prover(plain, devices=[0]))
    p.close()
    p, res["load_from_memory_s"] = timed(lambda: zkp_amd.Prover(zk, devices=[0]))
    res["table_bytes_per_device"] = p.msm_config()["table_bytes_per_device"]
    p.close()
    res["cpu_threads"] = len(os.sched_getaffinity(0))
    res["note"] = ("load_* = zkp_prover_load_file / _mem end to end: read + inflate + merge (host), parse + validate, "
                   "one H2D of the points, base-table build on the GPU; files in the page cache")
    shutil.rmtree(work, ignore_errors=True)
    line = json.dumps(res)
    print(line)
    if out:
        with open(out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
