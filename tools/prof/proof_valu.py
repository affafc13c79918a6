#!/usr/bin/env python3
"""Whole-proof VALU budget from one rocprofv3 --pmc pass of the valu set over the short bench command
(tools/gpu/pmc.sh <tag> valu): every dispatch of a proof, grouped from one k_build_abc to the next.

The collection serialises dispatches, so per-dispatch counters and times are each kernel alone; instruction
counts do not depend on concurrency.  Per proof and per kernel class:
    busy SIMD-cycles = (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) x 4 / 1024   (the counted VALU busy of
                       tools/prof/valu_counted.py, summed instead of divided by a kernel's own cycles)
    t_valu(f) = busy SIMD-cycles / f: the proof's VALU work if every SIMD issued every quad-cycle at clock f
and the sum of the dispatches' serialised times.  Against the bench's concurrent ms per proof this says how
much of a proof's span the VALU work fills.
usage: proof_valu.py <run_counter_collection.csv> <bench line json> [out.json]
(round 6: tools/gpu/pmc.sh pw2 valu on the final library, three whole proofs kept in profiles/proof_valu_r06/,
the span from profiles/bench_r06_d.json -> profiles/proof_valu_r06.json)"""
import collections
import csv
import json
import re
import statistics
import sys

SIMDS = 1024


def klass(name):
    n = name
    if "k_accumulate" in n:
        return "accumulate G2" if "Fq2" in n else "accumulate G1"
    if "k_ntt" in n or "k_coset" in n or "k_pass_table" in n:
        return "NTT"
    if re.search(r"k_(build_abc|join_abc)", n):
        return "QAP (buildABC, joinABC)"
    if re.search(r"k_(merge|reduce_segments|subset)", n):
        return "MSM finish (merges, reduction, subset sums)"
    if re.search(r"k_(hs_|scan_|tlen|lvl|digits|plan)", n):
        return "MSM plans (bucket sort, tasks)"
    if "witness_unpack" in n:
        return "witness expansion"
    return "other"


def dispatches(path):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        e = d.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]


def main():
    ds = dispatches(sys.argv[1])
    bench = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
    ms_proof = bench["ms_per_step"]
    starts = [i for i, e in enumerate(ds) if "k_build_abc" in e["name"]]
    proofs = []
    for a, b in zip(starts, starts[1:]):
        cls = collections.defaultdict(lambda: {"busy_simd_cycles": 0.0, "instr": 0.0, "serial_ms": 0.0})
        for e in ds[a:b]:
            c = cls[klass(e["name"])]
            c["busy_simd_cycles"] += (e["SQ_INSTS_VALU"] - e["SQ_ACTIVE_INST_VALU2"]) * 4 / SIMDS
            c["instr"] += e["SQ_INSTS_VALU"]
            c["serial_ms"] += e["ns"] / 1e6
        proofs.append(cls)
    out = {"source": sys.argv[1], "bench": sys.argv[2], "bench_ms_per_proof": ms_proof, "proofs": len(proofs), "classes": {}}
    keys = sorted({k for p in proofs for k in p})
    tot_busy = statistics.median(sum(c["busy_simd_cycles"] for c in p.values()) for p in proofs)
    tot_instr = statistics.median(sum(c["instr"] for c in p.values()) for p in proofs)
    for k in keys:
        busy = statistics.median(p[k]["busy_simd_cycles"] for p in proofs if k in p)
        out["classes"][k] = {
            "valu_instr_share": round(statistics.median(p[k]["instr"] for p in proofs if k in p) / tot_instr, 4),
            "busy_share": round(busy / tot_busy, 4),
            "serial_ms": round(statistics.median(p[k]["serial_ms"] for p in proofs if k in p), 3)}
    serial = statistics.median(sum(c["serial_ms"] for c in p.values()) for p in proofs)
    out["serial_ms_per_proof"] = round(serial, 3)
    out["valu_busy_simd_cycles_per_proof"] = round(tot_busy)
    out["t_valu_ms"] = {"%.1f GHz" % f: round(tot_busy / (f * 1e6), 3) for f in (1.8, 2.0, 2.2, 2.4)}
    out["span_filled_by_valu_work"] = {"%.1f GHz" % f: round(tot_busy / (f * 1e6) / ms_proof, 3) for f in (1.8, 2.0, 2.2, 2.4)}
    json.dump(out, open(sys.argv[3], "w") if len(sys.argv) > 3 else sys.stdout, indent=1)
    if len(sys.argv) > 3:
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
