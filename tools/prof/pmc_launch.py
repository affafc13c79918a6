#!/usr/bin/env python3
"""Per-launch-kind PMC figures of the bucket accumulation from rocprofv3 --pmc passes of one bench.py
command: k_accumulate<Fq> dispatches split by workgroup count (the H plan's grid vs the witness
plan's, from the bench line's roofline_launches[..]["workgroups"]), k_accumulate<Fq2> = B2.  Per
kind: SQ_INSTS_VALU per dispatch and per mixed addition (x 64 lanes: lane-instructions per addition,
the VERDICT r3 item 2 figure), and, when
the FETCH_SIZE / WRITE_SIZE passes are given, HBM bytes per dispatch (FETCH x1 for these random
64-B gathers: profiles/fetch_calibration_r02.json).
usage: pmc_launch.py <bench.json> <out.json> <counter_collection.csv>..."""
import collections
import csv
import json
import sys
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
import benchline  # noqa: E402


def main(bench_json, out, *files):
    line = benchline.detail(bench_json)
    kinds = line["roofline_launches"]["per_kind"]
    h_wg = set(kinds["H"]["workgroups"])
    w_wg = set(kinds["A"]["workgroups"])
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "k_accumulate" not in name:
                continue
            grid = int(r.get("Grid_Size") or r.get("Grid_Size_X"))
            wg = int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X"))
            blocks = grid // wg
            kind = "B2" if "Fq2" in name else ("H" if blocks in h_wg else ("W" if blocks in w_wg else None))
            if kind is None:
                continue
            vals[kind][(r["Counter_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))].append(float(r["Counter_Value"]))
    res = {"bench": bench_json, "kinds": {}}
    adds = {"H": kinds["H"]["mixed_adds_per_launch"], "W": kinds["A"]["mixed_adds_per_launch"],
            "B2": kinds["B2"]["mixed_adds_per_launch"]}
    for kind, d in vals.items():
        per = collections.defaultdict(list)
        for (cname, _), v in d.items():
            per[cname].append(sum(v))  # one dispatch: sum over the counter's instances
        avg = {c: sum(v) / len(v) for c, v in per.items()}
        o = {"dispatches": max(len(v) for v in per.values()), "counters_avg_per_dispatch": avg,
             "mixed_adds_per_dispatch": adds[kind]}
        if "SQ_INSTS_VALU" in avg:
            o["valu_lane_instructions_per_addition"] = round(avg["SQ_INSTS_VALU"] * 64 / adds[kind], 1)
        if "FETCH_SIZE" in avg:
            o["hbm_bytes_per_dispatch"] = (avg["FETCH_SIZE"] + avg.get("WRITE_SIZE", 0.0)) * 1024
        res["kinds"]["witness (A, B1, C)" if kind == "W" else kind] = o
    txt = json.dumps(res, indent=1)
    print(txt)
    open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
