#!/usr/bin/env python3
"""Per-launch PMC summary of the bucket-accumulate kernels from three rocprofv3 --pmc
passes of the same bench command (FETCH_SIZE; WRITE_SIZE; SQ_INSTS_VALU + SQ_WAVES ...).
HBM bytes per launch = FETCH_SIZE + WRITE_SIZE (KB units).  The guide's x2 on FETCH_SIZE holds for
coalesced 16-B/lane streams only; the accumulate's bytes are random 64-B base gathers, for which
FETCH_SIZE reads the bytes exactly (calibrated on a known byte count: profiles/fetch_calibration_r02.json,
tools/ubench/gather_fetch.hip: gather x1.00, stream x0.50).  VALU issue fraction =
SQ_INSTS_VALU x 64 lanes / launch time / measured issue peak (35.4 T lane-op/s,
profiles/ubench_r01.txt: v_mul_lo_u32 / v_add_co_u32).
usage: pmc_accumulate.py <fetch.csv> <write.csv> <sq.csv> <out.json>"""
import collections, csv, json, sys
from summarize import short

PEAK = 35.4e12


def load(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        if not k.startswith("k_accumulate"):
            continue
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[k][r["Counter_Name"]].append((float(r["Counter_Value"]), ns))
    return d


def main(fetch, write, sq, out):
    F, W, S = load(fetch), load(write), load(sq)
    res = {"sources": [fetch, write, sq], "peak_valu_lane_ops_per_s": PEAK, "kernels": {}}
    for k in F:
        f = [v for v, _ in F[k]["FETCH_SIZE"]]
        w = [v for v, _ in W.get(k, {}).get("WRITE_SIZE", [(0, 1)])]
        ins = S.get(k, {}).get("SQ_INSTS_VALU", [])
        e = {"launches": len(f), "FETCH_SIZE_kb_avg": sum(f) / len(f), "WRITE_SIZE_kb_avg": sum(w) / len(w),
             "hbm_bytes_per_launch": (sum(f) / len(f) + sum(w) / len(w)) * 1024,
             "correction": "FETCH_SIZE x1: random 64-B gathers (profiles/fetch_calibration_r02.json), KB units"}
        if ins:
            lane_ops = sum(v * 64 for v, _ in ins) / (sum(ns for _, ns in ins) * 1e-9)
            e.update({"valu_insts_per_launch": sum(v for v, _ in ins) / len(ins),
                      "valu_lane_ops_per_s": lane_ops, "valu_issue_frac": round(lane_ops / PEAK, 3)})
        res["kernels"][k] = e
    g1 = res["kernels"].get("k_accumulate<Fq >") or res["kernels"].get("k_accumulate<Fq>")
    if g1:
        res["hbm_bytes_per_launch"] = g1["hbm_bytes_per_launch"]
        res["valu_issue_frac"] = g1.get("valu_issue_frac")
        res["kernel"] = "k_accumulate<Fq>"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
