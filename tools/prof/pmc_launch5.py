#!/usr/bin/env python3
"""Round-5 per-launch-kind PMC summary of the bucket accumulation (profiles/pmc_launch_r05.json, read by
bench.py): for each kind (H, the witness launches A/B1/C, B2) the cycle accounting of pmc_stall.py
(effective clock from GRBM_GUI_ACTIVE, VALU issue fraction at that clock and at 2.4 GHz, the wave-cycle
split, lane-instructions per addition) from the SQ pass, HBM bytes per dispatch from the FETCH_SIZE
(x1: random 64-B gathers, profiles/fetch_calibration_r02.json) and WRITE_SIZE passes, and the L1 TLB
(UTCL1) miss share from the TCP pass -- all passes of the same bench command (273c6e8:tools/gpu/r5/pmc.sh).
usage: pmc_launch5.py <pmc dir> <out.json>"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_stall  # noqa: E402
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
import benchline  # noqa: E402


def per_kind(d, name):
    bench = benchline.detail(os.path.join(d, name + ".json"))
    kinds = bench["roofline_launches"]["per_kind"]
    hwg, wwg = set(kinds["H"]["workgroups"]), set(kinds["A"]["workgroups"])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(os.path.join(d, name, "run_counter_collection.csv"))):
        if "k_accumulate" not in r["Kernel_Name"]:
            continue
        b = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
        k = "B2" if "Fq2" in r["Kernel_Name"] else ("H" if b in hwg else ("W" if b in wwg else None))
        if k:
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in agg[k].items()} for k in agg}


def main(d, out, source=None):
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        pmc_stall.acc(os.path.join(d, "sq.json"), os.path.join(d, "sq", "run_counter_collection.csv"), "/tmp/_sq.json")
    sq = json.load(open("/tmp/_sq.json"))["kinds"]
    fetch, write = per_kind(d, "fetch"), per_kind(d, "write")
    tcp = per_kind(d, "tcp") if os.path.isdir(os.path.join(d, "tcp")) else {}
    res = {"source": source or ("rocprofv3 --pmc passes of `bench.py --steps 4 --warmup 1 --batch 0 --no-kernels "
                                "--no-bool0-line` (tools/gpu/r5/pmc.sh): SQ+GRBM; FETCH_SIZE; WRITE_SIZE + TCC_HIT_sum; "
                                "TCP UTCL1; split per launch kind by tools/prof/pmc_launch5.py"),
           "kinds": {}}
    for k, label in (("H", "H"), ("W", "witness (A, B1, C)"), ("B2", "B2")):
        s = sq[label]
        o = {key: s[key] for key in ("dispatches", "wall_ms", "clock_GHz", "valu_issue_frac", "valu_issue_frac_2p4",
                                      "waves_per_simd", "wave_cycles_split", "mixed_adds_per_dispatch") if key in s}
        o["valu_lane_instructions_per_addition"] = s["valu_lane_instructions_per_unit"]
        if k in fetch and k in write:
            o["hbm_bytes_per_dispatch"] = (fetch[k]["FETCH_SIZE"] + write[k]["WRITE_SIZE"]) * 1024
            o["hbm_bytes_per_addition"] = round(o["hbm_bytes_per_dispatch"] / s["mixed_adds_per_dispatch"], 1)
        if k in tcp:
            t = tcp[k]
            o["utcl1_translation_miss_share"] = round(
                t["TCP_UTCL1_TRANSLATION_MISS_sum"] / (t["TCP_UTCL1_TRANSLATION_MISS_sum"] + t["TCP_UTCL1_TRANSLATION_HIT_sum"]), 3)
            o["utcl1_misses_per_addition"] = round(t["TCP_UTCL1_TRANSLATION_MISS_sum"] / s["mixed_adds_per_dispatch"], 2)
        res["kinds"][label] = o
    h = res["kinds"]["H"]
    res["hbm_bytes_per_launch"] = h.get("hbm_bytes_per_dispatch")
    res["valu_issue_frac"] = h["valu_issue_frac"]
    res["clock_GHz"] = h["clock_GHz"]
    res["valu_lane_instructions_per_addition"] = h["valu_lane_instructions_per_addition"]
    res["note"] = ("valu_issue_frac = SQ_INSTS_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the share of VALU issue "
                   "slots used at the clock the launch ran (clock_GHz = GRBM_GUI_ACTIVE / 8 / wall time); the counter "
                   "collection serialises dispatches, so each launch ran alone")
    txt = json.dumps(res, indent=1)
    open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:4])
