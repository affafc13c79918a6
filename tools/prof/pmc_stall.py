#!/usr/bin/env python3
"""Where a kernel's cycles go, per bucket-accumulate launch kind (or per NTT kernel), from ONE
rocprofv3 --pmc pass with SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT (the counter collection
serialises dispatches, so every launch runs alone).  Per dispatch (averaged per kind):

* effective clock = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / dispatch wall time
  (/opt/skills/guides/MI355X_MICROARCH.md, DVFS give-back);
* valu_issue_frac = SQ_INSTS_VALU x 4 cycles (one wave64 VALU instruction per SIMD per 4 clocks)
  / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the share of the SIMDs' VALU issue slots used, at the clock
  the kernel actually ran;
* valu_issue_frac_2p4 = the same against 2.4 GHz x wall time (the issue ceiling at the max clock);
* the wave-cycle split: SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue
  stalls), SQ_ACTIVE_INST_ANY (issuing), each / SQ_WAVE_CYCLES (the guide: disjoint, ~ sum to 1);
* waves per SIMD = SQ_WAVE_CYCLES (quad-cycles) x 4 / (1024 x cycles).

usage: pmc_stall.py acc <bench.json> <counter_collection.csv> [out.json]
       pmc_stall.py ntt <counter_collection.csv> [out.json]"""
import collections
import csv
import json
import re
import sys
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
import benchline  # noqa: E402

SIMDS = 1024
MAXCLK_GHZ = 2.4


def rows_by_dispatch(path):
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = disp[r.get("Dispatch_Id") or r.get("Correlation_Id")]
        d["name"] = r["Kernel_Name"]
        grid = int(r.get("Grid_Size") or r.get("Grid_Size_X"))
        wg = int(r.get("Workgroup_Size") or r.get("Workgroup_Size_X"))
        d["blocks"] = grid // wg
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(disp.values())


def summarize(ds, work=None):
    n = len(ds)
    keys = set().union(*(d.keys() for d in ds)) - {"name", "blocks"}
    avg = {k: sum(d.get(k, 0.0) for d in ds) / n for k in keys}
    o = {"dispatches": n, "wall_ms": round(avg["ns"] / 1e6, 4)}
    cyc = avg["GRBM_GUI_ACTIVE"] / 8.0 if "GRBM_GUI_ACTIVE" in avg else None
    if cyc:
        o["clock_GHz"] = round(cyc / avg["ns"], 3)
    if "SQ_INSTS_VALU" in avg:
        if cyc:
            o["valu_issue_frac"] = round(avg["SQ_INSTS_VALU"] * 4 / (SIMDS * cyc), 4)
        o["valu_issue_frac_2p4"] = round(avg["SQ_INSTS_VALU"] * 4 / (SIMDS * MAXCLK_GHZ * avg["ns"]), 4)
        if work:
            o["valu_lane_instructions_per_unit"] = round(avg["SQ_INSTS_VALU"] * 64 / work, 1)
    if cyc and "SQ_ACTIVE_INST_VALU" in avg:
        pass  # SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU (it counts instructions): not a cycle measure
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        if cyc:
            o["waves_per_simd"] = round(wc * 4 / (SIMDS * cyc), 3)
        o["wave_cycles_split"] = {k.lower()[3:]: round(avg[k] / wc, 4)
                                  for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in avg}
    o["counters_avg_per_dispatch"] = {k: v for k, v in sorted(avg.items()) if k != "ns"}
    return o


def acc(bench_json, path, out=None):
    line = benchline.detail(bench_json)
    kinds = line["roofline_launches"]["per_kind"]
    h_wg = set(kinds["H"]["workgroups"])
    w_wg = set(kinds["A"]["workgroups"])
    groups = collections.defaultdict(list)
    for d in rows_by_dispatch(path):
        if "k_accumulate" not in d["name"]:
            continue
        k = "B2" if "Fq2" in d["name"] else ("H" if d["blocks"] in h_wg else ("W" if d["blocks"] in w_wg else None))
        if k:
            groups[k].append(d)
    adds = {"H": kinds["H"]["mixed_adds_per_launch"], "W": kinds["A"]["mixed_adds_per_launch"],
            "B2": kinds["B2"]["mixed_adds_per_launch"]}
    res = {"source": path, "bench": bench_json, "kinds": {}}
    for k, ds in groups.items():
        res["kinds"]["witness (A, B1, C)" if k == "W" else k] = dict(summarize(ds, adds[k]), mixed_adds_per_dispatch=adds[k])
    emit(res, out)


def ntt(path, out=None):
    groups = collections.defaultdict(list)
    for d in rows_by_dispatch(path):
        if "k_ntt" in d["name"]:
            m = re.search(r"k_ntt<(\d+)|k_nttILi(\d+)E", d["name"])
            groups["k_ntt<%s>" % (m.group(1) or m.group(2) if m else "?")].append(d)
    res = {"source": path, "kernels": {k: summarize(v) for k, v in groups.items()}}
    emit(res, out)


def emit(res, out):
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "acc":
        acc(*sys.argv[2:])
    else:
        ntt(*sys.argv[2:])
