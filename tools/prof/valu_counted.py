#!/usr/bin/env python3
"""Counted VALU busy from one rocprofv3 --pmc pass per workload with SQ_INSTS_VALU,
SQ_ACTIVE_INST_VALU2, SQ_INSTS_VALU_INT32, SQ_INSTS_VALU_INT64, SQ_ACTIVE_INST_VALU, SQ_THREAD_CYCLES_VALU,
SQ_WAVES, SQ_WAVE_CYCLES and GRBM_GUI_ACTIVE (tools/gpu/pmc.sh valu ntt + ubench.sh valu_rates (the round-6 call: f1362da:tools/gpu/r6/valu.sh); raw rows in profiles/pmc_valu_r06/).

The round-5 issue model priced every VALU instruction at one quad-cycle (4 clocks) of its SIMD.  gfx950
executes the full-rate class (v_and/or/xor/add/sub/mov/lshrrev_b32 ... e32, v_bitop3) in 2 clocks, but a
single wave issues at most one VALU instruction per quad-cycle: two full-rate instructions share a quad-
cycle only when two WAVES issue them together, which SQ_ACTIVE_INST_VALU2 counts ("quad-cycles in which two
VALU instructions are issued").  So the VALU's busy quad-cycles are SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2,
measured, not modelled:
    valu_busy_counted = (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
Calibration (the same pass over tools/ubench/valu_rates.hip, one opcode per kernel, 4 waves per SIMD):
full-rate opcodes co-issue in ~0.9 of their instructions (VALU2 / VALU ~0.45), every other opcode in
< 0.002.  SQ_ACTIVE_INST_VALU equals SQ_INSTS_VALU in every row (it counts instructions, not cycles), so it
is not used.
usage: valu_counted.py [--check]   (writes / checks profiles/pmc_valu_r06.json)"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D = os.path.join(ROOT, "profiles", "pmc_valu_r06")
SIMDS = 1024


def dispatches(name):
    out = collections.OrderedDict()
    for r in csv.DictReader(open(os.path.join(D, name))):
        e = out.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"],
                                                     "blocks": int(r["Grid_Size"]) // int(r["Workgroup_Size"])})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return list(out.values())


def line(ds, work=None):
    keys = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64",
            "GRBM_GUI_ACTIVE", "ns")
    s = {k: sum(d[k] for d in ds) for k in keys}
    cyc = s["GRBM_GUI_ACTIVE"] / 8.0
    i = s["SQ_INSTS_VALU"]
    o = {"dispatches": len(ds),
         "clock_GHz": round(cyc / s["ns"], 3),
         "valu_issue_frac_4cyc": round(i * 4 / (SIMDS * cyc), 4),
         "dual_issue_quad_cycles_per_instr": round(s["SQ_ACTIVE_INST_VALU2"] / i, 4),
         "valu_busy_counted": round((i - s["SQ_ACTIVE_INST_VALU2"]) * 4 / (SIMDS * cyc), 4),
         "int32_share": round(s["SQ_INSTS_VALU_INT32"] / i, 4),
         "int64_share": round(s["SQ_INSTS_VALU_INT64"] / i, 4)}
    if work:
        o["valu_lane_instructions_per_unit"] = round(i * 64 / len(ds) / work, 1)
    return o


def summarise():
    res = {"source": "profiles/pmc_valu_r06/ (tools/gpu/pmc.sh valu ntt + ubench.sh valu_rates (the round-6 call: f1362da:tools/gpu/r6/valu.sh))", "opcodes_alone": {}, "accumulate": {},
           "ntt": {}}
    for d in dispatches("ub_counter_collection.csv"):
        op = re.sub(r"^k_", "", d["name"].split("(")[0])
        if op not in res["opcodes_alone"]:  # first launch per opcode (the tool launches each twice)
            res["opcodes_alone"][op] = line([d])
    kinds = json.load(open(os.path.join(D, "acc_launch_kinds.json")))
    hwg, wwg = set(kinds["H"]["workgroups"]), set(kinds["A"]["workgroups"])
    groups = collections.defaultdict(list)
    for d in dispatches("acc_counter_collection.csv"):
        if "k_accumulate" not in d["name"]:
            continue
        k = "B2" if "Fq2" in d["name"] else ("H" if d["blocks"] in hwg else ("witness (A, B1, C)" if d["blocks"] in wwg else None))
        if k:
            groups[k].append(d)
    adds = {"H": kinds["H"]["mixed_adds_per_launch"], "witness (A, B1, C)": kinds["A"]["mixed_adds_per_launch"],
            "B2": kinds["B2"]["mixed_adds_per_launch"]}
    for k, ds in sorted(groups.items()):
        res["accumulate"][k] = line(ds, adds[k])
    for n in (23, 20):
        g = collections.defaultdict(list)
        for d in dispatches("ntt%d_counter_collection.csv" % n):
            m = re.search(r"k_ntt<(\d+)", d["name"])
            if m:
                g["k_ntt<%s>" % m.group(1)].append(d)
        res["ntt"]["2^%d" % n] = {k: line(v) for k, v in sorted(g.items())}
    return res


def main():
    res = summarise()
    out = os.path.join(ROOT, "profiles", "pmc_valu_r06.json")
    if "--check" in sys.argv:
        assert json.load(open(out)) == json.loads(json.dumps(res)), "profiles/pmc_valu_r06.json is stale"
        return
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("accumulate", "ntt")}, indent=1))


if __name__ == "__main__":
    main()
