#!/usr/bin/env python3
"""Summarise the batch-affine measurement (tools/ubench/affine_bench.hip) from the committed
rocprofv3 rows under profiles/affine_r06/ into profiles/affine_r06.json.

Passes (each `affine_bench 1 <B list>`: every timed launch once after one warm-up launch, dispatches in
program order: k_gen_points, k_fill_table, k_vals, k_iota, k_acc x2 (baseline), then per B: k_pairs x2,
k_acc x2 (accumulate of the pair sums), k_check):
  sq128_counters.csv            SQ_* + GRBM_GUI_ACTIVE, B = 128
  sq512_counter_collection.csv  SQ_* + GRBM_GUI_ACTIVE, B = 512
  fetch_/write_counter_collection.csv  FETCH_SIZE / WRITE_SIZE (KB), B = 128, 512
Per addition: the baseline's task additions (entries - tasks), the pair kernel's affine additions (one per
pair), the pair-sum accumulate's task additions.  Issue share in the round-5 form (SQ_INSTS_VALU x 4 cycles
/ (1024 SIMDs x GRBM_GUI_ACTIVE / 8)) so that it compares with profiles/pmc_launch_r05.json.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D = os.path.join(ROOT, "profiles", "affine_r06")

NB, PER, SA, SB = 1 << 19, 208, 48, 21
ENTRIES = NB * PER
NP = ENTRIES // 2
TASKS_A = NB * ((PER + SA - 1) // SA)
TASKS_B = NB * ((PER // 2 + SB - 1) // SB)
ADDS = {"baseline": ENTRIES - TASKS_A, "pairs": NP, "pair_sums": NP - TASKS_B}


def _rows(name):
    """{dispatch: (kernel, {counter: value}, duration_ns)} from a counter-collection csv of either form."""
    out = collections.OrderedDict()
    with open(os.path.join(D, name)) as f:
        for r in csv.DictReader(f):
            disp = int(r["Dispatch_Id"])
            kern = r["Kernel_Name"].split("(")[0].replace("void ", "")
            val = float(r.get("Counter_Value") or r.get("Counter_Value_sum"))
            if "Duration_ns" in r:
                dur = float(r["Duration_ns"])
            else:
                dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            k, cs, d0 = out.get(disp, (kern, {}, dur))
            cs[r["Counter_Name"]] = cs.get(r["Counter_Name"], 0.0) + val
            out[disp] = (k, cs, max(d0, dur))
    return out


def _label(rows, bs):
    """Attach (phase, B) to the timed dispatches: the second of each warm-up/timed pair."""
    seq = [(d, k, cs, dur) for d, (k, cs, dur) in rows.items() if k in ("k_acc", "k_pairs<1>")]
    out = []
    acc = [x for x in seq if x[1] == "k_acc"]
    prs = [x for x in seq if x[1] == "k_pairs<1>"]
    out.append(("baseline", None, acc[1]))
    for i, b in enumerate(bs):
        out.append(("pairs", b, prs[2 * i + 1]))
        out.append(("pair_sums", b, acc[2 * i + 3]))
    return out


def summarise():
    res = {"workload": {"buckets": NB, "entries_per_bucket": PER, "table_rows": 13 << 23,
                        "baseline_task_additions": ADDS["baseline"], "affine_pair_additions": ADDS["pairs"],
                        "pair_sum_task_additions": ADDS["pair_sums"]},
           "sq": {}, "bytes": {}}
    for name, bs in (("sq128_counters.csv", [128]), ("sq512_counter_collection.csv", [512])):
        for phase, b, (_, _, cs, dur) in _label(_rows(name), bs):
            clk = cs["GRBM_GUI_ACTIVE"] / 8.0
            key = phase if b is None else "%s_B%d" % (phase, b)
            res["sq"].setdefault(key, {
                "ms": round(dur / 1e6, 3),
                "valu_lane_instr_per_addition": round(cs["SQ_INSTS_VALU"] * 64 / ADDS[phase], 1),
                "valu_issue_frac_4cyc": round(cs["SQ_INSTS_VALU"] * 4 / (1024 * clk), 3),
                "clock_GHz": round(clk / (dur * 1e-9) / 1e9, 3),
                "wait_inst_any_frac": round(cs["SQ_WAIT_INST_ANY"] / cs["SQ_WAVE_CYCLES"], 3),
                "wait_any_frac": round(cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"], 3),
                "waves": int(cs["SQ_WAVES"])})
    fetch = _label(_rows("fetch_counter_collection.csv"), [128, 512])
    write = _label(_rows("write_counter_collection.csv"), [128, 512])
    for (phase, b, (_, _, fc, _)), (_, _, (_, _, wc, _)) in zip(fetch, write):
        key = phase if b is None else "%s_B%d" % (phase, b)
        byt = (fc["FETCH_SIZE"] + wc["WRITE_SIZE"]) * 1024
        res["bytes"][key] = {"fetch_GB": round(fc["FETCH_SIZE"] * 1024 / 1e9, 3),
                             "write_GB": round(wc["WRITE_SIZE"] * 1024 / 1e9, 3),
                             "bytes_per_addition": round(byt / ADDS[phase], 1)}
    base = res["sq"]["baseline"]
    # the pair pass replaces NP of the baseline's additions; at the baseline's own issue share and clock the
    # pair kernel plus the accumulate of the pair sums would take (instructions ratio) x the baseline time
    proj = {}
    for b in (128, 512):
        p, s = res["sq"].get("pairs_B%d" % b), res["sq"].get("pair_sums_B%d" % b)
        if not (p and s):
            continue
        instr = p["valu_lane_instr_per_addition"] * ADDS["pairs"] + s["valu_lane_instr_per_addition"] * ADDS["pair_sums"]
        instr0 = base["valu_lane_instr_per_addition"] * ADDS["baseline"]
        proj["B%d" % b] = {"instructions_vs_baseline": round(instr / instr0, 4),
                           "measured_total_ms": round(p["ms"] + s["ms"], 3),
                           "ms_if_issued_like_baseline": round(instr / instr0 * base["ms"], 3),
                           "baseline_ms": base["ms"]}
    res["projection_at_baseline_issue"] = proj
    return res


def main():
    res = summarise()
    out = os.path.join(ROOT, "profiles", "affine_r06.json")
    if "--check" in sys.argv:
        with open(out) as f:
            assert json.load(f) == json.loads(json.dumps(res)), "profiles/affine_r06.json is stale"
        return
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
