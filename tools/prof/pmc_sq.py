#!/usr/bin/env python3
"""Per-kernel SQ counter summary of a rocprofv3 --pmc CSV (SQ_WAVES, SQ_INSTS_VALU,
SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, SQ_ACTIVE_INST_VALU, SQ_WAIT_INST_ANY, SQ_WAIT_ANY,
SQ_ACTIVE_INST_ANY).  VALU lane-instructions/s = SQ_INSTS_VALU * 64 / kernel duration,
compared with the measured issue peak (profiles/ubench_r01.txt: v_mul_lo_u32 /
v_add_co_u32 35.4 T lane-ops/s; v_mad_u64_u32 32.3 T).
usage: pmc_sq.py <run_counter_collection.csv> [json_out]"""
import collections, csv, json, sys
from summarize import short

PEAK_LANE_OPS = 35.4e12


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(dict)
    for r in rows:
        d = (r["Dispatch_Id"])
        disp[d]["k"] = short(r["Kernel_Name"])
        disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
        disp[d]["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        disp[d]["vgpr"] = int(r["VGPR_Count"]) + int(r.get("Accum_VGPR_Count", 0) or 0)
    for d in disp.values():
        k = d["k"]
        per[k]["n"] += 1
        for key, v in d.items():
            if key not in ("k", "vgpr"):
                per[k][key] += v
        per[k]["vgpr"] = d["vgpr"]
    res = {}
    for k, v in sorted(per.items(), key=lambda x: -x[1]["ns"]):
        if v["ns"] < 1e6:
            continue
        lane_ops = v["SQ_INSTS_VALU"] * 64 / (v["ns"] * 1e-9)
        res[k] = {
            "launches": int(v["n"]), "ms_per_launch": round(v["ns"] / v["n"] / 1e6, 4), "vgpr+agpr": int(v["vgpr"]),
            "valu_insts_per_launch": v["SQ_INSTS_VALU"] / v["n"],
            "valu_lane_ops_per_s": lane_ops, "valu_issue_frac_of_peak": round(lane_ops / PEAK_LANE_OPS, 3),
            "active_valu_per_wave_cycle": round(v["SQ_ACTIVE_INST_VALU"] / max(1, v["SQ_WAVE_CYCLES"]), 3),
            "wait_inst_any_frac": round(v["SQ_WAIT_INST_ANY"] / max(1, v["SQ_WAVE_CYCLES"]), 3),
            "wait_any_frac": round(v["SQ_WAIT_ANY"] / max(1, v["SQ_WAVE_CYCLES"]), 3),
        }
        print("%-34s n=%3d %8.3f ms  VALU %6.2f T lane-op/s (%.0f%% of peak)  vgpr %d  wait_inst %.2f wait %.2f" % (
            k[:34], v["n"], v["ns"] / v["n"] / 1e6, lane_ops / 1e12, 100 * lane_ops / PEAK_LANE_OPS, v["vgpr"],
            res[k]["wait_inst_any_frac"], res[k]["wait_any_frac"]))
    if out:
        json.dump({"source": path, "peak_lane_ops_per_s": PEAK_LANE_OPS, "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
