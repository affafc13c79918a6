#!/usr/bin/env python3
"""NTT issue rate per launch kind, from a rocprofv3 kernel trace and a PMC pass of the same
command (tools/probe/ntt_run.py; 273c6e8:tools/gpu/r4/nttpmc.sh): per k_ntt kind, the median launch
duration, VALU lane-instructions per element and the issue rate (wave-level VALU instructions per
microsecond per CU), and per coset extension the credited butterfly products per instruction.
The ratio of the 2^20 and 2^23 rooflines factors into (credited products per instruction) x
(instructions per unit time): VERDICT r3 item 7.
usage: ntt_issue.py <dir with nttpmc20/, nttpmc23/, ntttr20/, ntttr23/>"""
import collections
import csv
import json
import os
import re
import statistics
import sys

CUS = 256


def kind(name):
    m = re.search(r"k_ntt<(\d+), ?(\d+)>", name)
    return "k_ntt<%s>" % m.group(1) if m else None


def main(d):
    out = {}
    for k in (20, 23):
        n = 1 << k
        dur = collections.defaultdict(list)
        for r in csv.DictReader(open(os.path.join(d, "ntttr%d" % k, "run_kernel_trace.csv"))):
            kk = kind(r["Kernel_Name"])
            if kk:
                dur[kk].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        pmc = collections.defaultdict(lambda: collections.defaultdict(float))
        kinds = {}
        for r in csv.DictReader(open(os.path.join(d, "nttpmc%d" % k, "run_counter_collection.csv"))):
            kk = kind(r["Kernel_Name"])
            if kk:
                pmc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                kinds[r["Dispatch_Id"]] = kk
        valu = collections.defaultdict(list)
        for did, c in pmc.items():
            valu[kinds[did]].append(c["SQ_INSTS_VALU"])
        res = {}
        for kk in sorted(dur):
            us = statistics.median(dur[kk])
            vi = statistics.median(valu[kk])
            res[kk] = {"launches": len(dur[kk]), "us_median": round(us, 1), "valu_lane_instr_per_element": round(vi * 64 / n),
                       "valu_wave_instr_per_us_per_cu": round(vi / us / CUS)}
        # one coset extension = 2 k_ntt<0> + 1 k_ntt<2> + 2 k_ntt<1>
        per = {"k_ntt<0>": 2, "k_ntt<2>": 1, "k_ntt<1>": 2}
        tot_us = sum(res[kk]["us_median"] * m for kk, m in per.items())
        tot_vi = sum(statistics.median(valu[kk]) * m for kk, m in per.items())
        res["coset_extension"] = {"kernel_us": round(tot_us, 1), "valu_lane_instr_per_element": round(tot_vi * 64 / n),
                                  "credited_products_per_element": k + 1,
                                  "credited_products_per_kilo_lane_instr": round(1000 * (k + 1) / (tot_vi * 64 / n), 3),
                                  "valu_wave_instr_per_us_per_cu": round(tot_vi / tot_us / CUS)}
        out["2^%d" % k] = res
    a, b = out["2^20"]["coset_extension"], out["2^23"]["coset_extension"]
    out["ratio_20_over_23"] = {"products_per_instr": round(a["credited_products_per_kilo_lane_instr"] / b["credited_products_per_kilo_lane_instr"], 3),
                               "issue_rate": round(a["valu_wave_instr_per_us_per_cu"] / b["valu_wave_instr_per_us_per_cu"], 3)}
    out["ratio_20_over_23"]["product"] = round(out["ratio_20_over_23"]["products_per_instr"] * out["ratio_20_over_23"]["issue_rate"], 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
