#!/usr/bin/env python3
"""One library's entry of profiles/ntt_issue_r05.json from the k_ntt rows of one rocprofv3 --pmc pass
(SQ + GRBM, 273c6e8:tools/gpu/r5/pmc.sh / ntt_root1.sh) of `tools/probe/ntt_run.py <k> 20`: per k_ntt mode the
clock, VALU issue and wave-cycle split of tools/prof/pmc_stall.py plus VALU lane-instructions per
element (SQ_INSTS_VALU x 64 / n); per coset extension 2 x k_ntt<0> + 2 x k_ntt<1> + k_ntt<2>.
usage: ntt_issue5.py <run_counter_collection.csv> <log_n>"""
import collections
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_stall  # noqa: E402

PER_EXTENSION = {"k_ntt<0>": 2, "k_ntt<1>": 2, "k_ntt<2>": 1}


def entry(path, k):
    n = 1 << k
    groups = collections.defaultdict(list)
    for d in pmc_stall.rows_by_dispatch(path):
        m = re.search(r"k_ntt<(\d+)", d["name"].replace(" ", ""))
        if m:
            groups["k_ntt<%s>" % m.group(1)].append(d)
    kernels = {}
    for kk, ds in sorted(groups.items()):
        s = pmc_stall.summarize(ds)
        o = {key: s[key] for key in ("dispatches", "wall_ms", "clock_GHz", "valu_issue_frac", "waves_per_simd",
                                      "wave_cycles_split") if key in s}
        o["valu_lane_instr_per_element"] = round(s["counters_avg_per_dispatch"]["SQ_INSTS_VALU"] * 64 / n, 1)
        kernels[kk] = o
    tot = sum(PER_EXTENSION[kk] * v["valu_lane_instr_per_element"] for kk, v in kernels.items())
    return {"kernels": kernels, "coset_extension_valu_lane_instr_per_element": round(tot, 1)}


if __name__ == "__main__":
    print(json.dumps(entry(sys.argv[1], int(sys.argv[2])), indent=1))
