#!/usr/bin/env python3
"""Per-proof kernel breakdown of a rocprofv3 --kernel-trace CSV of bench.py
(proofs delimited by k_build_abc; bench.py runs 1 warmup + `timed` proofs + 1 PCIe proof).
usage: breakdown.py <run_kernel_trace.csv> [timed=4] [--launches]"""
import collections, csv, sys
from summarize import short


def main(path, timed=4, launches=False):
    tr = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in tr if "k_build_abc" in r["Kernel_Name"]]
    t0, t1 = starts[1], starts[1 + timed]
    per = collections.defaultdict(lambda: [0, 0.0])
    rows = []
    for r in tr:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            k = short(r["Kernel_Name"])
            per[k][0] += 1
            per[k][1] += (e - s) / 1e6
            if s < starts[2]:
                rows.append((k, int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0), (e - s) / 1e3, (s - t0) / 1e3))
    tot = sum(v[1] for v in per.values())
    print("wall/proof %.2f ms  kernel-sum/proof %.2f ms" % ((t1 - t0) / timed / 1e6, tot / timed))
    for k, v in sorted(per.items(), key=lambda x: -x[1][1]):
        print("%-44s %6.1f %9.3f" % (k[:44], v[0] / timed, v[1] / timed))
    if launches:
        for k, g, us, at in rows:
            print("%10.1f %-40s grid=%-10d %9.1f us" % (at, k[:40], g, us))


if __name__ == "__main__":
    a = [x for x in sys.argv[1:] if not x.startswith("--")]
    main(a[0], int(a[1]) if len(a) > 1 else 4, "--launches" in sys.argv)
