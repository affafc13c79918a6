#!/usr/bin/env python3
"""Per-proof kernel time by kernel family from a serial (ZKP_SERIAL=1) rocprofv3 --stats
run of bench.py: load-time table kernels excluded, totals divided by the proof count
(number of k_build_abc launches).  usage: breakdown.py <run_kernel_stats.csv>"""
import collections, csv, re, sys

rows = list(csv.DictReader(open(sys.argv[1])))
proofs = sum(int(r["Calls"]) for r in rows if "k_build_abc" in r["Name"])
cat = collections.Counter()
for r in rows:
    n = r["Name"]
    if "extend_row" in n or "fixed_base" in n:
        continue
    m = re.search(r"(k_\w+)(<[^()]*?>)?\(", n)
    k = (m.group(1) + (m.group(2) or "").replace("zkp::", "")) if m else ("rocprim" if "rocprim" in n else n[:40])
    if "rocprim" in n:
        k = "rocprim (radix sort, scans)"
    cat[k] += float(r["TotalDurationNs"]) / proofs / 1e6
print("proofs %d, kernel time per proof %.3f ms" % (proofs, sum(cat.values())))
for k, v in cat.most_common():
    if v >= 0.01:
        print("%-48s %7.3f" % (k[:48], v))
