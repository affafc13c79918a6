#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc passes (one dispatch = one sample).
usage: pmc_by_kernel.py <kernel-regex> <run_counter_collection.csv>..."""
import collections, csv, re, sys


def main(pat, files):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in files:
        for r in csv.DictReader(open(f)):
            m = re.search(pat, r["Kernel_Name"])
            if not m:
                continue
            k, c = m.group(0), r["Counter_Name"]
            agg[k][c] += float(r["Counter_Value"])
            disp[k][c].add(r["Dispatch_Id"])
    for k in sorted(agg):
        print(k)
        for c, v in sorted(agg[k].items()):
            print("   %-22s %16.0f" % (c, v / max(1, len(disp[k][c]))))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
