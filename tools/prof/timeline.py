#!/usr/bin/env python3
"""Concurrent-stream timeline of one proof from a rocprofv3 kernel trace of bench.py:
kernels longer than 0.2 ms with start/end offsets, and how much of the proof span is
covered by the saturating kernels (accumulate, NTT, sort).
usage: timeline.py <run_kernel_trace.csv> [proof_index=2]"""
import csv, sys
from summarize import short


def main(path, idx=2):
    tr = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in tr if "k_build_abc" in r["Kernel_Name"]]
    t0, t1 = starts[idx], starts[idx + 1]
    rows = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, short(r["Kernel_Name"]))
            for r in tr if t0 <= int(r["Start_Timestamp"]) < t1]
    for s, e, k in rows:
        if e - s > 200000 or k.startswith(("k_hs_", "k_tlen", "k_lvl", "k_scan_", "k_bounds", "k_heavy", "k_task", "k_join")):
            print("%8.2f %8.2f %7.2f %s" % (s / 1e6, e / 1e6, (e - s) / 1e6, k))
    sat = [(s, e) for s, e, k in rows if k.startswith(("k_acc", "k_ntt", "rocprim", "k_hs_")) and e - s > 100000]
    ev = sorted([(s, 1) for s, e in sat] + [(e, -1) for s, e in sat])
    cur = last = cov = 0
    for t, d in ev:
        if cur > 0:
            cov += t - last
        cur += d
        last = t
    print("proof span %.2f ms, covered by saturating kernels %.2f ms" % ((t1 - t0) / 1e6, cov / 1e6))
    # GPU idle at the proof boundary: last kernel end of this proof -> first kernel of the next
    last_end = max(e for s, e, k in rows)
    print("last kernel of the proof ends at %.2f ms; GPU idle until the next proof's first kernel: %.2f ms"
          % (last_end / 1e6, (t1 - t0 - last_end) / 1e6))
    tail = sorted([(s, e, k) for s, e, k in rows if s >= last_end - 2e6], key=lambda x: x[0])
    for s, e, k in tail[-12:]:
        print("  tail %8.2f %8.2f %7.3f %s" % (s / 1e6, e / 1e6, (e - s) / 1e6, k))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
