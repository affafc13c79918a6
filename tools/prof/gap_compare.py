#!/usr/bin/env python3
"""Back-to-back vs gapped staged proofs in a rocprofv3 kernel trace of tools/probe/latency_probe.py:
proofs delimited by k_build_abc; for each proof the idle time before it, its span (first kernel start
to last kernel end) and, per kernel, the summed duration; then the per-kernel difference between the
median gapped proof (idle > 1 ms before it) and the median back-to-back one (idle < 0.5 ms) -- where
the ~1 ms of a proof started after a pause goes.
usage: gap_compare.py <run_kernel_trace.csv> [top=15]"""
import collections
import csv
import re
import statistics
import sys


def short(n):
    n = n.replace("zkp::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*", "", n)
    return n.replace("zkp::Fe<zkp::FqCfg>", "Fq").replace("zkp::Fq2", "Fq2").strip()


def main(path, top=15):
    tr = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(tr) if "k_build_abc" in r["Kernel_Name"]]
    proofs = []
    for j, i0 in enumerate(starts):
        i1 = starts[j + 1] if j + 1 < len(starts) else len(tr)
        ks = tr[i0:i1]
        s = int(ks[0]["Start_Timestamp"])
        e = max(int(r["End_Timestamp"]) for r in ks)
        prev_end = max(int(r["End_Timestamp"]) for r in tr[:i0]) if i0 else None
        per = collections.defaultdict(float)
        for r in ks:
            per[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        proofs.append({"gap": (s - prev_end) / 1e6 if prev_end else None, "span": (e - s) / 1e6, "per": per})
    b2b = [p for p in proofs if p["gap"] is not None and p["gap"] < 0.5]
    gapped = [p for p in proofs if p["gap"] is not None and p["gap"] > 1.0]
    print("proofs %d: back-to-back %d (span median %.3f ms), after > 1 ms idle %d (span median %.3f ms)"
          % (len(proofs), len(b2b), statistics.median(p["span"] for p in b2b) if b2b else 0, len(gapped),
             statistics.median(p["span"] for p in gapped) if gapped else 0))
    if not (b2b and gapped):
        return
    names = set().union(*[p["per"] for p in proofs])
    diff = []
    for n in names:
        a = statistics.median(p["per"].get(n, 0.0) for p in b2b)
        b = statistics.median(p["per"].get(n, 0.0) for p in gapped)
        diff.append((b - a, n, a, b))
    diff.sort(reverse=True)
    print("%-34s %10s %10s %10s" % ("kernel (summed per proof)", "b2b ms", "gapped ms", "diff"))
    for d, n, a, b in diff[:top]:
        print("%-34s %10.3f %10.3f %+10.3f" % (n[:34], a, b, d))
    print("sum of per-kernel differences %+.3f ms" % sum(d for d, *_ in diff))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15)
