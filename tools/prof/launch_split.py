#!/usr/bin/env python3
"""Per-launch-kind bucket-accumulate rooflines recomputed from a rocprofv3 kernel trace of bench.py
(VERDICT r3 item 1): the dispatches inside bench.py's "bench timed" ROCTx range (--marker-trace),
k_accumulate<Fq> split by workgroup count (the H plan's grid vs the witness plan's, from the bench
line's roofline_launches[...]["workgroups"]) and the witness launches by order (A, B1, C per proof),
k_accumulate<Fq2> = B2.  For each kind: the trace's average kernel duration and the frac it gives with
the bench line's own mixed additions per launch and peak -- to compare with the bench line's HIP-event
numbers.
usage: launch_split.py <kernel_trace.csv> <marker_api_trace.csv> <bench.json> [out.json]"""
import csv
import json
import sys
import os as _os, sys as _sys
_sys.path.insert(0, _os.path.dirname(_os.path.abspath(__file__)))
import benchline  # noqa: E402

MAC_PER_FPMUL, FPMUL_PER_MADD = 136, 11


def field(r, *names):
    for n in names:
        if n in r and r[n] != "":
            return r[n]
    raise KeyError("none of %s in %s" % (names, list(r)))


def timed_range(marker_csv):
    rows = list(csv.DictReader(open(marker_csv)))
    for r in rows:
        if any("bench timed" in str(v) for v in r.values()):
            return int(field(r, "Start_Timestamp")), int(field(r, "End_Timestamp"))
    raise SystemExit("no 'bench timed' range in %s (columns %s)" % (marker_csv, list(rows[0]) if rows else []))


def main(trace_csv, marker_csv, bench_json, out=None):
    line = benchline.detail(bench_json)
    per_kind = line["roofline_launches"]["per_kind"]
    peak = line["roofline"]["peak"]
    t0, t1 = timed_range(marker_csv)
    h_wg = set(per_kind["H"]["workgroups"])
    w_wg = set(per_kind["A"]["workgroups"]) if "A" in per_kind else set()
    if h_wg & w_wg:
        raise SystemExit("H and witness launches share a grid size %s: cannot split by grid" % (h_wg & w_wg))
    disp = []
    for r in csv.DictReader(open(trace_csv)):
        name = field(r, "Kernel_Name")
        if "k_accumulate" not in name:
            continue
        s, e = int(field(r, "Start_Timestamp")), int(field(r, "End_Timestamp"))
        if not (t0 <= s < t1):
            continue
        grid = int(field(r, "Grid_Size_X", "Grid_Size", "Grid_X"))
        wg = int(field(r, "Workgroup_Size_X", "Workgroup_Size", "Workgroup_X"))
        disp.append((s, e, "Fq2" in name, grid // wg))
    disp.sort()
    kinds = {"A": [], "B1": [], "C": [], "H": [], "B2": []}
    wi = 0
    for s, e, g2, blocks in disp:
        ms = (e - s) / 1e6
        if g2:
            kinds["B2"].append(ms)
        elif blocks in h_wg:
            kinds["H"].append(ms)
        elif blocks in w_wg:
            kinds[("A", "B1", "C")[wi % 3]].append(ms)
            wi += 1
        else:
            raise SystemExit("k_accumulate<Fq> dispatch with %d workgroups matches no launch kind" % blocks)
    res = {"trace": trace_csv, "timed_range_ns": [t0, t1], "peak": peak, "unit": line["roofline"]["unit"],
           "kinds": {}}
    for k, v in kinds.items():
        if not v or k not in per_kind:
            continue
        bl = per_kind[k]
        mac = bl["mixed_adds_per_launch"] * FPMUL_PER_MADD * MAC_PER_FPMUL * (3 if k == "B2" else 1)
        avg = sum(v) / len(v)
        frac = mac / (avg * 1e-3) / 1e12 / peak
        res["kinds"][k] = {"dispatches": len(v), "trace_avg_ms": round(avg, 4), "trace_frac": round(frac, 4),
                           "bench_avg_launch_ms": bl["avg_launch_ms"], "bench_frac": bl["frac"],
                           "frac_delta": round(frac - bl["frac"], 4) if bl["frac"] else None,
                           "bench_launches": bl["launches"]}
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
