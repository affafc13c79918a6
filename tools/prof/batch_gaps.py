#!/usr/bin/env python3
"""Where the batch line loses against the staged headline: from one rocprofv3 --kernel-trace
--marker-trace of bench.py, the dispatches inside its "bench timed" (staged proofs, witness in HBM) and
"batch timed" (zkp_prove_batch from host memory) ROCTx ranges, each summarised as
* proofs (k_build_abc dispatches) and ms per proof;
* GPU busy: the union of all kernel intervals over the range, and the idle time between kernels
  (total, and in gaps longer than 0.1 ms);
* the median duration of each accumulate launch kind (H, A/B1/C, B2: by grid size and field, as
  launch_split.py) and of the NTT / sort / witness-expansion kernels, so that a kernel slowed by the
  concurrent transfer shows next to its staged twin.
usage: batch_gaps.py <kernel_trace.csv> <marker_api_trace.csv> [out.json]"""
import collections
import csv
import json
import statistics
import sys


def ranges(marker_csv):
    out = {}
    for r in csv.DictReader(open(marker_csv)):
        name = r.get("Function") or r.get("Name") or ""
        if name in ("bench timed", "batch timed"):
            out[name] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    return out


def kind(name, grid, wg):
    if "k_accumulate" in name:
        if "Fq2" in name:
            return "k_accumulate B2"
        return "k_accumulate (grid %d)" % (grid // wg)
    for k in ("k_ntt<0", "k_ntt<1", "k_ntt<2", "k_build_abc", "k_join_abc", "k_hs_scatter1", "k_witness_unpack",
              "k_merge_final", "k_reduce_segments", "k_subset"):
        if k in name.replace(" ", ""):
            return k
    return None


def summarize(rows, t0, t1):
    ks = sorted((s, e, n, g, w) for s, e, n, g, w in rows if t0 <= s < t1)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _, _, _ in ks:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = t1 - t0
    proofs = sum(1 for _, _, n, _, _ in ks if "k_build_abc" in n)
    dur = collections.defaultdict(list)
    for s, e, n, g, w in ks:
        k = kind(n, g, w)
        if k:
            dur[k].append((e - s) / 1e6)
    acc = {k: v for k, v in dur.items() if k.startswith("k_accumulate (grid")}
    # drift over the range: per tenth of the span, the proofs started and the median H-launch time
    # (the accumulate grid with the longest launches), to separate a steady cost from a slow clock-down
    hk = max(acc, key=lambda k: statistics.median(acc[k])) if acc else None
    deciles = []
    for q in range(10):
        a, b = t0 + span * q // 10, t0 + span * (q + 1) // 10
        hs = [(e - s) / 1e6 for s, e, n, g, w in ks if a <= s < b and kind(n, g, w) == hk]
        deciles.append({"proofs_started": sum(1 for s, _, n, _, _ in ks if a <= s < b and "k_build_abc" in n),
                        "h_launch_median_ms": round(statistics.median(hs), 3) if hs else None})
    # the H launch: the accumulate grid with the most additions ~ the largest median duration
    return {"span_ms": round(span / 1e6, 2), "proofs": proofs,
            "ms_per_proof": round(span / 1e6 / proofs, 3) if proofs else None,
            "gpu_busy_frac": round(busy / span, 4), "idle_ms_per_proof": round((span - busy) / 1e6 / max(proofs, 1), 3),
            "idle_in_gaps_over_0.1ms_per_proof": round(sum(g for g in gaps if g > 100000) / 1e6 / max(proofs, 1), 3),
            "kernel_median_ms": {k: round(statistics.median(v), 4) for k, v in sorted(dur.items()) if len(v) >= 3},
            "accumulate_grids": sorted(acc, key=lambda k: -statistics.median(acc[k])),
            "by_tenth_of_span": deciles}


def main(trace_csv, marker_csv, out=None):
    rs = ranges(marker_csv)
    rows = []
    for r in csv.DictReader(open(trace_csv)):
        g = int(r.get("Grid_Size_X") or r.get("Grid_Size"))
        w = int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size"))
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], g, w))
    res = {name: summarize(rows, *rng) for name, rng in rs.items()}
    txt = json.dumps(res, indent=1)
    print(txt)
    if out:
        open(out, "w").write(txt + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
