#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py into per-proof kernel time
(proofs delimited by k_build_abc dispatches) + PMC traffic of k_accumulate.
usage: summarize.py <trace_kernel_trace.csv> <pmc_fetch.csv> <pmc_write.csv> <out.json> [timed_proofs]"""
import collections, csv, json, re, sys


def short(n):
    n = n.replace("zkp::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*", "", n)
    n = n.replace("zkp::Fe<zkp::FqCfg>", "Fq").replace("zkp::Fq2", "Fq2")
    if "rocprim" in n:
        m = re.search(r"detail::(\w+)", n)
        n = "rocprim::" + (m.group(1) if m else "kernel")
    return n.strip()


def main(tr_csv, fetch_csv, write_csv, out, timed=4):
    tr = sorted(csv.DictReader(open(tr_csv)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [int(r["Start_Timestamp"]) for r in tr if "k_build_abc" in r["Kernel_Name"]]
    # bench.py: 1 warmup proof, `timed` timed proofs, 1 PCIe-inclusive proof
    t0, t1 = starts[1], starts[1 + timed]
    per = collections.defaultdict(lambda: [0, 0.0])
    for r in tr:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            k = short(r["Kernel_Name"])
            per[k][0] += 1
            per[k][1] += (e - s) / 1e6
    rows = sorted(((k, c / timed, ms / timed, ms / c) for k, (c, ms) in per.items()), key=lambda x: -x[2])
    busy = sum(x[2] for x in rows)
    res = {"source": tr_csv, "timed_proofs": timed, "wall_ms_per_proof": (t1 - t0) / 1e6 / timed,
           "kernel_ms_per_proof_sum_over_streams": busy,
           "kernels": [{"kernel": k, "launches_per_proof": round(c, 2), "ms_per_proof": round(m, 3),
                        "avg_ms_per_launch": round(a, 4)} for k, c, m, a in rows]}

    def pmc(path):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            vals[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
        return vals
    try:
        f, w = pmc(fetch_csv), pmc(write_csv)
        acc = {}
        for k in f:
            fk, wk = f[k], w.get(k, [0])
            fetch_kb = sum(fk) / len(fk)
            write_kb = sum(wk) / len(wk)
            # MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of 16-B/lane loads on gfx950 -> x2; units KB
            acc[k] = {"launches": len(fk), "FETCH_SIZE_kb_avg": fetch_kb, "WRITE_SIZE_kb_avg": write_kb,
                      "hbm_bytes_per_launch_corrected": (2 * fetch_kb + write_kb) * 1024}
        res["pmc"] = acc
    except FileNotFoundError:
        pass
    json.dump(res, open(out, "w"), indent=1)
    print("wall ms/proof %.2f  kernel-ms/proof %.2f" % (res["wall_ms_per_proof"], busy))
    for k, c, m, a in rows[:25]:
        print("%-34s %6.2f launches %8.3f ms/proof  %8.4f ms/launch" % (k[:34], c, m, a))
    for k, v in res.get("pmc", {}).items():
        print("PMC", k, v)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4], int(sys.argv[5]) if len(sys.argv) > 5 else 4)
