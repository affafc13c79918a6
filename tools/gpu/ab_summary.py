#!/usr/bin/env python3
"""Summarise tools/gpu/ab.sh logs: ms/proof, NTT 2^23 ms, accumulate frac per run."""
import glob, json
for f in sorted(glob.glob("gpurun_out/ab_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            k = d.get("kernels_config1", {})
            ntt = (k.get("ntt_roofline") or {}).get("2^23 (Venmo domain)", {})
            iso = (d.get("roofline") or {}).get("isolated_launch", {})
            print("%-28s ms/proof %.3f  ntt23 %s  acc_frac %.4f  iso %s" % (f.split("/")[-1], d["ms_per_step"], ntt.get("ms"),
                  d["roofline"]["frac"], iso.get("frac") if isinstance(iso, dict) else iso))
