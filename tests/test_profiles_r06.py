"""Round-6 profile summaries recompute from the raw rocprofv3 rows committed beside them (no GPU needed).

* profiles/affine_r06.json (the batch-affine measurement): tools/prof/affine_summary.py
  over profiles/affine_r06/*.csv -- per-addition VALU instructions, issue share, HBM bytes, and the projection
  of the affine pair pass at the XYZZ kernel's own issue rate.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_affine_summary_recomputes():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "affine_summary.py"), "--check"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]


def test_affine_measurement_verdict():
    """What DESIGN.md §5 'Batch-affine accumulation' states: every measured pair pass + accumulate is slower
    than the XYZZ accumulate on the same buckets (and bit-identical in every bucket), the pair kernel runs
    latency-bound (issue share < 0.2), and it moves > 3x the XYZZ kernel's bytes per addition."""
    d = json.load(open(os.path.join(ROOT, "profiles", "affine_r06.json")))
    base = d["sq"]["baseline"]
    for b in ("B128", "B512"):
        assert d["projection_at_baseline_issue"][b]["measured_total_ms"] > 3 * base["ms"]
        assert d["sq"]["pairs_" + b]["valu_issue_frac_4cyc"] < 0.2
        assert d["bytes"]["pairs_" + b]["bytes_per_addition"] > 3 * d["bytes"]["baseline"]["bytes_per_addition"]
    for line in open(os.path.join(ROOT, "profiles", "affine_r06", "bench.txt")):
        r = json.loads(line)
        if "buckets_differing" in r:
            assert r["buckets_differing"] == 0 and r["vs_baseline"] > 1.0
