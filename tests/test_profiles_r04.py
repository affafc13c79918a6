"""The committed round-4 rocprof evidence reproduces the bench line's per-launch rooflines
(VERDICT r3 item 1): tools/prof/launch_split.py over profiles/rocprof_r04_accumulate_trace.csv
(k_accumulate dispatches of a rocprofv3 --kernel-trace of bench.py) and
profiles/rocprof_r04_marker_trace.csv (bench.py's ROCTx "bench timed" range) recomputes every launch
kind's frac of profiles/bench_r04_rocprof_run.json (the bench line of that same invocation) within
0.03.  CPU-only (reads committed files)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")


def test_launch_split_reproduces_bench_fracs(tmp_path):
    out = tmp_path / "split.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "launch_split.py"),
                    os.path.join(P, "rocprof_r04_accumulate_trace.csv"), os.path.join(P, "rocprof_r04_marker_trace.csv"),
                    os.path.join(P, "bench_r04_rocprof_run.json"), str(out)], check=True, capture_output=True, timeout=120)
    res = json.loads(out.read_text())
    assert set(res["kinds"]) == {"A", "B1", "C", "H", "B2"}
    for kind, v in res["kinds"].items():
        assert v["dispatches"] == v["bench_launches"], kind
        assert abs(v["frac_delta"]) <= 0.03, (kind, v)


def test_ntt_issue_rate_recomputes_from_committed_counters():
    """DESIGN §5 NTT: the 2^20 / 2^23 roofline ratio factors into credited
    products per instruction x issue rate; tools/prof/ntt_issue.py over the committed (k_ntt rows
    only) kernel traces and SQ counter passes reproduces profiles/ntt_issue_r04.json."""
    res = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "ntt_issue.py"),
                          os.path.join(P, "ntt_issue_r04")], check=True, capture_output=True, text=True, timeout=120)
    got = json.loads(res.stdout)
    assert got == json.load(open(os.path.join(P, "ntt_issue_r04.json")))
    r = got["ratio_20_over_23"]
    assert 0.95 < r["products_per_instr"] < 1.0 and r["issue_rate"] < 0.85
