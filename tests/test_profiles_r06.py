"""Round-6 profile summaries recompute from the raw rocprofv3 rows committed beside them (no GPU needed).

* profiles/affine_r06.json (the batch-affine measurement): tools/prof/affine_summary.py
  over profiles/affine_r06/*.csv -- per-addition VALU instructions, issue share, HBM bytes, and the projection
  of the affine pair pass at the XYZZ kernel's own issue rate.
"""
import json
import os
import subprocess
import sys

import pytest

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


def test_valu_counted_recomputes():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "valu_counted.py"), "--check"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]


def test_valu_counted_findings():
    """VERDICT r5 item 4, as DESIGN.md §5 states it: full-rate opcodes co-issue across waves (SQ_ACTIVE_INST_VALU2 ~
    0.45 of their instructions when alone), 4-clock opcodes never; the H launch's stream co-issues in < 3 % of
    its instructions, so its counted VALU busy stays within 0.02 of the 4-clock issue share and above 0.92."""
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_valu_r06.json")))
    ops = d["opcodes_alone"]
    for full in ("v_and_b32_e32", "v_add_u32_e32", "v_sub_u32_e32", "v_mov_b32_e32", "v_lshrrev_b32_e32"):
        assert ops[full]["dual_issue_quad_cycles_per_instr"] > 0.4
    for half in ("v_mad_u64_u32", "v_lshrrev_b64", "v_mul_lo_u32", "v_alignbit_b32", "v_add3_u32", "v_lshlrev_b32_e32"):
        assert ops[half]["dual_issue_quad_cycles_per_instr"] < 0.01
    h = d["accumulate"]["H"]
    assert h["dual_issue_quad_cycles_per_instr"] < 0.03
    assert h["valu_issue_frac_4cyc"] - h["valu_busy_counted"] < 0.02 and h["valu_busy_counted"] > 0.92
    assert h["valu_busy_counted"] == pytest.approx(
        h["valu_issue_frac_4cyc"] * (1 - h["dual_issue_quad_cycles_per_instr"]), abs=2e-4)


P = os.path.join(ROOT, "profiles")


def test_launch_split_r06_reproduces_bench_fracs(tmp_path):
    """The round-6 kernel trace (k_accumulate rows + the ROCTx "bench timed" range of the same bench
    invocation, tools/gpu/trace.sh) recomputes every launch kind's frac of profiles/bench_r06_rocprof_run.json
    within 0.01, and the committed launch_split_r06.json is that output."""
    out = tmp_path / "split.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "launch_split.py"),
                    os.path.join(P, "rocprof_r06_accumulate_trace.csv"), os.path.join(P, "rocprof_r06_marker_trace.csv"),
                    os.path.join(P, "bench_r06_rocprof_run.json"), str(out)], check=True, capture_output=True, timeout=120)
    res = json.loads(out.read_text())
    assert set(res["kinds"]) == {"A", "B1", "C", "H", "B2"}
    for kind, v in res["kinds"].items():
        assert v["dispatches"] == v["bench_launches"], kind
        assert abs(v["frac_delta"]) <= 0.01, (kind, v)
    assert res["kinds"] == json.load(open(os.path.join(P, "launch_split_r06.json")))["kinds"]


def test_pmc_launch_r06_recomputes(tmp_path):
    """profiles/pmc_launch_r06.json (what bench.py's roofline `traffic`, issue share and clock read) from the
    committed k_accumulate rows of the round-6 SQ / FETCH_SIZE / WRITE_SIZE passes (tools/gpu/pmc.sh)."""
    out = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "pmc_launch5.py"),
                    os.path.join(P, "pmc_launch_r06"), str(out), "x"], check=True, capture_output=True, timeout=120)
    got = json.loads(out.read_text())
    want = json.load(open(os.path.join(P, "pmc_launch_r06.json")))
    assert got["kinds"] == want["kinds"]
    h = got["kinds"]["H"]
    assert h["valu_issue_frac"] > 0.9 and 1.3 < h["hbm_bytes_per_addition"] / 68 < 1.6


def test_proof_valu_r06_recomputes(tmp_path):
    """profiles/proof_valu_r06.json (a proof's VALU work against its span) from the committed
    per-dispatch counters of three whole proofs: the classes' instruction shares sum to 1, the G1
    accumulations are the largest share, and the VALU work fills most of the bench's ms per proof."""
    out = tmp_path / "pv.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "proof_valu.py"),
                    os.path.join(ROOT, "profiles", "proof_valu_r06", "valu_counter_collection.csv"),
                    os.path.join(ROOT, "profiles", "bench_r06_d.json"), str(out)],
                   check=True, capture_output=True, timeout=120)
    got = json.load(open(out))
    want = json.load(open(os.path.join(ROOT, "profiles", "proof_valu_r06.json")))
    for k in ("classes", "valu_busy_simd_cycles_per_proof", "t_valu_ms", "span_filled_by_valu_work", "proofs"):
        assert got[k] == want[k], k
    assert got["proofs"] == 3
    assert abs(sum(c["valu_instr_share"] for c in got["classes"].values()) - 1) < 1e-3
    assert max(got["classes"], key=lambda k: got["classes"][k]["valu_instr_share"]) == "accumulate G1"
    assert 0.8 < got["span_filled_by_valu_work"]["2.0 GHz"] < 1.0
