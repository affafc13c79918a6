"""The committed round-5 counter evidence recomputes the numbers the bench line and DESIGN.md quote
(VERDICT r4 items 1, 2, 7).  CPU-only (reads committed files):

* profiles/pmc_launch_r05.json (per launch kind: effective clock, VALU issue at that clock, the
  wave-cycle split, lane-instructions and HBM bytes per addition) from the committed k_accumulate rows
  of the four rocprofv3 --pmc passes (profiles/pmc_launch_r05/) by tools/prof/pmc_launch5.py;
* the H launch's frac gap to the witness launches factors into clock x issue x instructions;
* profiles/ntt_issue_r05.json's per-element instruction counts from the committed k_ntt rows;
* profiles/ubench_r05.json's peak is the best row of the sweep it lists."""
import io
import contextlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
sys.path.insert(0, os.path.join(ROOT, "tools", "prof"))


def test_pmc_launch_summary_recomputes(tmp_path):
    out = tmp_path / "pmc.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "pmc_launch5.py"),
                    os.path.join(P, "pmc_launch_r05"), str(out)], check=True, capture_output=True, timeout=120)
    got = json.loads(out.read_text())
    want = json.load(open(os.path.join(P, "pmc_launch_r05.json")))
    assert got["kinds"] == want["kinds"]
    h, w = got["kinds"]["H"], got["kinds"]["witness (A, B1, C)"]
    # issue-bound: the H launch uses >= 0.9 of its issue slots, at a clock well below the witness launches'
    assert h["valu_issue_frac"] > 0.9 and h["clock_GHz"] < 0.85 * w["clock_GHz"]
    # clock x issue x instructions per addition account for the frac ratio within a few percent
    model = (h["clock_GHz"] / w["clock_GHz"]) * (h["valu_issue_frac"] / w["valu_issue_frac"]) * (
        w["valu_lane_instructions_per_addition"] / h["valu_lane_instructions_per_addition"])
    measured = (h["mixed_adds_per_dispatch"] / h["wall_ms"]) / (w["mixed_adds_per_dispatch"] / w["wall_ms"])
    assert abs(model / measured - 1) < 0.03, (model, measured)
    # traffic: ~1.5x the 68 B per-addition minimum
    assert 1.3 < h["hbm_bytes_per_addition"] / 68 < 1.6


def test_ntt_instruction_counts_recompute():
    import pmc_stall
    want = json.load(open(os.path.join(P, "ntt_issue_r05.json")))["sizes"]
    for k in (23, 20):
        for v in ("base", "cur", "root1"):
            with contextlib.redirect_stdout(io.StringIO()):
                pmc_stall.ntt(os.path.join(P, "ntt_issue_r05", "ntt%d_%s.csv" % (k, v)), None)
            # recompute per-element counts from the rows directly
            ds = pmc_stall.rows_by_dispatch(os.path.join(P, "ntt_issue_r05", "ntt%d_%s.csv" % (k, v)))
            per = {}
            for d in ds:
                m = [x for x in ("<0", "<1", "<2") if "k_ntt" + x in d["name"].replace(" ", "")]
                per.setdefault(m[0][1], []).append(d["SQ_INSTS_VALU"] * 64 / (1 << k))
            tot = sum((2 if mode in "01" else 1) * sum(x) / len(x) for mode, x in per.items())
            assert abs(tot - want["2^%d" % k][v]["coset_extension_valu_lane_instr_per_element"]) < 1.0
    assert want["2^23"]["cur"]["coset_extension_valu_lane_instr_per_element"] < 0.94 * \
        want["2^23"]["base"]["coset_extension_valu_lane_instr_per_element"]
    # the trivial last-pair root: a quarter product per element per DFT fewer (2^23: six DFTs, 1.5 of 25 products)
    assert want["2^23"]["root1"]["coset_extension_valu_lane_instr_per_element"] < 0.97 * \
        want["2^23"]["cur"]["coset_extension_valu_lane_instr_per_element"]
    import ntt_issue5
    for k in (23, 20):
        got = ntt_issue5.entry(os.path.join(P, "ntt_issue_r05", "ntt%d_root1.csv" % k), k)
        assert got == want["2^%d" % k]["root1"]


def test_ubench_peak_is_best_sweep_row():
    u = json.load(open(os.path.join(P, "ubench_r05.json")))
    assert u["v_mad_u64_u32_tops"] == max(r["tops"] for r in u["sweep"])
    assert len(u["sweep"]) == 15 and abs(u["issue_ceiling_tops"] - 256 * 64 * 2.4e9 / 1e12) < 1e-3


def test_launch_split_r05_reproduces_bench_fracs(tmp_path):
    """The round-5 kernel trace (k_accumulate rows + the ROCTx "bench timed" range of the same bench
    invocation) recomputes every launch kind's frac of profiles/bench_r05_rocprof_run.json within 0.01."""
    out = tmp_path / "split.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "launch_split.py"),
                    os.path.join(P, "rocprof_r05_accumulate_trace.csv"), os.path.join(P, "rocprof_r05_marker_trace.csv"),
                    os.path.join(P, "bench_r05_rocprof_run.json"), str(out)], check=True, capture_output=True, timeout=120)
    res = json.loads(out.read_text())
    assert set(res["kinds"]) == {"A", "B1", "C", "H", "B2"}
    for kind, v in res["kinds"].items():
        assert v["dispatches"] == v["bench_launches"], kind
        assert abs(v["frac_delta"]) <= 0.01, (kind, v)
    bench = json.loads(open(os.path.join(P, "bench_r05_rocprof_run.json")).read())
    assert bench["roofline"]["valu_issue_frac_pmc"] is not None and bench["roofline"]["clock_GHz_pmc"] is not None


def test_host_capacity_covers_eight_gpus():
    """profiles/host_capacity_r05.json: 8 concurrent encoder groups on the GPU box's
    16-core quota keep up with 8 GPUs' worth of proofs for both witness mixes."""
    d = json.load(open(os.path.join(P, "host_capacity_r05.json")))
    best = {}
    for r in d["host_capacity"]:
        if r["groups"] == 8:
            best[r["bool_pct"]] = max(best.get(r["bool_pct"], 0), r["witnesses_per_s"])
    assert best[70] > 2 * 320 and best[0] > 2 * 160
