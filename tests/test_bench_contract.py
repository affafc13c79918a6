"""The committed bench lines under profiles/ keep the driver's bench.py contract.

Checks the JSON shape the driver parses (metric/value/unit/steps/..., config.workload), that
`value` is the throughput `ms_per_step` implies, and that the roofline object is internally
consistent: `achieved` = algorithmic MACs per launch / average launch time (DESIGN.md §5:
11 Fp-mul per mixed add, 136 MAC per Fp-mul) and `frac` = achieved / peak.
No GPU and no library needed.
"""
import json
import pathlib

import pytest

PROFILES = pathlib.Path(__file__).resolve().parent.parent / "profiles"
LINES = ["bench_r01.json", "bench_r01_recheck.json", "bench_r05_final.json", "bench_r06_a.json", "bench_r06_b.json",
         "bench_r06_c.json", "bench_r06_d.json"]
REQUIRED = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
            "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]


def _load(name):
    path = PROFILES / name
    if not path.exists():
        pytest.skip(f"{name} not committed")
    return json.loads(path.read_text().strip().splitlines()[-1])


@pytest.mark.parametrize("name", LINES)
def test_contract_keys(name):
    d = _load(name)
    for k in REQUIRED:
        assert k in d, k
    assert d["unit"] == "proofs/s" and d["higher_is_better"] is True
    assert d["scaling"] in ("weak", "strong")
    assert "workload" in d["config"]
    assert d["n_gpus"] >= 1 and d["steps"] >= 1
    # whole-job throughput: one proof per step per rank
    assert d["value"] == pytest.approx(1000.0 * d["n_gpus"] / d["ms_per_step"], rel=0.02)


@pytest.mark.parametrize("name", LINES)
def test_roofline_consistent(name):
    r = _load(name)["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-3)
    assert 0.0 < r["frac"] < 1.0
    w = r["algorithmic_work_per_launch"]
    mac = w["mixed_adds"] * w["fp_mul_per_add"] * w["mac_per_fp_mul"]
    assert r["achieved"] == pytest.approx(mac / (r["avg_launch_ms"] * 1e-3) / 1e12, rel=0.01)


@pytest.mark.parametrize("name", LINES)
def test_cpu_baseline(name):
    c = _load(name)["cpu_baseline"]
    assert c["kind"] in ("port", "reference")
    assert c["cores"] >= 1 and c["value"] > 0 and c["sample"]
    assert c.get("bit_exact_vs_gpu") is True


def test_gpus_more_than_visible_fails_loudly():
    """`bench.py --gpus N` without torchrun drives N devices from one process; with fewer
    visible GPUs (none here, one on the test box) it must exit non-zero with a message instead
    of printing a line measured on fewer devices."""
    import os
    import subprocess
    import sys
    root = PROFILES.parent
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "64", "--cpu-baseline", "none"],
                       cwd=str(root), env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "--gpus 64 requested" in p.stderr and "--rehearsal" in p.stderr
    assert p.stdout.strip() == ""


def test_round5_line_fields():
    """The round-5 default bench line (profiles/bench_r05_final.json) carries what VERDICT r4 asked for:
    verified batch proofs, the counted VALU issue and clock beside the H roofline, the issue-ceiling
    fraction consistent with `achieved`, the fixed-base label of the MSM kernel line with its table
    build time, and the NTT's counted instructions per element."""
    d = _load("bench_r05_final.json")
    b = d["batch_pcie_inclusive"]
    assert b["verified"] == "%d/%d" % (b["proofs_per_rank"], b["proofs_per_rank"]) and b["all_proofs_ok"]
    assert b["verify_before_return_mode"] == 2 and b["vs_staged_headline"] > 0.95
    r = d["roofline"]
    assert 0.9 < r["valu_issue_frac_pmc"] < 1.0 and 1.5 < r["clock_GHz_pmc"] < 2.5
    assert r["frac_vs_issue_ceiling"] == pytest.approx(r["achieved"] / r["issue_ceiling"], rel=1e-3)
    assert r["issue_ceiling"] == pytest.approx(256 * 64 * 2.4e9 / 1e12, rel=1e-4)
    k = d["kernels_config1"]
    assert k["msm_kind"].startswith("fixed-base") and k["msm_g1_2^20_table_build_ms"] > 0
    ntt = k["ntt_roofline"]["2^23 (Venmo domain)"]
    assert ntt["valu_lane_instr_per_element_pmc"] < 6000
    assert d["all_proofs_ok"] and d["cpu_baseline"]["bit_exact_vs_gpu"]


@pytest.mark.parametrize("name", ["bench_r06_b.json", "bench_r06_c.json", "bench_r06_d.json"])
def test_round6_compact_line(name):
    """the driver keeps the last 8 KB of stdout, so the contract line (the LAST line)
    stays below 6,000 bytes and carries both halves of the metric (proofs/s and the 1-proof latency), the
    verified batch, the sustained >= 30-s rate, the roofline and cpu_baseline; the detail object is the
    line before it."""
    path = PROFILES / name
    if not path.exists():
        pytest.skip("%s not committed" % name)
    lines = path.read_text().strip().splitlines()
    last = lines[-1]
    assert len(last.encode()) < 6000
    d = json.loads(last)
    assert d["latency_ms"] > 0 and d["latency_ms_staged"] > 0
    b = d["batch_pcie_inclusive"]
    assert b["verified"] == "%d/%d" % (b["proofs_per_rank"], b["proofs_per_rank"]) and b["all_proofs_ok"]
    su = d["sustained"]
    assert su["seconds"] >= 30 and su["all_proofs_ok"] and su["proofs"] >= 1000
    assert su["vs_value"] == pytest.approx(su["proofs_per_s"] / d["value"], rel=1e-3)
    if su["vs_value"] < 0.98:
        assert "value_note" in d
    assert "bench_detail" in json.loads(lines[-2])
