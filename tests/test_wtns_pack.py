"""The compact witness transfer format (csrc/wtns_pack.hpp, decoded on the device by qap.hip
k_witness_unpack): tools/hosttest/wtns_pack_test encodes witnesses of uniform, all-small, 70 %
small and lane-pattern mixes (2^32, 2^32 - 1, top-word-only values, whole blocks of one kind) at
sizes 1, 63, 64, 65, 64K, 128K - 1, 3 x 64K + 37, 4 x 64K and four random ones (chunks encoded in descending or
shuffled order), decodes every signal the way the kernel does and
compares it with the input.  CPU-only; the GPU side is tests/test_gpu_witness_transfer.py."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_wtns_pack_roundtrip(tmp_path):
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "wtns_pack_test")
    subprocess.run([gxx, "-O2", "-std=c++17", "-pthread", os.path.join(ROOT, "tools", "hosttest", "wtns_pack_test.cpp"),
                    "-o", exe], check=True, timeout=300)
    out = subprocess.run([exe, "100000", "2"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ok roundtrip" in out.stdout


def test_host_capacity_probe_runs(tmp_path):
    """tools/hosttest/host_capacity (the configs[3] host-side probe): G concurrent
    encoder groups report witnesses/s and the host-memory traffic; a tiny run here checks that it
    builds and that its numbers hang together (every group encoded, payload per witness between the
    all-bits floor and 32 B per signal)."""
    import json
    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "host_capacity")
    subprocess.run([gxx, "-O2", "-std=c++17", "-pthread", os.path.join(ROOT, "tools", "hosttest", "host_capacity.cpp"),
                    "-o", exe], check=True, timeout=300)
    for pct in ("70", "0"):
        out = subprocess.run([exe, "70000", "2", "2", "0.3", pct], capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stdout + out.stderr
        r = json.loads(out.stdout.strip().splitlines()[-1])
        assert r["witnesses"] >= 2 and r["witnesses_per_s"] > 0
        mb = r["pcie_payload_MB_per_witness"]
        meta = 2 * 7 * 1024 * 4 / 1e6  # two 64K-signal chunks, 7 metadata words per 64-signal block
        assert 70000 * 32 * 0.05 / 1e6 < mb <= 70000 * 32 / 1e6 + meta + 0.01
