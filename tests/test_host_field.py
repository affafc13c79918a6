"""The device field and curve code (csrc/field.hpp, curve.hpp: __host__ __device__)
compiled for the host by hipcc and checked op by op against the oracle -- the lazy
reductions (lsub/rsub/sub_2x/mul2/mul4, Fq2 products) at their extreme operand
ranges, and XYZZ additions/doublings.  CPU-only: exercises the exact arithmetic the
kernels run, without a GPU."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HT = os.path.join(ROOT, "tools", "hosttest")


@pytest.fixture(scope="module")
def field_host(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("fh") / "field_host")
    subprocess.run([hipcc, "-O1", "-std=c++17", os.path.join(HT, "field_host.cpp"), "-o", out], check=True,
                   timeout=300)
    return out


def test_device_field_ops_on_host(field_host, monkeypatch):
    monkeypatch.setenv("FIELD_HOST_BIN", field_host)
    sys.path.insert(0, HT)
    try:
        import importlib
        import check_field
        importlib.reload(check_field)
        assert check_field.main(n=120)
        assert check_field.curve_check(n=12)
    finally:
        sys.path.remove(HT)
