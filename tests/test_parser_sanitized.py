"""Host parser robustness: the .zkey / .wtns / gzip readers built with
AddressSanitizer + UndefinedBehaviorSanitizer (host-only C++, no device) and fed every
truncation on a grid, section-length fields set to extremes and seeded byte flips of the golden
files; every input must parse or raise ZkpError, with no sanitizer report."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zk-p2p-onramp_amd", "csrc")
HT = os.path.join(ROOT, "tools", "hosttest")


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = str(tmp_path_factory.mktemp("pf") / "parse_fuzz")
    srcs = [os.path.join(HT, "parse_fuzz.cpp")] + [os.path.join(CSRC, f) for f in
                                                    ("zkey_parse.cpp", "host_ec.cpp", "zkey_io.cpp")]
    # host code only: every sanitizer flag behind -Xarch_host (no device code is built or run)
    subprocess.run([hipcc, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-Xarch_host",
                    "-fsanitize=address,undefined", "-Xarch_host", "-fno-sanitize-recover=all", *srcs, "-o", out,
                    "-lz", "-lpthread"], check=True)
    return out


@pytest.mark.parametrize("name", ["tiny", "small"])
def test_parsers_under_sanitizers(fuzz_bin, golden_dir, name):
    zk = os.path.join(golden_dir, "circuit_%s.zkey" % name)
    wt = os.path.join(golden_dir, "circuit_%s.wtns" % name)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
    r = subprocess.run([fuzz_bin, zk, wt, "7", "3000"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "parse_fuzz:" in r.stdout
