"""configs[1]'s Fr NTT at its own size, full-vector bit-exact.

The GPU transforms (`zkp_ntt_fr`: mode 0 Fr.fft, 1 Fr.ifft, 2 the coset extension ifft ->
batchApplyKey(1, Fr.w[k+1]) -> fft) of 2^20 uniform Fr values -- SplitMix64 seed
0x5A4B5032 stream 2, SURVEY.md §8d D2 S20-NTT -- and a 2^23 coset extension (the Venmo domain) are
compared element by element with the C++ oracle's radix-2 NTT (oracle/cpu/groth16_cpu.cpp g16cpu_ntt,
itself pinned to the golden vectors by tests/test_cpu_oracle.py).  Every output, not a sample.
"""
import os

import pytest

import zkp_amd
from zkp_amd import synth

pytestmark = pytest.mark.gpu

SEED = 0x5A4B5032
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.fixture(scope="module")
def co():
    from oracle import cpu_oracle
    return cpu_oracle


def _first_diff(a: bytes, b: bytes):
    for i in range(0, min(len(a), len(b)), 32):
        if a[i:i + 32] != b[i:i + 32]:
            return i // 32
    return None


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_ntt_2_20_full_vector(co, mode):
    raw = synth.scalars(SEED, 2, 1 << 20)
    got = zkp_amd.ntt_fr_bytes(raw, mode)
    want = co.ntt(raw, mode, threads=THREADS)
    assert got == want, "first differing element %s" % _first_diff(got, want)


def test_ntt_2_23_coset_extension_full_vector(co):
    raw = synth.scalars(SEED, 2, 1 << 23)
    got = zkp_amd.ntt_fr_bytes(raw, 2)
    want = co.ntt(raw, 2, threads=THREADS)
    assert got == want, "first differing element %s" % _first_diff(got, want)


def test_ntt_2_20_edge_values(co):
    """0, 1, r - 1 and runs of equal values (2^20 elements: every pass of the 7+7+6 split sees them)."""
    r = zkp_amd.R_MOD
    n = 1 << 20
    vals = [0, 1, r - 1, 2, r - 2] * (n // 5) + [r - 1] * (n % 5)
    raw = b"".join(v.to_bytes(32, "little") for v in vals)
    for mode in (0, 1, 2):
        got = zkp_amd.ntt_fr_bytes(raw, mode)
        want = co.ntt(raw, mode, threads=THREADS)
        assert got == want, (mode, _first_diff(got, want))


@pytest.mark.parametrize("k", [16, 18, 19, 21, 22])
def test_ntt_other_sizes_full_vector(co, k):
    """Every pass split between the pinned sizes (16 = 8+8, 18 = 6+6+6, 19 = 7+6+6, 21 = 7+7+7, 22 = 8+7+7):
    the three transforms full-vector against the C++ oracle on a SplitMix stream of their own."""
    raw = synth.scalars(SEED + k, 2, 1 << k)
    for mode in (0, 1, 2):
        got = zkp_amd.ntt_fr_bytes(raw, mode)
        want = co.ntt(raw, mode, threads=THREADS)
        assert got == want, (mode, _first_diff(got, want))
