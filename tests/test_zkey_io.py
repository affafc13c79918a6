"""§8f row 2: chunked / compressed zkey ingestion (host only, no GPU).

The app stores the key as circuit.zkey{b..k}.gz (reference app/src/helpers/zkp.ts:11-13,
51-68; circuit/server-scripts/upload_chunked_keys_to_s3.sh:13-22).  The chunk layout
belongs to an un-vendored snarkjs fork, so both plausible layouts are exercised: a byte
split of one binfile and per-chunk binfiles holding disjoint sections ("parity
unpinned" for the fork's exact layout; both must give back the original key)."""
import gzip
import os
import struct

import pytest

from oracle import binfile
import zkp_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
SUFFIX = "bcdefghijk"


def _orig(name="small"):
    return open(os.path.join(GOLD, "circuit_%s.zkey" % name), "rb").read()


def _sections(buf):
    nsec = struct.unpack_from("<I", buf, 8)[0]
    pos, out = 12, []
    for _ in range(nsec):
        sid, ln = struct.unpack_from("<IQ", buf, pos)
        out.append((sid, buf[pos + 12:pos + 12 + ln]))
        pos += 12 + ln
    return out


def _binfile(secs, version=1):
    return b"zkey" + struct.pack("<II", version, len(secs)) + b"".join(
        struct.pack("<IQ", sid, len(d)) + d for sid, d in secs)


def test_plain_and_gzip(tmp_path):
    z = _orig()
    (tmp_path / "a.zkey").write_bytes(z)
    assert zkp_amd.read_zkey(str(tmp_path / "a.zkey")) == z
    (tmp_path / "b.zkey.gz").write_bytes(gzip.compress(z))
    assert zkp_amd.read_zkey(str(tmp_path / "b.zkey")) == z          # path.gz fallback
    (tmp_path / "c.zkey").write_bytes(gzip.compress(z[:500]) + gzip.compress(z[500:]))  # 2 gzip members
    assert zkp_amd.read_zkey(str(tmp_path / "c.zkey")) == z


def test_byte_split_chunks_b_to_k_gz(tmp_path):
    z = _orig("venmo_mini")
    step = (len(z) + 9) // 10
    for i, s in enumerate(SUFFIX):
        part = z[i * step:(i + 1) * step]
        if i % 2:
            (tmp_path / ("circuit.zkey%s.gz" % s)).write_bytes(gzip.compress(part))
        else:
            (tmp_path / ("circuit.zkey%s" % s)).write_bytes(part)
    assert zkp_amd.read_zkey(str(tmp_path / "circuit.zkey")) == z


def test_byte_split_chunks_multi_member(tmp_path):
    # chunks are inflated in parallel into one buffer sized from the gzip trailers; a chunk of
    # several gzip members (trailer = last member only) takes the fallback path, same bytes back
    z = _orig("venmo_mini")
    step = (len(z) + 3) // 4
    for i, s in enumerate(SUFFIX[:4]):
        part = z[i * step:(i + 1) * step]
        blob = gzip.compress(part[:100]) + gzip.compress(part[100:]) if i == 1 else gzip.compress(part)
        (tmp_path / ("circuit.zkey%s.gz" % s)).write_bytes(blob)
    assert zkp_amd.read_zkey(str(tmp_path / "circuit.zkey")) == z


def test_section_split_chunks(tmp_path):
    z = _orig("small")
    secs = _sections(z)
    groups = [secs[:3], secs[3:5], secs[5:6], secs[6:]]
    paths = []
    for s, g in zip(SUFFIX, groups):
        p = tmp_path / ("circuit.zkey%s.gz" % s)
        p.write_bytes(gzip.compress(_binfile(g)))
        paths.append(str(p))
    merged = zkp_amd.read_zkey(str(tmp_path / "circuit.zkey"))
    assert merged == z  # snarkjs writes sections in ascending id order: same bytes back
    assert zkp_amd.read_zkey(list(reversed(paths))) == z  # explicit list, any order
    assert binfile.read_zkey(merged).n_vars == binfile.read_zkey(z).n_vars


def test_errors(tmp_path):
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.read_zkey(str(tmp_path / "missing.zkey"))
    assert e.value.status == 2
    (tmp_path / "bad.zkey").write_bytes(gzip.compress(_orig())[:200])
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.read_zkey(str(tmp_path / "bad.zkey"))
    assert e.value.status == 3
    secs = _sections(_orig())
    (tmp_path / "d.zkeyb").write_bytes(_binfile(secs[:4]))
    (tmp_path / "d.zkeyc").write_bytes(_binfile(secs[3:]))  # section 4 twice
    with pytest.raises(zkp_amd.ZkpError) as e:
        zkp_amd.read_zkey(str(tmp_path / "d.zkey"))
    assert e.value.status == 3 and "twice" in e.value.message
