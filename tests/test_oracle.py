"""CPU: the oracle (plain-C restatement of the reference inflate) pinned against the golden
vectors produced by the real reference (tests/golden/make_golden.py) and against zlib."""
import hashlib
import json
import os
import sys
import random
import zlib

import pytest

from oracle_bind import CheckerError, Oracle, Reference

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLD)
from zgen import stream_of  # noqa: E402
MAN = json.load(open(os.path.join(GOLD, "manifest.json")))
VECS = [v for v in MAN["vectors"] if "stream" in v or "zgen" in v]


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("v", VECS, ids=[v["name"] for v in VECS])
def test_oracle_matches_reference_vector(oracle, v):
    s = stream_of(v, GOLD)
    if v.get("reference_reads_past_buffer"):
        # the reference's result depends on the byte after the buffer (A-9); ours errors
        with pytest.raises(CheckerError):
            oracle.inflate(s)
        return
    if not v["ref_ok"]:
        with pytest.raises(CheckerError):
            oracle.inflate(s)
        return
    out = oracle.inflate(s)
    assert len(out) == v["out_len"] and sha(out) == v["out_sha256"]
    if "expect" in v:
        assert out == open(os.path.join(GOLD, v["expect"]), "rb").read()


def test_reference_zlib_fixtures(oracle):
    for v in MAN["vectors"]:
        if "zlib_file" in v:
            d = open(os.path.join(GOLD, v["zlib_file"]), "rb").read()
            out = oracle.inflate(d[2:])
            assert sha(out) == v["out_sha256"] and len(out) == v["out_len"]
            assert out == zlib.decompress(d)


def test_lossy_reference_level2_decodes_pinned(oracle):
    """The reference's own level-2 stream of test.bmp is valid but lossy (A-1): the oracle
    reproduces the reference's (wrong) bytes exactly -- the first difference is at byte 26."""
    s = open(os.path.join(GOLD, "streams", "ref_L2_test.bmp.deflate"), "rb").read()
    out = oracle.inflate(s)
    orig = open(os.path.join(GOLD, "test.bmp"), "rb").read()
    assert out == open(os.path.join(GOLD, "expect", "ref_L2_test.bmp.bin"), "rb").read()
    diff = next(i for i in range(len(orig)) if out[i] != orig[i])
    assert diff == 26


def test_rfc_mode_crafted(oracle):
    """A-11 / A-12: the reference throws, RFC mode decodes as zlib does."""
    assert oracle.inflate(bytes.fromhex("0d83050100000040b6f27f84c40d"), rfc=True) == b"ababa"
    assert oracle.inflate(bytes.fromhex("0d89250100000080b6c2ff1140100027"), rfc=True) == b"abbbb"
    with pytest.raises(CheckerError):
        oracle.inflate(bytes.fromhex("0d83050100000040b6f27f84c40d"))


@pytest.mark.parametrize("seed", range(6))
def test_oracle_vs_zlib_random(oracle, seed):
    rng = random.Random(seed)
    n = rng.choice([0, 1, 2, 3, 258, 32767, 32768, 32769, 65537, rng.randrange(1, 200000)])
    alphabet = bytes(rng.sample(range(256), rng.randrange(1, 256)))
    data = bytes(rng.choice(alphabet) for _ in range(n))
    for lvl in (0, 1, 6, 9):
        for st in (zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE):
            z = zlib.compressobj(lvl, zlib.DEFLATED, -15, 9, st)
            s = z.compress(data) + z.flush()
            assert oracle.inflate(s) == data


@pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_equals_compiled_reference_on_fresh_streams(oracle):
    ref = Reference()
    rng = random.Random(7)
    for _ in range(10):
        n = rng.randrange(0, 70000)
        data = bytes(rng.randrange(0, 8) * 17 for _ in range(n))
        for lvl in (1, 6):
            z = zlib.compressobj(lvl, zlib.DEFLATED, -15)
            s = z.compress(data) + z.flush()
            assert oracle.inflate(s) == ref.decompress(s) == data


def test_oracle_quirk_path5_stream_matches_reference():
    """The quirk section (bad NLEN, BTYPE 3, far copy at a block start, A-11, A-12) in the
    middle of a 2 MiB-output zlib-1 stream: the oracle gives the compiled reference's SHA-256
    (tests/golden/quirk_streams.py, manifest 'quirk_path5')."""
    import hashlib
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import dmx
    import quirk_streams as Q
    from oracle_bind import Oracle
    q = json.load(open(os.path.join(GOLD, "manifest.json")))["quirk_path5"]
    orc = Oracle()
    text = dmx.corpus("text", q["text_len"], offset=q["text_offset"])
    s1, sec, b = Q.path5_stream(text)
    s = Q.finish_path5(s1, sec, b, orc.inflate(s1 + sec + b"\x03\x00"))
    assert len(s) == q["stream_len"] and hashlib.sha256(s).hexdigest() == q["stream_sha256"]
    out = orc.inflate(s)
    assert len(out) == q["out_len"] and hashlib.sha256(out).hexdigest() == q["out_sha256"]


@pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built (no /root/reference)")
def test_config0_test_bmp_round_trip_on_cpu(oracle):
    """BASELINE config 0: deflate::compress + inflate::decompress of test.bmp on the CPU (the
    reference's own case, deflate.hpp:779-815 / inflate.hpp:326).  Level 1 (literals only)
    round-trips exactly; level 2 (the "fast" matcher, getMatches) is lossy by SURVEY A-1, and the
    oracle must give the reference's own lossy bytes for it -- the checker the GPU tests rely on
    agrees with the reference on the reference's streams."""
    ref = Reference()
    data = open(os.path.join(GOLD, "test.bmp"), "rb").read()
    s1 = ref.compress(data, 1)
    assert ref.decompress(s1) == data == oracle.inflate(s1)
    s2 = ref.compress(data, 2)
    out = ref.decompress(s2)
    assert len(s2) < len(data) and len(out) == len(data)
    assert oracle.inflate(s2) == out
    assert out == open(os.path.join(GOLD, "expect", "ref_L2_test.bmp.bin"), "rb").read()
