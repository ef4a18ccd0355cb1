"""GPU: the two resolve kernels of path 4 (inflate_lanes.hip, round 6) on streams that mix both
kinds of segment in one call -- short token lists (long periodic copies filled by a 256-thread
workgroup, stored segments) and long ones (text-like, the one-wave kernel's ticket list) -- at 32
and 64 KiB segments, every period class of the workgroup fill (d < 16, d < 64, d >= 64, copies
ending inside or at the end of a segment, followed by literals).  Bytes are compared with the
input (our deflate's round trip) and with the oracle; the inflate must stay on path 4."""
import random

import pytest

import dmx

pytestmark = pytest.mark.gpu


def _segments(seed):
    rnd = random.Random(seed)
    text = dmx.corpus("text", 1 << 20)
    segs = []
    for k, d in enumerate((1, 2, 3, 5, 7, 13, 16, 17, 31, 63, 64, 65, 100, 251, 1000, 4095, 9000, 20000)):
        head = rnd.randrange(0, 3000)
        tail = rnd.choice((0, 0, 5, 700, 5000))
        pre = bytes(rnd.getrandbits(8) for _ in range(head))
        pat = bytes(rnd.getrandbits(8) for _ in range(d))
        body = (pat * (32768 // d + 2))[:32768 - head - tail]
        post = bytes(rnd.getrandbits(8) for _ in range(tail))
        segs.append(pre + body + post)
        # a text-like segment (a long token list) and a random one (stored) between them
        o = rnd.randrange(0, len(text) - 32768)
        segs.append(text[o:o + 32768])
        if k % 3 == 0:
            segs.append(bytes(rnd.getrandbits(8) for _ in range(32768)))
    return segs


@pytest.mark.parametrize("seg_bytes", [32768, 65536])
def test_resolve_kernels_mixed_segments(oracle, seg_bytes):
    c = dmx.Context(segment_bytes=seg_bytes)
    try:
        for seed in (1, 2):
            d = b"".join(_segments(seed))
            s = c.compress(d, 2)
            out = c.decompress(s)
            assert c.stats().path == 4
            assert out == d
            assert oracle.inflate(s) == d
            # a ragged end: the last segment short, with a long copy reaching the stream's end
            d2 = d + b"xyz" * 3000
            s2 = c.compress(d2, 2)
            assert c.decompress(s2) == d2 and c.stats().path == 4
    finally:
        c.close()
