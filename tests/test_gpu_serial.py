"""The serial decoder (k_inflate_serial), the safety net for every stream the parallel paths
decline: forced with dev_inflate_pass (7 = the serial decoder alone), it must
give the oracle's bytes -- realDecompress, /root/reference/include/inflate.hpp:277-322 -- and
errors, at >= 30 MB/s on a 16 MiB stream (the reference inflates zlib streams
at ~25-48 MB/s on one CPU core)."""
import time
import zlib

import pytest

import dmx
import streams
from oracle_bind import CheckerError

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sctx():
    c = dmx.Context(inflate_pass=7)
    yield c
    c.close()


def _run(c, s, n):
    import torch
    d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    d_o = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    c.set_timing(True)
    olen = c.inflate_device(d_in.data_ptr(), len(s), d_o.data_ptr(), n + 64)
    ms = c.stats().ms_device_total
    path = c.stats().path
    c.set_timing(False)
    return d_o[:olen].cpu().numpy().tobytes(), path, ms


# MB/s floors of the forced serial decoder on 16 MiB (one MI355X, round 5: bmp Z_FIXED 35.7, mixed
# zlib-6 29.5, text zlib-1 13.6, one literal-only fixed block 10.9; round 4: 2.7 MB/s on the last).
# The decoder is one wavefront (the stream is one dependency chain): it decodes the token at 128
# consecutive bit offsets at once and walks the true chain four tokens per scalar step.
FLOOR = {("bmp", "zfixed"): 30, ("mixed", "zlib6"): 25, ("text", "zlib1"): 11, ("mixed", "single"): 9}


@pytest.mark.parametrize("kind,shape", [("mixed", "zlib6"), ("text", "zlib1"), ("mixed", "single"),
                                        ("bmp", "zfixed")])
def test_serial_16MiB(sctx, oracle, kind, shape):
    data = dmx.corpus(kind, 16 << 20)
    s = {"zlib6": lambda: streams.zlib_raw(data, 6), "zlib1": lambda: streams.zlib_raw(data, 1),
         "single": lambda: streams.single_fixed_block(data), "zfixed": lambda: streams.zfixed(data)}[shape]()
    out, path, ms = _run(sctx, s, len(data))
    assert path == 2
    assert out == data == oracle.inflate(s)
    mbps = len(data) / ms / 1e3
    print(f"serial {kind} {shape}: stream {len(s)} B, {ms:.1f} ms = {mbps:.1f} MB/s")
    assert mbps >= FLOOR[(kind, shape)], (kind, shape, mbps)


def test_serial_host_api_and_errors(sctx, oracle):
    """Host API (output buffer grown by the driver) and the reference's error codes: a truncated
    stream over-reads (DMX_ERR_OVERREAD), a stored block at the end is short."""
    data = dmx.corpus("text", 3 << 20) + dmx.corpus("zeros", 1 << 20)
    s = streams.zlib_raw(data, 9)
    assert sctx.decompress(s) == data
    assert sctx.stats().path == 2
    for cut in (len(s) // 2, len(s) - 1):
        t = s[:cut]
        try:
            want = oracle.inflate(t)
        except CheckerError as e:  # the oracle's codes: -1 over-read, -2 bad data
            want = {-1: dmx.DMX_ERR_OVERREAD, -2: dmx.DMX_ERR_DATA}[e.code]
        try:
            got = sctx.decompress(t)
        except dmx.DmxError as e:
            got = e.code
        assert got == want, (cut, got if isinstance(got, int) else len(got), want if isinstance(want, int) else len(want))
