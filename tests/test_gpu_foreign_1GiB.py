"""Path 5 at BASELINE scale on third-party streams: zlib level-1 raw streams
of the 1 GiB text, mixed and zeros corpora (SURVEY section 6 times the
reference on exactly these) inflated on the block-parallel path, the output's SHA-256 against
the survey's 1 GiB values, and the time against the reference's own inflate::decompress on one
core of this host (timed on a 128 MiB slice's zlib-1 stream and scaled by 8: the reference is
linear in its input, one 1 GiB run would take 10-30 s per corpus)."""
import hashlib
import time
import zlib

import pytest

import dmx
from oracle_bind import Reference

pytestmark = pytest.mark.gpu
GiB = 1 << 30
SHA_1GIB = {
    "zeros": "49bc20df15e412a64472421e13fe86ff1c5165e18b2afccf160d4dc19fe68a14",
    "text": "aebbaba8601a2913c661e467890bcd8e08ce790595c946c733cbd5fb934ef89e",
    "mixed": "f83fe2d63b39efbe8763cfbb1cb559de5fc87e0fa3be742d09b5bb98bc79125a",
}


def _zlib1(data):
    z = zlib.compressobj(1, zlib.DEFLATED, -15)
    return z.compress(data) + z.flush()


@pytest.mark.parametrize("kind", ["text", "mixed", "zeros"])
def test_path5_zlib1_1GiB(ctx, kind):
    import torch
    data = dmx.corpus(kind, GiB)
    s = _zlib1(data)
    d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    d_o = torch.empty(GiB + 64, dtype=torch.uint8, device="cuda")
    ctx.set_timing(True)
    best = 1e30
    for _ in range(3):
        olen = ctx.inflate_device(d_in.data_ptr(), len(s), d_o.data_ptr(), d_o.numel())
        best = min(best, ctx.stats().ms_device_total)
    path = ctx.stats().path
    ctx.set_timing(False)
    assert olen == GiB
    assert path == 5
    h = hashlib.sha256(d_o[:GiB].cpu().numpy().tobytes()).hexdigest()
    assert h == SHA_1GIB[kind]
    ref_ms = None
    if Reference.available():
        part = _zlib1(data[:GiB // 8])
        t = time.perf_counter()
        Reference().decompress(part)
        ref_ms = (time.perf_counter() - t) * 1e3 * 8
    print(f"{kind}: zlib-1 stream {len(s)} B, GPU {best:.2f} ms ({GiB / best / 1e6:.1f} GB/s), "
          f"reference 1 core ~{ref_ms if ref_ms is None else round(ref_ms)} ms (128 MiB x 8)")
    if ref_ms is not None:
        assert best < ref_ms
