"""GPU parity at BASELINE.json's full sizes: the 1 GiB streams our deflate
writes are decoded by decoders that are not ours -- zlib for the whole stream, the oracle (the
CPU restatement of the reference inflate) for a marker-cut prefix -- and by our GPU inflate.

Config C5: level 3 on the 1 GiB text corpus.  Level 2 on 1 GiB text, zeros and
bmp (config C2 is the repeat corpus, test_gpu_parity.test_device_roundtrip_1GiB_repeat_checksum).
"""
import hashlib
import zlib

import pytest

import dmx

pytestmark = pytest.mark.gpu
N = 1 << 30
PREFIX_SEGMENTS = 2048  # 64 MiB of output at 32 KiB segments
# SHA-256 of the 1 GiB corpora
SHA_1GIB = {
    "text": "aebbaba8601a2913c661e467890bcd8e08ce790595c946c733cbd5fb934ef89e",
    "zeros": "49bc20df15e412a64472421e13fe86ff1c5165e18b2afccf160d4dc19fe68a14",
}


def _device_corpus(kind):
    import torch
    host = torch.empty(N, dtype=torch.uint8).pin_memory()
    dmx.corpus_into(kind, N, host.data_ptr())
    return host, host.cuda()


def _zlib_whole(stream):
    """Raw inflate of the whole stream by zlib in bounded steps: (decoded bytes, SHA-256)."""
    z = zlib.decompressobj(-15)
    h = hashlib.sha256()
    total = 0
    view = memoryview(stream)
    for pos in range(0, len(view), 16 << 20):
        buf = view[pos: pos + (16 << 20)]
        while buf and not z.eof:
            out = z.decompress(buf, 64 << 20)
            h.update(out)
            total += len(out)
            buf = z.unconsumed_tail
        if z.eof:
            break
    assert z.eof, "zlib: the stream has no final block"
    assert not z.unused_data and pos + (16 << 20) >= len(view), "zlib: bytes after the final block"
    return total, h.hexdigest()


def _check_large(ctx, oracle, kind, level, min_ratio):
    import torch
    host, d_in = _device_corpus(kind)
    want = SHA_1GIB.get(kind) or hashlib.sha256(host.numpy().tobytes()).hexdigest()
    cap = dmx.deflate_bound(N) + 64
    d_c = torch.empty(cap, dtype=torch.uint8, device="cuda")
    clen = ctx.deflate_device(d_in.data_ptr(), N, level, d_c.data_ptr(), cap)
    assert N / clen >= min_ratio, (kind, level, N / clen)
    stream = d_c[:clen].cpu().numpy().tobytes()
    # 1. zlib decodes the whole stream to the corpus
    total, digest = _zlib_whole(stream)
    assert total == N and digest == want
    # 2. the oracle decodes a prefix cut at a segment start (closed with an empty final block)
    starts = ctx.segment_starts_device(d_c.data_ptr(), clen)
    assert len(starts) >= PREFIX_SEGMENTS
    cut = starts[PREFIX_SEGMENTS - 1]
    dec = oracle.inflate(stream[:cut] + b"\x03\x00")
    assert len(dec) == PREFIX_SEGMENTS * 32768 and dec == host[: len(dec)].numpy().tobytes()
    # 3. our GPU inflate
    d_o = torch.empty(N + 64, dtype=torch.uint8, device="cuda")
    olen = ctx.inflate_device(d_c.data_ptr(), clen, d_o.data_ptr(), N + 64)
    assert olen == N and torch.equal(d_o[:N], d_in)


def test_c5_level3_1GiB_text(ctx, oracle):
    """Config C5 at full size: 1 GiB text at level 3 (persistent segment loop, chain search under
    full occupancy); ratio at least 2.62 (the reference's L3 gives 2.574 on 1 MiB)."""
    _check_large(ctx, oracle, "text", 3, 2.62)


@pytest.mark.parametrize("kind,min_ratio", [("text", 2.5), ("zeros", 600.0), ("bmp", 100.0)])
def test_level2_1GiB_streams_decode_elsewhere(ctx, oracle, kind, min_ratio):
    """The 1 GiB level-2 streams of the bench corpora decode with zlib and the oracle too, so no
    large stream is checked by our own inflate alone."""
    _check_large(ctx, oracle, kind, 2, min_ratio)
