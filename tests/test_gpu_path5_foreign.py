"""Block-parallel inflate (path 5) of third-party streams the header scan cannot split (VERDICT
r3 item 2): runs of fixed-code blocks (zlib Z_FIXED, the reference's own level-1 output), one
huge block, and zlib-1 zeros.  Each is checked bit-exact against the oracle (the CPU restatement
of the reference inflate, inflate.hpp:277-322) and timed against the reference's own inflate on
one core of the same host; the decode must take path 5 (virtual units), not the serial decoder.
"""
import time
import zlib

import pytest

import dmx
import streams
from oracle_bind import Reference

pytestmark = pytest.mark.gpu


def _gpu_inflate(ctx, s, n, reps=3):
    import torch
    d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
    d_o = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    ctx.set_timing(True)
    best = 1e30
    for _ in range(reps):
        olen = ctx.inflate_device(d_in.data_ptr(), len(s), d_o.data_ptr(), n + 64)
        best = min(best, ctx.stats().ms_device_total)
    path = ctx.stats().path
    ctx.set_timing(False)
    return d_o[:olen].cpu().numpy().tobytes(), path, best


def _ref_ms(s):
    """The reference's inflate::decompress of the stream on one host core (compiled from its
    headers, oracle/_ref), best of 2; None without the reference build."""
    if not Reference.available():
        return None
    r = Reference()
    best = 1e30
    for _ in range(2):
        t = time.perf_counter()
        r.decompress(s)
        best = min(best, (time.perf_counter() - t) * 1e3)
    return best


CASES = {
    "zfixed_text_64MiB": lambda: (dmx.corpus("text", 64 << 20), None),
    "zlib1_zeros_256MiB": lambda: (dmx.corpus("zeros", 256 << 20), None),
    "single_block_16MiB": lambda: (dmx.corpus("mixed", 16 << 20), None),
    "zfixed_mixed_32MiB": lambda: (dmx.corpus("mixed", 32 << 20), None),
    "single_block_open_8MiB": lambda: (dmx.corpus("text", 8 << 20), None),
}


def _stream(name, data):
    if name.startswith("zfixed"):
        return streams.zfixed(data)
    if name.startswith("zlib1"):
        return streams.zlib_raw(data, 1)
    if "open" in name:  # a non-final block, then an empty final fixed block
        return streams.single_fixed_block(data, final=False, close=True)
    return streams.single_fixed_block(data)


@pytest.mark.parametrize("name", sorted(CASES))
def test_path5_streams_without_unit_starts(ctx, oracle, name):
    data, _ = CASES[name]()
    s = _stream(name, data)
    out, path, ms = _gpu_inflate(ctx, s, len(data))
    assert out == data
    assert path == 5, f"{name}: path {path}"
    assert oracle.inflate(s) == data
    ref = _ref_ms(s)
    print(f"{name}: stream {len(s)} B, GPU {ms:.3f} ms ({len(data) / ms / 1e6:.2f} GB/s), "
          f"reference 1 core {ref if ref is None else round(ref, 1)} ms")
    if ref is not None:
        assert ms < ref, (name, ms, ref)


def test_path5_reference_fixed_block_stream(ctx, oracle):
    """The reference's own level-2 output of periodic data is a fixed-code block per 32 KiB
    chunk with no marker and no dynamic header (SURVEY A-4: 2,049 fixed blocks on the repeat
    corpus); it is lossy (A-1), so the expected bytes are the oracle's -- the reference inflate's
    -- not the input."""
    if not Reference.available():
        pytest.skip("reference build (oracle/_ref) not present")
    data = dmx.corpus("repeat", 8 << 20)
    s = Reference().compress(data, 2)
    want = oracle.inflate(s)
    out, path, ms = _gpu_inflate(ctx, s, len(want))
    assert out == want
    assert path == 5


def _unmark(sync_flushed, filler):
    """A sync-flushed stream ends in the empty stored block 000|pad|00 00 FF FF; give that block
    a payload instead (LEN = len(filler)), so the junction carries no 00 00 FF FF marker and
    its stored header (not byte-aligned, after a Huffman block) is no scanned start."""
    assert sync_flushed.endswith(b"\x00\x00\xff\xff")
    n = len(filler)
    return sync_flushed[:-4] + n.to_bytes(2, "little") + (n ^ 0xFFFF).to_bytes(2, "little") + filler


@pytest.mark.parametrize("final_fixed", [False, True])
def test_path5_dynamic_then_fixed_run(ctx, oracle, final_fixed):
    """Dynamic blocks, a small stored block, then a long run of fixed-code blocks (zlib Z_FIXED)
    and (optionally) a huge final fixed block: the dynamic unit ends at the first far fixed
    header and repair units decode the run lane-parallel."""
    a = dmx.corpus("text", 3 << 20)
    b = dmx.corpus("mixed", 6 << 20, offset=5 << 20)
    c = dmx.corpus("bmp", 4 << 20)
    f1, f2 = b"gap-1", b"gap-2!"
    z = zlib.compressobj(6, zlib.DEFLATED, -15)
    s1 = _unmark(z.compress(a) + z.flush(zlib.Z_SYNC_FLUSH), f1)
    zf = zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_FIXED)
    if final_fixed:
        s2 = _unmark(zf.compress(b) + zf.flush(zlib.Z_SYNC_FLUSH), f2) + streams.single_fixed_block(c)
        want = a + f1 + b + f2 + c
    else:
        s2 = zf.compress(b) + zf.flush()
        want = a + f1 + b
    s = s1 + s2
    assert b"\x00\x00\xff\xff" not in s[len(s1) - 16: len(s1) + 16]
    out, path, ms = _gpu_inflate(ctx, s, len(want))
    assert out == want == oracle.inflate(s)
    assert path == 5


@pytest.mark.parametrize("name", ["single_block_2MiB", "zfixed_mixed_4MiB", "zfixed_text_2MiB"])
def test_path5_regions_serial_units(oracle, name):
    """The same shapes with DMX_CFG_FB_SERIAL (every unit decoded by one wavefront, the serial
    replay and window hand-off): the A/B reference of the lane-parallel unit decoder."""
    kind, mib = {"single_block_2MiB": ("mixed", 2), "zfixed_mixed_4MiB": ("mixed", 4),
                 "zfixed_text_2MiB": ("text", 2)}[name]
    data = dmx.corpus(kind, mib << 20)
    s = streams.single_fixed_block(data) if name.startswith("single") else streams.zfixed(data)
    c = dmx.Context(fb_serial=True)
    try:
        out, path, ms = _gpu_inflate(c, s, len(data), reps=1)
    finally:
        c.close()
    assert out == data == oracle.inflate(s)
    assert path == 5


def _ref_err_ms(s):
    """The reference's inflate::decompress of a broken stream on one host core: (ms, raised)."""
    if not Reference.available():
        return None, None
    r = Reference()
    t = time.perf_counter()
    raised = False
    try:
        r.decompress(s)
    except Exception:
        raised = True
    return (time.perf_counter() - t) * 1e3, raised


def test_path5_truncated_stream_reports_error_from_chain(ctx, oracle):
    """A truncated third-party stream: the chain of units is valid from bit 0
    up to the unit that runs out of input, and that unit's over-read is the error realDecompress
    (inflate.hpp:277-322, Bitwrapper inflate.hpp:81-108) throws -- reported from the chain, not
    by a serial re-decode from bit 0; faster than the reference reaches the same error."""
    import torch
    data = dmx.corpus("text", 256 << 20)
    s = streams.zlib_raw(data, 1)
    d_o = torch.empty(len(data) + 64, dtype=torch.uint8, device="cuda")
    for cut in (len(s) * 2 // 3 + 12345, len(s) - 3):
        t = s[:cut]
        from oracle_bind import CheckerError
        with pytest.raises(CheckerError) as oe:
            oracle.inflate(t)
        want = {-1: dmx.DMX_ERR_OVERREAD, -2: dmx.DMX_ERR_DATA}[oe.value.code]
        d_in = torch.frombuffer(bytearray(t), dtype=torch.uint8).cuda()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with pytest.raises(dmx.DmxError) as ge:
            ctx.inflate_device(d_in.data_ptr(), len(t), d_o.data_ptr(), d_o.numel())
        ms = (time.perf_counter() - t0) * 1e3
        assert ge.value.code == want
        assert ctx.stats().path == 5
        ref, raised = _ref_err_ms(t)
        print(f"truncated at {cut} of {len(s)}: GPU {ms:.1f} ms ({dmx.strerror(want)}), reference 1 core "
              f"{ref if ref is None else round(ref, 1)} ms")
        if ref is not None:
            assert raised
            assert ms < ref, (cut, ms, ref)


def _fixed_bits(data, final):
    """One fixed-code block of literals as a bit array (sending order), not byte-padded."""
    import numpy as np
    a = np.frombuffer(bytes(data), dtype=np.uint8).astype(np.uint32)
    code = np.where(a < 144, 0x30 + a, 0x190 + a - 144)
    ln = np.where(a < 144, 8, 9)
    j = np.arange(9, dtype=np.uint32)
    bits = ((code[:, None] >> np.maximum(ln[:, None] - 1 - j[None, :], 0)) & 1).astype(np.uint8)
    body = bits[j[None, :] < ln[:, None]]
    head = np.array([1 if final else 0, 1, 0], dtype=np.uint8)
    return np.concatenate([head, body, np.zeros(7, dtype=np.uint8)])


def test_path5_unlisted_dynamic_header_inside_fixed_run(ctx, oracle):
    """A dynamic block inside a long fixed-code run whose header the scan's check rejects (its
    lit/len code is incomplete -- valid for the reference's decoder, inflate.hpp:136-224, but
    not a candidate the check accepts): the region map meets a dynamic header that is not a
    listed start, so the region has no token path.  That region's span is decoded by repair
    units on the block-parallel path (it used to send the whole stream to the serial
    decoder); the bytes are the oracle's."""
    import numpy as np
    from golden.quirk_streams import BitWriter, canonical, rle_ops, write_dynamic_header
    a = dmx.corpus("mixed", 1 << 20, offset=11)
    b = dmx.corpus("text", 1 << 20, offset=22)
    # the dynamic block: 16 literals 'a'..'p' and end of block at 5 bits -- 17/32 of the code
    # space (incomplete); two distance codes of one bit
    L = [0] * 257
    for s in list(range(ord("a"), ord("a") + 16)) + [256]:
        L[s] = 5
    lc = canonical(L)
    payload = bytes((ord("a") + (i * 7) % 16) for i in range(5000))
    bw = BitWriter()
    bw.put(0, 1)
    bw.put(2, 2)
    write_dynamic_header(bw, rle_ops(L) + rle_ops([1, 1]), 257, 2)
    for ch in payload:
        bw.put_code(*lc[ch])
    bw.put_code(*lc[256])
    nbits = 8 * len(bw.out) + bw.n
    dyn = np.unpackbits(np.frombuffer(bytes(bw.out) + bytes([bw.acc & 0xFF]), dtype=np.uint8),
                        bitorder="little")[:nbits]
    allbits = np.concatenate([_fixed_bits(a, False), dyn, _fixed_bits(b, True)])
    s = np.packbits(allbits, bitorder="little").tobytes()
    want = oracle.inflate(s)
    assert want == a + payload + b
    out, path, ms = _gpu_inflate(ctx, s, len(want), reps=1)
    assert out == want
    assert path == 5
