"""Config C4 at its full size on one GPU: 8 GiB of the mixed corpus as eight
1 GiB shards, and a compressed stream of more than 4 GiB.  These are the runs that push 64-bit
offsets through every kernel: segment indices past 2^17, input and output offsets past 4 GiB,
marker-scan and candidate positions past 4 GiB, token-list offsets past 2^32 bytes.

Block size: C4 names 64 KiB blocks (dmx_config.segment_bytes = 65536: one DEFLATE block per
64 KiB of input, its two 32 KiB halves matched independently under one Huffman code); the
reference's chunk is 32 KiB (deflate.hpp:689-697), libdmx's default.  Both are run at full size."""
import gc

import pytest

import dmx

pytestmark = pytest.mark.gpu
GiB = 1 << 30


def _release():
    import torch
    gc.collect()
    torch.cuda.empty_cache()


def _log(msg):
    print(f"[c4] {msg}", flush=True)


def _first_diff(a, b, chunk=256 << 20):
    """First index where two equal-length device tensors differ (None if equal), by chunks."""
    import torch
    for o in range(0, a.numel(), chunk):
        x, y = a[o:o + chunk], b[o:o + chunk]
        if not torch.equal(x, y):
            return o + int((x != y).to(torch.uint8).argmax())
    return None


def _device_corpus(kind, n, chunk=GiB):
    """kind[0, n) on the device, generated on the host one chunk at a time (bounded host RAM)."""
    import torch
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    host = torch.empty(min(chunk, n), dtype=torch.uint8).pin_memory()
    for b in range(0, n, chunk):
        m = min(chunk, n - b)
        dmx.corpus_into(kind, m, host.data_ptr(), offset=b)
        d[b:b + m].copy_(host[:m])
    return d


def test_c4_full_8GiB_mixed_shards_one_gpu(ctx, oracle):
    """The whole C4 workload on one GPU: 8 shards of 1 GiB deflated NOT_FINAL except the last,
    written back to back into one stream (the byte concatenation the RCCL gather produces),
    then that > 2 GiB stream inflated into 8 GiB and compared shard by shard.  The same 8 GiB in
    ONE deflate call must give the identical stream (segments are independent, deflate.hpp:697),
    and shard 3's stream closed with an empty final block decodes with the oracle."""
    import torch
    world, per = 8, GiB
    n = world * per
    d_in = _device_corpus("mixed", n)
    _log("corpus on the device")
    cap = world * (dmx.deflate_bound(per) + 64)
    stream = torch.empty(cap, dtype=torch.uint8, device="cuda")
    offs = [0]
    for r in range(world):
        L = ctx.deflate_device(d_in.data_ptr() + r * per, per, 2, stream.data_ptr() + offs[-1],
                               cap - offs[-1], not_final=(r < world - 1))
        offs.append(offs[-1] + L)
    total = offs[-1]
    _log(f"8 shards deflated: {offs}")
    assert total > 2 * GiB  # bit offsets past 2^34
    # one call over the whole 8 GiB: the same bytes
    one = torch.empty(dmx.deflate_bound(n) + 64, dtype=torch.uint8, device="cuda")
    L1 = ctx.deflate_device(d_in.data_ptr(), n, 2, one.data_ptr(), one.numel())
    _log(f"one call: {L1} bytes")
    assert L1 == total
    diff = _first_diff(one[:total], stream[:total])
    assert diff is None, f"first difference at byte {diff} of {total}"
    del one
    _release()
    # shard 3 (offsets 3..4 GiB of the input) closed with 03 00, through the oracle
    s3 = stream[offs[3]:offs[4]].cpu().numpy().tobytes() + b"\x03\x00"
    assert oracle.inflate(s3) == dmx.corpus("mixed", per, offset=3 * per)
    _log("shard 3 matches the oracle")
    del s3
    gc.collect()
    # the whole stream back into 8 GiB on the device
    out = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    try:
        olen = ctx.inflate_device(stream.data_ptr(), total, out.data_ptr(), n + 64)
    except Exception as e:
        _log(f"inflate raised {e!r}")
        raise
    _log(f"inflated {olen} bytes on path {ctx.stats().path}")
    assert olen == n
    assert ctx.stats().path == 4
    for r in range(world):
        diff = _first_diff(out[r * per:(r + 1) * per], d_in[r * per:(r + 1) * per])
        assert diff is None, f"shard {r}: first difference at byte {diff}"
    del d_in, stream, out
    _release()


def test_c4_64KiB_blocks_8GiB_mixed(oracle):
    """C4 as stated: 8 GiB of mixed data as 64 KiB DEFLATE blocks in eight 1 GiB shards (NOT_FINAL
    except the last, concatenated as the RCCL gather does), shard 5 checked by the oracle, the
    whole stream inflated on the lane path with 64 KiB slots and compared on the device."""
    import torch
    c = dmx.Context(segment_bytes=65536)
    try:
        world, per = 8, GiB
        n = world * per
        d_in = _device_corpus("mixed", n)
        cap = world * (dmx.deflate_bound(per) + 64)
        stream = torch.empty(cap, dtype=torch.uint8, device="cuda")
        offs = [0]
        for r in range(world):
            L = c.deflate_device(d_in.data_ptr() + r * per, per, 2, stream.data_ptr() + offs[-1],
                                 cap - offs[-1], not_final=(r < world - 1))
            offs.append(offs[-1] + L)
        total = offs[-1]
        _log(f"64 KiB blocks: 8 shards deflated, ratio {n / total:.4f}")
        s5 = stream[offs[5]:offs[6]].cpu().numpy().tobytes() + b"\x03\x00"
        assert oracle.inflate(s5) == dmx.corpus("mixed", per, offset=5 * per)
        del s5
        gc.collect()
        out = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
        olen = c.inflate_device(stream.data_ptr(), total, out.data_ptr(), n + 64)
        _log(f"inflated {olen} bytes on path {c.stats().path}")
        assert olen == n
        assert c.stats().path == 4
        for r in range(world):
            diff = _first_diff(out[r * per:(r + 1) * per], d_in[r * per:(r + 1) * per])
            assert diff is None, f"shard {r}: first difference at byte {diff}"
        del d_in, stream, out
    finally:
        c.close()
        _release()


def test_stream_over_4GiB_random(ctx):
    """A compressed stream of more than 4 GiB (5 GiB of random data: stored segments), one
    deflate call and one inflate call, compared on the device; the segment index reaches past
    byte 2^32 of the stream."""
    import torch
    n = 5 * GiB
    d_in = _device_corpus("random", n)
    _log("corpus on the device")
    cap = dmx.deflate_bound(n) + 64
    stream = torch.empty(cap, dtype=torch.uint8, device="cuda")
    total = ctx.deflate_device(d_in.data_ptr(), n, 2, stream.data_ptr(), cap)
    _log(f"deflated: {total} bytes")
    assert total > 4 * GiB
    out = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    olen = ctx.inflate_device(stream.data_ptr(), total, out.data_ptr(), n + 64)
    _log(f"inflated {olen} bytes on path {ctx.stats().path}")
    assert olen == n
    diff = _first_diff(out[:n], d_in)
    assert diff is None, f"first difference at byte {diff}"
    # the tail of the stream (past 4 GiB) is plain stored segments: check one by hand
    seg = n // 32768 - 1  # the last segment: BFINAL stored block of 32 KiB
    tail = stream[total - 32768 - 5: total].cpu().numpy().tobytes()
    assert tail[0] == 1 and tail[1:5] == b"\x00\x80\xff\x7f"
    assert tail[5:] == d_in[seg * 32768:].cpu().numpy().tobytes()
    del d_in, stream, out
    _release()
