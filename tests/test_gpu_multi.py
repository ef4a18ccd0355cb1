"""Single-process multi-GPU through the C-ABI (dmx_config.n_gpus) and the
non-blocking device deflate.  On a one-GPU box the shards are virtual: every sub-context lives on
device 0, which exercises the split, the per-shard streams and the reassembly exactly as on a
node (the reference's chunks are independent, deflate.hpp:689-697)."""
import pytest

import dmx

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("g", [2, 3, 8])
def test_n_gpus_host_api_matches_one_device(ctx, oracle, g):
    data = dmx.corpus("mixed", 9 << 20, offset=12345)
    one = ctx.compress(data, 2)
    multi = dmx.Context(n_gpus=g)
    try:
        s = multi.compress(data, 2)
        assert s == one  # shards NOT_FINAL + the last final: the one-device bytes
        assert multi.stats().shards == g
        assert multi.decompress(s) == data
        assert multi.stats().shards == g  # the stream was split at proven segment starts
        assert multi.decompress(s, cap=1000) == data[:1000]
        assert oracle.inflate(s) == data
        # a stream without markers (zlib's) does not split: one device decodes it
        import zlib
        z = zlib.compressobj(6, zlib.DEFLATED, -15)
        zs = z.compress(data) + z.flush()
        assert multi.decompress(zs) == data
        # small inputs stay on one device
        assert multi.compress(data[:1000], 2) == ctx.compress(data[:1000], 2)
    finally:
        multi.close()


def test_deflate_device_async_leaves_length_on_device(ctx):
    import torch
    data = dmx.corpus("text", 5 << 20)
    d_in = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    cap = dmx.deflate_bound(len(data)) + 64
    a = torch.empty(cap, dtype=torch.uint8, device="cuda")
    b = torch.empty(cap, dtype=torch.uint8, device="cuda")
    d_len = torch.zeros(2, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ctx.deflate_device_async(d_in.data_ptr(), len(data), 2, a.data_ptr(), cap, d_len.data_ptr(), stream=st)
    ctx.deflate_device_async(d_in.data_ptr(), len(data), 3, b.data_ptr(), cap, d_len.data_ptr() + 8, stream=st,
                             not_final=True)
    torch.cuda.synchronize()
    la, lb = (int(x) for x in d_len.tolist())
    n2 = ctx.deflate_device(d_in.data_ptr(), len(data), 2, b.data_ptr(), cap)
    assert la == n2
    ref = b[:n2].clone()
    assert torch.equal(a[:la], ref)
    assert ctx.decompress(a[:la].cpu().numpy().tobytes()) == data
    assert lb > 0
    # too small: the length says so, the call itself does not fail
    ctx.deflate_device_async(d_in.data_ptr(), len(data), 2, a.data_ptr(), 1000, d_len.data_ptr(), stream=st)
    torch.cuda.synchronize()
    assert int(d_len[0]) == la > 1000


def test_n_gpus_concatenated_streams_match_one_device(ctx, oracle):
    """Two libdmx streams back to back: the reference stops at the first BFINAL block, so the
    split decode must give exactly the one-device result (a piece that ends at an
    early BFINAL no longer passes as complete; the stream falls back to one device)."""
    a = dmx.corpus("mixed", 6 << 20, offset=7)
    b = dmx.corpus("text", 6 << 20, offset=99)
    s = ctx.compress(a, 2) + ctx.compress(b, 2)
    want = oracle.inflate(s)
    assert want == a
    assert ctx.decompress(s) == want
    multi = dmx.Context(n_gpus=2)
    try:
        assert multi.decompress(s) == want
    finally:
        multi.close()


def test_deflate_gather_waits_for_current_stream(ctx):
    """shard.deflate_gather compresses on a side stream: an input still being written by work
    queued on torch's current stream must be waited for.  World size 1 over gloo:
    no P2P, only the side-stream ordering is exercised."""
    import socket
    import torch
    import torch.distributed as dist
    import shard
    own_pg = not dist.is_initialized()
    if own_pg:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        data = dmx.corpus("text", 8 << 20, offset=5)
        src = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
        d_in = torch.zeros_like(src)
        torch.cuda.synchronize()
        # delay the current stream, then write the input behind the delay (all asynchronous)
        x = torch.full((2048, 2048), 1.0 / 2048, device="cuda")
        for _ in range(40):
            x = x @ x
        d_in.copy_(src)
        out = torch.empty(dmx.deflate_bound(len(data)) + 1024, dtype=torch.uint8, device="cuda")
        total, mine = shard.deflate_gather(ctx, d_in, len(data), 2, out=out)
        torch.cuda.synchronize()
        assert total == mine > 0
        assert ctx.decompress(out[:total].cpu().numpy().tobytes()) == data
    finally:
        if own_pg:
            dist.destroy_process_group()


def test_n_gpus_bound():
    """A garbage n_gpus (e.g. from a caller built against another dmx_config layout) is
    DMX_ERR_ARG, not thousands of sub-contexts."""
    with pytest.raises(dmx.DmxError) as e:
        dmx.Context(n_gpus=1 << 20)
    assert e.value.code == dmx.DMX_ERR_ARG


@pytest.mark.parametrize("seg", [32768, 65536])
def test_inflate_device_async(oracle, seg):
    """dmx_inflate_device_async: libdmx-layout streams decode with no host
    synchronisation -- the candidate count stays on the device -- and give the synchronous
    call's bytes; a stream of another layout (zlib's), a too-small cap or a piece whose first
    segment reaches back report status 1 for the caller's synchronous fallback.  Two calls on
    different streams are ordered by the context."""
    import zlib
    import torch
    c = dmx.Context(segment_bytes=seg)
    try:
        data = dmx.corpus("mixed", (24 << 20) + 777, offset=3)
        s = c.compress(data, 2)
        d_in = torch.frombuffer(bytearray(s), dtype=torch.uint8).cuda()
        d_o = torch.zeros(len(data) + 64, dtype=torch.uint8, device="cuda")
        d_r = torch.full((2,), 7, dtype=torch.int64, device="cuda")
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        c.inflate_device_async(d_in.data_ptr(), len(s), d_o.data_ptr(), d_o.numel(), d_r.data_ptr(),
                               stream=s1.cuda_stream)
        # a second call on another stream into another buffer: ordered behind the first
        d_o2 = torch.zeros_like(d_o)
        d_r2 = torch.full((2,), 7, dtype=torch.int64, device="cuda")
        c.inflate_device_async(d_in.data_ptr(), len(s), d_o2.data_ptr(), d_o2.numel(), d_r2.data_ptr(),
                               stream=s2.cuda_stream)
        torch.cuda.synchronize()
        for r, o in ((d_r, d_o), (d_r2, d_o2)):
            n, st = (int(x) for x in r.tolist())
            assert (n, st) == (len(data), 0)
            assert o[:n].cpu().numpy().tobytes() == data
        # another layout: status 1, and the synchronous call decodes it
        z = zlib.compressobj(1, zlib.DEFLATED, -15)
        zs = z.compress(data) + z.flush()
        d_z = torch.frombuffer(bytearray(zs), dtype=torch.uint8).cuda()
        c.inflate_device_async(d_z.data_ptr(), len(zs), d_o.data_ptr(), d_o.numel(), d_r.data_ptr())
        torch.cuda.synchronize()
        assert int(d_r[1]) == 1
        assert c.inflate_device(d_z.data_ptr(), len(zs), d_o.data_ptr(), d_o.numel()) == len(data)
        # output beyond cap: status 1
        c.inflate_device_async(d_in.data_ptr(), len(s), d_o.data_ptr(), len(data) // 2, d_r.data_ptr())
        torch.cuda.synchronize()
        assert int(d_r[1]) == 1
        # a piece cut at a proven segment start, closed with an empty final block, piece mode
        starts = c.segment_starts_device(d_in.data_ptr(), len(s))
        cut = starts[len(starts) // 2]
        piece = s[cut:]
        d_p = torch.frombuffer(bytearray(piece), dtype=torch.uint8).cuda()
        c.inflate_device_async(d_p.data_ptr(), len(piece), d_o.data_ptr(), d_o.numel(), d_r.data_ptr(), piece=True)
        torch.cuda.synchronize()
        n, st = (int(x) for x in d_r.tolist())
        assert st == 0
        want = oracle.inflate(piece)
        assert d_o[:n].cpu().numpy().tobytes() == want == data[len(data) - len(want):]
    finally:
        c.close()
