"""CPU, world_size 2 over gloo: the shard -> gather -> concatenate path of bench.py /
SURVEY 8(e).  GPU shards are stood in for by host-built shards in libdmx's segment format
(stored segments, each ending on an empty stored block; BFINAL only on the last rank's last
block), which is what dmx_deflate_device(..., DMX_DEFLATE_NOT_FINAL) produces at level 0."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import shard

SEG = 32768


def stored_shard(data, final):
    out = bytearray()
    for i in range(0, max(1, len(data)), SEG):
        chunk = data[i:i + SEG]
        last = final and i + SEG >= len(data)
        n = len(chunk)
        out += bytes([1 if last else 0]) + n.to_bytes(2, "little") + (n ^ 0xFFFF).to_bytes(2, "little") + chunk
        if not last:
            out += b"\x00\x00\x00\xff\xff"
    return bytes(out)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import dmx
    data = dmx.corpus("mixed", total)
    b, e = shard.shard_range(total, rank, world, SEG)
    local = stored_shard(data[b:e], final=(rank == world - 1))
    t = torch.frombuffer(bytearray(local), dtype=torch.uint8)
    out = torch.empty(2 * total + 1024, dtype=torch.uint8) if rank == 0 else None
    n = shard.gather_stream(t, len(local), out)
    if rank == 0:
        q.put(bytes(out[:n].numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_concatenates_valid_stream(oracle, world):
    total = 5 * SEG + 1234
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    stream = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    import dmx
    assert oracle.inflate(stream) == dmx.corpus("mixed", total)


def test_shard_ranges_cover_and_align():
    for total in (0, 1, SEG, 10 * SEG + 5, 1 << 30):
        for world in (1, 2, 3, 8):
            rs = [shard.shard_range(total, r, world, SEG) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            for (b0, e0), (b1, e1) in zip(rs, rs[1:]):
                assert e0 == b1 and (b1 % SEG == 0 or b1 == total)


# ---------------------------------------------------------------------------------------
# real libdmx output (tests/golden/dmx/, made on the GPU by make_dmx_fixtures.py)
# ---------------------------------------------------------------------------------------
GOLD_DMX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dmx")


def _dmx_manifest():
    import json
    return json.load(open(os.path.join(GOLD_DMX, "manifest.json")))


def _read(name):
    return open(os.path.join(GOLD_DMX, name), "rb").read()


def _markers(s):
    """Candidate segment starts: the byte after every 00 00 FF FF (what
    dmx_segment_starts_device returns on the GPU)."""
    out, i = [], s.find(b"\x00\x00\xff\xff")
    while i >= 0:
        out.append(i + 4)
        i = s.find(b"\x00\x00\xff\xff", i + 1)
    return out


def _gather_worker(rank, world, port, level, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = _read(f"mixed1M_L{level}_shard{rank}.deflate")
    t = torch.frombuffer(bytearray(local), dtype=torch.uint8)
    out = torch.empty(4 << 20, dtype=torch.uint8) if rank == 0 else None
    n = shard.gather_stream(t, len(local), out)
    if rank == 0:
        q.put(bytes(out[:n].numpy()))
    dist.destroy_process_group()


def _oracle_decode(orc):
    def decode(piece, first):  # the checker stands in for the GPU inflate on this CPU-only host
        return torch.frombuffer(bytearray(orc.inflate(piece.numpy().tobytes(), piece=not first)),
                                dtype=torch.uint8)
    return decode


def _oracle_decode_async(orc, refuse_rank=None):
    """Stand-in for Context.inflate_device_async: {bytes, status} in a tensor, status 1 when the
    piece does not decode (or, refuse_rank, always on that rank: the synchronous retry runs)."""
    def decode_async(piece, first):
        buf = torch.zeros(8 << 20, dtype=torch.uint8)
        res = torch.tensor([0, 1], dtype=torch.int64)
        if dist.get_rank() != refuse_rank:
            try:
                b = orc.inflate(piece.numpy().tobytes(), piece=not first)
                buf[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8) if b else buf[:0]
                res = torch.tensor([len(b), 0], dtype=torch.int64)
            except Exception:
                pass
        return res, buf
    return decode_async


def _oracle_check(orc, s):
    """Stand-in for Context.segment_check_device: the segment at c must decode in piece mode up
    to the first 00 00 FF FF after it (or to the stream end, as the final segment)."""
    def check(cands):
        ends = []
        for c in cands:
            m = s.find(b"\x00\x00\xff\xff", c)
            e = m + 4 if m >= 0 else len(s)
            piece = s[c:e] + (b"\x03\x00" if m >= 0 else b"")
            try:  # the decode must end exactly at the piece's end (no early BFINAL in garbage)
                _, used = orc.inflate_consumed(piece, piece=True)
                ends.append(e if used == len(piece) else None)
            except Exception:
                ends.append(None)
        return ends
    return check


def _scatter_case(name):
    """(stream, candidate starts) of a named case."""
    import zlib
    if name == "corrupt-split":  # a false marker as the only cut: the pieces fail, rank 0 decodes whole
        s = _read("mixed1M_L0_shard0.deflate") + _read("mixed1M_L0_shard1.deflate")
        return s, [len(s) // 2 + 7]
    if name == "false-marker":  # stored data holding 00 00 FF FF next to every cut target
        import dmx
        data = bytearray(dmx.corpus("random", 12 * SEG + 999, offset=5))
        for i in range(1000, len(data) - 8, 4 * 1024 + 3):
            data[i:i + 4] = b"\x00\x00\xff\xff"
        s = stored_shard(bytes(data), final=True)
        return s, _markers(s)
    if name == "sync-flush":  # zlib sync flush: markers at real block boundaries, window carried over
        import dmx
        d = dmx.corpus("text", 6 * SEG, offset=3)
        z = zlib.compressobj(6, zlib.DEFLATED, -15)
        s = b"".join(z.compress(d[i:i + SEG]) + z.flush(zlib.Z_SYNC_FLUSH) for i in range(0, len(d), SEG)) + z.flush()
        return s, _markers(s)
    if name == "garbage":  # not a deflate stream at all: every rank must raise, none may hang
        return bytes(range(256)) * 64, [1000, 5000]
    s = _read(name)
    return s, _markers(s)


def _scatter_worker(rank, world, port, name, use_check, out_cap, q, mode=None):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle_bind import Oracle
    orc = Oracle()
    s, starts = _scatter_case(name)
    stream = torch.frombuffer(bytearray(s), dtype=torch.uint8) if rank == 0 else torch.empty(0, dtype=torch.uint8)
    out = torch.empty(out_cap, dtype=torch.uint8) if rank == 0 else None
    try:
        da = None
        if mode == "async":
            da = _oracle_decode_async(orc)
        elif mode == "async-refuse":
            da = _oracle_decode_async(orc, refuse_rank=world - 1)
        total, ok = shard.scatter_inflate(stream, len(s) if rank == 0 else 0, _oracle_decode(orc),
                                          starts=starts if rank == 0 else None, out=out,
                                          check=_oracle_check(orc, s) if use_check else None, decode_async=da)
        res = (bytes(out[:total].numpy()), ok)
    except Exception as e:  # every rank reports (a rank that hung would time the test out)
        res = ("raised", type(e).__name__)
    q.put((rank, res))
    dist.destroy_process_group()


def _run(target, world, *args, all_ranks=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world if all_ranks else 1)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    if all_ranks:
        return dict(res)
    return res[0]


@pytest.mark.parametrize("level", [0, 2])
def test_gather_of_libdmx_shards(oracle, level):
    """Two NOT_FINAL / final shards made by dmx_deflate_device on the GPU, gathered over gloo:
    the concatenation is one valid stream of the whole corpus."""
    import dmx  # noqa: F401
    import hashlib
    m = _dmx_manifest()
    stream = _run(_gather_worker, 2, level)
    assert stream == _read(f"mixed1M_L{level}_shard0.deflate") + _read(f"mixed1M_L{level}_shard1.deflate")
    dec = oracle.inflate(stream)
    assert hashlib.sha256(dec).hexdigest() == hashlib.sha256(
        b"".join(oracle.inflate(_read(s["file"]) + (b"\x03\x00" if s["not_final"] else b""))
                 for s in m["streams"] if s["file"].startswith(f"mixed1M_L{level}_shard"))).hexdigest()
    assert len(dec) == m["corpus_total"]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("use_check", [False, True])
def test_scatter_inflate_libdmx_stream(oracle, world, use_check):
    """SURVEY 8(e) inflate: rank 0 cuts a libdmx stream at segment starts (raw candidates, or only
    those the segment check proves), every rank decodes its piece, the pieces gather back to
    rank 0 bit-exact."""
    import hashlib
    m = _dmx_manifest()
    full = next(s for s in m["streams"] if s["file"] == "mixed1M_L2.deflate")
    res = _run(_scatter_worker, world, "mixed1M_L2.deflate", use_check, 4 << 20, all_ranks=True)
    dec, ok = res[0]
    assert ok
    assert hashlib.sha256(dec).hexdigest() == full["out_sha256"]


def _scatter_worker_mode(rank, world, port, name, use_check, out_cap, mode, q):
    _scatter_worker(rank, world, port, name, use_check, out_cap, q, mode)


@pytest.mark.parametrize("mode", ["async", "async-refuse"])
def test_scatter_inflate_async_decode(oracle, mode):
    """the pieces decode through decode_async (dmx_inflate_device_async on a
    GPU) with their statuses in the ranks' one all_gather; a rank whose status says "not the lane
    path" decodes its piece again synchronously.  Same bytes either way; a corrupt split still
    falls back to rank 0's whole decode."""
    import hashlib
    m = _dmx_manifest()
    full = next(s for s in m["streams"] if s["file"] == "mixed1M_L2.deflate")
    res = _run(_scatter_worker_mode, 3, "mixed1M_L2.deflate", True, 4 << 20, mode, all_ranks=True)
    dec, ok = res[0]
    assert ok
    assert hashlib.sha256(dec).hexdigest() == full["out_sha256"]
    s = _read("mixed1M_L0_shard0.deflate") + _read("mixed1M_L0_shard1.deflate")
    dec, ok = _run(_scatter_worker_mode, 2, "corrupt-split", False, 4 << 20, mode, all_ranks=True)[0]
    assert not ok
    assert dec == oracle.inflate(s)


def test_scatter_inflate_false_marker_falls_back(oracle):
    """A cut at a 00 00 FF FF that is not a segment start: the piece before it over-reads, all
    ranks see the failure, rank 0 decodes the stream whole (same bytes)."""
    s = _read("mixed1M_L0_shard0.deflate") + _read("mixed1M_L0_shard1.deflate")
    dec, ok = _run(_scatter_worker, 2, "corrupt-split", False, 4 << 20, all_ranks=True)[0]
    assert not ok
    assert dec == oracle.inflate(s)


@pytest.mark.parametrize("world", [2, 3])
def test_scatter_inflate_false_markers_still_split(oracle, world):
    """00 00 FF FF inside stored data next to every cut target: the segment check rejects those
    candidates, the cuts move to proven segment starts, the split still happens (ok) and the
    bytes are exact; without the check a false cut is taken and the run falls back."""
    s, _ = _scatter_case("false-marker")
    dec, ok = _run(_scatter_worker, world, "false-marker", True, 1 << 20, all_ranks=True)[0]
    assert ok and dec == oracle.inflate(s)
    dec, ok = _run(_scatter_worker, world, "false-marker", False, 1 << 20, all_ranks=True)[0]
    assert dec == oracle.inflate(s)


@pytest.mark.parametrize("use_check", [False, True])
def test_scatter_inflate_sync_flush_stream_never_drops_bytes(oracle, use_check):
    """a zlib Z_SYNC_FLUSH stream has 00 00 FF FF at real block boundaries but its
    window carries across them.  Pieces after the first decode in piece mode, so a reference
    before the cut fails instead of silently copying nothing: the result is exact either way
    (the check refuses the cuts, or the pieces fail and rank 0 decodes whole)."""
    s, _ = _scatter_case("sync-flush")
    want = oracle.inflate(s)
    dec, ok = _run(_scatter_worker, 2, "sync-flush", use_check, 1 << 20, all_ranks=True)[0]
    assert dec == want
    if not use_check:
        assert not ok


def test_scatter_inflate_errors_raise_on_every_rank():
    """a stream that does not decode, or an output buffer that is too small, raises on
    every rank (no rank left blocking in a collective)."""
    res = _run(_scatter_worker, 2, "garbage", False, 1 << 20, all_ranks=True)
    assert res[0][0] == "raised" and res[1][0] == "raised"
    res = _run(_scatter_worker, 3, "mixed1M_L2.deflate", False, 1000, all_ranks=True)
    assert all(r[0] == "raised" and r[1] == "ValueError" for r in res.values())


class _HostDeflate:
    """CPU stand-in for dmx.Context.deflate_device: stored segments in libdmx's layout, read
    from and written to host pointers (torch CPU tensors)."""

    def deflate_device(self, d_in, n, level, d_out, cap, not_final=False):
        import ctypes
        s = stored_shard(ctypes.string_at(d_in, n), final=not not_final)
        assert len(s) <= cap
        ctypes.memmove(d_out, s, len(s))
        return len(s)


class _HostDeflateAsync(_HostDeflate):
    """The same with dmx.Context.deflate_device_async's interface: the length goes to an 8-byte
    buffer (here a host int64), as the GPU path of shard.deflate_gather uses it."""

    def deflate_device_async(self, d_in, n, level, d_out, cap, d_len, stream=None, not_final=False):
        import ctypes
        ctypes.c_int64.from_address(d_len).value = self.deflate_device(d_in, n, level, d_out, cap, not_final)


def _deflate_gather_worker(rank, world, port, total, sub, cuts, *rest):
    codec, q = rest if len(rest) == 2 else ("sync", rest[0])
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import dmx
    data = dmx.corpus("mixed", total)
    b, e = (cuts[rank], cuts[rank + 1]) if cuts else shard.shard_range(total, rank, world, SEG)
    d_in = torch.frombuffer(bytearray(data[b:e] or b"\0"), dtype=torch.uint8)
    out = torch.empty(2 * total + 4096, dtype=torch.uint8) if rank == 0 else None
    c = _HostDeflateAsync() if codec == "async" else _HostDeflate()
    n, mine = shard.deflate_gather(c, d_in, e - b, 0, out=out, sub=sub)
    q.put((rank, bytes(out[:n].numpy()) if rank == 0 else mine))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,sub", [(2, 3), (3, 4)])
def test_deflate_gather_pipelined_async_codec(oracle, world, sub):
    """The codec's non-blocking deflate (lengths left in device buffers, read one step late)."""
    import dmx
    total = 11 * SEG + 777
    res = _run(_deflate_gather_worker, world, total, sub, None, "async", all_ranks=True)
    assert oracle.inflate(res[0]) == dmx.corpus("mixed", total)


@pytest.mark.parametrize("world,sub", [(2, 3), (3, 4)])
def test_deflate_gather_pipelined(oracle, world, sub):
    """The pipelined gather (sub-shards sent while the next compresses) assembles the same
    single valid stream as the one-shot gather: the oracle decodes it to the corpus."""
    import dmx
    total = 11 * SEG + 777
    res = _run(_deflate_gather_worker, world, total, sub, None, all_ranks=True)
    stream = res[0]
    assert oracle.inflate(stream) == dmx.corpus("mixed", total)
    assert len(stream) == sum(v if r else 0 for r, v in res.items()) + \
        len(stream) - sum(v for r, v in res.items() if r)


@pytest.mark.parametrize("last_bytes", [0, 100, 2 * SEG, 3 * SEG])
def test_deflate_gather_short_last_shard(oracle, last_bytes):
    """the last rank's last NON-EMPTY sub-shard carries BFINAL.  A last shard of 0
    bytes (empty final block), of 100 bytes (sub-shards 1..3 empty) and of 2 or 3 segments with
    sub = 4 (trailing sub-shards empty) must all gather into a stream that ends in BFINAL."""
    import dmx
    first = 3 * SEG + 555
    total = first + last_bytes
    res = _run(_deflate_gather_worker, 2, total, 4, [0, first, total], all_ranks=True)
    stream = res[0]
    assert oracle.inflate(stream) == dmx.corpus("mixed", total)


def test_split_points():
    starts = [10, 20, 35, 50, 90]
    assert shard.split_points(starts, 100, 2) == [0, 50, 100]
    assert shard.split_points(starts, 100, 4) == [0, 20, 50, 90, 100]
    assert shard.split_points([], 100, 3) == [0, 0, 0, 100]
    c = shard.split_points(starts, 100, 8)
    assert c[0] == 0 and c[-1] == 100 and all(a <= b for a, b in zip(c, c[1:]))


class _HostCodec(_HostDeflate):
    """CPU stand-in for the dmx.Context entry points bench.dist_step calls, on host pointers:
    stored-segment deflate, the oracle as inflate (piece mode for pieces), a byte search for the
    segment starts and the oracle for the cut check."""

    def __init__(self):
        from oracle_bind import Oracle
        self.orc = Oracle()

    def _inflate(self, d_in, n, d_out, cap, piece):
        import ctypes
        out = self.orc.inflate(ctypes.string_at(d_in, n), piece=piece)
        if len(out) > cap:
            raise RuntimeError("capacity")
        ctypes.memmove(d_out, out, len(out))
        return len(out)

    def inflate_device(self, d_in, n, d_out, cap, stream=None):
        return self._inflate(d_in, n, d_out, cap, False)

    def inflate_piece_device(self, d_in, n, d_out, cap, stream=None):
        return self._inflate(d_in, n, d_out, cap, True)

    def inflate_device_async(self, d_in, n, d_out, cap, d_result, stream=None, piece=False):
        """{bytes, status} at d_result (int64 pair); status 1 when the piece does not decode here,
        so dist_step's synchronous retry runs (as on the GPU for a stream the lane path declines)."""
        import ctypes
        res = (ctypes.c_int64 * 2).from_address(d_result)
        try:
            res[0], res[1] = self._inflate(d_in, n, d_out, cap, piece), 0
        except Exception:
            res[0], res[1] = 0, 1

    def segment_starts_device(self, d_in, n, stream=None):
        import ctypes
        return _markers(ctypes.string_at(d_in, n))

    def segment_check_device(self, d_in, n, starts, stream=None):
        import ctypes
        return _oracle_check(self.orc, ctypes.string_at(d_in, n))(starts)


def _bench_worker(rank, world, port, per, sub, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import dmx
    dev = torch.device("cpu")
    run = bench.Runner(torch, _HostCodec(), dev, per, None)
    run.d_in[:per].copy_(torch.frombuffer(bytearray(dmx.corpus("mixed", per, offset=rank * per)), dtype=torch.uint8))
    total_n = world * per
    gathered = torch.empty(world * run.bound + 64, dtype=torch.uint8) if rank == 0 else None
    run.grow_out(total_n + 64 if rank == 0 else 2 * per + 4096)
    _, clen, olen, ok = bench.dist_step(torch, run.ctx, dev, run, 0, gathered, sub, None)
    good = bench.dist_verify(torch, dist, run, "mixed", olen, ok, dev, total_n)
    q.put((rank, (clen, olen, ok, good)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_distributed_step(world):
    """bench.py's N > 1 step on gloo with host stand-ins for the GPU codec: pipelined deflate +
    gather of one stream, proven cuts, piece-mode inflate on every rank; the decoded pieces
    together are the whole input (dist_verify), and the split held (ok)."""
    per = 7 * SEG + 1000
    res = _run(_bench_worker, world, per, 3, all_ranks=True)
    assert all(v[3] for v in res.values()), res
    assert all(v[2] for v in res.values()), res
    assert sum(v[1] for v in res.values()) == world * per
