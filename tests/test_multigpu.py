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


def _scatter_worker(rank, world, port, name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle_bind import Oracle
    orc = Oracle()

    def decode(piece):  # the checker stands in for the GPU inflate on this CPU-only host
        return torch.frombuffer(bytearray(orc.inflate(piece.numpy().tobytes())), dtype=torch.uint8)

    if name == "corrupt-split":  # a false marker as the cut: the pieces fail, rank 0 decodes whole
        s = _read("mixed1M_L0_shard0.deflate") + _read("mixed1M_L0_shard1.deflate")
        starts = [len(s) // 2 + 7]
    else:
        s = _read(name)
        starts = _markers(s)
    stream = torch.frombuffer(bytearray(s), dtype=torch.uint8) if rank == 0 else torch.empty(0, dtype=torch.uint8)
    out = torch.empty(4 << 20, dtype=torch.uint8) if rank == 0 else None
    total, ok = shard.scatter_inflate(stream, len(s) if rank == 0 else 0, decode,
                                      starts=starts if rank == 0 else None, out=out)
    if rank == 0:
        q.put((bytes(out[:total].numpy()), ok))
    dist.destroy_process_group()


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return res


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
def test_scatter_inflate_libdmx_stream(oracle, world):
    """SURVEY 8(e) inflate: rank 0 cuts a libdmx stream at segment starts, every rank decodes its
    piece, the pieces gather back to rank 0 bit-exact."""
    import hashlib
    m = _dmx_manifest()
    full = next(s for s in m["streams"] if s["file"] == "mixed1M_L2.deflate")
    dec, ok = _run(_scatter_worker, world, "mixed1M_L2.deflate")
    assert ok
    assert hashlib.sha256(dec).hexdigest() == full["out_sha256"]


def test_scatter_inflate_false_marker_falls_back(oracle):
    """A cut at a 00 00 FF FF that is not a segment start: the piece before it over-reads, all
    ranks see the failure, rank 0 decodes the stream whole (same bytes)."""
    s = _read("mixed1M_L0_shard0.deflate") + _read("mixed1M_L0_shard1.deflate")
    dec, ok = _run(_scatter_worker, 2, "corrupt-split")
    assert not ok
    assert dec == oracle.inflate(s)


def test_split_points():
    starts = [10, 20, 35, 50, 90]
    assert shard.split_points(starts, 100, 2) == [0, 50, 100]
    assert shard.split_points(starts, 100, 4) == [0, 20, 50, 90, 100]
    assert shard.split_points([], 100, 3) == [0, 0, 0, 100]
    c = shard.split_points(starts, 100, 8)
    assert c[0] == 0 and c[-1] == 100 and all(a <= b for a, b in zip(c, c[1:]))
