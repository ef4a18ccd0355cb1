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
