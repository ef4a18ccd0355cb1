"""Multi-GPU sharding of one DEFLATE stream.

Each rank compresses its contiguous shard of the input with DMX_DEFLATE_NOT_FINAL (every
segment, hence the shard, ends byte-aligned on an empty stored block), except the last rank
whose final block carries BFINAL.  The stream is the byte concatenation of the shards in rank
order; the one exchange step is a gather of the compressed shards to rank 0 over
torch.distributed (RCCL over xGMI on MI355X nodes, gloo for the CPU tests):

  1. all_gather of the per-rank compressed byte counts,
  2. rank 0 receives every shard at its prefix offset (batched P2P), others send.
"""
import torch
import torch.distributed as dist


def shard_range(total, rank, world, align):
    """Contiguous [begin, end) of rank's shard, boundaries rounded to `align` (segment size)."""
    per = -(-total // world)
    per = -(-per // align) * align
    b = min(total, rank * per)
    return b, min(total, b + per)


def gather_sizes(clen, device):
    world = dist.get_world_size()
    sz = torch.tensor([clen], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, sz)
    return [int(s.item()) for s in sizes]


def gather_stream(local, clen, out=None):
    """Gather the compressed shards (local[:clen] on every rank) into out on rank 0.

    Returns the total stream length on every rank; on rank 0 out[:total] holds the stream.
    """
    rank, world = dist.get_rank(), dist.get_world_size()
    sizes = gather_sizes(clen, local.device)
    total = sum(sizes)
    if world == 1:
        if out is not None:
            out[:clen].copy_(local[:clen])
        return total
    if rank == 0:
        if out is None or out.numel() < total:
            raise ValueError("rank 0 needs an output buffer of at least the total stream size")
        offs = [sum(sizes[:r]) for r in range(world)]
        out[: sizes[0]].copy_(local[: sizes[0]])
        ops = [dist.P2POp(dist.irecv, out[offs[r]: offs[r] + sizes[r]], r) for r in range(1, world) if sizes[r]]
    else:
        ops = [dist.P2POp(dist.isend, local[:clen], 0)] if clen else []
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return total


# ---------------------------------------------------------------------------------------------
# inflate across ranks ("Inflate (our streams)"): rank 0 indexes the segment
# markers, cuts the stream into one contiguous piece per rank at segment starts, sends each rank
# its piece, every rank decodes its piece locally, and the decoded pieces are gathered back to
# rank 0 at their prefix offsets.
# ---------------------------------------------------------------------------------------------
FINAL_EMPTY = (0x03, 0x00)  # an empty final fixed-Huffman block: closes a NOT_FINAL piece


def split_points(starts, total, world):
    """Piece boundaries [0, c_1, ..., c_{world-1}, total]: c_r is the candidate segment start
    nearest r * total / world (boundaries strictly increase; a rank may get an empty piece)."""
    import bisect
    cuts = [0]
    for r in range(1, world):
        target = r * total // world
        i = bisect.bisect_left(starts, target)
        best = None
        for j in (i - 1, i):
            if 0 <= j < len(starts) and starts[j] > cuts[-1] and starts[j] < total:
                if best is None or abs(starts[j] - target) < abs(best - target):
                    best = starts[j]
        cuts.append(best if best is not None else cuts[-1])
    cuts.append(total)
    return cuts


def scatter_inflate(stream, clen, decode, starts=None, out=None):
    """Inflate one stream held by rank 0 (stream[:clen]) on all ranks.

    decode(piece) -> 1-D uint8 tensor of decoded bytes, raising on a decode error (libdmx's
    inflate_device on a GPU; tests pass a checker).  starts: rank 0's candidate segment starts
    (Context.segment_starts_device).  Returns (total decoded bytes, ok); on rank 0, out[:total]
    receives the decoded stream.  A false candidate (00 00 FF FF inside stored data) makes the
    piece before it fail; then every rank agrees on ok == False and rank 0 decodes the stream
    whole, so the result never depends on the split.
    """
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = stream.device
    cut = torch.zeros(world + 1, dtype=torch.int64, device=dev)
    if rank == 0:
        cut.copy_(torch.tensor(split_points(sorted(starts or []), clen, world), dtype=torch.int64))
    dist.broadcast(cut, 0)
    cuts = [int(x) for x in cut.tolist()]
    lo, hi = cuts[rank], cuts[rank + 1]
    closes = rank < world - 1
    piece = torch.empty(hi - lo + 2, dtype=torch.uint8, device=dev)
    if rank == 0:
        piece[: hi - lo].copy_(stream[lo:hi])
        ops = [dist.P2POp(dist.isend, stream[cuts[r]: cuts[r + 1]], r) for r in range(1, world)
               if cuts[r + 1] > cuts[r]]
    else:
        ops = [dist.P2POp(dist.irecv, piece[: hi - lo], 0)] if hi > lo else []
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    plen = hi - lo
    if closes and plen:
        piece[plen: plen + 2].copy_(torch.tensor(FINAL_EMPTY, dtype=torch.uint8))
        plen += 2
    dec, ok = None, 1
    if plen:
        try:
            dec = decode(piece[:plen])
        except Exception:
            ok = 0
    state = torch.tensor([ok, 0 if dec is None else dec.numel()], dtype=torch.int64, device=dev)
    states = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(states, state)
    oks = [int(s[0].item()) for s in states]
    sizes = [int(s[1].item()) for s in states]
    if not all(oks):
        total = 0
        if rank == 0:
            full = decode(stream[:clen])
            total = full.numel()
            if out is not None:
                out[:total].copy_(full)
        t = torch.tensor([total], dtype=torch.int64, device=dev)
        dist.broadcast(t, 0)
        return int(t.item()), False
    total = sum(sizes)
    if rank == 0:
        if out is None or out.numel() < total:
            raise ValueError("rank 0 needs an output buffer of at least the decoded size")
        offs = [sum(sizes[:r]) for r in range(world)]
        if sizes[0]:
            out[: sizes[0]].copy_(dec)
        ops = [dist.P2POp(dist.irecv, out[offs[r]: offs[r] + sizes[r]], r) for r in range(1, world) if sizes[r]]
    else:
        ops = [dist.P2POp(dist.isend, dec, 0)] if sizes[rank] else []
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return total, True
