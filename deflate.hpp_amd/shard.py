"""Multi-GPU sharding of one DEFLATE stream.

Each rank compresses its contiguous shard of the input with DMX_DEFLATE_NOT_FINAL (every
segment, hence the shard, ends byte-aligned on an empty stored block), except the last rank
whose final block carries BFINAL.  The stream is the byte concatenation of the shards in rank
order; the one exchange step is a gather of the compressed shards to rank 0 over
torch.distributed (RCCL over xGMI on MI355X nodes, gloo for the CPU tests):

  1. all_gather of the per-rank compressed byte counts (and rank 0's output capacity, so that
     every rank sees a too-small buffer and raises together instead of one rank leaving the
     collective),
  2. rank 0 receives every shard at its prefix offset (batched P2P), others send.

deflate_gather() pipelines this: the shard is compressed in sub-shards, and each sub-shard's
bytes go to rank 0 (into a staging slot) while the next one compresses; rank 0 compresses its
own shard straight into the output and packs the other ranks' slots behind it at the end.
"""
import torch
import torch.distributed as dist


def shard_range(total, rank, world, align):
    """Contiguous [begin, end) of rank's shard, boundaries rounded to `align` (segment size)."""
    per = -(-total // world)
    per = -(-per // align) * align
    b = min(total, rank * per)
    return b, min(total, b + per)


def _all_gather_ints(vals, device):
    world = dist.get_world_size()
    t = torch.tensor(vals, dtype=torch.int64, device=device)
    parts = [torch.zeros(len(vals), dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(parts, t)
    return [[int(x) for x in p.tolist()] for p in parts]


def gather_sizes(clen, device):
    return [s[0] for s in _all_gather_ints([clen], device)]


def _p2p(ops):
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


def gather_stream(local, clen, out=None):
    """Gather the compressed shards (local[:clen] on every rank) into out on rank 0.

    Returns the total stream length on every rank; on rank 0 out[:total] holds the stream.
    Raises ValueError on EVERY rank when rank 0's out is too small; out=None only asks for the
    total (nothing is copied, the shards stay where they are).
    """
    rank, world = dist.get_rank(), dist.get_world_size()
    cap = out.numel() if (rank == 0 and out is not None) else -1
    st = _all_gather_ints([clen, cap, 1 if out is None else 0], local.device)
    sizes = [s[0] for s in st]
    total = sum(sizes)
    if st[0][2]:  # no output buffer on rank 0: the total only
        return total
    if total and st[0][1] < total:
        raise ValueError("rank 0 needs an output buffer of at least the total stream size")
    if world == 1:
        if clen:
            out[:clen].copy_(local[:clen])
        return total
    if rank == 0:
        offs = [sum(sizes[:r]) for r in range(world)]
        out[: sizes[0]].copy_(local[: sizes[0]])
        ops = [dist.P2POp(dist.irecv, out[offs[r]: offs[r] + sizes[r]], r) for r in range(1, world) if sizes[r]]
    else:
        ops = [dist.P2POp(dist.isend, local[:clen], 0)] if clen else []
    _p2p(ops)
    return total


def deflate_gather(ctx, d_in, n, level, out=None, sub=4, align=32768):
    """Compress this rank's device-resident shard d_in[:n] and gather every rank's stream on
    rank 0, the transfers pipelined behind the compression.

    The shard is cut into `sub` sub-shards (multiples of `align`), each compressed NOT_FINAL
    except the last rank's last NON-EMPTY one, which carries BFINAL (a last rank with no bytes
    emits the empty final block 03 00, so the gathered stream always ends in BFINAL).  After
    sub-shard k every rank r >= 1 sends its length and then its bytes to rank 0 (asynchronous
    P2P) and goes on compressing k + 1.  Rank 0 compresses its own shard straight into `out`
    (its bytes open the stream), posts the length receives of step k before compressing k + 1
    and reads them only after it (one step of lag: rank 0's compression never waits for the
    other ranks), then posts the payload receives into a per-rank staging buffer of the shard
    bound; at the end it packs ranks 1.. behind its own bytes (rank order, then k).
    ctx: dmx.Context on this rank's GPU.  Returns (total stream bytes, this rank's bytes) on
    every rank; raises ValueError on every rank when rank 0's out is too small.
    """
    import dmx
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = d_in.device
    last = rank == world - 1
    cuts = [min(n, -(-(n * k // sub) // align) * align) for k in range(sub + 1)]
    cuts[-1] = n
    nonempty = [k for k in range(sub) if cuts[k + 1] > cuts[k]]
    fin_k = (nonempty[-1] if nonempty else -1) if last else None
    slot = dmx.deflate_bound(max([1] + [b - a for a, b in zip(cuts, cuts[1:])])) + 64
    cap0 = out.numel() if (rank == 0 and out is not None) else -1
    direct = rank == 0 and cap0 >= sub * slot  # rank 0 compresses into out (room for any result)
    stage = None if direct else torch.empty(sub * slot, dtype=torch.uint8, device=dev)
    lens = [0] * sub
    rlens = [[0] * sub for _ in range(world)]
    rstage = [None] * world
    if rank == 0:
        for r in range(1, world):
            rstage[r] = torch.empty(sub * slot, dtype=torch.uint8, device=dev)
    pend, keep = [], []
    lag = None  # rank 0: (k, length tensors) whose payload receives are still to be posted

    def post_payloads(k, got):  # the payload receives of step k (its lengths have arrived)
        ops = []
        for r in range(1, world):
            Lr = int(got[r].item())
            rlens[r][k] = Lr
            if Lr:
                ops.append(dist.P2POp(dist.irecv, rstage[r][k * slot: k * slot + Lr], r))
        return ops

    o0 = 0
    for k in range(sub):
        a, b = cuts[k], cuts[k + 1]
        L = 0
        if b > a or k == fin_k or (fin_k == -1 and k == sub - 1):
            final = k == fin_k or (fin_k == -1 and k == sub - 1)
            if direct:
                dst, cap = out.data_ptr() + o0, slot
            else:
                dst, cap = stage.data_ptr() + k * slot, slot
            L = ctx.deflate_device(d_in.data_ptr() + a, b - a, level, dst, cap, not_final=not final)
        lens[k] = L
        if direct:
            o0 += L
        if world == 1:
            continue
        if rank == 0:
            # receives are posted in the order each rank sends (length k, payload k, length
            # k + 1, ...): P2P matching per peer is in posting order (RCCL, gloo)
            got = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
            ops = []
            if lag is not None:
                for q in lag[2]:
                    q.wait()
                ops = post_payloads(lag[0], lag[1])
            ops += [dist.P2POp(dist.irecv, got[r], r) for r in range(1, world)]
            reqs = dist.batch_isend_irecv(ops)
            lag = (k, got, reqs)
        else:
            lt = torch.tensor([L], dtype=torch.int64, device=dev)
            keep.append(lt)
            ops = [dist.P2POp(dist.isend, lt, 0)]
            if L:
                ops.append(dist.P2POp(dist.isend, stage[k * slot: k * slot + L], 0))
            pend += dist.batch_isend_irecv(ops)
    if lag is not None:
        for q in lag[2]:
            q.wait()
        ops = post_payloads(lag[0], lag[1])
        if ops:
            pend += dist.batch_isend_irecv(ops)
    for q in pend:
        q.wait()
    mine = sum(lens)
    st = _all_gather_ints([mine, cap0], dev) if world > 1 else [[mine, cap0]]
    total = sum(x[0] for x in st)
    if total and st[0][1] < total:
        raise ValueError("rank 0 needs an output buffer of at least the total stream size")
    if rank == 0:
        rlens[0] = lens
        rstage[0] = stage
        o = o0 if direct else 0
        for r in range(1 if direct else 0, world):
            for k in range(sub):
                L = rlens[r][k]
                if L:
                    out[o: o + L].copy_(rstage[r][k * slot: k * slot + L])
                    o += L
    return total, mine


# ---------------------------------------------------------------------------------------------
# inflate across ranks ("Inflate (our streams)"): rank 0 indexes the segment
# markers, picks one cut per rank among them -- only starts whose segment decodes to a closing
# marker (check) -- sends each rank its piece, every rank decodes its piece locally (pieces
# after the first in piece mode: a reference before the piece is an error, never silently
# dropped), and the decoded pieces are gathered back to rank 0 at their prefix offsets.
# ---------------------------------------------------------------------------------------------
FINAL_EMPTY = (0x03, 0x00)  # an empty final fixed-Huffman block: closes a NOT_FINAL piece
CHECK_NEAREST = 8           # candidates tried per cut, nearest to its target first


def _target(starts, total, world, r, balance):
    """Where cut r aims: r / world of the stream's bytes, or (balance == "count") the start of
    the (r / world)-th candidate segment -- equal output for libdmx's equal-size segments."""
    if balance == "count" and starts:
        return starts[min(len(starts) - 1, r * len(starts) // world)]
    return r * total // world


def split_points(starts, total, world, valid=None, balance="bytes"):
    """Piece boundaries [0, c_1, ..., c_{world-1}, total]: c_r is the candidate segment start
    nearest its target (_target) among those valid(start) accepts (boundaries strictly increase;
    a rank may get an empty piece)."""
    import bisect
    cuts = [0]
    for r in range(1, world):
        target = _target(starts, total, world, r, balance)
        i = bisect.bisect_left(starts, target)
        order = sorted((j for j in range(max(0, i - CHECK_NEAREST), min(len(starts), i + CHECK_NEAREST))),
                       key=lambda j: (abs(starts[j] - target), starts[j]))
        best = None
        for j in order:
            s = starts[j]
            if cuts[-1] < s < total and (valid is None or valid(s)):
                best = s
                break
        cuts.append(best if best is not None else cuts[-1])
    cuts.append(total)
    return cuts


def pick_cuts(starts, total, world, check=None, balance="bytes"):
    """split_points with the candidates near each target proven first by check(list of starts)
    -> list of end bytes (None: the segment does not decode) -- one batched call."""
    import bisect
    starts = sorted(starts)
    if check is None:
        return split_points(starts, total, world, balance=balance)
    near = set()
    for r in range(1, world):
        i = bisect.bisect_left(starts, _target(starts, total, world, r, balance))
        near.update(starts[max(0, i - CHECK_NEAREST): i + CHECK_NEAREST])
    near = sorted(s for s in near if 0 < s < total)
    ends = check(near) if near else []
    # the segment must end where a segment starts (its closing marker), or at the stream end
    # (its BFINAL block): a garbage start that stops early on some lenient block never does
    known = set(starts)
    ok = {s for s, e in zip(near, ends) if e is not None and s < e and (e in known or e == total)}
    return split_points(starts, total, world, valid=lambda s: s in ok, balance=balance)


def scatter_inflate(stream, clen, decode, starts=None, out=None, check=None, gather=True, balance="bytes"):
    """Inflate one stream held by rank 0 (stream[:clen]) on all ranks.

    decode(piece, first) -> 1-D uint8 tensor of decoded bytes, raising on a decode error; first
    is False for every piece but rank 0's, which must then be decoded in piece mode (libdmx's
    inflate_piece_device; tests pass a checker).  starts: rank 0's candidate segment starts
    (Context.segment_starts_device).  check: rank 0's cut-point proof (Context.
    segment_check_device), None to cut at raw candidates.  Returns (total decoded bytes, ok);
    on rank 0, out[:total] receives the decoded stream.  ok == False: a piece failed (a false
    candidate), every rank saw it, and rank 0 decoded the stream whole -- the result never
    depends on the split.  A stream that does not decode at all, or an out that is too small,
    raises on every rank.  gather=False leaves every rank's decoded piece where it was decoded
    (decode's own buffer; bench.py at N > 1): no byte goes back to rank 0 and out is unused
    except for the whole-stream fallback.  balance: cut targets by stream bytes, or by
    candidate count ("count": equal output for libdmx's equal-size segments).
    """
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = stream.device
    cut = torch.zeros(world + 1, dtype=torch.int64, device=dev)
    if rank == 0:
        try:
            cut.copy_(torch.tensor(pick_cuts(starts or [], clen, world, check, balance), dtype=torch.int64))
        except Exception:  # no split (rank 0 alone decodes) rather than a rank left in the collective
            cut.copy_(torch.tensor([0] + [clen] * world, dtype=torch.int64))
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
    _p2p(ops)
    plen = hi - lo
    if closes and plen:
        piece[plen: plen + 2].copy_(torch.tensor(FINAL_EMPTY, dtype=torch.uint8))
        plen += 2
    dec, ok = None, 1
    if plen:
        try:
            dec = decode(piece[:plen], rank == 0)
        except Exception:
            ok = 0
    cap = out.numel() if (rank == 0 and out is not None) else -1
    st = _all_gather_ints([ok, 0 if dec is None else dec.numel(), cap], dev)
    oks = [s[0] for s in st]
    sizes = [s[1] for s in st]
    if not all(oks):
        total = -1
        if rank == 0:
            try:
                full = decode(stream[:clen], True)
                total = full.numel()
                if total <= cap:
                    if total:
                        out[:total].copy_(full)
                else:
                    total = -2
            except Exception:
                total = -1
        t = torch.tensor([total], dtype=torch.int64, device=dev)
        dist.broadcast(t, 0)
        total = int(t.item())
        if total == -2:
            raise ValueError("rank 0 needs an output buffer of at least the decoded size")
        if total < 0:
            raise RuntimeError("scatter_inflate: the stream does not decode")
        return total, False
    total = sum(sizes)
    if not gather:
        return total, True
    if total and st[0][2] < total:
        raise ValueError("rank 0 needs an output buffer of at least the decoded size")
    if rank == 0:
        offs = [sum(sizes[:r]) for r in range(world)]
        if sizes[0]:
            out[: sizes[0]].copy_(dec)
        ops = [dist.P2POp(dist.irecv, out[offs[r]: offs[r] + sizes[r]], r) for r in range(1, world) if sizes[r]]
    else:
        ops = [dist.P2POp(dist.isend, dec, 0)] if sizes[rank] else []
    _p2p(ops)
    return total, True
