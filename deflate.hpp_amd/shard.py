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

deflate_gather() pipelines this: ranks 1.. compress their shard in sub-shards on a side stream,
and each sub-shard's bytes go to rank 0 while the next one compresses; rank 0 compresses its own
shard straight into the output (one non-blocking call) and packs the other ranks' sub-shards
behind it at the end.
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


class _Lens:
    """Per-step compressed lengths that stay on the device while the next step compresses; each
    is read on the host one step later through a pinned copy and an event on the compression
    stream (never an .item() that would wait for the work behind it).  CPU tensors (the gloo
    tests) are read directly."""

    def __init__(self, count, dev):
        self.dev = dev
        self.d = torch.zeros(max(1, count), dtype=torch.int64, device=dev)
        self.cuda = dev.type == "cuda"
        self.h = torch.zeros(max(1, count), dtype=torch.int64, pin_memory=self.cuda)
        self.ev = [None] * max(1, count)
        self.stream = torch.cuda.Stream(dev) if self.cuda else None
        if self.cuda:
            # a pool stream does not order itself behind torch's current stream: the input (and
            # rank 0's output) may have been written by work still queued there
            self.stream.wait_stream(torch.cuda.current_stream(dev))

    def use(self, *tensors):
        """Tensors allocated on torch's current stream and read or written on the side stream:
        the caching allocator must not hand their memory out again before that work is done."""
        if self.cuda:
            for t in tensors:
                if t is not None and t.is_cuda:
                    t.record_stream(self.stream)

    def ptr(self, k):
        return self.d.data_ptr() + 8 * k

    def issued(self, k):  # after step k's compression was enqueued on self.stream
        if self.cuda:
            with torch.cuda.stream(self.stream):
                self.h[k].copy_(self.d[k], non_blocking=True)
                self.ev[k] = torch.cuda.Event()
                self.ev[k].record(self.stream)

    def read(self, k):  # the host value of step k; torch's stream then also waits for step k
        if not self.cuda:
            return int(self.d[k])
        self.ev[k].synchronize()
        torch.cuda.current_stream(self.dev).wait_event(self.ev[k])
        return int(self.h[k])


def _deflate(ctx, lens, k, src, n, level, dst, cap, not_final):
    """Enqueue one device deflate (length into lens step k): dmx's non-blocking call on the
    compression stream, or -- a codec without it (the CPU stand-in) -- the blocking one."""
    if hasattr(ctx, "deflate_device_async"):
        ctx.deflate_device_async(src, n, level, dst, cap, lens.ptr(k),
                                 stream=lens.stream.cuda_stream if lens.cuda else None, not_final=not_final)
    else:
        lens.d[k] = ctx.deflate_device(src, n, level, dst, cap, not_final=not_final)
    lens.issued(k)


def deflate_gather(ctx, d_in, n, level, out=None, sub=4, align=32768):
    """Compress this rank's device-resident shard d_in[:n] and gather every rank's stream on
    rank 0, the transfers pipelined behind the compression.

    Ranks r >= 1 cut the shard into `sub` sub-shards (multiples of `align`), each compressed
    NOT_FINAL except the last rank's last NON-EMPTY one, which carries BFINAL (a last rank with
    no bytes emits the empty final block 03 00, so the gathered stream always ends in BFINAL).
    Sub-shard k is enqueued on a side stream; then the length of k - 1 is read (it finished
    while k runs) and its length and bytes go to rank 0 by P2P.  Rank 0 compresses its whole
    shard with one non-blocking call straight into `out` (its bytes open the stream) and, while
    that runs, receives the other ranks' sub-shards: each length first, then the bytes into a
    buffer of exactly that size (staging = the compressed bytes of ranks 1.., not a worst-case
    bound per rank and step).  The stream is rank-major (rank r's input shard follows rank
    r - 1's), and rank r's offset is known only once every rank before it has finished, so
    rank 0 packs the received sub-shards behind its own bytes at the end: that copy of
    (world - 1) / world of the stream is inherent to the byte order.
    ctx: dmx.Context on this rank's GPU.  Returns (total stream bytes, this rank's bytes) on
    every rank; raises ValueError on every rank when rank 0's out is too small.
    """
    import dmx
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = d_in.device
    last = rank == world - 1
    cap0 = out.numel() if (rank == 0 and out is not None) else -1
    if rank == 0:
        # rank 0: one call; BFINAL only when it is also the last rank
        lens = _Lens(1, dev)
        need = dmx.deflate_bound(max(1, n)) + 64
        direct = cap0 >= need
        stage = None if direct else torch.empty(need, dtype=torch.uint8, device=dev)
        dst = out.data_ptr() if direct else stage.data_ptr()
        lens.use(d_in, out, stage)
        own = n > 0 or world == 1  # (an empty first shard adds no bytes; alone it is 03 00)
        if own:
            _deflate(ctx, lens, 0, d_in.data_ptr(), n, level, dst, need, world > 1)
        rbufs = [[None] * sub for _ in range(world)]
        lag = None  # (k, length tensors, requests) of the step whose payload receives are pending
        for k in range(sub if world > 1 else 0):
            got = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
            ops = []
            if lag is not None:  # receives in each sender's order: length k-1, bytes k-1, length k
                for q in lag[2]:
                    q.wait()
                for r in range(1, world):
                    L = int(lag[1][r].item())
                    if L:
                        rbufs[r][lag[0]] = torch.empty(L, dtype=torch.uint8, device=dev)
                        ops.append(dist.P2POp(dist.irecv, rbufs[r][lag[0]], r))
            ops += [dist.P2POp(dist.irecv, got[r], r) for r in range(1, world)]
            lag = (k, got, dist.batch_isend_irecv(ops))
        pend = []
        if lag is not None:
            for q in lag[2]:
                q.wait()
            ops = []
            for r in range(1, world):
                L = int(lag[1][r].item())
                if L:
                    rbufs[r][lag[0]] = torch.empty(L, dtype=torch.uint8, device=dev)
                    ops.append(dist.P2POp(dist.irecv, rbufs[r][lag[0]], r))
            if ops:
                pend = dist.batch_isend_irecv(ops)
        for q in pend:
            q.wait()
        mine = lens.read(0) if own else 0
    else:
        cuts = [min(n, -(-(n * k // sub) // align) * align) for k in range(sub + 1)]
        cuts[-1] = n
        nonempty = [k for k in range(sub) if cuts[k + 1] > cuts[k]]
        fin_k = (nonempty[-1] if nonempty else sub - 1) if last else None
        slot = dmx.deflate_bound(max([1] + [b - a for a, b in zip(cuts, cuts[1:])])) + 64
        stage = torch.empty(sub * slot, dtype=torch.uint8, device=dev)
        lens = _Lens(sub, dev)
        lens.use(d_in, stage)
        emitted = [False] * sub
        pend, keep = [], []

        def send(j):  # step j's length, then its bytes
            L = lens.read(j) if emitted[j] else 0
            lt = torch.tensor([L], dtype=torch.int64, device=dev)
            keep.append(lt)
            ops = [dist.P2POp(dist.isend, lt, 0)]
            if L:
                ops.append(dist.P2POp(dist.isend, stage[j * slot: j * slot + L], 0))
            pend.extend(dist.batch_isend_irecv(ops))
            return L

        mine = 0
        for k in range(sub):
            a, b = cuts[k], cuts[k + 1]
            if b > a or k == fin_k:
                _deflate(ctx, lens, k, d_in.data_ptr() + a, b - a, level, stage.data_ptr() + k * slot, slot,
                         k != fin_k)
                emitted[k] = True
            if k:
                mine += send(k - 1)
        mine += send(sub - 1)
        for q in pend:
            q.wait()
    st = _all_gather_ints([mine, cap0], dev) if world > 1 else [[mine, cap0]]
    total = sum(x[0] for x in st)
    if total and st[0][1] < total:
        raise ValueError("rank 0 needs an output buffer of at least the total stream size")
    if rank == 0:
        o = mine
        if not direct and mine:
            out[:mine].copy_(stage[:mine])
        for r in range(1, world):
            for k in range(sub):
                t = rbufs[r][k]
                if t is not None:
                    out[o: o + t.numel()].copy_(t)
                    o += t.numel()
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


def scatter_inflate(stream, clen, decode, starts=None, out=None, check=None, gather=True, balance="bytes",
                    decode_async=None):
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
    decode_async(piece, first) -> (res, buf): the same decode enqueued without a host sync
    (libdmx's dmx_inflate_device_async): res is a device int64 pair {bytes, status}, buf the
    output tensor.  The statuses travel in the one all_gather the ranks need anyway; a rank whose
    status is 1 (a piece the lane path does not take) decodes it again with decode().
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
    cap = out.numel() if (rank == 0 and out is not None) else -1
    st = None
    if decode_async is not None:
        # {ok, bytes, cap, status} per rank from device values: no host read before the gather
        res, buf = decode_async(piece[:plen], rank == 0) if plen else (None, None)
        mine = torch.tensor([1, 0, cap, 0], dtype=torch.int64, device=dev)
        if res is not None:
            mine[1:2].copy_(res[0:1])
            mine[3:4].copy_(res[1:2])
        parts = [torch.zeros(4, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.all_gather(parts, mine)
        st = [[int(x) for x in p.tolist()] for p in parts]
        if st[rank][3] == 0 and res is not None:
            dec = buf[: st[rank][1]]
        if any(x[3] != 0 for x in st):  # some rank needs the synchronous decode of its piece
            if st[rank][3] != 0:
                try:
                    dec = decode(piece[:plen], rank == 0)
                except Exception:
                    ok = 0
            st = _all_gather_ints([ok, 0 if dec is None else dec.numel(), cap], dev)
    elif plen:
        try:
            dec = decode(piece[:plen], rank == 0)
        except Exception:
            ok = 0
    if st is None:
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
