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
