"""Multi-GPU sharding of independent buffers: one process per GPU, buffers
assigned to ranks with no data-path collective, and one gather of the variable-length
compressed outputs to a destination rank at the end (RCCL over xGMI with the "nccl"
backend; gloo on CPU for the tests).

The batch is embarrassingly parallel -- every buffer is its own Brotli stream -- so the
only exchange is the final gather, sized by one all_gather of per-rank byte counts and done
as a single padded gather (RCCL has no gatherv; padding to the largest shard costs at most
the spread between ranks, small next to the shard itself).
"""
import torch
import torch.distributed as dist


def shard_indices(sizes, world, rank):
    """Size-balanced assignment (longest-processing-time greedy, deterministic): the
    indices of `sizes` that `rank` owns, in ascending order."""
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))
    load = [0] * world
    owner = [0] * len(sizes)
    for i in order:
        r = min(range(world), key=lambda q: (load[q], q))
        owner[i] = r
        load[r] += sizes[i]
    return [i for i in range(len(sizes)) if owner[i] == rank]


def gather_shards(local, lengths, dst=0, group=None):
    """Gather every rank's packed byte shard to `dst`.

    local:   1-D uint8 tensor holding this rank's streams back to back (on the backend's
             device: CUDA for nccl, CPU for gloo)
    lengths: list of this rank's stream lengths (sum <= local.numel())
    dst:     the destination's rank WITHIN `group` (= the global rank when group is None)
    Returns, on dst, a list over group ranks of (packed uint8 tensor, [lengths]); None elsewhere.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    # torch.distributed.gather takes a global rank for dst
    gdst = dst if group is None else dist.get_global_rank(group, dst)
    dev = local.device
    nbytes = int(sum(lengths))
    meta = torch.tensor([nbytes, len(lengths)], dtype=torch.int64, device=dev)
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    metas = [(int(m[0]), int(m[1])) for m in metas]
    max_bytes = max(1, max(m[0] for m in metas))
    max_count = max(1, max(m[1] for m in metas))
    # one padded gather for the bytes, one for the per-stream lengths
    send = torch.zeros(max_bytes, dtype=torch.uint8, device=dev)
    send[:nbytes] = local[:nbytes]
    lens = torch.zeros(max_count, dtype=torch.int64, device=dev)
    if lengths:
        lens[:len(lengths)] = torch.tensor(lengths, dtype=torch.int64, device=dev)
    if rank == dst:
        bufs = [torch.empty(max_bytes, dtype=torch.uint8, device=dev) for _ in range(world)]
        lbufs = [torch.empty(max_count, dtype=torch.int64, device=dev) for _ in range(world)]
        dist.gather(send, bufs, dst=gdst, group=group)
        dist.gather(lens, lbufs, dst=gdst, group=group)
        return [(bufs[r][:metas[r][0]], [int(x) for x in lbufs[r][:metas[r][1]].tolist()]) for r in range(world)]
    dist.gather(send, None, dst=gdst, group=group)
    dist.gather(lens, None, dst=gdst, group=group)
    return None
