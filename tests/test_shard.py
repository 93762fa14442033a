"""The N > 1 path on CPU: world_size-2 gloo processes shard a batch of buffers and gather
their variable-length outputs to rank 0 (brotli_amd.shard, used by bench.py with RCCL).

The per-rank "encode" here is a length-changing byte transform (the GPU encoder is covered
by the gpu tests): what is checked is that every buffer is owned by exactly one rank and
that rank 0 reassembles every output in the original order."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from brotli_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _transform(b):
    return bytes(reversed(b)) + bytes([len(b) % 251])


def _worker(rank, world, port, sizes, out_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    bufs = [bytes((i * 7 + j) & 0xFF for j in range(n)) for i, n in enumerate(sizes)]
    mine = shard.shard_indices(sizes, world, rank)
    outs = [_transform(bufs[i]) for i in mine]
    packed = torch.tensor(list(b''.join(outs)) or [0], dtype=torch.uint8)
    got = shard.gather_shards(packed, [len(o) for o in outs], dst=0)
    own = torch.zeros(len(sizes), dtype=torch.int64)
    for i in mine:
        own[i] = 1
    dist.all_reduce(own)
    if rank == 0:
        assign = [shard.shard_indices(sizes, world, r) for r in range(world)]
        result = [None] * len(sizes)
        for r, (data, lens) in enumerate(got):
            raw = bytes(data.tolist())
            off = 0
            for idx, ln in zip(assign[r], lens):
                result[idx] = raw[off:off + ln]
                off += ln
        ok = all(result[i] == _transform(bufs[i]) for i in range(len(sizes)))
        out_q.put((ok, own.tolist(), [len(a) for a in assign]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('sizes', [[5, 900, 0, 33, 1024, 77, 300, 1], [100] * 7, [3]])
def test_gloo_world2_shard_and_gather(sizes):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, own, counts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert ok
    assert own == [1] * len(sizes)   # every buffer encoded by exactly one rank
    assert sum(counts) == len(sizes)


def test_shard_balance():
    sizes = [1 << 20] * 1024
    parts = [shard.shard_indices(sizes, 8, r) for r in range(8)]
    assert sorted(sum(parts, [])) == list(range(1024))
    assert all(len(p) == 128 for p in parts)


def _sub_worker(rank, world, port, out_q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    group = dist.new_group([1, 2])   # a subgroup whose rank 0 is global rank 1
    if rank in (1, 2):
        payload = bytes([rank]) * (10 + rank)
        packed = torch.tensor(list(payload), dtype=torch.uint8)
        got = shard.gather_shards(packed, [len(payload)], dst=0, group=group)
        if rank == 1:
            out_q.put([(bytes(d.tolist()), lens) for d, lens in got])
        else:
            assert got is None
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_subgroup_gather_dst_is_group_rank():
    """gather_shards(dst=0, group=g) delivers to g's rank 0 (global rank 1), not global rank 0."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sub_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == [(b'\x01' * 11, [11]), (b'\x02' * 12, [12])]
