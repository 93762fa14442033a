#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: encode+decode MB/s at q11 lgwin=22 on 1/2/4/8 MI355X.

Workload (one "step" = one pass of the hot path over one batch):
  C4 per-GPU shard: 1024 independent 1 MiB enwik-style text buffers per GPU, resident in
  HBM, quality 11, lgwin 22, GENERIC mode.  A step encodes the shard (mib_ctx_encode:
  packed compressed streams in HBM), gathers the compressed shards to rank 0 over RCCL
  (N > 1; the only collective) and decodes the shard back
  (mib_ctx_decode) into HBM.  Round-trip bit-exactness is checked on device after the
  warmup steps (outside the timed region).
  value = uncompressed MB (10^6 B) processed by all ranks / step time (max over ranks).
  scaling "weak": per-GPU work fixed as N grows.

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 via torch.distributed.run
(one rank per GPU, backend nccl = RCCL).

roofline: the step's dominant kernel (largest device time, HIP events recorded by the
library on the launch stream), achieved = algorithmic bytes of one launch (input +
output bytes of the streams it processed) / its mean launch time;
peak = 8.0 TB/s HBM3E (MI355X_MICROARCH.md).  traffic = HBM bytes per launch from the
rocprofv3 PMC passes committed in profiles/ (scripts/collect_pmc.sh), or null.

cpu_baseline: the oracle (CPU restatement of the reference's q11 encoder + decoder,
oracle/) on a bounded sample of the same workload, one buffer per host thread, rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))

MIB = 1 << 20
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--streams', type=int, default=1024, help='buffers per GPU')
    ap.add_argument('--size', type=int, default=MIB, help='bytes per buffer')
    ap.add_argument('--quality', type=int, default=11)
    ap.add_argument('--lgwin', type=int, default=22)
    ap.add_argument('--cpu-sample', type=int, default=-1, help='buffers in the CPU baseline sample (-1 auto)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-gather', action='store_true')
    return ap.parse_args()


def cpu_baseline(args):
    """Oracle q11 encode + decode of 1 MiB buffers, one per thread (ctypes drops the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import _oracle
    from brotli_amd import datagen
    threads = max(1, min(16, os.cpu_count() or 1))
    nbuf = args.cpu_sample if args.cpu_sample > 0 else threads
    bufs = [datagen.enwik_text(args.size, 2000 + i) for i in range(nbuf)]
    _oracle.lib()

    def one(d):
        e = _oracle.encode(d, args.quality, args.lgwin)
        assert _oracle.decode(e) == d
        return len(e)

    t0 = time.time()
    with ThreadPoolExecutor(threads) as ex:
        sizes = list(ex.map(one, bufs))
    dt = time.time() - t0
    return {'value': round(nbuf * args.size / 1e6 / dt, 4), 'unit': 'MB/s', 'cores': min(threads, nbuf),
            'kind': 'port',
            'sample': '%d x %d B enwik-style buffers (seeds 2000+i), oracle q%d encode + decode, %d threads, %.1f s wall, '
                      'ratio %.4f' % (nbuf, args.size, args.quality, min(threads, nbuf), dt,
                                      sum(sizes) / (nbuf * args.size))}


def load_traffic(kernel, launch_bytes):
    """HBM bytes per launch of `kernel` from profiles/pmc_summary.json (collect_pmc.sh)."""
    p = os.path.join(ROOT, 'profiles', 'pmc_summary.json')
    try:
        with open(p) as f:
            d = json.load(f)
        k = d['kernels'][kernel]
        return int(k['hbm_bytes_per_launch'])
    except Exception:
        return None


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args)   # before any device work

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)
    import brotli_amd
    from brotli_amd import datagen, shard

    k, size = args.streams, args.size
    total = k * size
    data = datagen.enwik_device(total, 2000 + rank, dev)
    in_off = [i * size for i in range(k + 1)]
    cap = total + total // 8 + 4096 * k
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    # output slots with room for a one-metablock stream's ring: the decoder writes in place
    slot = size + 4096
    dec = torch.empty(k * slot, dtype=torch.uint8, device=dev)
    dec_off = [i * slot for i in range(k + 1)]
    ctx = brotli_amd.DeviceContext(local, profiling=True)
    opts = {'quality': args.quality, 'lgwin': args.lgwin}

    def step(times):
        out_off = ctx.encode(data.data_ptr(), in_off, comp.data_ptr(), cap, opts)
        for name, (ms, n) in ctx.kernel_times().items():
            t = times.setdefault(name, [0.0, 0])
            t[0] += ms
            t[1] += n
        if world > 1 and not args.no_gather:
            # the one collective: RCCL gather of the variable-length compressed shards to rank 0
            lens = [out_off[i + 1] - out_off[i] for i in range(k)]
            shard.gather_shards(comp[:out_off[-1]], lens, dst=0)
        sizes, status = ctx.decode(comp.data_ptr(), out_off, dec.data_ptr(), dec_off)
        for name, (ms, n) in ctx.kernel_times().items():
            t = times.setdefault(name, [0.0, 0])
            t[0] += ms
            t[1] += n
        return out_off, sizes, status

    for w in range(max(1, args.warmup)):
        out_off, sizes, status = step({})
    torch.cuda.synchronize()
    bad = [i for i in range(k) if status[i] != 0 or sizes[i] != size]
    if bad or not torch.equal(dec.view(k, slot)[:, :size], data.view(k, size)):
        raise SystemExit('round trip FAILED on rank %d: %d bad streams' % (rank, len(bad)))
    comp_bytes = out_off[-1]

    times = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out_off, sizes, status = step(times)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        cb = torch.tensor([comp_bytes], dtype=torch.int64, device=dev)
        dist.all_reduce(cb)
        comp_all = int(cb.item())
    else:
        comp_all = comp_bytes
    if rank == 0:
        ms_step = dt * 1e3 / args.steps
        mb = world * total / 1e6
        enc_ms = sum(v[0] for n, v in times.items() if n != 'decode_streams_kernel') / args.steps
        dec_ms = times.get('decode_streams_kernel', [0.0, 1])[0] / args.steps
        dom = max(times.items(), key=lambda kv: kv[1][0])
        dom_name, (dom_ms, dom_n) = dom[0], dom[1]
        # a kernel launched L times per step covers 1/L of the shard per launch
        launches_per_step = max(1, dom_n // args.steps)
        launch_bytes = (total + comp_bytes) // launches_per_step
        avg_ms = dom_ms / max(1, dom_n)
        achieved = launch_bytes / (avg_ms * 1e-3) / 1e9
        res = {
            'metric': 'encode+decode MB/s at q11 lgwin=22',
            'value': round(mb / dt * args.steps, 3),
            'unit': 'MB/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(ms_step, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'u8',
            'data': 'synthetic',
            'config': {'workload': 'C4 per-GPU shard: %d x %d B enwik-style text, q%d lgwin%d GENERIC, encode -> %s'
                                   'decode round trip (bit-exact checked)' % (
                                       k, size, args.quality, args.lgwin, 'RCCL gather -> ' if world > 1 else ''),
                       'streams_per_gpu': k, 'bytes_per_stream': size, 'quality': args.quality, 'lgwin': args.lgwin,
                       'parallelism': 'shard%d' % world},
            'encode_MBps': round(mb / (enc_ms * 1e-3), 3) if enc_ms else None,
            'decode_MBps': round(mb / (dec_ms * 1e-3), 3) if dec_ms else None,
            'compressed_ratio': round(comp_all / (world * total), 5),
            'kernel_ms_per_step': {n: round(v[0] / args.steps, 3) for n, v in sorted(times.items())},
            'roofline': {'bound': 'hbm', 'kernel': dom_name, 'achieved': round(achieved, 3), 'peak': PEAK_HBM_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / PEAK_HBM_GBS, 6),
                         'traffic': load_traffic(dom_name, launch_bytes),
                         'algorithmic_bytes_per_launch': launch_bytes, 'avg_launch_ms': round(avg_ms, 3)},
            'cpu_baseline': cpu,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
