#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric: encode+decode MB/s at q11 lgwin=22 on 1/2/4/8 MI355X.

Workloads (one "step" = one pass of the hot path over one batch; inputs are
resident in HBM when the timed region starts):
  c4 (default)  C4 per-GPU shard: 1024 independent 1 MiB enwik-style text buffers per GPU,
                q11, lgwin 22, GENERIC -- the configuration the metric's 1/2/4/8-GPU
                numbers are quoted on.
  c3            C3: 1024 x 256 KiB WOFF2-transformed glyf tables per GPU (glyph sets drawn from
                the reference's Inter bench font, jittered per seed), q11, FONT.
  c2            C2: one 64 MiB enwik-style buffer, q11 GENERIC (one stream: replicas at N > 1).
  c5            C5's shape per GPU: one stream streamed through BrotliEncoder.update() in 1 MiB
                chunks (history window carried on the device), q9 lgwin 24 TEXT, then decoded
                (64 MiB by default: --size for more).
  ref           decode of the reference's own bench streams (noto-tc etc.), one stream per
                call: the single-stream latency case of the reference's README.
  latency       one brotliEncode + one brotliDecode per call of the reference's encode bench
                inputs (13 B .. 45 KB) and C1 through the host API, next to README.md:88-94.
A step encodes the batch (mib_ctx_encode: packed compressed streams in HBM), gathers the
compressed shards to rank 0 over RCCL (N > 1, c3/c4; the only collective)
and decodes them back (mib_ctx_decode) into HBM.  The round trip is checked bit-exact on
device after the warmup steps (outside the timed region).
  value = uncompressed MB (10^6 B) processed by all ranks / step time (max over ranks).
  scaling "weak": per-GPU work fixed as N grows.

Launch: python bench.py [--gpus N --steps K --warmup W --workload c4|c3|c2]; N > 1 via
torch.distributed.run (one rank per GPU, backend nccl = RCCL).

roofline: the step's dominant kernel (largest device time, HIP events recorded by the
library on the launch stream); achieved = algorithmic bytes of one launch (input + output
bytes of the streams it processed) / its mean launch time; peak = 8.0 TB/s
HBM3E (MI355X_MICROARCH.md).  traffic = HBM bytes per launch from the rocprofv3 PMC passes
committed in profiles/ (scripts/collect_pmc.py), or null.

cpu_baseline: the oracle (CPU restatement of the reference's q11 encoder + decoder,
oracle/) on a bounded sample of the SAME buffers the GPU encoded (copied back from HBM),
one buffer per host thread on every core of this process's CPU share, rank 0 only.  The
same sample gives the compressed-size comparison GPU vs reference (ref-fixed) vs Node's
native brotli (when `node` exists), all on identical bytes.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))

MIB = 1 << 20
PEAK_HBM_GBS = 8000.0
WORKLOADS = {
    # name: (streams per GPU, bytes per stream, mode, seed base, generator)
    'c4': (1024, MIB, 0, 2000, 'enwik'),
    'c3': (1024, 256 * 1024, 2, 1000, 'glyf'),
    'c2': (1, 64 * MIB, 0, 2, 'enwik'),
    # C5's per-GPU stream: 1 GiB through BrotliEncoder.update() in 1 MiB chunks, q9 lgwin 24,
    # custom dictionary, then one decode of the whole stream
    'c5': (1, 1024 * MIB, 1, 5000, 'enwik'),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--workload', default='c4', choices=sorted(WORKLOADS) + ['ref', 'latency'])
    ap.add_argument('--streams', type=int, default=-1, help='buffers per GPU (-1: the workload\'s)')
    ap.add_argument('--size', type=int, default=-1, help='bytes per buffer (-1: the workload\'s)')
    ap.add_argument('--quality', type=int, default=11)
    ap.add_argument('--lgwin', type=int, default=22)
    ap.add_argument('--cpu-seconds', type=float, default=10.0, help='target wall time of the CPU baseline sample')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-gather', action='store_true')
    ap.add_argument('--kernel-events', default=None, choices=['all', 'decode'],
                    help='c4/c3/c2: HIP events around every kernel of the timed steps (all), or the decoder\'s '
                         'only, the encoder\'s table then from one untimed step after them (decode). Default: '
                         'decode, except c3, whose dominant kernel is the encoder\'s DP (events on every kernel '
                         'cost C4 ~1.3 %% of its MB/s, 2.3 %% of its encode)')
    ap.add_argument('--stream-chunk', type=int, default=32, help='c5: BrotliEncoder streamChunk in MiB (0: the reference\'s cadence)')
    ap.add_argument('--gpus-in-lib', type=int, default=0,
                    help='host-API leg: the batch through mib_*_batch_n with N shards against the one-context batch')
    return ap.parse_args()


def cpu_share():
    """CPUs this process may use: its affinity mask, capped by a cgroup CPU quota and by the
    box's per-GPU share (OMP_NUM_THREADS is set to it on the GPU boxes; os.cpu_count()
    shows the whole machine there)."""
    n = len(os.sched_getaffinity(0))
    if os.environ.get('OMP_NUM_THREADS', '').isdigit():
        n = min(n, int(os.environ['OMP_NUM_THREADS']))
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, p = f.read().split()
        if q != 'max':
            n = min(n, max(1, int(int(q) // int(p))))
    except Exception:
        pass
    return max(1, n)


def make_inputs(wl, k, size, rank, dev):
    """The batch, generated straight into HBM (k streams of `size` bytes, packed)."""
    import numpy as np
    import torch
    from brotli_amd import datagen
    _, _, _, seed0, gen = WORKLOADS[wl]
    if gen == 'enwik':
        # one device-generated text, cut into k buffers (seed per rank)
        return datagen.enwik_device(k * size, seed0 + rank * 7919, dev)
    # C3: WOFF2-transformed glyf tables of glyph sets drawn from the reference's Inter bench
    # font, jittered per seed (the GPU's own glyf transform, §8 f4)
    bufs = datagen.glyf_font_batch(k, size, seed0 + rank * k, workers=max(1, min(16, cpu_share())))
    host = np.frombuffer(b''.join(bufs), dtype=np.uint8)
    return torch.from_numpy(host.copy()).to(dev)


def node_native(sample, quality, lgwin, mode):
    """Node's bundled native brotli (zlib.brotliCompressSync) on the same sample: sizes."""
    try:
        subprocess.run(['node', '--version'], check=True, capture_output=True, timeout=30)
    except Exception:
        return None
    with tempfile.TemporaryDirectory() as td:
        paths = []
        for i, b in enumerate(sample):
            p = os.path.join(td, '%d.bin' % i)
            with open(p, 'wb') as f:
                f.write(b)
            paths.append(p)
        js = ("const z=require('zlib'),fs=require('fs');let t=0,s=0;const c=z.constants;"
              "for(const p of process.argv.slice(1)){const d=fs.readFileSync(p);const t0=process.hrtime.bigint();"
              "const e=z.brotliCompressSync(d,{params:{[c.BROTLI_PARAM_QUALITY]:%d,[c.BROTLI_PARAM_LGWIN]:%d,"
              "[c.BROTLI_PARAM_MODE]:%d,[c.BROTLI_PARAM_SIZE_HINT]:d.length}});t+=Number(process.hrtime.bigint()-t0);s+=e.length;}"
              "console.log(JSON.stringify({bytes:s,ns:t}));" % (quality, lgwin, mode))
        # one node process per host thread of this process's CPU share, the buffers dealt out
        groups = [paths[g::max(1, min(cpu_share(), len(paths)))] for g in range(max(1, min(cpu_share(), len(paths))))]
        try:
            procs = [subprocess.Popen(['node', '-e', js] + g, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL) for g in groups]
            out = {'bytes': 0, 'ns': 0}
            for pr in procs:
                so, _ = pr.communicate(timeout=600)
                if pr.returncode != 0:
                    return None
                r = json.loads(so.decode().strip().splitlines()[-1])
                out['bytes'] += r['bytes']
                out['ns'] += r['ns']   # (summed over processes: one core's time)
            return out
        except Exception:
            return None


def cpu_baseline(sample, gpu_sizes, args, mode, what):
    """Oracle q11 encode + decode of the sample buffers, one per thread (ctypes drops the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    import _oracle
    _oracle.lib()
    threads = cpu_share()

    bad = []

    def one(d):
        e = _oracle.encode(d, args.quality, args.lgwin, mode)
        if _oracle.decode(e) != d:   # the reference encoder's own output failing its round trip
            bad.append(d)
            if os.environ.get('BENCH_DUMP_DIR'):
                os.makedirs(os.environ['BENCH_DUMP_DIR'], exist_ok=True)
                with open(os.path.join(os.environ['BENCH_DUMP_DIR'], 'oracle_bad_%d.bin' % len(bad)), 'wb') as f:
                    f.write(d)
                with open(os.path.join(os.environ['BENCH_DUMP_DIR'], 'oracle_bad_%d.br' % len(bad)), 'wb') as f:
                    f.write(e)
        return len(e)

    # bounded: whole rounds of `threads` buffers until the target time is reached
    sizes, done, t0 = [], 0, time.time()
    with ThreadPoolExecutor(threads) as ex:
        while done < len(sample) and (time.time() - t0) < args.cpu_seconds:
            batch = sample[done:done + threads]
            sizes += list(ex.map(one, batch))
            done += len(batch)
    dt = time.time() - t0
    nbytes = sum(len(b) for b in sample[:done])
    ratio_ref = sum(sizes) / nbytes
    ratio_gpu = sum(gpu_sizes[:done]) / nbytes
    nn = min(done, 32)   # native brotli q11 runs ~1 MB/s a core: a sub-sample, one node process per thread
    nat = node_native(sample[:nn], args.quality, args.lgwin, mode)
    nn_bytes = sum(len(b) for b in sample[:nn])
    return {'value': round(nbytes / 1e6 / dt, 4), 'unit': 'MB/s', 'cores': min(threads, done), 'kind': 'port',
            'sample': '%d x %d B %s (the first buffers the GPU encoded, copied back), oracle q%d encode + decode, '
                      '%d threads (host nproc %d, CPU share %d), %.1f s wall' % (
                          done, len(sample[0]), what, args.quality, min(threads, done), os.cpu_count() or 0,
                          threads, dt)}, {
        'sample_buffers': done, 'oracle_roundtrip_failures': len(bad), 'gpu': round(ratio_gpu, 5), 'oracle_ref_fixed': round(ratio_ref, 5),
        'gpu_vs_ref_fixed': round(ratio_gpu / ratio_ref, 4),
        'node_native_sample_buffers': nn if nat else 0,
        'node_native_brotli': round(nat['bytes'] / nn_bytes, 5) if nat else None,
        'gpu_vs_node_native': round(sum(gpu_sizes[:nn]) / nat['bytes'], 4) if nat else None,
        'node_native_MBps_1thread': round(nn_bytes / 1e6 / (nat['ns'] * 1e-9), 3) if nat else None}


def load_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` in `workload` from profiles/pmc_summary.json (the
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes, scripts/collect_pmc.py), or None."""
    p = os.path.join(ROOT, 'profiles', 'pmc_summary.json')
    try:
        with open(p) as f:
            d = json.load(f)
        k = d['workloads'][workload]['kernels'] if 'workloads' in d else d['kernels']
        return int(k[kernel]['hbm_bytes_per_launch'])
    except Exception:
        return None


def run_stream(args, rank, world, local):
    """C5 leg: one stream per GPU through the streaming encoder in 1 MiB host chunks with the
    C5 custom dictionary (PCIe inside: update() takes host bytes, the API the reference
    exposes), then brotliDecode of the whole stream with the dictionary; both timed."""
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)
    import brotli_amd
    from brotli_amd import datagen
    size = args.size if args.size > 0 else WORKLOADS['c5'][1]
    q = 9 if args.quality == 11 else args.quality
    lg = 24 if args.lgwin == 22 else args.lgwin
    data = datagen.c5_stream(size, 5000 + rank, dev)
    cdict = datagen.c5_dictionary()
    # throughput mode (streamChunk, brotli_amd.h): device encodes of >= 32 MiB growing with the
    # stream; --stream-chunk 0 measures the reference's cadence (every update() encodes its
    # complete blocks)
    opts = {'quality': q, 'lgwin': lg, 'mode': 1, 'customDictionary': cdict, 'streamChunk': args.stream_chunk * MIB}
    step = MIB

    view = memoryview(data)   # update() gets views of the stream, as Uint8Array.subarray gives

    def enc():
        e = brotli_amd.BrotliEncoder(opts)
        parts = [e.update(view[p:p + step]) for p in range(0, size, step)]
        parts.append(e.finish())
        return b''.join(parts)
    for _ in range(max(1, args.warmup)):
        stream = enc()
    if brotli_amd.brotliDecode(stream, {'customDictionary': cdict}) != data:
        raise SystemExit('c5 round trip FAILED')
    if world > 1:
        dist.barrier()
    # The encode loop runs without kernel events (a reference-cadence update() is one launch
    # sequence of ~2.8 ms, with ~25 event pairs in it); the decode loop times the
    # decoder (its kernel is the leg's dominant one: the roofline's launch time comes from the
    # timed region); one more, untimed, encode fills the encoder's kernel table.
    brotli_amd.default_profiling(False)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        stream = enc()
    t1 = time.perf_counter()
    brotli_amd.default_profiling('decode')
    for _ in range(args.steps):
        out = brotli_amd.brotliDecode(stream, {'customDictionary': cdict})
    t2 = time.perf_counter()
    times = brotli_amd.default_kernel_times()   # (the decoder's: the timed region)
    brotli_amd.default_profiling(True)
    enc()   # (untimed: the encoder's kernel table, one step)
    enc_times = brotli_amd.default_kernel_times()
    brotli_amd.default_profiling(False)
    assert out == data
    del out
    te, td = (t1 - t0) / args.steps, (t2 - t1) / args.steps
    dt = te + td
    if world > 1:
        t = torch.tensor([dt, te, td], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, te, td = (float(x) for x in t.tolist())
    if rank == 0:
        mb = world * size / 1e6
        # the dominant kernel: the longest launch of the timed region's (the decoder's: every
        # encoder launch covers one device chunk of the stream and is far shorter); decode
        # launches cover the whole stream
        dom_name, (dom_ms, dom_n) = max(times.items(), key=lambda kv: kv[1][0] / max(1, kv[1][1]))
        launches_per_step = max(1, dom_n // args.steps)
        launch_bytes = (size + len(stream)) // launches_per_step
        avg_ms = dom_ms / max(1, dom_n)
        achieved = launch_bytes / (avg_ms * 1e-3) / 1e9
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            # decode: the oracle (reference decoder restated) decodes the same stream with the
            # same dictionary on one host thread (it is one bit-serial stream).  encode: the
            # oracle's restatement of the reference's q9 path (hash chains + greedy,
            # backward-references.ts:14-134; pinned by tests/golden/encode_ref_q5_9.json) on the
            # stream's first 1 MiB pieces, one-shot at lgwin 22 (the reference's q5-9 path has
            # no custom dictionary and indexes its ring wrongly past 2^lgwin: bugs C/E), one
            # piece per host thread; value = 1 / (1 / encode + 1 / decode), as the GPU's
            from concurrent.futures import ThreadPoolExecutor
            sys.path.insert(0, os.path.join(ROOT, 'tests'))
            import _oracle
            _oracle.lib()
            c0 = time.perf_counter()
            got = _oracle.decode(stream, dictionary=cdict)
            ct = time.perf_counter() - c0
            ok = got == data
            del got
            threads = cpu_share()
            pieces = [bytes(view[k * MIB:(k + 1) * MIB]) for k in range(min(threads, size // MIB))]
            e0 = time.perf_counter()
            with ThreadPoolExecutor(threads) as ex:
                encs = list(ex.map(lambda b: _oracle.encode(b, q, 22, 1), pieces))
            et = time.perf_counter() - e0
            eok = all(_oracle.decode(x) == b for x, b in zip(encs, pieces))
            enc_mbps = len(pieces) * MIB / 1e6 / et
            dec_mbps = size / 1e6 / ct
            cpu = {'value': round(1.0 / (1.0 / enc_mbps + 1.0 / dec_mbps), 4), 'unit': 'MB/s', 'cores': threads,
                   'kind': 'port', 'encode_MBps': round(enc_mbps, 4), 'decode_MBps': round(dec_mbps, 3),
                   'compressed_ratio_sample': round(sum(map(len, encs)) / (len(pieces) * MIB), 5),
                   'sample': 'encode: %d x 1 MiB pieces of the stream, oracle q%d lgwin22 TEXT one-shot (the '
                             'reference\'s hash-chain path restated), one piece per host thread, %.1f s, round trip %s; '
                             'decode: the whole %d B C5 stream, oracle decoder with the dictionary, one host thread, '
                             '%.1f s, %s' % (len(pieces), q, et, 'ok' if eok else 'FAILED', size, ct,
                                             'bit-exact' if ok else 'MISMATCH')}
        print(json.dumps({
            'metric': 'encode+decode MB/s at q11 lgwin=22', 'value': round(mb / dt, 3), 'unit': 'MB/s',
            'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(dt * 1e3, 3),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u8', 'data': 'synthetic',
            'config': {'workload': 'C5 per GPU: one %d B enwik-style stream, BrotliEncoder.update() in 1 MiB host '
                                   'chunks, q%d lgwin%d TEXT, %d B custom dictionary, then brotliDecode of the stream '
                                   'with it (host buffers: PCIe included)' % (size, q, lg, len(cdict)),
                       'name': 'c5', 'bytes_per_stream': size, 'quality': q, 'lgwin': lg,
                       'stream_chunk_MiB': args.stream_chunk,
                       'custom_dictionary_bytes': len(cdict), 'parallelism': 'replicas%d' % world},
            'encode_MBps': round(mb / te, 3), 'decode_MBps': round(mb / td, 3),
            'compressed_ratio': round(len(stream) / size, 5),
            'kernel_ms_per_step': dict(sorted(list({n: round(v[0] / args.steps, 3) for n, v in times.items()}.items()) +
                                              list({n: round(v[0], 3) for n, v in enc_times.items()}.items()))),
            'kernel_times_from': 'decoder: the timed decode loop; encoder: one untimed encode step after it (the '
                                 'timed encode loop runs without kernel events)',
            'roofline': {'bound': 'hbm', 'kernel': dom_name, 'achieved': round(achieved, 3), 'peak': PEAK_HBM_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / PEAK_HBM_GBS, 6),
                         'traffic': load_traffic(dom_name, 'c5' if args.stream_chunk else 'c5cad'),
                         'algorithmic_bytes_per_launch': launch_bytes, 'avg_launch_ms': round(avg_ms, 3)},
            'cpu_baseline': cpu}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# The reference's encode bench inputs (bench/encode.bench.ts:5-16) and its published q11 encode
# times (README.md:88-94, "unstated, M2 Max implied"), plus C1's 45,000 B enwik-style slice.
LATENCY_INPUTS = [
    ('short 13 B', lambda: b'Hello, World!', 0.001),
    ('medium 4.5 KB', lambda: b'The quick brown fox jumps over the lazy dog. ' * 100, 0.27),
    ('long 45 KB', lambda: b'The quick brown fox jumps over the lazy dog. ' * 1000, 3.0),
    ('html 8 KB', lambda: b'<!DOCTYPE html><html><head><title>Test</title></head><body>' + b'<p>Content</p>' * 500
     + b'</body></html>', None),
    ('C1 enwik 45,000 B', None, None),
]


def run_latency(args):
    """latency leg: ONE brotliEncode (q11) and ONE brotliDecode per call through the drop-in
    host API (host buffers in and out: PCIe, launch and synchronisation included), median of
    `steps` x 20 calls per input, next to the reference's published single-call encode times;
    the oracle (the reference's q11 encoder restated) times the same calls on one host core."""
    import statistics
    import brotli_amd
    from brotli_amd import datagen
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    rows = []
    reps = max(1, args.steps) * 20
    for name, make, ref_ms in LATENCY_INPUTS:
        data = make() if make else datagen.enwik_text(45000, 1)
        for _ in range(max(1, args.warmup) * 3):
            enc = brotli_amd.brotliEncode(data, {'quality': 11})
            assert brotli_amd.brotliDecode(enc) == data
        te, td = [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            enc = brotli_amd.brotliEncode(data, {'quality': 11})
            t1 = time.perf_counter()
            out = brotli_amd.brotliDecode(enc)
            t2 = time.perf_counter()
            te.append(t1 - t0)
            td.append(t2 - t1)
        assert out == data
        row = {'input': name, 'bytes': len(data), 'compressed': len(enc),
               'encode_ms_median': round(statistics.median(te) * 1e3, 4),
               'decode_ms_median': round(statistics.median(td) * 1e3, 4),
               'ref_encode_ms_published': ref_ms}
        if not args.no_cpu_baseline:
            import _oracle
            t0 = time.perf_counter()
            n = 0
            while n < 5 or time.perf_counter() - t0 < 0.5:
                e = _oracle.encode(data, 11, 22)
                n += 1
            row['oracle_encode_ms'] = round((time.perf_counter() - t0) / n * 1e3, 4)
            row['oracle_compressed'] = len(e)
        rows.append(row)
    tot_b = sum(r['bytes'] for r in rows)
    tot_s = sum((r['encode_ms_median'] + r['decode_ms_median']) * 1e-3 for r in rows)
    cpu = None
    if not args.no_cpu_baseline:
        cpu = {'value': round(tot_b / 1e6 / sum(r['oracle_encode_ms'] * 1e-3 for r in rows), 4), 'unit': 'MB/s',
               'cores': 1, 'kind': 'port',
               'sample': 'the same inputs, one oracle q11 encode per call on one host thread (encode only)'}
    print(json.dumps({
        'metric': 'single-call brotliEncode + brotliDecode latency (host API)', 'value': round(tot_b / 1e6 / tot_s, 4),
        'unit': 'MB/s', 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(tot_s * 1e3, 4),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u8', 'data': 'reference bench inputs',
        'config': {'workload': 'one call per input: the reference encode bench inputs (bench/encode.bench.ts) and C1 '
                               '(45,000 B enwik-style), q11 lgwin 22, host buffers', 'name': 'latency',
                   'parallelism': 'replicas1'},
        'inputs': rows, 'roofline': None, 'cpu_baseline': cpu}), flush=True)


# The reference's own bench streams (tests/golden/bench, bench/fixtures of the reference) and
# its decode times: README.md:79-82 (Apple M2 Max, Node 22) and SURVEY.md §6 (the survey
# host: Xeon, Node 12, 1 thread).
REF_STREAMS = [('enc-ttf', 2.3, 5.6), ('enc-otf', 2.2, 4.2), ('enc-var-ttf', 5.8, 10.6), ('noto-tc', 47.0, 85.9),
               ('html-content', None, None), ('random-binary', None, None)]


def run_ref(args):
    """ref leg: decode each of the reference's bench streams ALONE (one stream per call, input
    and output in HBM: single-stream latency, the case the reference's README times), then all
    of them in one call; the oracle decodes the same streams on one host core."""
    import torch
    import brotli_amd
    sys.path.insert(0, os.path.join(ROOT, 'tests'))
    dev = torch.device('cuda', 0)
    ctx = brotli_amd.DeviceContext(0, profiling=True)
    gold = os.path.join(ROOT, 'tests', 'golden', 'bench')
    streams = []
    for name, m2, host in REF_STREAMS:
        with open(os.path.join(gold, name + '.br'), 'rb') as f:
            enc = f.read()
        n = brotli_amd.brotliDecodedSize(enc)
        if n <= 0:
            n = len(brotli_amd.brotliDecode(enc))
        streams.append((name, m2, host, enc, n))
    per = []
    tot_out, tot_s = 0, 0.0
    for name, m2, host, enc, n in streams:
        src = torch.tensor(list(enc), dtype=torch.uint8, device=dev)
        out = torch.empty(n + 4096, dtype=torch.uint8, device=dev)
        for _ in range(max(1, args.warmup)):
            sizes, st = ctx.decode(src.data_ptr(), [0, len(enc)], out.data_ptr(), [0, n + 4096])
        assert st == [0] and sizes == [n], (name, st, sizes)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        kern = 0.0
        for _ in range(args.steps):
            ctx.decode(src.data_ptr(), [0, len(enc)], out.data_ptr(), [0, n + 4096])
            kern += sum(ms for nm, (ms, c) in ctx.kernel_times().items() if nm.startswith('decode'))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        tot_out += n
        tot_s += dt
        per.append({'stream': name, 'out_bytes': n, 'in_bytes': len(enc), 'ms': round(dt * 1e3, 3),
                    'kernel_ms': round(kern / args.steps, 3), 'MBps': round(n / dt / 1e6, 2),
                    'ref_ms_m2max': m2, 'ref_ms_survey_host': host})
    # all streams in one call (one wave each)
    cat = b''.join(s[3] for s in streams)
    ioff, ooff = [0], [0]
    for s_ in streams:
        ioff.append(ioff[-1] + len(s_[3]))
        ooff.append(ooff[-1] + s_[4] + 4096)
    src = torch.tensor(list(cat), dtype=torch.uint8, device=dev)
    out = torch.empty(ooff[-1], dtype=torch.uint8, device=dev)
    ctx.decode(src.data_ptr(), ioff, out.data_ptr(), ooff)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.decode(src.data_ptr(), ioff, out.data_ptr(), ooff)
    torch.cuda.synchronize()
    batch_ms = (time.perf_counter() - t0) / args.steps * 1e3
    cpu = None
    if not args.no_cpu_baseline:
        import _oracle
        t0 = time.perf_counter()
        for s_ in streams:
            assert isinstance(_oracle.decode(s_[3]), bytes)
        ct = time.perf_counter() - t0
        cpu = {'value': round(tot_out / ct / 1e6, 3), 'unit': 'MB/s', 'cores': 1, 'kind': 'port',
               'sample': 'the same %d streams, oracle decoder (reference decoder restated), one host thread, %.2f s'
                         % (len(streams), ct)}
    print(json.dumps({
        'metric': 'decode MB/s of the reference bench streams (single stream per call)', 'value': round(tot_out / tot_s / 1e6, 3),
        'unit': 'MB/s', 'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(tot_s * 1e3, 3),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u8', 'data': 'reference fixtures',
        'config': {'workload': 'decode of the reference bench streams (tests/golden/bench/*.br), one stream per call, '
                               'input/output in HBM', 'name': 'ref', 'parallelism': 'replicas1'},
        'streams': per, 'all_streams_one_call_ms': round(batch_ms, 3), 'roofline': None, 'cpu_baseline': cpu}),
          flush=True)


def run_in_lib(args):
    """in-library sharding leg: the workload's batch as host buffers through
    the C ABI's sharded batch calls (mib_encode_batch_n / mib_decode_batch_n: a context per
    shard, pinned one-copy staging, shard s on device s % ndev) against the one-context batch
    (mib_encode_batch / mib_decode_batch) on the same buffers.  On one GPU all N shards share
    device 0, so this times the sharding machinery's overhead, not multi-GPU scaling."""
    import brotli_amd
    import torch
    wl = args.workload
    k0, size0, mode, _, gen = WORKLOADS[wl]
    k = args.streams if args.streams > 0 else k0
    size = args.size if args.size > 0 else size0
    dev = torch.device('cuda', 0)
    data = make_inputs(wl, k, size, 0, dev).cpu().numpy().tobytes()
    bufs = [data[i * size:(i + 1) * size] for i in range(k)]
    del data
    opts = {'quality': args.quality, 'lgwin': args.lgwin, 'mode': mode}
    n = args.gpus_in_lib

    def leg(gpus):
        comp = brotli_amd.encode_batch(bufs, opts, gpus=gpus)
        out = brotli_amd.decode_batch(comp, gpus=gpus)
        return comp, out

    ref_comp = None
    for g in (None, n):
        for _ in range(max(1, args.warmup)):
            comp, out = leg(g)
            if out != bufs:
                raise SystemExit('in-library leg: round trip FAILED (gpus=%s)' % g)
            if ref_comp is None:
                ref_comp = comp
            elif comp != ref_comp:
                raise SystemExit('in-library leg: sharded streams differ from the one-context batch')
    res = {}
    del comp, out
    for g in (None, n):
        te = td = 0.0
        for _ in range(args.steps):
            t0 = time.perf_counter()
            comp = brotli_amd.encode_batch(bufs, opts, gpus=g)
            t1 = time.perf_counter()
            out = brotli_amd.decode_batch(comp, gpus=g)
            t2 = time.perf_counter()
            te += t1 - t0
            td += t2 - t1
            # (the caller's results are freed outside the timed calls: releasing 1,024 x 1 MiB
            # bytes objects took Python 57-108 ms on the MI355X box, scripts/host_xfer_probe.py)
            del comp, out
        res['one_context' if g is None else 'shards'] = {'encode_ms': round(te * 1e3 / args.steps, 3),
                                                         'decode_ms': round(td * 1e3 / args.steps, 3)}
    one = res['one_context']['encode_ms'] + res['one_context']['decode_ms']
    sh = res['shards']['encode_ms'] + res['shards']['decode_ms']
    total = k * size
    print(json.dumps({
        'metric': 'encode+decode MB/s at q11 lgwin=22, host buffers through the sharded C-ABI batch calls',
        'value': round(total / 1e6 / (sh * 1e-3), 3), 'unit': 'MB/s', 'n_gpus': 1, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(sh, 3), 'higher_is_better': True, 'scaling': 'weak',
        'vs_baseline': None, 'dtype': 'u8', 'data': 'synthetic',
        'config': {'workload': '%s batch (%d x %d B) as host buffers: mib_encode_batch_n + mib_decode_batch_n with %d '
                               'shards on device 0 vs mib_encode_batch + mib_decode_batch (PCIe included)'
                               % (wl, k, size, n), 'name': 'in_lib', 'shards': n, 'parallelism': 'shards%d_on_1gpu' % n},
        'legs': res, 'shard_overhead': round(sh / one - 1.0, 4), 'roofline': None, 'cpu_baseline': None}), flush=True)


def datagen_device(total, seed, dev):
    from brotli_amd import datagen
    return datagen.enwik_device(total, seed, dev)


def main():
    args = parse()
    wl = args.workload
    if wl == 'ref':
        return run_ref(args)
    if wl == 'latency':
        return run_latency(args)
    if args.gpus_in_lib > 0:
        return run_in_lib(args)
    if wl == 'c5':
        return run_stream(args, int(os.environ.get('RANK', '0')), int(os.environ.get('WORLD_SIZE', '1')),
                          int(os.environ.get('LOCAL_RANK', '0')))
    k0, size0, mode, _, gen = WORKLOADS[wl]
    k = args.streams if args.streams > 0 else k0
    size = args.size if args.size > 0 else size0
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1:
        dist.init_process_group('nccl', device_id=dev)
    import brotli_amd
    from brotli_amd import shard

    total = k * size
    data = make_inputs(wl, k, size, rank, dev)
    in_off = [i * size for i in range(k + 1)]
    cap = total + total // 8 + 4096 * k
    comp = torch.empty(cap, dtype=torch.uint8, device=dev)
    slot = size + 4096   # decoded output slots (+ the decoder's slack)
    dec = torch.empty(k * slot, dtype=torch.uint8, device=dev)
    dec_off = [i * slot for i in range(k + 1)]
    ctx = brotli_amd.DeviceContext(local, profiling=True)
    opts = {'quality': args.quality, 'lgwin': args.lgwin, 'mode': mode}
    gather = world > 1 and k > 1 and not args.no_gather

    def step(times):
        t0 = time.perf_counter()
        out_off = ctx.encode(data.data_ptr(), in_off, comp.data_ptr(), cap, opts)
        wall = times.setdefault(' encode_wall', [0.0, 0])
        wall[0] += (time.perf_counter() - t0) * 1e3
        wall[1] += 1
        for name, (ms, n) in ctx.kernel_times().items():
            t = times.setdefault(name, [0.0, 0])
            t[0] += ms
            t[1] += n
        if gather:
            # the one collective: RCCL gather of the variable-length compressed shards to rank 0
            lens = [out_off[i + 1] - out_off[i] for i in range(k)]
            shard.gather_shards(comp[:out_off[-1]], lens, dst=0)
        t0 = time.perf_counter()
        sizes, status = ctx.decode(comp.data_ptr(), out_off, dec.data_ptr(), dec_off)
        wall = times.setdefault(' decode_wall', [0.0, 0])
        wall[0] += (time.perf_counter() - t0) * 1e3
        wall[1] += 1
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
    gpu_sizes = [out_off[i + 1] - out_off[i] for i in range(k)]

    times = {}
    if args.kernel_events is None:
        args.kernel_events = 'all' if wl == 'c3' else 'decode'
    if args.kernel_events == 'decode':
        ctx.set_profiling('decode')
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
    timed = set(times)   # (the kernels the timed steps' events measured: the roofline's candidates)
    if args.kernel_events == 'decode':   # the encoder's kernel table: one untimed step, scaled
        ctx.set_profiling(True)
        extra = {}
        step(extra)
        torch.cuda.synchronize()
        for n, (ms, c) in extra.items():
            if n not in times:
                times[n] = [ms * args.steps, c * args.steps]
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        cb = torch.tensor([comp_bytes], dtype=torch.int64, device=dev)
        dist.all_reduce(cb)
        comp_all = int(cb.item())
    else:
        comp_all = comp_bytes

    cpu, ratios = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the CPU sample: the first buffers of the same batch (C2: 1 MiB slices of its one buffer)
        piece = min(size, MIB)
        nsamp = min(max(1, total // piece), 16 * cpu_share())
        host = data[:nsamp * piece].cpu().numpy().tobytes()
        sample = [host[i * piece:(i + 1) * piece] for i in range(nsamp)]
        if piece == size:
            samp_gpu = gpu_sizes[:nsamp]
        else:   # GPU sizes of the slices: encode them alone on the device
            s_in = torch.frombuffer(bytearray(host), dtype=torch.uint8).to(dev)
            s_cap = nsamp * (piece + piece // 8 + 4096)
            s_out = torch.empty(s_cap, dtype=torch.uint8, device=dev)
            s_off = ctx.encode(s_in.data_ptr(), [i * piece for i in range(nsamp + 1)], s_out.data_ptr(), s_cap, opts)
            samp_gpu = [s_off[i + 1] - s_off[i] for i in range(nsamp)]
        what = {'enwik': 'enwik-style text', 'glyf': 'WOFF2-transformed glyf tables'}[gen]
        cpu, ratios = cpu_baseline(sample, samp_gpu, args, mode, what)

    if rank == 0:
        ms_step = dt * 1e3 / args.steps
        mb = world * total / 1e6
        # encode / decode rates from each call's wall time (the encode's two lanes overlap
        # their kernels, so kernel times no longer add up to it); kernel times below
        walls = {n: times.pop(n) for n in list(times) if n.startswith(' ')}
        enc_ms = walls[' encode_wall'][0] / args.steps
        dec_ms = walls[' decode_wall'][0] / args.steps
        # the dominant kernel: the longest launch (the encode lanes' kernels run concurrently,
        # so their summed time is not time on the chip's clock)
        dom_name, (dom_ms, dom_n) = max(((n, v) for n, v in times.items() if n in timed),
                                        key=lambda kv: kv[1][0] / max(1, kv[1][1]))
        # a kernel launched L times per step covers 1/L of the batch per launch
        launches_per_step = max(1, dom_n // args.steps)
        launch_bytes = (total + comp_bytes) // launches_per_step
        avg_ms = dom_ms / max(1, dom_n)
        achieved = launch_bytes / (avg_ms * 1e-3) / 1e9
        desc = {'c4': 'C4 per-GPU shard: %d x %d B enwik-style text, q%d lgwin%d GENERIC',
                'c3': 'C3: %d x %d B WOFF2-transformed glyf tables (glyph sets from the reference\'s Inter font, jittered per seed), q%d lgwin%d FONT',
                'c2': 'C2: %d x %d B enwik-style text (one stream), q%d lgwin%d GENERIC'}[wl] % (
                    k, size, args.quality, args.lgwin)
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
            'config': {'workload': desc + ', encode -> %sdecode round trip (bit-exact checked)' % (
                           'RCCL gather -> ' if gather else ''),
                       'name': wl, 'streams_per_gpu': k, 'bytes_per_stream': size, 'quality': args.quality,
                       'lgwin': args.lgwin, 'mode': mode,
                       'parallelism': ('shard%d' % world) if k > 1 else ('replicas%d' % world)},
            'encode_MBps': round(mb / (enc_ms * 1e-3), 3) if enc_ms else None,
            'decode_MBps': round(mb / (dec_ms * 1e-3), 3) if dec_ms else None,
            'compressed_ratio': round(comp_all / (world * total), 5),
            'ratio_same_sample': ratios,
            'kernel_ms_per_step': {n: round(v[0] / args.steps, 3) for n, v in sorted(times.items())},
            'kernel_events': args.kernel_events,
            'roofline': {'bound': 'hbm', 'kernel': dom_name, 'achieved': round(achieved, 3), 'peak': PEAK_HBM_GBS,
                         'unit': 'GB/s', 'frac': round(achieved / PEAK_HBM_GBS, 6),
                         'traffic': load_traffic(dom_name, wl),
                         'algorithmic_bytes_per_launch': launch_bytes, 'avg_launch_ms': round(avg_ms, 3)},
            'cpu_baseline': cpu,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
