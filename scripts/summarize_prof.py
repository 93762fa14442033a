"""Turn a gpurun_out/prof_<tag> rocprofv3 run (scripts/gpu_profile.sh) into the committed
evidence: profiles/<tag>_kernel_stats.csv and profiles/pmc_summary.json.

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 / launches: FETCH_SIZE and
WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts 1/2 of the bytes of wide
streaming reads (MI355X_MICROARCH.md, HBM section), so it is doubled.  The correction is
exact only for 16 B/lane streaming reads; byte-granular gathers are uncalibrated."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def short(name):
    n = name.split('(')[0]
    n = n.replace('void ', '').strip()
    for pre in ('mib::enc::', 'mib::'):
        if n.startswith(pre):
            n = n[len(pre):]
    return n


def main(tag):
    base = os.path.join(ROOT, 'gpurun_out', 'prof_' + tag)
    stats = glob.glob(os.path.join(base, 'trace', '**', '*kernel_stats.csv'), recursive=True)
    os.makedirs(os.path.join(ROOT, 'profiles'), exist_ok=True)
    if stats:
        shutil.copy(stats[0], os.path.join(ROOT, 'profiles', '%s_kernel_stats.csv' % tag))
    per = {}
    for kind in ('fetch', 'write'):
        for r in rows(os.path.join(base, kind, '**', '*counter_collection.csv')):
            k = short(r.get('Kernel_Name', ''))
            d = per.setdefault(k, {'FETCH_SIZE': 0.0, 'WRITE_SIZE': 0.0, 'dispatches': set()})
            d[r['Counter_Name']] = d.get(r['Counter_Name'], 0.0) + float(r['Counter_Value'])
            d['dispatches'].add((kind, r.get('Dispatch_Id')))
    kernels = {}
    for k, d in per.items():
        n = max(1, len([x for x in d['dispatches'] if x[0] == 'fetch']))
        fetch = d['FETCH_SIZE'] * 1024 / n
        write = d['WRITE_SIZE'] * 1024 / n
        kernels[k] = {'launches_per_pass': n, 'fetch_bytes_raw': fetch, 'write_bytes': write,
                      'hbm_bytes_per_launch': int(2 * fetch + write)}
    # bench.py names kernels by its event labels; map the HIP symbol names onto them
    alias = {'decode_streams_kernel': 'decode_streams_kernel', 'find_matches_kernel': 'find_matches',
             'dp_kernel': 'dp_parse', 'emit_kernel': 'emit', 'assemble_kernel': 'assemble'}
    for src, dst in alias.items():   # templated kernels: the first instantiation with the base name
        hit = [k for k in sorted(kernels) if k == src or k.startswith(src + '<') and 'true' in k]
        hit = hit or [k for k in sorted(kernels) if k.startswith(src + '<')]
        if hit:
            kernels[dst] = kernels[hit[0]]
    with open(os.path.join(ROOT, 'profiles', 'pmc_summary.json'), 'w') as f:
        json.dump({'tag': tag, 'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of '
                   'bench.py --steps 1 --warmup 1 (scripts/gpu_profile.sh)',
                   'correction': 'hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B); gfx950 FETCH_SIZE halves wide reads',
                   'kernels': kernels}, f, indent=1, sort_keys=True)
    print(json.dumps(kernels, indent=1)[:3000])


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'r01')
