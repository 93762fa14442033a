"""Turn a gpurun_out/prof_<tag> run (scripts/gpu_profile_all.sh) into committed evidence:
profiles/<tag>/<workload>_kernel_stats.csv, profiles/pmc_summary.json (HBM bytes per launch
per workload and kernel) and profiles/<tag>/sq_counters.json.

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 / launches: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE tallies each 128 B memory-side read request
(TCC_EA0_RDREQ) at 64 B, hence the doubling.  Calibrated per access width in round 5
(scripts/probe/traffic_probe.hip, profiles/r05/traffic_calibration.json): 1, 4, 16 and 32-byte
gathers and 1-byte LDS-DMA loads each make exactly one 128 B request per missed line, so the
doubled figure is the line traffic for the gather-bound kernels too (a 36 B access across a
128 B boundary is two requests).  Requests served by the Infinity Cache are counted as well.  SQ counters are in the SQ's units (cycle counters
in quad-cycles), summed over a kernel's dispatches and divided by their number."""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(pattern):
    out = []
    for p in glob.glob(pattern, recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def short(name):
    n = name.split('(')[0].replace('void ', '').strip()
    for pre in ('mib::enc::', 'mib::'):
        if n.startswith(pre):
            n = n[len(pre):]
    return n


# bench.py names kernels by its HIP-event labels: map symbol prefixes onto them
ALIAS = {'decode_streams_kernel': 'decode_streams_kernel', 'decode_parts_kernel': 'decode_parts_kernel',
         'find_matches_kernel': 'find_matches', 'emit_kernel': 'emit', 'huffman_kernel': 'huffman',
         'cluster_kernel': 'cluster', 'backtrack_kernel': 'backtrack'}


def main(tag):
    base = os.path.join(ROOT, 'gpurun_out', 'prof_' + tag)
    dst = os.path.join(ROOT, 'profiles', tag)
    os.makedirs(dst, exist_ok=True)
    summary = {'tag': tag, 'source': 'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of bench.py --steps 1 '
                                      '--warmup 1 --workload <w> (scripts/gpu_profile_all.sh)',
               'correction': 'hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB -> B); gfx950 FETCH_SIZE tallies each 128 B read request at 64 B, '
                             'for every access width (profiles/r05/traffic_calibration.json)',
               'workloads': {}}
    for tr in sorted(glob.glob(os.path.join(base, 'trace_*'))):
        if not os.path.isdir(tr):
            continue
        w = os.path.basename(tr)[len('trace_'):]
        st = glob.glob(os.path.join(tr, '**', '*kernel_stats.csv'), recursive=True)
        if st:
            shutil.copy(st[0], os.path.join(dst, '%s_kernel_stats.csv' % w))
        per = defaultdict(lambda: {'FETCH_SIZE': 0.0, 'WRITE_SIZE': 0.0, 'disp': set()})
        for kind in ('fetch', 'write'):
            for r in rows(os.path.join(base, '%s_%s' % (kind, w), '**', '*counter_collection.csv')):
                d = per[short(r.get('Kernel_Name', ''))]
                d[r['Counter_Name']] += float(r['Counter_Value'])
                d['disp'].add((kind, r.get('Dispatch_Id')))
        kernels = {}
        for k, d in per.items():
            n = max(1, len([x for x in d['disp'] if x[0] == 'fetch']))
            fetch, write = d['FETCH_SIZE'] * 1024 / n, d['WRITE_SIZE'] * 1024 / n
            kernels[k] = {'launches_per_pass': n, 'fetch_bytes_raw': round(fetch), 'write_bytes': round(write),
                          'hbm_bytes_per_launch': int(2 * fetch + write)}
        for src, name in ALIAS.items():
            hit = sorted(k for k in kernels if k == src or k.startswith(src + '<'))
            if hit:   # templated kernels: the instantiation with the most traffic
                kernels[name] = max((kernels[h] for h in hit), key=lambda v: v['hbm_bytes_per_launch'])
        dp = sorted(k for k in kernels if k.startswith('dp_kernel<'))
        if dp:   # the second (model) iteration is the bench's dp_parse
            model = [k for k in dp if ', true' in k] or dp
            kernels['dp_parse'] = max((kernels[h] for h in model), key=lambda v: v['hbm_bytes_per_launch'])
        summary['workloads'][w] = {'kernels': kernels}
    with open(os.path.join(ROOT, 'profiles', 'pmc_summary.json'), 'w') as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    sq = {}
    for d in sorted(glob.glob(os.path.join(base, 'sq[12]_*')) + glob.glob(os.path.join(base, 'sqref[12]_*'))):
        if not os.path.isdir(d):
            continue
        b = os.path.basename(d)
        k = b[4:] if b.startswith('sq1_') or b.startswith('sq2_') else b[7:] + ' (ref leg: one foreign stream per call)'
        acc = defaultdict(float)
        disp = set()
        for r in rows(os.path.join(d, '**', '*counter_collection.csv')):
            acc[r['Counter_Name']] += float(r['Counter_Value'])
            disp.add(r.get('Dispatch_Id'))
        e = sq.setdefault(k, {'dispatches': 0})
        e['dispatches'] = max(e['dispatches'], len(disp))
        for c, v in acc.items():
            e[c] = round(v / max(1, len(disp)))
    for k, e in sq.items():
        if e.get('SQ_WAVE_CYCLES'):
            e['wait_any_share'] = round(e.get('SQ_WAIT_ANY', 0) / e['SQ_WAVE_CYCLES'], 3)
            e['active_inst_share'] = round(e.get('SQ_ACTIVE_INST_ANY', 0) / e['SQ_WAVE_CYCLES'], 3)
    with open(os.path.join(dst, 'sq_counters.json'), 'w') as f:
        json.dump({'source': 'rocprofv3 --pmc (two passes of 8 SQ counters) on bench.py c4 (and --workload ref where named), --kernel-include-regex',
                   'units': 'SQ units (cycle counters in quad-cycles), per dispatch', 'kernels': sq}, f, indent=1,
                  sort_keys=True)
    for w, v in summary['workloads'].items():
        top = sorted(v['kernels'].items(), key=lambda kv: -kv[1]['hbm_bytes_per_launch'])[:6]
        print(w, [(k, round(x['hbm_bytes_per_launch'] / 1e9, 2)) for k, x in top])
    print(json.dumps(sq, indent=1)[:3000])


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'r03')
