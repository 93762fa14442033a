#!/usr/bin/env python3
"""Encode-phase timeline of a bench step from a rocprofv3 kernel trace (run_kernel_trace.csv).

The window is the last step's encode: from the first encoder kernel after the second-to-last
decode_streams_kernel (or decode_parts_kernel) to the start of the last one.  Prints the window, the time any kernel
runs (union), per stream busy time, and the largest idle gaps with the kernels around them.
usage: timeline.py run_kernel_trace.csv [ngaps=12]"""
import csv
import sys


def main():
    path = sys.argv[1]
    ngaps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'].split('(')[0].replace('void ', ''),
                     r.get('Stream_Id', r.get('Queue_Id'))))
    rows.sort()
    dec = [x for x in rows if 'decode_streams_kernel' in x[2] or 'decode_parts_kernel' in x[2]]
    if len(dec) < 2:
        print('need two decode launches')
        return
    lo, hi = dec[-2][1], dec[-1][0]
    enc = [x for x in rows if x[0] >= lo and x[1] <= hi and 'mib::enc' in x[2]]
    if enc:   # (from the first encoder kernel: the bench's checks of the step before are not encode)
        lo = enc[0][0]
    win = [x for x in rows if x[0] >= lo and x[1] <= hi]
    wall = hi - lo
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    last_end, last_name = lo, 'window start'
    for s, e, n, q in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            gap = s - (cur_e if cur_e is not None else lo)
            if gap > 0:
                gaps.append((gap, cur_e if cur_e is not None else lo, last_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        last_name = n if e >= (cur_e or 0) else last_name
    if cur_e is not None:
        busy += cur_e - cur_s
        if hi > cur_e:
            gaps.append((hi - cur_e, cur_e, last_name, 'window end'))
    per = {}
    for s, e, n, q in win:
        per[q] = per.get(q, 0) + (e - s)
    print('encode window %.3f ms, kernels %d, any-kernel busy %.3f ms (%.1f %%), idle %.3f ms' % (
        wall / 1e6, len(win), busy / 1e6, 100.0 * busy / wall, (wall - busy) / 1e6))
    for q, v in sorted(per.items()):
        print('  stream %s: kernel time %.3f ms' % (q, v / 1e6))
    print('largest idle gaps (nothing running):')
    for g, at, a, b in sorted(gaps, reverse=True)[:ngaps]:
        print('  %8.3f ms at +%.3f ms  after %s  before %s' % (g / 1e6, (at - lo) / 1e6, a[:60], b[:60]))


if __name__ == '__main__':
    main()
