#!/usr/bin/env python3
"""Static instruction counts of one device function, by basic block and by source section.

Input: device assembly with line tables, e.g.
  hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -gline-tables-only -x hip \
        --cuda-device-only -S brotli-lib_amd/csrc/decode.hip -o /tmp/decg.s
Usage:
  isa_sections.py ASM FUNC_SYMBOL [--sections name:lo-hi,...] [--blocks] [--listing OUT]

Each instruction is classed as rocprof's SQ_INSTS_* counters class them (SALU = scalar ALU
and scalar compares, SMEM = scalar loads, VALU = v_* including v_readlane / v_readfirstlane,
LDS = ds_*, VMEM = global_/buffer_/flat_, BRANCH = s_branch / s_cbranch_*, WAIT = s_waitcnt and
other SOPP that no ALU counter sees).  A block's source section is the section holding the
most of its instructions' decode.hip lines (.loc of file 0); lines of inlined helpers (the
reader lambdas) are outside every section and take their block's other lines' section, or the
section of the block before when a block has no other line.
"""
import re
import sys
from collections import Counter, OrderedDict


def cls(m):
    if m.startswith('s_waitcnt') or m in ('s_nop', 's_setprio', 's_sleep', 's_endpgm', 's_barrier'):
        return 'WAIT'
    if m.startswith('s_cbranch') or m == 's_branch' or m.startswith('s_setpc') or m.startswith('s_swappc'):
        return 'BRANCH'
    if m.startswith('s_load') or m.startswith('s_buffer_load') or m.startswith('s_dcache'):
        return 'SMEM'
    if m.startswith('s_'):
        return 'SALU'
    if m.startswith('v_'):
        return 'VALU'
    if m.startswith('ds_'):
        return 'LDS'
    if m.startswith(('global_', 'buffer_', 'flat_', 'scratch_')):
        return 'VMEM'
    return 'OTHER'


def parse(path, func):
    blocks = OrderedDict()
    cur = None
    line = None
    inside = False
    raw = []
    with open(path) as f:
        for ln in f:
            s = ln.rstrip('\n')
            if not inside:
                if s.startswith(func + ':'):
                    inside = True
                    cur = func
                    blocks[cur] = {'ins': [], 'lines': Counter(), 'succ': []}
                continue
            if s.startswith('.Lfunc_end'):
                break
            m = re.match(r'^(\.LBB\d+_\d+):', s)
            if m:
                cur = m.group(1)
                blocks[cur] = {'ins': [], 'lines': Counter(), 'succ': []}
                raw.append(s)
                continue
            m = re.match(r'^\s*\.loc\s+(\d+)\s+(\d+)', s)
            if m:
                line = int(m.group(2)) if m.group(1) == '0' else None
                continue
            st = s.strip()
            if not st or st.startswith(('.', ';')):
                continue
            mn = st.split()[0]
            b = blocks[cur]
            b['ins'].append((mn, line, st))
            if line is not None:
                b['lines'][line] += 1
            t = re.search(r'(\.LBB\d+_\d+)', st)
            if t and cls(mn) == 'BRANCH':
                b['succ'].append(t.group(1))
            raw.append('%-6s %5s  %s' % (cls(mn), line if line is not None else '', st))
    return blocks, raw


def main():
    a = sys.argv[1:]
    if len(a) < 2:
        print(__doc__)
        sys.exit(2)
    path, func = a[0], a[1]
    secs = []
    show_blocks = '--blocks' in a
    listing = None
    if '--sections' in a:
        for it in a[a.index('--sections') + 1].split(','):
            nm, rg = it.split(':')
            lo, hi = rg.split('-')
            secs.append((nm, int(lo), int(hi)))
    if '--listing' in a:
        listing = a[a.index('--listing') + 1]
    blocks, raw = parse(path, func)
    order = list(blocks)
    pos = {k: i for i, k in enumerate(order)}
    prev = 'entry'
    tot = Counter()
    bysec = OrderedDict()
    for k in order:
        b = blocks[k]
        votes = Counter()
        for l, n in b['lines'].items():
            for nm, lo, hi in secs:
                if lo <= l <= hi:
                    votes[nm] += n
        sec = votes.most_common(1)[0][0] if votes else prev
        prev = sec
        c = Counter(cls(mn) for mn, _, _ in b['ins'])
        tot.update(c)
        bysec.setdefault(sec, Counter()).update(c)
        b['sec'] = sec
        b['cls'] = c
        if show_blocks:
            back = [t for t in b['succ'] if t in pos and pos[t] <= pos[k]]
            ls = sorted(b['lines'])
            print('%-14s %-10s n=%3d SALU=%3d VALU=%3d LDS=%2d VMEM=%2d SMEM=%2d BR=%2d WAIT=%2d lines=%s%s' % (
                k, sec, len(b['ins']), c['SALU'], c['VALU'], c['LDS'], c['VMEM'], c['SMEM'], c['BRANCH'], c['WAIT'],
                ('%d-%d' % (ls[0], ls[-1])) if ls else '-', ('  back->' + ','.join(back)) if back else ''))
    print('section totals (static):')
    for sec, c in bysec.items():
        print('  %-10s n=%4d SALU=%4d VALU=%4d LDS=%3d VMEM=%3d SMEM=%3d BR=%3d WAIT=%3d' % (
            sec, sum(c.values()), c['SALU'], c['VALU'], c['LDS'], c['VMEM'], c['SMEM'], c['BRANCH'], c['WAIT']))
    print('  %-10s n=%4d' % ('all', sum(tot.values())))
    if listing:
        with open(listing, 'w') as f:
            f.write('\n'.join(raw) + '\n')


if __name__ == '__main__':
    main()
