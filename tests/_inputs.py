"""Resolve the input specs used by the golden fixtures (tests/golden/*.json).

A spec is a small dict; the bytes are reproduced from committed data files
(tests/golden/vectors = the reference's canonical corpus, tests/golden/bench = its bench
fixtures) or from the deterministic generators in brotli_amd.datagen, so no golden input
has to be stored twice and nothing here reads /root/reference.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'brotli-lib_amd', 'python'))
from brotli_amd import datagen  # noqa: E402

GOLDEN = os.path.join(HERE, 'golden')


def resolve(spec):
    k = spec['kind']
    if k == 'file':
        with open(os.path.join(GOLDEN, spec['path']), 'rb') as f:
            data = f.read()
        off = spec.get('off', 0)
        ln = spec.get('len', len(data) - off)
        return data[off:off + ln]
    if k == 'xorshift':
        nxt = datagen.xorshift32(spec['seed'])
        for _ in range(spec.get('skip', 0)):
            nxt()
        return datagen.random_bytes(spec['len'], nxt)
    if k == 'ramp':
        return datagen.ramp(spec['len'])
    if k == 'fox':
        return datagen.fox(spec['repeats'])
    if k == 'enwik':
        return datagen.enwik_text(spec['len'], spec['seed'])
    if k == 'glyf':
        return datagen.glyf_stream(spec['len'], spec['seed'])
    if k == 'text':
        return spec['s'].encode('utf-8')
    if k == 'repeat':
        return bytes([spec['byte']]) * spec['len']
    raise ValueError(spec)
