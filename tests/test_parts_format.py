"""The part index format on the CPU (no GPU): a stream the GPU encoder wrote with a part index
(tests/golden/parts/parts_enwik300k.br, made by make_fixture.py) decodes with the oracle to its
input, and every index entry equals the reference decoder's own state at that point."""
import os

import numpy as np

import _inputs
import _oracle
import _parts
from brotli_amd import datagen

FIX = os.path.join(_inputs.GOLDEN, 'parts', 'parts_enwik300k.br')


def test_fixture_index_matches_oracle_states():
    with open(FIX, 'rb') as f:
        enc = f.read()
    data = datagen.enwik_text(300000, 21)
    assert _oracle.decode(enc) == data
    ents, total = _parts.read_chain(enc)
    assert total == len(data) and len(ents) >= 4
    got = _oracle.probe(enc, ents['pos'])
    assert np.all(got['flags'] & 1)
    for f in ('bit', 'pos', 'mb_bit', 'mb_pos', 'ring', 'p1', 'p2'):
        assert np.array_equal(got[f], ents[f]), f
    mid = (ents['flags'] & _parts.AT_MB) == 0
    for f in ('blen', 'type', 'prev'):
        assert np.array_equal(got[f][mid], ents[f][mid]), f


def test_fixture_is_plain_brotli_after_the_index():
    # the index is one metadata metablock right after the window bits: dropping its payload's
    # meaning changes nothing -- a zeroed payload still decodes to the same bytes
    with open(FIX, 'rb') as f:
        enc = bytearray(f.read())
    r = _parts._Bits(enc, 0)
    assert r.get(1) == 1 and r.get(3) == 5   # lgwin 22: window bits 1 + 101
    assert r.get(1) == 0 and r.get(2) == 3 and r.get(1) == 0
    nb = r.get(2)
    length = r.get(8 * nb) + 1
    pay = (r.bit + 7) >> 3
    enc[pay:pay + length] = bytes(length)
    assert _oracle.decode(bytes(enc)) == datagen.enwik_text(300000, 21)
