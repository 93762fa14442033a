"""The oracle (CPU restatement of the reference) checked against the reference's own
golden data: canonical vectors, bench streams, ref-fixed encoder outputs and the error
corpus produced by running the reference itself (oracle/refgen/make_goldens.py)."""
import base64
import hashlib
import json
import os

import pytest

import _inputs
import _oracle

G = _inputs.GOLDEN


def _load(name):
    with open(os.path.join(G, name)) as f:
        return json.load(f)['cases']


def test_canonical_vectors_bit_exact():
    """test/brotli.test.ts:88-101 runs the 22 *.compressed; we also run the 23 *.compressed.NN."""
    n = 0
    for nm in sorted(os.listdir(os.path.join(G, 'vectors'))):
        if '.compressed' not in nm:
            continue
        base = nm.split('.compressed')[0]
        with open(os.path.join(G, 'vectors', nm), 'rb') as f:
            comp = f.read()
        with open(os.path.join(G, 'vectors', base), 'rb') as f:
            exp = f.read()
        assert _oracle.decode(comp) == exp, nm
        n += 1
    assert n == 45


def test_decode_vectors_match_reference_hashes():
    for c in _load('decode_vectors.json'):
        with open(os.path.join(G, c['path']), 'rb') as f:
            out = _oracle.decode(f.read())
        assert not isinstance(out, int), c['path']
        assert hashlib.sha256(out).hexdigest() == c['sha256'], c['path']


def test_decode_error_corpus_matches_reference():
    """Corrupted / truncated / random streams: same output hash or same 'Brotli error code: N'."""
    n = 0
    for c in _load('decode_errors.json'):
        if c.get('hang'):
            continue   # the reference never returns on this one; covered separately
        out = _oracle.decode(base64.b64decode(c['in_b64']))
        if 'error' in c:
            assert isinstance(out, int) and c['error'] == 'Brotli error code: %d' % out, c
        else:
            assert not isinstance(out, int) and hashlib.sha256(out).hexdigest() == c['sha256']
        n += 1
    assert n > 600


@pytest.mark.parametrize('chunk', [0, 1])
def test_encode_matches_ref_fixed(chunk):
    """brotliEncode byte-identical to the A+B-fixed reference (q0 / q10 / q11, FONT, lgwin 10..24)."""
    cases = _load('encode_ref_fixed.json')
    cases = cases[chunk::2]
    for c in cases:
        data = _inputs.resolve(c['input'])
        o = c['opts']
        out = _oracle.encode(data, o.get('quality', 11), o.get('lgwin', 22), o.get('mode', 0))
        assert hashlib.sha256(out).hexdigest() == c['sha256'], (c['input'], o)
        # ref-fixed still emits one invalid stream (compressed_repeated: packed extra bits
        # overflow, Bug F metablock.ts:283-286); it must fail exactly as native brotli says.
        assert (_oracle.decode(out) == data) == c['native_roundtrip'], (c['input'], o)


def test_encode_q5_9_matches_reference():
    """brotliEncode at qualities 5-9 (hash chains + greedy, backward-references.ts:14-134,
    hash-chains.ts:68-153) byte-identical to the reference run as is (86 cases: text, binary,
    fonts in FONT mode, TEXT mode, lgwin 16 / 22 / 24, up to 4 MiB at q9 lgwin 22); the golden
    streams all decode to their inputs under native brotli, and under the oracle decoder."""
    cases = _load('encode_ref_q5_9.json')
    assert len(cases) == 86
    for c in cases:
        data = _inputs.resolve(c['input'])
        o = c['opts']
        out = _oracle.encode(data, o['quality'], o.get('lgwin', 22), o.get('mode', 0))
        assert hashlib.sha256(out).hexdigest() == c['sha256'], (c['input'], o)
        assert c['native_roundtrip']
        if len(data) <= 300000:
            assert _oracle.decode(out) == data


def test_peek_decoded_size():
    assert _oracle.peek_size(_oracle.encode(b'x' * 1000)) == 1000
    assert _oracle.peek_size(_oracle.encode(b'')) == 0


def test_oracle_decoder_is_thread_safe():
    """bench.py's cpu_baseline runs the oracle on many threads at once: concurrent decodes of
    streams with different prefix codes must each give their own bytes."""
    from concurrent.futures import ThreadPoolExecutor
    pairs = []
    for nm in sorted(os.listdir(os.path.join(G, 'vectors'))):
        if nm.endswith('.compressed'):
            with open(os.path.join(G, 'vectors', nm), 'rb') as f:
                comp = f.read()
            with open(os.path.join(G, 'vectors', nm[:-len('.compressed')]), 'rb') as f:
                pairs.append((comp, f.read()))
    work = pairs * 12
    with ThreadPoolExecutor(8) as ex:
        got = list(ex.map(lambda p: _oracle.decode(p[0]) == p[1], work))
    assert all(got)


def test_compound_dictionary_matches_reference():
    """customDictionary (compound dictionary, engine.ts:142-159,946-1011): the oracle decodes
    the reference-decoded corpus (oracle/refgen/make_compound.py) to the same bytes / errors,
    including the reference's rule that a dictionary copy must end at the dictionary's end
    (-9 otherwise) and its TypeError past the end (-1000 here)."""
    n_ok = 0
    for c in _load('decode_compound.json'):
        data = base64.b64decode(c['in_b64'])
        out = _oracle.decode(data, dictionary=_inputs.resolve(c['dict']))
        if 'error' not in c:
            assert not isinstance(out, int) and hashlib.sha256(out).hexdigest() == c['sha256'], c
            n_ok += 1
        elif c['error'].startswith('Brotli error code: '):
            assert out == int(c['error'].split(': ')[1]), (c, out)
        else:
            assert 'subarray' in c['error'] and out == -1000, (c, out)
    assert n_ok > 100


def test_bt_matches_match_reference():
    """The oracle's binary-tree match finder (hash-binary-tree.ts:57-227, Bug B fixed) gives
    the reference's per-position match lists (tests/golden/bt_matches.json)."""
    for c in _load('bt_matches.json'):
        data = _inputs.resolve(c['input'])
        got = _oracle.bt_matches(data, c.get('lgwin', 22))
        exp = [(i, [tuple(m) for m in ms]) for i, ms in c['lists']]
        assert got == exp, c['input']
