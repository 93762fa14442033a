"""Static-dictionary references in the encoder (RFC 7932 section 8): where the
window holds no match, a word of the RFC dictionary that the input repeats in full becomes a
copy whose distance points past the window (identity transform).  The reference encoder has
none (its static-dict.ts is dead code), so parity here is the round trip: the oracle (the
reference decoder restated), the HIP decoder and native brotli return the input, and the
oracle decoder sees the word references."""
import shutil
import subprocess

import pytest

import _oracle
import brotli_amd
from brotli_amd import datagen

pytestmark = pytest.mark.gpu

WORDS = (b'international', b'information', b'development', b'environment', b'government', b'understanding',
         b'management', b'experience', b'particular', b'performance', b'available', b'community', b'technology',
         b'everything', b'interesting', b'particularly', b'different', b'important', b'university', b'education')


def _prose():
    # every word once: nothing for the window to find
    return b'The ' + b', '.join(WORDS) + b' and so on.'


def test_words_become_dictionary_references():
    data = _prose()
    enc = brotli_amd.brotliEncode(data, {'quality': 11})
    r0 = _oracle.word_refs()
    assert _oracle.decode(enc) == data
    assert _oracle.word_refs() - r0 >= 5, 'the encoder emitted no dictionary references'
    assert brotli_amd.brotliDecode(enc) == data
    assert len(enc) < len(data) * 0.8


@pytest.mark.parametrize('seed', [3, 4])
def test_text_with_words_round_trips(seed):
    # words in a larger text, segment ends and the part index included (3 MiB)
    data = datagen.enwik_text(3 << 20, seed)[:(3 << 20) - 77] + _prose()
    enc = brotli_amd.brotliEncode(data, {'quality': 11})
    assert _oracle.decode(enc) == data
    assert brotli_amd.brotliDecode(enc) == data


def test_large_window_distances_are_not_words():
    # lgwin 24: window distances use bit 23, which marks words only where they are enabled
    part = datagen.enwik_text(6 << 20, 8)
    data = part + datagen.enwik_text(3 << 20, 9) + part[:(3 << 20)]
    enc = brotli_amd.brotliEncode(data, {'quality': 11, 'lgwin': 24})
    assert brotli_amd.brotliDecode(enc) == data
    assert _oracle.decode(enc) == data


@pytest.mark.skipif(shutil.which('node') is None, reason='node not installed')
def test_native_brotli_decodes_words(tmp_path):
    data = _prose() * 1 + datagen.enwik_text(100000, 5)
    enc = brotli_amd.brotliEncode(data, {'quality': 11})
    p = tmp_path / 'w.br'
    p.write_bytes(enc)
    js = ("const z=require('zlib'),fs=require('fs');"
          "process.stdout.write(z.brotliDecompressSync(fs.readFileSync(process.argv[1])).toString('latin1'))")
    out = subprocess.run(['node', '-e', js, str(p)], capture_output=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout == data
