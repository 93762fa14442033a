"""Regenerate parts_enwik300k.br: a GPU-encoded stream with a part index (64 KiB parts forced by
MIB_PART_MIN / MIB_PART_BITS) that the CPU tests check against the oracle.  Run on an MI355X:
    MIB_PART_MIN=65537 MIB_PART_BITS=16 python3 tests/golden/parts/make_fixture.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402

data = datagen.enwik_text(300000, 21)
enc = brotli_amd.brotliEncode(data, {'quality': 11, 'lgwin': 22})
assert brotli_amd.brotliDecode(enc) == data
out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, 'parts_enwik300k.br')
with open(out, 'wb') as f:
    f.write(enc)
print(out, len(enc), brotli_amd.part_stats())
