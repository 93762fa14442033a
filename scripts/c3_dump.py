"""Encode a few C3 (glyf-like, FONT) buffers on the GPU and save the streams for analysis."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'brotli-lib_amd', 'python'))
import brotli_amd
from brotli_amd import datagen
out = sys.argv[1]
os.makedirs(out, exist_ok=True)
for i in range(4):
    d = datagen.glyf_stream(262144, 1000 + i)
    e = brotli_amd.brotliEncode(d, {'quality': 11, 'lgwin': 22, 'mode': 2})
    open(os.path.join(out, 'c3_%d.br' % i), 'wb').write(e)
    print(i, len(e) / len(d))
