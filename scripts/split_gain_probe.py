"""The block split's cost per (metablock, category) (experiment build, MIB_SPLIT_PRINT=n prints
the first n metablocks' one-type and split costs): C4 / C3 streams against the heterogeneous
input of test_more_than_four_command_and_distance_block_types."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'brotli-lib_amd', 'python'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import brotli_amd  # noqa: E402
from brotli_amd import datagen  # noqa: E402
import test_gpu_encode  # noqa: E402

print('== kinds', flush=True)
brotli_amd.brotliEncode(test_gpu_encode._kinds_input())
print('== c4', flush=True)
brotli_amd.encode_batch([datagen.enwik_text(1 << 20, 100 + i) for i in range(4)])
print('== c3', flush=True)
brotli_amd.encode_batch(datagen.glyf_font_batch(4, 1 << 18, 1000, workers=4), {'mode': 2})
