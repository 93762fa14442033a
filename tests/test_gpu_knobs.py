"""The shipped library ignores the environment.

The A/B scripts steer experiment builds through MIB_* variables (common.h `knob`); a server
that happens to carry one of them in its environment must still get the same stream bytes.
A fresh child interpreter is started with every knob that ever changed output set to a
value that would change it (MIB_FM_SORTED_STORE made streams that decode to wrong bytes),
before it makes any GPU call; its C4-shaped batch (1 MiB text buffers, q11, GENERIC) and a
FONT-mode batch must equal the parent's byte for byte and round-trip.
"""
import hashlib
import json
import os
import subprocess
import sys

import pytest

import brotli_amd
from brotli_amd import datagen

pytestmark = pytest.mark.gpu
MIB = 1 << 20

KNOBS = {
    'MIB_FM_SORTED_STORE': '1', 'MIB_LIT_TREES': '64', 'MIB_HASH_BYTES': '5', 'MIB_CMD_PENALTY': '6',
    'MIB_SPLIT_BT': '1,1,1', 'MIB_DP_KS': '1', 'MIB_REP': '1', 'MIB_DICT': '0', 'MIB_DP_PIECES': '0',
    'MIB_CTX_MODE': '2', 'MIB_DEPTH': '4', 'MIB_ZOPFLI_ITERS': '1', 'MIB_ZOPFLI_SAMPLE': '8192',
    'MIB_MB_BITS': '18', 'MIB_PART_MIN': '1048576', 'MIB_PART_BITS': '17', 'MIB_PART_LAG': '0',
    'MIB_DICT_SPAN': '0', 'MIB_ENC_LANES': '1', 'MIB_FM_TILE': '512', 'MIB_STREAM_CHUNK': '1',
    'MIB_DEC_GRID': '7', 'MIB_CODES_NT': '256', 'MIB_HISTO_NT': '256', 'MIB_SIZES_NT': '256',
}

CHILD = r'''
import hashlib, json, sys
sys.path.insert(0, sys.argv[1])
import brotli_amd
from brotli_amd import datagen
MIB = 1 << 20
d = datagen.enwik_text(32 * MIB, 4242)
bufs = [d[i:i + MIB] for i in range(0, len(d), MIB)]
res = {}
for mode in (0, 2):
    outs = brotli_amd.encode_batch(bufs, {'quality': 11, 'lgwin': 22, 'mode': mode})
    assert brotli_amd.decode_batch(outs) == bufs
    res[str(mode)] = [hashlib.sha256(o).hexdigest() for o in outs]
e = brotli_amd.BrotliEncoder({'quality': 9, 'lgwin': 24})
s = b''.join([e.update(d[i:i + 4 * MIB]) for i in range(0, 12 * MIB, 4 * MIB)] + [e.finish()])
assert brotli_amd.brotliDecode(s) == d[:12 * MIB]
res['stream'] = hashlib.sha256(s).hexdigest()
print(json.dumps(res))
'''


def _run_child(env):
    py = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'brotli-lib_amd', 'python')
    out = subprocess.run([sys.executable, '-c', CHILD, py], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_environment_knobs_do_not_change_stream_bytes():
    base = {k: v for k, v in os.environ.items() if not k.startswith('MIB_')}
    clean = _run_child(base)
    knobbed = _run_child(dict(base, **KNOBS))
    assert knobbed == clean
    # and the parent (this process) agrees with both on the C4-shaped batch
    d = datagen.enwik_text(32 * MIB, 4242)
    outs = brotli_amd.encode_batch([d[i:i + MIB] for i in range(0, len(d), MIB)], {'quality': 11, 'lgwin': 22})
    assert [hashlib.sha256(o).hexdigest() for o in outs] == clean['0']
