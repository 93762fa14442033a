"""The Node-API drop-in (brotli-lib_amd/node) exercised by tests/node/addon_test.js on the GPU."""
import os
import shutil
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_node_addon_surface():
    node = shutil.which('node')
    if node is None:
        pytest.skip('node is not installed')
    addon = os.path.join(ROOT, 'brotli-lib_amd', 'node', 'brotli_amd.node')
    assert os.path.exists(addon), 'run __graft_entry__.build() first'
    r = subprocess.run([node, os.path.join(ROOT, 'tests', 'node', 'addon_test.js')], capture_output=True, text=True,
                       timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stderr[-4000:]
    assert 'ALL OK' in r.stdout
