import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'brotli-lib_amd', 'python'))


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP path)')


def has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if has_gpu():
        return
    skip = pytest.mark.skip(reason='no GPU in this container')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)


def pytest_assertrepr_compare(config, op, left, right):
    """Large byte strings that differ: where, not a diff (difflib on MiBs of bytes runs for
    minutes, and a silent GPU test run is taken to be hung)."""
    if op == '==' and isinstance(left, (bytes, bytearray)) and isinstance(right, (bytes, bytearray)) \
            and max(len(left), len(right)) > 512:
        n = min(len(left), len(right))
        first = next((i for i in range(n) if left[i] != right[i]), n)
        return ['bytes differ: lengths %d vs %d, first difference at offset %d' % (len(left), len(right), first)]
    if op == '==' and isinstance(left, list) and isinstance(right, list) and len(left) == len(right) and \
            any(isinstance(x, (bytes, bytearray)) and len(x) > 512 for x in left[:4]):
        bad = [i for i in range(len(left)) if left[i] != right[i]]
        return ['lists of byte strings differ at %d of %d items, first %s' % (len(bad), len(left), bad[:8])]
    return None
