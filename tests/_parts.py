"""Reader of the part index (brotli-lib_amd/csrc/parts.h) a stream carries in its first
metadata metablock(s): test infrastructure, independent of the C++ reader in runtime.cpp."""
import numpy as np

MAGIC = 0x3170424D
VALID, AT_MB = 1, 2
HEAD_DTYPE = np.dtype([('magic', '<u4'), ('version', '<u2'), ('entry_bytes', '<u2'), ('nentries', '<u4'),
                       ('lgwin', '<u4'), ('next_byte', '<u8'), ('total', '<u8')])
ENTRY_DTYPE = np.dtype([('bit', '<u8'), ('pos', '<u8'), ('mb_bit', '<u8'), ('mb_pos', '<u8'), ('ring', '<u4', 4),
                        ('blen', '<u4', 3), ('type', 'u1', 3), ('prev', 'u1', 3), ('p1', 'u1'), ('p2', 'u1'),
                        ('flags', '<u4')])
assert HEAD_DTYPE.itemsize == 32 and ENTRY_DTYPE.itemsize == 72


class _Bits:
    def __init__(self, b, bit):
        self.b, self.bit = b, bit

    def get(self, n):
        v = 0
        for i in range(n):
            byte = self.b[self.bit >> 3] if (self.bit >> 3) < len(self.b) else 0
            v |= ((byte >> (self.bit & 7)) & 1) << i
            self.bit += 1
        return v


def index_block(stream, at=0):
    """(payload byte offset, payload length) of the metadata block at byte `at` (window bits
    first when at == 0), or None when there is none"""
    r = _Bits(stream, 8 * at)
    if at == 0 and r.get(1):
        if r.get(3) == 0:
            r.get(3)
    if r.get(1) != 0 or r.get(2) != 3 or r.get(1) != 0:
        return None
    nb = r.get(2)
    if nb == 0:
        return None
    length = r.get(8 * nb) + 1
    return (r.bit + 7) >> 3, length


def read_index(stream, at=0):
    """(head, entries) of the index block at byte `at` (window bits first when at == 0), or None"""
    r = _Bits(stream, 8 * at)
    lgwin = None
    if at == 0:
        if r.get(1) == 0:
            lgwin = 16
        else:
            m = r.get(3)
            if m:
                lgwin = 17 + m
            else:
                k = r.get(3)
                lgwin = 8 + k if k else 17
    if r.get(1) != 0 or r.get(2) != 3 or r.get(1) != 0:
        return None
    nb = r.get(2)
    if nb == 0:
        return None
    length = r.get(8 * nb) + 1
    pay = (r.bit + 7) >> 3
    head = np.frombuffer(bytes(stream[pay:pay + 32]), dtype=HEAD_DTYPE)[0]
    if int(head['magic']) != MAGIC:
        return None
    n = int(head['nentries'])
    assert 32 + 72 * n <= length
    ents = np.frombuffer(bytes(stream[pay + 32:pay + 32 + 72 * n]), dtype=ENTRY_DTYPE)
    if lgwin is not None:
        assert int(head['lgwin']) == lgwin
    return head, ents


def read_chain(stream):
    """every valid entry of the stream's index chain and the stream's total, or None"""
    at, valid, total = 0, [], None
    while True:
        got = read_index(stream, at)
        if got is None:
            break
        head, ents = got
        valid.append(ents[(ents['flags'] & VALID) != 0])
        total = int(head['total'])
        if int(head['next_byte']) == 0:
            break
        at = int(head['next_byte'])
    if not valid:
        return None
    return np.concatenate(valid), total
