"""Geec block (extblock) structure: the tx oracle's split against hand-built blocks, and the
C-ABI entry eges_block_senders_raw on blocks whose structure it rejects or that select no list
(both answered on the host before any GPU work, so these run without a GPU). The GPU side is
tests/test_gpu_block.py."""
import ctypes

import numpy as np
import pytest

from eges_amd import txs
from oracle import txoracle as T


def block(fake=2, geec=1, n=3, **kw):
    f = [txs.fake_tx(data_len=100) for _ in range(fake)]
    g = [txs.fake_tx(data_len=17, is_geec=True, data=b"udp payload %d" % i) for i in range(geec)]
    t = [txs.encode_geec_tx(i, 1, 21000, b"\x22" * 20, 1, b"", False, 37, 5 + i, 7 + i) for i in range(n)]
    return txs.geec_extblock(f, g, t, **kw), (f, g, t)


def test_split_well_formed():
    raw, (f, g, t) = block(5, 2, 9)
    lists = T.split_extblock(raw)
    assert [len(x) for x in lists] == [5, 2, 9]
    assert lists[0] == f and lists[1] == g and lists[2] == t
    empty, _ = block(0, 0, 0)
    assert [len(x) for x in T.split_extblock(empty)] == [0, 0, 0]


def malformed():
    raw, _ = block()
    items = []
    s = T._Stream(raw)
    s.list_start()
    while s.pos < s.ends[-1]:
        st = s.pos
        k, size, _ = s.kind()
        if k != "byte":
            s.content(size)
        items.append(s.b[st:s.pos])
    assert len(items) == 6
    yield "trailing byte", raw + b"\x00"
    yield "five elements", T.enc_list(items[:5])
    yield "seven elements", T.enc_list(items + [b"\xc0"])
    yield "header not a list", T.enc_list([b"\x83abc"] + items[1:])
    yield "txs not a list", T.enc_list(items[:3] + [b"\x80"] + items[4:])
    yield "confirm non-empty string", T.enc_list(items[:5] + [b"\x81\x99"])
    yield "truncated", raw[:-3]
    yield "not a list", b"\x83abc"
    yield "tx item overruns its list", T.enc_list(items[:3] + [b"\xc2\xc3\x01"] + items[4:])
    yield "non-canonical list size", T.enc_list(items[:3] + [b"\xf8\x02\xc1\x01"] + items[4:])


@pytest.mark.parametrize("name,raw", list(malformed()), ids=[m[0] for m in malformed()])
def test_malformed_blocks(name, raw):
    with pytest.raises(T.DecodeError):
        T.split_extblock(raw)
    # the C-ABI rejects the same structure on the host (no GPU work is started)
    from eges_amd._lib import lib
    counts = np.zeros(3, np.uint32)
    bst = ctypes.c_int(-1)
    buf = np.frombuffer(raw, np.uint8)
    rc = lib.eges_block_senders_raw(ctypes.c_void_p(buf.ctypes.data), len(raw), 7, 2, txs.GEEC_CHAIN_ID, 0, None, None,
                                    ctypes.c_void_p(counts.ctypes.data), ctypes.byref(bst))
    assert rc == 0 and bst.value == T.DECODE_FAILED and not counts.any()


def test_counts_without_selection():
    """A sizing call (cap 0) returns EGES_E_INVALID_ARG with counts and block_status valid, on the
    host. With nothing selected, every list still goes through the GPU decoder (rlp.DecodeBytes
    decodes all of them): no fallback without a device."""
    import torch
    from eges_amd._lib import EGES_E_INVALID_ARG, EGES_E_NODEVICE, lib
    raw, _ = block(4, 3, 11)
    counts = np.zeros(3, np.uint32)
    bst = ctypes.c_int(-1)
    buf = np.frombuffer(raw, np.uint8)
    rc = lib.eges_block_senders_raw(ctypes.c_void_p(buf.ctypes.data), len(raw), 7, 2, txs.GEEC_CHAIN_ID, 0, None, None,
                                    ctypes.c_void_p(counts.ctypes.data), ctypes.byref(bst))
    assert rc == EGES_E_INVALID_ARG and bst.value == 0 and counts.tolist() == [4, 3, 11]
    if torch.cuda.is_available():
        return
    counts[:] = 0
    rc = lib.eges_block_senders_raw(ctypes.c_void_p(buf.ctypes.data), len(raw), 0, 2, txs.GEEC_CHAIN_ID, 0, None, None,
                                    ctypes.c_void_p(counts.ctypes.data), ctypes.byref(bst))
    assert rc == EGES_E_NODEVICE and counts.tolist() == [4, 3, 11]
