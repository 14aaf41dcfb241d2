"""Batch entry points over numpy host buffers and torch device tensors.

Thin, allocation-only wrappers around libeges.so; all arithmetic happens in the HIP kernels.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib


def _u8(a, shape_tail, name):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    if a.ndim != 1 + len(shape_tail) or tuple(a.shape[1:]) != tuple(shape_tail):
        raise ValueError(f"{name}: expected shape (n, {', '.join(map(str, shape_tail))}), got {a.shape}")
    return a


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def init(device_mask=0):
    check(lib.eges_init(device_mask, 0))
    return lib.eges_device_count()


def device_count():
    return lib.eges_device_count()


def set_knob(name, value):
    """eges_test_set_knob: change an engine knob (its environment name) while the engine runs."""
    check(lib.eges_test_set_knob(name.encode(), int(value)))


def get_knob(name):
    v = ctypes.c_longlong()
    check(lib.eges_test_get_knob(name.encode(), ctypes.byref(v)))
    return v.value


class knob:
    """with knob("EGES_LAT_MAX", 0): ... sets a knob for the block and restores it after."""

    def __init__(self, name, value):
        self.name, self.value = name, value

    def __enter__(self):
        self.old = get_knob(self.name)
        set_knob(self.name, self.value)
        return self

    def __exit__(self, *a):
        set_knob(self.name, self.old)


def diag_counters(device=0, reset=False):
    """eges_diag_counters: {name: count} of the rare exact branches the kernels ran (DIAG_NAMES)."""
    out = (ctypes.c_uint64 * _lib.DIAG_COUNT)()
    check(lib.eges_diag_counters(device, out, _lib.DIAG_COUNT, 1 if reset else 0))
    return {n: int(out[i]) for i, n in enumerate(_lib.DIAG_NAMES)}


def _out(buf, n, w, name):
    """a caller-supplied output array (reused across calls, e.g. a buffer pool) or a fresh one"""
    shape = (n, w) if w else (n,)
    if buf is None:
        return np.zeros(shape, np.uint8)
    if not (isinstance(buf, np.ndarray) and buf.dtype == np.uint8 and buf.shape == shape and buf.flags.c_contiguous
            and buf.flags.writeable):
        raise ValueError(f"{name}: expected a writable C-contiguous uint8 array of shape {shape}")
    return buf


def ecrecover_batch(msg, sig, want_pub=True, want_addr=True, out_pub=None, out_addr=None, out_status=None):
    """crypto.Ecrecover over n items: msg (n,32), sig (n,65) -> (pub (n,65)|None, addr (n,20)|None, status (n,)).
    out_* optionally supply the output arrays (written in place and returned)."""
    msg = _u8(msg, (32,), "msg")
    sig = _u8(sig, (65,), "sig")
    n = msg.shape[0]
    if sig.shape[0] != n:
        raise ValueError("msg/sig length mismatch")
    pub = _out(out_pub, n, 65, "out_pub") if want_pub else None
    addr = _out(out_addr, n, 20, "out_addr") if want_addr else None
    status = _out(out_status, n, 0, "out_status")
    if n:
        check(lib.eges_ecrecover_batch(_p(msg), _p(sig), n, _p(pub), _p(addr), _p(status)))
    return pub, addr, status


def sender_batch(sighash, r, s, v, vflags, signer, chain_id):
    """types.Sender over n items (big-endian 32-byte r/s/v + EGES_VF_* flags) -> (addr (n,20), status (n,))."""
    sighash = _u8(sighash, (32,), "sighash")
    r = _u8(r, (32,), "r")
    s = _u8(s, (32,), "s")
    v = _u8(v, (32,), "v")
    n = sighash.shape[0]
    vflags = np.zeros(n, np.uint8) if vflags is None else np.ascontiguousarray(vflags, dtype=np.uint8)
    addr = np.zeros((n, 20), np.uint8)
    status = np.zeros(n, np.uint8)
    if n:
        check(lib.eges_sender_batch(_p(sighash), _p(r), _p(s), _p(v), _p(vflags), n, int(signer), int(chain_id),
                                    _p(addr), _p(status)))
    return addr, status


def pack_raw(raws):
    """List of per-transaction RLP byte strings -> (raw uint8 buffer, offsets uint64 (n+1,))."""
    raws = [bytes(x) for x in raws]
    offsets = np.zeros(len(raws) + 1, np.uint64)
    if raws:
        offsets[1:] = np.cumsum([len(x) for x in raws], dtype=np.uint64)
    raw = np.frombuffer(b"".join(raws), np.uint8).copy() if offsets[-1] else np.zeros(1, np.uint8)
    return raw, offsets


def sender_raw_batch(raws, signer, chain_id, want_sighash=False):
    """types.Sender over wire-format transactions (a list of txdata RLP encodings, or a
    (raw, offsets) pair as pack_raw returns) -> (addr (n,20), status (n,), sighash (n,32)|None).
    Decoding, signing hash and recovery all run on the GPU (eges_sender_raw_batch)."""
    raw, offsets = raws if isinstance(raws, tuple) else pack_raw(raws)
    raw = np.ascontiguousarray(raw, np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = offsets.shape[0] - 1
    addr = np.zeros((n, 20), np.uint8)
    status = np.zeros(n, np.uint8)
    sighash = np.zeros((n, 32), np.uint8) if want_sighash else None
    if n > 0:
        check(lib.eges_sender_raw_batch(_p(raw), _p(offsets), n, int(signer), int(chain_id), _p(addr), _p(status),
                                        _p(sighash)))
    return addr, status, sighash


def block_senders_raw(block, lists=_lib.LIST_TXS, signer=_lib.SIGNER_EIP155, chain_id=None, cap=None):
    """Senders of a whole Geec block (extblock RLP, core/types/block.go:188-195) through
    eges_block_senders_raw -> (addr (m,20), status (m,), counts (3,), block_status) for the
    selected lists (bits: 1 FakeTxs, 2 GeecTxs, 4 Txs), concatenated in list order."""
    from .txs import GEEC_CHAIN_ID
    chain_id = GEEC_CHAIN_ID if chain_id is None else chain_id
    blk = np.frombuffer(bytes(block), np.uint8) if len(block) else np.zeros(1, np.uint8)
    cap = cap if cap is not None else max(1, len(block) // 2)
    addr = np.zeros((cap, 20), np.uint8)
    status = np.zeros(cap, np.uint8)
    counts = np.zeros(3, np.uint32)
    bst = ctypes.c_int(-1)
    check(lib.eges_block_senders_raw(_p(blk), len(block), int(lists), int(signer), int(chain_id), cap, _p(addr),
                                     _p(status), _p(counts), ctypes.byref(bst)))
    m = sum(int(counts[k]) for k in range(3) if lists & (1 << k))  # 0 when the structure fails
    return addr[:m].copy(), status[:m].copy(), counts, bst.value


def ecrecover_precompile_batch(inputs):
    """The EVM ECRECOVER precompile (core/vm/contracts.go:77-101) over a list of call inputs
    (bytes of any length) -> (out (n,32), status (n,)); item i returns out[i] when status[i] == 0
    and nil otherwise."""
    n = len(inputs)
    buf = np.zeros((n, 128), np.uint8)
    inlen = np.zeros(n, np.uint32)
    for i, x in enumerate(inputs):
        x = bytes(x)[:128]
        buf[i, :len(x)] = np.frombuffer(x, np.uint8)
        inlen[i] = len(x)
    out = np.zeros((n, 32), np.uint8)
    status = np.zeros(n, np.uint8)
    if n:
        check(lib.eges_ecrecover_precompile_batch(_p(buf), _p(inlen), n, _p(out), _p(status)))
    return out, status


def verify_batch(pub, publen, msg, sig):
    """crypto.VerifySignature over n items: pub (n,65) left-aligned, publen (n,), msg (n,32), sig (n,64) -> ok (n,)."""
    pub = _u8(pub, (65,), "pub")
    msg = _u8(msg, (32,), "msg")
    sig = _u8(sig, (64,), "sig")
    publen = np.ascontiguousarray(publen, dtype=np.uint8)
    n = pub.shape[0]
    ok = np.zeros(n, np.uint8)
    if n:
        check(lib.eges_verify_batch(_p(pub), _p(publen), _p(msg), _p(sig), n, _p(ok)))
    return ok


def keccak256(data):
    data = bytes(data)
    a = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    out = np.zeros(32, np.uint8)
    lib.eges_keccak256(_p(a), len(data), _p(out))
    return out.tobytes()


# ------------------------------------------------------------------ torch device tensors
def _tp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _dchk(t, tail, name, n, dev, dtype=None, optional=False):
    """Validate a device tensor handed to a *_dev entry: dtype (uint8 unless given), C-contiguous,
    shape (n, *tail), on `dev`. The C-ABI takes raw pointers and sizes, so a sliced, short or
    foreign-device tensor would otherwise be read or written out of bounds."""
    import torch
    if t is None:
        if optional:
            return None
        raise ValueError(f"{name}: required")
    want = dtype or torch.uint8
    dts = want if isinstance(want, tuple) else (want,)
    if t.dtype not in dts:
        raise ValueError(f"{name}: dtype {t.dtype}, expected {' or '.join(map(str, dts))}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if t.device != dev:
        raise ValueError(f"{name}: on {t.device}, expected {dev}")
    shape = (n,) + tuple(tail)
    if tuple(t.shape) != shape:
        raise ValueError(f"{name}: shape {tuple(t.shape)}, expected {shape}")
    return t


def _stream_of(t):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def ecrecover_batch_dev(msg, sig, pub=None, addr=None, status=None, stream=None):
    """Device-resident batch: uint8 CUDA(HIP) tensors msg (n,32), sig (n,65); outputs allocated if None.
    Enqueued on `stream` (default: torch's current stream of the tensors' device); asynchronous."""
    import torch
    n = msg.shape[0]
    dev = msg.device
    if addr is None:
        addr = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    if status is None:
        status = torch.empty((n,), dtype=torch.uint8, device=dev)
    _dchk(msg, (32,), "msg", n, dev)
    _dchk(sig, (65,), "sig", n, dev)
    _dchk(pub, (65,), "pub", n, dev, optional=True)
    _dchk(addr, (20,), "addr", n, dev)
    _dchk(status, (), "status", n, dev)
    st = ctypes.c_void_p(stream) if stream is not None else _stream_of(msg)
    check(lib.eges_ecrecover_batch_dev(dev.index, _tp(msg), _tp(sig), n, _tp(pub), _tp(addr), _tp(status), st))
    return pub, addr, status


def synth_sign_dev(first_index, n, device, stream=None):
    """Deterministic synthetic signed batch on `device` -> (msg (n,32), sig (n,65), expected addr (n,20))."""
    import torch
    dev = torch.device("cuda", device) if isinstance(device, int) else device
    msg = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    sig = torch.empty((n, 65), dtype=torch.uint8, device=dev)
    addr = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(stream) if stream is not None else _stream_of(msg)
    check(lib.eges_synth_sign_dev(dev.index, int(first_index), n, _tp(msg), _tp(sig), _tp(addr), st))
    return msg, sig, addr


def synth_sign_msg_dev(msg, first_index=0, stream=None):
    """Sign caller-supplied 32-byte hashes (uint8 device tensor (n,32)) with the synthetic keys of
    indices first_index.. -> (sig (n,65), expected addr (n,20))."""
    import torch
    n = msg.shape[0]
    dev = msg.device
    sig = torch.empty((n, 65), dtype=torch.uint8, device=dev)
    addr = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    _dchk(msg, (32,), "msg", n, dev)
    st = ctypes.c_void_p(stream) if stream is not None else _stream_of(msg)
    check(lib.eges_synth_sign_msg_dev(dev.index, int(first_index), n, _tp(msg), _tp(sig), _tp(addr), st))
    return sig, addr


def verify_batch_dev(pub, publen, msg, sig, ok=None, stream=None):
    """crypto.VerifySignature over device tensors: pub (n,65) left-aligned, publen (n,), msg (n,32),
    sig (n,64) -> ok (n,) uint8. Asynchronous on `stream`."""
    import torch
    n = msg.shape[0]
    if ok is None:
        ok = torch.empty((n,), dtype=torch.uint8, device=msg.device)
    dev = msg.device
    _dchk(pub, (65,), "pub", n, dev)
    _dchk(publen, (), "publen", n, dev)
    _dchk(msg, (32,), "msg", n, dev)
    _dchk(sig, (64,), "sig", n, dev)
    _dchk(ok, (), "ok", n, dev)
    st = ctypes.c_void_p(stream) if stream is not None else _stream_of(msg)
    check(lib.eges_verify_batch_dev(msg.device.index, _tp(pub), _tp(publen), _tp(msg), _tp(sig), n, _tp(ok), st))
    return ok


def sender_batch_dev(sighash, r, s, v, vflags, signer, chain_id, addr=None, status=None, stream=None):
    """types.Sender over device tensors (n,32) x4 + vflags (n,) -> (addr (n,20), status (n,))."""
    import torch
    n = sighash.shape[0]
    dev = sighash.device
    if addr is None:
        addr = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    if status is None:
        status = torch.empty((n,), dtype=torch.uint8, device=dev)
    for t, name in ((sighash, "sighash"), (r, "r"), (s, "s"), (v, "v")):
        _dchk(t, (32,), name, n, dev)
    _dchk(vflags, (), "vflags", n, dev, optional=True)
    _dchk(addr, (20,), "addr", n, dev)
    _dchk(status, (), "status", n, dev)
    st = ctypes.c_void_p(stream) if stream is not None else _stream_of(sighash)
    check(lib.eges_sender_batch_dev(dev.index, _tp(sighash), _tp(r), _tp(s), _tp(v), _tp(vflags), n, int(signer),
                                    int(chain_id), _tp(addr), _tp(status), st))
    return addr, status


def sender_raw_batch_dev(raw, offsets, signer, chain_id, addr=None, status=None, sighash=None, stream=None):
    """types.Sender over wire-format transactions resident on the device: raw uint8 tensor,
    offsets int64/uint64 tensor (n+1,) (item i = raw[offsets[i]-offsets[0] : offsets[i+1]-offsets[0]])
    -> (addr (n,20), status (n,)). Asynchronous on `stream`."""
    import torch
    n = offsets.shape[0] - 1
    dev = raw.device
    if addr is None:
        addr = torch.empty((n, 20), dtype=torch.uint8, device=dev)
    if status is None:
        status = torch.empty((n,), dtype=torch.uint8, device=dev)
    if raw.dtype != torch.uint8 or raw.dim() != 1 or not raw.is_contiguous() or raw.device != dev:
        raise ValueError("raw: expected a contiguous 1-D uint8 tensor on the device")
    _dchk(offsets, (), "offsets", n + 1, dev, dtype=(torch.int64, torch.uint64))
    _dchk(addr, (20,), "addr", n, dev)
    _dchk(status, (), "status", n, dev)
    _dchk(sighash, (32,), "sighash", n, dev, optional=True)
    st = ctypes.c_void_p(stream) if stream is not None else _stream_of(raw)
    check(lib.eges_sender_raw_batch_dev(dev.index, _tp(raw), _tp(offsets), n, int(signer), int(chain_id), _tp(addr),
                                        _tp(status), _tp(sighash), st))
    return addr, status


def ecrecover_precompile_batch_dev(input, inlen=None, out=None, status=None, stream=None):
    """The ECRECOVER precompile over device tensors: input (n,128) uint8, inlen (n,) int32 or None
    -> (out (n,32), status (n,)). Asynchronous on `stream`."""
    import torch
    n = input.shape[0]
    dev = input.device
    if out is None:
        out = torch.empty((n, 32), dtype=torch.uint8, device=dev)
    if status is None:
        status = torch.empty((n,), dtype=torch.uint8, device=dev)
    _dchk(input, (128,), "input", n, dev)
    _dchk(inlen, (), "inlen", n, dev, dtype=(torch.int32, torch.uint32), optional=True)
    _dchk(out, (32,), "out", n, dev)
    _dchk(status, (), "status", n, dev)
    st = ctypes.c_void_p(stream) if stream is not None else _stream_of(input)
    check(lib.eges_ecrecover_precompile_batch_dev(dev.index, _tp(input), _tp(inlen), n, _tp(out), _tp(status), st))
    return out, status
