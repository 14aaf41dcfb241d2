"""The resident servers (capi.hip Resident, k_recover_lat.hip lat_resident_kernel /
lat_resident_block_kernel): coalesced eges_ecdsa_recover / eges_ecdsa_verify groups go to
split-form workgroups, and latency-kernel blocks above the three-wave form's range to a
narrow-form grid, that stay resident and poll a job word in coherent pinned memory instead of a
launch per call. Every golden item through them against the fixtures; device-wide calls between
(the servers stop first and restart on the next call); idle exits and restarts; the servers
switched off. EGES_DIAG_RESIDENT counts the jobs they served."""
import ctypes
import time

import numpy as np
import pytest

from conftest import load_golden
from eges_amd import _lib

pytestmark = pytest.mark.gpu


class knobs:
    def __init__(self, engine, kv):
        self.engine, self.kv = engine, kv

    def __enter__(self):
        self.old = {k: self.engine.get_knob(k) for k in self.kv}
        for k, v in self.kv.items():
            self.engine.set_knob(k, v)

    def __exit__(self, *a):
        for k, v in self.old.items():
            self.engine.set_knob(k, v)


def _single_recover(msg, sig):
    out = (ctypes.c_ubyte * 65)()
    rc = _lib.lib.eges_ecdsa_recover(out, sig.tobytes(), msg.tobytes())
    return rc, bytes(out)


def test_resident_single_recover_golden(engine):
    g = load_golden("recover.npz")
    engine.diag_counters(reset=True)
    calls = 0
    with knobs(engine, {"EGES_RESIDENT": 1}):
        for i in range(len(g["msg"])):
            if g["sig"][i][64] >= 4:
                continue  # checkSignature rejects these before the C call (secp256.go:171-179)
            rc, pub = _single_recover(g["msg"][i], g["sig"][i])
            want = 1 if g["status"][i] == 0 else 0
            assert rc == want, (i, rc, int(g["status"][i]))
            if rc == 1:
                assert pub == g["pub"][i].tobytes(), i
            calls += 1
    d = engine.diag_counters(reset=True)
    assert d["resident"] >= calls, (d, calls)


def test_resident_single_verify_golden(engine):
    gv = load_golden("verify.npz")
    engine.diag_counters(reset=True)
    with knobs(engine, {"EGES_RESIDENT": 1}):
        for i in range(len(gv["msg"])):
            plen = int(gv["publen"][i])
            if plen not in (33, 65):
                continue
            rc = _lib.lib.eges_ecdsa_verify(gv["sig"][i].tobytes(), gv["msg"][i].tobytes(), gv["pub"][i][:plen].tobytes(),
                                            plen)
            assert rc == int(gv["ok"][i]), (i, rc)
    assert engine.diag_counters(reset=True)["resident"] > 0


def test_resident_stops_for_batches_and_restarts(engine):
    """single calls and batch calls alternating: every batch stops the server first (it would
    share the CUs), the next single call starts it again"""
    g = load_golden("recover.npz")
    ok = np.nonzero((g["status"] == 0) & (g["sig"][:, 64] < 4))[0]
    engine.diag_counters(reset=True)
    with knobs(engine, {"EGES_RESIDENT": 1}):
        for rep in range(40):
            i = int(ok[(rep * 37) % len(ok)])
            rc, pub = _single_recover(g["msg"][i], g["sig"][i])
            assert rc == 1 and pub == g["pub"][i].tobytes(), (rep, i)
            sel = np.arange(rep * 50, rep * 50 + 3000) % len(g["msg"])
            bp, _, bs = engine.ecrecover_batch(g["msg"][sel], g["sig"][sel])  # mid-size: device-wide
            assert np.array_equal(bs, g["status"][sel]) and np.array_equal(bp, g["pub"][sel]), rep
    assert engine.diag_counters(reset=True)["resident"] >= 40


def test_resident_idle_exit_and_restart(engine):
    g = load_golden("recover.npz")
    ok = np.nonzero((g["status"] == 0) & (g["sig"][:, 64] < 4))[0]
    engine.diag_counters(reset=True)
    with knobs(engine, {"EGES_RESIDENT": 1, "EGES_RESIDENT_IDLE_MS": 4}):
        for rep in range(12):
            i = int(ok[rep])
            rc, pub = _single_recover(g["msg"][i], g["sig"][i])
            assert rc == 1 and pub == g["pub"][i].tobytes(), rep
            time.sleep(0.001 * (rep % 4) * 3)  # 0, 3, 6, 9 ms: across the server's idle bound
    assert engine.diag_counters(reset=True)["resident"] >= 12


def test_resident_off_uses_the_lanes(engine):
    g = load_golden("recover.npz")
    i = int(np.nonzero((g["status"] == 0) & (g["sig"][:, 64] < 4))[0][0])
    engine.diag_counters(reset=True)
    with knobs(engine, {"EGES_RESIDENT": 0}):
        rc, pub = _single_recover(g["msg"][i], g["sig"][i])
    assert rc == 1 and pub == g["pub"][i].tobytes()
    assert engine.diag_counters(reset=True)["resident"] == 0


# ---- the block server: latency-kernel blocks above the three-wave form's range (narrow form)
def _sender_block(engine, n, first):
    import torch
    from eges_amd import txs
    h = txs.geec_block(first, n, payload=100)
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(h).cuda(), first)
    torch.cuda.synchronize()
    sig_h, exp = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    r, s, v = txs.sender_rows(sig_h, txs.GEEC_CHAIN_ID)
    return h, r, s, v, exp


def test_block_server_sender_blocks(engine):
    """1000-transaction blocks (C3) through eges_sender_batch, one after another, with single calls
    between them (both servers resident at once)"""
    from eges_amd import txs
    g = load_golden("recover.npz")
    i1 = int(np.nonzero((g["status"] == 0) & (g["sig"][:, 64] < 4))[0][0])
    engine.diag_counters(reset=True)
    with knobs(engine, {"EGES_RESIDENT": 1, "EGES_RESIDENT_BLOCK": 1}):
        for rep, n in enumerate([1000, 1000, 777, 449, 1000]):
            h, r, s, v, exp = _sender_block(engine, n, 100000 * rep)
            addr, st = engine.sender_batch(h, r, s, v, None, _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID)
            assert (st == 0).all() and np.array_equal(addr, exp), (rep, n)
            rc, pub = _single_recover(g["msg"][i1], g["sig"][i1])
            assert rc == 1 and pub == g["pub"][i1].tobytes()
    assert engine.diag_counters(reset=True)["resident"] >= 10


def test_block_server_recover_golden_tiled(engine):
    """every golden recovery item (all reject classes) in 600-item blocks, pub + address + status"""
    g = load_golden("recover.npz")
    n = len(g["msg"])
    engine.diag_counters(reset=True)
    with knobs(engine, {"EGES_RESIDENT_BLOCK": 1}):
        for a in range(0, n, 600):
            sel = np.arange(a, min(n, a + 600))
            if len(sel) <= 448:
                sel = np.arange(a, a + 600) % n
            pub, addr, st = engine.ecrecover_batch(g["msg"][sel], g["sig"][sel])
            assert np.array_equal(st, g["status"][sel]) and np.array_equal(pub, g["pub"][sel]), a
    assert engine.diag_counters(reset=True)["resident"] >= n // 600
    with knobs(engine, {"EGES_RESIDENT_BLOCK": 0}):
        sel = np.arange(0, 600)
        pub0, addr0, st0 = engine.ecrecover_batch(g["msg"][sel], g["sig"][sel])
    assert engine.diag_counters(reset=True)["resident"] == 0
    assert np.array_equal(st0, g["status"][sel]) and np.array_equal(pub0, g["pub"][sel])


def test_block_server_stops_for_device_work_and_idles_out(engine):
    from eges_amd import txs
    g = load_golden("recover.npz")
    engine.diag_counters(reset=True)
    with knobs(engine, {"EGES_RESIDENT_BLOCK": 1, "EGES_RESIDENT_IDLE_MS": 4}):
        for rep in range(6):
            h, r, s, v, exp = _sender_block(engine, 800, 7000 * rep)
            addr, st = engine.sender_batch(h, r, s, v, None, _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID)
            assert (st == 0).all() and np.array_equal(addr, exp), rep
            if rep % 2:
                sel = np.arange(0, 3000) % len(g["msg"])  # a mid-size batch: device-wide work
                pub, _, st2 = engine.ecrecover_batch(g["msg"][sel], g["sig"][sel])
                assert np.array_equal(st2, g["status"][sel]) and np.array_equal(pub, g["pub"][sel])
            else:
                time.sleep(0.01)  # past the server's idle bound
    assert engine.diag_counters(reset=True)["resident"] >= 6
