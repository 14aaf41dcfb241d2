"""The latency kernel's three-wave form (k_recover_lat.hip FORM_TRI, EGES_LAT_TRI_MAX): wave 0
runs windows [0, TRI_W0) of both GLV halves, wave 2 the rest of both halves against a table of
D = 2^(5 TRI_W0) R', wave 1 the scalar work and u1 G, the roots come from the helper workgroups.
Every golden recovery / sender item, wire-format transactions, synthetic batches up to the form's
one-generation bound, the forced exact redo, the root fallback and the hand-off faults, each
against the fixtures or the other forms byte for byte. EGES_DIAG_LAT_TRI shows the form ran (the
engine falls back to the narrow form above the occupancy bound)."""
import ctypes

import numpy as np
import pytest

from conftest import load_golden
from eges_amd import _lib

pytestmark = pytest.mark.gpu

ALL = 1 << 20
TRI = {"EGES_LAT_MAX": ALL, "EGES_LAT_WIDE_MAX": 0, "EGES_LAT_TRI_MAX": ALL}
NARROW = {"EGES_LAT_MAX": ALL, "EGES_LAT_WIDE_MAX": 0, "EGES_LAT_TRI_MAX": 0}
LANE = {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 0}
CHUNK = 900  # under the form's one-generation bound (3 n + helpers <= 12 x CUs)


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


def _recover_chunks(engine, msg, sig, kv):
    pubs, addrs, sts = [], [], []
    with knobs(engine, kv):
        for a in range(0, len(msg), CHUNK):
            p, d, s = engine.ecrecover_batch(msg[a:a + CHUNK], sig[a:a + CHUNK])
            pubs.append(p)
            addrs.append(d)
            sts.append(s)
    return np.concatenate(pubs), np.concatenate(addrs), np.concatenate(sts)


def test_tri_golden_recover(engine):
    g = load_golden("recover.npz")
    engine.diag_counters(reset=True)
    pub, addr, st = _recover_chunks(engine, g["msg"], g["sig"], TRI)
    d = engine.diag_counters(reset=True)
    assert d["lat_tri"] == -(-len(g["msg"]) // CHUNK), d
    names = list(g["kind_names"])
    bad = np.nonzero(st != g["status"])[0]
    assert bad.size == 0, [(int(i), names[g["kind"][i]], int(st[i]), int(g["status"][i])) for i in bad[:20]]
    assert np.array_equal(pub, g["pub"])
    pub2, addr2, st2 = _recover_chunks(engine, g["msg"], g["sig"], NARROW)
    assert engine.diag_counters(reset=True)["lat_tri"] == 0
    assert np.array_equal(addr, addr2) and np.array_equal(st, st2) and np.array_equal(pub, pub2)


def test_tri_golden_sender(engine):
    g = load_golden("sender.npz")
    keys = sorted(set(zip(g["signer"].tolist(), g["chain_id"].tolist())))
    engine.diag_counters(reset=True)
    for signer, cid in keys:
        sel = np.nonzero((g["signer"] == signer) & (g["chain_id"] == cid))[0]
        for a in range(0, len(sel), CHUNK):
            s = sel[a:a + CHUNK]
            with knobs(engine, TRI):
                addr, st = engine.sender_batch(g["sighash"][s], g["r"][s], g["s"][s], g["v"][s], g["vflags"][s],
                                               signer, cid)
            assert np.array_equal(st, g["status"][s]) and np.array_equal(addr, g["addr"][s]), (signer, cid)
    assert engine.diag_counters(reset=True)["lat_tri"] >= len(keys)


@pytest.mark.parametrize("n", [257, 511, 1000])
def test_tri_sizes_against_lane_serial(engine, n):
    msg, sig, exp = engine.synth_sign_dev(7_000_000 + n, n, 0)
    m, s, e = msg.cpu().numpy(), sig.cpu().numpy(), exp.cpu().numpy()
    engine.diag_counters(reset=True)
    with knobs(engine, TRI):
        pub, addr, st = engine.ecrecover_batch(m, s)
    assert engine.diag_counters(reset=True)["lat_tri"] == 1
    assert (st == 0).all() and np.array_equal(addr, e)
    with knobs(engine, LANE):
        pub2, _, _ = engine.ecrecover_batch(m, s)
    assert np.array_equal(pub, pub2)


def test_tri_wire_form(engine):
    """wire-format Geec transactions through the three-wave form (in-kernel decode + sighash)"""
    import torch

    from eges_amd import txs
    n = 600
    h = txs.c1_sighashes(0, n)
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(h).cuda(), 0)
    torch.cuda.synchronize()
    sig_h, exp = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    packed = engine.pack_raw(txs.c1_raw(0, sig_h))
    engine.diag_counters(reset=True)
    with knobs(engine, TRI):
        addr, st, hs = engine.sender_raw_batch(packed, _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID, want_sighash=True)
    assert engine.diag_counters(reset=True)["lat_tri"] == 1
    assert (st == 0).all() and np.array_equal(addr, exp)
    assert np.array_equal(hs, h)


def test_tri_forced_redo_and_root_fallback_golden(engine):
    """EGES_TEST_FORCE_REDO (every exact redo pass: both R' loops, D's loop, the comb) and
    EGES_TEST_ROOT_HELPERS=0 (every wave computes its own root): golden outputs unchanged."""
    g = load_golden("recover.npz")
    engine.diag_counters(reset=True)
    pub, addr, st = _recover_chunks(engine, g["msg"], g["sig"], dict(TRI, EGES_TEST_FORCE_REDO=1))
    d = engine.diag_counters(reset=True)
    assert np.array_equal(st, g["status"]) and np.array_equal(pub, g["pub"])
    assert d["lat_redo"] > 0 and d["comb_redo"] > 0 and d["lat_tri"] > 0, d
    pub, addr, st = _recover_chunks(engine, g["msg"], g["sig"], dict(TRI, EGES_TEST_ROOT_HELPERS=0))
    assert np.array_equal(st, g["status"]) and np.array_equal(pub, g["pub"])
    engine.diag_counters(reset=True)


@pytest.mark.parametrize("flag", [0, 2, 4])  # F_DIG, F_G, F_HI
def test_tri_skipped_flag_faults_one_item(engine, flag):
    g = load_golden("recover.npz")
    n = 300
    msg, sig = np.ascontiguousarray(g["msg"][:n]), np.ascontiguousarray(g["sig"][:n])
    pub = np.full((n, 65), 0xAB, np.uint8)
    addr = np.full((n, 20), 0xAB, np.uint8)
    st = np.full(n, 0xEE, np.uint8)
    P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    engine.diag_counters(reset=True)
    with knobs(engine, dict(TRI, EGES_TEST_SKIP_FLAG=flag + 1)):
        rc = _lib.lib.eges_ecrecover_batch(P(msg), P(sig), n, P(pub), P(addr), P(st))
    assert rc == -3  # EGES_E_HIP
    assert st[0] == _lib.ENGINE_FAULT and not pub[0].any() and not addr[0].any()
    assert np.array_equal(st[1:], g["status"][1:n]) and np.array_equal(pub[1:], g["pub"][1:n])
    assert engine.diag_counters(reset=True)["handoff"] >= 1
    with knobs(engine, TRI):
        p2, _, s2 = engine.ecrecover_batch(msg, sig)
    assert np.array_equal(s2, g["status"][:n]) and np.array_equal(p2, g["pub"][:n])
