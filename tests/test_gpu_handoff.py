"""Bounded, reporting hand-offs between the waves of a workgroup (handoff.cuh).

The mid-size kernel (both forms) and the latency kernels' split form pass results between their
waves through LDS flags and counters. A test-only knob (EGES_TEST_SKIP_FLAG = k + 1) makes the
first workgroup's producer of flag k skip publishing it once per launch: its consumers must time
out (about a second), the workgroup's items must come back as EGES_ENGINE_FAULT with no address,
the host-buffer call must fail with EGES_E_HIP, EGES_DIAG_HANDOFF must count it, every other
item must still be exact, and the next call (knob reset) must be exact again.

Flag indices (k_recover_mid.hip / k_recover_lat.hip enums): bucket form BF_DIG 0, BF_Y 1,
BF_G 2, BF_Q2 3, BF_PARSED 7, BF_STAGE_FREE 8, BF_A1 12; windowed form MF_DIG 0, MF_HB 3;
latency split form F_DIG 0, F_HI 4."""
import ctypes

import numpy as np
import pytest

from conftest import load_golden
from eges_amd import _lib

pytestmark = pytest.mark.gpu

BUCKET = {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2}
WINDOWED = dict(BUCKET, EGES_MID_FORM=0)
BUCKET2 = dict(BUCKET, EGES_BKT2=2)  # two workgroups per CU, ring in the workspace (round 6)
SPLIT = {"EGES_LAT_MAX": 1 << 20, "EGES_LAT_WIDE_MAX": 1 << 20}


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


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _recover_raw(msg, sig):
    """eges_ecrecover_batch without the raising wrapper: (rc, pub, addr, status)."""
    n = msg.shape[0]
    pub = np.full((n, 65), 0xAB, np.uint8)
    addr = np.full((n, 20), 0xAB, np.uint8)
    st = np.full(n, 0xEE, np.uint8)
    rc = _lib.lib.eges_ecrecover_batch(_p(msg), _p(sig), n, _p(pub), _p(addr), _p(st))
    return rc, pub, addr, st


def _check_fault(engine, form, flag, n_fault, golden="recover.npz", n=None):
    g = load_golden(golden)
    msg, sig = np.ascontiguousarray(g["msg"]), np.ascontiguousarray(g["sig"])
    if n is not None:
        msg, sig = msg[:n].copy(), sig[:n].copy()
    exp_st, exp_pub = g["status"][:len(msg)], g["pub"][:len(msg)]
    engine.diag_counters(reset=True)
    with knobs(engine, dict(form, EGES_TEST_SKIP_FLAG=flag + 1)):
        rc, pub, addr, st = _recover_raw(msg, sig)
    assert rc == -3, rc  # EGES_E_HIP
    assert "hand-off" in _lib.lib.eges_last_error().decode()
    assert (st[:n_fault] == _lib.ENGINE_FAULT).all(), st[:n_fault]
    assert not pub[:n_fault].any() and not addr[:n_fault].any()
    assert np.array_equal(st[n_fault:], exp_st[n_fault:])
    assert np.array_equal(pub[n_fault:], exp_pub[n_fault:])
    assert engine.diag_counters()["handoff"] >= 1
    # the knob is back to 0: the same call is exact again
    with knobs(engine, form):
        rc, pub, addr, st = _recover_raw(msg, sig)
    assert rc == 0
    assert np.array_equal(st, exp_st) and np.array_equal(pub, exp_pub)
    assert engine.diag_counters(reset=True)["handoff"] >= 1  # (only the faulted call counted)


@pytest.mark.parametrize("flag", [0, 2, 3, 12])
def test_bucket_form_skipped_flag_faults_one_workgroup(engine, flag):
    _check_fault(engine, BUCKET, flag, 64)


@pytest.mark.parametrize("flag", [0, 2, 3, 12])
def test_bucket2_form_skipped_flag_faults_one_workgroup(engine, flag):
    _check_fault(engine, BUCKET2, flag, 64)


@pytest.mark.parametrize("flag", [0, 3])
def test_windowed_form_skipped_flag_faults_one_workgroup(engine, flag):
    _check_fault(engine, WINDOWED, flag, 64)


@pytest.mark.parametrize("flag", [0, 4])
def test_latency_split_form_skipped_flag_faults_one_item(engine, flag):
    _check_fault(engine, SPLIT, flag, 1, n=48)


@pytest.mark.parametrize("flag", [7, 8])
def test_bucket_wire_form_skipped_flag_faults_one_workgroup(engine, flag):
    """wire-format batches in the bucket form (S decodes, X reads R from the LDS stage)"""
    import torch
    from eges_amd import txs
    n = 300
    h = txs.c1_sighashes(0, n)
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(h).cuda(), 0)
    torch.cuda.synchronize()
    sig_h, exp = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    raw, off = engine.pack_raw(txs.c1_raw(0, sig_h))
    addr = np.full((n, 20), 0xAB, np.uint8)
    st = np.full(n, 0xEE, np.uint8)
    form = dict(BUCKET, EGES_WIRE_FUSED=1)
    with knobs(engine, dict(form, EGES_TEST_SKIP_FLAG=flag + 1)):
        rc = _lib.lib.eges_sender_raw_batch(_p(raw), _p(off), n, _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID, _p(addr), _p(st),
                                            None)
    assert rc == -3
    assert (st[:64] == _lib.ENGINE_FAULT).all() and not addr[:64].any()
    assert (st[64:] == 0).all() and np.array_equal(addr[64:], exp[64:])
    with knobs(engine, form):
        a2, s2, _ = engine.sender_raw_batch((raw, off), _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID)
    assert (s2 == 0).all() and np.array_equal(a2, exp)
    engine.diag_counters(reset=True)


def test_bucket_wire_form_delayed_x_keeps_the_stage(engine):
    """in the bucket form's wire path wave S's u1 G part shares LDS with the staged
    encodings wave X reads R from. EGES_TEST_DELAY_X holds every X wave back ~0.7 ms before that
    read, long after S would otherwise have written its part: S must wait for X's first published
    point (the stage's release), so every address stays exact."""
    import torch
    from eges_amd import txs
    n = 2000
    h = txs.c1_sighashes(0, n)
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(h).cuda(), 0)
    torch.cuda.synchronize()
    sig_h, exp = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    packed = engine.pack_raw(txs.c1_raw(0, sig_h))
    engine.diag_counters(reset=True)
    with knobs(engine, dict(BUCKET, EGES_WIRE_FUSED=1, EGES_TEST_DELAY_X=200)):
        a, s_, _ = engine.sender_raw_batch(packed, _lib.SIGNER_EIP155, txs.GEEC_CHAIN_ID)
    assert (s_ == 0).all() and np.array_equal(a, exp)
    assert engine.diag_counters(reset=True)["handoff"] == 0


def test_verify_split_form_skipped_flag_faults_one_item(engine):
    g = load_golden("verify.npz")
    n = 40
    pub, publen, msg, sig = (np.ascontiguousarray(g[k][:n]) for k in ("pub", "publen", "msg", "sig"))
    ok = np.full(n, 0xEE, np.uint8)
    with knobs(engine, dict(SPLIT, EGES_TEST_SKIP_FLAG=1)):
        rc = _lib.lib.eges_verify_batch(_p(pub), _p(publen), _p(msg), _p(sig), n, _p(ok))
    assert rc == -3
    assert "hand-off" in _lib.lib.eges_last_error().decode()
    assert ok[0] == 0  # (ok stays 0 / 1; the call's error and EGES_DIAG_HANDOFF say why)
    assert np.array_equal(ok[1:], g["ok"][1:n])
    with knobs(engine, SPLIT):
        assert np.array_equal(engine.verify_batch(pub, publen, msg, sig), g["ok"][:n])
    engine.diag_counters(reset=True)


@pytest.mark.parametrize("two", [False, True])
def test_verify_bucket_form_skipped_flag_faults_one_workgroup(engine, two):
    """the bucket form's VerifySignature mode (one and two workgroups per CU): a skipped digit flag
    faults workgroup 0's items"""
    g = load_golden("verify.npz")
    n = 300
    rep = -(-n // len(g["pub"]))
    pub, publen, msg, sig, exp = (np.ascontiguousarray(np.concatenate([g[k]] * rep)[:n])
                                  for k in ("pub", "publen", "msg", "sig", "ok"))
    ok = np.full(n, 0xEE, np.uint8)
    with knobs(engine, dict(BUCKET2 if two else BUCKET, EGES_TEST_SKIP_FLAG=1)):
        rc = _lib.lib.eges_verify_batch(_p(pub), _p(publen), _p(msg), _p(sig), n, _p(ok))
    assert rc == -3
    assert (ok[:64] == 0).all()
    assert np.array_equal(ok[64:], exp[64:])
    engine.diag_counters(reset=True)


@pytest.mark.parametrize("form", ["split", "bucket"])
def test_verify_dev_fault_is_never_truthy(engine, form):
    """the device-resident VerifySignature entry returns without a sync, so a faulted
    item must not reach the caller as a nonzero ok byte: it is 0, and EGES_DIAG_HANDOFF counts it"""
    import torch
    g = load_golden("verify.npz")
    n = 40 if form == "split" else 300
    rep = -(-n // len(g["pub"]))
    cols = [np.ascontiguousarray(np.concatenate([g[k]] * rep)[:n]) for k in ("pub", "publen", "msg", "sig", "ok")]
    pub, publen, msg, sig, exp = cols
    nf = 1 if form == "split" else 64
    assert exp[:nf].any()  # some of the faulted items are valid signatures
    d = [torch.from_numpy(x).cuda() for x in (pub, publen, msg, sig)]
    ok = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    engine.diag_counters(reset=True)
    with knobs(engine, dict(SPLIT if form == "split" else BUCKET, EGES_TEST_SKIP_FLAG=1)):
        engine.verify_batch_dev(*d, ok=ok)
        torch.cuda.synchronize()
    got = ok.cpu().numpy()
    assert set(np.unique(got).tolist()) <= {0, 1}
    assert not got[:nf].any() and np.array_equal(got[nf:], exp[nf:])
    assert engine.diag_counters(reset=True)["handoff"] >= 1
