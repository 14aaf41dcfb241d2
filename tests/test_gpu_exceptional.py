"""Exceptional sums (acc == +-P) forced through every kernel form and entry, pinned to the oracle,
with the engine's diagnostic counters showing which exact branch ran.

Reference: libsecp256k1 resolves a == b / a == -b inline (group_impl.h:414-461, doubling at
:440) inside ecmult (ecmult_impl.h:369-399); attacker-chosen (msg, r, s) reach it through the
EVM precompile (core/vm/contracts.go:78-101) and secp256k1_ext_ecdsa_recover (ext.h:30-47).

Which sums can be exceptional is pinned on CPU by tests/test_exceptional_model.py (the
R-table loops and the comb cannot meet one; R-part against G-part can). Here:
  - constructed inputs (tests/ecmodel.py recover_cases / verify_cases: R = rho G with rho known)
    reach the lane-serial loop's exact redo (window 0) and the latency forms' exact joins, both
    the doubling and the infinity branch, through batch, precompile and single-item entries;
  - EGES_TEST_FORCE_REDO runs every unchecked loop's exact redo on the golden sets (the redo
    code of the forms whose poisoning no input can cause), outputs byte for byte unchanged.
"""
import ctypes
import random

import numpy as np
import pytest

import ecmodel as M
from conftest import load_golden

pytestmark = pytest.mark.gpu

LAT_ALL = 1 << 20
FORMS = {  # knob settings per form (recovery / verification)
    "lane_serial": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 0},
    "narrow": {"EGES_LAT_MAX": LAT_ALL, "EGES_LAT_WIDE_MAX": 0, "EGES_LAT_TRI_MAX": 0},
    "split": {"EGES_LAT_MAX": LAT_ALL, "EGES_LAT_WIDE_MAX": LAT_ALL},
    # (recovery batches under the three-wave form's occupancy bound; verification runs narrow)
    "tri": {"EGES_LAT_MAX": LAT_ALL, "EGES_LAT_WIDE_MAX": 0, "EGES_LAT_TRI_MAX": LAT_ALL},
    "mid": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": LAT_ALL, "EGES_MID_FORM": 0},
    "mid_bucket": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": LAT_ALL, "EGES_MID_FORM": 2},
    # the bucket form at two workgroups per CU (ring and parts in the workspace; round 6)
    "mid_bucket2": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": LAT_ALL, "EGES_MID_FORM": 2, "EGES_BKT2": 2},
}


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


def _recover_inputs(seed=11, count=8):
    cases = M.recover_cases(random.Random(seed), count)
    msgs, sigs = [], []
    for kind, sign, rho, R, u1, u2 in cases:
        m, s = M.recover_input(rho, R, u1, u2)
        msgs.append(m)
        sigs.append(s)
    msg = np.frombuffer(b"".join(msgs), np.uint8).reshape(-1, 32)
    sig = np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 65)
    return cases, msg, sig


def _expected_recover(oracle, msg, sig):
    st, pub = [], []
    for i in range(len(msg)):
        s, p = oracle.recover_pubkey(msg[i].tobytes(), sig[i].tobytes())
        st.append(s)
        pub.append(p if s == 0 else bytes(65))
    return np.array(st, np.uint8), np.frombuffer(b"".join(pub), np.uint8).reshape(-1, 65)


def _check_model(cases, st, pub):
    """the oracle's outputs agree with the model's point u2 rho + u1 (the constructions are what
    they claim to be)"""
    for i, (kind, sign, rho, R, u1, u2) in enumerate(cases):
        q = (u2 * rho + u1) % M.N
        if q == 0:
            assert st[i] == 6, (i, kind)  # EGES_RECOVER_FAILED: Q at infinity
        else:
            Q = M.ec_mul(q)
            assert st[i] == 0 and pub[i].tobytes() == b"\x04" + Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big")


def test_recover_exceptional_sums_every_form(engine, oracle):
    cases, msg, sig = _recover_inputs()
    est, epub = _expected_recover(oracle, msg, sig)
    _check_model(cases, est, epub)
    assert (est == 6).any() and (est == 0).any()
    kinds = np.array([c[0] for c in cases])
    for form, kv in FORMS.items():
        engine.diag_counters(reset=True)
        with knobs(engine, kv):
            pub, addr, st = engine.ecrecover_batch(msg, sig)
        d = engine.diag_counters(reset=True)
        assert np.array_equal(st, est), (form, np.nonzero(st != est)[0])
        assert np.array_equal(pub, epub), form
        for i in np.nonzero(est == 0)[0]:
            assert addr[i].tobytes() == oracle.pub_to_addr(epub[i].tobytes())
        if form == "lane_serial":
            # window 0: the u1 G addition meets u2 R == +-u1 G, the wave redoes its loop exactly
            assert d["ls_redo"] > 0 and d["ls_exc"] > 0, d
        elif form == "mid":
            # the split1 / split2 constructions meet the windowed form's joins ((A + u1 G) + H, as split)
            assert d["mid_join"] > 0 and d["mid_redo"] == 0 and d["mid_exc"] == 0, d
        elif form in ("mid_bucket", "mid_bucket2"):
            # the ls / join constructions (u2 R == +-u1 G) meet the bucket form's final join
            assert d["mid_join"] > 0 and d["mid_redo"] == 0 and d["mid_exc"] == 0, d
        else:
            assert d["join_dbl"] > 0 and d["join_inf"] > 0, (form, d)
            assert d["lat_redo"] == 0 and d["comb_redo"] == 0 and d["lat_exc"] == 0, (form, d)
    # kinds split1 / split2 target the split (and windowed) form's joins; the three-wave form joins
    # (A + H) + u1 G and meets the "join" kind's branches
    assert {"ls", "join", "split1", "split2"} == set(kinds.tolist())


def test_recover_exceptional_sums_reference_lib(engine):
    """the same inputs through the reference libsecp256k1 (oracle/_ref, compiled in place)"""
    from oracle import RefLib, have_ref
    if not have_ref():
        pytest.skip("oracle/_ref not built")
    ref = RefLib()
    _, msg, sig = _recover_inputs()
    pub, addr, st = engine.ecrecover_batch(msg, sig)
    for i in range(len(msg)):
        ok, rpub = ref.ecrecover(msg[i].tobytes(), sig[i].tobytes())
        assert (st[i] == 0) == bool(ok), i
        if ok:
            assert pub[i].tobytes() == rpub, i


def test_precompile_and_single_item_exceptional(engine, oracle):
    """The attacker-facing entries: the EVM ECRECOVER precompile (both latency forms and the
    mid-size kernel) and the
    coalesced single-item secp256k1_ext_ecdsa_recover replacement."""
    from eges_amd._lib import lib
    cases, msg, sig = _recover_inputs(seed=12)
    est, epub = _expected_recover(oracle, msg, sig)
    inputs = [msg[i].tobytes() + bytes(31) + bytes([27 + sig[i, 64]]) + sig[i, :64].tobytes() for i in range(len(msg))]
    for form in ("narrow", "split", "mid", "mid_bucket", "mid_bucket2"):
        engine.diag_counters(reset=True)
        with knobs(engine, FORMS[form]):
            out, st = engine.ecrecover_precompile_batch(inputs)
        d = engine.diag_counters(reset=True)
        if form in ("mid", "mid_bucket", "mid_bucket2"):
            assert d["mid_join"] > 0, d
        else:
            assert d["join_dbl"] > 0 and d["join_inf"] > 0, (form, d)
        for i in range(len(msg)):
            if est[i] == 0:
                assert st[i] == 0 and out[i].tobytes() == bytes(12) + oracle.pub_to_addr(epub[i].tobytes()), (form, i)
            else:
                assert st[i] == 6 and not out[i].any(), (form, i)
    engine.diag_counters(reset=True)
    for i in range(len(msg)):
        out = (ctypes.c_ubyte * 65)()
        rc = lib.eges_ecdsa_recover(out, sig[i].tobytes(), msg[i].tobytes())
        assert rc == (1 if est[i] == 0 else 0), i
        if rc:
            assert bytes(out) == epub[i].tobytes(), i
    d = engine.diag_counters(reset=True)
    assert d["join_dbl"] + d["join_inf"] > 0, d


def test_verify_exceptional_sums_every_form(engine, oracle):
    from eges_amd._lib import lib
    cases = M.verify_cases(random.Random(13), 6)
    n = len(cases)
    pub = np.zeros((n, 65), np.uint8)
    msg = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    for i, (kind, sign, rho, p, m, s) in enumerate(cases):
        pub[i] = np.frombuffer(p, np.uint8)
        msg[i] = np.frombuffer(m, np.uint8)
        sig[i] = np.frombuffer(s, np.uint8)
    publen = np.full(n, 65, np.uint8)
    exp = np.array([oracle.verify(pub[i].tobytes(), msg[i].tobytes(), sig[i].tobytes()) for i in range(n)], np.uint8)
    assert exp.sum() >= 1  # valid signatures through the doubling branch
    for form, kv in FORMS.items():
        engine.diag_counters(reset=True)
        with knobs(engine, kv):
            ok = engine.verify_batch(pub, publen, msg, sig)
        d = engine.diag_counters(reset=True)
        assert np.array_equal(ok, exp), (form, np.nonzero(ok != exp)[0])
        if form == "lane_serial":
            assert d["ls_redo"] > 0 and d["ls_exc"] > 0, d
        elif form == "mid":  # (verification has no windowed mid-size form: lane-serial runs)
            assert d["ls_redo"] > 0 and d["ls_exc"] > 0, d
        elif form in ("mid_bucket", "mid_bucket2"):  # the bucket form's verify mode: the exact final join
            assert d["mid_join"] > 0 and d["mid_exc"] == 0, d
        else:
            assert d["join_dbl"] > 0 and d["join_inf"] > 0, (form, d)
    for i in range(n):
        assert lib.eges_ecdsa_verify(sig[i].tobytes(), msg[i].tobytes(), pub[i].tobytes(), 65) == exp[i], i


def test_forced_redo_every_form_golden(engine):
    """EGES_TEST_FORCE_REDO: every form runs its exact redo pass (the lane-serial loop, the R'
    loops, the split form's high loops, the comb) on every wave; the golden fixtures' outputs are
    unchanged byte for byte and the counters show each redo ran."""
    g = load_golden("recover.npz")
    gv = load_golden("verify.npz")
    for form, kv in FORMS.items():
        engine.diag_counters(reset=True)
        with knobs(engine, dict(kv, EGES_TEST_FORCE_REDO=1)):
            pub, addr, st = engine.ecrecover_batch(g["msg"], g["sig"])
            ok = engine.verify_batch(gv["pub"], gv["publen"], gv["msg"], gv["sig"])
        d = engine.diag_counters(reset=True)
        assert np.array_equal(st, g["status"]) and np.array_equal(pub, g["pub"]), form
        assert np.array_equal(ok, gv["ok"]), form
        if form == "lane_serial":
            assert d["ls_redo"] > 0, d
        elif form == "mid":
            assert d["mid_redo"] > 0 and d["ls_redo"] > 0, d  # recovery: mid-size; verification: lane-serial
        elif form in ("mid_bucket", "mid_bucket2"):
            assert d["mid_redo"] > 0, d  # recovery and verification both on the bucket form
        else:
            assert d["lat_redo"] > 0 and d["comb_redo"] > 0, (form, d)
