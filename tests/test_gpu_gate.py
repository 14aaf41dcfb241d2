"""Host-buffer calls that launch before their inputs are copied (EGES_GATE = 1, the default:
hostpath.hip run_host_shard GateOpen, handoff.cuh gate_wait / gate_done): the fused mid-size kernels
(bucket, windowed) wait at the call's gate word while the host copies the inputs into the pinned
buffer, and their last workgroup stores the completion word the host waits on. The latency forms
run ungated either way (measured slower gated). Every golden recovery and sender item through
each form with the gate on and off, byte for byte the fixtures, and many back-to-back calls of
changing sizes across the routes (the gate's sequence advancing per call)."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

FORMS = {
    "narrow": {"EGES_LAT_MAX": 1 << 20, "EGES_LAT_WIDE_MAX": 0, "EGES_LAT_TRI_MAX": 0},
    "tri": {"EGES_LAT_MAX": 1 << 20, "EGES_LAT_WIDE_MAX": 0, "EGES_LAT_TRI_MAX": 1 << 20},
    "split": {"EGES_LAT_MAX": 1 << 20, "EGES_LAT_WIDE_MAX": 1 << 20},
    "bucket": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2},
    "windowed": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 0},
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


@pytest.mark.parametrize("form", sorted(FORMS))
@pytest.mark.parametrize("gate", [1, 0])
def test_gate_recover_and_sender_golden(engine, form, gate):
    g = load_golden("recover.npz")
    gs = load_golden("sender.npz")
    with knobs(engine, dict(FORMS[form], EGES_GATE=gate, EGES_RESIDENT=0)):
        pub, addr, st = engine.ecrecover_batch(g["msg"], g["sig"])
        assert np.array_equal(st, g["status"]) and np.array_equal(pub, g["pub"]), form
        for signer, cid in sorted(set(zip(gs["signer"].tolist(), gs["chain_id"].tolist()))):
            sel = np.nonzero((gs["signer"] == signer) & (gs["chain_id"] == cid))[0]
            a, s_ = engine.sender_batch(gs["sighash"][sel], gs["r"][sel], gs["s"][sel], gs["v"][sel],
                                        gs["vflags"][sel], int(signer), int(cid))
            assert np.array_equal(s_, gs["status"][sel]) and np.array_equal(a, gs["addr"][sel]), (form, signer, cid)


def test_gate_back_to_back_sizes(engine):
    """300 calls whose sizes walk across the split / three-wave / narrow / mid-size routes, each
    checked: a stale gate or input from the previous call would show as a wrong item"""
    g = load_golden("recover.npz")
    n_all = len(g["msg"])
    rng = np.random.default_rng(7)
    with knobs(engine, {"EGES_GATE": 1, "EGES_RESIDENT": 0}):
        for rep in range(300):
            n = int(rng.choice([1, 2, 17, 200, 300, 449, 1000, 1536, 2500]))
            sel = (np.arange(n) + rep * 131) % n_all
            pub, addr, st = engine.ecrecover_batch(g["msg"][sel], g["sig"][sel])
            assert np.array_equal(st, g["status"][sel]) and np.array_equal(pub, g["pub"][sel]), (rep, n)
