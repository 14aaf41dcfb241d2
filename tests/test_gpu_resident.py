"""The resident single-call server (single.hip Resident, k_recover_lat.hip lat_resident_kernel):
coalesced eges_ecdsa_recover / eges_ecdsa_verify groups go to split-form workgroups that stay
resident and poll a job word in coherent pinned memory instead of a launch per call. Every golden
item through it against the fixtures; device-wide calls between (the server stops first and
restarts on the next call); idle exits and restarts; the server switched off. EGES_DIAG_RESIDENT
counts the jobs it served. (Round 4's resident block server measured slower and was removed in
round 5.)"""
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
    with knobs(engine, {"EGES_RESIDENT": 1, "EGES_RESIDENT_IDLE_US": 4000}):
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


def test_resident_idle_window_and_another_process(engine):
    """the resident server's workgroups keep polling for EGES_RESIDENT_IDLE_US
    after a call, on CUs another process may want. A second process launches a 1M batch right
    after this process's single call (the server alive for EGES_RESIDENT_IDLE_US, 0.5 ms by default)
    and after the same call on a lane (no server), alternating. ADVICE r5: the server's liveness at
    each launch request is recorded (eges_diag_resident_running) and must have been seen, so the
    'alive' case did overlap the other kernel; the slowdown is reported (bench.py carries it as
    secondary.single.resident_tax) and only guarded loosely here (< 10 % in the median: the
    server's 16 workgroups hold 16 of the 512 resident recover blocks' places for at most the idle
    window), so clock noise on a shared box cannot fail the suite."""
    import os
    import subprocess
    import sys
    g = load_golden("recover.npz")
    i = int(np.nonzero((g["status"] == 0) & (g["sig"][:, 64] < 4))[0][0])
    here = os.path.dirname(os.path.abspath(__file__))
    child = subprocess.Popen([sys.executable, "-u", os.path.join(here, "gpu_child.py"), "other_process_kernels"],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        assert child.stdout.readline().strip() == "ready"

        def other(with_server):
            # the same sequence either way (one single call, then the other process's launch at
            # once), so both see the same GPU clock state; only whether the server is alive differs
            engine.set_knob("EGES_RESIDENT", 1 if with_server else 0)
            rc, _ = _single_recover(g["msg"][i], g["sig"][i])
            assert rc == 1
            if with_server:
                alive.append(_lib.lib.eges_diag_resident_running(0) == 1)
            child.stdin.write("go\n")
            child.stdin.flush()
            return float(child.stdout.readline())

        with knobs(engine, {"EGES_RESIDENT": 1}):
            on, off, alive = [], [], []
            for _ in range(8):
                time.sleep(0.02)  # (the previous server idles out first)
                on.append(other(True))
                time.sleep(0.02)
                off.append(other(False))
        child.stdin.close()
        out = child.stdout.read()
        assert child.wait(timeout=60) == 0 and '"ok": true' in out, out
    finally:
        if child.poll() is None:
            child.kill()
    m_on, m_off = float(np.median(on)), float(np.median(off))
    print(f"other process 1M kernel: server alive {m_on:.3f} ms, stopped {m_off:.3f} ms, "
          f"server running at {sum(alive)}/{len(alive)} launch requests")
    assert sum(alive) >= len(alive) // 2, alive
    assert m_on <= 1.10 * m_off, (on, off)
