"""Concurrent callers through the C-ABI (SURVEY §8(b) threading contract).

The reference calls one read-only libsecp256k1 context from any goroutine with no locks
(crypto/secp256k1/secp256.go:45-52). libeges must give the same answers when several host
threads call its batch and single-item entries at once (ctypes releases the GIL for the
call). Every result is checked bit-exactly against the golden fixtures.
"""
import ctypes
import threading

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


def test_concurrent_batch_and_single_item_callers(engine):
    from eges_amd._lib import lib
    g = load_golden("recover.npz")
    msg, sig, exp_pub, exp_st = g["msg"], g["sig"], g["pub"], g["status"]
    n = msg.shape[0]
    errors = []

    def batch_worker(t):
        try:
            for rep in range(3):
                lo = (t * 397 + rep * 131) % n
                sel = np.arange(lo, lo + 700) % n  # ragged, wraps around the fixture
                pub, _, st = engine.ecrecover_batch(msg[sel], sig[sel])
                if not np.array_equal(st, exp_st[sel]) or not np.array_equal(pub, exp_pub[sel]):
                    errors.append(("batch", t, rep))
        except Exception as e:  # surfaced in the main thread
            errors.append(("batch-exc", t, repr(e)))

    def single_worker(t):
        try:
            out = (ctypes.c_ubyte * 65)()
            for i in range(t, n, 97):
                m = msg[i].tobytes()
                s = sig[i].tobytes()
                if s[64] >= 4:
                    continue  # checkSignature rejects these before the C call (secp256.go:171-179)
                rc = lib.eges_ecdsa_recover(out, s, m)
                want = 1 if exp_st[i] == 0 else 0
                if rc != want or (rc == 1 and bytes(out) != exp_pub[i].tobytes()):
                    errors.append(("single", t, i, rc))
        except Exception as e:
            errors.append(("single-exc", t, repr(e)))

    threads = [threading.Thread(target=batch_worker, args=(t,)) for t in range(4)]
    threads += [threading.Thread(target=single_worker, args=(t,)) for t in range(4)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a caller thread did not return"
    assert not errors, errors[:10]


def test_coalesced_single_item_callers(engine):
    """8 threads x 2000 single eges_ecdsa_recover calls (the reference's per-goroutine
    secp256k1_ext_ecdsa_recover, ext.h:30-47): coalesced into shared batches (single.hip
    Coalescer), every result bit-exact against the golden fixture. Rates printed for the record."""
    import time
    from eges_amd._lib import lib
    g = load_golden("recover.npz")
    msg, sig, exp_pub, exp_st = g["msg"], g["sig"], g["pub"], g["status"]
    idx = [i for i in range(msg.shape[0]) if sig[i, 64] < 4]  # checkSignature filters recid >= 4 in Go
    per_thread, nthreads = 2000, 8
    errors = []
    lat = []

    def worker(t):
        out = (ctypes.c_ubyte * 65)()
        try:
            for k in range(per_thread):
                i = idx[(t * 7919 + k * 31) % len(idx)]
                t0 = time.perf_counter()
                rc = lib.eges_ecdsa_recover(out, sig[i].tobytes(), msg[i].tobytes())
                if t == 0:
                    lat.append(time.perf_counter() - t0)
                want = 1 if exp_st[i] == 0 else 0
                if rc != want or (rc == 1 and bytes(out) != exp_pub[i].tobytes()):
                    errors.append((t, k, i, rc))
        except Exception as e:
            errors.append(("exc", t, repr(e)))

    # single caller first (p50 latency of one call), then 8 concurrent callers
    one = (ctypes.c_ubyte * 65)()
    ts = []
    for k in range(200):
        i = idx[k % len(idx)]
        t0 = time.perf_counter()
        lib.eges_ecdsa_recover(one, sig[i].tobytes(), msg[i].tobytes())
        ts.append(time.perf_counter() - t0)
    threads = [threading.Thread(target=worker, args=(t,)) for t in range(nthreads)]
    t0 = time.perf_counter()
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=200)
    dt = time.perf_counter() - t0
    assert not any(th.is_alive() for th in threads), "a caller thread did not return"
    assert not errors, errors[:10]
    print(f"\nsingle eges_ecdsa_recover p50 {np.median(ts[20:]) * 1e3:.3f} ms (one caller); "
          f"{nthreads} callers x {per_thread}: {nthreads * per_thread / dt:.0f} recoveries/s, "
          f"p50 {np.median(lat) * 1e3:.3f} ms per call")


def test_coalesced_recover_and_verify_many_callers(engine):
    """24 threads at once, 12 through eges_ecdsa_recover and 12 through eges_ecdsa_verify (the
    reference's ext.h:30-47 / :58-75 per-call seams): both coalescers share the device's lanes,
    more callers than the coalescer lets spin (single.hip EGES_COALESCE_SPINNERS), so the blocking
    path runs too. Every result against the golden fixtures (recover.npz, verify.npz)."""
    from eges_amd._lib import lib
    gr = load_golden("recover.npz")
    gv = load_golden("verify.npz")
    ridx = [i for i in range(gr["msg"].shape[0]) if gr["sig"][i, 64] < 4]
    errors = []

    def rec_worker(t):
        out = (ctypes.c_ubyte * 65)()
        try:
            for k in range(300):
                i = ridx[(t * 4099 + k * 37) % len(ridx)]
                rc = lib.eges_ecdsa_recover(out, gr["sig"][i].tobytes(), gr["msg"][i].tobytes())
                want = 1 if gr["status"][i] == 0 else 0
                if rc != want or (rc == 1 and bytes(out) != gr["pub"][i].tobytes()):
                    errors.append(("recover", t, k, i, rc))
        except Exception as e:
            errors.append(("recover-exc", t, repr(e)))

    def ver_worker(t):
        try:
            n = gv["msg"].shape[0]
            for k in range(300):
                i = (t * 577 + k * 13) % n
                plen = int(gv["publen"][i])
                rc = lib.eges_ecdsa_verify(gv["sig"][i].tobytes(), gv["msg"][i].tobytes(), gv["pub"][i][:plen].tobytes(),
                                           plen)
                if rc != int(gv["ok"][i]):
                    errors.append(("verify", t, k, i, rc, int(gv["ok"][i])))
        except Exception as e:
            errors.append(("verify-exc", t, repr(e)))

    threads = [threading.Thread(target=rec_worker, args=(t,)) for t in range(12)]
    threads += [threading.Thread(target=ver_worker, args=(t,)) for t in range(12)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=150)
    assert not any(th.is_alive() for th in threads), "a caller thread did not return"
    assert not errors, errors[:10]


def test_concurrent_mid_size_callers(engine):
    """Host threads calling the mid-size band at once (round 6): batches of 24,000 (the bucket form
    at two workgroups per CU, its ring in the device workspace), 9,000 (one workgroup per CU) and
    3,000 signatures, gated host-buffer recover and VerifySignature calls, beside single-item
    callers on the resident server. The device workspace and the input gate are per device, so
    these calls must serialize on it without mixing; every result is checked against the
    synthetic signer's addresses (and the verify calls against all-valid / wrong-key rows)."""
    import torch
    from eges_amd._lib import lib
    n = 24_000
    msg_d, sig_d, addr_d = engine.synth_sign_dev(77 << 20, n, 0)
    pub_d = torch.empty((n, 65), dtype=torch.uint8, device="cuda")
    engine.ecrecover_batch_dev(msg_d, sig_d, pub=pub_d)
    torch.cuda.synchronize()
    msg, sig, exp, pub = (x.cpu().numpy() for x in (msg_d, sig_d, addr_d, pub_d))
    sig64 = np.ascontiguousarray(sig[:, :64])
    publen = np.full(n, 65, np.uint8)
    wrong = np.roll(pub, 1, axis=0)  # another signer's key: every item rejected
    errors = []

    def recover_worker(t):
        try:
            for rep, m in enumerate((24_000, 9_000, 3_000)):
                lo = (t * 1_009 + rep * 211) % (n - m + 1)
                sl = slice(lo, lo + m)
                _, addr, st = engine.ecrecover_batch(msg[sl], sig[sl], want_pub=False)
                if int(st.max()) != 0 or not np.array_equal(addr, exp[sl]):
                    errors.append(("recover", t, m, int((addr != exp[sl]).any(axis=1).sum())))
        except Exception as e:  # surfaced in the main thread
            errors.append(("recover-exc", t, repr(e)))

    def verify_worker(t):
        try:
            for rep, m in enumerate((20_000, 6_000)):
                lo = (t * 733 + rep * 97) % (n - m + 1)
                sl = slice(lo, lo + m)
                keys = pub if (t + rep) % 2 == 0 else wrong
                ok = engine.verify_batch(keys[sl], publen[sl], msg[sl], sig64[sl])
                want = 1 if keys is pub else 0
                if int((ok != want).sum()):
                    errors.append(("verify", t, m, int((ok != want).sum())))
        except Exception as e:
            errors.append(("verify-exc", t, repr(e)))

    def single_worker(t):
        try:
            out = (ctypes.c_ubyte * 65)()
            for i in range(t, 4_000, 37):
                rc = lib.eges_ecdsa_recover(out, sig[i].tobytes(), msg[i].tobytes())
                if rc != 1 or bytes(out) != pub[i].tobytes():
                    errors.append(("single", t, i, rc))
        except Exception as e:
            errors.append(("single-exc", t, repr(e)))

    threads = [threading.Thread(target=recover_worker, args=(t,)) for t in range(3)]
    threads += [threading.Thread(target=verify_worker, args=(t,)) for t in range(2)]
    threads += [threading.Thread(target=single_worker, args=(t,)) for t in range(2)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=110)
    assert not any(th.is_alive() for th in threads), "a caller thread did not return"
    assert not errors, errors[:10]
