"""The latency kernels (k_recover_lat.hip: one signature per wave, recover and verify) against the
throughput kernels and the golden fixtures. Batches up to EGES_LAT_MAX signatures take the latency kernel;
EGES_LAT_MAX=0 (eges_test_set_knob) forces the lane-serial kernel, so every
case runs both ways and must agree byte for byte, and with the reference-generated fixtures."""
import time

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


class env_knob:
    """Sets engine knobs (eges_test_set_knob; the engine reads no environment after init) for
    the duration of a with-block."""

    def __init__(self, v):
        self.kv = self.knobs(v)

    def __enter__(self):
        import eges_amd
        self.old = {k: eges_amd.get_knob(k) for k in self.kv}
        for k, v in self.kv.items():
            eges_amd.set_knob(k, v)

    def __exit__(self, *a):
        import eges_amd
        for k, v in self.old.items():
            eges_amd.set_knob(k, v)


class lat_max(env_knob):
    """batches up to v take the latency kernels; lat_max(0) forces the lane-serial kernel (the
    mid-size kernel, k_recover_mid.hip, is switched off too; tests/test_gpu_mid.py covers it)"""

    @staticmethod
    def knobs(v):
        return {"EGES_LAT_MAX": v} if v else {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 0}


class wide_max(env_knob):  # latency batches up to this size use the split (4-wave) form; wide_max(0): narrow
    @staticmethod
    def knobs(v):
        return {"EGES_LAT_WIDE_MAX": v} if v else {"EGES_LAT_WIDE_MAX": 0, "EGES_LAT_TRI_MAX": 0}


class root_helpers(env_knob):  # 0: the narrow form launches no root-helper workgroups
    @staticmethod
    def knobs(v):
        return {"EGES_TEST_ROOT_HELPERS": v}


def test_wide_kernel_golden_recover(engine):
    """Every golden recovery item (all reject classes) through the split form, the narrow form
    and the lane-serial kernel: byte for byte the same, and the fixtures'."""
    g = load_golden("recover.npz")
    with lat_max(1 << 20), wide_max(1 << 20):
        pub, addr, st = engine.ecrecover_batch(g["msg"], g["sig"])
    names = list(g["kind_names"])
    bad = np.nonzero(st != g["status"])[0]
    assert bad.size == 0, [(int(i), names[g["kind"][i]], int(st[i]), int(g["status"][i])) for i in bad[:20]]
    assert np.array_equal(pub, g["pub"])
    with lat_max(1 << 20), wide_max(0):
        pub2, addr2, st2 = engine.ecrecover_batch(g["msg"], g["sig"])
    assert np.array_equal(pub, pub2) and np.array_equal(addr, addr2) and np.array_equal(st, st2)
    g2 = load_golden("sender.npz")
    keys = sorted(set(zip(g2["signer"].tolist(), g2["chain_id"].tolist())))
    for signer, cid in keys:
        sel = np.nonzero((g2["signer"] == signer) & (g2["chain_id"] == cid))[0]
        with lat_max(1 << 20), wide_max(1 << 20):
            a, s_ = engine.sender_batch(g2["sighash"][sel], g2["r"][sel], g2["s"][sel], g2["v"][sel],
                                        g2["vflags"][sel], signer, cid)
        assert np.array_equal(s_, g2["status"][sel]) and np.array_equal(a, g2["addr"][sel])


def test_lat_kernel_golden_recover(engine):
    g = load_golden("recover.npz")
    with lat_max(1 << 20):
        pub, addr, st = engine.ecrecover_batch(g["msg"], g["sig"])
    names = list(g["kind_names"])
    bad = np.nonzero(st != g["status"])[0]
    assert bad.size == 0, [(int(i), names[g["kind"][i]], int(st[i]), int(g["status"][i])) for i in bad[:20]]
    assert np.array_equal(pub, g["pub"])
    with lat_max(0):
        pub2, addr2, st2 = engine.ecrecover_batch(g["msg"], g["sig"])
    assert np.array_equal(addr, addr2) and np.array_equal(st, st2)




def test_narrow_root_fetch_fallback_golden(engine):
    """The narrow form's R.y normally comes from its lane-serial root-helper workgroups
    (k_recover_lat.hip root_helper / root_fetch). Without them every signature wave waits out
    root_fetch's bound and takes its own-root path: every golden item must still match the
    fixtures byte for byte (and the helper path's result)."""
    g = load_golden("recover.npz")
    with lat_max(1 << 20), wide_max(0):
        pub, addr, st = engine.ecrecover_batch(g["msg"], g["sig"])
        with root_helpers(0):
            pub2, addr2, st2 = engine.ecrecover_batch(g["msg"], g["sig"])
    assert np.array_equal(st, g["status"]) and np.array_equal(pub, g["pub"])
    assert np.array_equal(pub, pub2) and np.array_equal(addr, addr2) and np.array_equal(st, st2)


def test_lat_kernel_golden_sender(engine):
    g = load_golden("sender.npz")
    keys = sorted(set(zip(g["signer"].tolist(), g["chain_id"].tolist())))
    for signer, cid in keys:
        sel = np.nonzero((g["signer"] == signer) & (g["chain_id"] == cid))[0]
        with lat_max(1 << 20):
            addr, st = engine.sender_batch(g["sighash"][sel], g["r"][sel], g["s"][sel], g["v"][sel], g["vflags"][sel],
                                           signer, cid)
        assert np.array_equal(st, g["status"][sel]) and np.array_equal(addr, g["addr"][sel])


def test_lat_verify_golden(engine):
    """VerifySignature's 591 golden items (every key encoding and reject class) through the
    verify latency kernel and through the lane-serial verify kernel."""
    g = load_golden("verify.npz")
    names = list(g["kind_names"])
    with lat_max(1 << 20):
        ok = engine.verify_batch(g["pub"], g["publen"], g["msg"], g["sig"])
    bad = np.nonzero(ok != g["ok"])[0]
    assert bad.size == 0, [(int(i), names[g["kind"][i]], int(ok[i]), int(g["ok"][i])) for i in bad[:20]]
    with lat_max(0):
        ok2 = engine.verify_batch(g["pub"], g["publen"], g["msg"], g["sig"])
    assert np.array_equal(ok, ok2)
    with lat_max(1 << 20), wide_max(1 << 20):
        ok3 = engine.verify_batch(g["pub"], g["publen"], g["msg"], g["sig"])
    assert np.array_equal(ok, ok3)


@pytest.mark.parametrize("n", [1, 3, 64, 1000])
def test_lat_verify_sizes(engine, n):
    """Synthetic signatures, compressed and uncompressed keys, every 3rd message altered; both
    kernels agree and match the construction."""
    import torch
    msg, sig, _ = engine.synth_sign_dev(52_000 + n, n, 0)
    torch.cuda.synchronize()
    mh, sh = msg.cpu().numpy(), sig.cpu().numpy()
    pub, _, st = engine.ecrecover_batch(mh, sh)
    assert (st == 0).all()
    pk = pub.copy()
    lens = np.full(n, 65, np.uint8)
    comp = np.arange(n) % 2 == 1  # odd items as 33-byte keys
    pk[comp, 0] = 2 + (pub[comp, 64] & 1)
    pk[comp, 33:] = 0
    lens[comp] = 33
    mm = mh.copy()
    mm[::3, 0] ^= 1
    with lat_max(1 << 20):
        ok = engine.verify_batch(pk, lens, mm, sh[:, :64])
    with lat_max(0):
        ok2 = engine.verify_batch(pk, lens, mm, sh[:, :64])
    with lat_max(1 << 20), wide_max(1 << 20):
        ok3 = engine.verify_batch(pk, lens, mm, sh[:, :64])
    assert np.array_equal(ok, ok2) and np.array_equal(ok, ok3)
    assert ok.tolist() == [0 if i % 3 == 0 else 1 for i in range(n)]


@pytest.mark.parametrize("n", [1, 2, 15, 16, 17, 1000, 4097])
def test_lat_kernel_sizes_and_adversarial(engine, n):
    """Ragged sizes around the 16-signature block, C3's 1000, and the adversarial mix's classes."""
    import torch
    from eges_amd import workloads
    msg, sig, exp = engine.synth_sign_dev(31_000 + n, n, 0)
    torch.cuda.synchronize()
    sig_h = sig.cpu().numpy()
    kind = workloads.adversarial_mix(sig_h, frac=0.3 if n > 16 else 0.0, seed=n)
    mh = msg.cpu().numpy()
    with lat_max(1 << 20):
        p1, a1, s1 = engine.ecrecover_batch(mh, sig_h)
    with lat_max(0):
        p2, a2, s2 = engine.ecrecover_batch(mh, sig_h)
    with lat_max(1 << 20), wide_max(1 << 20):
        p3, a3, s3 = engine.ecrecover_batch(mh, sig_h)
    assert np.array_equal(s1, s2) and np.array_equal(p1, p2) and np.array_equal(a1, a2)
    assert np.array_equal(s1, s3) and np.array_equal(p1, p3) and np.array_equal(a1, a3)
    assert np.array_equal(s1, workloads.expected_status(kind, "ecrecover"))
    ok = s1 == 0
    assert np.array_equal(a1[ok], exp.cpu().numpy()[ok])


def test_lat_kernel_block_latency_record(engine):
    """C3's shape through eges_sender_batch on both kernels (printed for the record)."""
    import torch
    from eges_amd import txs
    from eges_amd._lib import SIGNER_EIP155
    sighash = txs.geec_block(7000, 1000, payload=100)
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(sighash).to("cuda:0"), 7000)
    torch.cuda.synchronize()
    r, s, v = txs.sender_rows(sig_d.cpu().numpy(), txs.GEEC_CHAIN_ID)
    out = {}
    for name, lm in (("latency", 1 << 20), ("lane-serial", 0)):
        with lat_max(lm):
            ts = []
            for i in range(12):
                t0 = time.perf_counter()
                addr, st = engine.sender_batch(sighash, r, s, v, None, SIGNER_EIP155, txs.GEEC_CHAIN_ID)
                ts.append(time.perf_counter() - t0)
            assert (st == 0).all() and np.array_equal(addr, exp_d.cpu().numpy())
            out[name] = float(np.median(ts[2:])) * 1e3
    print(f"\n1000-tx block via eges_sender_batch: latency kernel {out['latency']:.3f} ms, "
          f"lane-serial kernel {out['lane-serial']:.3f} ms")


def test_split_boundaries_structured_scalars(engine, oracle):
    """u2 = s / r chosen so that whole partial sums of the split form are empty or sit at its
    boundaries: u2 = 1, 2, lambda (GLV halves (0, 1)), 2^k around the split point 2^75 and the
    5-bit / 4-bit window edges, n - 1, n - lambda; each with u1 = -z / r for three z: 0 (no G
    part), the golden item's message, and -s (u1 = u2: Q = u2 (R + G)). Every item through the
    split (4-wave) and the narrow form must equal the oracle (pinned by the reference libsecp256k1)."""
    from eges_amd.workloads import N
    lam = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
    g = load_golden("recover.npz")
    base = [i for i in range(len(g["kind"])) if g["status"][i] == 0][:3]
    u2s = [1, 2, 3, lam, (N - lam) % N, N - 1, 1 << 74, 1 << 75, (1 << 75) - 1, (1 << 75) + 1, 1 << 76, 1 << 80,
           1 << 128, (1 << 129) - 1, 1 << 200, 31 << 70, 15 << 75]
    msgs, sigs = [], []
    for i in base:
        sig = g["sig"][i].tobytes()
        r = int.from_bytes(sig[:32], "big")
        for u2 in u2s:
            s = u2 * r % N
            for z in (0, int.from_bytes(g["msg"][i].tobytes(), "big") % N, (N - s) % N):
                msgs.append(z.to_bytes(32, "big"))
                sigs.append(sig[:32] + s.to_bytes(32, "big") + sig[64:])
    m = np.frombuffer(b"".join(msgs), np.uint8).reshape(-1, 32)
    sg = np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 65)
    assert len(m) <= 256  # the split form
    with lat_max(1 << 20):
        pub, addr, st = engine.ecrecover_batch(m, sg)
        with wide_max(0):
            pub2, addr2, st2 = engine.ecrecover_batch(m, sg)
    assert np.array_equal(pub, pub2) and np.array_equal(st, st2)
    for k in range(len(m)):
        ost, opub = oracle.recover_pubkey(m[k].tobytes(), sg[k].tobytes())
        assert int(st[k]) == ost, (k, int(st[k]), ost)
        if ost == 0:
            assert pub[k].tobytes() == opub, k
