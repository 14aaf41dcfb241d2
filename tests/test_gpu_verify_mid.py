"""crypto.VerifySignature on the mid-size kernel's bucket form (k_recover_mid.hip verify mode:
s^-1, u1 = z/s, u2 = r/s on wave S, the key's R' chain on wave X, buckets on Y1 / Y2, x(Q) == r
checked projectively on Y1): batches between the latency kernels' cut and
64 x CUs items take it. Every item equals the reference-generated fixtures and the lane-serial
verify kernel."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

BUCKET = {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2}
LANE = {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 0}


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


def test_verify_bucket_golden(engine):
    """every golden verify item (33/65-byte and hybrid keys, off-curve, high-s, overflow,
    zero r / s, wrong key): byte for byte the fixtures (reference libsecp256k1)"""
    g = load_golden("verify.npz")
    with knobs(engine, BUCKET):
        ok = engine.verify_batch(g["pub"], g["publen"], g["msg"], g["sig"])
    names = list(g["kind_names"])
    bad = np.nonzero(ok != g["ok"])[0]
    assert bad.size == 0, [(int(i), names[g["kind"][i]], int(ok[i]), int(g["ok"][i])) for i in bad[:20]]


def test_verify_bucket_tiled_ragged_dev(engine):
    """the golden set tiled to 10,007 items (ragged last workgroup) through the device entry,
    bucket form vs lane-serial kernel vs fixtures"""
    import torch
    g = load_golden("verify.npz")
    n = 10007
    rep = -(-n // len(g["pub"]))
    cols = {k: np.ascontiguousarray(np.concatenate([g[k]] * rep)[:n]) for k in ("pub", "publen", "msg", "sig", "ok")}
    dev = {k: torch.from_numpy(cols[k]).cuda() for k in ("pub", "publen", "msg", "sig")}
    outs = {}
    for name, kv in (("bucket", BUCKET), ("bucket2", dict(BUCKET, EGES_BKT2=2)), ("lane", LANE)):
        with knobs(engine, kv):
            ok = engine.verify_batch_dev(dev["pub"], dev["publen"], dev["msg"], dev["sig"])
            torch.cuda.synchronize()
        outs[name] = ok.cpu().numpy()
    assert np.array_equal(outs["bucket"], cols["ok"])
    assert np.array_equal(outs["bucket2"], cols["ok"])
    assert np.array_equal(outs["lane"], cols["ok"])


def test_verify_bucket_synthetic_mix(engine):
    """4,099 synthetic signatures, a quarter with 33-byte keys, every tenth with a wrong key or a
    high s: the bucket form equals the lane-serial kernel item for item"""
    import torch
    from eges_amd import workloads
    n = 4099
    msg, sig, _ = engine.synth_sign_dev(4242, n, 0)
    pub = torch.empty((n, 65), dtype=torch.uint8, device="cuda")
    engine.ecrecover_batch_dev(msg, sig, pub=pub)
    torch.cuda.synchronize()
    pub_h, sig_h, msg_h = pub.cpu().numpy(), sig.cpu().numpy()[:, :64].copy(), msg.cpu().numpy()
    publen = np.full(n, 65, np.uint8)
    comp = np.arange(n) % 4 == 1
    odd = pub_h[:, 64] & 1
    pub_h[comp, 0] = 2 + odd[comp]
    pub_h[comp, 33:] = 0
    publen[comp] = 33
    for i in range(0, n, 10):
        if i % 20 == 0:
            pub_h[i] = pub_h[(i + 1) % n]
            publen[i] = publen[(i + 1) % n]
        else:
            s_ = int.from_bytes(sig_h[i, 32:64].tobytes(), "big")
            sig_h[i, 32:64] = np.frombuffer((workloads.N - s_).to_bytes(32, "big"), np.uint8)
    with knobs(engine, BUCKET):
        ok_b = engine.verify_batch(pub_h, publen, msg_h, sig_h)
    with knobs(engine, LANE):
        ok_l = engine.verify_batch(pub_h, publen, msg_h, sig_h)
    assert np.array_equal(ok_b, ok_l)
    assert ok_b.sum() > n * 8 // 10 and ok_b[::10].sum() == 0


def test_verify_bucket_two_generations(engine):
    """EGES_VERIFY_MID_GENS = 2 routes a batch of up to 2 x 64 x CUs items to the bucket form (two
    generations of workgroups) instead of the lane-serial kernel: with the forced redo only the
    mid-size kernel bumps mid_redo, so the counters show which form ran; the golden set tiled past
    one generation (ragged last workgroup) equals the fixtures under both routings"""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    g = load_golden("verify.npz")
    n = 64 * cus + 64 * (cus // 2) + 37  # 1.5 generations
    rep = -(-n // len(g["pub"]))
    cols = {k: np.ascontiguousarray(np.concatenate([g[k]] * rep)[:n]) for k in ("pub", "publen", "msg", "sig", "ok")}
    dev = {k: torch.from_numpy(cols[k]).cuda() for k in ("pub", "publen", "msg", "sig")}
    # (round 6: 1.5 generations at one workgroup per CU are one at two per CU, EGES_BKT2, the
    # default; without it the lane-serial kernel runs)
    for gens, b2, form in ((2, 0, "mid_redo"), (1, 0, "ls_redo"), (1, 1, "mid_redo")):
        engine.diag_counters(reset=True)
        with knobs(engine, {"EGES_VERIFY_MID_GENS": gens, "EGES_TEST_FORCE_REDO": 1, "EGES_BKT2": b2}):
            ok = engine.verify_batch_dev(dev["pub"], dev["publen"], dev["msg"], dev["sig"])
            torch.cuda.synchronize()
        d = engine.diag_counters(reset=True)
        assert np.array_equal(ok.cpu().numpy(), cols["ok"]), (gens, b2)
        assert d[form] > 0, (gens, b2, d)
        assert d["mid_redo" if form == "ls_redo" else "ls_redo"] == 0, (gens, d)
