"""types.Sender rows classified inside the recover kernels (EGES_SENDER_FUSED = 1, the default:
sender.cuh sender_parse_wave / sender_parse_lane, no prep_sender_kernel launch) against the
reference-generated fixtures and against the separate prep_sender path (EGES_SENDER_FUSED = 0),
for every kernel form that takes them: the latency kernels (narrow with root helpers, split) and
the mid-size kernel (bucket, windowed). Misaligned device rows fall back to prep_sender."""
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
    "bucket2": {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 2, "EGES_BKT2": 2},
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
@pytest.mark.parametrize("fused", [1, 0])
def test_sender_golden_fused_and_prep(engine, form, fused):
    """every golden sender item (all Go error classes, every signer) byte for byte the fixtures"""
    g = load_golden("sender.npz")
    with knobs(engine, dict(FORMS[form], EGES_SENDER_FUSED=fused)):
        for signer, cid in sorted(set(zip(g["signer"].tolist(), g["chain_id"].tolist()))):
            sel = np.nonzero((g["signer"] == signer) & (g["chain_id"] == cid))[0]
            a, s_ = engine.sender_batch(g["sighash"][sel], g["r"][sel], g["s"][sel], g["v"][sel], g["vflags"][sel],
                                        int(signer), int(cid))
            bad = np.nonzero(s_ != g["status"][sel])[0]
            assert bad.size == 0, (signer, cid, [(int(sel[i]), int(s_[i]), int(g["status"][sel][i])) for i in bad[:10]])
            assert np.array_equal(a, g["addr"][sel]), (signer, cid)


@pytest.mark.parametrize("form", ["narrow", "bucket"])
def test_sender_dev_misaligned_rows_fall_back(engine, form):
    """device rows at an odd byte offset: not 4-byte aligned, so the prep_sender path runs; the
    results equal the fixtures either way"""
    import torch
    g = load_golden("sender.npz")
    signer, cid = 2, int(g["chain_id"][g["signer"] == 2][0])
    sel = np.nonzero((g["signer"] == signer) & (g["chain_id"] == cid))[0]
    n = len(sel)

    def odd(x, w):
        buf = torch.zeros(n * w + 1, dtype=torch.uint8, device="cuda")
        buf[1:] = torch.from_numpy(np.ascontiguousarray(x).reshape(-1)).cuda()
        return buf[1:].view(n, w) if w > 1 else buf[1:]

    rows = [odd(g[k][sel], 32) for k in ("sighash", "r", "s", "v")]
    vf = torch.from_numpy(np.ascontiguousarray(g["vflags"][sel])).cuda()
    with knobs(engine, FORMS[form]):
        addr, st = engine.sender_batch_dev(*rows, vf, signer, cid)
        torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), g["status"][sel])
    assert np.array_equal(addr.cpu().numpy(), g["addr"][sel])
