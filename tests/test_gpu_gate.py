"""Host-buffer calls that launch before their inputs are copied (EGES_GATE = 1, the default:
hostpath.hip run_host_shard GateOpen, handoff.cuh gate_wait): the fused mid-size kernels (bucket,
windowed) wait at the call's gate word while the host copies the inputs into the pinned buffer;
the host reads the outputs after the stream's completion signal. The latency forms
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


def _c1_batch(engine, first, n):
    """n C1-shaped transfers (nonce first + i) signed by the GPU synthetic signer,
    as wire bytes, with their signers' addresses"""
    import torch
    from eges_amd import txs
    sighash = txs.c1_sighashes(first, n)
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(sighash).cuda(), first)
    torch.cuda.synchronize()
    sig, exp = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    return txs.c1_raw(first, sig), exp


@pytest.mark.parametrize("step", [1, 3, 16, 0])
def test_gate_pieces_wire_and_golden(engine, step):
    """The progressive gate (EGES_GATE_STEP workgroups per piece; 0 = one piece): the host opens
    the inputs piece by piece in workgroup order while each mid-size workgroup waits for its own
    piece only. Two different 10k wire-format batches alternate (a workgroup that read its
    inputs before its piece was copied would return the other batch's sender), and the golden
    recovery and sender fixtures tiled to 7,000 items go through the bucket and windowed forms."""
    from eges_amd import txs
    from eges_amd._lib import SIGNER_EIP155
    batches = [_c1_batch(engine, first, 10000) for first in (0, 50000)]
    with knobs(engine, {"EGES_GATE": 1, "EGES_GATE_STEP": step, "EGES_RESIDENT": 0}):
        for rep in range(6):
            raws, exp = batches[rep % 2]
            addr, st, _ = engine.sender_raw_batch(raws, SIGNER_EIP155, txs.GEEC_CHAIN_ID)
            bad = np.nonzero((st != 0) | (addr != exp).any(axis=1))[0]
            assert bad.size == 0, (step, rep, bad[:10].tolist())
    g = load_golden("recover.npz")
    gs = load_golden("sender.npz")
    n = 7000
    idx = [np.arange(n) % len(g["msg"]), (np.arange(n) * 7 + 3) % len(g["msg"])]
    sel = np.nonzero((gs["signer"] == 2) & (gs["chain_id"] == 930412))[0]
    sidx = [sel[np.arange(n) % len(sel)], sel[(np.arange(n) * 5 + 1) % len(sel)]]
    for form in ("bucket", "windowed", "bucket2"):
        with knobs(engine, dict(FORMS[form], EGES_GATE=1, EGES_GATE_STEP=step, EGES_RESIDENT=0)):
            for rep in range(4):
                i = idx[rep % 2]
                pub, _, st = engine.ecrecover_batch(g["msg"][i], g["sig"][i])
                assert np.array_equal(st, g["status"][i]) and np.array_equal(pub, g["pub"][i]), (form, step, rep)
                k = sidx[rep % 2]
                a, s_ = engine.sender_batch(gs["sighash"][k], gs["r"][k], gs["s"][k], gs["v"][k], gs["vflags"][k], 2,
                                            930412)
                assert np.array_equal(s_, gs["status"][k]) and np.array_equal(a, gs["addr"][k]), (form, step, rep)


def test_gated_outputs_reread_after_drain(engine):
    """a gated mid-size call returns its outputs from the pinned buffer (round 5:
    at the last workgroup's completion word, which round 6 found can reach the host before the
    outputs stored ahead of it, handoff.cuh; now at the stream's completion signal). With
    EGES_TEST_RECHECK the call then synchronises the stream again, re-reads the pinned outputs and
    fails if any byte differs from what it returned. C1-sized recover calls
    (10k signatures) and C1 wire-format calls (10k transfers), two different batches alternating
    (a byte read before its store arrived would be the other batch's), 40 calls each, every
    returned address and status also checked against its signer."""
    import torch
    from eges_amd import txs
    from eges_amd._lib import SIGNER_EIP155
    sets = []
    for first in (11 << 20, 23 << 20):
        m, s, e = engine.synth_sign_dev(first, 10000, 0)
        torch.cuda.synchronize()
        sets.append((m.cpu().numpy(), s.cpu().numpy(), e.cpu().numpy()))
    wires = [_c1_batch(engine, first, 10000) for first in (0, 70000)]
    with knobs(engine, {"EGES_GATE": 1, "EGES_RESIDENT": 0, "EGES_TEST_RECHECK": 1}):
        for rep in range(40):
            m, s, e = sets[rep % 2]
            _, addr, st = engine.ecrecover_batch(m, s, want_pub=False)
            assert (st == 0).all() and np.array_equal(addr, e), rep
            raws, exp = wires[rep % 2]
            a, st2, _ = engine.sender_raw_batch(raws, SIGNER_EIP155, txs.GEEC_CHAIN_ID)
            assert (st2 == 0).all() and np.array_equal(a, exp), rep


def test_resident_outputs_reread(engine):
    """The resident single-call server publishes each job with the same primitive (outputs, then a
    system-scope release and the done word the host polls). With EGES_TEST_RECHECK the call returns
    a snapshot taken at the done word and fails if the live outputs differ 200 us later: 400
    single recoveries alternating two golden items, every one checked."""
    from test_gpu_resident import _single_recover
    g = load_golden("recover.npz")
    ok = np.nonzero((g["status"] == 0) & (g["sig"][:, 64] < 4))[0][:2]
    with knobs(engine, {"EGES_RESIDENT": 1, "EGES_TEST_RECHECK": 1}):
        engine.diag_counters(reset=True)
        for rep in range(400):
            i = int(ok[rep % 2])
            rc, pub = _single_recover(g["msg"][i], g["sig"][i])
            assert rc == 1 and pub == g["pub"][i].tobytes(), rep
        assert engine.diag_counters(reset=True)["resident"] >= 300
