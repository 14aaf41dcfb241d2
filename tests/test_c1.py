"""BASELINE.json configs[0] (C1): types.Sender over synthetic EIP-155-signed transfers, as
SURVEY.md §8(d) specifies them: key_i = Keccak256("eges-key" || u64le(i)) mod n, to =
Keccak256("eges-to" || u64le(i))[12:], nonce i, gasPrice 1, gas 21000, value 1, empty data,
chainId 930412, signed with RFC6979 nonces exactly as secp256k1.Sign does (secp256.go:70-99;
the reference libsecp256k1 built in place, oracle/_ref). Expected senders come from the
reference's own pubkey_create, independently of any recovery code.

CPU: the oracle's Sender restatement reproduces every sender. GPU: the same transactions
through eges_sender_raw_batch (wire bytes: GPU decode + sighash + recovery) and
eges_sender_batch (SoA rows) are bit-exact, and the GPU synthetic signer's keys match the
reference-derived addresses (pins the bench's input generator).
"""
import numpy as np
import pytest

from eges_amd import txs

N_CPU = 200
N_GPU = 10000  # configs[0]'s full size


def _ref():
    from oracle import RefLib, have_ref
    if not have_ref():
        pytest.skip("oracle/_ref (reference libsecp256k1) not built")
    return RefLib()


def _c1_signed(ref, n):
    """(sighash, sig65, expected addr) of C1 transfers 0..n-1 via the reference signer."""
    from oracle.pyoracle import _p
    h = txs.c1_sighashes(0, n)
    sig = np.zeros((n, 65), np.uint8)
    addr = np.zeros((n, 20), np.uint8)
    pub = np.zeros(65, np.uint8)
    for i in range(n):
        key = np.frombuffer(txs.c1_key(i).to_bytes(32, "big"), np.uint8)
        assert ref.L.eref_sign(_p(sig[i]), _p(np.ascontiguousarray(h[i])), _p(key)) == 1
        assert ref.L.eref_pubkey(_p(pub), _p(key)) == 1
        addr[i] = np.frombuffer(txs._keccak(pub[1:].tobytes())[12:], np.uint8)
    return h, sig, addr


def test_c1_senders_oracle():
    from oracle import Oracle
    ref = _ref()
    o = Oracle()
    h, sig, addr = _c1_signed(ref, N_CPU)
    r, s, v = txs.sender_rows(sig)
    for i in range(N_CPU):
        st, a = o.sender(2, txs.GEEC_CHAIN_ID, h[i].tobytes(), r[i].tobytes(), s[i].tobytes(), v[i].tobytes(), 0)
        assert st == 0 and a == addr[i].tobytes(), i
    # the wire form decodes back to the same fields and sighash
    raw = txs.c1_raw(0, sig[:5])
    for i, b in enumerate(raw):
        d = txs.decode_geec_tx(b)
        assert (d["nonce"], d["price"], d["gas"], d["to"], d["value"], d["data"], d["is_geec"]) == \
            (i, 1, 21000, txs.c1_to(i), 1, b"", False)
        hh, *_ = txs.sender_inputs([d], txs.GEEC_CHAIN_ID)
        assert np.array_equal(hh[0], h[i])


@pytest.mark.gpu
def test_c1_senders_gpu(engine):
    import torch
    from eges_amd._lib import SIGNER_EIP155
    ref = _ref()
    h, sig, addr = _c1_signed(ref, N_GPU)
    r, s, v = txs.sender_rows(sig)
    # every recover form that can take the batch: the engine's default dispatch, the mid-size
    # kernel, the lane-serial kernel (knobs, eges_test_set_knob)
    forms = [{}, {"EGES_WIRE_FUSED": 0}, {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 1 << 20, "EGES_MID_FORM": 0},
             {"EGES_LAT_MAX": 0, "EGES_MID_MAX": 0}]
    for kv in forms:
        old = {k: engine.get_knob(k) for k in kv}
        try:
            for k, x in kv.items():
                engine.set_knob(k, x)
            a1, st1, sh = engine.sender_raw_batch(txs.c1_raw(0, sig), SIGNER_EIP155, txs.GEEC_CHAIN_ID,
                                                  want_sighash=True)
            assert (st1 == 0).all(), (kv, np.nonzero(st1)[0][:10])
            assert np.array_equal(sh, h)
            assert np.array_equal(a1, addr), kv
            a2, st2 = engine.sender_batch(h, r, s, v, None, SIGNER_EIP155, txs.GEEC_CHAIN_ID)
            assert (st2 == 0).all() and np.array_equal(a2, addr), kv
        finally:
            for k, x in old.items():
                engine.set_knob(k, x)
    # the GPU synthetic signer (bench.py --config c1) uses the same keys
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(h[:512]).cuda(), 0)
    torch.cuda.synchronize()
    assert np.array_equal(exp_d.cpu().numpy(), addr[:512])
