"""CPU tests of the host-side workload helpers against the oracle and the reference's vectors:
sighash RLP (core/types/transaction_test.go:33-62), EIP-155 senders of the Vitalik vectors
(transaction_signing_test.go:79-116) through eges_amd.txs -> oracle Sender, the Geec block
shape, and the C5 adversarial mix whose expected statuses must equal the oracle's.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from eges_amd import txs, workloads


def vectors():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)["items"]


def test_frontier_sighash_vectors():
    for v in vectors()["sighash_go"]:
        h = txs.frontier_sighash(v["nonce"], v["price"], v["gas"], bytes.fromhex(v["to"]), v["value"],
                                 bytes.fromhex(v["data"]))
        assert h.hex() == v["hash"], v["cite"]


def test_eip155_vitalik_senders_through_host_rows(oracle):
    vs = vectors()["eip155_vitalik"]
    decoded = [txs.decode_geec_tx(bytes.fromhex(t["rlp"])) for t in vs["txs"]]
    h, r, s, v, vf = txs.sender_inputs(decoded, vs["chain_id"])
    for i, t in enumerate(vs["txs"]):
        st, addr = oracle.sender(2, vs["chain_id"], h[i].tobytes(), r[i].tobytes(), s[i].tobytes(), v[i].tobytes(),
                                 int(vf[i]))
        assert st == 0 and addr.hex() == t["addr"]


def test_geec_tx_roundtrip_10_fields():
    to = bytes(range(20))
    raw = txs.rlp_list([txs.rlp_uint(7), txs.rlp_uint(1), txs.rlp_uint(21000), txs.rlp_bytes(to), txs.rlp_uint(5),
                        txs.rlp_bytes(bytes(100)), b"\x01", txs.rlp_uint(txs.eip155_v(1, txs.GEEC_CHAIN_ID)),
                        txs.rlp_uint(12345), txs.rlp_uint(678)])
    d = txs.decode_geec_tx(raw)
    assert d == dict(nonce=7, price=1, gas=21000, to=to, value=5, data=bytes(100), is_geec=True,
                     v=1 + 35 + 2 * txs.GEEC_CHAIN_ID, r=12345, s=678)


def test_geec_block_shape():
    b = txs.geec_block(0, n=16)
    assert b.shape == (16, 32) and len({x.tobytes() for x in b}) == 16
    assert np.array_equal(b[3], txs.geec_block(3, n=1)[0])


def _signed_batch(n, seed):
    from oracle import RefLib, have_ref
    if not have_ref():
        pytest.skip("oracle/_ref not built here")
    ref = RefLib()
    rng = np.random.default_rng(seed)
    msg = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    keys = [int.from_bytes(rng.bytes(32), "big") % (workloads.N - 1) + 1 for _ in range(n)]
    sig = np.zeros((n, 65), np.uint8)
    pub = np.zeros((n, 65), np.uint8)
    import ctypes
    for i, k in enumerate(keys):
        kb = np.frombuffer(k.to_bytes(32, "big"), np.uint8)
        assert ref.L.eref_sign(ctypes.c_void_p(sig[i].ctypes.data), ctypes.c_void_p(msg[i].ctypes.data),
                               ctypes.c_void_p(kb.ctypes.data)) == 1
        assert ref.L.eref_pubkey(ctypes.c_void_p(pub[i].ctypes.data), ctypes.c_void_p(kb.ctypes.data)) == 1
    return msg, sig, pub


def test_adversarial_mix_matches_oracle(oracle):
    msg, sig, pub = _signed_batch(160, 3)
    kind = workloads.adversarial_mix(sig, frac=0.9, seed=11)
    assert set(kind.tolist()) == set(range(len(workloads.KIND_NAMES)))
    exp_e = workloads.expected_status(kind, "ecrecover")
    exp_s = workloads.expected_status(kind, "sender")
    r, s, v = workloads.sender_rows_mixed(sig, kind, txs.GEEC_CHAIN_ID)
    for i in range(len(kind)):
        st, p = oracle.recover_pubkey(msg[i].tobytes(), sig[i].tobytes())
        assert st == exp_e[i], (i, workloads.KIND_NAMES[kind[i]], st)
        if st == 0:
            assert p == pub[i].tobytes()  # high-s malleation recovers the same key
        st2, addr = oracle.sender(2, txs.GEEC_CHAIN_ID, msg[i].tobytes(), r[i].tobytes(), s[i].tobytes(),
                                  v[i].tobytes(), 0)
        assert st2 == exp_s[i], (i, workloads.KIND_NAMES[kind[i]], st2)
        if st2 == 0:
            assert addr == oracle.pub_to_addr(pub[i].tobytes())
