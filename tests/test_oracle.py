"""CPU tests: pin the oracle (oracle/oracle.c) against the reference's own vectors and the
golden fixtures (generated from the reference libsecp256k1 compiled in place), and cross-check
it against oracle/_ref where that library is present.

Mirrors the reference's tests: crypto/signature_test.go:37-86, crypto/crypto_test.go:37-41,
:59-87, :148-190, crypto/sha3/sha3_test.go:79-117, core/types/transaction_signing_test.go:79-138,
core/types/transaction_test.go:54-127, libsecp256k1 src/modules/recovery/tests_impl.h:209-380.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
HALF_N = N // 2


def vectors():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)["items"]


# ------------------------------------------------------------------ Keccak
def test_keccak_kats(oracle):
    with open(os.path.join(GOLDEN, "keccak_kats.json")) as f:
        k = json.load(f)
    for v in k["keccak256"]:
        assert oracle.keccak256(bytes.fromhex(v["in"])).hex() == v["out"]
    assert len(k["sha3"]) >= 64
    for v in k["sha3"]:  # same permutation, SHA-3 domain byte (sha3_test.go:79-117)
        outlen = int(v["fn"].split("-")[1]) // 8
        assert oracle.sponge(bytes.fromhex(v["msg"]), outlen, v["rate"], v["ds"]).hex() == v["digest"], v


def test_keccak_abc(oracle):  # crypto/crypto_test.go:37-41
    assert oracle.keccak256(b"abc").hex() == vectors()["keccak_abc"]["out"]


# ------------------------------------------------------------------ Ecrecover / Verify
def test_ecrecover_go_vector(oracle):  # crypto/signature_test.go:37-45
    v = vectors()["ecrecover_go"]
    st, pub = oracle.recover_pubkey(bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]))
    assert st == 0 and pub.hex() == v["pub"]


def test_verify_go_vectors(oracle):  # crypto/signature_test.go:47-86
    v = vectors()["ecrecover_go"]
    msg, sig = bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"])[:64]
    pub, pubc = bytes.fromhex(v["pub"]), bytes.fromhex(v["pubc"])
    assert oracle.verify(pub, msg, sig) == 1
    assert oracle.verify(pubc, msg, sig) == 1
    assert oracle.verify(b"", msg, sig) == 0
    assert oracle.verify(pub, b"", sig) == 0
    assert oracle.verify(pub, msg, b"") == 0
    assert oracle.verify(pub, msg, sig + b"\x01\x02\x03") == 0
    assert oracle.verify(pub, msg, sig[:-2]) == 0
    wrong = bytearray(pub)
    wrong[10] += 1
    assert oracle.verify(bytes(wrong), msg, sig) == 0
    m = vectors()["verify_malleable_go"]
    assert oracle.verify(bytes.fromhex(m["key"]), bytes.fromhex(m["msg"]), bytes.fromhex(m["sig"])) == 0


def test_recovery_edge_vectors(oracle):  # tests_impl.h:209-380
    e = vectors()["secp_edge"]
    msg, sig = bytes.fromhex(e["msg"]), bytes.fromhex(e["sig_key0"])
    for recid in range(4):
        st, _ = oracle.recover_pubkey(msg, sig + bytes([recid]))
        assert (st == 0) == (recid in e["key0_ok_recids"])
    four = (4).to_bytes(32, "big")
    for recid in range(4):  # (r, s) = (4, 4) recovers with every recid
        assert oracle.recover_pubkey(msg, four + four + bytes([recid]))[0] == 0
    one, zero = (1).to_bytes(32, "big"), bytes(32)
    assert oracle.recover_pubkey(msg, one + one + b"\0")[0] == 0
    assert oracle.recover_pubkey(msg, zero + one + b"\0")[0] == 6
    assert oracle.recover_pubkey(msg, one + zero + b"\0")[0] == 6


def test_invalid_recovery_id(oracle):  # crypto/secp256k1/secp256_test.go:87-96
    v = vectors()["ecrecover_go"]
    sig = bytearray(bytes.fromhex(v["sig"]))
    sig[64] = 99
    assert oracle.recover_pubkey(bytes.fromhex(v["msg"]), bytes(sig))[0] == 5


def test_recover_golden(oracle):
    g = load_golden("recover.npz")
    pub, addr, st = oracle.recover_batch(g["msg"], g["sig"])
    assert np.array_equal(st, g["status"])
    assert np.array_equal(pub, g["pub"])
    # every reject class is represented
    kinds = set(g["kind_names"][g["kind"][g["status"] != 0]])
    assert {"recid_ge4", "overflow", "zero_rs", "infinity", "edge_r"} <= kinds


def test_verify_golden(oracle):
    g = load_golden("verify.npz")
    for i in range(len(g["ok"])):
        pub = g["pub"][i][: g["publen"][i]].tobytes()
        assert oracle.verify(pub, g["msg"][i].tobytes(), g["sig"][i].tobytes()) == g["ok"][i], i


def test_sender_golden(oracle):
    g = load_golden("sender.npz")
    for i in range(len(g["status"])):
        st, addr = oracle.sender(g["signer"][i], g["chain_id"][i], g["sighash"][i].tobytes(), g["r"][i].tobytes(),
                                 g["s"][i].tobytes(), g["v"][i].tobytes(), g["vflags"][i])
        assert st == g["status"][i], (i, g["kind_names"][g["kind"][i]])
        assert addr == g["addr"][i].tobytes()


def test_test_priv_address(oracle):  # crypto/crypto_test.go:31-32,59-87 via a recover round trip
    from oracle import RefLib, have_ref
    if not have_ref():
        pytest.skip("oracle/_ref not built here")
    ref = RefLib()
    v = vectors()["test_priv"]
    import ctypes
    pub = np.zeros(65, np.uint8)
    key = np.frombuffer(bytes.fromhex(v["priv"]), np.uint8)
    assert ref.L.eref_pubkey(ctypes.c_void_p(pub.ctypes.data), ctypes.c_void_p(key.ctypes.data)) == 1
    assert oracle.pub_to_addr(pub.tobytes()).hex() == v["addr"]


# ------------------------------------------------------------------ restatement vs compiled reference
def test_oracle_matches_reference_random(oracle):
    from oracle import RefLib, have_ref
    if not have_ref():
        pytest.skip("oracle/_ref not built here")
    ref = RefLib()
    rng = np.random.default_rng(7)
    n = 300
    msg = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    sig = rng.integers(0, 256, (n, 65), dtype=np.uint8)
    sig[:, 64] = rng.integers(0, 4, n)
    sig[: n // 2, 0] = 0  # push half below n so they parse
    for i in range(n):
        r1, p1 = ref.ecrecover(msg[i].tobytes(), sig[i].tobytes())
        st, p2 = oracle.recover_pubkey(msg[i].tobytes(), sig[i].tobytes())
        assert (r1 == 1) == (st == 0)
        if r1 == 1:
            assert p1 == p2


def test_validate_signature_values_table(oracle):  # crypto/crypto_test.go:148-190 through Sender
    one = (1).to_bytes(32, "big")
    zero = bytes(32)
    nm1 = (N - 1).to_bytes(32, "big")
    nn = N.to_bytes(32, "big")
    h = bytes(32)
    cases = [  # (v, r, s, valid under Frontier rules)
        (0, one, one, True), (1, one, one, True), (2, one, one, False), (3, one, one, False),
        (0, zero, zero, False), (0, zero, one, False), (0, one, zero, False),
        (0, nm1, nm1, True), (0, nn, nm1, False), (0, nm1, nn, False), (0, nn, nn, False),
    ]
    for v, r, s, valid in cases:
        st, _ = oracle.sender(0, 0, h, r, s, (27 + v).to_bytes(32, "big"), 0)
        # valid range => passes ValidateSignatureValues; recovery itself may still fail (6)
        assert (st != 2) == valid, (v, valid, st)


def test_ref_backed_sender_reproduces_golden():
    """oracle/_ref eref_sender_batch_mt (oracle.c's Go-layer Sender rules over the reference
    libsecp256k1's recovery; the 1M Sender-mode GPU check uses it) reproduces every golden sender
    item: status and address, every signer and chain id."""
    import numpy as np
    from oracle import RefLib, have_ref
    if not have_ref():
        pytest.skip("oracle/_ref not built")
    from conftest import load_golden
    g = load_golden("sender.npz")
    ref = RefLib()
    for signer, cid in sorted(set(zip(g["signer"].tolist(), g["chain_id"].tolist()))):
        sel = np.nonzero((g["signer"] == signer) & (g["chain_id"] == cid))[0]
        a, st = ref.sender_batch_mt(signer, cid, g["sighash"][sel], g["r"][sel], g["s"][sel], g["v"][sel],
                                    g["vflags"][sel], 4)
        assert np.array_equal(st, g["status"][sel]), (signer, cid)
        assert np.array_equal(a, g["addr"][sel]), (signer, cid)


def test_ref_verify_batch_mt_golden():
    """oracle/_ref's multi-threaded VerifySignature (the GPU tests' item-for-item checker at
    size) gives the golden fixtures' results on all 591 items, on 1 and on 7 threads."""
    from oracle import RefLib, have_ref
    if not have_ref():
        pytest.skip("oracle/_ref not built")
    g = load_golden("verify.npz")
    for t in (1, 7):
        ok = RefLib().verify_batch_mt(g["pub"], g["publen"], g["msg"], g["sig"], t)
        assert np.array_equal(ok, g["ok"]), t
