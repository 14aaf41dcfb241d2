"""GPU parity of the wire-format decoder (k_txhash.hip) on the reference's own RLP vectors.

Each vector of rlp/decode_test.go (tests/golden/rlp_decode.json) is spliced into the field of a
10-field Geec txdata list (core/types/transaction.go:59-76) whose Go type it was written for:
uint -> Nonce / GasLimit, *big.Int -> Price / Amount / V / R / S, []byte -> Payload,
bool -> IsGeecTxn. Every vector the reference rejects must give EGES_DECODE_FAILED; every
accepted one must decode to the vector's value in the oracle, and the GPU's status, sender and
signing hash must equal the oracle's item for item. Vectors whose outcome depends on being at the
end of the input (input-limit / EOF cases) are spliced into the last field only. The base
transaction is the reference's TestChainId vector (tests/golden/chain_id.json)."""
import json
import os

import numpy as np
import pytest

from oracle import txoracle as T

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("wire_form")]
HERE = os.path.dirname(os.path.abspath(__file__))

FIELDS = {"uint": (0, 2), "uint32": (0, 2), "bigint": (1, 4, 7, 8, 9), "bytes": (5,), "bool": (6,)}
STREAM_TYPES = {"Uint": "uint", "Bytes": "bytes", "Bool": "bool", "Kind": "bytes", "List": "bytes"}
# 20-byte analogs of decode_test.go:406-418 for the *common.Address field (rlp:"nil"): derived
# from the same decodeByteArray rules (not reference vectors); "80" / "C0" decode as nil.
ADDR_CASES = [("94" + "11" * 20, True), ("02", False), ("820000", False), ("C3010203", False),
              ("95" + "11" * 21, False), ("93" + "11" * 19, False), ("8105", False), ("80", True), ("C0", True),
              ("C101", False)]


def load(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


def split_items(raw):
    s = T._Stream(raw)
    s.list_start()
    items = []
    while s.pos < s.ends[-1]:
        start = s.pos
        k, size, _ = s.kind()
        if k != "byte":
            s.content(size)
        items.append(s.b[start:s.pos])
    return items


def splice(items, j, enc):
    return T.enc_list(items[:j] + [enc] + items[j + 1:])


def build_cases():
    base = bytes.fromhex(load("chain_id.json")["raw10"])
    items = split_items(base)
    assert len(items) == 10
    cases = []  # (raw, reference_ok or None, field, expected value or None, label)
    vecs = load("rlp_decode.json")
    for v in vecs["decode"]:
        typ = v["type"]
        if typ not in FIELDS or (typ == "uint32" and v["line"] == 375):  # 5-byte value: fits uint64
            continue
        for j in FIELDS[typ]:
            cases.append((splice(items, j, bytes.fromhex(v["input"])), v["ok"], j, v.get("value"), f"L{v['line']}"))
    for v in vecs["stream"]:
        end_bound = not v["ok"] and v["error"] in ("ErrValueTooLarge", "io.EOF")
        fields = (9,) if end_bound else FIELDS[STREAM_TYPES[v["call"]]]
        for j in fields:
            cases.append((splice(items, j, bytes.fromhex(v["input"])), v["ok"], j, v.get("value"), f"S{v['line']}"))
    for enc, ok in ADDR_CASES:
        cases.append((splice(items, 3, bytes.fromhex(enc)), ok, 3, None, f"addr-{enc[:6]}"))
    # struct element count (decode_test.go:452-472 rules on txdata): too few / too many / not a list
    for k in range(10):
        cases.append((T.enc_list(items[:k]), False, None, None, f"fields-{k}"))
    cases.append((T.enc_list(items + [b"\x01"]), False, None, None, "fields-11"))
    cases.append((b"\x83\x22\x22\x22", False, None, None, "not-a-list"))
    cases.append((base + b"\x00", False, None, None, "trailing"))
    cases.append((base, True, None, None, "base"))
    return cases


def test_reference_rlp_vectors_on_gpu(engine, oracle):
    cases = build_cases()
    raws = [c[0] for c in cases]
    addr, st, sh = engine.sender_raw_batch(raws, 2, 1, want_sighash=True)
    n_rej = 0
    for i, (raw, ref_ok, field, value, label) in enumerate(cases):
        ost, oaddr, oh = T.sender_raw(oracle, raw, 2, 1)
        # the oracle agrees with the reference's verdict on the vector
        if ref_ok is False:
            assert ost == T.DECODE_FAILED, (label, field, raw.hex())
            n_rej += 1
        elif ref_ok is True:
            assert ost != T.DECODE_FAILED, (label, field, raw.hex())
            if field is not None and value is not None:
                d = T.decode_txdata(raw)
                got = d[T.TXDATA_FIELDS[field]]
                got = got.hex() if isinstance(got, bytes) else got
                assert got == value, (label, field, got, value)
        # the GPU agrees with the oracle item for item
        assert int(st[i]) == ost, (label, field, raw.hex(), int(st[i]), ost)
        assert addr[i].tobytes() == oaddr, (label, field)
        assert sh[i].tobytes() == oh, (label, field)
    assert n_rej > 60


def test_chain_id_mismatch_vector_gpu(engine):
    """core/types/transaction_signing_test.go:118-138 through eges_sender_raw_batch."""
    v = load("chain_id.json")
    raw10 = bytes.fromhex(v["raw10"])
    for case in v["cases"]:
        addr, st, sh = engine.sender_raw_batch([raw10, raw10], 2, case["signer_chain_id"], want_sighash=True)
        assert (st == case["status"]).all()
        if case["status"] == 0:
            assert addr[0].tobytes().hex() == case["addr"] and sh[0].tobytes().hex() == v["sighash_chain1"]
        else:
            assert not addr.any()
    _, st, _ = engine.sender_raw_batch([bytes.fromhex(v["raw9"])], 2, 1)
    assert int(st[0]) == T.DECODE_FAILED
