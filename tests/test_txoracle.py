"""CPU tests of the wire-format transaction oracle (oracle/txoracle.py) against the reference's
own vectors: the Vitalik EIP-155 transactions (core/types/transaction_signing_test.go:79-116)
and the Homestead recipient transactions (core/types/transaction_test.go:82-127), re-encoded
in the 10-field Geec txdata form (core/types/transaction.go:59-76); plus the rlp/decode.go
rejection rules the GPU decoder (eges_amd/csrc/k_txhash.hip) must reproduce."""
import json
import os

import pytest

from conftest import GOLDEN
from eges_amd import txs
from oracle import txoracle as T


def vectors():
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        return json.load(f)["items"]


def test_vitalik_vectors_nine_fields_do_not_decode():
    # the Geec struct has 10 fields: the standard encoding runs out of elements (decode.go:428)
    for t in vectors()["eip155_vitalik"]["txs"]:
        with pytest.raises(T.DecodeError):
            T.decode_txdata(bytes.fromhex(t["rlp"]))


def test_vitalik_vectors_geec_form_senders(oracle):
    vs = vectors()["eip155_vitalik"]
    for t in vs["txs"]:
        raw = T.to_geec10(bytes.fromhex(t["rlp"]))
        d = T.decode_txdata(raw)
        assert d["is_geec"] is False
        st, addr, h = T.sender_raw(oracle, raw, 2, vs["chain_id"])
        assert st == 0 and addr.hex() == t["addr"]
        # the lenient host decoder agrees on every field
        assert {k: v for k, v in txs.decode_geec_tx(raw).items()} == d


def test_homestead_recipient_vectors(oracle):
    hv = vectors()["homestead_recipients"]
    for raw9 in hv["txs"]:
        raw = T.to_geec10(bytes.fromhex(raw9))
        for signer in (1, 2):  # Homestead, and EIP155 falling back for V = 27/28
            st, addr, _ = T.sender_raw(oracle, raw, signer, 930412)
            assert st == 0 and addr.hex() == hv["addr"]


def _tx(nonce=b"\x01", price=b"\x01", gas=b"\x82\x52\x08", to=b"\x80", value=b"\x05", data=b"\x80", geec=b"\x80",
        v=b"\x25", r=b"\xa0" + bytes([7] * 32), s=b"\xa0" + bytes([9] * 32), extra=()):
    """A txdata list from already-encoded items (so non-canonical items can be placed)."""
    return T.enc_list([nonce, price, gas, to, value, data, geec, v, r, s, *extra])


TO20 = b"\x94" + bytes(range(1, 21))

# (name, raw, decodes?) — each rejection cites the decode.go rule
DECODE_CASES = [
    ("plain", _tx(to=TO20), True),
    ("nil to as empty string", _tx(), True),
    ("nil to as empty list", _tx(to=b"\xc0"), True),                           # makeOptionalPtrDecoder :472
    ("to 19 bytes", _tx(to=b"\x93" + bytes(19)), False),                         # decodeByteArray :407
    ("to single byte", _tx(to=b"\x05"), False),                                  # :398-400
    ("to as list", _tx(to=b"\xd4" + bytes(20)), False),                          # :421
    ("nonce zero", _tx(nonce=b"\x80"), True),
    ("nonce 0x00 byte", _tx(nonce=b"\x00"), False),                              # uint ErrCanonInt :715
    ("nonce 9 bytes", _tx(nonce=b"\x89" + bytes([1] * 9)), False),               # uint overflow :723
    ("gas leading zero", _tx(gas=b"\x83\x00\x52\x08"), False),                   # readUint :1002 -> ErrCanonInt
    ("gas 0x8105", _tx(gas=b"\x81\x05"), False),                                  # uint :733
    ("gas 0x8180", _tx(gas=b"\x81\x80"), True),
    ("geec true", _tx(geec=b"\x01"), True),
    ("geec 0x00", _tx(geec=b"\x00"), False),                                     # uint ErrCanonInt :715
    ("geec 2", _tx(geec=b"\x02"), False),                                        # Bool :752
    ("geec 0x8101", _tx(geec=b"\x81\x01"), False),                               # :733 ErrCanonSize
    ("geec 0x8180", _tx(geec=b"\x81\x80"), False),                               # invalid boolean
    ("price leading zero", _tx(price=b"\x82\x00\x01"), False),                   # decodeBigInt :265
    ("price 0x00", _tx(price=b"\x00"), False),
    ("price 0x8105", _tx(price=b"\x81\x05"), False),                             # Bytes :683
    ("price zero", _tx(price=b"\x80"), True),
    ("value long 33 bytes", _tx(value=b"\xa1" + b"\x01" + bytes(32)), True),
    ("v wide", _tx(v=b"\xa1" + b"\x01" + bytes(32)), True),
    ("r as list", _tx(r=b"\xc0"), False),
    ("payload single byte", _tx(data=b"\x05"), True),
    ("payload 0x8105", _tx(data=b"\x81\x05"), False),                             # Bytes :683
    ("payload as list", _tx(data=b"\xc1\x05"), False),
    ("payload long", _tx(data=T.enc_bytes(bytes(300))), True),
    ("11 fields", _tx(extra=(b"\x80",)), False),                                 # too many :434
    ("9 fields", T.enc_list([b"\x01", b"\x01", b"\x82\x52\x08", b"\x80", b"\x05", b"\x80", b"\x25",
                             b"\xa0" + bytes([7] * 32), b"\xa0" + bytes([9] * 32)]), False),  # too few :428
]


def test_decode_acceptance_table():
    for name, raw, ok in DECODE_CASES:
        try:
            T.decode_txdata(raw)
            got = True
        except T.DecodeError:
            got = False
        assert got == ok, name


def test_decode_framing_rules():
    good = _tx(to=TO20)
    T.decode_txdata(good)
    bad = [
        good + b"\x00",                        # trailing bytes: ErrMoreThanOneValue (DecodeBytes :125)
        good[:-1],                             # value larger than the input (Kind :892)
        b"",                                   # EOF
        b"\x80",                               # not a list
        b"\xf9\x00" + good[2:],                # length with a leading zero (readUint :1002)
        b"\xb8\x05hello",                      # long string form for 5 bytes (readKind :951)
    ]
    for raw in bad:
        with pytest.raises(T.DecodeError):
            T.decode_txdata(raw)
    # a long-form list header whose declared size is below 56: ErrCanonSize (readKind :980)
    short = _tx(r=b"\x01", s=b"\x01")
    assert short[0] < 0xf8 and len(short) - 1 < 56
    T.decode_txdata(short)
    with pytest.raises(T.DecodeError):
        T.decode_txdata(bytes([0xf8, len(short) - 1]) + short[1:])


def test_nil_to_forms_hash_alike(oracle):
    a, b = _tx(), _tx(to=b"\xc0")
    da, db = T.decode_txdata(a), T.decode_txdata(b)
    assert da == db and da["to"] is None
    for signer in (0, 2):
        assert T.signing_payload(da, signer, 930412) == T.signing_payload(db, signer, 930412)


def test_signing_payload_matches_host_helpers():
    raw = _tx(to=TO20, data=T.enc_bytes(bytes(100)), v=T.enc_uint(txs.eip155_v(1, txs.GEEC_CHAIN_ID)))
    d = T.decode_txdata(raw)
    from eges_amd.engine import keccak256
    h = keccak256(T.signing_payload(d, 2, txs.GEEC_CHAIN_ID))
    assert h == txs.eip155_sighash(d["nonce"], d["price"], d["gas"], d["to"], d["value"], d["data"], txs.GEEC_CHAIN_ID)
    h0 = keccak256(T.signing_payload(d, 0, txs.GEEC_CHAIN_ID))
    assert h0 == txs.frontier_sighash(d["nonce"], d["price"], d["gas"], d["to"], d["value"], d["data"])


# core/vm/contracts_test.go:390-395 (BenchmarkPrecompiledEcrecover sample)
PRECOMPILE_VECTOR = ("38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e"
                     "000000000000000000000000000000000000000000000000000000000000001b"
                     "38d18acb67d25c8bb9942764b62f18e17054f66a817bd4295423adf9ed98873e"
                     "789d1dd423d25f0772d2748d60f7e4b81bb14d086eba8e8e8efb6dcff8a4ae02",
                     "000000000000000000000000ceaccac640adf55b2028469bd36ba501f28b699d")


def precompile_cases():
    """(input, expected status) around the reference vector: the pre-checks of Run and padding."""
    good = bytes.fromhex(PRECOMPILE_VECTOR[0])
    N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    flip = lambda b, i, x: b[:i] + bytes([x]) + b[i + 1:]
    cases = [(good, 0), (good + b"\x99" * 40, 0),                      # longer input: first 128 bytes
             (flip(good, 40, 1), 2),                                   # input[32:63] not zero
             (flip(good, 63, 0x1c), None),                             # v = 1: another key or failure
             (flip(good, 63, 0x1d), 2), (flip(good, 63, 0x00), 2),     # v not 27/28 (byte wrap)
             (good[:64] + bytes(32) + good[96:], 2),                   # r = 0
             (good[:96] + bytes(32), 2),                               # s = 0
             (good[:64] + N.to_bytes(32, "big") + good[96:], 2),       # r = N
             (good[:96] + (N - 1).to_bytes(32, "big"), 0),             # high s allowed (homestead = false)
             (good[:64] + (5).to_bytes(32, "big") + good[96:], 6),     # x = 5: not on the curve
             (good[:100], None), (b"", 2), (good[:127], None), (good[:64], 2)]  # right-padded short inputs
    return cases


def test_precompile_reference_vector(oracle):
    st, out = T.precompile_ecrecover(oracle, bytes.fromhex(PRECOMPILE_VECTOR[0]))
    assert st == 0 and out.hex() == PRECOMPILE_VECTOR[1]
    for inp, exp in precompile_cases():
        st, out = T.precompile_ecrecover(oracle, inp)
        if exp is not None:
            assert st == exp, inp.hex()
        assert (out is None) == (st != 0)
