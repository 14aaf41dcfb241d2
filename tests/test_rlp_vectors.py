"""The reference's own RLP decoder vectors (rlp/decode_test.go, transcribed as data into
tests/golden/rlp_decode.json) against the tx oracle's decoder (oracle/txoracle.py), per Go
target type; and the chain-id mismatch vector (core/types/transaction_signing_test.go:118-138,
tests/golden/chain_id.json) through the oracle's sender. The GPU side of both is in
tests/test_gpu_rlp.py: every rule here must give EGES_DECODE_FAILED there."""
import json
import os

import pytest

from oracle import txoracle as T

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


def reader_for(typ):
    """Go target type of a decodeTests vector -> reader(stream)."""
    if typ == "bool":
        return lambda s: s.boolean()
    if typ == "uint32":
        return lambda s: s.uint(32)
    if typ == "uint":
        return lambda s: s.uint(64)
    if typ == "bytes":
        return lambda s: s.bytes_()
    if typ == "bigint":
        return lambda s: s.bigint()
    if typ.startswith("bytearray:"):
        n = int(typ.split(":")[1])
        return lambda s: s.byte_array(n)
    if typ == "struct:uint,bytes":  # simplestruct{A uint; B string}
        return lambda s: T.decode_struct(s, [lambda: s.uint(64), s.bytes_])
    raise KeyError(typ)


STREAM_CALLS = {"Uint": lambda s: s.uint(64), "Bytes": lambda s: s.bytes_(), "Bool": lambda s: s.boolean(),
                "Kind": lambda s: s.kind(), "List": lambda s: s.list_start()}


def norm(v):
    if isinstance(v, bytes):
        return v.hex()
    if isinstance(v, list):
        return [norm(x) for x in v]
    return v


@pytest.mark.parametrize("vec", load("rlp_decode.json")["decode"], ids=lambda v: f"L{v['line']}-{v['type']}")
def test_decode_vectors(vec):
    raw = bytes.fromhex(vec["input"])
    rd = reader_for(vec["type"])
    if vec["ok"]:
        assert norm(T.decode_bytes(raw, rd)) == vec["value"]
    else:
        with pytest.raises(T.DecodeError):
            T.decode_bytes(raw, rd)


@pytest.mark.parametrize("vec", load("rlp_decode.json")["stream"], ids=lambda v: f"L{v['line']}-{v['call']}")
def test_stream_vectors(vec):
    s = T._Stream(bytes.fromhex(vec["input"]))
    call = STREAM_CALLS[vec["call"]]
    if vec["ok"]:
        assert norm(call(s)) == vec["value"]
    else:
        with pytest.raises(T.DecodeError):
            call(s)


def test_chain_id_mismatch_vector(oracle):
    """TestChainId: the tx signed under EIP155Signer(1) fails under EIP155Signer(2) with
    ErrInvalidChainId and recovers defaultTestKey's address under EIP155Signer(1); the 9-field
    original does not decode as this fork's 10-field txdata."""
    v = load("chain_id.json")
    raw10 = bytes.fromhex(v["raw10"])
    for case in v["cases"]:
        st, addr, h = T.sender_raw(oracle, raw10, 2, case["signer_chain_id"])
        assert st == case["status"]
        if st == 0:
            assert addr.hex() == case["addr"] and h.hex() == v["sighash_chain1"]
    st, _, _ = T.sender_raw(oracle, bytes.fromhex(v["raw9"]), 2, 1)
    assert st == T.DECODE_FAILED
