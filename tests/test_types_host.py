"""CPU tests of the host-side Go-layer mirror (include/eges_types.hpp, eges_amd/host/): its
Transaction decoder / encoder, isProtectedV and Signer.Hash against the tx oracle on the
reference's own RLP vectors (rlp/decode_test.go, spliced into txdata as tests/test_gpu_rlp.py
does) plus a mutation fuzz, and the signer / sender-cache unit checks of tests/cpp/test_types.cpp
(Signer.Equal, MakeSigner, cache hits without any engine call). No engine compute here."""
import os
import random
import subprocess

import pytest

from oracle import txoracle as T
from test_gpu_rlp import build_cases

HERE = os.path.dirname(os.path.abspath(__file__))
DRIVER = os.path.join(HERE, "cpp", "test_types")


def run_driver(mode, lines, tmp_path):
    assert os.path.exists(DRIVER), "tests/cpp/test_types not built (build() / make -C eges_amd/host)"
    f = tmp_path / f"{mode}.txt"
    f.write_text("\n".join(lines) + "\n")
    p = subprocess.run([DRIVER, mode, str(f)], capture_output=True, text=True, timeout=600)
    return p


def encode(d):
    """EncodeRLP of a decoded txdata (rlp/encode.go: a nil recipient encodes as 0x80)."""
    return T.enc_list([T.enc_uint(d["nonce"]), T.enc_uint(d["price"]), T.enc_uint(d["gas"]),
                       T.enc_bytes(d["to"]) if d["to"] is not None else b"\x80", T.enc_uint(d["value"]),
                       T.enc_bytes(d["data"]), b"\x01" if d["is_geec"] else b"\x80", T.enc_uint(d["v"]),
                       T.enc_uint(d["r"]), T.enc_uint(d["s"])])


def fuzz_cases(n=400, seed=1):
    rnd = random.Random(seed)
    base = [c[0] for c in build_cases() if c[4] == "base"][0]
    out = []
    for _ in range(n):
        b = bytearray(base)
        op = rnd.randrange(4)
        if op == 0:
            b[rnd.randrange(len(b))] ^= 1 << rnd.randrange(8)
        elif op == 1:
            del b[rnd.randrange(len(b)):]
        elif op == 2:
            i = rnd.randrange(len(b))
            b[i:i] = bytes([rnd.randrange(256)])
        else:
            b[rnd.randrange(len(b))] = rnd.choice((0x00, 0x7F, 0x80, 0x81, 0xB8, 0xC0, 0xF8))
        out.append(bytes(b))
    return out


def test_mirror_decode_hash_protected(oracle, tmp_path):
    raws = [c[0] for c in build_cases()] + fuzz_cases()
    p = run_driver("cpu", [r.hex() for r in raws], tmp_path)
    out = p.stdout.splitlines()
    unit = [l for l in out if not l.startswith("vec ") and not l.startswith("failed")]
    assert unit and all(l.startswith("ok ") for l in unit), unit
    vec = [l.split() for l in out if l.startswith("vec ")]
    assert len(vec) == len(raws)
    n_ok = 0
    for raw, v in zip(raws, vec):
        try:
            d = T.decode_txdata(raw)
        except T.DecodeError:
            assert v[1] == "0", raw.hex()
            continue
        n_ok += 1
        # decoded, re-encoded as the reference encodes (equal to the input unless it used a
        # non-canonical-but-accepted form such as 0xC0 for the nil recipient), isProtectedV
        assert v[1:4] == ["1", "1" if encode(d) == raw else "0", "1" if T.is_protected_v(d["v"]) else "0"], (raw.hex(), v)
        assert v[4] == oracle.keccak256(T.signing_payload(d, 0, 0)).hex()
        # EIP155Signer.Hash is the EIP-155 payload whatever V is (Sender picks the hash, not Hash)
        assert v[5] == oracle.keccak256(T.signing_payload(dict(d, v=37), 2, 930412)).hex()
    assert n_ok > 50 and len(raws) - n_ok > 100
    assert p.returncode == 0, p.stdout[-2000:]
