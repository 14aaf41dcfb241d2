"""GPU parity of the wire-format sender path (eges_sender_raw_batch / _dev, k_txhash.hip):
RLP decode + signing hash + Keccak + recovery on the GPU, checked item by item (status, sighash,
address) against oracle/txoracle.py — on the reference's own vectors (10-field Geec form, and
the 9-field originals that the Geec struct rejects), the decode-rule table of test_txoracle.py,
a seeded mutation fuzz over signed Geec transactions (truncations, byte flips, non-canonical
items, nil `to` as 0xC0, IsGeecTxn values, unprotected / wide / mismatched V, multi-block
payloads, 9-field lists, string headers) and a 1000-tx Geec block through the device entry;
plus the EVM ECRECOVER precompile batch (eges_ecrecover_precompile_batch / _dev)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import txoracle as T

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("wire_form")]

CHAIN = 930412  # genesis.json.template chainId
SIGNERS = (0, 1, 2)


def _check(engine, oracle, raws, signer, chain_id):
    addr, st, sh = engine.sender_raw_batch(raws, signer, chain_id, want_sighash=True)
    for i, raw in enumerate(raws):
        ost, oaddr, oh = T.sender_raw(oracle, raw, signer, chain_id)
        assert int(st[i]) == ost, (i, raw.hex(), int(st[i]), ost)
        assert addr[i].tobytes() == oaddr, (i, raw.hex())
        if ost != T.DECODE_FAILED:
            assert sh[i].tobytes() == oh, (i, raw.hex())
        else:
            assert not sh[i].any()
    return addr, st


def test_reference_vectors(engine, oracle):
    with open(os.path.join(GOLDEN, "vectors.json")) as f:
        items = json.load(f)["items"]
    vs = items["eip155_vitalik"]
    raws = [T.to_geec10(bytes.fromhex(t["rlp"])) for t in vs["txs"]]
    addr, st = _check(engine, oracle, raws, 2, vs["chain_id"])
    assert (st == 0).all()
    assert [a.tobytes().hex() for a in addr] == [t["addr"] for t in vs["txs"]]
    nine = [bytes.fromhex(t["rlp"]) for t in vs["txs"]]
    _, st9 = _check(engine, oracle, nine, 2, vs["chain_id"])
    assert (st9 == T.DECODE_FAILED).all()
    hv = items["homestead_recipients"]
    for signer in SIGNERS:
        addr, st = _check(engine, oracle, [T.to_geec10(bytes.fromhex(x)) for x in hv["txs"]], signer, CHAIN)
        assert (st == 0).all() and all(a.tobytes().hex() == hv["addr"] for a in addr)


def test_decode_rule_table(engine, oracle):
    from test_txoracle import DECODE_CASES
    raws = [raw for _, raw, _ in DECODE_CASES] + [b"", b"\x80", b"\xc0", b"\xf8"]
    for signer in SIGNERS:
        _, st = _check(engine, oracle, raws, signer, CHAIN)
        for (name, _, ok), s in zip(DECODE_CASES, st):
            assert (s != T.DECODE_FAILED) == ok, name


def _geec_fields(i, rng, payload_len):
    to = None if i % 7 == 0 else rng.bytes(20)
    return dict(nonce=int(rng.integers(0, 1 << 62)) if i % 3 else i, price=int(rng.integers(0, 1 << 40)),
                gas=21000 + i, to=to, value=int(rng.integers(0, 1 << 60)) if i % 4 else 0,
                data=rng.bytes(payload_len), is_geec=bool(i % 2))


def _encode(d, v, r, s, geec_item=None, to_item=None):
    to_enc = to_item if to_item is not None else (T.enc_bytes(d["to"]) if d["to"] is not None else b"\x80")
    items = [T.enc_uint(d["nonce"]), T.enc_uint(d["price"]), T.enc_uint(d["gas"]), to_enc, T.enc_uint(d["value"]),
             T.enc_bytes(d["data"]), geec_item if geec_item is not None else (b"\x01" if d["is_geec"] else b"\x80"),
             T.enc_uint(v), T.enc_uint(r), T.enc_uint(s)]
    return T.enc_list(items)


def _signed_txs(engine, first, n, payload_fn, rng, protected=True):
    """n signed Geec transactions (EIP-155 V when `protected`, else V = 27/28), signed on the GPU
    with the synthetic keys of indices first.. over the oracle's signing hash.
    -> (raws, fields, sig (n,65), expected addr (n,20))."""
    import torch
    fields = [_geec_fields(first + i, rng, payload_fn(i)) for i in range(n)]
    h = np.zeros((n, 32), np.uint8)
    for i, d in enumerate(fields):
        h[i] = np.frombuffer(engine.keccak256(T.signing_payload(dict(d, v=37 if protected else 27), 2, CHAIN)),
                             np.uint8)
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(h).to("cuda:0"), first)
    torch.cuda.synchronize()
    sig, exp = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    raws = []
    for i, d in enumerate(fields):
        rec = int(sig[i, 64])
        v = rec + 35 + 2 * CHAIN if protected else rec + 27
        raws.append(_encode(d, v, int.from_bytes(sig[i, :32].tobytes(), "big"),
                            int.from_bytes(sig[i, 32:64].tobytes(), "big")))
    return raws, fields, sig, exp


def _mutate(raw, d, sig, rng):
    """One seeded mutation of a signed tx -> its new encoding (the oracle decides the outcome)."""
    k = int(rng.integers(0, 14))
    r = int.from_bytes(sig[:32].tobytes(), "big")
    s = int.from_bytes(sig[32:64].tobytes(), "big")
    v = int(sig[64]) + 35 + 2 * CHAIN
    if k == 0:
        return raw
    if k == 1:  # one bit flipped anywhere
        b = bytearray(raw)
        j = int(rng.integers(0, len(b)))
        b[j] ^= 1 << int(rng.integers(0, 8))
        return bytes(b)
    if k == 2:  # truncated
        return raw[:int(rng.integers(0, len(raw)))]
    if k == 3:  # trailing byte
        return raw + bytes([int(rng.integers(0, 256))])
    if k == 4:  # payload changed: the signature no longer matches (another sender or a failure)
        return _encode(dict(d, data=d["data"] + b"\x00"), v, r, s)
    if k == 5:
        return _encode(d, v, r, s, geec_item=[b"\x01", b"\x00", b"\x02", b"\x81\x01", b"\x80", b"\xc0"][int(rng.integers(0, 6))])
    if k == 6:  # unprotected V: Frontier hash
        return _encode(d, int(sig[64]) + 27, r, s)
    if k == 7:  # chain id mismatch
        return _encode(d, v + 2, r, s)
    if k == 8:  # V wider than 256 bits
        return _encode(d, v + (1 << 300), r, s)
    if k == 9:  # R wider than 256 bits
        return _encode(d, v, r + (1 << 256), s)
    if k == 10:  # high S
        return _encode(d, v, r, (1 << 256) - 1 - s)
    if k == 11:  # standard 9-field encoding
        return T.enc_list([T.enc_uint(d["nonce"]), T.enc_uint(d["price"]), T.enc_uint(d["gas"]),
                           T.enc_bytes(d["to"]) if d["to"] is not None else b"\x80", T.enc_uint(d["value"]),
                           T.enc_bytes(d["data"]), T.enc_uint(v), T.enc_uint(r), T.enc_uint(s)])
    if k == 12:  # the list body under a string header
        body = raw[1:] if raw[0] < 0xf8 else raw[1 + raw[0] - 0xf7:]
        return bytes([0xb9]) + len(body).to_bytes(2, "big") + body
    # k == 13: nil `to` sent as an empty list (decodes as nil; the hash re-encodes it as 0x80)
    return _encode(d, v, r, s, to_item=b"\xc0") if d["to"] is None else raw


def test_mutation_fuzz(engine, oracle):
    rng = np.random.default_rng(2024)
    n = 1500
    raws, fields, sig, exp = _signed_txs(engine, 10_000, n, lambda i: [0, 1, 55, 100, 135, 136, 300, 2000][i % 8], rng)
    addr, st = _check(engine, oracle, raws, 2, CHAIN)  # unmutated: the synthetic keys' addresses
    assert (st == 0).all() and np.array_equal(addr, exp)
    mutated = [_mutate(raws[i], fields[i], sig[i], rng) for i in range(n)]
    seen = set()
    # batches up to 8192 items decode one transaction per wave (k_txhash.hip), larger ones one per
    # lane: the lane-serial form (forced by EGES_TXROWS_WAVE_MAX=0) must agree item by item
    for signer in SIGNERS:
        addr, st = _check(engine, oracle, mutated, signer, CHAIN)
        seen |= set(np.unique(st).tolist())
        _, _, sh = engine.sender_raw_batch(mutated, signer, CHAIN, want_sighash=True)
        with engine.knob("EGES_TXROWS_WAVE_MAX", 0):
            addr1, st1, sh1 = engine.sender_raw_batch(mutated, signer, CHAIN, want_sighash=True)
        assert np.array_equal(st1, st) and np.array_equal(addr1, addr) and np.array_equal(sh1, sh)
    assert {0, 1, 2, T.DECODE_FAILED} <= seen, seen


def test_unprotected_txs(engine, oracle):
    rng = np.random.default_rng(5)
    raws, _, _, exp = _signed_txs(engine, 50_000, 64, lambda i: 100, rng, protected=False)
    for signer in SIGNERS:
        addr, st = _check(engine, oracle, raws, signer, CHAIN)
        assert (st == 0).all() and np.array_equal(addr, exp)


def test_geec_block_device_entry(engine, oracle):
    """C3's shape: 1000 EIP-155 transfers with a 100-byte payload, resident on the device."""
    import torch
    rng = np.random.default_rng(77)
    raws, _, _, exp = _signed_txs(engine, 90_000, 1000, lambda i: 100, rng)
    raw, off = engine.pack_raw(raws)
    raw_d = torch.from_numpy(raw).to("cuda:0")
    off_d = torch.from_numpy(off.astype(np.int64)).to("cuda:0")
    addr_d, st_d = engine.sender_raw_batch_dev(raw_d, off_d, 2, CHAIN)
    torch.cuda.synchronize()
    assert (st_d.cpu().numpy() == 0).all() and np.array_equal(addr_d.cpu().numpy(), exp)
    for i in (0, 511, 999):
        ost, oaddr, _ = T.sender_raw(oracle, raws[i], 2, CHAIN)
        assert ost == 0 and oaddr == exp[i].tobytes()
    # offsets that are positions in a larger buffer: only differences from offsets[0] matter
    a2, s2 = engine.sender_raw_batch_dev(raw_d, off_d + 37, 2, CHAIN)
    torch.cuda.synchronize()
    assert torch.equal(a2, addr_d) and torch.equal(s2, st_d)


def test_ecrecover_precompile(engine, oracle):
    """EVM ECRECOVER precompile (core/vm/contracts.go:77-101) through eges_ecrecover_precompile_batch:
    the reference's sample (contracts_test.go:390-395), the pre-check cases, and synthetic
    signatures with seeded mutations, every output word and status against the oracle."""
    import torch
    from test_txoracle import PRECOMPILE_VECTOR, precompile_cases
    inputs = [bytes.fromhex(PRECOMPILE_VECTOR[0])] + [c for c, _ in precompile_cases()]
    msg, sig, exp = engine.synth_sign_dev(123_000, 600, 0)
    torch.cuda.synchronize()
    msg, sig, exp = msg.cpu().numpy(), sig.cpu().numpy(), exp.cpu().numpy()
    rng = np.random.default_rng(31)
    for i in range(600):
        word = bytes(31) + bytes([27 + int(sig[i, 64])])
        x = msg[i].tobytes() + word + sig[i, :64].tobytes()
        k = i % 6
        if k == 1:
            j = int(rng.integers(0, 128))
            x = x[:j] + bytes([x[j] ^ (1 << int(rng.integers(0, 8)))]) + x[j + 1:]
        elif k == 2:
            x = x[:int(rng.integers(0, 129))]
        elif k == 3:
            x = x + rng.bytes(int(rng.integers(1, 64)))
        inputs.append(x)
    out, st = engine.ecrecover_precompile_batch(inputs)
    for i, x in enumerate(inputs):
        ost, oout = T.precompile_ecrecover(oracle, x)
        assert int(st[i]) == ost, (i, x.hex())
        assert out[i].tobytes() == (oout if oout is not None else bytes(32)), (i, x.hex())
    assert out[0].tobytes().hex() == PRECOMPILE_VECTOR[1]
    base = len(inputs) - 600
    for i in range(0, 600, 6):  # unmutated synthetic items: the signer's address
        assert st[base + i] == 0 and out[base + i, 12:].tobytes() == exp[i].tobytes()
    # device entry, fixed 128-byte records
    buf = np.zeros((len(inputs), 128), np.uint8)
    ln = np.zeros(len(inputs), np.int32)
    for i, x in enumerate(inputs):
        x = x[:128]
        buf[i, :len(x)] = np.frombuffer(x, np.uint8)
        ln[i] = len(x)
    o2, s2 = engine.ecrecover_precompile_batch_dev(torch.from_numpy(buf).cuda(), torch.from_numpy(ln).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(o2.cpu().numpy(), out) and np.array_equal(s2.cpu().numpy(), st)


def test_short_tx_with_long_signing_header(engine, oracle):
    """Unsigned Geec transactions with short payloads: the encoding's list header is one byte (a
    body <= 55 bytes) while the EIP-155 signing payload's is two (the chain-id tail pushes it past
    55). Regression: the signing-payload reader once loaded the byte before such an encoding (an
    aperture violation when it sat at the start of a wave's LDS stage, found by
    tools/sanitize_host.cpp). Alone, first in a batch, between signed items, and as an unselected
    (decode-only) and a selected list of a block; every result against the oracle."""
    from eges_amd import txs
    short = [txs.encode_geec_tx(0, 1, 21000, b"\x22" * 20, 7, b"\x41" * n, True, 0, 0, 0) for n in (22, 23, 10, 30)]
    assert len(short[0]) == 55 and len(short[1]) == 56  # one-byte list headers; payload bodies 56, 57
    for signer in SIGNERS:
        _check(engine, oracle, short, signer, CHAIN)
        _check(engine, oracle, short[:1], signer, CHAIN)
    tx_raws = _signed_txs(engine, 770_000, 40, lambda i: i % 50, np.random.default_rng(5))[0]
    mixed = [short[1]] + tx_raws[:20] + short + tx_raws[20:]
    _check(engine, oracle, mixed, 2, CHAIN)
    for lists in (0, 2, 4, 7):
        raw = txs.geec_extblock(short[:2], short, tx_raws)
        addr, st, counts, bst = engine.block_senders_raw(raw, lists=lists)
        ost, oaddr, _, obst = T.block_senders(oracle, raw, lists, 2, txs.GEEC_CHAIN_ID)
        assert bst == obst and st.tolist() == ost and [a.tobytes() for a in addr] == oaddr, lists
