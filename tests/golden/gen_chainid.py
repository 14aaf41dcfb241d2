#!/usr/bin/env python3
"""Generate tests/golden/chain_id.json: the reference's chain-id mismatch vector.

TEST INFRASTRUCTURE (build container only: needs /root/reference for oracle/_ref).
core/types/transaction_signing_test.go:118-138 (TestChainId): defaultTestKey
(core/types/transaction_test.go:82-86) signs NewTransaction(0, common.Address{}, 0, 0, 0, nil)
with NewEIP155Signer(1); Sender(NewEIP155Signer(2), tx) must be ErrInvalidChainId and
Sender(NewEIP155Signer(1), tx) must succeed. SignTx goes through crypto.Sign ->
secp256k1.Sign (RFC6979 nonces, crypto/secp256k1/secp256.go:70-99), so the signature is
deterministic; it is produced here by the reference libsecp256k1 compiled in place.
The transaction is written both as the standard 9-field RLP and as this fork's 10-field Geec
txdata (IsGeecTxn = false before V, core/types/transaction.go:59-76).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import (N, Ref, rlp_bytes, rlp_int, rlp_list, tx_sighash)  # noqa: E402

KEY = int("45a915e4d060149eb4365960e6a7a45f334393093061116b197e3240065ff2d8", 16)  # transaction_test.go:83


def main():
    ref = Ref()
    to = bytes(20)  # common.Address{}
    h = tx_sighash(ref, 0, 0, 0, to, 0, b"", chain_id=1)
    sig = ref.sign(h, KEY)
    r, s, recid = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:64], "big"), sig[64]
    assert 0 < s <= N // 2
    v = recid + 35 + 2 * 1  # EIP155Signer.SignatureValues (transaction_signing.go:141-152)
    head = [rlp_int(0), rlp_int(0), rlp_int(0), rlp_bytes(to), rlp_int(0), rlp_bytes(b"")]
    tail = [rlp_int(v), rlp_int(r), rlp_int(s)]
    raw9 = rlp_list(head + tail)
    raw10 = rlp_list(head + [rlp_bytes(b"")] + tail)  # IsGeecTxn = false encodes as 0x80
    addr = ref.addr(ref.pubkey(KEY))
    st, pub = ref.ecrecover(h, sig)
    assert st == 0 and ref.addr(pub) == addr
    doc = {"cite": "core/types/transaction_signing_test.go:118-138 (TestChainId), key transaction_test.go:82-86",
           "generator": "tests/golden/gen_chainid.py (reference libsecp256k1 RFC6979 signature, oracle/_ref)",
           "key": f"{KEY:064x}", "sighash_chain1": h.hex(), "sig": sig.hex(), "v": v,
           "raw9": raw9.hex(), "raw10": raw10.hex(), "addr": addr.hex(),
           "cases": [{"signer_chain_id": 2, "status": 1, "note": "ErrInvalidChainId"},
                     {"signer_chain_id": 1, "status": 0, "addr": addr.hex()}]}
    with open(os.path.join(HERE, "chain_id.json"), "w") as f:
        json.dump(doc, f, indent=1, sort_keys=True)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
