"""A whole Geec block through eges_block_senders_raw:
a synthetic 1000-transaction block (configs[2]'s shape: EIP-155 transfers with a 100-byte
payload in Txs) plus the leader's unsigned FakeTxs padding and GeecTxs (consensus/geec/geec.go:
333-339, geec_api.go:33-35), every selected item against the tx oracle (oracle/txoracle.py
block_senders) item for item, and the block-level status of a block with one undecodable tx."""
import numpy as np
import pytest

from eges_amd import txs
from oracle import txoracle as T

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("wire_form")]


def signed_block(engine, first, n, payload=100):
    import torch
    sighash = txs.geec_block(first, n, payload=payload)
    sig_d, exp_d = engine.synth_sign_msg_dev(torch.from_numpy(sighash).to("cuda:0"), first)
    torch.cuda.synchronize()
    sig = sig_d.cpu().numpy()
    return txs.geec_block_raw(first, sig, payload=payload), exp_d.cpu().numpy()


def test_geec_block_1000_txs(engine, oracle):
    tx_raws, exp = signed_block(engine, 880_000, 1000)
    fake = [txs.fake_tx(data_len=100) for _ in range(40)]
    geec = [txs.fake_tx(data_len=23, is_geec=True, data=b"geec udp txn %03d......." % i) for i in range(12)]
    raw = txs.geec_extblock(fake, geec, tx_raws)
    # Txs only: the signed transfers
    addr, st, counts, bst = engine.block_senders_raw(raw, lists=txs_mask("txs"))
    assert bst == 0 and counts.tolist() == [40, 12, 1000]
    assert (st == 0).all() and np.array_equal(addr, exp)
    # all three lists, against the oracle item for item
    addr, st, counts, bst = engine.block_senders_raw(raw, lists=7)
    osts, oaddrs, ocounts, obst = T.block_senders(oracle, raw, 7, 2, txs.GEEC_CHAIN_ID)
    assert counts.tolist() == ocounts and bst == obst == 0
    assert st.tolist() == osts
    assert [a.tobytes() for a in addr] == oaddrs
    # the unsigned placeholders (V = R = S = 0) fail as types.Sender would: ErrInvalidChainId
    assert (st[:52] == 1).all() and (st[52:] == 0).all()


def test_geec_block_with_undecodable_tx(engine, oracle):
    tx_raws, exp = signed_block(engine, 990_000, 64)
    bad = T.enc_list([tx_raws[17][2:-5]])  # a list whose single element is not a txdata
    tx_raws = tx_raws[:17] + [bad] + tx_raws[18:]
    raw = txs.geec_extblock([], [], tx_raws)
    addr, st, counts, bst = engine.block_senders_raw(raw, lists=4)
    osts, oaddrs, _, obst = T.block_senders(oracle, raw, 4, 2, txs.GEEC_CHAIN_ID)
    assert bst == obst == T.DECODE_FAILED
    assert st.tolist() == osts and int(st[17]) == T.DECODE_FAILED
    assert [a.tobytes() for a in addr] == oaddrs
    ok = np.arange(64) != 17
    assert np.array_equal(addr[ok], exp[ok])


def test_undecodable_tx_in_an_unselected_list(engine, oracle):
    """rlp.DecodeBytes(block) decodes FakeTxs and GeecTxs too: a Txs-only call (the Geec
    validator's selection) still fails a block whose FakeTx does not decode."""
    tx_raws, exp = signed_block(engine, 991_000, 32)
    fake = [txs.fake_tx(data_len=100) for _ in range(5)]
    fake[3] = T.enc_list([fake[3][2:-7]])  # not a txdata
    geec = [txs.fake_tx(data_len=23, is_geec=True, data=b"geec udp txn %03d......." % i) for i in range(3)]
    for f, g, bad in ((fake, geec, True), (geec, fake, True), (geec, geec, False)):
        raw = txs.geec_extblock(f, g, tx_raws)
        addr, st, counts, bst = engine.block_senders_raw(raw, lists=txs_mask("txs"))
        _, _, _, obst = T.block_senders(oracle, raw, txs_mask("txs"), 2, txs.GEEC_CHAIN_ID)
        assert bst == obst == (T.DECODE_FAILED if bad else 0)
        assert (st == 0).all() and np.array_equal(addr, exp)  # the selected list is still recovered


def txs_mask(name):
    from eges_amd import _lib
    return {"fake": _lib.LIST_FAKE, "geec": _lib.LIST_GEEC, "txs": _lib.LIST_TXS}[name]
