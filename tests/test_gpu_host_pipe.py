"""Host-buffer shards of at least 512k items (hostpath.hip run_host_shard): the chunked path (the
copy stream moves chunk i + 1 in while chunk i computes) on ragged batches of several kinds,
against the fixtures item for item. Round 4's pinned-slot pipeline (run_host_pipe) and second
compute stream measured slower and were removed in round 5."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


class knobs:
    def __init__(self, engine, kv):
        self.engine, self.kv = engine, kv

    def __enter__(self):
        self.old = {k: self.engine.get_knob(k) for k in self.kv}
        for k, v in self.kv.items():
            self.engine.set_knob(k, v)

    def __exit__(self, *a):
        for k, v in self.old.items():
            self.engine.set_knob(k, v)


def _tile(a, n):
    rep = -(-n // len(a))
    return np.ascontiguousarray(np.concatenate([a] * rep)[:n])


def test_chunked_path_golden_tiled(engine):
    """the chunked host path on a ragged 5-chunk batch: recovery and types.Sender rows"""
    g = load_golden("recover.npz")
    n = 600011
    msg, sig = _tile(g["msg"], n), _tile(g["sig"], n)
    with knobs(engine, {"EGES_HOST_PARTS": 5}):
        pub, addr, st = engine.ecrecover_batch(msg, sig)
    assert np.array_equal(st, _tile(g["status"], n))
    assert np.array_equal(pub, _tile(g["pub"], n))
    gs = load_golden("sender.npz")
    sel = np.nonzero((gs["signer"] == 2) & (gs["chain_id"] == 930412))[0]
    cols = {k: _tile(gs[k][sel], n) for k in ("sighash", "r", "s", "v", "vflags", "status", "addr")}
    with knobs(engine, {"EGES_HOST_PARTS": 5}):
        a, s_ = engine.sender_batch(cols["sighash"], cols["r"], cols["s"], cols["v"], cols["vflags"], 2, 930412)
    assert np.array_equal(s_, cols["status"]) and np.array_equal(a, cols["addr"])


def test_chunked_path_verify_golden_tiled(engine):
    g = load_golden("verify.npz")
    n = 524309
    cols = {k: _tile(g[k], n) for k in ("pub", "publen", "msg", "sig", "ok")}
    with knobs(engine, {"EGES_HOST_PARTS": 3}):
        ok = engine.verify_batch(cols["pub"], cols["publen"], cols["msg"], cols["sig"])
    assert np.array_equal(ok, cols["ok"])


def _golden_addr(g):
    """The golden fixture's addresses: Keccak-256(pub[1:])[12:] for every accepted item, zeros
    for the rejected ones (crypto.go:194-197; the engine's host Keccak, pinned by the KATs)."""
    import eges_amd
    out = np.zeros((len(g["status"]), 20), np.uint8)
    for i in np.nonzero(g["status"] == 0)[0]:
        out[i] = np.frombuffer(eges_amd.keccak256(g["pub"][i][1:].tobytes())[12:], np.uint8)
    return out


@pytest.mark.parametrize("n", [600011, 1 << 20, 1 << 21])
def test_one_launch_path_golden_tiled(engine, n):
    """run_host_one (the default for host-buffer ecrecover shards of 512k .. 2M): one lane-serial
    launch fed piece by piece, outputs copied block by block; every reject class of the golden
    fixture, ragged and at the chunk limit, statuses, keys and addresses item for item, and the
    same bytes as the chunked path (EGES_HOST_ONE=0)."""
    g = load_golden("recover.npz")
    msg, sig = _tile(g["msg"], n), _tile(g["sig"], n)
    pub, addr, st = engine.ecrecover_batch(msg, sig)
    assert np.array_equal(st, _tile(g["status"], n))
    assert np.array_equal(pub, _tile(g["pub"], n))
    assert np.array_equal(addr, _tile(_golden_addr(g), n))
    if n == 600011:
        with knobs(engine, {"EGES_HOST_ONE": 0}):
            pub0, addr0, st0 = engine.ecrecover_batch(msg, sig)
        assert np.array_equal(pub0, pub) and np.array_equal(addr0, addr) and np.array_equal(st0, st)
        # addresses only (no key output), then keys only: the pinned output layout without a part
        _, a2, s2 = engine.ecrecover_batch(msg, sig, want_pub=False)
        assert np.array_equal(a2, addr) and np.array_equal(s2, st)
        p3, _, s3 = engine.ecrecover_batch(msg, sig, want_addr=False)
        assert np.array_equal(p3, pub) and np.array_equal(s3, st)


def test_one_launch_path_synthetic_repeat(engine):
    """1M synthetic signatures through the one-launch form, four calls in a row alternating two
    different batches into the same output arrays: the staging and output buffers hold the
    other batch's bytes at every call, so an input read before its piece was published, or an
    output copied before its block was done, shows up as a wrong address (round 5: glibc's
    non-temporal memcpy stores overtook the piece word until it was fenced)."""
    import torch
    n = 1 << 20
    sets = []
    for first in (123_456_789, 987_654_321):
        msg, sig, exp = engine.synth_sign_dev(first, n, 0)
        torch.cuda.synchronize()
        sets.append((msg.cpu().numpy(), sig.cpu().numpy(), exp.cpu().numpy()))
    oa, os_ = np.zeros((n, 20), np.uint8), np.zeros(n, np.uint8)
    for i in range(4):
        mh, sh, eh = sets[i % 2]
        os_.fill(0xEE)
        engine.ecrecover_batch(mh, sh, want_pub=False, out_addr=oa, out_status=os_)
        bad = np.nonzero((oa != eh).any(axis=1))[0]
        assert (os_ == 0).all() and bad.size == 0, (i, bad.size, bad[:10].tolist())
