"""Host-buffer shards of at least 512k items (hostpath.hip run_host_shard): the chunked path (the
copy stream moves chunk i + 1 in while chunk i computes) on ragged batches of several kinds,
against the fixtures item for item. Round 4's pinned-slot pipeline (run_host_pipe) and second
compute stream, and round 5's one-launch form fed piece by piece (profiles/r05), measured slower
and were removed."""
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



def test_host_gens_above_grid_mult(engine):
    """EGES_HOST_GENS larger than the device's EGES_GRID_MULT (default 2): the chunk launch's
    grid is clamped to the generations the workspace was sized for (route.hip
    launch_recover_pass) instead of being refused with EGES_E_HIP. Two chunks of
    ~300k items each would ask for more blocks than ws_blocks at 8 generations."""
    g = load_golden("recover.npz")
    n = 600011
    msg, sig = _tile(g["msg"], n), _tile(g["sig"], n)
    with knobs(engine, {"EGES_HOST_PARTS": 2, "EGES_HOST_GENS": 8}):
        pub, addr, st = engine.ecrecover_batch(msg, sig)
    assert np.array_equal(st, _tile(g["status"], n))
    assert np.array_equal(pub, _tile(g["pub"], n))
