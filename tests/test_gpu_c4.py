"""configs[3] (C4) on the GPU: the full 64M-signature batch through the device entry, every
address checked against the synthetic signer, an oracle sample across every pass boundary and a
1M random-index sample against the reference libsecp256k1 (oracle/_ref);
and the in-library multi-device split (hostpath.hip run_host with ndev > 1) and a small-grid device
run in child processes with the engine's test-only knobs (tests/gpu_child.py)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PASS = 1 << 21  # signatures per device pass (launch.h PASS_MAX)


def test_c4_full_64m_batch(engine, oracle):
    import torch
    n = 64 << 20  # BASELINE configs[3]: 64M signatures (one GPU's strong-scaled shard = the whole batch)
    msg, sig, exp = engine.synth_sign_dev(0, n, 0)
    addr = torch.empty((n, 20), dtype=torch.uint8, device=msg.device)
    st = torch.empty((n,), dtype=torch.uint8, device=msg.device)
    engine.ecrecover_batch_dev(msg, sig, addr=addr, status=st)
    torch.cuda.synchronize()
    assert int((st != 0).sum().item()) == 0
    assert torch.equal(addr, exp), "an address of the 64M batch differs from the signer's"
    # oracle sample: ~62 items around each of the 32 pass boundaries (the overlapped launches
    # alternate streams and workspaces there), 2,000 in total
    idx = []
    for b in range(0, n + 1, PASS):
        idx += [i for i in range(b - 31, b + 31) if 0 <= i < n]
    idx = np.array(sorted(set(idx))[:2000], np.int64)
    sel = torch.from_numpy(idx).to(msg.device)
    m, s, a = msg[sel].cpu().numpy(), sig[sel].cpu().numpy(), addr[sel].cpu().numpy()
    for j in range(len(idx)):
        ost, opub = oracle.recover_pubkey(m[j].tobytes(), s[j].tobytes())
        assert ost == 0 and oracle.pub_to_addr(opub) == a[j].tobytes(), int(idx[j])
    # a 1M random-index sample of the 64M batch against the reference libsecp256k1 itself
    # (oracle/_ref, its recovery + the address, on the host cores): independent of the GPU signer
    from oracle import RefLib, have_ref
    if have_ref():
        rng = np.random.default_rng(64)
        ridx = np.unique(rng.integers(0, n, size=(1 << 20) + (1 << 16)))[: 1 << 20].astype(np.int64)
        sel = torch.from_numpy(ridx).to(msg.device)
        m, s, a = msg[sel].cpu().numpy(), sig[sel].cpu().numpy(), addr[sel].cpu().numpy()
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
        _, raddr, ret = RefLib().ecrecover_batch_mt(m, s, threads)
        assert (ret == 1).all()
        bad = np.nonzero((raddr != a).any(axis=1))[0]
        assert bad.size == 0, ridx[bad[:10]].tolist()
    del msg, sig, exp, addr, st
    torch.cuda.empty_cache()


def _child(mode, env_extra, timeout=240):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "gpu_child.py"), mode], env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_logical_devices_shard_split():
    out = _child("logical_devices", {"EGES_TEST_LOGICAL_DEVICES": "2"})
    assert out["devices"] == 2
    assert out["same_as_single"] and out["correct"] and out["golden"], out


def test_small_resident_grid_multi_pass():
    """EGES_TEST_MAX_BLOCKS=8: grid_for_lane_serial raises a full pass to 256 blocks, 32x the
    resident grid; the workspace must cover it."""
    out = _child("small_grid", {"EGES_TEST_MAX_BLOCKS": "8"})
    assert out["ok_dev"] and out["ok_host"], out


def test_records_all_gather_over_rccl():
    """The optional records exchange (eges_amd.shard.all_gather_records) on device tensors
    through the "nccl" (RCCL) backend, world size 1, in a child process."""
    out = _child("allgather_nccl", {"EGES_TEST_PORT": str(29000 + os.getpid() % 1000)})
    assert out["ok"] and out["backend"] == "nccl", out

