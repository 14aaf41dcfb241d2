"""Child process for GPU tests that need the engine initialised under test-only knobs
(EGES_TEST_MAX_BLOCKS, EGES_TEST_LOGICAL_DEVICES), which are read once at eges_init. Run by
tests/test_gpu_c4.py as `python tests/gpu_child.py <mode>`; prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def tiled_golden(n):
    """The golden recover fixture tiled to n items: (msg, sig, pub, status)."""
    import numpy as np
    from conftest import load_golden
    g = load_golden("recover.npz")
    idx = np.arange(n) % g["msg"].shape[0]
    return g["msg"][idx], g["sig"][idx], g["pub"][idx], g["status"][idx]


def small_grid():
    """A device whose resident grid is far below the blocks a full pass needs: a multi-pass
    device batch and a multi-pass verify batch must still be bit-exact (the workspace is sized
    for the larger grid, engine.hip init_device)."""
    import numpy as np
    import torch
    import eges_amd
    from eges_amd._lib import lib
    eges_amd.init(1)
    n = (1 << 21) + 3001  # two passes of the device entry
    msg, sig, pub, st = tiled_golden(n)
    dev = torch.device("cuda", 0)
    pd = torch.empty((n, 65), dtype=torch.uint8, device=dev)
    _, _, sd = eges_amd.ecrecover_batch_dev(torch.from_numpy(msg).to(dev), torch.from_numpy(sig).to(dev), pub=pd)
    torch.cuda.synchronize()
    ok_dev = bool(np.array_equal(sd.cpu().numpy(), st) and np.array_equal(pd.cpu().numpy(), pub))
    # host-buffer entry (pipelined chunks) on the same small grid
    m2 = 300_001
    p2, _, s2 = eges_amd.ecrecover_batch(msg[:m2], sig[:m2])
    ok_host = bool(np.array_equal(s2, st[:m2]) and np.array_equal(p2, pub[:m2]))
    return {"ok_dev": ok_dev, "ok_host": ok_host, "devices": int(lib.eges_device_count())}


def logical_devices():
    """Two logical devices on one GPU: run_host splits a host-buffer batch into two contiguous
    shards on two threads (hostpath.hip run_host); the result must equal the device-resident
    single-device result byte for byte, and the synthetic signer's addresses."""
    import numpy as np
    import torch
    import eges_amd
    from eges_amd._lib import lib
    eges_amd.init(1)
    ndev = int(lib.eges_device_count())
    n = 400_003
    msg, sig, exp = eges_amd.synth_sign_dev(77_000_000, n, 0)
    pub_d = torch.empty((n, 65), dtype=torch.uint8, device=msg.device)
    _, addr_d, st_d = eges_amd.ecrecover_batch_dev(msg, sig, pub=pub_d)
    torch.cuda.synchronize()
    mh, sh = msg.cpu().numpy(), sig.cpu().numpy()
    pub, addr, st = eges_amd.ecrecover_batch(mh, sh)
    same = bool(np.array_equal(pub, pub_d.cpu().numpy()) and np.array_equal(addr, addr_d.cpu().numpy())
                and np.array_equal(st, st_d.cpu().numpy()))
    correct = bool((st == 0).all() and np.array_equal(addr, exp.cpu().numpy()))
    # golden fixture through the split path too (every reject class)
    gm, gs, gp, gst = tiled_golden(200_000)
    p3, _, s3 = eges_amd.ecrecover_batch(gm, gs)
    golden = bool(np.array_equal(s3, gst) and np.array_equal(p3, gp))
    return {"devices": ndev, "same_as_single": same, "correct": correct, "golden": golden}


def allgather_nccl():
    """eges_amd.shard.all_gather_records over the "nccl" backend (RCCL), world size 1: the
    device-resident (address, status) records of a golden batch go through the collective and
    come back equal (the exchange of SURVEY §8(e) on the real backend; N > 1 is gloo-tested)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    import eges_amd
    from eges_amd.shard import all_gather_records
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("EGES_TEST_PORT", "29541"),
                      RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    eges_amd.init(1)
    n = 4099
    msg, sig, pub, st = tiled_golden(n)
    _, addr, sd = eges_amd.ecrecover_batch_dev(torch.from_numpy(msg).to(dev), torch.from_numpy(sig).to(dev))
    rec = torch.cat([addr.reshape(n, 20), sd.reshape(n, 1).to(torch.uint8)], 1).contiguous()
    got = all_gather_records(rec, n)
    torch.cuda.synchronize()
    ok = bool(got.device.type == "cuda" and torch.equal(got, rec)
              and np.array_equal(got[:, 20].cpu().numpy(), st.astype(np.uint8)))
    backend = dist.get_backend()
    dist.destroy_process_group()
    return {"ok": ok, "backend": backend}


def other_process_kernels():
    """A second process on the same GPU (test_gpu_resident.py): a device-resident 1M batch,
    timed with HIP events each time a line "go" arrives on stdin; prints one number per launch
    (ms), then "bye" at EOF. The engine of this process never starts a resident server."""
    import torch
    import eges_amd
    eges_amd.init(1)
    eges_amd.set_knob("EGES_RESIDENT", 0)
    n = 1 << 20
    msg, sig, exp = eges_amd.synth_sign_dev(5 << 30, n, 0)
    addr = torch.empty((n, 20), dtype=torch.uint8, device=msg.device)
    st = torch.empty((n,), dtype=torch.uint8, device=msg.device)
    s = torch.cuda.Stream()
    for _ in range(2):
        eges_amd.ecrecover_batch_dev(msg, sig, addr=addr, status=st, stream=s.cuda_stream)
    torch.cuda.synchronize()
    print("ready", flush=True)
    ok = True
    for line in sys.stdin:
        if line.strip() != "go":
            continue
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        eges_amd.ecrecover_batch_dev(msg, sig, addr=addr, status=st, stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(addr, exp))
        print(f"{e0.elapsed_time(e1):.4f}", flush=True)
    return {"ok": ok}


if __name__ == "__main__":
    mode = sys.argv[1]
    out = {"small_grid": small_grid, "logical_devices": logical_devices, "allgather_nccl": allgather_nccl,
           "other_process_kernels": other_process_kernels}[mode]()
    print(json.dumps(out), flush=True)
