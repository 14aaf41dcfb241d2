#!/usr/bin/env python3
"""bench.py — secp256k1 ecrecover + Keccak address throughput on MI355X.

Metric (BASELINE.json): "secp256k1 ecrecover+address/sec at 1/8 MI355X; % of INT32 VALU peak".
Workload (BASELINE.json configs[1]): 1M random-key secp256k1 signatures, batch ecrecover +
Keccak address on one MI355X. One step = one pass of the hot path over the per-GPU batch
(device-resident inputs -> 20-byte addresses + status bytes). Multi-GPU: one process per GPU
(torch.distributed.run), each rank recovers its own contiguous index shard of the synthetic
signature stream — no data-path collective ("scaling": "weak"); a barrier brackets the timed
region and the max time over ranks is reported.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic work per recovered address: INT32 lane-ops of the reference
# algorithm = 80 x 3085.2 field ops + 128 x 301 scalar ops + 6,300 (Keccak-f) = 291,644.
W_RECOVER = 291_644
# INT32 VALU peak of one MI355X for the multiply/carry instruction class the kernel is made of
# (256 CU x 64 lane-ops/clk x 2.4 GHz; tools/ubench_valu.hip measures
# v_mad_u64_u32 / v_add_co / v_addc at 4.4-4.9 cyc per wave64 instruction per SIMD, i.e. this
# rate; only v_add_u32/v_bitop3 issue at the 2x rate).
PEAK_INT32_OPS = 256 * 64 * 2.4e9  # 3.93e13 lane-ops/s


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1 << 20, help="signatures per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def cpu_baseline(msg_h, sig_h, target_s):
    """Reference libsecp256k1 (compiled in place, oracle/_ref) on the host cores: the
    goroutine-parallel types.Sender/Ecrecover path restated as one pthread per core.
    Returns the cpu_baseline object or None."""
    import numpy as np
    try:
        from oracle import Oracle, RefLib, have_ref
    except Exception:
        return None
    threads = min(16, os.cpu_count() or 1)  # the GPU box grants 16 CPUs per GPU
    if have_ref():
        ref = RefLib()
        # calibrate on a small slice, then size the sample to ~target_s
        n0 = min(len(msg_h), 4000)
        t0 = time.perf_counter()
        ref.ecrecover_batch_mt(msg_h[:n0], sig_h[:n0], threads)
        dt = time.perf_counter() - t0
        n = int(min(len(msg_h), max(n0, n0 * target_s / max(dt, 1e-6))))
        t0 = time.perf_counter()
        _, _, ret = ref.ecrecover_batch_mt(msg_h[:n], sig_h[:n], threads)
        dt = time.perf_counter() - t0
        assert (ret == 1).all()
        return {"value": round(n / dt, 1), "unit": "sigs/s", "cores": threads, "kind": "reference",
                "sample": f"first {n} signatures of the same synthetic batch: reference libsecp256k1 ecrecover "
                          f"(cgo build flags) + Keccak address, {threads} pthreads, {dt:.1f} s"}
    o = Oracle()
    n = 200
    t0 = time.perf_counter()
    o.recover_batch(msg_h[:n], sig_h[:n])
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "sigs/s", "cores": 1, "kind": "port",
            "sample": f"first {n} of the batch, oracle restatement, 1 thread"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    import eges_amd
    from eges_amd._lib import check, lib

    eges_amd.init(1 << local)
    dev = torch.device("cuda", local)
    B = args.batch

    # synthetic device-resident input: this rank's contiguous index shard
    msg, sig, exp_addr = eges_amd.synth_sign_dev(rank * B, B, local)
    addr = torch.empty((B, 20), dtype=torch.uint8, device=dev)
    status = torch.empty((B,), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    # a dedicated stream: the engine's kernels and the timing events share it
    stream = torch.cuda.Stream(dev)
    sp = ctypes.c_void_p(stream.cuda_stream)

    def step():
        check(lib.eges_ecrecover_batch_dev(local, ctypes.c_void_p(msg.data_ptr()), ctypes.c_void_p(sig.data_ptr()), B,
                                           None, ctypes.c_void_p(addr.data_ptr()), ctypes.c_void_p(status.data_ptr()),
                                           sp))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness of the measured path: every address equals the signer's (by construction)
    ok = bool((status == 0).all().item()) and bool(torch.equal(addr, exp_addr))

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    if world > 1:
        t = torch.tensor([elapsed, kern_ms, 0.0 if ok else 1.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, bad = t.tolist()
        ok = bad == 0.0

    total_sigs = B * world * args.steps
    value = total_sigs / elapsed
    per_gpu_rate = B / (kern_ms / 1e3)  # from HIP events on the launch stream
    achieved = per_gpu_rate * W_RECOVER / 1e12
    peak = PEAK_INT32_OPS / 1e12
    traffic = None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tf):
        try:
            with open(tf) as f:
                tj = json.load(f)
            if tj.get("batch") == B:
                traffic = tj.get("bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(msg.cpu().numpy(), sig.cpu().numpy(), args.cpu_seconds)
        line = {
            "metric": "secp256k1 ecrecover+address/sec at 1/8 MI355X; % of INT32 VALU peak",
            "value": round(value, 1),
            "unit": "sigs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "configs[1]: 1M random-key secp256k1 signatures, batch ecrecover + Keccak address "
                                   "per MI355X (inputs resident in HBM)",
                       "batch_per_gpu": B, "parallelism": f"index-sharded x{world}", "correct": ok},
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": round(peak, 2),
                         "unit": "T INT32 lane-ops/s (reference-algorithm accounting, SURVEY.md 8(d))",
                         "frac": round(achieved / peak, 4), "traffic": traffic,
                         "kernel_ms": round(kern_ms, 3)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
