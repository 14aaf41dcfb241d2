#!/usr/bin/env python3
"""bench.py — secp256k1 ecrecover + Keccak address throughput on MI355X.

Metric (BASELINE.json): "secp256k1 ecrecover+address/sec at 1/8 MI355X; % of INT32 VALU peak".

--config c2 (default; BASELINE.json configs[1]): 1M random-key secp256k1 signatures per GPU,
  batch ecrecover + Keccak address. One step = one pass of the hot path over the per-GPU batch
  (device-resident inputs -> 20-byte addresses + status bytes). Multi-GPU: one process per GPU
  (torch.distributed.run), each rank recovers its own contiguous index shard of the synthetic
  signature stream — no data-path collective ("scaling": "weak"); a barrier brackets the
  timed region and the max time over ranks is reported.
--config c4 (configs[3]): a fixed 64M-signature batch split by index across the ranks
  (eges_amd.shard.shard_range; "scaling": "strong"); every address checked.
--config c3 (configs[2]): Geec block import, 1000 EIP-155 transactions with a 100-byte payload
  per block, sender recovery through the host-buffer C-ABI (H2D + kernels + D2H) -> per-block
  latency (median, p99) next to the reference's serial per-transaction loop on one core.
--config c3raw: the same block handed over as wire bytes (10-field Geec txdata RLP) through
  eges_sender_raw_batch: RLP decode, signing-hash RLP + Keccak and recovery all on the GPU.
--config c5 (configs[4]): 10% invalid signatures (high-s, bad recid / chain id, r >= n, s >= n,
  non-residue R, zero r / s) through crypto.Ecrecover and types.Sender semantics, statuses
  checked bit-exact against their by-construction expectation, plus VerifySignature mode.
--config c1 (configs[0]): types.Sender over 10k EIP-155 transfers (SURVEY.md §8(d) C1 shape:
  nonce i, gasPrice 1, gas 21000, value 1, empty data, chainId 930412) handed over as wire bytes
  through eges_sender_raw_batch -> txs/s, next to the reference libsecp256k1 on all host cores.
--config verify: crypto.VerifySignature throughput (65-byte and 33-byte keys).
--config c2host: configs[1]'s batch handed over as host (pageable) buffers through
  eges_ecrecover_batch — the PCIe-inclusive rate a Go caller sees (never `value` of the c2 line).
--config c4host: configs[3]'s batch as host buffers through eges_ecrecover_batch with every
  visible device open in one process (the library's own multi-device split, capi run_host).

The c2 line also carries a `secondary` object (outside the timed region). At every N it holds
`c4_strong`: configs[3]'s fixed 64M batch split by shard_range over the ranks, every address
checked, each rank's HIP-event kernel ms and the max/min imbalance, and the strong-scaled rate
(so the driver's 1/2/4/8 runs of the default line give the configs[3] curve too); at N > 1 also
`c4_host_all_devices` (rank 0 runs --config c4host as a child, the other ranks wait on a gloo
barrier). At N = 1 also: C3's block latency (median / p99 over 50 blocks, from sender rows and
from wire bytes), C1's 10k transfers from wire bytes, C5 over the same 1M batch (ecrecover and
sender statuses, mismatch counts), the same 1M batch as host buffers (c2_host) and the
single-item seam under concurrent callers.

Multi-GPU: `--gpus N` without a launcher starts `torch.distributed.run --nproc-per-node N` on this
script as a child process (no exec) and exits with its code; under a launcher WORLD_SIZE must
equal N. Every line carries `ranks`: each rank's device index, PCI address and UUID, gathered
through the process group. `--stub` rehearses the rank logic on the CPU (gloo, a timed sleep as
the step, no GPU and no libeges): tests/test_shard.py runs it at world size 2.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--c4-total T]
                       [--config c1|c2|c2host|c3|c3raw|c4|c4host|c5|verify]
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "secp256k1 ecrecover+address/sec at 1/8 MI355X; % of INT32 VALU peak"
# Algorithmic work per recovered address: INT32 lane-ops of the reference
# algorithm = 80 x 3085.2 field ops + 128 x 301 scalar ops + 6,300 (Keccak-f) = 291,644.
W_RECOVER = 291_644
W_VERIFY65 = 242_216
# Algorithmic HBM bytes per recovered address: 32 B msg + 65 B sig in, 20 B
# address + 1 B status out
ALGO_BYTES = 118
# The roofline's `peak` / `frac`: the guide's INT32 VALU peak (MI355X_MICROARCH.md "Wave
# scheduling": one wave64 VALU instruction per 2 cycles per SIMD), 1024 SIMDs x 32 lane-ops/clk x
# 2.4 GHz = 7.86e13 lane-ops/s. The same achieved rate is also given against two named ceilings
# of the instruction class the kernel is made of (bench line "peaks_T"):
#  - SURVEY.md §8(d)'s contract, 256 CU x 64 lane-ops/clk x 2.4 GHz = 3.93e13: the 64-bit MAD /
#    carry class issues at half the full rate (tools/ubench_valu.hip: v_mad_u64_u32 / v_add_co /
#    v_addc 4.4-4.9 cyc per wave64 instruction per SIMD; only v_add_u32 / v_bitop3 at ~2.5);
#  - measured: v_mad_u64_u32 at 4 waves/SIMD, 31.6e12 lane-ops/s (profiles/r01/ubench_valu.txt).
PEAK_GUIDE_VALU = 1024 * 32 * 2.4e9
PEAK_INT32_OPS = 256 * 64 * 2.4e9  # SURVEY contract / MAD-class ceiling, 3.93e13 lane-ops/s
PEAK_MEASURED_MAD = 31.61e12
C4_TOTAL = 64 << 20


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=None, help="c2: signatures per GPU; c4: total signatures")
    ap.add_argument("--config", default="c2", choices=["c1", "c2", "c2host", "c3", "c3raw", "c4", "c4host", "c5",
                                                           "verify"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="c2: skip the secondary C1 / C3 / C5 measurements")
    ap.add_argument("--stub", action="store_true", help="CPU rehearsal of the rank logic (gloo, sleep as the step)")
    ap.add_argument("--other-process-kernels", action="store_true",
                    help="(internal) the second process of secondary.single.resident_tax")
    ap.add_argument("--c4-total", type=int, default=None,
                    help="c2: the secondary configs[3] strong-scaled leg's total batch (default 64M; 0 skips it)")
    return ap.parse_args()


def launch_ranks(args):
    """--gpus N: one process per GPU. Without a torch.distributed launcher (WORLD_SIZE unset),
    start `python -m torch.distributed.run --nproc-per-node N` on this script as a CHILD process
    (nothing here has touched the GPU; no exec) and exit with its return code; its rank 0
    prints the JSON line. Under a launcher, WORLD_SIZE must be N."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}", file=sys.stderr, flush=True)
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def host_cpus():
    """CPUs granted to this process on the box: nproc (os.cpu_count()), affinity
    (len(sched_getaffinity)), the cgroup CPU quota (None when unset) and the threads the
    baseline uses: one pthread per granted CPU, i.e. the affinity count, capped by a cgroup
    quota when one is set (more threads than the quota would only time-share)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except Exception:
        quota = None
    threads = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    return {"nproc": nproc, "affinity": aff, "cgroup_cpus": quota, "threads": threads}


def cpu_baseline(msg_h, sig_h, target_s, gpu_addr=None):
    """Reference libsecp256k1 (compiled in place, oracle/_ref) on the host cores: the
    goroutine-parallel types.Sender/Ecrecover path restated as one pthread per granted CPU.
    With gpu_addr (the addresses the timed GPU steps wrote), the reference's addresses for the
    sample are compared with them item for item. Returns the cpu_baseline object or None."""
    try:
        from oracle import Oracle, RefLib, have_ref
    except Exception:
        return None
    host = host_cpus()
    threads = int(os.environ.get("EGES_CPU_THREADS", host["threads"]))
    if have_ref():
        ref = RefLib()
        # calibrate on a small slice, then size the sample to ~target_s
        n0 = min(len(msg_h), 4000)
        t0 = time.perf_counter()
        ref.ecrecover_batch_mt(msg_h[:n0], sig_h[:n0], threads)
        dt = time.perf_counter() - t0
        n = int(min(len(msg_h), max(n0, n0 * target_s / max(dt, 1e-6))))
        t0 = time.perf_counter()
        _, addr_ref, ret = ref.ecrecover_batch_mt(msg_h[:n], sig_h[:n], threads)
        dt = time.perf_counter() - t0
        assert (ret == 1).all()
        agree = None
        if gpu_addr is not None:
            bad = int((addr_ref != gpu_addr[:n]).any(axis=1).sum())
            agree = {"items": n, "mismatches": bad,
                     "note": "the timed GPU steps' addresses vs the reference libsecp256k1's, item for item"}
        rate = n / dt
        return {"value": round(rate, 1), "unit": "sigs/s", "cores": threads, "kind": "reference",
                "reference_check": agree, "host": dict(host, threads=threads),
                "ratio_basis": "the GPU/CPU ratio is per granted CPU set of the host (all threads above), "
                               "not per core",
                # per-core and whole-socket figures beside the granted-set one (VERDICT r5
                # item 6): the measured per-thread rate, and that rate times every host thread (nproc),
                # an extrapolation (the box grants `threads` of them)
                "per_thread": round(rate / threads, 1),
                "whole_host_extrapolated": {"threads": host["nproc"], "sigs_per_s": round(rate / threads * host["nproc"], 1),
                                            "basis": "per_thread x nproc (not measured: this process may use "
                                                     f"{threads} of the host's {host['nproc']} threads)"},
                "sample": f"first {n} signatures of the same synthetic batch: reference libsecp256k1 ecrecover "
                          f"(cgo build flags) + Keccak address, {threads} pthreads, {dt:.1f} s"}
    o = Oracle()
    n = 200
    t0 = time.perf_counter()
    o.recover_batch(msg_h[:n], sig_h[:n])
    dt = time.perf_counter() - t0
    return {"value": round(n / dt, 1), "unit": "sigs/s", "cores": 1, "kind": "port", "host": dict(host, threads=1),
            "sample": f"first {n} of the batch, oracle restatement, 1 thread"}


def kernel_src_hash():
    """SHA-256 over the kernel sources and headers libeges.so is built from. The GPU box gets no
    .git, so a PMC summary is tied to the sources it was collected from, not to a commit id."""
    import glob
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "eges_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cuh"))
                   + glob.glob(os.path.join(csrc, "*.h"))) + [os.path.join(ROOT, "include", "eges.h")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def read_pmc(kernel, batch):
    """Counter summary of `kernel` launched on `batch` items, from profiles/pmc_traffic.json
    (tools/pmc.sh + tools/pmc_summary.py: one entry per (config, kernel), each with its own launch
    size), only when it was collected from the same kernel sources; else None."""
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(tf) as f:
            tj = json.load(f)
    except Exception:
        return None
    if tj.get("src_sha256") != kernel_src_hash():
        return None
    for ent in tj.get("entries", []):
        if ent.get("kernel") == kernel and ent.get("batch") == batch:
            return ent
    return None


class Ctx:
    def __init__(self, args):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.args = torch, dist, args
        self.stub = args.stub
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # rehearsal knobs for a 1-GPU box (tools/rehearse_dist.sh): every rank on one device,
        # gloo for the timing collectives. The driver's multi-GPU runs leave both unset.
        if "EGES_BENCH_DEVICE" in os.environ:
            self.local = int(os.environ["EGES_BENCH_DEVICE"])
        if not self.stub:
            # bind the rank's GPU before the process group exists, so RCCL's barrier uses it
            torch.cuda.set_device(self.local)
        if self.world > 1:
            backend = "gloo" if self.stub else (os.environ.get("EGES_BENCH_BACKEND") or "nccl")
            dist.init_process_group(backend=backend)
        # host-side collectives (per-rank summaries, the barrier while rank 0's child uses every
        # GPU): gloo, so no RCCL kernel waits on a device meanwhile
        self.cpu_group = (dist.new_group(backend="gloo") if backend != "gloo" else dist.group.WORLD) \
            if self.world > 1 else None
        self.ranks = self.gather_ranks()
        if self.stub:
            return
        import eges_amd
        self.eges = eges_amd
        # c4host opens every visible device in this one process (the library splits the batch)
        eges_amd.init(0 if args.config == "c4host" else 1 << self.local)
        self.dev = torch.device("cuda", self.local)
        # a dedicated stream: the engine's kernels and the timing events share it
        self.stream = torch.cuda.Stream(self.dev)
        self.sp = self.stream.cuda_stream

    def gather_ranks(self):
        """Each rank's device identity (index, PCI address, UUID), all-gathered through the process
        group, so the line shows how many distinct GPUs the ranks ran on."""
        me = {"rank": self.rank, "local_rank": self.local, "host": socket.gethostname()}
        if self.stub:
            me["device"] = "cpu (stub)"
        else:
            p = self.torch.cuda.get_device_properties(self.local)
            me.update(device=self.local, name=p.name,
                      pci=f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", uuid=str(p.uuid))
        if self.world == 1:
            return [me]
        out = [None] * self.world
        self.dist.all_gather_object(out, me)
        return out

    def sync(self):
        if not self.stub:
            self.torch.cuda.synchronize()

    def timed(self, step, reset=None):
        """W untimed steps, then K steps between barrier + synchronize on both sides; returns
        (max elapsed over ranks, mean per-step time from HIP events on the engine's stream).
        `reset` (untimed) clears the outputs after the warmup, so the check that follows reads
        what the timed steps wrote."""
        torch, dist, a = self.torch, self.dist, self.args
        for _ in range(a.warmup):
            step()
        self.sync()
        if reset is not None:
            reset()
            self.sync()
        evs = [] if self.stub else [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                                    for _ in range(a.steps)]
        if self.world > 1:
            dist.barrier()
        self.sync()
        t0 = time.perf_counter()
        for i in range(a.steps):
            if evs:
                evs[i][0].record(self.stream)
            step()
            if evs:
                evs[i][1].record(self.stream)
        self.sync()
        if self.world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kern_ms = (sum(x.elapsed_time(y) for x, y in evs) / a.steps) if evs else elapsed * 1e3 / a.steps
        return elapsed, kern_ms

    def reduce_max(self, *vals):
        if self.world == 1:
            return vals
        dev = "cpu" if self.stub else self.dev
        t = self.torch.tensor(list(vals), dtype=self.torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return tuple(t.tolist())

    def finish(self, line, ok):
        line["ranks"] = self.ranks
        line["distinct_devices"] = len({(r.get("host"), r.get("pci"), r.get("uuid"), r.get("device")) for r in self.ranks})
        if self.rank == 0:
            print(json.dumps(line), flush=True)
        if self.world > 1:
            self.dist.destroy_process_group()
        if not ok:
            sys.exit(1)


def roofline(per_gpu_rate, work, batch, kern_ms, kernel="eges::recover_kernel"):
    """Roofline object of the dominant kernel. `frac` keeps the SURVEY.md 8(d) contract
    denominator; the same achieved rate is also given against the guide's VALU issue rate and
    the measured v_mad_u64_u32 rate, each named. With a PMC summary of the same kernel sources:
    HBM-side traffic and the counter-derived VALU utilisation."""
    achieved = per_gpu_rate * work
    r = {"bound": "valu", "kernel": kernel, "batch": batch, "achieved": round(achieved / 1e12, 3),
         "peak": round(PEAK_GUIDE_VALU / 1e12, 2),
         "unit": "T INT32 lane-ops/s (reference-algorithm accounting, SURVEY.md 8(d); peak: MI355X_MICROARCH.md "
                 "VALU issue, 1024 SIMDs x 32 lanes/clk x 2.4 GHz)",
         "frac": round(achieved / PEAK_GUIDE_VALU, 4),
         "frac_vs_survey_contract": round(achieved / PEAK_INT32_OPS, 4),
         "frac_vs_measured_mad_rate": round(achieved / PEAK_MEASURED_MAD, 4),
         "peaks_T": {"guide_valu_issue": round(PEAK_GUIDE_VALU / 1e12, 2),
                     "survey_contract_mad_class": round(PEAK_INT32_OPS / 1e12, 2),
                     "measured_v_mad_u64_u32": round(PEAK_MEASURED_MAD / 1e12, 2)},
         "traffic": None, "kernel_ms": round(kern_ms, 4),
         "kernel_ms_source": "HIP events on the launch stream around each timed step"}
    pmc = read_pmc(kernel, batch)
    if pmc:
        # FETCH_SIZE (KB, x2: gfx950 correction) + WRITE_SIZE (KB): L2 <-> fabric (MALL / HBM) bytes
        r["traffic"] = pmc.get("bytes_per_launch")
        insts = pmc.get("SQ_INSTS_VALU")
        if insts and batch:
            lane_insts = insts * 64
            r["counters"] = {
                "source": f"profiles/pmc_traffic.json entry {pmc.get('config')}/{kernel} (PMC passes of the same "
                          "kernel sources, src_sha256), per launch of this batch size",
                "valu_lane_insts_per_sig": round(lane_insts / batch),
                "salu_insts_per_sig": round(pmc["SQ_INSTS_SALU"] / batch, 1) if pmc.get("SQ_INSTS_SALU") else None,
                "int64_class_share": round(pmc.get("SQ_INSTS_VALU_INT64", 0) / insts, 4),
                "waves_per_launch": pmc.get("SQ_WAVES"),
                "valu_util_vs_guide": round(lane_insts / (kern_ms / 1e3) / PEAK_GUIDE_VALU, 4),
                "valu_util_vs_survey_contract": round(lane_insts / (kern_ms / 1e3) / PEAK_INT32_OPS, 4)}
            # what the waves wait on, and how much of the traffic the L2 absorbs:
            # the share of wave-cycles spent waiting on anything (memory, LDS, dependencies) and the
            # L2 hit rate; traffic_vs_algorithmic = fabric bytes per launch / (ALGO_BYTES x batch)
            cn = r["counters"]
            if pmc.get("SQ_WAIT_ANY") and pmc.get("SQ_WAVE_CYCLES"):
                cn["wait_any_share_of_wave_cycles"] = round(pmc["SQ_WAIT_ANY"] / pmc["SQ_WAVE_CYCLES"], 4)
            if pmc.get("SQ_WAIT_INST_ANY") and pmc.get("SQ_WAVE_CYCLES"):
                cn["wait_inst_any_share_of_wave_cycles"] = round(pmc["SQ_WAIT_INST_ANY"] / pmc["SQ_WAVE_CYCLES"], 4)
            hit, miss = pmc.get("TCC_HIT_sum"), pmc.get("TCC_MISS_sum")
            if hit is not None and miss is not None and hit + miss > 0:
                cn["l2_hit_rate"] = round(hit / (hit + miss), 4)
            if r["traffic"]:
                cn["traffic_vs_algorithmic"] = round(r["traffic"] / (ALGO_BYTES * batch), 1)
            cn["bound_note"] = ("VALU issue-bound, not traffic-bound, when valu_util is near the measured "
                                "v_mad_u64_u32 rate (frac_vs_measured_mad_rate) and the wait share is small; "
                                "the fabric traffic is the per-lane R-table workspace and fixed-base gathers, "
                                "mostly served by the Infinity Cache (DESIGN.md section 4)")
    return r


# ------------------------------------------------------------------ c2 / c4: throughput
def run_throughput(c, strong):
    a = c.args
    from eges_amd.shard import shard_range
    if strong:
        total = a.batch or C4_TOTAL
        shards = [shard_range(total, r, c.world) for r in range(c.world)]
    else:
        B0 = a.batch or (1 << 20)
        shards = [(r * B0, (r + 1) * B0) for r in range(c.world)]
        total = B0 * c.world
    lo, hi = shards[c.rank]
    B = hi - lo
    wl = ("configs[3]: 64M-signature batch sharded by index across the GPUs, batch ecrecover + Keccak address"
          if strong else "configs[1]: 1M random-key secp256k1 signatures, batch ecrecover + Keccak address per "
          "MI355X (inputs resident in HBM)")
    if c.stub:
        elapsed, kern_ms, ok = run_stub(c, B)
        line = {"metric": METRIC, "value": round(total * a.steps / elapsed, 1), "unit": "sigs/s", "n_gpus": c.world,
                "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 3),
                "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
                "dtype": "u32", "data": "stub: rank-logic rehearsal on the CPU (sleep as the step, no GPU)",
                "config": {"workload": wl, "batch_per_gpu": B, "shards": shards, "total_batch": total,
                           "parallelism": f"index-sharded x{c.world}", "correct": ok}}
        c4_total = C4_TOTAL if a.c4_total is None else a.c4_total
        if not strong and not a.no_secondary and c4_total > 0:
            sec = {"note": "stub legs", "c4_strong": measure_c4_strong(c, c4_total)}
            if c.world > 1:
                sec["c4_host_all_devices"] = measure_host_all_devices(c, c4_total)
            ok = ok and all(v.get("correct", True) for v in sec.values() if isinstance(v, dict))
            ok = c.reduce_max(0.0 if ok else 1.0)[0] == 0.0
            line["secondary"] = sec
            line["config"]["correct"] = ok
        c.finish(line, ok)
        return
    torch = c.torch
    # synthetic device-resident input: this rank's contiguous index shard
    msg, sig, exp_addr = c.eges.synth_sign_dev(lo, B, c.local)
    addr = torch.empty((B, 20), dtype=torch.uint8, device=c.dev)
    status = torch.empty((B,), dtype=torch.uint8, device=c.dev)
    torch.cuda.synchronize()
    from eges_amd._lib import check, lib

    def step():
        check(lib.eges_ecrecover_batch_dev(c.local, ctypes.c_void_p(msg.data_ptr()), ctypes.c_void_p(sig.data_ptr()), B,
                                           None, ctypes.c_void_p(addr.data_ptr()), ctypes.c_void_p(status.data_ptr()),
                                           ctypes.c_void_p(c.sp)))

    def reset():
        addr.zero_()
        status.fill_(0xFF)

    elapsed, kern_ms = c.timed(step, reset)
    # correctness of the measured launches: every address the timed steps wrote equals the
    # signer's (by construction)
    ok = bool((status == 0).all().item()) and bool(torch.equal(addr, exp_addr))
    elapsed, kern_ms, bad = c.reduce_max(elapsed, kern_ms, 0.0 if ok else 1.0)
    ok = bad == 0.0
    value = total * a.steps / elapsed
    per_gpu_rate = B / (kern_ms / 1e3)  # from HIP events on the launch stream
    cpu = None
    if c.rank == 0 and not a.no_cpu_baseline and c.world == 1 and not strong:
        cpu = cpu_baseline(msg.cpu().numpy(), sig.cpu().numpy(), a.cpu_seconds, gpu_addr=addr.cpu().numpy())
        if cpu and (cpu.get("reference_check") or {}).get("mismatches"):
            ok = False
    line = {"metric": METRIC, "value": round(value, 1), "unit": "sigs/s", "n_gpus": c.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed * 1e3 / a.steps, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": wl, "batch_per_gpu": B, "shards": shards, "total_batch": total,
                       "parallelism": f"index-sharded x{c.world}", "correct": ok},
            "roofline": roofline(per_gpu_rate, W_RECOVER, B, kern_ms), "cpu_baseline": cpu}
    if cpu and cpu.get("kind") == "reference":
        cpu["gpu_vs"] = {"granted_set": round(value / cpu["value"], 1), "per_thread": round(value / cpu["per_thread"], 1),
                         "whole_host_extrapolated": round(value / cpu["whole_host_extrapolated"]["sigs_per_s"], 1)}
    sec = {"note": "measured after the timed C2 region, same processes; not part of value"}
    c4_total = C4_TOTAL if a.c4_total is None else a.c4_total
    if not strong and not a.no_secondary and c4_total > 0:
        # configs[3] at every N: the driver's 1/2/4/8 runs of this default line are its curve
        sec["c4_strong"] = measure_c4_strong(c, c4_total)
        if c.world > 1:
            sec["c4_host_all_devices"] = measure_host_all_devices(c, c4_total)
            if c.rank == 0:
                line["secondary"] = sec
                ok = ok and all(v.get("correct", True) for v in sec.values() if isinstance(v, dict))
                line["config"]["correct"] = ok
            ok = c.reduce_max(0.0 if ok else 1.0)[0] == 0.0
    if c.world == 1 and not strong and not a.no_secondary:
        # the other configs, after the timed region (about a second): C3 and C1 latency, C5 statuses
        sec["c3_block"] = measure_block(c, 1000, raw_mode=False, warmup=3, iters=50, cpu=False)
        sec["c3_block_wire"] = measure_block(c, 1000, raw_mode=True, warmup=3, iters=50, cpu=False)
        sec["c1_transfers"] = measure_c1(c, 10000, warmup=3, iters=20, cpu=False)
        sec["c5_adversarial"] = measure_c5(c, B, msg, sig, exp_addr, steps=1, warmup=1)
        # the same 1M batch handed over as host buffers
        sec["c2_host"] = measure_host(c, msg.cpu().numpy(), sig.cpu().numpy(), exp_addr.cpu().numpy(), steps=6,
                                      warmup=2)
        # as many synchronous callers as the reference baseline's threads (the box's granted CPUs)
        ref = cpu if cpu and cpu.get("kind") == "reference" else None
        sec["single"] = measure_single(ref["cores"] if ref else 16, 2000, ref["value"] if ref else None,
                                       ref_one_call_us(msg.cpu().numpy(), sig.cpu().numpy()))
        sec["single"]["resident_tax"] = measure_resident_tax(c, msg[0].cpu().numpy(), sig[0].cpu().numpy())
        line["secondary"] = sec
        ok = ok and all(v.get("correct", True) for v in sec.values() if isinstance(v, dict))
        line["config"]["correct"] = ok
    c.finish(line, ok)


def run_stub(c, B):
    """The rank logic of run_throughput on the CPU: timed steps between barriers, max over ranks,
    the correctness reduce (EGES_BENCH_STUB_BAD_RANK makes one rank report a mismatch)."""
    def step():
        time.sleep(0.002)
    elapsed, kern_ms = c.timed(step)
    ok = str(c.rank) != os.environ.get("EGES_BENCH_STUB_BAD_RANK", "")
    elapsed, kern_ms, bad = c.reduce_max(elapsed, kern_ms, 0.0 if ok else 1.0)
    return elapsed, kern_ms, bad == 0.0


def with_steps(c, steps, warmup, fn):
    """fn() with the context's step / warmup counts temporarily replaced (secondary legs)."""
    saved = (c.args.steps, c.args.warmup)
    c.args.steps, c.args.warmup = steps, warmup
    try:
        return fn()
    finally:
        c.args.steps, c.args.warmup = saved


def strong_summary(total, shards, steps, per_rank):
    """The configs[3] leg's numbers from every rank's (elapsed s, kernel ms, ok) triple: the
    strong-scaled rate (all ranks' items / the slowest rank's elapsed time), each rank's kernel
    ms from HIP events, and the imbalance max / min over the ranks that hold work."""
    els = [p[0] for p in per_rank]
    kms = [p[1] for p in per_rank]
    busy = [k for k, (lo, hi) in zip(kms, shards) if hi > lo]
    el = max(els)
    return {"total_batch": total, "shards": [list(s) for s in shards], "steps": steps,
            "sigs_per_s": round(total * steps / el, 1), "ms_per_step": round(el * 1e3 / steps, 3),
            "rank_kernel_ms": [round(k, 4) for k in kms],
            "rank_elapsed_ms_per_step": [round(e * 1e3 / steps, 3) for e in els],
            "imbalance_max_over_min": round(max(busy) / min(busy), 4) if busy and min(busy) > 0 else None,
            "correct": all(bool(p[2]) for p in per_rank), "scaling": "strong"}


def measure_c4_strong(c, total, steps=2, warmup=1):
    """configs[3] inside the default line: the fixed batch of `total`
    signatures split by shard_range over the ranks, each rank's shard synthesised on its GPU,
    `steps` timed passes between barriers, every address the timed passes wrote checked against
    its signer's. Per-rank numbers are all-gathered so rank 0's line shows the imbalance. With
    --stub the step is a sleep proportional to the shard (the rank logic on the CPU)."""
    from eges_amd.shard import shard_range
    shards = [shard_range(total, r, c.world) for r in range(c.world)]
    lo, hi = shards[c.rank]
    B = hi - lo
    if c.stub:
        unit = max(1, shards[0][1] - shards[0][0])

        def step():
            time.sleep(0.002 * B / unit)
        elapsed, kern_ms = with_steps(c, steps, warmup, lambda: c.timed(step))
        ok = str(c.rank) != os.environ.get("EGES_BENCH_STUB_BAD_RANK", "")
    else:
        torch = c.torch
        from eges_amd._lib import check, lib
        ok = True
        elapsed, kern_ms = 0.0, 0.0
        if B:
            msg, sig, exp_addr = c.eges.synth_sign_dev(lo, B, c.local, stream=c.sp)
            addr = torch.empty((B, 20), dtype=torch.uint8, device=c.dev)
            status = torch.empty((B,), dtype=torch.uint8, device=c.dev)
            torch.cuda.synchronize()

            def step():
                check(lib.eges_ecrecover_batch_dev(c.local, ctypes.c_void_p(msg.data_ptr()),
                                                   ctypes.c_void_p(sig.data_ptr()), B, None,
                                                   ctypes.c_void_p(addr.data_ptr()), ctypes.c_void_p(status.data_ptr()),
                                                   ctypes.c_void_p(c.sp)))

            def reset():
                addr.zero_()
                status.fill_(0xFF)
        else:  # an empty shard (total < world): the rank still joins the barriers
            def step():
                pass
            reset = None
        elapsed, kern_ms = with_steps(c, steps, warmup, lambda: c.timed(step, reset))
        if B:
            ok = bool((status == 0).all().item()) and bool(torch.equal(addr, exp_addr))
            del msg, sig, exp_addr, addr, status
            torch.cuda.empty_cache()
    mine = (elapsed, kern_ms, ok)
    if c.world == 1:
        per_rank = [mine]
    else:
        per_rank = [None] * c.world
        c.dist.all_gather_object(per_rank, mine, group=c.cpu_group)
    out = strong_summary(total, shards, steps, per_rank)
    out["workload"] = ("configs[3]: the fixed batch sharded by index across the ranks (eges_amd.shard.shard_range), "
                       "device-resident inputs, every address checked")
    out["kernel_ms_source"] = "HIP events on each rank's launch stream around each timed step"
    return out


def measure_host_all_devices(c, total):
    """The Go caller's multi-GPU path: rank 0 starts bench.py --config
    c4host as a child process (no launcher environment) after the ranks' own legs; the child
    opens every visible device in one process and hands the fixed batch over as host buffers
    through eges_ecrecover_batch, which splits it over the devices in-library (capi run_host).
    The other ranks wait at a barrier meanwhile. Returns the child's line (rank 0) or None."""
    out = None
    if c.rank == 0:
        env = {k: v for k, v in os.environ.items()
               if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                            "ROLE_WORLD_SIZE", "TORCHELASTIC_RUN_ID", "MASTER_PORT")}
        cmd = [sys.executable, os.path.abspath(__file__), "--config", "c4host", "--batch", str(total),
               "--steps", "2", "--warmup", "1"] + (["--stub"] if c.stub else [])
        try:
            cp = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
            lines = [ln for ln in cp.stdout.splitlines() if ln.startswith("{")]
            out = json.loads(lines[-1]) if lines else {"note": f"c4host child rc {cp.returncode}: {cp.stderr[-500:]}",
                                                       "correct": False}
            if cp.returncode != 0:
                out["correct"] = False
        except Exception as e:  # noqa: BLE001
            out = {"note": f"c4host child failed: {e}", "correct": False}
    if c.world > 1:
        c.dist.barrier(group=c.cpu_group)
    return out


# ------------------------------------------------------------------ c3: Geec block latency
def dev_kernel_ms(c, step, reps=20, warmup=3):
    """Mean span of one device-resident launch of `step` (everything on the bench stream c.sp),
    from HIP events around each launch: the dominant kernel's duration for a one-kernel step."""
    torch = c.torch
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in evs:
        e0.record(c.stream)
        step()
        e1.record(c.stream)
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in evs) / reps


def measure_block(c, n, raw_mode, warmup, iters, cpu=True):
    """A Geec block of n EIP-155 transactions (100-byte payload) through eges_sender_batch (host
    buffers) or, raw_mode, as wire bytes through eges_sender_raw_batch: per-block latency."""
    import numpy as np
    torch = c.torch
    from eges_amd import txs
    from eges_amd._lib import SIGNER_EIP155
    sighash = txs.geec_block(0, n, payload=100)
    sig_d, exp_d = c.eges.synth_sign_msg_dev(torch.from_numpy(sighash).to(c.dev), 0, stream=c.sp)
    torch.cuda.synchronize()
    sig_h, exp_h = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    r, s, v = txs.sender_rows(sig_h, txs.GEEC_CHAIN_ID)
    if raw_mode:  # the block's transactions as the wire carries them (10-field Geec txdata RLP)
        raw, offs = c.eges.pack_raw(txs.geec_block_raw(0, sig_h, payload=100))
    # the C-ABI call itself on preallocated host buffers (what a cgo caller pays), not the numpy
    # wrapper: every timed call's outputs are checked after it
    from eges_amd._lib import check, lib
    addr = np.zeros((n, 20), np.uint8)
    st = np.zeros(n, np.uint8)
    P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    vf = np.zeros(n, np.uint8)
    if raw_mode:
        args = (P(raw), P(offs), n, SIGNER_EIP155, txs.GEEC_CHAIN_ID, P(addr), P(st), None)
        fn = lib.eges_sender_raw_batch
    else:
        sighash, r, s, v = (np.ascontiguousarray(x) for x in (sighash, r, s, v))
        args = (P(sighash), P(r), P(s), P(v), P(vf), n, SIGNER_EIP155, txs.GEEC_CHAIN_ID, P(addr), P(st))
        fn = lib.eges_sender_batch
    lat = []
    ok = True
    for i in range(warmup + iters):
        addr.fill(0)
        st.fill(0xEE)
        t0 = time.perf_counter()
        rc = fn(*args)
        dt = time.perf_counter() - t0
        check(rc)
        if i >= warmup:
            lat.append(dt)
        ok = ok and bool((st == 0).all()) and np.array_equal(addr, exp_h)
    lat = np.array(lat) * 1e3
    # the dominant kernel's roofline: the same block device-resident through the *_dev entry (one
    # launch with the sender rows / wire bytes classified in-kernel), HIP events on the bench stream
    if raw_mode:
        rd, od = torch.from_numpy(raw).to(c.dev), torch.from_numpy(offs.astype(np.int64)).to(c.dev)
        ad, sd = torch.empty((n, 20), dtype=torch.uint8, device=c.dev), torch.empty(n, dtype=torch.uint8, device=c.dev)
        kms = dev_kernel_ms(c, lambda: c.eges.sender_raw_batch_dev(rd, od, SIGNER_EIP155, txs.GEEC_CHAIN_ID, addr=ad,
                                                                   status=sd, stream=c.sp))
    else:
        hd, rr, sr, vr, vd = (torch.from_numpy(np.ascontiguousarray(x)).to(c.dev) for x in (sighash, r, s, v, vf))
        ad, sd = torch.empty((n, 20), dtype=torch.uint8, device=c.dev), torch.empty(n, dtype=torch.uint8, device=c.dev)
        kms = dev_kernel_ms(c, lambda: c.eges.sender_batch_dev(hd, rr, sr, vr, vd, SIGNER_EIP155, txs.GEEC_CHAIN_ID,
                                                               addr=ad, status=sd, stream=c.sp))
    torch.cuda.synchronize()
    ok = ok and bool((sd == 0).all().item()) and np.array_equal(ad.cpu().numpy(), exp_h)
    out = {"median_ms": round(float(np.median(lat)), 3), "p99_ms": round(float(np.percentile(lat, 99)), 3),
           "blocks": iters, "txs": n, "correct": ok,
           "native_caller": None if raw_mode else native_block(n, iters),
           "roofline": roofline(n / (kms / 1e3), W_RECOVER, n, kms, kernel="eges::recover_lat_kernel"),
           "path": ("wire-format txdata RLP through eges_sender_raw_batch (H2D + decode + sighash RLP/Keccak + "
                    "recovery kernels + D2H)" if raw_mode else "host buffers through eges_sender_batch (H2D + "
                    "kernels + D2H)") + "; timed around the C-ABI call (ctypes, preallocated outputs)"}
    if cpu:
        out["cpu"] = None
        try:
            from oracle import RefLib, have_ref
            if have_ref():
                ref = RefLib()
                t0 = time.perf_counter()
                ref.ecrecover_batch_mt(sighash, sig_h, 1)
                dt = time.perf_counter() - t0
                out["cpu"] = {"value": round(dt * 1e3, 3), "unit": "ms/block", "cores": 1, "kind": "reference",
                              "sample": f"one {n}-tx block: the reference's serial per-tx ecrecover + Keccak address "
                                        "(types.Sender inside StateProcessor.Process, state_processor.go:73-93), "
                                        "1 core; " + ("sighash RLP + Keccak excluded on the CPU side only (the GPU "
                                                      "value includes decode and sighash)" if raw_mode else
                                                      "sighash RLP cost excluded on both sides")}
        except Exception:
            out["cpu"] = None
    return out


def native_block(n, iters):
    """The same block size through eges_sender_batch from a native caller (tools/block_bench, built
    by build(): preallocated host buffers, every result checked), as a child process on the same
    GPU: what a cgo caller pays per block, without the Python ctypes call's own overhead."""
    exe = os.path.join(ROOT, "tools", "block_bench")
    if not os.path.exists(exe):
        return None
    try:
        cp = subprocess.run([exe, str(n), str(max(iters, 300))], capture_output=True, text=True, timeout=120)
        m = json.loads(cp.stdout.strip().splitlines()[-1])
        return {"median_ms": round(m["median_ms"], 4), "p99_ms": round(m["p99_ms"], 4), "blocks": m["iters"],
                "correct": m["errors"] == 0 and cp.returncode == 0, "path": "tools/block_bench (C++ caller)"}
    except Exception as e:  # noqa: BLE001
        return {"note": f"block_bench failed: {e}"}


def run_block_latency(c):
    a = c.args
    n = a.batch or 1000
    raw_mode = a.config == "c3raw"
    iters = max(50, a.steps * 20)
    m = measure_block(c, n, raw_mode, a.warmup, iters, cpu=not a.no_cpu_baseline)
    line = {"metric": "Geec block sender recovery latency (1000 EIP-155 txs, 100-byte payload)"
                      + (", from wire bytes" if raw_mode else ""),
            "value": m["median_ms"], "unit": "ms/block", "p99_ms": m["p99_ms"],
            "sigs_per_s": round(n / (m["median_ms"] / 1e3), 1), "n_gpus": 1, "steps": iters, "warmup": a.warmup,
            "higher_is_better": False, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "configs[2]: Geec block import, 1000 txns/block (txnSize 100), EIP155Signer(930412), "
                                   + m["path"], "correct": m["correct"]}, "roofline": m.get("roofline"),
            "cpu_baseline": m.get("cpu"), "native_caller": m.get("native_caller")}
    nc = m.get("native_caller") or {}
    c.finish(line, m["correct"] and nc.get("correct", True))


# ------------------------------------------------------------------ single-item seam
def ref_one_call_us(msg_h, sig_h, n=4000):
    """The reference's per-call cost on one host thread: secp256k1_ext_ecdsa_recover (ext.h:30-47,
    what crypto.Ecrecover reaches through signature_cgo.go:31-44) over n items serially, no
    Keccak, averaged (oracle/_ref; the cgo call overhead itself is not included)."""
    try:
        from oracle import RefLib, have_ref
        if not have_ref():
            return None
        ref = RefLib()
        ref.ecrecover_batch_mt(msg_h[:200], sig_h[:200], 1, want_addr=False)  # warm
        t0 = time.perf_counter()
        _, _, ret = ref.ecrecover_batch_mt(msg_h[:n], sig_h[:n], 1, want_addr=False)
        dt = time.perf_counter() - t0
        return round(dt / min(n, len(msg_h)) * 1e6, 2) if (ret == 1).all() else None
    except Exception:  # noqa: BLE001
        return None


def measure_single(callers=16, calls=2000, ref_rate=None, ref_one_us=None):
    """The per-call cgo seam (eges_ecdsa_recover, replacing ext.h:30-47 under
    crypto.Ecrecover, signature_cgo.go:31-44): tools/single_bench (native threads, built by
    build()) as a child process on the same GPU: one caller's p50 / p99, then `callers` synchronous
    callers x `calls` calls, every result checked. ref_rate: the reference libsecp256k1 on the same
    host with the same number of threads, each calling secp256k1_ext_ecdsa_recover once per item
    (oracle/_ref eref_ecrecover_batch_mt = cpu_baseline)."""
    exe = os.path.join(ROOT, "tools", "single_bench")
    if not os.path.exists(exe):
        return {"note": "tools/single_bench not built", "correct": True}
    try:
        cp = subprocess.run([exe, str(callers), str(calls)], capture_output=True, text=True, timeout=240)
        m = json.loads(cp.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        return {"note": f"single_bench failed: {e}", "correct": False}
    out = {"p50_ms_one_caller": m["p50_ms_one_caller"], "p99_ms_one_caller": m["p99_ms_one_caller"],
           "verify_p50_ms_one_caller": m["verify_p50_ms_one_caller"], "callers": callers,
           "calls_per_caller": calls, "recoveries_per_s": m["recoveries_per_s"], "errors": m["errors"],
           "correct": m["errors"] == 0 and cp.returncode == 0,
           "path": "eges_ecdsa_recover (the per-call seam; concurrent callers coalesced into shared launches)"}
    if ref_rate:
        out["reference_same_threads_per_s"] = ref_rate
        out["vs_reference"] = round(m["recoveries_per_s"] / ref_rate, 3)
    if ref_one_us:
        # one caller: the reference's serial per-call cost beside this seam's p50
        out["reference_one_call_us"] = ref_one_us
        out["one_caller_vs_reference"] = round(ref_one_us / (m["p50_ms_one_caller"] * 1e3), 3)
    return out


def other_process_kernels():
    """--other-process-kernels: the second process of measure_resident_tax. A device-resident 1M
    batch on device 0, timed with HIP events each time a line "go" arrives on stdin; prints one
    number per launch (ms). Its own engine never starts a resident server."""
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
    print("ok" if ok else "wrong", flush=True)


def measure_resident_tax(c, msg1, sig1, reps=8):
    """What the resident single-call server costs another tenant of the GPU:
    a second process launches a device-resident 1M batch right after one single recovery of this
    process, alternately with the server alive (EGES_RESIDENT=1: its workgroups poll for
    EGES_RESIDENT_IDLE_US after the call) and without it; the medians of the other process's kernel
    time, their ratio, and how often the server was still running when the other launch was
    requested (eges_diag_resident_running)."""
    import numpy as np
    from eges_amd._lib import lib
    dev = c.dev.index if c.dev.index is not None else 0
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    try:
        child = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--other-process-kernels"],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env)
    except Exception as e:  # noqa: BLE001
        return {"note": f"second process failed to start: {e}"}
    out = {"note": "second process did not finish"}
    try:
        if child.stdout.readline().strip() != "ready":
            return {"note": "second process not ready"}
        old = c.eges.get_knob("EGES_RESIDENT")
        pub = (ctypes.c_ubyte * 65)()
        on, off, alive = [], [], []
        for rep in range(2 * reps):
            with_server = rep % 2 == 0
            c.eges.set_knob("EGES_RESIDENT", 1 if with_server else 0)
            time.sleep(0.02)  # (a previous server idles out first)
            rc = lib.eges_ecdsa_recover(pub, sig1.tobytes(), msg1.tobytes())
            if with_server:
                alive.append(lib.eges_diag_resident_running(dev) == 1)
            child.stdin.write("go\n")
            child.stdin.flush()
            ms = float(child.stdout.readline())
            (on if with_server else off).append(ms)
            if rc != 1:
                return {"note": "single recovery failed", "correct": False}
        c.eges.set_knob("EGES_RESIDENT", old)
        child.stdin.close()
        tail = child.stdout.read().strip()
        child.wait(timeout=60)
        m_on, m_off = float(np.median(on)), float(np.median(off))
        out = {"other_process_1m_kernel_ms_server_alive": round(m_on, 4), "other_process_1m_kernel_ms_no_server": round(m_off, 4),
               "slowdown": round(m_on / m_off - 1.0, 4), "server_alive_at_launch": f"{sum(alive)}/{len(alive)}",
               "idle_window_us": c.eges.get_knob("EGES_RESIDENT_IDLE_US"), "resident_workgroups": c.eges.get_knob("EGES_RESIDENT_WGS"),
               "pairs": reps, "correct": tail.endswith("ok")}
    finally:
        if child.poll() is None:
            child.kill()
    return out


# ------------------------------------------------------------------ c1: 10k EIP-155 transfers
def measure_c1(c, n, warmup, iters, cpu=True):
    import numpy as np
    torch = c.torch
    from eges_amd import txs
    from eges_amd._lib import SIGNER_EIP155
    sighash = txs.c1_sighashes(0, n)
    # the GPU synthetic signer uses C1's keys (tests/test_c1.py pins them against the reference's
    # pubkey_create); its nonces are not RFC6979, which does not change what recovery computes
    sig_d, exp_d = c.eges.synth_sign_msg_dev(torch.from_numpy(sighash).to(c.dev), 0, stream=c.sp)
    torch.cuda.synchronize()
    sig_h, exp_h = sig_d.cpu().numpy(), exp_d.cpu().numpy()
    packed = c.eges.pack_raw(txs.c1_raw(0, sig_h))
    # the C-ABI call itself on preallocated host buffers (what a cgo caller pays), as in
    # measure_block: every timed call's outputs are checked after it
    from eges_amd._lib import check, lib
    P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    addr = np.zeros((n, 20), np.uint8)
    st = np.zeros(n, np.uint8)
    args = (P(packed[0]), P(packed[1]), n, SIGNER_EIP155, txs.GEEC_CHAIN_ID, P(addr), P(st), None)
    lat = []
    ok = True
    for i in range(warmup + iters):
        addr.fill(0)
        st.fill(0xEE)
        t0 = time.perf_counter()
        rc = lib.eges_sender_raw_batch(*args)
        dt = time.perf_counter() - t0
        check(rc)
        if i >= warmup:
            lat.append(dt)
        ok = ok and bool((st == 0).all()) and np.array_equal(addr, exp_h)
    med = float(np.median(lat))
    # the dominant kernel's roofline: the batch device-resident through eges_sender_raw_batch_dev
    # (one launch of the bucket form with decode + sighash fused in), HIP events on the bench stream
    raw, offs = packed
    rd, od = torch.from_numpy(raw).to(c.dev), torch.from_numpy(offs.astype(np.int64)).to(c.dev)
    ad, sd = torch.empty((n, 20), dtype=torch.uint8, device=c.dev), torch.empty(n, dtype=torch.uint8, device=c.dev)
    kms = dev_kernel_ms(c, lambda: c.eges.sender_raw_batch_dev(rd, od, SIGNER_EIP155, txs.GEEC_CHAIN_ID, addr=ad,
                                                               status=sd, stream=c.sp))
    torch.cuda.synchronize()
    ok = ok and bool((sd == 0).all().item()) and np.array_equal(ad.cpu().numpy(), exp_h)
    out = {"txs_per_s": round(n / med, 1), "median_ms": round(med * 1e3, 3),
           "p99_ms": round(float(np.percentile(np.array(lat) * 1e3, 99)), 3), "txs": n, "batches": iters,
           "correct": ok, "path": "wire-format txdata RLP through eges_sender_raw_batch; timed around the C-ABI "
                                   "call (ctypes, preallocated outputs)",
           "roofline": dict(roofline(n / (kms / 1e3), W_RECOVER, n, kms, kernel="eges::recover_bkt_kernel"),
                            note="W excludes the fused RLP decode and signing-hash Keccak (conservative)")}
    if cpu:
        out["cpu"] = None
        try:
            from oracle import RefLib, have_ref
            if have_ref():
                ref = RefLib()
                threads = int(os.environ.get("EGES_CPU_THREADS", host_cpus()["threads"]))
                t0 = time.perf_counter()
                ref.ecrecover_batch_mt(sighash, sig_h, 1)
                dt1 = time.perf_counter() - t0
                t0 = time.perf_counter()
                _, _, ret = ref.ecrecover_batch_mt(sighash, sig_h, threads)
                dtn = time.perf_counter() - t0
                assert (ret == 1).all()
                out["cpu"] = {"value": round(n / dtn, 1), "unit": "txs/s", "cores": threads, "kind": "reference",
                              "single_core_txs_per_s": round(n / dt1, 1),
                              "sample": f"the same {n} transfers: reference libsecp256k1 ecrecover (cgo build flags) + "
                                        f"Keccak address, {threads} pthreads ({dtn:.2f} s; 1 core {dt1:.2f} s); sighash "
                                        "RLP + Keccak excluded on the CPU side only (the GPU value includes decode and "
                                        "sighash)"}
        except Exception:
            out["cpu"] = None
    return out


def run_c1(c):
    a = c.args
    n = a.batch or 10000
    iters = max(20, a.steps * 4)
    m = measure_c1(c, n, a.warmup, iters, cpu=not a.no_cpu_baseline)
    line = {"metric": "types.Sender over 10k synthetic EIP-155-signed transfers (configs[0]), from wire bytes",
            "value": m["txs_per_s"], "unit": "txs/s", "ms_per_batch": m["median_ms"], "p99_ms": m["p99_ms"],
            "n_gpus": 1, "steps": iters, "warmup": a.warmup, "higher_is_better": True, "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": f"configs[0]: {n} EIP-155 transfers (nonce i, gasPrice 1, gas 21000, value 1, "
                                   "empty data, chainId 930412) as 10-field txdata RLP through eges_sender_raw_batch "
                                   "(pageable host buffers: H2D + GPU decode + sighash RLP/Keccak + recovery + D2H)",
                       "correct": m["correct"]}, "roofline": m.get("roofline"), "cpu_baseline": m.get("cpu")}
    if m.get("cpu"):
        line["vs_cpu"] = round(m["txs_per_s"] / m["cpu"]["value"], 1)
    c.finish(line, m["correct"])


# ------------------------------------------------------------------ c5: adversarial mix
def measure_c5(c, B, msg, sig, exp_addr, steps, warmup):
    """configs[4] over a device-resident batch (msg, sig valid low-s signatures, exp_addr their
    addresses): 10 % mutated over 7 reject classes, through crypto.Ecrecover and types.Sender
    (EIP155Signer) semantics; every status against its by-construction expectation, every
    accepted item's address against the signer's."""
    import numpy as np
    torch = c.torch
    from eges_amd import txs, workloads
    from eges_amd._lib import SIGNER_EIP155
    sig_h = sig.cpu().numpy()
    kind = workloads.adversarial_mix(sig_h, frac=0.10)
    exp_e = workloads.expected_status(kind, "ecrecover")
    exp_s = workloads.expected_status(kind, "sender")
    r, s, v = workloads.sender_rows_mixed(sig_h, kind, txs.GEEC_CHAIN_ID)
    sig_m = torch.from_numpy(sig_h).to(c.dev)
    rd, sd, vd = (torch.from_numpy(x).to(c.dev) for x in (r, s, v))
    vf = torch.zeros(B, dtype=torch.uint8, device=c.dev)
    addr = torch.empty((B, 20), dtype=torch.uint8, device=c.dev)
    st = torch.empty((B,), dtype=torch.uint8, device=c.dev)
    addr2 = torch.empty((B, 20), dtype=torch.uint8, device=c.dev)
    st2 = torch.empty((B,), dtype=torch.uint8, device=c.dev)

    def step_e():
        c.eges.ecrecover_batch_dev(msg, sig_m, addr=addr, status=st, stream=c.sp)

    def step_s():
        c.eges.sender_batch_dev(msg, rd, sd, vd, vf, SIGNER_EIP155, txs.GEEC_CHAIN_ID, addr=addr2, status=st2,
                                stream=c.sp)

    def reset_e():
        addr.fill_(0xAB)
        st.fill_(0xFF)

    def reset_s():
        addr2.fill_(0xAB)
        st2.fill_(0xFF)

    saved = (c.args.steps, c.args.warmup)
    c.args.steps, c.args.warmup = steps, warmup
    try:
        el_e, _ = c.timed(step_e, reset_e)
        el_s, _ = c.timed(step_s, reset_s)
    finally:
        c.args.steps, c.args.warmup = saved
    got_e, got_s = st.cpu().numpy(), st2.cpu().numpy()
    a_e, a_s, ex = addr.cpu().numpy(), addr2.cpu().numpy(), exp_addr.cpu().numpy()
    okm_e = got_e == 0
    okm_s = got_s == 0
    mism = {"ecrecover_status": int((got_e != exp_e).sum()), "sender_status": int((got_s != exp_s).sum()),
            "ecrecover_addr": int((a_e[okm_e] != ex[okm_e]).any(axis=1).sum()) + int(a_e[~okm_e].any(axis=1).sum()),
            "sender_addr": int((a_s[okm_s] != ex[okm_s]).any(axis=1).sum()) + int(a_s[~okm_s].any(axis=1).sum())}
    return {"batch": B, "sender_sigs_per_s": round(B * steps / el_s, 1), "ecrecover_sigs_per_s": round(B * steps / el_e, 1),
            "kinds": {workloads.KIND_NAMES[k]: int((kind == k).sum()) for k in range(len(workloads.KIND_NAMES))},
            "mismatches": mism, "correct": not any(mism.values())}


def run_adversarial(c):
    a = c.args
    B = a.batch or (1 << 20)
    msg, sig, exp_addr = c.eges.synth_sign_dev(0, B, c.local, stream=c.sp)
    c.torch.cuda.synchronize()
    m = measure_c5(c, B, msg, sig, exp_addr, a.steps, a.warmup)
    line = {"metric": "adversarial-mix sender recovery, bit-exact statuses", "value": m["sender_sigs_per_s"],
            "unit": "sigs/s", "ecrecover_sigs_per_s": m["ecrecover_sigs_per_s"], "n_gpus": 1, "steps": a.steps,
            "warmup": a.warmup, "higher_is_better": True, "dtype": "u32", "data": "synthetic",
            "config": {"workload": "configs[4]: 10% invalid (high-s, bad recid / chain id, r>=n, s>=n, non-residue R, "
                                   "zero r/s); types.Sender (EIP155Signer 930412) and crypto.Ecrecover semantics",
                       "batch": B, "kinds": m["kinds"], "correct": m["correct"], "mismatches": m["mismatches"]}}
    c.finish(line, m["correct"])


# ------------------------------------------------------------------ verify mode
def run_verify(c):
    import numpy as np
    torch, a = c.torch, c.args
    from eges_amd import workloads
    B = a.batch or (1 << 20)
    msg, sig, _ = c.eges.synth_sign_dev(0, B, c.local, stream=c.sp)
    pub = torch.empty((B, 65), dtype=torch.uint8, device=c.dev)
    c.eges.ecrecover_batch_dev(msg, sig, pub=pub, stream=c.sp)
    torch.cuda.synchronize()
    pub_h, sig_h = pub.cpu().numpy(), sig.cpu().numpy()[:, :64].copy()
    n_ = B
    publen = np.full(n_, 65, np.uint8)
    expect = np.ones(n_, np.uint8)
    rng = np.random.default_rng(7)
    # a quarter compressed (02/03 || X), 10% mutated: high-s, wrong key, hybrid 06/07 prefixes
    comp = rng.random(n_) < 0.25
    odd = (pub_h[:, 64] & 1).astype(np.uint8)
    pub_c = pub_h.copy()
    pub_c[comp, 0] = 2 + odd[comp]
    pub_c[comp, 33:] = 0
    publen[comp] = 33
    mut = np.nonzero(rng.random(n_) < 0.10)[0]
    cls = rng.integers(0, 3, len(mut))
    for i, k in zip(mut.tolist(), cls.tolist()):
        if k == 0:  # high-s: VerifySignature always rejects (secp256k1.c:293-308)
            s_ = int.from_bytes(sig_h[i, 32:64].tobytes(), "big")
            sig_h[i, 32:64] = np.frombuffer((workloads.N - s_).to_bytes(32, "big"), np.uint8)
            expect[i] = 0
        elif k == 1:  # wrong key
            j = (i + 1) % n_
            pub_c[i], publen[i] = pub_h[j], 65
            expect[i] = 0
        else:  # hybrid encoding with the right parity is accepted (eckey_impl.h:21-29)
            pub_c[i], publen[i] = pub_h[i], 65
            pub_c[i, 0] = 6 + odd[i]
    pd, ld, sd = (torch.from_numpy(x).to(c.dev) for x in (pub_c, publen, sig_h))
    ok_d = torch.empty((B,), dtype=torch.uint8, device=c.dev)

    def step():
        c.eges.verify_batch_dev(pd, ld, msg, sd, ok=ok_d, stream=c.sp)

    elapsed, kern_ms = c.timed(step, lambda: ok_d.fill_(0xFF))
    got = ok_d.cpu().numpy()
    ok = bool(np.array_equal(got, expect))
    line = {"metric": "crypto.VerifySignature/sec on 1 MI355X", "value": round(B * a.steps / elapsed, 1),
            "unit": "sigs/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "higher_is_better": True,
            "dtype": "u32", "data": "synthetic",
            "config": {"workload": "VerifySignature over 1M signatures: 75% 65-byte / 25% 33-byte keys, 10% mutated "
                                   "(high-s, wrong key, hybrid 06/07)", "batch": B, "correct": ok,
                       "mismatches": int((got != expect).sum())},
            "roofline": roofline(B / (kern_ms / 1e3), W_VERIFY65, B, kern_ms, kernel="eges::verify_kernel")}
    c.finish(line, ok)


# ------------------------------------------------------------------ c2host: host buffers
def measure_host(c, msg_h, sig_h, exp_h, steps, warmup, fresh_reps=3):
    """configs[1]'s batch as host (pageable) buffers through eges_ecrecover_batch (the cgo path of
    signature_cgo.go:31): H2D + prep + recover + D2H in one synchronous call. The caller's output
    arrays are reused across calls (a buffer pool); fresh arrays cost their first-touch page faults
    inside the call, reported beside it as fresh_outputs_sigs_per_s."""
    import numpy as np
    B = msg_h.shape[0]
    out = {}
    oa, os_ = np.zeros((B, 20), np.uint8), np.zeros(B, np.uint8)

    def step(fresh=False):
        out["r"] = c.eges.ecrecover_batch(msg_h, sig_h, want_pub=False, out_addr=None if fresh else oa,
                                          out_status=None if fresh else os_)

    for _ in range(warmup):
        step()
    os_.fill(0xFF)
    oa.fill(0)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    elapsed = time.perf_counter() - t0
    _, addr, st = out["r"]
    ok = bool((st == 0).all()) and np.array_equal(addr, exp_h)
    fresh = None
    if fresh_reps:
        tf = time.perf_counter()
        for _ in range(fresh_reps):
            step(fresh=True)
        fresh = round(B * fresh_reps / (time.perf_counter() - tf), 1)
        _, addr, st = out["r"]
        ok = ok and bool((st == 0).all()) and np.array_equal(addr, exp_h)
    return {"batch": B, "sigs_per_s": round(B * steps / elapsed, 1), "ms_per_call": round(elapsed * 1e3 / steps, 3),
            "steps": steps, "fresh_outputs_sigs_per_s": fresh, "correct": ok}


def run_host_throughput(c):
    torch, a = c.torch, c.args
    B = a.batch or (1 << 20)
    msg, sig, exp_addr = c.eges.synth_sign_dev(0, B, c.local)
    torch.cuda.synchronize()
    r = measure_host(c, msg.cpu().numpy(), sig.cpu().numpy(), exp_addr.cpu().numpy(), a.steps, a.warmup)
    ok = r["correct"]
    line = {"metric": "secp256k1 ecrecover+address/sec, host buffers (PCIe-inclusive)", "value": r["sigs_per_s"],
            "unit": "sigs/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": r["ms_per_call"], "higher_is_better": True, "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "configs[1] batch through eges_ecrecover_batch: pageable host msg/sig in, host "
                                   "addresses + statuses out (H2D + prep + recover + D2H, synchronous call) into "
                                   "reused output arrays",
                       "batch": B, "correct": ok},
            "fresh_outputs_sigs_per_s": r["fresh_outputs_sigs_per_s"]}
    c.finish(line, ok)


def run_c4host(c):
    """--config c4host: configs[3]'s fixed batch handed over as host (pageable) buffers through
    eges_ecrecover_batch with every visible device open in this one process (eges_init(0)): the
    library splits the batch into contiguous shards, one host thread per device (capi run_host),
    the path a Go node with several GPUs takes. Inputs are synthesised on each device for its
    own shard and brought to the host first (untimed); every address is checked."""
    a = c.args
    total = a.batch or C4_TOTAL
    if c.stub:
        t0 = time.perf_counter()
        time.sleep(0.002 * a.steps)
        el = time.perf_counter() - t0
        line = {"metric": "secp256k1 ecrecover+address/sec, host buffers over every device of one process",
                "value": round(total * a.steps / el, 1), "unit": "sigs/s", "devices": 0, "steps": a.steps,
                "data": "stub", "config": {"workload": "c4host stub", "total_batch": total, "correct": True}}
        c.finish(line, True)
        return
    import numpy as np
    torch = c.torch
    from eges_amd.shard import shard_range
    nd = c.eges.device_count()  # every visible gfx950 device (Ctx called eges_init(0))
    msg_h = np.empty((total, 32), np.uint8)
    sig_h = np.empty((total, 65), np.uint8)
    exp_h = np.empty((total, 20), np.uint8)
    ng = torch.cuda.device_count()  # (the synthesis runs per physical device)
    for d in range(ng):
        lo, hi = shard_range(total, d, ng)
        for s0 in range(lo, hi, 1 << 24):  # 16M-signature pieces bound the device memory used
            s1 = min(hi, s0 + (1 << 24))
            with torch.cuda.device(d):
                m, s, e = c.eges.synth_sign_dev(s0, s1 - s0, d)
                torch.cuda.synchronize(d)
                msg_h[s0:s1], sig_h[s0:s1], exp_h[s0:s1] = m.cpu().numpy(), s.cpu().numpy(), e.cpu().numpy()
                del m, s, e
    r = measure_host(c, msg_h, sig_h, exp_h, a.steps, a.warmup, fresh_reps=0)
    line = {"metric": "secp256k1 ecrecover+address/sec, host buffers over every device of one process",
            "value": r["sigs_per_s"], "unit": "sigs/s", "devices": nd, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": r["ms_per_call"], "higher_is_better": True, "dtype": "u32", "data": "synthetic",
            "config": {"workload": f"configs[3] batch of {total} signatures through eges_ecrecover_batch: pageable "
                                   "host msg/sig in, host addresses + statuses out, split over every device in-library "
                                   "(one host thread per device), reused output arrays",
                       "total_batch": total, "shards": [list(shard_range(total, d, nd)) for d in range(nd)],
                       "correct": r["correct"]}}
    c.finish(line, r["correct"])


def main():
    args = parse()
    if args.other_process_kernels:
        other_process_kernels()
        return
    launch_ranks(args)  # --gpus N: one process per GPU (before anything touches the GPU)
    c = Ctx(args)
    if args.stub and args.config not in ("c2", "c4", "c4host"):
        sys.exit("bench.py: --stub rehearses the c2 / c4 / c4host rank logic only")
    if args.config == "c4host":
        run_c4host(c)
        return
    if args.config == "c1":
        run_c1(c)
    elif args.config == "c2":
        run_throughput(c, strong=False)
    elif args.config == "c4":
        run_throughput(c, strong=True)
    elif args.config in ("c3", "c3raw"):
        run_block_latency(c)
    elif args.config == "c2host":
        run_host_throughput(c)
    elif args.config == "c5":
        run_adversarial(c)
    else:
        run_verify(c)


if __name__ == "__main__":
    main()
