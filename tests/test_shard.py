"""Multi-rank sharding of the batch path on CPU (gloo, world_size 2): every rank takes its
contiguous index range (eges_amd.shard, the rule bench.py and libeges.so use), computes the
per-item work of its shard with host code, and the gathered result must equal the
single-process result for the whole batch — no item lost, duplicated or reordered."""
import os
import socket

import numpy as np
import pytest

from eges_amd.shard import gather_shards, shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 1000, 1 << 20, 1000003):
        for world in (1, 2, 3, 4, 8):
            cover = []
            prev_hi = 0
            for r in range(world):
                lo, hi = shard_range(n, r, world)
                assert lo == prev_hi and lo <= hi
                prev_hi = hi
                cover.append(hi - lo)
            assert prev_hi == n and sum(cover) == n
            assert max(cover) - min(cover) <= -(-n // world)
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _item_work(idx):
    """Per-signature stand-in computed on the host: the address-derivation Keccak of a
    synthetic 64-byte public key (libeges.so's host Keccak-256, crypto.go:194-197)."""
    import eges_amd
    out = np.zeros((len(idx), 20), np.uint8)
    for k, i in enumerate(idx):
        pub = int(i).to_bytes(8, "little") * 8
        out[k] = np.frombuffer(eges_amd.keccak256(pub)[12:], np.uint8)
    return out


def _rank_main(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n, rank, world)
    mine = _item_work(range(lo, hi))
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    if rank == 0:
        q.put(gather_shards(parts))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n", [1001, 2])
def test_gloo_two_ranks_gather_equals_single(n):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.array_equal(got, _item_work(range(n)))


def _records(idx):
    """[len(idx), 21] (address, status) records of the stand-in work, status = index mod 7."""
    addr = _item_work(idx)
    st = np.array([i % 7 for i in idx], np.uint8).reshape(-1, 1)
    return np.concatenate([addr, st], 1) if len(addr) else np.zeros((0, 21), np.uint8)


def _rank_all_gather(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from eges_amd.shard import all_gather_records
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n, rank, world)
    got = all_gather_records(torch.from_numpy(_records(range(lo, hi))), n)
    bad = 0
    try:
        all_gather_records(torch.zeros((hi - lo + 1, 21), dtype=torch.uint8), n)
    except ValueError:
        bad = 1
    # only rank 1's shard is malformed: both ranks must raise (no rank left in the all-gather)
    shard = torch.from_numpy(_records(range(lo, hi + (1 if rank == 1 else 0))))
    try:
        all_gather_records(shard, n)
    except ValueError:
        bad += 1
    q.put((rank, got.numpy().copy(), bad))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [1001, 2, 1])
def test_gloo_all_gather_records_every_rank(n):
    """eges_amd.shard.all_gather_records (the optional exchange of SURVEY §8(e)): every rank
    ends with the whole batch's records in index order, shards ragged or empty."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_all_gather, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = _records(range(n))
    for rank, got, bad in outs:
        assert got.shape == (n, 21) and np.array_equal(got, want), rank
        assert bad == 2  # a shard of the wrong size (on every rank, or on one) is refused on every rank


def _bench(args, env_extra=None, timeout=240):
    """bench.py as the driver runs it (no launcher: --gpus N starts torch.distributed.run itself)."""
    import json
    import subprocess
    import sys

    from conftest import ROOT
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.parametrize("config", ["c2", "c4"])
def test_bench_rank_logic_two_ranks(config):
    """bench.py's own rank logic at world size 2 on the CPU (--stub: gloo, a timed sleep as the
    step): --gpus 2 launches two ranks, each takes its shard (weak: its own batch; strong:
    shard_range of the fixed total), times between barriers, the max over ranks and the
    correctness reduce come back to rank 0, whose line names both ranks."""
    rc, line, err = _bench(["--stub", "--gpus", "2", "--steps", "3", "--warmup", "1", "--config", config,
                            "--batch", "1001", "--c4-total", "3001"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2 and len(line["ranks"]) == 2
    assert sorted(r["rank"] for r in line["ranks"]) == [0, 1]
    sh = line["config"]["shards"]
    if config == "c4":
        assert sh == [list(shard_range(1001, r, 2)) for r in range(2)] and line["scaling"] == "strong"
        assert line["config"]["total_batch"] == 1001
    else:
        assert sh == [[0, 1001], [1001, 2002]] and line["scaling"] == "weak"
        assert line["config"]["total_batch"] == 2002
    # value = all ranks' items / the max elapsed over ranks (3 steps of >= 2 ms each)
    assert line["ms_per_step"] >= 2.0
    assert abs(line["value"] - line["config"]["total_batch"] * 3 / (line["ms_per_step"] * 3 / 1e3)) \
        <= 1e-3 * line["value"] + 1.0
    assert line["config"]["correct"] is True
    if config == "c2":
        # the configs[3] strong-scaled leg every default line carries
        c4 = line["secondary"]["c4_strong"]
        assert c4["shards"] == [list(shard_range(3001, r, 2)) for r in range(2)] and c4["scaling"] == "strong"
        assert len(c4["rank_kernel_ms"]) == 2 and len(c4["rank_elapsed_ms_per_step"]) == 2
        assert c4["imbalance_max_over_min"] >= 1.0 and c4["correct"] is True
        assert abs(c4["sigs_per_s"] - 3001 * c4["steps"] / (c4["ms_per_step"] * c4["steps"] / 1e3)) <= 1e-3 * c4["sigs_per_s"] + 1
        # rank 0's child over every device of one process (stubbed: no GPU here)
        assert line["secondary"]["c4_host_all_devices"]["config"]["total_batch"] == 3001


def test_bench_correctness_reduce_and_world_check():
    """one rank's mismatch fails the whole line (rc != 0, correct false on rank 0); a launcher
    whose WORLD_SIZE differs from --gpus is refused"""
    rc, line, _ = _bench(["--stub", "--gpus", "2", "--steps", "2", "--warmup", "0"], {"EGES_BENCH_STUB_BAD_RANK": "1"})
    assert rc != 0 and line["config"]["correct"] is False
    assert line["secondary"]["c4_strong"]["correct"] is False  # the bad rank's strong-leg check reaches rank 0
    rc, line, err = _bench(["--stub", "--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc == 2 and line is None and "WORLD_SIZE=3" in err


def test_strong_summary_imbalance():
    """bench.strong_summary: the slowest rank sets the rate, idle (empty) shards are left out of
    the imbalance, and one rank's failed check fails the leg."""
    import importlib.util
    from conftest import ROOT
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    sh = [shard_range(3, r, 4) for r in range(4)]  # [0,1) [1,2) [2,3) [3,3)
    s = b.strong_summary(3, sh, 2, [(0.2, 10.0, True), (0.4, 20.0, True), (0.3, 15.0, True), (0.1, 0.0, True)])
    assert s["ms_per_step"] == 200.0 and s["sigs_per_s"] == 15.0
    assert s["imbalance_max_over_min"] == 2.0 and s["correct"] is True
    s = b.strong_summary(3, sh, 2, [(0.2, 10.0, True), (0.4, 20.0, False), (0.3, 15.0, True), (0.1, 0.0, True)])
    assert s["correct"] is False
