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
