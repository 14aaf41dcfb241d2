"""Index sharding of a signature batch across ranks / devices.

Every signature is independent, so a batch of n items splits into contiguous index ranges,
one per rank: rank g gets [g * ceil(n / G), min(n, (g + 1) * ceil(n / G))). No data-path
collective is needed; each rank returns its own 21-byte (address, status) records and the
caller concatenates them in rank order. libeges.so applies the same rule to the devices of
one process (hostpath.hip, run_host).
"""


def shard_range(n, rank, world):
    """Contiguous [lo, hi) index range of `rank` out of `world` for a batch of n items."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    if n < 0:
        raise ValueError("n < 0")
    per = -(-n // world) if n else 0
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    return lo, hi


def gather_shards(parts):
    """Concatenate per-rank results (numpy arrays, rank order) into one batch."""
    import numpy as np
    parts = [np.asarray(p) for p in parts]
    return np.concatenate(parts, axis=0) if parts else np.zeros(0)


RECORD = 21  # one item's result: 20-byte address + 1 status byte (eges_recover_* outputs)


def all_gather_records(local, n, group=None):
    """Optional exchange for consumers that want the whole batch's senders on every rank
    (no reference analog — the Go node recovers on one host).

    `local` is this rank's [hi - lo, 21] uint8 tensor of (address, status) records for its
    shard_range(n, rank, world) slice, on the rank's device (RCCL over xGMI with the "nccl"
    backend) or on the CPU (gloo). Every shard is padded to ceil(n / world) records so the
    collective is one fixed-size all-gather; the result is the [n, 21] batch in index order on
    every rank. It is outside the recovery path: bench.py's timed region never calls it.

    The ranks first agree on whether every shard is well formed (one MIN all-reduce of a 0/1
    flag), so a bad shard on one rank raises ValueError on every rank instead of leaving the
    others blocked in the all-gather until the process-group timeout.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_range(n, rank, world)
    good = local.dtype == torch.uint8 and local.dim() == 2 and tuple(local.shape) == (hi - lo, RECORD)
    flag = torch.tensor([1 if good else 0], dtype=torch.int32, device=local.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    if not good:
        raise ValueError(f"rank {rank}: expected uint8 [{hi - lo}, {RECORD}] records, got "
                         f"{local.dtype} {tuple(local.shape)}")
    if int(flag.item()) == 0:
        raise ValueError(f"rank {rank}: another rank passed a malformed shard; no records exchanged")
    per = -(-n // world) if n else 0
    if per == 0:
        return local.new_zeros((0, RECORD))
    send = local.new_zeros((per, RECORD))
    send[: hi - lo] = local
    recv = [local.new_empty((per, RECORD)) for _ in range(world)]
    dist.all_gather(recv, send, group=group)
    rows = [recv[g][: shard_range(n, g, world)[1] - shard_range(n, g, world)[0]] for g in range(world)]
    return torch.cat(rows, 0)
