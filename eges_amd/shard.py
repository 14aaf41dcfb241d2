"""Index sharding of a signature batch across ranks / devices.

Every signature is independent, so a batch of n items splits into contiguous index ranges,
one per rank: rank g gets [g * ceil(n / G), min(n, (g + 1) * ceil(n / G))). No data-path
collective is needed; each rank returns its own 21-byte (address, status) records and the
caller concatenates them in rank order. libeges.so applies the same rule to the devices of
one process (capi.hip, run_host).
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
