"""Host copy cost of a C1-sized wire batch into pinned memory (single-threaded memmove, as the
engine's pinned staging does), median of 50 (tools/passes/gpu_c1k.sh)."""
import ctypes
import time

import numpy as np
import torch

for nbytes in (1_100_000, 210_000):
    src = np.random.default_rng(0).integers(0, 255, nbytes, dtype=np.uint8)
    dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        ctypes.memmove(dst.data_ptr(), src.ctypes.data, nbytes)
        ts.append(time.perf_counter() - t0)
    print(f"memmove {nbytes} B into pinned: median {1e6 * sorted(ts)[25]:.1f} us")
