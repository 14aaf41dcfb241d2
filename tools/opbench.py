"""Per-operation cost on the GPU (SIMD-cycles per lane-op at 2.4 GHz nominal, 2 waves/SIMD)."""
import ctypes
import os

import torch  # noqa: F401  (share the HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "eges_amd", "libeges_selftest.so"))
lib.eges_opbench.restype = ctypes.c_double
lib.eges_opbench.argtypes = [ctypes.c_int, ctypes.c_int]
names = ["fe_mul", "fe_sqr", "gej_double", "gej_add_ge", "fe_normalize(add)", "normalize_weak(sub)", "sc_mul",
         "fe_is_zero+add+nw"]
reps = [4000, 4000, 500, 400, 4000, 4000, 2000, 2000]
for i, n in enumerate(names):
    print(f"{n:24s} {lib.eges_opbench(i, reps[i]):8.2f} SIMD-cycles/lane-op")
