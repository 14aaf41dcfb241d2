"""Same-box A/B of the row-form inversion latency (tools/passes/gpu_r04_c.sh): the product selftest
library (scalar-ALU divsteps in assembly, EGES_DIVSTEPS_ASM=1) against tools/abbase's build of
the compiled C loop (EGES_DIVSTEPS_ASM=0), alternating; mean s_memtime cycles per inversion at
one wave per CU. Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = {"asm": os.path.join(ROOT, "eges_amd", "libeges_selftest.so"),
        "c": os.path.join(ROOT, "tools", "abbase", "libeges_selftest.so")}
import torch  # noqa: E402,F401  (share the HIP runtime)
out = {k: {"mod_p": [], "mod_n": []} for k in libs}
L = {}
for k, p in libs.items():
    L[k] = ctypes.CDLL(p)
    L[k].eges_inv_latency.argtypes = [ctypes.c_int, ctypes.c_int]
    L[k].eges_inv_latency.restype = ctypes.c_double
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for k in libs:
        out[k]["mod_p"].append(round(L[k].eges_inv_latency(0, 64)))
        out[k]["mod_n"].append(round(L[k].eges_inv_latency(1, 64)))
print(json.dumps({"metric": "row-form inversion, cycles per inversion (one wave per CU)", **out}))
