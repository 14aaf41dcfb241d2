"""How the resident single-call server's idle window (EGES_RESIDENT_IDLE_US) delays another
process's kernel on the same GPU: this process makes one eges_ecdsa_recover call (the server starts
and polls for the idle window) and a second process (tests/gpu_child.py other_process_kernels)
launches a device-resident 1M batch right after; the same with the server stopped. Medians over
6 alternating pairs per idle value; one JSON line per value."""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import ctypes
    import eges_amd
    from eges_amd import _lib
    from conftest import load_golden
    eges_amd.init(1)
    g = load_golden("recover.npz")
    i = int(np.nonzero((g["status"] == 0) & (g["sig"][:, 64] < 4))[0][0])

    def single():
        out = (ctypes.c_ubyte * 65)()
        return _lib.lib.eges_ecdsa_recover(out, g["sig"][i].tobytes(), g["msg"][i].tobytes())

    child = subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "gpu_child.py"), "other_process_kernels"],
                             stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    assert child.stdout.readline().strip() == "ready"

    def go():
        child.stdin.write("go\n")
        child.stdin.flush()
        return float(child.stdout.readline())

    try:
        for idle in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4000,2000,1000,500").split(",")]:
            eges_amd.set_knob("EGES_RESIDENT_IDLE_US", idle)
            on, off = [], []
            for _ in range(6):
                eges_amd.set_knob("EGES_RESIDENT", 1)
                assert single() == 1
                on.append(go())
                time.sleep(0.02)
                eges_amd.set_knob("EGES_RESIDENT", 0)
                single()
                time.sleep(0.02)
                off.append(go())
            print(json.dumps({"idle_us": idle, "other_kernel_ms_server_alive": round(float(np.median(on)), 3),
                              "other_kernel_ms_server_stopped": round(float(np.median(off)), 3),
                              "ratio": round(float(np.median(on)) / float(np.median(off)), 4), "on": on, "off": off}),
                  flush=True)
    finally:
        child.stdin.close()
        child.wait(timeout=60)
    eges_amd.set_knob("EGES_RESIDENT", 1)


if __name__ == "__main__":
    main()
