"""CPU tests of the C-ABI library: it loads, exports every symbol include/eges.h declares, and
fails loudly (no CPU fallback) when no GPU is present. No compute calls are made here."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "eges.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(eges_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entries():
    syms = declared_symbols()
    for must in ("eges_init", "eges_ecdsa_recover", "eges_ecdsa_verify", "eges_ecrecover_batch",
                 "eges_sender_batch", "eges_verify_batch", "eges_ecrecover_batch_dev"):
        assert must in syms


def test_library_exports_all_declared_symbols():
    from eges_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    # the Python binding covers the same set
    assert set(_lib.SIGNATURES) == set(declared_symbols())


def test_host_keccak_matches_kat():
    import eges_amd
    assert eges_amd.keccak256(b"abc").hex() == "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"
    assert eges_amd.keccak256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    # multi-block (> 136 bytes) against the oracle restatement
    from oracle import Oracle
    o = Oracle()
    for n in (135, 136, 137, 300, 1000):
        data = bytes((i * 7 + 3) & 0xFF for i in range(n))
        assert eges_amd.keccak256(data) == o.keccak256(data)


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import numpy as np

    import eges_amd
    from eges_amd._lib import EGES_E_NODEVICE, EgesError
    with pytest.raises(EgesError) as ei:
        eges_amd.ecrecover_batch(np.zeros((1, 32), np.uint8), np.zeros((1, 65), np.uint8))
    assert ei.value.rc == EGES_E_NODEVICE
    # single-item entry returns 0 (failure), exactly like the replaced C function would on error
    from eges_amd._lib import lib
    pub = (ctypes.c_ubyte * 65)()
    sig = (ctypes.c_ubyte * 65)()
    msg = (ctypes.c_ubyte * 32)()
    assert lib.eges_ecdsa_recover(pub, sig, msg) == 0


def test_null_and_empty_inputs():
    from eges_amd._lib import EGES_E_NULLPTR, EGES_SUCCESS, lib
    assert lib.eges_ecrecover_batch(None, None, 0, None, None, None) == EGES_SUCCESS  # n == 0 is a no-op
    assert lib.eges_ecrecover_batch(None, None, 5, None, None, None) == EGES_E_NULLPTR
    assert lib.eges_verify_batch(None, None, None, None, 3, None) == EGES_E_NULLPTR
    assert lib.eges_abi_version() == 1


def test_knobs_set_and_read_without_gpu():
    """Engine knobs are changed through eges_test_set_knob, not the environment (read once, at the
    first eges_init): the setter works before init and without a device, unknown names fail."""
    import eges_amd
    from eges_amd._lib import EGES_E_INVALID_ARG, EgesError, lib
    old = eges_amd.get_knob("EGES_LAT_MAX")
    with eges_amd.knob("EGES_LAT_MAX", 17):
        assert eges_amd.get_knob("EGES_LAT_MAX") == 17
    assert eges_amd.get_knob("EGES_LAT_MAX") == old
    for name in ("EGES_LAT_WIDE_MAX", "EGES_MID_MAX", "EGES_MID_FORM", "EGES_WIRE_FUSED", "EGES_TXROWS_WAVE_MAX", "EGES_TEST_ROOT_HELPERS",
                 "EGES_OVERLAP", "EGES_TEST_FORCE_REDO", "EGES_COALESCE_GATHER_US", "EGES_COALESCE_SPIN_US",
                 "EGES_COALESCE_SPINNERS"):
        eges_amd.get_knob(name)
    # the defaults DESIGN.md documents (measured choices: the resident single-call server and the
    # input gate on); round 5 removed the measured-slower pinned pipeline, second host stream and
    # resident block server, so their names are unknown now
    defaults = {"EGES_RESIDENT": 1, "EGES_GATE": 1, "EGES_GATE_STEP": 8, "EGES_VERIFY_MID_GENS": 2, "EGES_HOST_PARTS": 8,
                "EGES_LAT_TRI_MAX": 448, "EGES_SENDER_FUSED": 1}
    for name, want in defaults.items():
        assert eges_amd.get_knob(name) == want, name
    for name in ("EGES_RESIDENT_WGS", "EGES_RESIDENT_CAP", "EGES_RESIDENT_IDLE_US", "EGES_TEST_DELAY_X",
                 "EGES_TEST_SKIP_FLAG"):
        eges_amd.get_knob(name)
    for gone in ("EGES_HOST_PIPE", "EGES_PIPE_SEG", "EGES_HOST_STREAMS", "EGES_RESIDENT_BLOCK",
                 "EGES_RESIDENT_BLOCK_CAP", "EGES_HOST_ONE", "EGES_HOST_FEEDERS", "EGES_TEST_HOST_ONE"):
        assert lib.eges_test_set_knob(gone.encode(), 1) == EGES_E_INVALID_ARG, gone
    assert lib.eges_test_set_knob(b"EGES_NO_SUCH_KNOB", 1) == EGES_E_INVALID_ARG
    with pytest.raises(EgesError):
        eges_amd.get_knob("EGES_NO_SUCH_KNOB")


def test_no_getenv_on_call_paths():
    """The product sources read the environment only in eges_init / init_device / knobs_load_env
    (VERDICT r2 item 5): no getenv in any kernel launcher or call path."""
    import glob
    for f in glob.glob(os.path.join(ROOT, "eges_amd", "csrc", "*.hip")) + glob.glob(
            os.path.join(ROOT, "eges_amd", "csrc", "*.cuh")):
        if os.path.basename(f) == "selftest.hip":
            continue
        src = open(f).read()
        n = len(re.findall(r"getenv\(", src))
        if os.path.basename(f) == "engine.hip":
            # env_int (init_device / eges_init) and knobs_load_env
            assert n == 2, n
        else:
            assert n == 0, f
        for m in re.finditer(r"env_int\(\"(EGES_[A-Z_]+)\"", src):
            assert os.path.basename(f) in ("engine.hip", "capi.hip"), f
            assert m.group(1) in ("EGES_GRID_MULT", "EGES_TEST_MAX_BLOCKS", "EGES_TEST_LOGICAL_DEVICES"), m.group(1)
