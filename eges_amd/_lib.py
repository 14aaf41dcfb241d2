"""ctypes binding of libeges.so (include/eges.h).

The shared library is built in-tree (eges_amd/libeges.so, see __graft_entry__.build()).
There is no Python or CPU fallback: if the library is missing this module raises on import,
and every compute entry returns EGES_E_NODEVICE when no gfx950 GPU is usable.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# EGES_LIB: another build of the library in this directory (same-box A/B runs); default libeges.so
LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ.get("EGES_LIB", "libeges.so")))
# Same-box A/B tooling only (tools/passes/gpu_*.sh): another build of the same sources, e.g. with one
# optimisation compiled out, in place of the product library.
if os.environ.get("EGES_AB_LIB"):
    LIB_PATH = os.path.abspath(os.environ["EGES_AB_LIB"])

# include/eges.h
EGES_OK = 0
EGES_INVALID_CHAIN_ID = 1
EGES_INVALID_SIG = 2
EGES_INVALID_MSG_LEN = 3
EGES_INVALID_SIG_LEN = 4
EGES_INVALID_RECOVERY_ID = 5
EGES_RECOVER_FAILED = 6
EGES_DECODE_FAILED = 7

EGES_SUCCESS = 0
EGES_E_NULLPTR = -1
EGES_E_NODEVICE = -2
EGES_E_HIP = -3
EGES_E_INVALID_ARG = -4
EGES_E_NOMEM = -5

SIGNER_FRONTIER = 0
SIGNER_HOMESTEAD = 1
SIGNER_EIP155 = 2

LIST_FAKE = 1
LIST_GEEC = 2
LIST_TXS = 4

VF_V_WIDE = 1
VF_R_WIDE = 2
VF_S_WIDE = 4

# every symbol include/eges.h declares, with (restype, argtypes)
_P = ctypes.c_void_p
_SZ = ctypes.c_size_t
_U64 = ctypes.c_uint64
_I = ctypes.c_int
_U32 = ctypes.c_uint32
SIGNATURES = {
    "eges_init": (_I, [_U32, _U32]),
    "eges_shutdown": (None, []),
    "eges_device_count": (_I, []),
    "eges_last_error": (ctypes.c_char_p, []),
    "eges_abi_version": (_I, []),
    "eges_ecdsa_recover": (_I, [_P, _P, _P]),
    "eges_ecdsa_verify": (_I, [_P, _P, _P, _SZ]),
    "eges_ecrecover_batch": (_I, [_P, _P, _SZ, _P, _P, _P]),
    "eges_sender_batch": (_I, [_P, _P, _P, _P, _P, _SZ, _I, _U64, _P, _P]),
    "eges_sender_raw_batch": (_I, [_P, _P, _SZ, _I, _U64, _P, _P, _P]),
    "eges_ecrecover_precompile_batch": (_I, [_P, _P, _SZ, _P, _P]),
    "eges_block_senders_raw": (_I, [_P, _SZ, _U32, _I, _U64, _SZ, _P, _P, _P, _P]),
    "eges_verify_batch": (_I, [_P, _P, _P, _P, _SZ, _P]),
    "eges_ecrecover_batch_dev": (_I, [_I, _P, _P, _SZ, _P, _P, _P, _P]),
    "eges_sender_batch_dev": (_I, [_I, _P, _P, _P, _P, _P, _SZ, _I, _U64, _P, _P, _P]),
    "eges_sender_raw_batch_dev": (_I, [_I, _P, _P, _SZ, _I, _U64, _P, _P, _P, _P]),
    "eges_ecrecover_precompile_batch_dev": (_I, [_I, _P, _P, _SZ, _P, _P, _P]),
    "eges_verify_batch_dev": (_I, [_I, _P, _P, _P, _P, _SZ, _P, _P]),
    "eges_keccak256": (None, [_P, _SZ, _P]),
    "eges_synth_sign_dev": (_I, [_I, _U64, _SZ, _P, _P, _P, _P]),
    "eges_synth_sign_msg_dev": (_I, [_I, _U64, _SZ, _P, _P, _P, _P]),
    "eges_diag_counters": (_I, [_I, _P, _SZ, _I]),
    "eges_diag_resident_running": (_I, [_I]),
    "eges_test_set_knob": (_I, [ctypes.c_char_p, ctypes.c_longlong]),
    "eges_test_get_knob": (_I, [ctypes.c_char_p, _P]),
}

# EGES_DIAG_* (include/eges.h): rare exact branches the kernels count
DIAG_NAMES = ["ls_redo", "ls_exc", "lat_redo", "lat_exc", "comb_redo", "join_dbl", "join_inf", "mid_redo",
              "mid_exc", "mid_join", "handoff", "lat_tri", "resident"]
ENGINE_FAULT = 255  # EGES_ENGINE_FAULT: an item whose in-kernel wave hand-off timed out
DIAG_COUNT = 16


class EgesError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__(f"eges error {rc}: {msg}")
        self.rc = rc


def _bind_process_hip_runtime():
    """Make libeges.so share the process's HIP runtime with PyTorch.

    torch's wheel ships its own libamdhip64 (SONAME libamdhip64.so.7, loaded as "libamdhip64.so"
    from torch/lib). If libeges.so were loaded first, its NEEDED libamdhip64.so.7 would pull the
    /opt/rocm copy and torch would later load a second runtime that cannot open the GPU. Loading
    torch first lets the dynamic loader satisfy libeges.so's NEEDED entry with torch's copy, so
    device pointers and streams are shared between the two.
    """
    try:
        import torch  # noqa: F401
    except Exception:  # torch is optional for the host-buffer API
        pass


def _load():
    _bind_process_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc):
    if rc != EGES_SUCCESS:
        raise EgesError(rc, lib.eges_last_error().decode(errors="replace"))
    return rc
