"""eges_amd — MI355X-native batched secp256k1 sender recovery for the EGES / Geec chain.

Hot path: crypto.Ecrecover -> Keccak-256 address (and crypto.VerifySignature, types.Sender),
executed by hand-written HIP kernels for gfx950 behind the C-ABI in include/eges.h.
The Python modules mirror the reference's Go API (crypto, crypto/secp256k1, core/types) so
the parity tests read like the reference's own tests.
"""
from . import _lib  # noqa: F401  (raises ImportError if libeges.so is missing: no fallback)
from .engine import (block_senders_raw, device_count, diag_counters, get_knob, knob, set_knob, ecrecover_batch, ecrecover_batch_dev, init, keccak256,  # noqa: F401
                     ecrecover_precompile_batch, ecrecover_precompile_batch_dev, pack_raw, sender_batch, sender_batch_dev, sender_raw_batch, sender_raw_batch_dev,
                     synth_sign_dev, synth_sign_msg_dev, verify_batch, verify_batch_dev)

__all__ = ["init", "device_count", "ecrecover_batch", "sender_batch", "verify_batch", "keccak256",
           "ecrecover_batch_dev", "sender_batch_dev", "verify_batch_dev", "synth_sign_dev", "synth_sign_msg_dev",
           "pack_raw", "sender_raw_batch", "sender_raw_batch_dev", "ecrecover_precompile_batch",
           "ecrecover_precompile_batch_dev", "block_senders_raw", "set_knob", "get_knob", "knob", "diag_counters"]
