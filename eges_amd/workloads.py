"""Synthetic workloads of BASELINE.json configs[4] (C5): an adversarial mix of invalid
signatures whose expected status is known by construction.

adversarial_mix() mutates ~frac of a batch of valid, low-s signatures, uniformly over the
reject classes below, and returns per item the class and the exact status the reference
returns for it in each mode:
  - crypto.Ecrecover (crypto/secp256k1/secp256.go:105-122, recovery/main_impl.h:38-121):
      HIGH_S      s -> n - s, recid ^ 1: accepted, same public key (Frontier-style malleability)
      BAD_RECID   recid in 4..255: ErrInvalidRecoveryID (secp256.go:175-177)
      R_GE_N      r in [n, 2^256): parse_compact overflow -> ErrRecoverFailed
      S_GE_N      s in [n, 2^256): same
      NONRESIDUE  r < n with r^3 + 7 a non-residue mod p, recid < 2: ErrRecoverFailed
      ZERO_R      r = 0: ErrRecoverFailed (main_impl.h:96-98)
      ZERO_S      s = 0: same
  - types.Sender with EIP155Signer(chain_id) (transaction_signing.go:127-137,222-247): the same
    items with V = recid + 35 + 2 chain_id; HIGH_S, R_GE_N, S_GE_N, ZERO_R, ZERO_S ->
    ErrInvalidSig (crypto.ValidateSignatureValues, crypto.go:181-192, homestead low-s);
    NONRESIDUE -> ErrRecoverFailed; BAD_RECID becomes a V of another chain id (1) ->
    ErrInvalidChainId.
"""
import numpy as np

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
P = 2**256 - 2**32 - 977

VALID, HIGH_S, BAD_RECID, R_GE_N, S_GE_N, NONRESIDUE, ZERO_R, ZERO_S = range(8)
KIND_NAMES = ["valid", "high_s", "bad_recid", "r_ge_n", "s_ge_n", "nonresidue", "zero_r", "zero_s"]

# statuses (include/eges.h)
OK, INVALID_CHAIN_ID, INVALID_SIG, INVALID_RECOVERY_ID, RECOVER_FAILED = 0, 1, 2, 5, 6

EXPECT_ECRECOVER = {VALID: OK, HIGH_S: OK, BAD_RECID: INVALID_RECOVERY_ID, R_GE_N: RECOVER_FAILED,
                    S_GE_N: RECOVER_FAILED, NONRESIDUE: RECOVER_FAILED, ZERO_R: RECOVER_FAILED,
                    ZERO_S: RECOVER_FAILED}
EXPECT_SENDER = {VALID: OK, HIGH_S: INVALID_SIG, BAD_RECID: INVALID_CHAIN_ID, R_GE_N: INVALID_SIG,
                 S_GE_N: INVALID_SIG, NONRESIDUE: RECOVER_FAILED, ZERO_R: INVALID_SIG, ZERO_S: INVALID_SIG}


def _be(x):
    return np.frombuffer(int(x).to_bytes(32, "big"), np.uint8)


def _nonresidue_x(rng):
    """A random x < n with x^3 + 7 a quadratic non-residue mod p (no curve point has x)."""
    while True:
        x = int.from_bytes(rng.bytes(32), "big") % N
        if pow((x * x * x + 7) % P, (P - 1) // 2, P) == P - 1:
            return x


def _be_rows(xs):
    """32-byte big-endian rows of a list of Python ints (one join, no per-item arrays)."""
    return np.frombuffer(b"".join(int(x).to_bytes(32, "big") for x in xs), np.uint8).reshape(-1, 32)


def adversarial_mix(sig, frac=0.10, seed=20191015):
    """Mutate ~frac of sig (n, 65) uint8 (R || S || recid, valid low-s signatures) in place.
    Returns kind (n,) uint8. The per-mode expectation is expected_status(kind, mode).
    Vectorised per class (1M signatures in well under a second); non-residue x values come from
    a pool of 256 drawn per call."""
    rng = np.random.default_rng(seed)
    n = sig.shape[0]
    kind = np.zeros(n, np.uint8)
    m = int(round(n * frac))
    if m == 0:
        return kind
    idx = rng.choice(n, m, replace=False)
    cls = rng.integers(1, len(KIND_NAMES), m).astype(np.uint8)
    kind[idx] = cls
    at = {c: np.sort(idx[cls == c]) for c in range(1, len(KIND_NAMES))}
    i = at[HIGH_S]
    if i.size:
        sig[i, 32:64] = _be_rows(N - int.from_bytes(sig[k, 32:64].tobytes(), "big") for k in i.tolist())
        sig[i, 64] ^= 1
    i = at[BAD_RECID]
    sig[i, 64] = rng.integers(4, 256, i.size).astype(np.uint8)
    for c, lo in ((R_GE_N, 0), (S_GE_N, 32)):
        i = at[c]
        if i.size:
            sig[i, lo:lo + 32] = _be_rows(N + int(o) for o in rng.integers(0, 2**62, i.size).tolist())
    i = at[NONRESIDUE]
    if i.size:
        pool = _be_rows(_nonresidue_x(rng) for _ in range(256))
        sig[i, 0:32] = pool[rng.integers(0, 256, i.size)]
        sig[i, 64] &= 1
    sig[at[ZERO_R], 0:32] = 0
    sig[at[ZERO_S], 32:64] = 0
    return kind


def expected_status(kind, mode):
    """Per-item status the reference returns: mode 'ecrecover' or 'sender' (EIP-155)."""
    table = EXPECT_ECRECOVER if mode == "ecrecover" else EXPECT_SENDER
    lut = np.array([table[k] for k in range(len(KIND_NAMES))], np.uint8)
    return lut[kind]


def sender_rows_mixed(sig, kind, chain_id, other_chain_id=1):
    """r, s, v rows for an EIP155Signer(chain_id) batch over the mixed signatures: BAD_RECID
    items carry V of other_chain_id (with their recid reduced to 0/1)."""
    n = sig.shape[0]
    r = sig[:, :32].copy()
    s = sig[:, 32:64].copy()
    v = np.zeros((n, 32), np.uint8)
    bad = kind == BAD_RECID
    vv = np.where(bad, (sig[:, 64] & 1).astype(np.uint64) + np.uint64(35 + 2 * other_chain_id),
                  sig[:, 64].astype(np.uint64) + np.uint64(35 + 2 * chain_id))
    for k in range(8):
        v[:, 31 - k] = ((vv >> np.uint64(8 * k)) & np.uint64(0xFF)).astype(np.uint8)
    return r, s, v
