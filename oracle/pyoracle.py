"""ctypes wrappers of the oracle libraries (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py)."""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libeges_ref.so")


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


# EGES_ORACLE_RECORD=<file>: append every call made through these wrappers (inputs and outputs)
# to <file>, so that `make -C oracle sanitize` can replay the Python tests' exact calls in the
# ASan/UBSan build (oracle/sanitize_main.c --replay). Record: u8 op, u8 nfields, then per field
# u32 length + bytes; ints are 8-byte little-endian.
_RECORD = os.environ.get("EGES_ORACLE_RECORD")
OPS = dict(keccak256=1, sponge=2, recover_pubkey=3, recover_batch=4, verify=5, sender=6, pub_to_addr=7,
           eref_ecrecover=8, eref_batch_mt=9)


def _rec(op, *fields):
    if not _RECORD:
        return
    out = bytearray([OPS[op], len(fields)])
    for f in fields:
        b = int(f).to_bytes(8, "little", signed=True) if isinstance(f, (int, np.integer)) else bytes(f)
        out += len(b).to_bytes(4, "little") + b
    with open(_RECORD, "ab") as fh:
        fh.write(out)


def have_ref():
    return os.path.exists(REF_SO)


class Oracle:
    """This repo's CPU restatement (oracle/oracle.c)."""

    def __init__(self):
        if not os.path.exists(ORACLE_SO):
            raise FileNotFoundError(f"{ORACLE_SO} missing: run `make -C oracle`")
        L = ctypes.CDLL(ORACLE_SO)
        P, SZ, I, U64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
        L.oracle_keccak256.argtypes = [P, SZ, P]
        L.oracle_sponge.argtypes = [P, SZ, P, SZ, I, ctypes.c_ubyte]
        L.oracle_ext_ecdsa_recover.argtypes = [P, P, P]
        L.oracle_recover_pubkey.argtypes = [P, P, P]
        L.oracle_ext_ecdsa_verify.argtypes = [P, P, P, SZ]
        L.oracle_verify_signature.argtypes = [P, SZ, P, SZ, P, SZ]
        L.oracle_sender.argtypes = [P, I, U64, P, P, P, P, I]
        L.oracle_pub_to_addr.argtypes = [P, P]
        L.oracle_recover_batch.argtypes = [SZ, P, P, P, P, P]
        self.L = L

    def keccak256(self, data: bytes) -> bytes:
        a = np.frombuffer(bytes(data) or b"\0", np.uint8)
        out = np.zeros(32, np.uint8)
        self.L.oracle_keccak256(_p(a), len(data), _p(out))
        _rec("keccak256", bytes(data), out)
        return out.tobytes()

    def sponge(self, data: bytes, outlen: int, rate: int, ds: int) -> bytes:
        a = np.frombuffer(bytes(data) or b"\0", np.uint8)
        out = np.zeros(outlen, np.uint8)
        self.L.oracle_sponge(_p(a), len(data), _p(out), outlen, rate, ds)
        _rec("sponge", bytes(data), outlen, rate, ds, out)
        return out.tobytes()

    def recover_pubkey(self, msg: bytes, sig: bytes):
        """secp256k1.RecoverPubkey -> (status, pub65)."""
        m = np.frombuffer(bytes(msg), np.uint8)
        s = np.frombuffer(bytes(sig), np.uint8)
        pub = np.zeros(65, np.uint8)
        st = self.L.oracle_recover_pubkey(_p(pub), _p(s), _p(m))
        _rec("recover_pubkey", m, s, st, pub)
        return st, pub.tobytes()

    def recover_batch(self, msg, sig):
        msg = np.ascontiguousarray(msg, np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8)
        n = msg.shape[0]
        pub = np.zeros((n, 65), np.uint8)
        addr = np.zeros((n, 20), np.uint8)
        st = np.zeros(n, np.uint8)
        self.L.oracle_recover_batch(n, _p(msg), _p(sig), _p(pub), _p(addr), _p(st))
        _rec("recover_batch", n, msg, sig, pub, addr, st)
        return pub, addr, st

    def verify(self, pub: bytes, msg: bytes, sig: bytes) -> int:
        p = np.frombuffer(bytes(pub) or b"\0", np.uint8)
        m = np.frombuffer(bytes(msg) or b"\0", np.uint8)
        s = np.frombuffer(bytes(sig) or b"\0", np.uint8)
        ok = self.L.oracle_verify_signature(_p(p), len(pub), _p(m), len(msg), _p(s), len(sig))
        _rec("verify", bytes(pub), bytes(msg), bytes(sig), ok)
        return ok

    def sender(self, signer, chain_id, sighash, r32, s32, v32, vflags):
        out = np.zeros(20, np.uint8)
        args = [np.frombuffer(bytes(x), np.uint8) for x in (sighash, r32, s32, v32)]
        st = self.L.oracle_sender(_p(out), int(signer), int(chain_id), *[_p(a) for a in args], int(vflags))
        _rec("sender", int(signer), int(chain_id).to_bytes(8, "little"), *args, int(vflags), st, out)
        return st, out.tobytes()

    def pub_to_addr(self, pub65: bytes) -> bytes:
        p = np.frombuffer(bytes(pub65), np.uint8)
        out = np.zeros(20, np.uint8)
        self.L.oracle_pub_to_addr(_p(out), _p(p))
        _rec("pub_to_addr", p, out)
        return out.tobytes()


class RefLib:
    """The reference libsecp256k1 compiled in place (oracle/_ref)."""

    def __init__(self):
        if not have_ref():
            raise FileNotFoundError(f"{REF_SO} missing")
        L = ctypes.CDLL(REF_SO)
        P, SZ, I = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.eref_ecrecover.argtypes = [P, P, P]
        L.eref_verify.argtypes = [P, P, P, SZ]
        L.eref_sign.argtypes = [P, P, P]
        L.eref_pubkey.argtypes = [P, P]
        L.eref_ecrecover_batch_mt.argtypes = [SZ, P, P, P, P, P, I]
        L.eref_sender_batch_mt.argtypes = [SZ, I, ctypes.c_ulonglong, P, P, P, P, P, P, P, I]
        L.eref_verify_batch_mt.argtypes = [SZ, P, P, P, P, P, I]
        self.L = L

    def ecrecover(self, msg: bytes, sig: bytes):
        m = np.frombuffer(bytes(msg), np.uint8)
        s = np.frombuffer(bytes(sig), np.uint8)
        pub = np.zeros(65, np.uint8)
        r = self.L.eref_ecrecover(_p(pub), _p(s), _p(m))
        _rec("eref_ecrecover", m, s, r, pub)
        return r, pub.tobytes()

    def ecrecover_batch_mt(self, msg, sig, nthreads, want_addr=True):
        """want_addr=False: the recovery alone (secp256k1_ext_ecdsa_recover per item, no Keccak),
        addr comes back None."""
        msg = np.ascontiguousarray(msg, np.uint8)
        sig = np.ascontiguousarray(sig, np.uint8)
        n = msg.shape[0]
        pub = np.zeros((n, 65), np.uint8)
        addr = np.zeros((n, 20), np.uint8) if want_addr else None
        ret = np.zeros(n, np.int8)
        self.L.eref_ecrecover_batch_mt(n, _p(msg), _p(sig), _p(pub), _p(addr) if want_addr else None, _p(ret),
                                       int(nthreads))
        _rec("eref_batch_mt", n, msg, sig, int(nthreads), pub, addr, ret)
        return pub, addr, ret

    def sender_batch_mt(self, signer, chain_id, sighash, r, s, v, vflags, nthreads):
        """types.Sender: oracle.c's Go-layer rules over the reference's recovery -> (addr, status)."""
        sighash, r, s, v = (np.ascontiguousarray(x, np.uint8) for x in (sighash, r, s, v))
        n = sighash.shape[0]
        vflags = np.zeros(n, np.uint8) if vflags is None else np.ascontiguousarray(vflags, np.uint8)
        addr = np.zeros((n, 20), np.uint8)
        st = np.zeros(n, np.uint8)
        self.L.eref_sender_batch_mt(n, int(signer), int(chain_id), _p(sighash), _p(r), _p(s), _p(v), _p(vflags), _p(addr),
                                    _p(st), int(nthreads))
        return addr, st

    def verify_batch_mt(self, pub, publen, msg, sig64, nthreads):
        """crypto.VerifySignature per item (secp256.go:126-134 over ext.h:58-75): pub [n, 65]
        (the first publen[i] bytes used), msg [n, 32], sig64 [n, 64] -> ok [n] (1 / 0; 255 = the
        reference's illegal-argument callback fired)."""
        pub, publen, msg, sig64 = (np.ascontiguousarray(x, np.uint8) for x in (pub, publen, msg, sig64))
        n = msg.shape[0]
        ok = np.zeros(n, np.uint8)
        self.L.eref_verify_batch_mt(n, _p(pub), _p(publen), _p(msg), _p(sig64), _p(ok), int(nthreads))
        return ok
