"""Host-side transaction helpers around the sender-recovery batch (not GPU work).

Restates what core/types does before it calls into crypto:
  - RLP of the signing payload and its Keccak-256: EIP155Signer.Hash
    (core/types/transaction_signing.go:155-165) and FrontierSigner.Hash (:207-216) through
    rlpHash (core/types/block.go:134-139); integers and byte strings as rlp/encode.go.
  - V encoding of EIP155Signer.SignatureValues (:141-151): V = recid + 35 + 2 * chainId.
  - The 10-field Geec txdata wire form [nonce, price, gas, to, value, payload, IsGeecTxn, V, R, S]
    (core/types/transaction.go:59-76; bools as rlp/encode.go:408-415) -> the SoA rows that
    eges_sender_batch takes.
Keccak-256 is libeges.so's host implementation (eges_keccak256).
"""
import numpy as np

GEEC_CHAIN_ID = 930412  # genesis.json.template:3-5 (Homestead and EIP-155 active at block 0)


# ------------------------------------------------------------------ RLP (rlp/encode.go)
def rlp_bytes(b):
    b = bytes(b)
    if len(b) == 1 and b[0] < 0x80:
        return b
    return _rlp_len(len(b), 0x80) + b


def _rlp_len(n, off):
    if n < 56:
        return bytes([off + n])
    nb = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([off + 55 + len(nb)]) + nb


def rlp_uint(x):
    return rlp_bytes(x.to_bytes((x.bit_length() + 7) // 8, "big") if x else b"")


def rlp_list(items):
    body = b"".join(items)
    return _rlp_len(len(body), 0xC0) + body


def rlp_decode(b):
    """Decode one RLP item (bytes or nested lists of bytes)."""
    def item(i):
        p = b[i]
        if p < 0x80:
            return b[i:i + 1], i + 1
        if p < 0xB8:
            n = p - 0x80
            return b[i + 1:i + 1 + n], i + 1 + n
        if p < 0xC0:
            ll = p - 0xB7
            n = int.from_bytes(b[i + 1:i + 1 + ll], "big")
            return b[i + 1 + ll:i + 1 + ll + n], i + 1 + ll + n
        if p < 0xF8:
            n, j = p - 0xC0, i + 1
        else:
            ll = p - 0xF7
            n, j = int.from_bytes(b[i + 1:i + 1 + ll], "big"), i + 1 + ll
        out, end = [], j + n
        while j < end:
            x, j = item(j)
            out.append(x)
        return out, end
    v, _ = item(0)
    return v


# ------------------------------------------------------------------ sighashes
def _keccak(data):
    from .engine import keccak256
    return keccak256(data)


def frontier_sighash(nonce, price, gas, to, value, data):
    """FrontierSigner.Hash / HomesteadSigner.Hash (transaction_signing.go:207-216)."""
    return _keccak(rlp_list([rlp_uint(nonce), rlp_uint(price), rlp_uint(gas), rlp_bytes(to or b""),
                             rlp_uint(value), rlp_bytes(data)]))


def eip155_sighash(nonce, price, gas, to, value, data, chain_id):
    """EIP155Signer.Hash (transaction_signing.go:155-165)."""
    return _keccak(rlp_list([rlp_uint(nonce), rlp_uint(price), rlp_uint(gas), rlp_bytes(to or b""),
                             rlp_uint(value), rlp_bytes(data), rlp_uint(chain_id), rlp_uint(0), rlp_uint(0)]))


def eip155_v(recid, chain_id):
    """EIP155Signer.SignatureValues (transaction_signing.go:141-151)."""
    return int(recid) + 35 + 2 * int(chain_id)


def be32(x):
    """Left-padded 32-byte big-endian encoding; returns (bytes, wide flag)."""
    x = int(x)
    if x >= 1 << 256:
        return bytes(32), True
    return x.to_bytes(32, "big"), False


# ------------------------------------------------------------------ Geec blocks
def geec_block(first, n=1000, payload=100, chain_id=GEEC_CHAIN_ID):
    """A synthetic Geec block: n EIP-155 transfers shaped like the leader's block filler
    (consensus/geec/geec.go:333-339: NewTransaction(nonce, coinbase, 0, 0, 0, make([]byte,
    txnSize)), txnPerBlock 1000 and txnSize 100 from config-test.json). The nonce is the global
    index first + i, so every sighash differs. Returns sighash (n, 32) uint8."""
    coinbase = _keccak(b"eges-coinbase")[12:]
    data = bytes(payload)
    out = np.zeros((n, 32), np.uint8)
    for i in range(n):
        out[i] = np.frombuffer(eip155_sighash(first + i, 0, 0, coinbase, 0, data, chain_id), np.uint8)
    return out


def geec_block_raw(first, sig65, payload=100, chain_id=GEEC_CHAIN_ID, is_geec=True):
    """The transactions of geec_block(first, len(sig65), payload) as the wire carries them: the
    10-field Geec txdata RLP [nonce, price, gas, to, value, payload, IsGeecTxn, V, R, S]
    (core/types/transaction.go:59-76; the leader marks its filler txs with SetIsGeec,
    consensus/geec/geec_api.go:35), signed with sig65 (R || S || recid) under EIP155Signer."""
    coinbase = _keccak(b"eges-coinbase")[12:]
    data = rlp_bytes(bytes(payload))
    out = []
    for i, sg in enumerate(np.ascontiguousarray(sig65, np.uint8)):
        v = eip155_v(int(sg[64]), chain_id)
        r = int.from_bytes(sg[:32].tobytes(), "big")
        s = int.from_bytes(sg[32:64].tobytes(), "big")
        out.append(rlp_list([rlp_uint(first + i), rlp_uint(0), rlp_uint(0), rlp_bytes(coinbase), rlp_uint(0), data,
                             b"\x01" if is_geec else b"\x80", rlp_uint(v), rlp_uint(r), rlp_uint(s)]))
    return out


def encode_geec_tx(nonce, price, gas, to, value, data, is_geec, v, r, s):
    """One transaction in the 10-field Geec txdata wire form (core/types/transaction.go:59-76)."""
    return rlp_list([rlp_uint(nonce), rlp_uint(price), rlp_uint(gas), rlp_bytes(to or b""), rlp_uint(value),
                     rlp_bytes(data), b"\x01" if is_geec else b"\x80", rlp_uint(v), rlp_uint(r), rlp_uint(s)])


# ------------------------------------------------------------------ C1: 10k EIP-155 transfers
C1_PRICE, C1_GAS, C1_VALUE = 1, 21000, 1


def c1_key(i):
    """SURVEY.md §8(d) C1 key of transfer i: Keccak256("eges-key" || u64le(i)) mod n, skipping 0
    (the same derivation as the GPU synthetic signer, k_synth.hip)."""
    from .workloads import N
    k = int.from_bytes(_keccak(b"eges-key" + int(i).to_bytes(8, "little")), "big") % N
    return k or 1


def c1_to(i):
    """Recipient of transfer i: Keccak256("eges-to" || u64le(i))[12:]."""
    return _keccak(b"eges-to" + int(i).to_bytes(8, "little"))[12:]


def c1_sighashes(first, n, chain_id=GEEC_CHAIN_ID):
    """EIP155Signer(chain_id).Hash of C1 transfers first..first+n-1: nonce i, gasPrice 1,
    gas 21000, value 1, empty data (BASELINE.json configs[0]). Returns (n, 32) uint8."""
    out = np.zeros((n, 32), np.uint8)
    for j in range(n):
        i = first + j
        out[j] = np.frombuffer(eip155_sighash(i, C1_PRICE, C1_GAS, c1_to(i), C1_VALUE, b"", chain_id), np.uint8)
    return out


def c1_raw(first, sig65, chain_id=GEEC_CHAIN_ID):
    """C1 transfers signed with sig65 (R || S || recid) under EIP155Signer, as wire bytes
    (10-field txdata, IsGeecTxn false: ordinary user transfers)."""
    out = []
    for j, sg in enumerate(np.ascontiguousarray(sig65, np.uint8)):
        i = first + j
        out.append(encode_geec_tx(i, C1_PRICE, C1_GAS, c1_to(i), C1_VALUE, b"", False, eip155_v(int(sg[64]), chain_id),
                                  int.from_bytes(sg[:32].tobytes(), "big"), int.from_bytes(sg[32:64].tobytes(), "big")))
    return out


def sender_rows(sig65, chain_id=GEEC_CHAIN_ID):
    """R || S || recid signatures (n, 65) -> the r, s, v rows (n, 32) of eges_sender_batch for
    EIP-155-signed transactions (V = recid + 35 + 2 chainId)."""
    sig65 = np.ascontiguousarray(sig65, np.uint8)
    n = sig65.shape[0]
    r = sig65[:, :32].copy()
    s = sig65[:, 32:64].copy()
    v = np.zeros((n, 32), np.uint8)
    vv = sig65[:, 64].astype(np.uint64) + np.uint64(35 + 2 * chain_id)
    for k in range(8):
        v[:, 31 - k] = ((vv >> np.uint64(8 * k)) & np.uint64(0xFF)).astype(np.uint8)
    return r, s, v


def decode_geec_tx(raw):
    """10-field Geec txdata RLP -> dict(nonce, price, gas, to, value, data, is_geec, v, r, s)
    (core/types/transaction.go:59-76). Standard 9-field transactions are accepted too."""
    f = rlp_decode(raw)
    if len(f) not in (9, 10):
        raise ValueError(f"tx RLP has {len(f)} fields")
    ui = lambda b: int.from_bytes(b, "big")
    geec = len(f) == 10
    d = dict(nonce=ui(f[0]), price=ui(f[1]), gas=ui(f[2]), to=bytes(f[3]) or None, value=ui(f[4]), data=bytes(f[5]),
             is_geec=bool(geec and f[6] == b"\x01"))
    d["v"], d["r"], d["s"] = (ui(x) for x in f[-3:])
    return d


def sender_inputs(txs, chain_id):
    """Decoded transactions -> (sighash, r, s, v, vflags) SoA rows for an EIP155Signer(chain_id)
    batch: protected txs carry the EIP-155 hash, unprotected ones (V 27/28) the Frontier hash
    HomesteadSigner.Sender would use (transaction_signing.go:127-130)."""
    n = len(txs)
    rows = [np.zeros((n, 32), np.uint8) for _ in range(4)]
    vflags = np.zeros(n, np.uint8)
    for i, t in enumerate(txs):
        protected = not (t["v"].bit_length() <= 8 and t["v"] in (27, 28))
        h = (eip155_sighash if protected else lambda *a: frontier_sighash(*a[:6]))(
            t["nonce"], t["price"], t["gas"], t["to"], t["value"], t["data"], chain_id)
        rows[0][i] = np.frombuffer(h, np.uint8)
        for k, (key, flag) in enumerate((("r", 2), ("s", 4), ("v", 1))):
            b, wide = be32(t[key])
            rows[1 + k][i] = np.frombuffer(b, np.uint8)
            vflags[i] |= flag if wide else 0
    return rows[0], rows[1], rows[2], rows[3], vflags


# ------------------------------------------------------------------ Geec blocks (extblock)
def geec_header(number=1, coinbase=b"\x11" * 20):
    """A Geec header's RLP (core/types/block.go:70-90: the 15 go-ethereum fields plus Regs and
    TrustRand). Its contents are not on the signature path; any well-formed list serves."""
    return rlp_list([rlp_bytes(b"\x00" * 32), rlp_bytes(b"\x1d" * 32), rlp_bytes(coinbase), rlp_bytes(b"\x00" * 32),
                     rlp_bytes(b"\x00" * 32), rlp_bytes(b"\x00" * 32), rlp_bytes(b"\x00" * 256), rlp_uint(1),
                     rlp_uint(number), rlp_uint(8_000_000), rlp_uint(0), rlp_uint(1_560_000_000), rlp_bytes(b""),
                     rlp_bytes(b"\x00" * 32), rlp_bytes(b"\x00" * 8), rlp_list([]), rlp_uint(7)])


def fake_tx(coinbase=b"\x11" * 20, data_len=100, is_geec=False, data=None):
    """types.NewTransaction(0, coinbase, 0, 0, 0, data) with V = R = S = 0: the placeholders the
    Geec leader pads blocks with (consensus/geec/geec.go:333-339) and, with IsGeecTxn set, the
    unsigned UDP payload transactions (consensus/geec/geec_api.go:33-35)."""
    return encode_geec_tx(0, 0, 0, coinbase, 0, bytes(data_len) if data is None else data, is_geec, 0, 0, 0)


def geec_extblock(fake, geec, txs, header=None, uncles=(), confirm=None):
    """extblock RLP (core/types/block.go:188-195): [Header, FakeTxs, GeecTxs, Txs, Uncles,
    Confirm]; confirm None encodes the nil pointer (0xC0, rlp/encode.go nil struct pointer)."""
    return rlp_list([header or geec_header(), rlp_list(list(fake)), rlp_list(list(geec)), rlp_list(list(txs)),
                     rlp_list(list(uncles)), confirm if confirm is not None else rlp_list([])])
