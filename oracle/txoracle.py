"""Wire-format transaction oracle — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Pure-Python restatement of what the reference does from raw transaction bytes to a sender:
  - rlp.DecodeBytes(raw, &tx) for the Geec txdata struct (core/types/transaction.go:59-76,
    DecodeRLP :157-165) with the reference decoder's acceptance rules (rlp/decode.go):
      DecodeBytes + trailing-bytes check ............ :119-129
      Stream.Kind bound checks ....................... :874-907
      readKind / readUint (canonical sizes) .......... :937-1008
      Stream.Bytes (single byte < 0x80 rule) ......... :668-688
      Stream.uint / Bool ............................. :707-756
      decodeBigInt (leading zero bytes) .............. :254-269
      decodeByteArray ([N]byte, [20]byte Recipient) .. :390-413
      makeOptionalPtrDecoder (rlp:"nil") ............. :464-490
      struct decoder: too few / too many elements .... :418-435
  - the signer's Hash (FrontierSigner.Hash transaction_signing.go:207-216, EIP155Signer.Hash
    :155-165) re-encoded with rlp/encode.go's rules and Keccak-256'd (rlpHash, block.go:134-139);
    EIP155Signer.Sender (:127-137) picks the Frontier hash for unprotected V (isProtectedV,
    transaction.go:142-149);
  - the sender itself through the C oracle's Sender (oracle.c, pinned by oracle/_ref);
  - the EVM ECRECOVER precompile's Run (core/vm/contracts.go:77-101), pinned by the reference's
    own sample (contracts_test.go:390-395).
  - the extblock list structure of a whole Geec block (core/types/block.go:188-195,273-282)
    around it (split_extblock / block_senders).
Pinned by: the reference's Vitalik EIP-155 vectors (transaction_signing_test.go:79-116) and the
Homestead recipient vectors (transaction_test.go:82-127), re-encoded in the 10-field Geec form;
the 9-field originals must fail to decode under the Geec struct.
"""

DECODE_FAILED = 7  # include/eges.h EGES_DECODE_FAILED


class DecodeError(Exception):
    pass


class _Stream:
    """Byte-level restatement of rlp.Stream over one input (limits as a stack of list ends)."""

    def __init__(self, b):
        self.b = bytes(b)
        self.pos = 0
        self.ends = [len(self.b)]  # top level: the input length (s.limited)

    def _byte(self):
        if self.pos >= self.ends[-1]:
            raise DecodeError("EOF / element too large")
        x = self.b[self.pos]
        self.pos += 1
        return x

    def _uint_be(self, n):
        if n == 0:
            return 0
        if n == 1:
            return self._byte()
        bs = bytes(self._byte() for _ in range(n))
        if bs[0] == 0:
            raise DecodeError("ErrCanonSize")
        return int.from_bytes(bs, "big")

    def kind(self):
        """-> (kind, size, byteval); kind in 'byte' / 'string' / 'list'. Consumes the header."""
        if self.pos == self.ends[-1]:
            raise DecodeError("EOL")
        b = self._byte()
        if b < 0x80:
            return "byte", 0, b
        if b < 0xB8:
            k, size = "string", b - 0x80
        elif b < 0xC0:
            size = self._uint_be(b - 0xB7)
            if size < 56:
                raise DecodeError("ErrCanonSize")
            k = "string"
        elif b < 0xF8:
            k, size = "list", b - 0xC0
        else:
            size = self._uint_be(b - 0xF7)
            if size < 56:
                raise DecodeError("ErrCanonSize")
            k = "list"
        if size > self.ends[-1] - self.pos:
            raise DecodeError("ErrElemTooLarge / ErrValueTooLarge")
        return k, size, None

    def content(self, size):
        c = self.b[self.pos:self.pos + size]
        self.pos += size
        return c

    # typed readers
    def bytes_(self):
        k, size, bv = self.kind()
        if k == "byte":
            return bytes([bv])
        if k == "list":
            raise DecodeError("ErrExpectedString")
        c = self.content(size)
        if size == 1 and c[0] < 128:
            raise DecodeError("ErrCanonSize")
        return c

    def uint(self, maxbits):
        k, size, bv = self.kind()
        if k == "byte":
            if bv == 0:
                raise DecodeError("ErrCanonInt")
            return bv
        if k == "list":
            raise DecodeError("ErrExpectedString")
        if size > maxbits // 8:
            raise DecodeError("uint overflow")
        c = self.content(size)
        if size >= 2 and c[0] == 0:
            raise DecodeError("ErrCanonInt")
        v = int.from_bytes(c, "big")
        if size > 0 and v < 128:
            raise DecodeError("ErrCanonSize")
        return v

    def bigint(self):
        c = self.bytes_()
        if len(c) > 0 and c[0] == 0:
            raise DecodeError("ErrCanonInt")
        return int.from_bytes(c, "big")

    def boolean(self):
        v = self.uint(8)
        if v not in (0, 1):
            raise DecodeError("invalid boolean")
        return v == 1

    def byte_array(self, n):
        """decodeByteArray into [n]byte (rlp/decode.go:390-413)."""
        k, size, bv = self.kind()
        if k == "byte":
            if n == 0:
                raise DecodeError("input string too long")
            if n > 1:
                raise DecodeError("input string too short")
            return bytes([bv])
        if k == "list":
            raise DecodeError("ErrExpectedString")
        if n < size:
            raise DecodeError("input string too long")
        if n > size:
            raise DecodeError("input string too short")
        c = self.content(size)
        if size == 1 and c[0] < 128:
            raise DecodeError("ErrCanonSize")
        return c

    def address_or_nil(self):
        """*common.Address with rlp:"nil" (makeOptionalPtrDecoder, rlp/decode.go:464-490): an
        empty string or list decodes as nil, anything else as [20]byte."""
        save = self.pos
        k, size, bv = self.kind()
        if size == 0 and k != "byte":
            return None
        self.pos = save  # decodeByteArray re-reads the same (cached) kind
        return self.byte_array(20)

    def list_start(self):
        k, size, _ = self.kind()
        if k != "list":
            raise DecodeError("ErrExpectedList")
        self.ends.append(self.pos + size)

    def list_end(self):
        if self.pos != self.ends[-1]:
            raise DecodeError("input list has too many elements")
        self.ends.pop()


def decode_struct(s, readers):
    """Struct decoder (rlp/decode.go:418-435): a list whose elements are read in field order;
    EOL before the last field is "too few elements", leftover elements "too many"."""
    s.list_start()
    try:
        vals = [r() for r in readers]
    except DecodeError as e:
        if str(e) == "EOL":
            raise DecodeError("too few elements")
        raise
    s.list_end()
    return vals


def decode_bytes(raw, reader):
    """rlp.DecodeBytes (rlp/decode.go:119-129): one value read by reader(stream), no trailing data."""
    s = _Stream(raw)
    v = reader(s)
    if s.pos != len(s.b):
        raise DecodeError("ErrMoreThanOneValue")
    return v


TXDATA_FIELDS = ("nonce", "price", "gas", "to", "value", "data", "is_geec", "v", "r", "s")


def txdata_readers(s):
    """Field readers of the Geec txdata struct, in order (core/types/transaction.go:59-76)."""
    return [lambda: s.uint(64), s.bigint, lambda: s.uint(64), s.address_or_nil, s.bigint, s.bytes_, s.boolean,
            s.bigint, s.bigint, s.bigint]


def decode_txdata(raw):
    """rlp.DecodeBytes(raw, &tx) for the Geec txdata struct -> dict, or raises DecodeError."""
    return decode_bytes(raw, lambda s: dict(zip(TXDATA_FIELDS, decode_struct(s, txdata_readers(s)))))


# ------------------------------------------------------------------ encoder (rlp/encode.go)
def _enc_len(n, off):
    if n < 56:
        return bytes([off + n])
    nb = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([off + 55 + len(nb)]) + nb


def enc_bytes(b):
    b = bytes(b)
    if len(b) == 1 and b[0] < 0x80:
        return b
    return _enc_len(len(b), 0x80) + b


def enc_uint(x):
    return enc_bytes(x.to_bytes((x.bit_length() + 7) // 8, "big") if x else b"")


def enc_list(items):
    body = b"".join(items)
    return _enc_len(len(body), 0xC0) + body


def is_protected_v(v):
    """transaction.go:142-149"""
    if v.bit_length() <= 8:
        return v not in (27, 28)
    return True


def signing_payload(d, signer, chain_id):
    """RLP that Signer.Hash Keccaks for a decoded tx under `signer` (0 Frontier, 1 Homestead,
    2 EIP155 with chain_id); EIP155Signer.Sender uses the Homestead (= Frontier) hash when V is
    unprotected (transaction_signing.go:127-130)."""
    fields = [enc_uint(d["nonce"]), enc_uint(d["price"]), enc_uint(d["gas"]),
              enc_bytes(d["to"]) if d["to"] is not None else b"\x80", enc_uint(d["value"]), enc_bytes(d["data"])]
    if signer == 2 and is_protected_v(d["v"]):
        fields += [enc_uint(chain_id), enc_uint(0), enc_uint(0)]
    return enc_list(fields)


def be32(x):
    """32-byte row + wide flag as eges_sender_batch takes them."""
    if x >= 1 << 256:
        return bytes(32), True
    return x.to_bytes(32, "big"), False


def sender_raw(oracle, raw, signer, chain_id):
    """types.Sender of one wire-format tx -> (status, addr20, sighash32)."""
    try:
        d = decode_txdata(raw)
    except DecodeError:
        return DECODE_FAILED, bytes(20), bytes(32)
    h = oracle.keccak256(signing_payload(d, signer, chain_id))
    (vb, vw), (rb, rw), (sb, sw) = be32(d["v"]), be32(d["r"]), be32(d["s"])
    flags = (1 if vw else 0) | (2 if rw else 0) | (4 if sw else 0)
    st, addr = oracle.sender(signer, chain_id, h, rb, sb, vb, flags)
    return st, (addr if st == 0 else bytes(20)), h


def split_extblock(raw):
    """Structure of rlp.DecodeBytes(raw, &block) (Block.DecodeRLP core/types/block.go:273-282 into
    extblock :188-195): [Header, FakeTxs, GeecTxs, Txs, Uncles, Confirm rlp:"nil"] -> the raw
    encodings of the three transaction lists' items, or DecodeError. Header / uncle / confirm
    field contents are not decoded (not on the signature path)."""
    s = _Stream(raw)
    s.list_start()
    lists = []
    for e in range(6):
        try:
            k, size, _ = s.kind()
        except DecodeError as err:
            raise DecodeError("too few elements" if str(err) == "EOL" else str(err))
        if e < 5 and k != "list":
            raise DecodeError("ErrExpectedList")
        if e == 5 and not (k == "list" or (k == "string" and size == 0)):
            raise DecodeError("confirm: expected list or nil")
        body = s.content(size) if k != "byte" else b""
        if 1 <= e <= 3:
            items = []
            t = _Stream(body)
            while t.pos < len(t.b):
                start = t.pos
                k2, size2, _ = t.kind()
                if k2 != "byte":
                    t.content(size2)
                items.append(t.b[start:t.pos])
            lists.append(items)
    s.list_end()
    if s.pos != len(s.b):
        raise DecodeError("ErrMoreThanOneValue")
    return lists


def block_senders(oracle, raw, lists_mask, signer, chain_id):
    """eges_block_senders_raw restated: (statuses, addrs, counts, block_status)."""
    try:
        lists = split_extblock(raw)
    except DecodeError:
        return [], [], [0, 0, 0], DECODE_FAILED
    sts, addrs = [], []
    bst = 0
    for k in range(3):
        if lists_mask & (1 << k):
            for item in lists[k]:
                st, addr, _ = sender_raw(oracle, item, signer, chain_id)
                sts.append(st)
                addrs.append(addr)
        else:
            # rlp.DecodeBytes decodes every transaction list of the block (extblock :188-195),
            # so an undecodable item of an unselected list fails the block too
            for item in lists[k]:
                try:
                    decode_txdata(item)
                except DecodeError:
                    bst = DECODE_FAILED
    if DECODE_FAILED in sts:
        bst = DECODE_FAILED
    return sts, addrs, [len(x) for x in lists], bst


def precompile_ecrecover(oracle, inp):
    """ECRECOVER precompile Run (core/vm/contracts.go:77-101) -> (status, 32-byte output or None).
    status: 0 ok, 2 rejected by the pre-checks (input[32:63] / ValidateSignatureValues with
    homestead = false), 6 crypto.Ecrecover failed."""
    inp = bytes(inp)
    if len(inp) < 128:
        inp = inp + bytes(128 - len(inp))  # common.RightPadBytes
    r = int.from_bytes(inp[64:96], "big")
    s = int.from_bytes(inp[96:128], "big")
    v = (inp[63] - 27) & 0xff
    N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    if any(inp[32:63]) or not (1 <= r < N and 1 <= s < N and v in (0, 1)):
        return 2, None
    st, pub = oracle.recover_pubkey(inp[:32], inp[64:128] + bytes([v]))
    if st != 0:
        return 6, None
    return 0, bytes(12) + oracle.keccak256(pub[1:])[12:]


def to_geec10(raw9):
    """A standard 9-field tx encoding -> the 10-field Geec form (IsGeecTxn = false inserted
    before V), keeping every other field's bytes."""
    s = _Stream(raw9)
    s.list_start()
    items = []
    while s.pos < s.ends[-1]:
        start = s.pos
        k, size, _ = s.kind()
        if k != "byte":
            s.content(size)
        items.append(s.b[start:s.pos])
    assert len(items) == 9
    return enc_list(items[:6] + [b"\x80"] + items[6:])
