"""Lane-level model of the row-form field product (eges_amd/csrc/fr.cuh fr_cols / fr_reduce,
the default "lean" reduction of round 5), checked on the CPU against Python big integers mod p
(the bounds its comments state were derived from a model that was not in the repo).

Every DPP move is modelled as the hardware does it on one 16-lane row (row_newbcast:I = lane I
of the row, row_shr:I / row_shl:I with zero fill), every v_mad_u64_u32 as a 32x32+64-bit
multiply-add, and every 32-bit add as a wrap-around add. The model asserts, for each
instruction, that no 64-bit column and no 32-bit limb wraps, and checks the bounds fr.cuh
states (columns < 2^63.9, n < 2^30.01, T < 2^60.8, t17 < 2^32, R < 2^55.01, e < 2^26.01,
z < 2^33.01). Inputs: every magnitude pair the formulas may issue (m(a) m(b) <= 6.5, limbs at
m (2^29 + 2^16)), lazy random limbs, and every fr_mul_sub<M, SH> preset (M 1..3, SH 0..3) with
the subtrahend at 0, at its largest and random. Same field values as libsecp256k1's
(field_10x26_impl.h:440,769); the representation is the engine's own."""
import random

import pytest

P = 2**256 - 2**32 - 977
M29 = (1 << 29) - 1
FOLD0 = 31264
U32 = 1 << 32
U64 = 1 << 64
LANES = 16
BOUNDS = {"col": 2**63.9, "n": 2**30.01, "T": 2**60.8, "R": 2**55.01, "e": 2**26.01, "z": 2**33.01}
seen = {k: 0 for k in list(BOUNDS) + ["t17", "out", "out0"]}


def bcast(x, i):
    return [x[i]] * LANES


def shr(x, i):
    return [x[L - i] if L >= i else 0 for L in range(LANES)]


def shl(x, i):
    return [x[L + i] if L + i < LANES else 0 for L in range(LANES)]


def mad64(a, b, c):
    assert 0 <= a < U32 and 0 <= b < U32 and 0 <= c < U64
    r = a * b + c
    assert r < U64, "64-bit column wraps"
    return r


def add32(*xs):
    r = sum(xs)
    assert r < U32, "32-bit limb wraps"
    return r


def kconst(m):
    """fr.cuh kconst<M>: M * 64p per lane (lanes 9..15: 0)"""
    kk = (0x3FFFFFFE * m) % U32
    out = []
    for L in range(LANES):
        v = kk if L <= 8 else 0
        if L == 0:
            v += (0x3FFF0BC0 * m - kk) % U32
        if L == 1:
            v += (0x3FFFFDFE * m - kk) % U32
        out.append(v % U32)
    return out


def cfold(L):
    return FOLD0 if L == 0 else 256 if L == 1 else 0


def fr_cols(col, a, b):
    """fr_cols: columns 0..15 of a * b on top of col (lane L = column L); a8, b8 for column 16"""
    col = [mad64(bcast(a, 0)[L], b[L], col[L]) for L in range(LANES)]
    c1 = [mad64(a[1], shr(b, 1)[L], 0) for L in range(LANES)]
    c2 = [mad64(a[2], shr(b, 2)[L], 0) for L in range(LANES)]
    for i, acc in ((3, col), (4, c1), (5, c2), (6, col), (7, c1)):
        sb = shr(b, i)
        for L in range(LANES):
            acc[L] = mad64(a[i], sb[L], acc[L])
    a8, b8 = a[8], b[8]
    sb = shr(b, 8)
    c2 = [mad64(a8, sb[L], c2[L]) for L in range(LANES)]
    out = []
    for L in range(LANES):
        v = col[L] + c1[L] + c2[L]
        assert v < U64
        out.append(v)
    seen["col"] = max(seen["col"], max(out))
    return out, a8, b8


def fr_reduce(col, a8, b8):
    p0 = [c & M29 for c in col]
    p1 = [(c >> 29) & M29 for c in col]  # v_alignbit(hi, lo, 29) & M29
    p2 = [c >> 58 for c in col]  # hi >> 26
    n = [add32(p0[L], shr(p1, 1)[L], shr(p2, 2)[L]) for L in range(LANES)]
    seen["n"] = max(seen["n"], max(n))
    s16 = [add32(p1[L], shr(p2, 1)[L]) for L in range(LANES)]
    T = mad64(a8, b8, s16[15])
    seen["T"] = max(seen["T"], T)
    t16 = T & M29
    t17 = add32((T >> 29) % U32, p2[15])
    assert T >> 29 < U32
    seen["t17"] = max(seen["t17"], t17)
    X = shl(n, 9)
    X[7] = t16
    Y = shl(n, 8)
    Y[0] = 0
    Y[8] = t16
    out = []
    R = []
    for L in range(LANES):
        c17 = (FOLD0 * 256 if L == 0 else 65536 if L == 1 else 0) + (FOLD0 if L == 8 else 0)
        R.append(mad64(Y[L], 256, mad64(X[L], FOLD0, mad64(c17, t17, n[L]))))
    seen["R"] = max(seen["R"], max(R))
    e = []
    for L in range(LANES):
        assert R[L] >> 29 < U32
        e.append(R[L] >> 29)
    seen["e"] = max(seen["e"], max(e[:9]))
    r = [R[L] & M29 if L <= 8 else 0 for L in range(LANES)]
    e7 = [e[L] if L <= 7 else 0 for L in range(LANES)]
    z = [mad64(e[8], cfold(L), r[L]) for L in range(LANES)]
    seen["z"] = max(seen["z"], max(z))
    zc = [zz >> 29 for zz in z]
    carry = [add32(e7[L], zc[L]) for L in range(LANES)]
    sc = shr(carry, 1)
    out = [add32(z[L] & M29, sc[L]) for L in range(LANES)]
    assert all(v == 0 for v in out[9:]), "lanes 9..15 must stay zero"
    seen["out"] = max(seen["out"], max(out[1:9]))
    seen["out0"] = max(seen["out0"], out[0])
    return out


def value(limbs):
    return sum(v << (29 * L) for L, v in enumerate(limbs[:9]))


def fr_mul_sub(a, b, c, m, sh):
    preset = [((kk - cc) % U32) << sh for kk, cc in zip(kconst(m), c)]
    for kk, cc in zip(kconst(m), c):
        assert cc <= kk, "subtrahend above M * 64p in a lane"
    col, a8, b8 = fr_cols(preset, a, b)
    return fr_reduce(col, a8, b8)


def row(limbs9):
    return list(limbs9) + [0] * (LANES - 9)


def at_magnitude(m, rnd=None):
    top = int(m * ((1 << 29) + (1 << 16)))
    if rnd is None:
        return row([top] * 9)
    return row([rnd.randrange(top + 1) for _ in range(9)])


PAIRS = [(1, 1), (1, 6.5), (6.5, 1), (2, 3), (3, 2), (2.5, 2.5), (2, 2), (1, 6), (6, 1), (3, 2.1)]


def check(a, b, c=None, m=1, sh=0):
    if c is None:
        col, a8, b8 = fr_cols([0] * LANES, a, b)
        out = fr_reduce(col, a8, b8)
        want = value(a) * value(b) % P
    else:
        out = fr_mul_sub(a, b, c, m, sh)
        want = (value(a) * value(b) - (value(c) << sh)) % P
    assert value(out) % P == want
    return out


@pytest.mark.parametrize("ma,mb", PAIRS)
def test_worst_magnitude_products(ma, mb):
    check(at_magnitude(ma), at_magnitude(mb))


def test_random_lazy_products():
    rnd = random.Random(20261018)
    for _ in range(400):
        ma, mb = rnd.choice(PAIRS)
        check(at_magnitude(ma, rnd), at_magnitude(mb, rnd))
    for _ in range(200):  # weak (reduced) field elements
        x, y = rnd.randrange(P), rnd.randrange(P)
        a = row([(x >> (29 * L)) & M29 for L in range(9)])
        b = row([(y >> (29 * L)) & M29 for L in range(9)])
        assert value(check(a, b)) % P == x * y % P


@pytest.mark.parametrize("m", [1, 2, 3])
@pytest.mark.parametrize("sh", [0, 1, 2, 3])
def test_mul_sub_presets(m, sh):
    rnd = random.Random(m * 10 + sh)
    k = kconst(m)
    big_c = row(k[:9])  # the largest subtrahend each lane allows: preset 0
    for ma, mb in PAIRS:
        a, b = at_magnitude(ma), at_magnitude(mb)
        check(a, b, row([0] * 9), m, sh)  # largest preset (M * 64p << SH)
        check(a, b, big_c, m, sh)
        for _ in range(20):
            c = row([rnd.randrange(k[L] + 1) for L in range(9)])
            check(at_magnitude(ma, rnd), at_magnitude(mb, rnd), c, m, sh)


def test_stated_bounds_hold():
    """runs last in this file: every bound fr.cuh's comments state held over all the above"""
    test_random_lazy_products()
    for ma, mb in PAIRS:
        check(at_magnitude(ma), at_magnitude(mb))
        check(at_magnitude(ma), at_magnitude(mb), row([0] * 9), 3, 3)
    for k, bound in BOUNDS.items():
        assert seen[k] < bound, (k, seen[k].bit_length(), bound)
    assert seen["t17"] < U32
    # the output is magnitude 1 in the engine's sense (limb 0 below 2^29, the others below
    # 2^29 + 2^26 as the comment states) and feeds the next product at m = 1
    assert seen["out0"] < 1 << 29
    assert seen["out"] < (1 << 29) + (1 << 26)
    out = check(at_magnitude(6.5), at_magnitude(1))
    check(out, at_magnitude(6.5))
