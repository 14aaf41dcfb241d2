"""GPU unit tests of the field / scalar / group layer (eges_amd/csrc/fe.cuh, sc.cuh, ge.cuh)
against Python big integers, through the self-test harness libeges_selftest.so.

Edge values: 0, 1, p-1, p, p+1, 2^256-1 (weak representations >= p), values with all-ones
limbs, and lazy-magnitude chains (fe.cuh magnitude rules)."""
import ctypes
import os
import random

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
LAM = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
OPS = dict(MUL=0, SQR=1, ADD=2, SUB=3, INV=4, SQRT=5, LAZY=6, NEG=7, EQZ=8, DBL=9, MADD=10, SCMUL=11, SCINV=12, GLV=13)


@pytest.fixture(scope="module")
def st():
    import torch  # noqa: F401  (share the HIP runtime, see eges_amd/_lib.py)
    lib = ctypes.CDLL(os.path.join(ROOT, "eges_amd", "libeges_selftest.so"))
    lib.eges_selftest.argtypes = [ctypes.c_int, ctypes.c_uint32] + [ctypes.c_void_p] * 7
    return lib


def enc(xs):
    a = np.zeros((len(xs), 8), np.uint32)
    for i, x in enumerate(xs):
        for k in range(8):
            a[i, k] = (x >> (32 * k)) & 0xFFFFFFFF
    return a


def dec(a):
    return [sum(int(a[i, k]) << (32 * k) for k in range(8)) for i in range(a.shape[0])]


def run(st, op, a, b=None, c=None, d=None):
    n = len(a)
    arrs = [enc(v if v is not None else [0] * n) for v in (a, b, c, d)]
    out = np.zeros((n, 8), np.uint32)
    out2 = np.zeros((n, 8), np.uint32)
    flag = np.zeros(n, np.uint32)
    p = lambda x: ctypes.c_void_p(x.ctypes.data)
    assert st.eges_selftest(OPS[op], n, *[p(x) for x in arrs], p(out), p(out2), p(flag)) == 0
    return dec(out), dec(out2), flag


def samples(rnd, n):
    edge = [0, 1, 2, P - 1, P, P + 1, 2**256 - 1, 2**256 - 2, 2**255, 2**26 - 1, 2**52 + 5, (2**256 - 1) // 3,
            sum(((1 << 26) - 1) << (26 * k) for k in range(10)) % 2**256,
            sum(((1 << 29) - 1) << (29 * k) for k in range(9)) % 2**256]
    xs = edge + [rnd.randrange(2**256) for _ in range(n - len(edge))]
    return xs


def test_field_ops(st):
    rnd = random.Random(11)
    a = samples(rnd, 512)
    b = list(reversed(samples(rnd, 512)))
    out, _, _ = run(st, "MUL", a, b)
    assert out == [(x * y) % P for x, y in zip(a, b)]
    out, _, _ = run(st, "SQR", a)
    assert out == [(x * x) % P for x in a]
    out, _, _ = run(st, "ADD", a, b)
    assert out == [(x + y) % P for x, y in zip(a, b)]
    out, _, _ = run(st, "SUB", a, b)
    assert out == [(x - y) % P for x, y in zip(a, b)]
    out, _, _ = run(st, "NEG", a)
    assert out == [(-x) % P for x in a]
    out, _, _ = run(st, "LAZY", a, b)
    assert out == [((2 * x) * (x + 2 * y) - 2 * y * (x - y)) % P for x, y in zip(a, b)]


def test_field_inv_sqrt(st):
    rnd = random.Random(12)
    a = [x for x in samples(rnd, 256) if x % P != 0]
    out, _, _ = run(st, "INV", a)
    assert out == [pow(x, P - 2, P) for x in a]
    out, _, flag = run(st, "SQRT", a)
    for x, r, f in zip(a, out, flag):
        is_sq = pow(x % P, (P - 1) // 2, P) == 1 or x % P == 0
        assert bool(f) == is_sq
        assert r == pow(x % P, (P + 1) // 4, P)


def test_field_equal_weak(st):
    rnd = random.Random(13)
    hi = [rnd.randrange(P, 2**256) for _ in range(64)] + [P, P + 1, 2**256 - 1]
    _, _, f = run(st, "EQZ", hi, [x - P for x in hi])
    assert f.tolist() == [1] * len(hi)
    _, _, f = run(st, "EQZ", hi, [(x - P + 1) % P for x in hi])
    assert f.tolist() == [0] * len(hi)


def ec_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    if p1[0] == p2[0]:
        if (p1[1] + p2[1]) % P == 0:
            return None
        l = 3 * p1[0] * p1[0] * pow(2 * p1[1], -1, P) % P
    else:
        l = (p2[1] - p1[1]) * pow(p2[0] - p1[0], -1, P) % P
    x = (l * l - p1[0] - p2[0]) % P
    return (x, (l * (p1[0] - x) - p1[1]) % P)


def ec_mul(k, pt):
    r = None
    while k:
        if k & 1:
            r = ec_add(r, pt)
        pt = ec_add(pt, pt)
        k >>= 1
    return r


def test_group_ops(st):
    rnd = random.Random(14)
    pts = [ec_mul(rnd.randrange(1, N), (GX, GY)) for _ in range(48)]
    xs, ys = [p[0] for p in pts], [p[1] for p in pts]
    ox, oy, _ = run(st, "DBL", xs, ys)
    for p, x, y in zip(pts, ox, oy):
        assert (x, y) == ec_mul(4, p)
    qs = [ec_mul(rnd.randrange(1, N), (GX, GY)) for _ in range(48)]
    # include exceptional cases: q == 2p (doubling) and q == -2p (infinity)
    qs[0] = ec_mul(2, pts[0])
    qs[1] = (ec_mul(2, pts[1])[0], (-ec_mul(2, pts[1])[1]) % P)
    ox, oy, fl = run(st, "MADD", xs, ys, [q[0] for q in qs], [q[1] for q in qs])
    assert fl[0] == 3 and fl[1] == 1
    for i in range(2, 48):
        assert fl[i] == 0
        assert (ox[i], oy[i]) == ec_add(ec_mul(2, pts[i]), qs[i])


def test_scalar_and_glv(st):
    rnd = random.Random(15)
    a = [0, 1, N - 1, N, N + 1, 2**256 - 1] + [rnd.randrange(2**256) for _ in range(250)]
    b = [rnd.randrange(2**256) for _ in a]
    out, _, _ = run(st, "SCMUL", a, b)
    assert out == [((x % N) * (y % N)) % N for x, y in zip(a, b)]
    nz = [x for x in a if x % N]
    out, _, _ = run(st, "SCINV", nz)
    assert out == [pow(x % N, N - 2, N) for x in nz]
    out, out2, fl = run(st, "GLV", a)
    for x, m1, m2, f in zip(a, out, out2, fl):
        k1 = -m1 if f & 1 else m1
        k2 = -m2 if f & 2 else m2
        assert (k1 + k2 * LAM - x) % N == 0
        assert abs(k1) < 2**129 and abs(k2) < 2**129


def test_ecmult_core_exceptional(st):
    """ecmult_core (unchecked Strauss + exact redo) on scalars chosen to hit P == +-Q mid-loop
    and an infinite result, against big-integer double-and-add."""
    lib = st
    lib.eges_selftest_ecmult.argtypes = [ctypes.c_uint32] + [ctypes.c_void_p] * 7
    rnd = random.Random(16)
    G = (GX, GY)
    cases = [(G, 1, 1), (G, 5, N - 5), (G, 7, 7), (G, 0, 3), (G, 3, 0), (G, 0, 0), (G, N - 1, 1),
             (ec_mul(2, G), 3, N - 6), (ec_mul(2, G), 3, 6), (ec_mul(LAM, G), 1, N - LAM),
             (ec_mul(LAM, G), 2, 2 * LAM % N)]
    for _ in range(8):
        a = rnd.randrange(1, N)
        cases.append((G, a, N - a))  # infinity
        cases.append((G, a, a))      # acc == p in the first windows
        k = rnd.randrange(1, N)
        b = rnd.randrange(1, N)
        cases.append((ec_mul(k, G), b, (N - b * k % N) % N))  # u_r*kG + u_g*G == infinity
    while len(cases) < 300:
        k = rnd.randrange(1, N)
        cases.append((ec_mul(k, G), rnd.randrange(N), rnd.randrange(N)))
    n = len(cases)
    px, py, ur, ug = (enc([c[0][0] for c in cases]), enc([c[0][1] for c in cases]), enc([c[1] for c in cases]),
                      enc([c[2] for c in cases]))
    ox = np.zeros((n, 8), np.uint32)
    oy = np.zeros((n, 8), np.uint32)
    fl = np.zeros(n, np.uint32)
    p = lambda x: ctypes.c_void_p(x.ctypes.data)
    assert lib.eges_selftest_ecmult(n, p(px), p(py), p(ur), p(ug), p(ox), p(oy), p(fl)) == 0
    xs, ys = dec(ox), dec(oy)
    for i, (pt, a, b) in enumerate(cases):
        exp = ec_add(ec_mul(a, pt), ec_mul(b, G))
        if exp is None:
            assert fl[i] == 1, i
        else:
            assert fl[i] == 0 and (xs[i], ys[i]) == exp, i
