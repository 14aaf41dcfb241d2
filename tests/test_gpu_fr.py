"""GPU unit tests of the row-form (limb-parallel) field layer of the latency kernel
(eges_amd/csrc/fr.cuh) against Python big integers, through libeges_selftest.so: every
operation on weak inputs (>= p, all-ones limbs), lazy magnitudes, long squaring chains, the
quad step (four products in the four rows of a wave), plus the latency of a dependent
squaring in row form vs the lane-serial form (printed, for the record)."""
import ctypes
import os
import random

import numpy as np
import pytest

from conftest import ROOT
from test_gpu_field import P, dec, enc, samples

pytestmark = pytest.mark.gpu
FR = dict(MUL=0, SQR=1, MULSUB=2, SUB=3, LAZY=4, NORMW=5, CHAIN=6, QUAD=7, QUAD2=8, INV=9, GADD=10, SCINV=11,
          MULSUB_MAX=12)
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


@pytest.fixture(scope="module")
def st():
    import torch  # noqa: F401  (share the HIP runtime, see eges_amd/_lib.py)
    lib = ctypes.CDLL(os.path.join(ROOT, "eges_amd", "libeges_selftest.so"))
    lib.eges_fr_selftest.argtypes = [ctypes.c_int, ctypes.c_uint32] + [ctypes.c_void_p] * 4
    lib.eges_fr_latency.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.eges_fr_latency.restype = ctypes.c_double
    return lib


def run(st, op, a, b, c):
    n = len(a)
    arrs = [enc(v) for v in (a, b, c)]
    out = np.zeros((n, 8), np.uint32)
    p = lambda x: ctypes.c_void_p(x.ctypes.data)
    assert st.eges_fr_selftest(FR[op], n, *[p(x) for x in arrs], p(out)) == 0
    return dec(out)


def expect(op, a, b, c):
    if op == "MUL":
        return a * b % P
    if op == "SQR":
        return a * a % P
    if op == "MULSUB":
        return (a * b - 4 * c) % P
    if op == "MULSUB_MAX":  # magnitudes 3 x 2 with the M = 3, SH = 3 preset (fr.cuh's bounds)
        return (2 * a * b - 40 * c) % P
    if op == "SUB":
        return (a - b) % P
    if op == "LAZY":
        return (2 * a * (a + 2 * b) - 2 * b * (a - b)) % P
    if op == "NORMW":
        return 7 * a % P
    if op == "CHAIN":
        return pow(a, 2**64, P) * b % P
    if op == "QUAD":  # rows 0..3 of one pass: ab, bc, ca, a^2 (each row's result told apart)
        return (a * b + 2 * b * c + 3 * c * a) * a * a % P
    if op == "QUAD2":
        return (a * b + 2 * c * c) % P
    if op == "INV":  # row-parallel safegcd (modinv_row.cuh); 0 -> 0
        return pow(a % P, P - 2, P)


def _lift(x, odd):
    y = pow((x**3 + 7) % P, (P + 1) // 4, P)
    assert y * y % P == (x**3 + 7) % P
    return (x, y if (y & 1) == odd else P - y)


def _add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if (p[1] + q[1]) % P == 0:
            return None
        lam = 3 * p[0] * p[0] * pow(2 * p[1], P - 2, P) % P
    else:
        lam = (q[1] - p[1]) * pow(q[0] - p[0], P - 2, P) % P
    x = (lam * lam - p[0] - q[0]) % P
    return (x, (lam * (p[0] - x) - p[1]) % P)


def test_fr_general_add(st):
    """gejq_add (the split latency kernel's joins) on points with different Z: random sums,
    a == b (doubling), a == -b (infinity), against big-integer affine addition."""
    rnd = random.Random(77)
    xs = []
    while len(xs) < 300:
        x = rnd.randrange(1, P)
        if pow((x**3 + 7) % P, (P - 1) // 2, P) == 1:
            xs.append(x)
    a, b, c = [], [], []
    for i in range(300):
        xa = xs[i]
        kind = i % 3
        xb = xs[(i * 7 + 1) % 300] if kind == 0 else xa
        zc = rnd.randrange(2, P)
        if kind == 1:  # b == a: same parity as a's even y
            zc -= zc & 1
        if kind == 2:  # b == -a
            zc |= 1
        a.append(xa), b.append(xb), c.append(zc)
    got = run(st, "GADD", a, b, c)
    for i in range(300):
        s = _add(_lift(a[i], 0), _lift(b[i], c[i] & 1))
        exp = 0 if s is None else s[0]
        assert got[i] == exp, (i, i % 3)


@pytest.mark.parametrize("op", [o for o in FR if o not in ("GADD", "SCINV")])
def test_fr_ops(st, op):
    rnd = random.Random(1234 + FR[op])
    n = 1500
    a, b, c = samples(rnd, n), samples(rnd, n)[::-1], samples(rnd, n)
    rnd.shuffle(c)
    got = run(st, op, a, b, c)
    bad = [i for i in range(n) if got[i] != expect(op, a[i], b[i], c[i])]
    assert not bad, [(i, hex(a[i]), hex(b[i]), hex(got[i])) for i in bad[:5]]


def test_fr_inv_edges(st):
    """Inverses of 0, 1, p - 1, p (weak zero), small and near-2^256 values, powers of two."""
    vals = [0, 1, 2, 3, P - 1, P - 2, P, P + 1, 2**255, 2**256 - 1 - P, (P + 1) // 2] + [2**k for k in range(0, 256, 17)]
    vals = [v for v in vals if v < 2**256]
    got = run(st, "INV", vals, vals, vals)
    bad = [(hex(v), hex(g)) for v, g in zip(vals, got) if g != expect("INV", v, 0, 0)]
    assert not bad, bad[:5]


def test_sc_inv_row(st):
    """sc_inv_row_var (r^-1 / s^-1 of the latency kernels: scalar-ALU divsteps, limb-parallel
    updates) against pow(a, n - 2, n): random scalars and edges (0 -> 0, 1, n - 1, powers of two,
    values with long runs of zero bits)"""
    rnd = random.Random(99)
    vals = [0, 1, 2, 3, N - 1, N - 2, (N + 1) // 2, 2**255 % N] + [2**k for k in range(0, 256, 13)]
    vals += [(2**k - 1) % N for k in range(1, 256, 19)] + [rnd.randrange(1, N) for _ in range(1500)]
    got = run(st, "SCINV", vals, vals, vals)
    bad = [(hex(v), hex(g)) for v, g in zip(vals, got) if g != (pow(v, N - 2, N) if v else 0)]
    assert not bad, bad[:5]


def test_inv_latency_record(st):
    st.eges_inv_latency.argtypes = [ctypes.c_int, ctypes.c_int]
    st.eges_inv_latency.restype = ctypes.c_double
    p, n = st.eges_inv_latency(0, 64), st.eges_inv_latency(1, 64)
    print(f"\nrow-form inversion at one wave per CU: mod p {p:.0f} cycles, mod n {n:.0f} cycles")
    assert p > 0 and n > 0


def test_fr_latency_record(st):
    lane = st.eges_fr_latency(0, 4000)
    row = st.eges_fr_latency(1, 4000)
    print(f"\ndependent squaring at one wave per CU: lane-serial {lane:.1f} ns, row form {row:.1f} ns "
          f"({lane / row:.2f}x)")
    assert row > 0 and lane > 0
