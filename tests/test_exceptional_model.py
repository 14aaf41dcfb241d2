"""Which exceptional sums (acc == +-P) each kernel form can meet (CPU; tests/ecmodel.py).

The reference resolves a == b / a == -b inline (libsecp256k1 group_impl.h:414-461, doubling at
:440). The engine's R-table loops and comb add without that check and redo a poisoned
accumulator; its partial sums are joined exactly. This file pins, on the
engine's exact digit schedules:
  - the R-table loops (lane-serial and latency, all windows) never meet an exceptional sum for
    the Babai-reduced GLV split the kernels compute, including the inputs VERDICT r2 proposed to
    force them (a + b lambda == +-j 2^-5w from a GLV decomposition): re-splitting such a scalar
    gives the reduced halves again, whose partial sums are too short to wrap mod n;
  - the comb (u_g canonical, < n) never does;
  - the split form's high loops never do (multiples of D below 2^60);
  - what IS reachable, and tests/test_gpu_exceptional.py forces on the GPU: R-part against G-part
    in the lane-serial loop (window 0) and the latency forms' joins.
"""
import random

import ecmodel as M


def test_glv_split_is_the_reduced_decomposition():
    rnd = random.Random(1)
    # the lattice the split reduces against: (a1, -|b1|) and (a2, a1) are both in
    # L = {(x, y): x + y lambda == 0 mod n}
    assert (M.GLV_A1 - M.GLV_B1 * M.LAM) % M.N == 0 and (M.GLV_A2 + M.GLV_A1 * M.LAM) % M.N == 0
    for k in [0, 1, M.N - 1, M.LAM, M.N - M.LAM, 2**128, 2**255] + [rnd.randrange(M.N) for _ in range(2000)]:
        k1, k2 = M.glv_split(k)
        assert (k1 + k2 * M.LAM - k) % M.N == 0
        assert abs(k1) < 2**129 and abs(k2) < 2**129
        # the bound the bucket form's 43 windows rely on (k_recover_mid.hip BK_WIN)
        assert abs(k1) < 0.64 * 2**128 and abs(k2) < 0.55 * 2**128
        # Babai coordinates of (k1, k2) in the basis v1 = (a1, -|b1|), v2 = (a2, a1) are within
        # 1/2 + 2^-120 of zero: (k1, k2) is the reduced representative of its coset
        det = M.GLV_A1 * M.GLV_A1 + M.GLV_A2 * M.GLV_B1  # == n
        assert det == M.N
        t1 = (k1 * M.GLV_A1 - k2 * M.GLV_A2) / det
        t2 = (k1 * M.GLV_B1 + k2 * M.GLV_A1) / det
        assert abs(t1) <= 0.5 + 2**-60 and abs(t2) <= 0.5 + 2**-60


def test_random_scalars_meet_no_exceptional_sum():
    rnd = random.Random(2)
    for _ in range(400):
        rho = rnd.randrange(1, M.N)
        u_r, u_g = rnd.randrange(1, M.N), rnd.randrange(1, M.N)
        want = (u_r * rho + u_g) % M.N
        for form in (M.lane_serial, M.narrow, M.split, M.tri, M.windowed, M.bucket):
            q, ev = form(u_r, u_g, rho)
            assert q == want and ev == [], (form.__name__, ev)


def test_verdict_construction_does_not_poison_the_r_loops():
    """VERDICT r2's recipe: partial sum before the R addition at window w congruent to +-j
    (a + b lambda == +-j / 32, (a, b) from a GLV decomposition), digit j at window w. The engine
    re-splits u_r itself: for every w, j and sign the R-table loops of every form stay clear."""
    rnd = random.Random(3)
    inv32 = pow(32, -1, M.N)
    hits = 0
    for w in range(M.RWIN):
        for j in (1, 2, 5, 16):
            for sign in (1, -1):
                a, b = M.glv_split(sign * j * inv32 % M.N)
                low = rnd.randrange(32**w) if w else 0
                e = rnd.randrange(-15, 17)
                u_r = ((a + b * M.LAM) * 32**(w + 1) + (j + e * M.LAM) * 32**w + low) % M.N
                rho = rnd.randrange(1, M.N)
                for form in (M.narrow, M.split, M.tri, M.windowed, M.bucket):
                    _, ev = form(u_r, rnd.randrange(1, M.N), rho)
                    assert not [x for x in ev if x[0] in ("lat_r", "lat_lo", "lat_hi", "lat_hi0", "lat_hi1", "bk0", "bk1")], (w, j, ev)
                _, ev = M.lane_serial(u_r, rnd.randrange(1, M.N), rho)
                assert ev == [], (w, j, ev)
                hits += 1
    assert hits == M.RWIN * 8


def test_comb_never_meets_an_exceptional_sum():
    """acc before digit k is (u mod 2^16k) G and the entry d 2^16k G with d != 0: as integers the
    entry is larger, and u < n keeps their sum or difference away from n."""
    ev = []
    rnd = random.Random(4)
    edge = [M.N - 1, M.N - 2, (M.N >> 240) << 240, ((M.N >> 240) << 240) - 1, 2**240 - 1, 2**240, 0xFFFF << 240]
    for u in [x for x in edge if 0 < x < M.N] + [rnd.randrange(1, M.N) for _ in range(2000)]:
        M.comb(u, ev)
    assert ev == []


def test_constructions_reach_every_reachable_branch():
    """tests/test_gpu_exceptional.py's inputs: each meets the exceptional sum it targets in its
    form, the results stay u_r rho + u_g, and the other forms compute the same point."""
    rnd = random.Random(5)
    seen = set()
    for kind, sign, rho, R, u1, u2 in M.recover_cases(rnd, 10):
        want = (u2 * rho + u1) % M.N
        res = {f.__name__: f(u2, u1, rho) for f in (M.lane_serial, M.narrow, M.split, M.tri, M.windowed)}
        for name, (q, ev) in res.items():
            assert (q if q is not None else 0) == want, (kind, name)
        br = "dbl" if sign == 1 else "inf"
        if kind == "ls":
            assert ("ls", br) in {(t, b) for t, b, _ in res["lane_serial"][1]}, res["lane_serial"][1]
            assert ("join", br) in {(t, b) for t, b, _ in res["narrow"][1]}
        elif kind == "join":
            for f in ("narrow", "tri"):
                assert ("join", br) in {(t, b) for t, b, _ in res[f][1]}, (f, res[f][1])
        else:
            for f in ("split", "windowed"):
                assert ("join", br) in {(t, b) for t, b, _ in res[f][1]}, (kind, f, res[f][1])
        seen |= {(kind, br)}
        # the R-table loops stay clear in every construction
        for name, (q, ev) in res.items():
            assert not [x for x in ev if x[0] in ("lat_r", "lat_lo", "lat_hi", "lat_hi0", "lat_hi1", "comb")]
    assert len(seen) == 8
    # recover inputs encode u1 = -z / r, u2 = s / r
    for kind, sign, rho, R, u1, u2 in M.recover_cases(rnd, 2):
        msg, sig = M.recover_input(rho, R, u1, u2)
        r, s, z = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:64], "big"), int.from_bytes(msg, "big")
        rinv = pow(r, -1, M.N)
        assert (-z * rinv) % M.N == u1 and s * rinv % M.N == u2 and sig[64] == R[1] & 1


def test_verify_constructions():
    rnd = random.Random(6)
    valid = 0
    for kind, sign, rho, pub, msg, sig in M.verify_cases(rnd, 4):
        r, s, z = int.from_bytes(sig[:32], "big"), int.from_bytes(sig[32:], "big"), int.from_bytes(msg, "big")
        assert 0 < s <= M.N // 2
        u1, u2 = z * pow(s, -1, M.N) % M.N, r * pow(s, -1, M.N) % M.N
        br = "dbl" if sign == 1 else "inf"
        form = {"ls": M.lane_serial, "join": M.narrow, "split1": M.split, "split2": M.split}[kind]
        q, ev = form(u2, u1, rho)
        tag = "ls" if kind == "ls" else "join"
        assert (tag, br) in {(t, b) for t, b, _ in ev}, (kind, ev)
        if kind == "ls" and sign == 1:
            Q = M.ec_mul(q)
            assert Q[0] % M.N == r  # a valid signature through the doubling branch
            valid += 1
    assert valid >= 1


def small_u2_cases():
    """u2 values whose digits leave buckets (or whole halves) empty: the bucket form's sums then
    join infinities; tests/test_gpu_mid.py runs them."""
    return [1, 2, 3, 4, 5, 6, 8, 16, 24, 2**3 * 3, 2**30 * 4, 2**129 - 1, M.LAM, 2 * M.LAM % M.N, M.N - 1, M.N - 2,
            M.N - 4, 3 * 2**60 + 2]


def test_bucket_form_schedule():
    """The mid-size kernel's bucket form (k_recover_mid.hip): neither its unchecked bucket
    additions nor its bucket sums ever meet +-P (edge, small and structured scalars included); the
    final join with u1 G does for the "join" constructions tests/test_gpu_mid.py uses, and the
    joined result is always u_r rho + u_g."""
    rnd = random.Random(7)
    for u2 in small_u2_cases() + [rnd.randrange(1, 2**k) for k in (3, 6, 9, 40, 130) for _ in range(20)]:
        for u1 in (1, rnd.randrange(1, M.N)):
            rho = rnd.randrange(1, M.N)
            q, ev = M.bucket(u2, u1, rho)
            assert (q if q is not None else 0) == (u2 * rho + u1) % M.N
            assert not [x for x in ev if x[0] in ("bk0", "bk1", "bsum", "join12")], (u2, ev)
    # the cases of tests/test_gpu_mid.py::test_bucket_exceptional_joins
    seen = set()
    for kind, sign, rho, R, u1, u2 in M.recover_cases(rnd, 6):
        q, ev = M.bucket(u2, u1, rho)
        assert (q if q is not None else 0) == (u2 * rho + u1) % M.N
        assert not [x for x in ev if x[0] in ("bk0", "bk1", "bsum", "join12")]
        if kind == "join":
            assert ("join", "dbl" if sign == 1 else "inf") in {(t, b) for t, b, _ in ev}
            seen.add(sign)
    assert seen == {1, -1}


def test_bucket_halves_never_join_exceptionally():
    """Q_1 == +-Q_2 needs k1 == +-lambda k2 (mod n) for the split's own output: k1 == -lambda k2
    means u2 == 0; k1 == lambda k2 puts (k1, k2) on the lattice {x == lambda y}, whose short
    vectors are not reduced representatives of the split (Babai rounding maps them elsewhere)."""
    v1, v2 = (M.GLV_A1, M.GLV_B1), (M.GLV_A2, -M.GLV_A1)
    for a, b in (v1, v2):
        assert (a - M.LAM * b) % M.N == 0
    for i in range(-6, 7):
        for j in range(-6, 7):
            if i or j:
                k = (i * v1[0] + j * v2[0], i * v1[1] + j * v2[1])
                assert M.glv_split((k[0] + M.LAM * k[1]) % M.N) != k
