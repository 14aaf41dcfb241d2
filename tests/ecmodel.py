"""Scalar-level model of the engine's multi-scalar schedules (test infrastructure, CPU only).

Restates, over exact integers mod n, how each kernel form splits Q = u_r R + u_g G into additions
(eges_amd/csrc/sc.cuh glv_split, core.cuh recode / strauss, k_recover_lat.hip recode_row /
recode_split / strauss_win / strauss_gcomb / high_wave / ecmult_deferred), so a test can say
in advance which addition of which form meets P == +-Q:

  lane-serial  one accumulator: 26 signed 5-bit windows of both GLV halves of u_r, with u_g's
               two 128-bit halves in 20-bit windows added every 4th window (core.cuh strauss)
  narrow       u_r R over the 26 windows (wave 0) and u_g G by the 16-bit comb (wave 1), joined
  split        windows [0, 15) of both halves (wave 0), the rest in 4-bit windows per half
               against D = 2^75 R (waves 2, 3, joined), u_g G by the comb; joins (A + G) + H
  tri          the three-wave form: windows [0, 20) on wave 0, the rest of both halves jointly
               on wave 2 against D = 2^100 R; joins (A + H) + G
  windowed     the mid-size kernel's windowed form: the split form's schedule
  bucket       the mid-size kernel: each GLV half in signed 3-bit windows, window k's digit d
               adds sign(d) 2^(3k) R into bucket |d| (bottom-up), Q_h = (B1 + B3) +
               2 ((B2 + B3) + 2 B4), then (Q_1 + Q_2) + u_g G (k_recover_mid.hip recover_bkt_body)

Points are tracked by their discrete log to base G (R = rho G with rho known to the test), so
"acc == +-P" is a congruence mod n. The reference resolves these sums with explicit branches
(libsecp256k1 group_impl.h:414-461); the engine adds without the check and either redoes a
poisoned accumulator exactly or joins partial sums with an exact addition. This model also
backs the reachability argument of DESIGN.md §3.1: the R-table loops never meet an exceptional
sum for a Babai-reduced GLV split, the comb never does for a canonical u_g, and the constructions
below reach every exceptional branch that is reachable at all.
"""
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
LAM = 0x5363AD4CC05C30E0A5261C028812645A122E22EA20816678DF02967C1B23BD72
BETA = 0x7AE96A2B657C07106E64479EAC3434E99CF0497512F58995C1396C28719501EE
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
G = (GX, GY)

# sc.cuh GLV constants (GLV_G1 / GLV_G2 / GLV_A1 / GLV_B1 / GLV_A2; b2 == a1)
GLV_G1 = 0x3086D221A7D46BCDE86C90E49284EB153DAA8A1471E8CA7FE893209A45DBB031
GLV_G2 = 0xE4437ED6010E88286F547FA90ABFE4C4221208AC9DF506C61571B4AE8AC47F71
GLV_A1 = 0x3086D221A7D46BCDE86C90E49284EB15
GLV_B1 = 0xE4437ED6010E88286F547FA90ABFE4C3  # |b1|
GLV_A2 = 0x114CA50F7A8E2F3F657C1108D9D44CFD8

RBITS, RWIN = 5, 26          # core.cuh
GBITS, GWIN, GSTEP = 20, 7, 4
CBITS, CWIN = 16, 16         # comb
SPLIT_W0, HBITS = 15, 4      # k_recover_lat.hip
TRI_W0 = 20
BK_BITS, BK_WIN, BK_NB = 3, 43, 4  # k_recover_mid.hip bucket form
HWIN = (130 - RBITS * SPLIT_W0 + HBITS) // HBITS


# ------------------------------------------------------------------ affine curve arithmetic
def ec_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = 3 * a[0] * a[0] * pow(2 * a[1], -1, P) % P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, P) % P
    x = (lam * lam - a[0] - b[0]) % P
    return x, (lam * (a[0] - x) - a[1]) % P


def ec_mul(k, pt=G):
    k %= N
    r = None
    while k:
        if k & 1:
            r = ec_add(r, pt)
        pt = ec_add(pt, pt)
        k >>= 1
    return r


# ------------------------------------------------------------------ the engine's decompositions
def glv_split(k):
    """sc.cuh glv_split, exactly: c_i = round(k g_i / 2^384), k1 = k - c1 a1 - c2 a2,
    k2 = c1 |b1| - c2 a1 (signed integers, |k_i| < 2^129)."""
    c1 = (k * GLV_G1 + (1 << 383)) >> 384
    c2 = (k * GLV_G2 + (1 << 383)) >> 384
    c1 &= (1 << 128) - 1
    c2 &= (1 << 128) - 1
    k1 = k - c1 * GLV_A1 - c2 * GLV_A2
    k2 = c1 * GLV_B1 - c2 * GLV_A1
    return k1, k2


def recode(k, W, NW, carry=0, out=None):
    """core.cuh recode / recode_row: signed W-bit digits of |k| (in [-(2^(W-1) - 1), 2^(W-1)]),
    negated for k < 0. Returns (digits, carry, remaining magnitude)."""
    m = abs(k) if out is None else k
    neg = k < 0 if out is None else out
    d = []
    for _ in range(NW):
        v = (m & ((1 << W) - 1)) + carry
        carry = 1 if v > (1 << (W - 1)) else 0
        v -= carry << W
        d.append(-v if neg else v)
        m >>= W
    return d, carry, m


def digits_narrow(u):
    k1, k2 = glv_split(u)
    return recode(k1, RBITS, RWIN)[0], recode(k2, RBITS, RWIN)[0]


def digits_split(u, w0=SPLIT_W0):
    """recode_split: w0 5-bit windows, then (carry included) the high part's 4-bit windows."""
    nh = (130 - RBITS * w0 + HBITS) // HBITS
    out = []
    for k in glv_split(u):
        lo, carry, m = recode(k, RBITS, w0)
        hi, _, _ = recode(m, HBITS, nh, carry=carry, out=k < 0)
        out.append((lo, hi))
    return out


def digits_g(u):
    """ecmult_core: u_g = lo + 2^128 hi, each in GWIN signed 20-bit windows."""
    lo, hi = u & ((1 << 128) - 1), u >> 128
    return recode(lo, GBITS, GWIN)[0], recode(hi, GBITS, GWIN)[0]


# ------------------------------------------------------------------ schedules
class Acc:
    """A running sum tracked by its discrete log; records every addition that meets +-P."""

    def __init__(self, events, tag):
        self.v, self.inf, self.events, self.tag = 0, True, events, tag

    def dbl(self, times):
        if not self.inf:
            self.v = self.v * pow(2, times, N) % N

    def add(self, p, where):
        p %= N
        if self.inf:
            self.v, self.inf = p, False
            return
        if self.v == p:
            self.events.append((self.tag, "dbl", where))
        elif (self.v + p) % N == 0:
            self.events.append((self.tag, "inf", where))
        self.v = (self.v + p) % N
        if self.v == 0:
            self.inf = True


def join(a, b, events, tag):
    """ecmult_deferred / high_wave's exact join; returns the sum (an Acc)."""
    r = Acc(events, tag)
    if a.inf:
        r.v, r.inf = b.v, b.inf
        return r
    if b.inf:
        r.v, r.inf = a.v, a.inf
        return r
    if a.v == b.v:
        events.append((tag, "dbl", None))
    elif (a.v + b.v) % N == 0:
        events.append((tag, "inf", None))
    r.v, r.inf = (a.v + b.v) % N, (a.v + b.v) % N == 0
    return r


def lane_serial(u_r, u_g, rho):
    """core.cuh strauss over R = rho G: events of the one accumulator. Returns (Q log or None, events)."""
    ev = []
    d0, d1 = digits_narrow(u_r)
    g0, g1 = digits_g(u_g)
    a = Acc(ev, "ls")
    for w in range(RWIN - 1, -1, -1):
        if w != RWIN - 1:
            a.dbl(RBITS)
        adds = [(d0[w], rho), (d1[w], rho * LAM)]
        if w % GSTEP == 0:
            adds += [(g0[w // GSTEP], 1), (g1[w // GSTEP], 1 << 128)]
        for j, (d, base) in enumerate(adds):
            if d:
                a.add(d * base, (w, j))
    return (None if a.inf else a.v), ev


def comb(u_g, ev):
    a = Acc(ev, "comb")
    for k in range(CWIN):
        d = (u_g >> (CBITS * k)) & ((1 << CBITS) - 1)
        if d:
            a.add(d << (CBITS * k), k)
    return a


def narrow(u_r, u_g, rho):
    """k_recover_lat.hip narrow form: wave 0's R' loop, wave 1's comb, one join."""
    ev = []
    d0, d1 = digits_narrow(u_r)
    a = Acc(ev, "lat_r")
    for w in range(RWIN - 1, -1, -1):
        if w != RWIN - 1:
            a.dbl(RBITS)
        for j, (d, base) in enumerate(((d0[w], rho), (d1[w], rho * LAM))):
            if d:
                a.add(d * base, (w, j))
    q = join(a, comb(u_g, ev), ev, "join")
    return (None if q.inf else q.v), ev


def split_parts(u_r, w0=SPLIT_W0):
    """The split form's low and high scalars (low + high == u_r mod n)."""
    nh = (130 - RBITS * w0 + HBITS) // HBITS
    (lo0, hi0), (lo1, hi1) = digits_split(u_r, w0)
    low = sum((lo0[w] + lo1[w] * LAM) * 32**w for w in range(w0)) % N
    high = sum((hi0[w] + hi1[w] * LAM) * 16**w for w in range(nh)) * 2**(RBITS * w0) % N
    return low, high


def _split_sums(u_r, rho, ev, w0, joint_high):
    """wave 0's low windows (tag lat_lo) and the high sum: one wave per half joined (lat_hi0 /
    lat_hi1, join_hi) or both halves on one wave (lat_hi)"""
    nh = (130 - RBITS * w0 + HBITS) // HBITS
    (lo0, hi0), (lo1, hi1) = digits_split(u_r, w0)
    a = Acc(ev, "lat_lo")
    for w in range(w0 - 1, -1, -1):
        if w != w0 - 1:
            a.dbl(RBITS)
        for j, (d, base) in enumerate(((lo0[w], rho), (lo1[w], rho * LAM))):
            if d:
                a.add(d * base, (w, j))
    D = rho * 2**(RBITS * w0)
    if joint_high:
        H = Acc(ev, "lat_hi")
        for w in range(nh - 1, -1, -1):
            if w != nh - 1:
                H.dbl(HBITS)
            for j, (hd, base) in enumerate(((hi0, D), (hi1, D * LAM))):
                if hd[w]:
                    H.add(hd[w] * base, (w, j))
        return a, H
    hs = []
    for j, (hd, base) in enumerate(((hi0, D), (hi1, D * LAM))):
        h = Acc(ev, f"lat_hi{j}")
        for w in range(nh - 1, -1, -1):
            if w != nh - 1:
                h.dbl(HBITS)
            if hd[w]:
                h.add(hd[w] * base, (w, j))
        hs.append(h)
    return a, join(hs[0], hs[1], ev, "join_hi")


def split(u_r, u_g, rho):
    """k_recover_lat.hip split form: wave 0 low windows, waves 2 / 3 high windows per half
    (joined on wave 2), wave 1 the comb; Q = (low + u_g G) + high. (Joining the R sums first, on
    E', puts a second join after the high waves' finish: measured slower, not kept.)"""
    ev = []
    a, H = _split_sums(u_r, rho, ev, SPLIT_W0, False)
    q = join(join(a, comb(u_g, ev), ev, "join"), H, ev, "join")
    return (None if q.inf else q.v), ev


def tri(u_r, u_g, rho):
    """k_recover_lat.hip three-wave form: wave 0 windows [0, TRI_W0), wave 2 the rest of both
    halves jointly; Q = (low + high) + u_g G."""
    ev = []
    a, H = _split_sums(u_r, rho, ev, TRI_W0, True)
    q = join(join(a, H, ev, "join_lohi"), comb(u_g, ev), ev, "join")
    return (None if q.inf else q.v), ev


def windowed(u_r, u_g, rho):
    """k_recover_mid.hip windowed form: the split form's schedule (joins (A + u_g G) + H)."""
    return split(u_r, u_g, rho)


def bucket(u_r, u_g, rho):
    """k_recover_mid.hip bucket form: buckets per half (tags bk0 / bk1, the unchecked additions),
    running sums (bsum) and the joins (join12: Q_1 + Q_2, join: + u_g G), all exact."""
    ev = []
    qs = []
    for h, k in enumerate(glv_split(u_r)):
        d = recode(k, BK_BITS, BK_WIN)[0]
        base = rho * (LAM if h else 1)
        B = [Acc(ev, f"bk{h}") for _ in range(BK_NB)]
        for j in range(BK_WIN):
            if d[j]:
                B[abs(d[j]) - 1].add((1 if d[j] > 0 else -1) * base * 2**(BK_BITS * j), j)
        # (B1 + B3) + 2 ((B2 + B3) + 2 B4)
        a = join(B[0], B[2], ev, "bsum")
        b = join(B[1], B[2], ev, "bsum")
        B[3].dbl(1)
        b = join(b, B[3], ev, "bsum")
        b.dbl(1)
        qs.append(join(a, b, ev, "bsum"))
    q = join(join(qs[0], qs[1], ev, "join12"), comb(u_g, ev), ev, "join")
    return (None if q.inf else q.v), ev


# ------------------------------------------------------------------ adversarial constructions
def point_for(rho):
    """R = rho G with x < n (so r = x and recid = parity of y; recid & 2 never arises here)."""
    while True:
        R = ec_mul(rho)
        if R[0] < N:
            return rho, R
        rho += 1


def recover_input(rho, R, u1, u2):
    """(msg32, sig65) whose recovery computes Q = u2 R + u1 G: u1 = -z / r, u2 = s / r."""
    r = R[0]
    z = (-u1 * r) % N
    s = (u2 * r) % N
    return z.to_bytes(32, "big"), r.to_bytes(32, "big") + s.to_bytes(32, "big") + bytes([R[1] & 1])


def recover_cases(rng, count=8):
    """Recovery inputs that make each form meet an exceptional sum, with the form and branch each
    targets: ("ls", "dbl"/"inf") the lane-serial loop at window 0 (u_g < 2^19, u_r R == +-u_g G),
    ("join", ...) the narrow and three-wave forms' final join (u_r R == +-u_g G), ("split1", ...)
    the split (and windowed) form's first join (low(u_r) R == +-u_g G), ("split2", ...) its second
    ((low R + u_g G) == +-high R)."""
    out = []
    for i in range(count):
        rho, R = point_for(rng.randrange(1, N))
        sign = 1 if i % 2 == 0 else -1
        g = [1, 2, 7, 1 << 19, rng.randrange(1, 1 << 19)][i % 5]
        out.append(("ls", sign, rho, R, g, sign * g * pow(rho, -1, N) % N))
        u1 = rng.randrange(1, N)
        out.append(("join", sign, rho, R, u1, sign * u1 * pow(rho, -1, N) % N))
        u2 = rng.randrange(1, N)
        low, high = split_parts(u2)
        out.append(("split1", sign, rho, R, sign * low * rho % N, u2))
        out.append(("split2", sign, rho, R, (sign * high * rho - low * rho) % N, u2))
    return out


def verify_cases(rng, count=8):
    """VerifySignature inputs (pub65, msg32, sig64, target): Q = u1 G + u2 P with P = rho G,
    u1 = z / s, u2 = r / s, s low. "ls" cases with sign +1 are valid signatures (r = x(2 g G))."""
    out = []
    half = N // 2
    i = 0
    while len(out) < 4 * count:
        rho, Pt = point_for(rng.randrange(1, N))
        pub = b"\x04" + Pt[0].to_bytes(32, "big") + Pt[1].to_bytes(32, "big")
        sign = 1 if i % 2 == 0 else -1
        i += 1
        # window 0 of the lane-serial loop: u1 = g, u2 rho = +-g
        g = rng.randrange(1, 1 << 19)
        r = ec_mul(2 * g)[0] % N if sign == 1 else rng.randrange(1, N)
        s = sign * r * rho * pow(g, -1, N) % N
        if s > half or s == 0:
            continue
        z = g * s % N
        cand = [("ls", sign, r, s, z)]
        r, s = rng.randrange(1, N), rng.randrange(1, half)
        u2 = r * pow(s, -1, N) % N
        cand.append(("join", sign, r, s, sign * u2 * rho * s % N))  # u1 = +-u2 rho
        low, high = split_parts(u2)
        cand.append(("split1", sign, r, s, sign * low * rho * s % N))
        cand.append(("split2", sign, r, s, (sign * high * rho - low * rho) * s % N))
        for kind, sg, r_, s_, z_ in cand:
            out.append((kind, sg, rho, pub, z_.to_bytes(32, "big"), r_.to_bytes(32, "big") + s_.to_bytes(32, "big")))
    return out
