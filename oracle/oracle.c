/*
 * TEST INFRASTRUCTURE ONLY — the CPU restatement ("oracle") of the reference's
 * sender-recovery path. Never linked into, called by, or shipped with the
 * product library (eges_amd/csrc, libeges.so). Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load it.
 *
 * It restates, in plain C with 4x64-bit limbs and obviously-correct (slow)
 * algorithms, what the reference computes:
 *   - Keccak-256 ............ crypto/sha3/keccakf.go:1-412 (permutation),
 *                             crypto/sha3/sha3.go:104-185 (sponge, pad 0x01/0x80),
 *                             crypto/sha3/hashes.go:16 (rate 136, dsbyte 0x01)
 *   - field mod p ........... libsecp256k1 src/field_10x26_impl.h (set_b32 rejects >= p, :323-345),
 *                             src/field_impl.h:38-134 (sqrt = x^((p+1)/4) + square check)
 *   - scalar mod n .......... src/scalar_8x32_impl.h:165-179 (set_b32 reduces, reports overflow),
 *                             :220-236 (is_high), src/scalar_impl.h:55-281 (inverse)
 *   - group law ............. src/group_impl.h:216-237 (set_xo_var), :301-518 (double/add incl.
 *                             infinity / P==Q / P==-Q cases)
 *   - ecmult ................ src/ecmult_impl.h:286-404 (u2*R + u1*G) as a plain joint
 *                             double-and-add over bits (same value, no wNAF)
 *   - recover ............... crypto/secp256k1/ext.h:30-47, src/modules/recovery/main_impl.h:38-58,
 *                             :87-121, :170-191; src/secp256k1.c:165-186 (serialize)
 *   - verify ................ crypto/secp256k1/ext.h:58-75, src/secp256k1.c:150-163, :228-247,
 *                             :293-308, src/eckey_impl.h:17-34, src/ecdsa_impl.h:203-271
 *   - Go wrapper checks ..... crypto/secp256k1/secp256.go:105-134,171-179
 *   - Sender / recoverPlain . core/types/transaction_signing.go:127-137,182-184,218-260,
 *                             core/types/transaction.go:142-149, crypto/crypto.go:181-192
 *
 * Parity of this restatement is pinned in tests/ against (a) the reference
 * libsecp256k1 compiled in place (oracle/_ref, see oracle/Makefile) and (b) the
 * golden vectors committed under tests/golden/ (Go test vectors, EIP-155
 * vectors, libsecp256k1 edge vectors).
 */
#include <stdint.h>
#include <string.h>
#include <stddef.h>

typedef unsigned __int128 u128;
typedef uint64_t u64;

/* ======================================================================== */
/* Keccak-256 (legacy padding 0x01), crypto/sha3                            */
/* ======================================================================== */
static const u64 KRC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808AULL, 0x8000000080008000ULL,
    0x000000000000808BULL, 0x0000000080000001ULL, 0x8000000080008081ULL, 0x8000000000008009ULL,
    0x000000000000008AULL, 0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000AULL,
    0x000000008000808BULL, 0x800000000000008BULL, 0x8000000000008089ULL, 0x8000000000008003ULL,
    0x8000000000008002ULL, 0x8000000000000080ULL, 0x000000000000800AULL, 0x800000008000000AULL,
    0x8000000080008081ULL, 0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};
static const int KROT[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};

static u64 rotl64(u64 x, int r) { return r ? (x << r) | (x >> (64 - r)) : x; }

/* Textbook theta / rho+pi / chi / iota over A[x + 5y]. */
void oracle_keccakf(u64 A[25]) {
    for (int round = 0; round < 24; ++round) {
        u64 C[5], D[5], B[25];
        for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
        for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rotl64(C[(x + 1) % 5], 1);
        for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(A[x + 5 * y], KROT[x + 5 * y]);
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                A[x + 5 * y] = B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= KRC[round];
    }
}

/* Generic sponge: rate in bytes, dsbyte as in sha3.go (0x01 Keccak, 0x06 SHA3). */
void oracle_sponge(const unsigned char *in, size_t len, unsigned char *out, size_t outlen, int rate, unsigned char ds) {
    u64 A[25];
    unsigned char blk[200];
    memset(A, 0, sizeof A);
    while (len >= (size_t)rate) {
        for (int i = 0; i < rate / 8; ++i) {
            u64 w = 0;
            for (int b = 0; b < 8; ++b) w |= (u64)in[8 * i + b] << (8 * b);
            A[i] ^= w;
        }
        oracle_keccakf(A);
        in += rate;
        len -= (size_t)rate;
    }
    memset(blk, 0, sizeof blk);
    memcpy(blk, in, len);
    blk[len] ^= ds;
    blk[rate - 1] ^= 0x80;
    for (int i = 0; i < rate / 8; ++i) {
        u64 w = 0;
        for (int b = 0; b < 8; ++b) w |= (u64)blk[8 * i + b] << (8 * b);
        A[i] ^= w;
    }
    oracle_keccakf(A);
    size_t o = 0;
    for (;;) {
        for (int i = 0; i < rate && o < outlen; ++i, ++o) out[o] = (unsigned char)(A[i / 8] >> (8 * (i % 8)));
        if (o >= outlen) break;
        oracle_keccakf(A);
    }
}

void oracle_keccak256(const unsigned char *in, size_t len, unsigned char out[32]) {
    oracle_sponge(in, len, out, 32, 136, 0x01);
}

/* ======================================================================== */
/* 256-bit integers, little-endian 4x64                                     */
/* ======================================================================== */
typedef struct { u64 v[4]; } u256;

static const u256 P = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const u256 N = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
/* 2^256 - p and 2^256 - n */
static const u64 PC[3] = {0x00000001000003D1ULL, 0, 0};
static const u64 NC[3] = {0x402DA1732FC9BEBFULL, 0x4551231950B75FC4ULL, 0x1ULL};
/* floor(n/2), crypto/crypto.go:39 */
static const u256 HALF_N = {{0xDFE92F46681B20A0ULL, 0x5D576E7357A4501DULL, 0xFFFFFFFFFFFFFFFFULL, 0x7FFFFFFFFFFFFFFFULL}};

static void u256_from_be(u256 *r, const unsigned char *b) {
    for (int i = 0; i < 4; ++i) {
        u64 w = 0;
        for (int j = 0; j < 8; ++j) w = (w << 8) | b[(3 - i) * 8 + j];
        r->v[i] = w;
    }
}
static void u256_to_be(unsigned char *b, const u256 *a) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (unsigned char)(a->v[i] >> (56 - 8 * j));
}
static int u256_cmp(const u256 *a, const u256 *b) {
    for (int i = 3; i >= 0; --i) {
        if (a->v[i] < b->v[i]) return -1;
        if (a->v[i] > b->v[i]) return 1;
    }
    return 0;
}
static int u256_is_zero(const u256 *a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }
static u64 u256_add(u256 *r, const u256 *a, const u256 *b) {
    u128 c = 0;
    for (int i = 0; i < 4; ++i) {
        c += (u128)a->v[i] + b->v[i];
        r->v[i] = (u64)c;
        c >>= 64;
    }
    return (u64)c;
}
static u64 u256_sub(u256 *r, const u256 *a, const u256 *b) {
    u64 borrow = 0;
    for (int i = 0; i < 4; ++i) {
        u128 d = (u128)a->v[i] - b->v[i] - borrow;
        r->v[i] = (u64)d;
        borrow = (u64)(d >> 64) & 1;
    }
    return borrow;
}

/* Reduce a 512-bit value x[8] modulo m = 2^256 - c (c has <= 3 limbs) by folding. */
static void mod_reduce512(u256 *r, const u64 x_in[8], const u64 c[3], const u256 *m) {
    u64 x[8];
    memcpy(x, x_in, sizeof x);
    for (;;) {
        int hi_zero = 1;
        for (int i = 4; i < 8; ++i) hi_zero &= (x[i] == 0);
        if (hi_zero) break;
        /* x = lo + hi * c */
        u64 t[8] = {x[0], x[1], x[2], x[3], 0, 0, 0, 0};
        for (int i = 0; i < 4; ++i) {
            u128 carry = 0;
            for (int j = 0; j < 3; ++j) {
                if (i + j >= 8) break;
                carry += (u128)x[4 + i] * c[j] + t[i + j];
                t[i + j] = (u64)carry;
                carry >>= 64;
            }
            for (int k = i + 3; k < 8 && carry; ++k) {
                carry += t[k];
                t[k] = (u64)carry;
                carry >>= 64;
            }
        }
        memcpy(x, t, sizeof x);
    }
    u256 v = {{x[0], x[1], x[2], x[3]}};
    while (u256_cmp(&v, m) >= 0) u256_sub(&v, &v, m);
    *r = v;
}

static void mul_wide(u64 out[8], const u256 *a, const u256 *b) {
    memset(out, 0, 8 * sizeof(u64));
    for (int i = 0; i < 4; ++i) {
        u128 carry = 0;
        for (int j = 0; j < 4; ++j) {
            carry += (u128)a->v[i] * b->v[j] + out[i + j];
            out[i + j] = (u64)carry;
            carry >>= 64;
        }
        out[i + 4] = (u64)carry;
    }
}

/* ---- field mod p ---- */
static void fe_mul(u256 *r, const u256 *a, const u256 *b) { u64 w[8]; mul_wide(w, a, b); mod_reduce512(r, w, PC, &P); }
static void fe_sqr(u256 *r, const u256 *a) { fe_mul(r, a, a); }
static void fe_add(u256 *r, const u256 *a, const u256 *b) {
    u64 w[8] = {0};
    u256 t;
    w[4] = u256_add(&t, a, b);
    memcpy(w, t.v, sizeof t.v);
    mod_reduce512(r, w, PC, &P);
}
static void fe_sub(u256 *r, const u256 *a, const u256 *b) {
    u256 t;
    if (u256_sub(&t, a, b)) u256_add(&t, &t, &P);
    *r = t;
}
static void fe_neg(u256 *r, const u256 *a) { u256 z = {{0, 0, 0, 0}}; fe_sub(r, &z, a); }
static void fe_set_u64(u256 *r, u64 x) { r->v[0] = x; r->v[1] = r->v[2] = r->v[3] = 0; }
static int fe_eq(const u256 *a, const u256 *b) { return u256_cmp(a, b) == 0; }
/* r = a^e (square-and-multiply, MSB first) */
static void fe_pow(u256 *r, const u256 *a, const u256 *e) {
    u256 acc;
    fe_set_u64(&acc, 1);
    for (int i = 255; i >= 0; --i) {
        fe_sqr(&acc, &acc);
        if ((e->v[i / 64] >> (i % 64)) & 1) fe_mul(&acc, &acc, a);
    }
    *r = acc;
}
static void fe_inv(u256 *r, const u256 *a) {
    u256 e = P;
    e.v[0] -= 2;
    fe_pow(r, a, &e);
}
/* field_impl.h:38-134: r = a^((p+1)/4); returns whether r^2 == a. */
static int fe_sqrt(u256 *r, const u256 *a) {
    u256 e = {{0xFFFFFFFFBFFFFF0CULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0x3FFFFFFFFFFFFFFFULL}};
    u256 t;
    fe_pow(r, a, &e);
    fe_sqr(&t, r);
    return fe_eq(&t, a);
}

/* ---- scalar mod n ---- */
/* scalar_8x32_impl.h:165-179: reduce b32 mod n, report overflow (value >= n). */
static int sc_set_b32(u256 *r, const unsigned char *b) {
    u256 t;
    u256_from_be(&t, b);
    int overflow = u256_cmp(&t, &N) >= 0;
    if (overflow) u256_sub(&t, &t, &N);
    *r = t;
    return overflow;
}
static void sc_mul(u256 *r, const u256 *a, const u256 *b) { u64 w[8]; mul_wide(w, a, b); mod_reduce512(r, w, NC, &N); }
static void sc_neg(u256 *r, const u256 *a) {
    if (u256_is_zero(a)) { *r = *a; return; }
    u256_sub(r, &N, a);
}
static void sc_inv(u256 *r, const u256 *a) {
    u256 e = N, acc;
    e.v[0] -= 2;
    fe_set_u64(&acc, 1);
    for (int i = 255; i >= 0; --i) {
        sc_mul(&acc, &acc, &acc);
        if ((e.v[i / 64] >> (i % 64)) & 1) sc_mul(&acc, &acc, a);
    }
    *r = acc;
}
static int sc_is_high(const u256 *a) { return u256_cmp(a, &HALF_N) > 0; }

/* ======================================================================== */
/* Group law (Jacobian, with every exceptional case)                        */
/* ======================================================================== */
typedef struct { u256 x, y; int inf; } ge;
typedef struct { u256 x, y, z; int inf; } gej;

static const ge GEN = {
    {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}},
    {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}}, 0};

static void gej_set_ge(gej *r, const ge *a) {
    r->x = a->x; r->y = a->y; fe_set_u64(&r->z, 1); r->inf = a->inf;
}
/* group_impl.h:301-354 (value-level): 2*(X,Y,Z) on y^2 = x^3 + 7 */
static void gej_double(gej *r, const gej *a) {
    if (a->inf || u256_is_zero(&a->y)) { r->inf = 1; return; }
    u256 A, B, C, D, E, F, t;
    fe_sqr(&A, &a->x);                 /* X^2 */
    fe_sqr(&B, &a->y);                 /* Y^2 */
    fe_sqr(&C, &B);                    /* Y^4 */
    fe_add(&t, &a->x, &B);
    fe_sqr(&t, &t);
    fe_sub(&t, &t, &A);
    fe_sub(&t, &t, &C);
    fe_add(&D, &t, &t);                /* D = 2((X+B)^2 - A - C) = 4XY^2 */
    fe_add(&E, &A, &A);
    fe_add(&E, &E, &A);                /* E = 3X^2 */
    fe_sqr(&F, &E);
    gej o;
    fe_add(&t, &D, &D);
    fe_sub(&o.x, &F, &t);              /* X3 = E^2 - 2D */
    fe_sub(&t, &D, &o.x);
    fe_mul(&t, &E, &t);
    u256 c8;
    fe_add(&c8, &C, &C); fe_add(&c8, &c8, &c8); fe_add(&c8, &c8, &c8);
    fe_sub(&o.y, &t, &c8);             /* Y3 = E(D - X3) - 8C */
    fe_mul(&o.z, &a->y, &a->z);
    fe_add(&o.z, &o.z, &o.z);          /* Z3 = 2YZ */
    o.inf = 0;
    *r = o;
}
/* group_impl.h:414-461 (value-level): (X,Y,Z) + affine (x,y), all cases */
static void gej_add_ge(gej *r, const gej *a, const ge *b) {
    if (b->inf) { *r = *a; return; }
    if (a->inf) { gej_set_ge(r, b); return; }
    u256 z2, u2, s2, h, rr, h2, h3, u1h2, t;
    fe_sqr(&z2, &a->z);
    fe_mul(&u2, &b->x, &z2);
    fe_mul(&s2, &b->y, &z2);
    fe_mul(&s2, &s2, &a->z);
    fe_sub(&h, &u2, &a->x);
    fe_sub(&rr, &s2, &a->y);
    if (u256_is_zero(&h)) {
        if (u256_is_zero(&rr)) { gej_double(r, a); return; }
        r->inf = 1;
        return;
    }
    fe_sqr(&h2, &h);
    fe_mul(&h3, &h2, &h);
    fe_mul(&u1h2, &a->x, &h2);
    gej o;
    fe_sqr(&o.x, &rr);
    fe_sub(&o.x, &o.x, &h3);
    fe_add(&t, &u1h2, &u1h2);
    fe_sub(&o.x, &o.x, &t);            /* X3 = R^2 - H^3 - 2 U1 H^2 */
    fe_sub(&t, &u1h2, &o.x);
    fe_mul(&t, &rr, &t);
    fe_mul(&o.y, &a->y, &h3);
    fe_sub(&o.y, &t, &o.y);            /* Y3 = R(U1H^2 - X3) - S1 H^3 */
    fe_mul(&o.z, &a->z, &h);           /* Z3 = Z1 H */
    o.inf = 0;
    *r = o;
}
static void ge_set_gej(ge *r, const gej *a) {
    if (a->inf) { r->inf = 1; return; }
    u256 zi, zi2, zi3;
    fe_inv(&zi, &a->z);
    fe_sqr(&zi2, &zi);
    fe_mul(&zi3, &zi2, &zi);
    fe_mul(&r->x, &a->x, &zi2);
    fe_mul(&r->y, &a->y, &zi3);
    r->inf = 0;
}
/* group_impl.h:216-237: lift x with requested y parity; 0 if x^3+7 is a non-residue. */
static int ge_set_xo(ge *r, const u256 *x, int odd) {
    u256 x3, c, y;
    fe_sqr(&x3, x);
    fe_mul(&x3, &x3, x);
    fe_set_u64(&c, 7);
    fe_add(&c, &x3, &c);
    if (!fe_sqrt(&y, &c)) return 0;
    if ((int)(y.v[0] & 1) != odd) fe_neg(&y, &y);
    r->x = *x; r->y = y; r->inf = 0;
    return 1;
}
/* group_impl.h:287-299 */
static int ge_is_valid(const ge *a) {
    if (a->inf) return 0;
    u256 y2, x3, c;
    fe_sqr(&y2, &a->y);
    fe_sqr(&x3, &a->x);
    fe_mul(&x3, &x3, &a->x);
    fe_set_u64(&c, 7);
    fe_add(&x3, &x3, &c);
    return fe_eq(&y2, &x3);
}
/* ecmult_impl.h:286 value: r = na*A + ng*G (joint double-and-add, MSB first) */
static void ecmult(gej *r, const ge *A, const u256 *na, const u256 *ng) {
    gej acc;
    acc.inf = 1;
    for (int i = 255; i >= 0; --i) {
        gej_double(&acc, &acc);
        if ((na->v[i / 64] >> (i % 64)) & 1) gej_add_ge(&acc, &acc, A);
        if ((ng->v[i / 64] >> (i % 64)) & 1) gej_add_ge(&acc, &acc, &GEN);
    }
    *r = acc;
}

/* ======================================================================== */
/* Recover / verify                                                         */
/* ======================================================================== */
/* secp256k1_ext_ecdsa_recover (ext.h:30-47). Returns 1 ok, 0 failure.
 * Precondition (Go checkSignature, secp256.go:171-179): sig65[64] < 4. */
int oracle_ext_ecdsa_recover(unsigned char pub65[65], const unsigned char sig65[65], const unsigned char msg32[32]) {
    int recid = sig65[64];
    u256 r, s, m;
    memset(pub65, 0, 65);
    if (recid < 0 || recid > 3) return -3; /* ARG_CHECK in parse_compact */
    /* parse_compact, recovery/main_impl.h:38-58: overflow => 0 */
    if (sc_set_b32(&r, sig65)) return 0;
    if (sc_set_b32(&s, sig65 + 32)) return 0;
    /* secp256k1_ecdsa_recover :183: message reduced mod n, overflow ignored */
    sc_set_b32(&m, msg32);
    /* sig_recover :87-121 */
    if (u256_is_zero(&r) || u256_is_zero(&s)) return 0;
    u256 fx = r;
    if (recid & 2) {
        u256 pmn;
        u256_sub(&pmn, &P, &N);
        if (u256_cmp(&fx, &pmn) >= 0) return 0;
        u256_add(&fx, &fx, &N);
    }
    ge X;
    if (!ge_set_xo(&X, &fx, recid & 1)) return 0;
    u256 rn, u1, u2;
    sc_inv(&rn, &r);
    sc_mul(&u1, &rn, &m);
    sc_neg(&u1, &u1);
    sc_mul(&u2, &rn, &s);
    gej Q;
    ecmult(&Q, &X, &u2, &u1);
    if (Q.inf) return 0;
    ge q;
    ge_set_gej(&q, &Q);
    /* ec_pubkey_serialize, uncompressed (eckey_impl.h:36-52) */
    pub65[0] = 0x04;
    u256_to_be(pub65 + 1, &q.x);
    u256_to_be(pub65 + 33, &q.y);
    return 1;
}

/* secp256k1.RecoverPubkey (secp256.go:105-122). Returns status:
 * 0 ok, 5 ErrInvalidRecoveryID, 6 ErrRecoverFailed. (lengths are fixed here) */
int oracle_recover_pubkey(unsigned char pub65[65], const unsigned char sig65[65], const unsigned char msg32[32]) {
    if (sig65[64] >= 4) { memset(pub65, 0, 65); return 5; }
    return oracle_ext_ecdsa_recover(pub65, sig65, msg32) == 1 ? 0 : 6;
}

/* eckey_pubkey_parse (eckey_impl.h:17-34) */
static int pubkey_parse(ge *elem, const unsigned char *pub, size_t size) {
    if (size == 33 && (pub[0] == 0x02 || pub[0] == 0x03)) {
        u256 x;
        u256_from_be(&x, pub + 1);
        if (u256_cmp(&x, &P) >= 0) return 0;
        return ge_set_xo(elem, &x, pub[0] == 0x03);
    } else if (size == 65 && (pub[0] == 0x04 || pub[0] == 0x06 || pub[0] == 0x07)) {
        u256 x, y;
        u256_from_be(&x, pub + 1);
        u256_from_be(&y, pub + 33);
        if (u256_cmp(&x, &P) >= 0 || u256_cmp(&y, &P) >= 0) return 0;
        elem->x = x; elem->y = y; elem->inf = 0;
        if ((pub[0] == 0x06 || pub[0] == 0x07) && (int)(y.v[0] & 1) != (pub[0] == 0x07)) return 0;
        return ge_is_valid(elem);
    }
    return 0;
}

/* secp256k1_ext_ecdsa_verify (ext.h:58-75) -> ecdsa_verify (secp256k1.c:293-308). */
int oracle_ext_ecdsa_verify(const unsigned char sig64[64], const unsigned char msg32[32], const unsigned char *pub,
                            size_t publen) {
    u256 r, s, m;
    if (sc_set_b32(&r, sig64)) return 0;
    if (sc_set_b32(&s, sig64 + 32)) return 0;
    ge Q;
    if (!pubkey_parse(&Q, pub, publen)) return 0;
    sc_set_b32(&m, msg32);
    if (sc_is_high(&s)) return 0;
    /* sig_verify, ecdsa_impl.h:203-271 */
    if (u256_is_zero(&r) || u256_is_zero(&s)) return 0;
    u256 sn, u1, u2;
    sc_inv(&sn, &s);
    sc_mul(&u1, &sn, &m);
    sc_mul(&u2, &sn, &r);
    gej pr;
    ecmult(&pr, &Q, &u2, &u1);
    if (pr.inf) return 0;
    ge a;
    ge_set_gej(&a, &pr);
    /* x(pr) mod n == r  <=>  x == r or (r + n < p and x == r + n) */
    if (fe_eq(&a.x, &r)) return 1;
    u256 pmn, rn;
    u256_sub(&pmn, &P, &N);
    if (u256_cmp(&r, &pmn) >= 0) return 0;
    u256_add(&rn, &r, &N);
    return fe_eq(&a.x, &rn);
}

/* crypto.VerifySignature (signature_cgo.go:66 -> secp256.go:126-134). */
int oracle_verify_signature(const unsigned char *pub, size_t publen, const unsigned char *msg, size_t msglen,
                            const unsigned char *sig, size_t siglen) {
    if (msglen != 32 || siglen != 64 || publen == 0) return 0;
    return oracle_ext_ecdsa_verify(sig, msg, pub, publen);
}

/* ======================================================================== */
/* types.Sender (EIP155 / Homestead / Frontier) — transaction_signing.go     */
/* ======================================================================== */
/* Status codes shared with include/eges.h */
enum { ST_OK = 0, ST_INVALID_CHAIN_ID = 1, ST_INVALID_SIG = 2, ST_INVALID_RECOVERY_ID = 5, ST_RECOVER_FAILED = 6 };
enum { SIGNER_FRONTIER = 0, SIGNER_HOMESTEAD = 1, SIGNER_EIP155 = 2 };
enum { VF_V_WIDE = 1, VF_R_WIDE = 2, VF_S_WIDE = 4 };

/* bit length of a 256-bit big-endian value */
static int bitlen_be(const unsigned char *b) {
    for (int i = 0; i < 32; ++i)
        if (b[i]) {
            int bl = 0;
            unsigned v = b[i];
            while (v) { ++bl; v >>= 1; }
            return (31 - i) * 8 + bl;
        }
    return 0;
}

/* recoverPlain (transaction_signing.go:222-247) with V already reduced to {27,28,...}
 * given as a 256-bit BE value vb (+ wide flag). */
/* The recovery recoverPlain ends in (crypto.Ecrecover): this restatement's own by default;
 * oracle_sender_with lets a caller put the reference libsecp256k1's in its place (ref_shim.c),
 * so that the Go-layer rules here are checked with the reference's recovery underneath. */
typedef int (*recover_fn)(unsigned char pub65[65], const unsigned char sig65[65], const unsigned char msg32[32]);

static int recover_plain(recover_fn rec, unsigned char addr20[20], const unsigned char sighash[32],
                         const unsigned char r32[32], const unsigned char s32[32], const unsigned char vb[32],
                         int v_wide, int r_wide, int s_wide, int homestead) {
    if (v_wide || bitlen_be(vb) > 8) return ST_INVALID_SIG;
    unsigned char V = (unsigned char)(vb[31] - 27); /* byte(Vb.Uint64() - 27) */
    /* ValidateSignatureValues (crypto.go:181-192) */
    u256 R, S, one = {{1, 0, 0, 0}};
    u256_from_be(&R, r32);
    u256_from_be(&S, s32);
    if (!r_wide && u256_cmp(&R, &one) < 0) return ST_INVALID_SIG;
    if (!s_wide && u256_cmp(&S, &one) < 0) return ST_INVALID_SIG;
    if (homestead && (s_wide || u256_cmp(&S, &HALF_N) > 0)) return ST_INVALID_SIG;
    if (r_wide || s_wide || u256_cmp(&R, &N) >= 0 || u256_cmp(&S, &N) >= 0 || !(V == 0 || V == 1))
        return ST_INVALID_SIG;
    unsigned char sig[65], pub[65], h[32];
    memcpy(sig, r32, 32);
    memcpy(sig + 32, s32, 32);
    sig[64] = V;
    int st = rec(pub, sig, sighash);
    if (st) return st;
    oracle_keccak256(pub + 1, 64, h);
    memcpy(addr20, h + 12, 20);
    return ST_OK;
}

/* 256-bit BE helpers for V arithmetic */
static void be_sub_u64(unsigned char *r, const unsigned char *a, u64 x) {
    int borrow = 0;
    for (int i = 31; i >= 0; --i) {
        int d = (int)a[i] - (int)(x & 0xff) - borrow;
        borrow = d < 0;
        r[i] = (unsigned char)(d & 0xff);
        x >>= 8;
    }
}

/* Signer.Sender for the three signers. v32 = V as 256-bit BE (VF_V_WIDE if V > 2^256).
 * chain_id is the EIP155 signer's chain id (uint64). Returns a status. `rec` recovers the key
 * (oracle_recover_pubkey's contract: 0 ok, else the status). */
int oracle_sender_with(recover_fn rec, unsigned char addr20[20], int signer, u64 chain_id,
                       const unsigned char sighash[32], const unsigned char r32[32], const unsigned char s32[32],
                       const unsigned char v32[32], int vflags) {
    int v_wide = vflags & VF_V_WIDE, r_wide = vflags & VF_R_WIDE, s_wide = vflags & VF_S_WIDE;
    memset(addr20, 0, 20);
    if (signer == SIGNER_FRONTIER) /* :218-220 */
        return recover_plain(rec, addr20, sighash, r32, s32, v32, v_wide, r_wide, s_wide, 0);
    if (signer == SIGNER_HOMESTEAD) /* :182-184 */
        return recover_plain(rec, addr20, sighash, r32, s32, v32, v_wide, r_wide, s_wide, 1);
    /* EIP155Signer.Sender :127-137 */
    int bl = v_wide ? 1000 : bitlen_be(v32);
    int prot; /* isProtectedV, transaction.go:142-149 */
    if (bl <= 8) prot = !(v32[31] == 27 || v32[31] == 28);
    else prot = 1;
    if (!prot) return recover_plain(rec, addr20, sighash, r32, s32, v32, v_wide, r_wide, s_wide, 1);
    /* deriveChainId (:250-260) compared with chain_id */
    int match;
    if (bl <= 64) {
        u64 v = 0;
        for (int i = 24; i < 32; ++i) v = (v << 8) | v32[i];
        u64 cid = (v == 27 || v == 28) ? 0 : (v - 35) / 2; /* uint64 wrap as in Go */
        match = (cid == chain_id);
    } else if (v_wide) {
        match = 0; /* (V-35)/2 >= 2^255 cannot equal a uint64 chain id */
    } else {
        /* big path: (V-35)/2 == chain_id  <=>  V-35 in {2c, 2c+1} */
        unsigned char t[32];
        be_sub_u64(t, v32, 35);
        /* V>=2^64 here so no underflow; compare t>>1 with chain_id */
        int hi_zero = 1;
        for (int i = 0; i < 23; ++i) hi_zero &= (t[i] == 0);
        u64 lo = 0;
        for (int i = 24; i < 32; ++i) lo = (lo << 8) | t[i];
        /* t >> 1 as 256-bit: need bits above 64 of (t>>1) zero */
        u64 sh = (lo >> 1) | ((u64)(t[23] & 1) << 63);
        hi_zero &= ((t[23] >> 1) == 0);
        match = hi_zero && sh == chain_id;
    }
    if (!match) return ST_INVALID_CHAIN_ID;
    /* V = V - 2*chainId - 8 (chainIdMul as big.Int, no wrap) */
    unsigned char vp[32];
    u128 mul = (u128)chain_id * 2 + 8;
    /* subtract a 128-bit value */
    {
        int borrow = 0;
        for (int i = 31; i >= 0; --i) {
            int d = (int)v32[i] - (int)(unsigned)(mul & 0xff) - borrow;
            borrow = d < 0;
            vp[i] = (unsigned char)(d & 0xff);
            mul >>= 8;
        }
        (void)borrow; /* V >= 2c+35 here, no underflow */
    }
    return recover_plain(rec, addr20, sighash, r32, s32, vp, 0, r_wide, s_wide, 1);
}

int oracle_sender(unsigned char addr20[20], int signer, u64 chain_id, const unsigned char sighash[32],
                  const unsigned char r32[32], const unsigned char s32[32], const unsigned char v32[32], int vflags) {
    return oracle_sender_with(oracle_recover_pubkey, addr20, signer, chain_id, sighash, r32, s32, v32, vflags);
}

/* Address from uncompressed pubkey (crypto.go:194-197 PubkeyToAddress / recoverPlain :245). */
void oracle_pub_to_addr(unsigned char addr20[20], const unsigned char pub65[65]) {
    unsigned char h[32];
    oracle_keccak256(pub65 + 1, 64, h);
    memcpy(addr20, h + 12, 20);
}

/* Batch helpers (one thread; tests use small sizes). */
void oracle_recover_batch(size_t n, const unsigned char *msg, const unsigned char *sig, unsigned char *pub_out,
                          unsigned char *addr_out, unsigned char *status) {
    for (size_t i = 0; i < n; ++i) {
        status[i] = (unsigned char)oracle_recover_pubkey(pub_out + 65 * i, sig + 65 * i, msg + 32 * i);
        if (status[i] == 0) oracle_pub_to_addr(addr_out + 20 * i, pub_out + 65 * i);
        else memset(addr_out + 20 * i, 0, 20);
    }
}
