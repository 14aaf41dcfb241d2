/*
 * TEST INFRASTRUCTURE ONLY — a standalone driver for the CPU sanitizer run of the checker
 * (VERDICT r1 item 10). `make -C oracle sanitize` compiles it with oracle.c and, where
 * /root/reference exists, ref_shim.c (the reference libsecp256k1 built in place) under
 * -fsanitize=address,undefined, and runs it: every oracle entry point and every eref_*
 * entry point on signed, mutated and random inputs, with the two checked against each other
 * item for item. Any sanitizer report aborts the run (-fno-sanitize-recover); a mismatch
 * exits 1. Without the reference tree it exercises the oracle alone (-DNO_REF).
 *
 * `--replay FILE` re-executes, in this sanitized build, every call that tests/test_oracle.py and
 * tests/test_txoracle.py made through oracle/pyoracle.py (recorded with EGES_ORACLE_RECORD, see
 * there), each input in an exact-size heap buffer, and checks every output byte for byte
 * against what the unsanitized libraries returned in the pytest run.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned long long u64;

void oracle_keccakf(u64 A[25]);
void oracle_sponge(const unsigned char *in, size_t len, unsigned char *out, size_t outlen, int rate, unsigned char ds);
void oracle_keccak256(const unsigned char *in, size_t len, unsigned char out[32]);
int oracle_ext_ecdsa_recover(unsigned char pub65[65], const unsigned char sig65[65], const unsigned char msg32[32]);
int oracle_recover_pubkey(unsigned char pub65[65], const unsigned char sig65[65], const unsigned char msg32[32]);
int oracle_ext_ecdsa_verify(const unsigned char sig64[64], const unsigned char msg32[32], const unsigned char *pub,
                            size_t publen);
int oracle_verify_signature(const unsigned char *pub, size_t publen, const unsigned char *msg, size_t msglen,
                            const unsigned char *sig, size_t siglen);
int oracle_sender(unsigned char addr20[20], int signer, u64 chain_id, const unsigned char sighash[32],
                  const unsigned char r32[32], const unsigned char s32[32], const unsigned char v32[32], int vflags);
void oracle_pub_to_addr(unsigned char addr20[20], const unsigned char pub65[65]);
void oracle_recover_batch(size_t n, const unsigned char *msg, const unsigned char *sig, unsigned char *pub_out,
                          unsigned char *addr_out, unsigned char *status);
#ifndef NO_REF
int eref_ecrecover(unsigned char *pub65, const unsigned char *sig65, const unsigned char *msg32);
int eref_verify(const unsigned char *sig64, const unsigned char *msg32, const unsigned char *pub, size_t publen);
int eref_sign(unsigned char *sig65, const unsigned char *msg32, const unsigned char *seckey32);
int eref_pubkey(unsigned char *pub65, const unsigned char *seckey32);
int eref_reencode(unsigned char *out, size_t outlen, const unsigned char *pub, size_t publen);
void eref_ecrecover_batch_mt(size_t n, const unsigned char *msg, const unsigned char *sig, unsigned char *pub_out,
                             unsigned char *addr_out, signed char *ret_out, int nthreads);
#endif

static u64 g_rng = 0x9e3779b97f4a7c15ull;
static u64 rnd(void) {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return g_rng;
}
static void fill(unsigned char *b, size_t n) {
    for (size_t i = 0; i < n; ++i) b[i] = (unsigned char)rnd();
}

static long g_checks = 0, g_fail = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        ++g_checks;                                    \
        if (!(c)) {                                    \
            ++g_fail;                                  \
            fprintf(stderr, "MISMATCH %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);              \
            fputc('\n', stderr);                       \
        }                                              \
    } while (0)

static const unsigned char N_BE[32] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                       0xff, 0xff, 0xff, 0xff, 0xfe, 0xba, 0xae, 0xdc, 0xe6, 0xaf, 0x48,
                                       0xa0, 0x3b, 0xbf, 0xd2, 0x5e, 0x8c, 0xd0, 0x36, 0x41, 0x41};

/* Keccak: known answers, every length across two rate boundaries, heap buffers of exact size. */
static void keccak_cases(void) {
    static const unsigned char empty[32] = {0xc5, 0xd2, 0x46, 0x01, 0x86, 0xf7, 0x23, 0x3c, 0x92, 0x7e, 0x7d,
                                            0xb2, 0xdc, 0xc7, 0x03, 0xc0, 0xe5, 0x00, 0xb6, 0x53, 0xca, 0x82,
                                            0x27, 0x3b, 0x7b, 0xfa, 0xd8, 0x04, 0x5d, 0x85, 0xa4, 0x70};
    unsigned char h[32];
    oracle_keccak256((const unsigned char *)"", 0, h);
    CHECK(!memcmp(h, empty, 32), "keccak256(\"\")");
    for (size_t len = 0; len <= 2 * 136 + 3; ++len) {
        unsigned char *in = malloc(len ? len : 1), out[64];
        fill(in, len);
        oracle_keccak256(in, len, h);
        oracle_sponge(in, len, out, 64, 136, 0x01); /* squeeze past 32 bytes */
        CHECK(!memcmp(h, out, 32), "sponge prefix len %zu", len);
        free(in);
    }
    u64 A[25] = {0};
    oracle_keccakf(A);
}

#ifndef NO_REF
static void cmp_recover(const unsigned char sig[65], const unsigned char msg[32], const char *what) {
    unsigned char po[65], pr[65];
    int o = oracle_ext_ecdsa_recover(po, sig, msg);
    memset(pr, 0, 65);
    int r = eref_ecrecover(pr, sig, msg);
    CHECK(o == r, "%s: recover rc oracle %d ref %d", what, o, r);
    if (o == 1 && r == 1) CHECK(!memcmp(po, pr, 65), "%s: pubkey", what);
}

/* Signed signatures, then every field mutated the ways the parse and lift reject. */
static void recover_cases(int n) {
    unsigned char key[32], msg[32], sig[65], pub[65], rec[65], a1[20], a2[20];
    for (int i = 0; i < n; ++i) {
        fill(key, 32);
        fill(msg, 32);
        if (!eref_sign(sig, msg, key)) continue;
        CHECK(eref_pubkey(pub, key) == 1, "pubkey");
        CHECK(oracle_recover_pubkey(rec, sig, msg) == 0 && !memcmp(rec, pub, 65), "sign/recover round trip %d", i);
        oracle_pub_to_addr(a1, rec);
        oracle_pub_to_addr(a2, pub);
        CHECK(!memcmp(a1, a2, 20), "address");
        cmp_recover(sig, msg, "signed");
        unsigned char m[65];
        memcpy(m, sig, 65);
        m[64] ^= 1;
        cmp_recover(m, msg, "flipped recid");
        memcpy(m, sig, 65);
        m[64] |= 2;
        cmp_recover(m, msg, "recid 2/3");
        memcpy(m, sig, 65);
        memset(m, 0, 32);
        cmp_recover(m, msg, "r = 0");
        memcpy(m, sig, 65);
        memset(m + 32, 0, 32);
        cmp_recover(m, msg, "s = 0");
        memcpy(m, sig, 65);
        memcpy(m, N_BE, 32);
        cmp_recover(m, msg, "r = n");
        memcpy(m, sig, 65);
        memcpy(m + 32, N_BE, 32);
        cmp_recover(m, msg, "s = n");
        memcpy(m, sig, 65);
        m[1 + (rnd() % 31)] ^= (unsigned char)(1u << (rnd() % 8));
        cmp_recover(m, msg, "bit flip in r");
        fill(m, 64);
        m[64] = (unsigned char)(rnd() & 3);
        cmp_recover(m, msg, "random r, s");
        m[64] = (unsigned char)(4 + rnd() % 252);
        CHECK(oracle_recover_pubkey(rec, m, msg) == 5, "recid >= 4 -> ErrInvalidRecoveryID");
        CHECK(eref_ecrecover(rec, m, msg) == -2, "ref recid >= 4");
        /* verify through every pubkey encoding */
        unsigned char enc33[33], enc65h[65];
        CHECK(eref_reencode(enc33, 33, pub, 65) == 1, "compress");
        memcpy(enc65h, pub, 65);
        enc65h[0] = (unsigned char)(0x06 | (pub[64] & 1));
        unsigned char s64[64];
        memcpy(s64, sig, 64);
        const unsigned char *pubs[3] = {pub, enc33, enc65h};
        const size_t lens[3] = {65, 33, 65};
        for (int k = 0; k < 3; ++k) {
            int o = oracle_ext_ecdsa_verify(s64, msg, pubs[k], lens[k]);
            int r = eref_verify(s64, msg, pubs[k], lens[k]);
            CHECK(o == r, "verify enc %d: %d vs %d", k, o, r);
            CHECK(oracle_verify_signature(pubs[k], lens[k], msg, 32, s64, 64) == o, "VerifySignature");
        }
        unsigned char junk[65];
        fill(junk, 65);
        size_t jl = rnd() % 66;
        if (jl) junk[0] = (unsigned char)(rnd() % 8);
        CHECK(oracle_ext_ecdsa_verify(s64, msg, junk, jl) == eref_verify(s64, msg, junk, jl), "verify junk pub len %zu",
              jl);
        CHECK(oracle_verify_signature(pub, 65, msg, 31, s64, 64) == 0, "msg length");
        CHECK(oracle_verify_signature(pub, 65, msg, 32, s64, 65) == 0, "sig length");
        CHECK(oracle_verify_signature(pub, 0, msg, 32, s64, 64) == 0, "empty pub");
    }
}

/* The reference's pthread harness (bench.py's cpu_baseline) under the same sanitizers. */
static void batch_cases(size_t n) {
    unsigned char *msg = malloc(32 * n), *sig = malloc(65 * n), *p1 = malloc(65 * n), *p2 = malloc(65 * n),
                  *a1 = malloc(20 * n), *a2 = malloc(20 * n), *st = malloc(n);
    signed char *rc = malloc(n);
    unsigned char key[32];
    for (size_t i = 0; i < n; ++i) {
        fill(key, 32);
        fill(msg + 32 * i, 32);
        if (!eref_sign(sig + 65 * i, msg + 32 * i, key) || i % 7 == 3) fill(sig + 65 * i, 64);
    }
    eref_ecrecover_batch_mt(n, msg, sig, p1, a1, rc, 4);
    oracle_recover_batch(n, msg, sig, p2, a2, st);
    for (size_t i = 0; i < n; ++i) {
        CHECK((rc[i] == 1) == (st[i] == 0), "batch rc %zu", i);
        if (st[i] == 0) CHECK(!memcmp(p1 + 65 * i, p2 + 65 * i, 65) && !memcmp(a1 + 20 * i, a2 + 20 * i, 20), "batch %zu", i);
    }
    free(msg), free(sig), free(p1), free(p2), free(a1), free(a2), free(st), free(rc);
}
#endif

/* types.Sender over the three signers and the V shapes EIP155 distinguishes. */
static void sender_cases(int n) {
    unsigned char sh[32], r[32], s[32], v[32], addr[20];
    const u64 cids[4] = {0, 1, 9999, 0xffffffffffffffffull};
    for (int i = 0; i < n; ++i) {
        fill(sh, 32);
        fill(r, 32);
        fill(s, 32);
        memset(v, 0, 32);
        const int shape = (int)(rnd() % 6);
        if (shape == 0) v[31] = (unsigned char)(27 + (rnd() & 1));
        if (shape == 1) { u64 x = rnd(); for (int k = 0; k < 8; ++k) v[31 - k] = (unsigned char)(x >> (8 * k)); }
        if (shape == 2) fill(v + 16, 16);
        if (shape == 3) fill(v, 32);
        if (shape == 4) v[31] = (unsigned char)(35 + 2 * 9999 % 256);
        for (int signer = 0; signer < 3; ++signer)
            for (int c = 0; c < 4; ++c) {
                int st = oracle_sender(addr, signer, cids[c], sh, r, s, v, (int)(rnd() % 8));
                CHECK(st >= 0 && st <= 6, "sender status %d", st);
            }
    }
}

/* ---- replay of recorded Python-test calls */
typedef struct {
    unsigned char *p;
    size_t n;
} field;

static long long fint(const field *f) {
    long long v = 0;
    memcpy(&v, f->p, f->n < 8 ? f->n : 8);
    return v;
}
static unsigned char *dup(const field *f) { /* exact-size copy: any overread is reported */
    unsigned char *q = malloc(f->n ? f->n : 1);
    memcpy(q, f->p, f->n);
    return q;
}
static void same(const unsigned char *got, const field *want, const char *what, long rec) {
    CHECK(!memcmp(got, want->p, want->n), "replay record %ld: %s differs", rec, what);
}

static long replay(const char *path) {
    FILE *fh = fopen(path, "rb");
    if (!fh) { perror(path); exit(2); }
    fseek(fh, 0, SEEK_END);
    const long sz = ftell(fh);
    fseek(fh, 0, SEEK_SET);
    unsigned char *buf = malloc(sz ? (size_t)sz : 1);
    if (fread(buf, 1, (size_t)sz, fh) != (size_t)sz) { perror("read"); exit(2); }
    fclose(fh);
    long rec = 0, pos = 0;
    while (pos < sz) {
        const int op = buf[pos], nf = buf[pos + 1];
        pos += 2;
        field f[16];
        for (int i = 0; i < nf && i < 16; ++i) {
            uint32_t len;
            memcpy(&len, buf + pos, 4);
            f[i].p = buf + pos + 4;
            f[i].n = len;
            pos += 4 + len;
        }
        unsigned char *a = NULL, *b = NULL, *c = NULL, *d = NULL, *o1 = NULL, *o2 = NULL, *o3 = NULL;
        switch (op) {
            case 1: /* keccak256: in -> out32 */
                a = dup(&f[0]), o1 = malloc(32);
                oracle_keccak256(a, f[0].n, o1);
                same(o1, &f[1], "keccak256", rec);
                break;
            case 2: /* sponge: in, outlen, rate, ds -> out */
                a = dup(&f[0]), o1 = malloc((size_t)fint(&f[1]) + 1);
                oracle_sponge(a, f[0].n, o1, (size_t)fint(&f[1]), (int)fint(&f[2]), (unsigned char)fint(&f[3]));
                same(o1, &f[4], "sponge", rec);
                break;
            case 3: /* recover_pubkey: msg, sig -> st, pub */
                a = dup(&f[0]), b = dup(&f[1]), o1 = malloc(65);
                CHECK(oracle_recover_pubkey(o1, b, a) == fint(&f[2]), "replay %ld: recover status", rec);
                same(o1, &f[3], "recover pub", rec);
                break;
            case 4: { /* recover_batch: n, msg, sig -> pub, addr, st */
                const size_t n = (size_t)fint(&f[0]);
                a = dup(&f[1]), b = dup(&f[2]), o1 = malloc(65 * n + 1), o2 = malloc(20 * n + 1), o3 = malloc(n + 1);
                oracle_recover_batch(n, a, b, o1, o2, o3);
                same(o1, &f[3], "batch pub", rec), same(o2, &f[4], "batch addr", rec), same(o3, &f[5], "batch st", rec);
                break;
            }
            case 5: /* verify: pub, msg, sig -> ok */
                a = dup(&f[0]), b = dup(&f[1]), c = dup(&f[2]);
                CHECK(oracle_verify_signature(a, f[0].n, b, f[1].n, c, f[2].n) == fint(&f[3]), "replay %ld: verify", rec);
                break;
            case 6: { /* sender: signer, chain, sighash, r, s, v, vflags -> st, addr */
                u64 chain;
                memcpy(&chain, f[1].p, 8);
                a = dup(&f[2]), b = dup(&f[3]), c = dup(&f[4]), d = dup(&f[5]), o1 = malloc(20);
                CHECK(oracle_sender(o1, (int)fint(&f[0]), chain, a, b, c, d, (int)fint(&f[6])) == fint(&f[7]),
                      "replay %ld: sender status", rec);
                same(o1, &f[8], "sender addr", rec);
                break;
            }
            case 7: /* pub_to_addr */
                a = dup(&f[0]), o1 = malloc(20);
                oracle_pub_to_addr(o1, a);
                same(o1, &f[1], "pub_to_addr", rec);
                break;
#ifndef NO_REF
            case 8: /* eref_ecrecover: msg, sig -> r, pub */
                a = dup(&f[0]), b = dup(&f[1]), o1 = calloc(65, 1);
                CHECK(eref_ecrecover(o1, b, a) == fint(&f[2]), "replay %ld: eref rc", rec);
                same(o1, &f[3], "eref pub", rec);
                break;
            case 9: { /* eref_batch_mt: n, msg, sig, nthreads -> pub, addr, ret */
                const size_t n = (size_t)fint(&f[0]);
                a = dup(&f[1]), b = dup(&f[2]), o1 = calloc(65 * n + 1, 1), o2 = calloc(20 * n + 1, 1), o3 = calloc(n + 1, 1);
                eref_ecrecover_batch_mt(n, a, b, o1, o2, (signed char *)o3, (int)fint(&f[3]));
                same(o1, &f[4], "eref batch pub", rec), same(o2, &f[5], "eref batch addr", rec);
                same(o3, &f[6], "eref batch ret", rec);
                break;
            }
#endif
            default:
                fprintf(stderr, "replay: unknown op %d (record %ld)\n", op, rec);
                exit(2);
        }
        free(a), free(b), free(c), free(d), free(o1), free(o2), free(o3);
        ++rec;
    }
    free(buf);
    return rec;
}

int main(int argc, char **argv) {
    if (argc > 2 && !strcmp(argv[1], "--replay")) {
        const long recs = replay(argv[2]);
        printf("sanitize_main --replay: %ld recorded test calls re-run, %ld checks, %ld mismatches\n", recs, g_checks,
               g_fail);
        return g_fail ? 1 : 0;
    }
    const int n = argc > 1 ? atoi(argv[1]) : 200;
    keccak_cases();
    sender_cases(n);
#ifndef NO_REF
    recover_cases(n);
    batch_cases(64);
#endif
    printf("sanitize_main: %ld checks, %ld mismatches (n=%d%s)\n", g_checks, g_fail, n,
#ifndef NO_REF
           ", oracle vs reference"
#else
           ", oracle only"
#endif
    );
    return g_fail ? 1 : 0;
}
