/*
 * TEST INFRASTRUCTURE ONLY — never linked into the product library.
 *
 * Build-time shim that compiles the REFERENCE libsecp256k1 in place, exactly
 * the way the reference's cgo preamble does (crypto/secp256k1/secp256.go:20-37:
 * one translation unit that #includes src/secp256k1.c, the recovery module and
 * ext.h, with USE_NUM_NONE / USE_FIELD_10X26 / USE_FIELD_INV_BUILTIN /
 * USE_SCALAR_8X32 / USE_SCALAR_INV_BUILTIN / NDEBUG). No reference source is
 * copied into this repository: the Makefile points -I at /root/reference and
 * the result lands in oracle/_ref/ (git-ignored).
 *
 * It exposes plain C entry points (eref_*) with the Go wrapper's pre-checks
 * (crypto/secp256k1/secp256.go:105-134,171-179) so that Python tests can drive
 * the reference the way crypto.Ecrecover / crypto.VerifySignature do, plus a
 * pthread harness (one worker per core) used as bench.py's cpu_baseline — the
 * goroutine-parallel CPU path BASELINE.json names, restated in C.
 */
#include "src/secp256k1.c"
#include "src/modules/recovery/main_impl.h"
#include "ext.h"

#include <pthread.h>
#include <stdint.h>
#include <string.h>

static secp256k1_context *g_ctx = NULL;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static __thread int g_illegal = 0;

/* secp256.go:50-51 route these to Go panics; here they set a thread-local flag. */
static void eref_illegal_cb(const char *msg, void *data) { (void)msg; (void)data; g_illegal = 1; }
static void eref_error_cb(const char *msg, void *data) { (void)msg; (void)data; g_illegal = 2; }

static void eref_init_once(void) {
    /* secp256.go:47-52 */
    g_ctx = secp256k1_context_create_sign_verify();
    secp256k1_context_set_illegal_callback(g_ctx, eref_illegal_cb, NULL);
    secp256k1_context_set_error_callback(g_ctx, eref_error_cb, NULL);
}

static secp256k1_context *ctx_get(void) {
    pthread_once(&g_once, eref_init_once);
    return g_ctx;
}

/* Go: secp256k1.RecoverPubkey (secp256.go:105-122).
 * Returns 1 ok, 0 ErrRecoverFailed, -2 ErrInvalidRecoveryID, -3 illegal-arg panic. */
int eref_ecrecover(unsigned char *pub65, const unsigned char *sig65, const unsigned char *msg32) {
    secp256k1_context *ctx = ctx_get();
    if (sig65[64] >= 4) return -2; /* checkSignature, secp256.go:175-177 */
    g_illegal = 0;
    int r = secp256k1_ext_ecdsa_recover(ctx, pub65, sig65, msg32);
    if (g_illegal) return -3;
    return r;
}

/* Go: secp256k1.VerifySignature (secp256.go:126-134) minus the length checks,
 * which the caller applies. Returns 1/0, -3 on illegal-arg panic. */
int eref_verify(const unsigned char *sig64, const unsigned char *msg32, const unsigned char *pub, size_t publen) {
    secp256k1_context *ctx = ctx_get();
    if (publen == 0) return 0;
    g_illegal = 0;
    int r = secp256k1_ext_ecdsa_verify(ctx, sig64, msg32, pub, publen);
    if (g_illegal) return -3;
    return r;
}

/* Go: secp256k1.Sign (secp256.go:70-99), RFC6979 nonces. Returns 1 ok, 0 fail. */
int eref_sign(unsigned char *sig65, const unsigned char *msg32, const unsigned char *seckey32) {
    secp256k1_context *ctx = ctx_get();
    secp256k1_ecdsa_recoverable_signature sig;
    int recid = 0;
    if (secp256k1_ec_seckey_verify(ctx, seckey32) != 1) return 0;
    if (!secp256k1_ecdsa_sign_recoverable(ctx, &sig, msg32, seckey32, secp256k1_nonce_function_rfc6979, NULL))
        return 0;
    secp256k1_ecdsa_recoverable_signature_serialize_compact(ctx, sig65, &recid, &sig);
    sig65[64] = (unsigned char)recid;
    return 1;
}

/* Public key of a secret key, 65-byte uncompressed. Returns 1 ok, 0 invalid key. */
int eref_pubkey(unsigned char *pub65, const unsigned char *seckey32) {
    secp256k1_context *ctx = ctx_get();
    secp256k1_pubkey pk;
    size_t len = 65;
    if (!secp256k1_ec_pubkey_create(ctx, &pk, seckey32)) return 0;
    return secp256k1_ec_pubkey_serialize(ctx, pub65, &len, &pk, SECP256K1_EC_UNCOMPRESSED);
}

/* Go: secp256k1.DecompressPubkey / CompressPubkey via ext_reencode_pubkey (ext.h:88). */
int eref_reencode(unsigned char *out, size_t outlen, const unsigned char *pub, size_t publen) {
    secp256k1_context *ctx = ctx_get();
    g_illegal = 0;
    int r = secp256k1_ext_reencode_pubkey(ctx, out, outlen, pub, publen);
    if (g_illegal) return -3;
    return r;
}

/* ---- pthread batch harness: the CPU baseline (one worker per core) ----
 * Per item: crypto.Ecrecover (reference C, exactly as cgo compiles it) then the address
 * Keccak256(pub[1:])[12:] (transaction_signing.go:245). The reference's Keccak is Go/asm and
 * cannot be built here; the oracle's C restatement of it (oracle.c, linked into this .so by
 * oracle/Makefile) stands in for it. */
void oracle_keccak256(const unsigned char *in, size_t len, unsigned char out[32]);

typedef struct {
    size_t lo, hi;
    const unsigned char *msg, *sig;
    unsigned char *pub, *addr;
    signed char *ret;
} eref_job;

static void *eref_worker(void *p) {
    eref_job *j = (eref_job *)p;
    unsigned char h[32];
    for (size_t i = j->lo; i < j->hi; ++i) {
        j->ret[i] = (signed char)eref_ecrecover(j->pub + 65 * i, j->sig + 65 * i, j->msg + 32 * i);
        if (j->addr) {
            if (j->ret[i] == 1) {
                oracle_keccak256(j->pub + 65 * i + 1, 64, h);
                memcpy(j->addr + 20 * i, h + 12, 20);
            } else {
                memset(j->addr + 20 * i, 0, 20);
            }
        }
    }
    return NULL;
}

/* Recover n signatures (msg n*32, sig n*65) with nthreads workers.
 * pub_out n*65, addr_out n*20 (may be NULL), ret_out n (codes as eref_ecrecover). */
void eref_ecrecover_batch_mt(size_t n, const unsigned char *msg, const unsigned char *sig, unsigned char *pub_out,
                             unsigned char *addr_out, signed char *ret_out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    ctx_get();
    pthread_t th[1024];
    eref_job jobs[1024];
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    int t;
    for (t = 0; t < nthreads; ++t) {
        size_t lo = (size_t)t * per, hi = lo + per;
        if (lo > n) lo = n;
        if (hi > n) hi = n;
        jobs[t].lo = lo; jobs[t].hi = hi; jobs[t].msg = msg; jobs[t].sig = sig;
        jobs[t].pub = pub_out; jobs[t].addr = addr_out; jobs[t].ret = ret_out;
        pthread_create(&th[t], NULL, eref_worker, &jobs[t]);
    }
    for (t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* ---- types.Sender over the reference libsecp256k1 (TEST INFRASTRUCTURE) ----
 * The Go-layer rules (EIP155Signer / HomesteadSigner / FrontierSigner.Sender, recoverPlain,
 * ValidateSignatureValues) are oracle.c's restatement (oracle_sender_with); the recovery under
 * them is the reference's secp256k1_ext_ecdsa_recover (eref_ecrecover), one pthread per worker.
 * Used by the GPU tests to check the engine's Sender statuses and addresses item for item at
 * configs[4]'s full size. */
int oracle_sender_with(int (*rec)(unsigned char *, const unsigned char *, const unsigned char *), unsigned char *addr20,
                       int signer, unsigned long long chain_id, const unsigned char *sighash, const unsigned char *r32,
                       const unsigned char *s32, const unsigned char *v32, int vflags);

static int eref_recover_status(unsigned char *pub65, const unsigned char *sig65, const unsigned char *msg32) {
    const int r = eref_ecrecover(pub65, sig65, msg32);
    return r == 1 ? 0 : r == -2 ? 5 /* EGES_INVALID_RECOVERY_ID */ : 6 /* EGES_RECOVER_FAILED */;
}

typedef struct {
    size_t lo, hi;
    int signer;
    unsigned long long chain_id;
    const unsigned char *h, *r, *s, *v, *f;
    unsigned char *addr, *status;
} eref_sender_job;

static void *eref_sender_worker(void *p) {
    eref_sender_job *j = (eref_sender_job *)p;
    for (size_t i = j->lo; i < j->hi; ++i)
        j->status[i] = (unsigned char)oracle_sender_with(eref_recover_status, j->addr + 20 * i, j->signer, j->chain_id,
                                                         j->h + 32 * i, j->r + 32 * i, j->s + 32 * i, j->v + 32 * i,
                                                         j->f ? j->f[i] : 0);
    return NULL;
}

void eref_sender_batch_mt(size_t n, int signer, unsigned long long chain_id, const unsigned char *sighash,
                          const unsigned char *r, const unsigned char *s, const unsigned char *v,
                          const unsigned char *vflags, unsigned char *addr_out, unsigned char *status_out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    ctx_get();
    pthread_t th[1024];
    eref_sender_job jobs[1024];
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    int t;
    for (t = 0; t < nthreads; ++t) {
        size_t lo = (size_t)t * per, hi = lo + per;
        if (lo > n) lo = n;
        if (hi > n) hi = n;
        eref_sender_job jb = {lo, hi, signer, chain_id, sighash, r, s, v, vflags, addr_out, status_out};
        jobs[t] = jb;
        pthread_create(&th[t], NULL, eref_sender_worker, &jobs[t]);
    }
    for (t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

/* ---- crypto.VerifySignature over the reference libsecp256k1 (TEST INFRASTRUCTURE) ----
 * Per item: eref_verify (secp256.go:126-134 -> ext.h:58-75) on pub[65*i .. 65*i+publen[i]),
 * msg[32*i], sig[64*i]; ok_out[i] = 1 valid, 0 invalid, 255 illegal-arg panic. One pthread per
 * worker; the GPU tests compare the engine's VerifySignature mode with it item for item. */
typedef struct {
    size_t lo, hi;
    const unsigned char *pub, *publen, *msg, *sig;
    unsigned char *ok;
} eref_verify_job;

static void *eref_verify_worker(void *p) {
    eref_verify_job *j = (eref_verify_job *)p;
    for (size_t i = j->lo; i < j->hi; ++i) {
        const int r = eref_verify(j->sig + 64 * i, j->msg + 32 * i, j->pub + 65 * i, j->publen[i]);
        j->ok[i] = (unsigned char)(r < 0 ? 255 : r);
    }
    return NULL;
}

void eref_verify_batch_mt(size_t n, const unsigned char *pub, const unsigned char *publen, const unsigned char *msg,
                          const unsigned char *sig, unsigned char *ok_out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    ctx_get();
    pthread_t th[1024];
    eref_verify_job jobs[1024];
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    int t;
    for (t = 0; t < nthreads; ++t) {
        size_t lo = (size_t)t * per, hi = lo + per;
        if (lo > n) lo = n;
        if (hi > n) hi = n;
        eref_verify_job jb = {lo, hi, pub, publen, msg, sig, ok_out};
        jobs[t] = jb;
        pthread_create(&th[t], NULL, eref_verify_worker, &jobs[t]);
    }
    for (t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}
