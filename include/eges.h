/*
 * eges.h — C-ABI of the MI355X-native secp256k1 sender-recovery engine (libeges.so).
 *
 * Drop-in boundary for the reference's cgo seam in crypto/secp256k1 (secp256.go:20-37,
 * ext.h:18-142): plain pointers and sizes, no torch / HIP types in any signature. A Go
 * binding is a one-line cgo call per entry.
 *
 * Conventions (mirroring the reference seam):
 *   - Single-item entries return exactly what the replaced C function returns (1 / 0).
 *   - Batch entries return an eges_rc call code (0 = success) and write one eges_status
 *     byte per item; item statuses are a 1:1 image of the Go errors the reference path
 *     returns for that item.
 *   - The caller owns every buffer; nothing is retained after return. Host-pointer entries
 *     are synchronous. *_dev entries take device pointers and a hipStream_t (as void*, NULL
 *     meaning the HIP null stream) and are asynchronous on that stream.
 *   - n == 0 is valid and a no-op. A NULL pointer where n > 0 needs it returns
 *     EGES_E_NULLPTR (never crashes).
 *   - Thread-safe. Concurrent single-item callers are coalesced into shared batches (group
 *     commit); batch calls from several threads run one after another on a device.
 *   - There is no CPU fallback: without a usable gfx950 device every compute entry fails
 *     with EGES_E_NODEVICE.
 */
#ifndef EGES_H
#define EGES_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EGES_ABI_VERSION 1

/* Per-item status: 1:1 image of the reference errors. */
typedef enum eges_status {
    EGES_OK = 0,
    EGES_INVALID_CHAIN_ID = 1,    /* types.ErrInvalidChainId  core/types/transaction_signing.go:30 */
    EGES_INVALID_SIG = 2,         /* types.ErrInvalidSig      core/types/transaction.go:36 (recoverPlain :223-229) */
    EGES_INVALID_MSG_LEN = 3,     /* secp256k1.ErrInvalidMsgLen        crypto/secp256k1/secp256.go:55 */
    EGES_INVALID_SIG_LEN = 4,     /* secp256k1.ErrInvalidSignatureLen  secp256.go:56 */
    EGES_INVALID_RECOVERY_ID = 5, /* secp256k1.ErrInvalidRecoveryID    secp256.go:57 */
    EGES_RECOVER_FAILED = 6,      /* secp256k1.ErrRecoverFailed        secp256.go:61 */
    EGES_DECODE_FAILED = 7,       /* rlp.DecodeBytes(raw, tx) error (transaction.go:157-165, rlp/decode.go):
                                     wire-format entries only; the reference never calls Sender */
    EGES_ENGINE_FAULT = 255       /* not a reference error: an internal hand-off between the waves of a
                                     kernel workgroup timed out, and the item got no result (no address
                                     is written). Host-buffer entries then return EGES_E_HIP; *_dev
                                     entries leave it in the status byte (and EGES_DIAG_HANDOFF counts
                                     it). Never produced by a call that returns EGES_SUCCESS. The
                                     VerifySignature entries never write it: their ok bytes stay 0 / 1
                                     (a faulted item reads 0, see eges_verify_batch). */
} eges_status;

/* Call-level return codes. */
typedef enum eges_rc {
    EGES_SUCCESS = 0,
    EGES_E_NULLPTR = -1,
    EGES_E_NODEVICE = -2,
    EGES_E_HIP = -3,
    EGES_E_INVALID_ARG = -4,
    EGES_E_NOMEM = -5
} eges_rc;

/* Signer kinds for eges_sender_batch (core/types/transaction_signing.go). */
typedef enum eges_signer {
    EGES_SIGNER_FRONTIER = 0,  /* FrontierSigner  :218-220 (homestead = false) */
    EGES_SIGNER_HOMESTEAD = 1, /* HomesteadSigner :182-184 (low-s enforced)     */
    EGES_SIGNER_EIP155 = 2     /* EIP155Signer    :127-137                      */
} eges_signer;

/* Per-item flags for eges_sender_batch: the big.Int did not fit in 256 bits. */
#define EGES_VF_V_WIDE 0x1u
#define EGES_VF_R_WIDE 0x2u
#define EGES_VF_S_WIDE 0x4u

/* ---------------------------------------------------------------- lifecycle */

/* Replaces the package init() that builds the context (secp256.go:45-52, ext.h:18-20):
 * selects devices (bit i of device_mask = HIP device i; 0 = all visible), uploads the
 * fixed-base tables and allocates staging. Idempotent. flags: reserved, pass 0. */
int eges_init(uint32_t device_mask, uint32_t flags);
void eges_shutdown(void);
/* Number of devices the engine is using (0 before eges_init / without a GPU). */
int eges_device_count(void);
/* Human-readable description of the last error on this thread. */
const char *eges_last_error(void);
int eges_abi_version(void);

/* ---------------------------------------------------------------- single item */

/* Replaces secp256k1_ext_ecdsa_recover (crypto/secp256k1/ext.h:30-47).
 * sig65 = R || S || recid, msg32 = hash. Returns 1 and writes the 65-byte uncompressed
 * public key on success, 0 on failure (including recid >= 4, which the reference's
 * parse_compact ARG_CHECK would reject). An engine failure (no device, HIP error) also returns 0
 * and leaves its text for eges_last_error on the calling thread ("" after a call that ran). */
int eges_ecdsa_recover(unsigned char *pubkey_out65, const unsigned char *sigdata65,
                       const unsigned char *msgdata32);

/* Replaces secp256k1_ext_ecdsa_verify (crypto/secp256k1/ext.h:58-75).
 * sig64 = R || S. Returns 1 if valid, 0 otherwise (low-s enforced); engine failures as above. */
int eges_ecdsa_verify(const unsigned char *sigdata64, const unsigned char *msgdata32,
                      const unsigned char *pubkeydata, size_t pubkeylen);

/* ---------------------------------------------------------------- batch, host buffers */

/* crypto.Ecrecover over a batch (crypto/signature_cgo.go:31 -> secp256.go:105-122).
 * msg: n*32, sig: n*65. Outputs (each may be NULL): pub_out n*65 (zeros on failure),
 * addr_out n*20 = Keccak256(pub[1:])[12:] (crypto.go:194-197), status n bytes:
 * EGES_OK / EGES_INVALID_RECOVERY_ID / EGES_RECOVER_FAILED. */
int eges_ecrecover_batch(const uint8_t *msg, const uint8_t *sig, size_t n, uint8_t *pub_out,
                         uint8_t *addr_out, uint8_t *status);

/* types.Sender over a batch (transaction_signing.go:72-89,127-137,182-184,218-247).
 * sighash n*32 = signer.Hash(tx) (the caller passes the Frontier hash for unprotected
 * txs under an EIP155 signer, as HomesteadSigner.Sender would use). r, s, v: n*32 each,
 * big-endian, left-padded; vflags n bytes of EGES_VF_*. chain_id: the EIP155 signer's
 * chain id (ignored for the other signers). Outputs: addr_out n*20, status n. */
int eges_sender_batch(const uint8_t *sighash, const uint8_t *r, const uint8_t *s, const uint8_t *v,
                      const uint8_t *vflags, size_t n, int signer, uint64_t chain_id, uint8_t *addr_out,
                      uint8_t *status);

/* types.Sender over a batch of wire-format transactions (SURVEY.md §8(f) N1 + N4): item i is the
 * RLP encoding of one Geec txdata (core/types/transaction.go:59-76, 10 fields) at
 * raw[offsets[i] - offsets[0], offsets[i+1] - offsets[0]) — offsets has n + 1 non-decreasing
 * entries (a block body's or TxMsg's tx list split at item boundaries, or txs concatenated).
 * On the GPU each item is decoded with the reference decoder's rules (rlp.DecodeBytes), its
 * signing hash built and Keccak-256'd (EIP155Signer.Hash for protected V under an EIP155
 * signer, else FrontierSigner.Hash: transaction_signing.go:127-137,155-165,207-216) and its
 * sender recovered exactly as eges_sender_batch. Outputs: addr_out n*20, status n
 * (EGES_DECODE_FAILED for items rlp.DecodeBytes rejects), sighash_out n*32 (nullable: the
 * signing hash, zeros for undecodable items). */
int eges_sender_raw_batch(const uint8_t *raw, const uint64_t *offsets, size_t n, int signer, uint64_t chain_id,
                          uint8_t *addr_out, uint8_t *status, uint8_t *sighash_out);

/* Senders of a whole Geec block: block is the RLP of one block as the
 * wire and the chain carry it, the extblock list of core/types/block.go:188-195
 * [Header, FakeTxs, GeecTxs, Txs, Uncles, Confirm]. The list structure is split as
 * rlp.DecodeBytes(block, &b) (Block.DecodeRLP, block.go:273-282) walks it; every transaction of
 * the lists selected by `lists` (bit 0 FakeTxs, bit 1 GeecTxs, bit 2 Txs) then goes through
 * eges_sender_raw_batch's path (GPU decode, signing hash, recovery). counts[3] receives the
 * item count of each list; addr_out / status (cap entries) receive the selected lists' results
 * concatenated in list order. *block_status = EGES_OK, or EGES_DECODE_FAILED when the block
 * structure (or a selected transaction) would make rlp.DecodeBytes fail; header, uncle and
 * confirm-message field contents are not decoded; the transactions of unselected lists are
 * decoded (not recovered) on the GPU, as rlp.DecodeBytes decodes them too. Returns
 * EGES_E_INVALID_ARG when more than cap transactions are selected (a sizing call): counts are
 * then valid, and *block_status covers the block's list structure only (EGES_DECODE_FAILED for a
 * structure error; EGES_OK does not yet mean that every transaction decodes, since none was
 * decoded). */
#define EGES_LIST_FAKE 0x1u
#define EGES_LIST_GEEC 0x2u
#define EGES_LIST_TXS 0x4u
int eges_block_senders_raw(const uint8_t *block, size_t len, uint32_t lists, int signer, uint64_t chain_id,
                           size_t cap, uint8_t *addr_out, uint8_t *status, uint32_t *counts, int *block_status);

/* The EVM ECRECOVER precompile (core/vm/contracts.go:77-101, address 0x01) over a batch: input
 * n*128 (hash, v, r, s as 32-byte words); inlen n (nullable = all 128): bytes at or past
 * inlen[i] read as zero, which is the RightPadBytes of :82 (a longer input passes its first 128
 * bytes, as Run reads no further). out32 n*32: 12 zero bytes + the address when status[i] ==
 * EGES_OK, all zero when Run returns nil — status EGES_INVALID_SIG for its pre-checks
 * (input[32:63] not zero, ValidateSignatureValues(input[63] - 27, r, s, homestead = false)) or
 * EGES_RECOVER_FAILED when crypto.Ecrecover fails. */
int eges_ecrecover_precompile_batch(const uint8_t *input, const uint32_t *inlen, size_t n, uint8_t *out32,
                                    uint8_t *status);

/* crypto.VerifySignature over a batch (signature_cgo.go:66 -> secp256.go:126-134).
 * pub: n*65 (each key left-aligned, publen[i] bytes valid: 33 or 65; 0 => false),
 * msg n*32, sig n*64. ok_out n bytes, always 0 or 1. An item whose in-kernel wave hand-off timed
 * out reads 0; the call then returns EGES_E_HIP (eges_verify_batch_dev cannot: it returns before
 * the kernels run, so there EGES_DIAG_HANDOFF is the only report). */
int eges_verify_batch(const uint8_t *pub, const uint8_t *publen, const uint8_t *msg, const uint8_t *sig,
                      size_t n, uint8_t *ok_out);

/* ---------------------------------------------------------------- batch, device buffers */
/* Same semantics; all pointers are device pointers on `device`, work is enqueued on
 * `stream` (a hipStream_t; NULL = the HIP null stream, exactly as in HIP) and the call
 * returns without synchronising. Engine work is serialised across streams on a device. */
int eges_ecrecover_batch_dev(int device, const uint8_t *msg, const uint8_t *sig, size_t n, uint8_t *pub_out,
                             uint8_t *addr_out, uint8_t *status, void *stream);
int eges_sender_batch_dev(int device, const uint8_t *sighash, const uint8_t *r, const uint8_t *s,
                          const uint8_t *v, const uint8_t *vflags, size_t n, int signer, uint64_t chain_id,
                          uint8_t *addr_out, uint8_t *status, void *stream);
/* offsets: device array of n + 1 entries, same meaning as above. */
int eges_sender_raw_batch_dev(int device, const uint8_t *raw, const uint64_t *offsets, size_t n, int signer,
                              uint64_t chain_id, uint8_t *addr_out, uint8_t *status, uint8_t *sighash_out,
                              void *stream);
int eges_ecrecover_precompile_batch_dev(int device, const uint8_t *input, const uint32_t *inlen, size_t n,
                                        uint8_t *out32, uint8_t *status, void *stream);
int eges_verify_batch_dev(int device, const uint8_t *pub, const uint8_t *publen, const uint8_t *msg,
                          const uint8_t *sig, size_t n, uint8_t *ok_out, void *stream);

/* ---------------------------------------------------------------- utilities */

/* Keccak-256 (crypto.Keccak256, crypto/crypto.go:43-49), host implementation. */
void eges_keccak256(const uint8_t *data, size_t len, uint8_t *out32);

/* Synthetic workload generator (not on the hot path): on `device`, signs n messages with
 * deterministic keys. Item i (global index first_index + i):
 *   key_i = Keccak256("eges-key" || le64(i)) mod n (0 -> 1), msg_i = Keccak256("eges-msg" || le64(i)),
 *   nonce_i = Keccak256("eges-nonce" || le64(i)) mod n (0 -> 1), low-s normalised.
 * Writes msg n*32, sig n*65 (R||S||recid) and the expected address n*20 (from key_i*G).
 * Device pointers, asynchronous on stream. */
int eges_synth_sign_dev(int device, uint64_t first_index, size_t n, uint8_t *msg, uint8_t *sig,
                        uint8_t *addr_expected, void *stream);

/* Same signer over caller-supplied message hashes msg_in (n*32, device): item i signs
 * msg_in[i] with key_i and nonce_i as above (used for synthetic Geec blocks whose messages are
 * EIP-155 sighashes). */
int eges_synth_sign_msg_dev(int device, uint64_t first_index, size_t n, const uint8_t *msg_in, uint8_t *sig,
                            uint8_t *addr_expected, void *stream);

/* ---------------------------------------------------------------- diagnostics and tests */

/* Counters the kernels bump (once per wave) when a rare exact branch runs. The reference takes
 * these branches inline (group_impl.h:414-461 gej_add_ge_var's a == b doubling and a == -b
 * infinity); this engine adds without the check and redoes a poisoned accumulator exactly
 * (DESIGN.md §3.1), or joins partial sums with an exact addition (§3.3). */
#define EGES_DIAG_LS_REDO 0   /* lane-serial kernels: exact redo of a wave's Strauss loop */
#define EGES_DIAG_LS_EXC 1    /* lane-serial checked addition met P == +-Q (doubling / infinity) */
#define EGES_DIAG_LAT_REDO 2  /* latency kernels: exact redo of an R' Strauss part */
#define EGES_DIAG_LAT_EXC 3   /* latency kernels: checked addition met P == +-Q */
#define EGES_DIAG_COMB_REDO 4 /* latency kernels: exact redo of the u1*G comb */
#define EGES_DIAG_JOIN_DBL 5  /* latency kernels: partial sums joined with a == b (doubling) */
#define EGES_DIAG_JOIN_INF 6  /* latency kernels: partial sums joined with a == -b (infinity) */
#define EGES_DIAG_MID_REDO 7  /* mid-size kernel: exact redo of an R' Strauss part */
#define EGES_DIAG_MID_EXC 8   /* mid-size kernel: checked addition met P == +-Q */
#define EGES_DIAG_MID_JOIN 9  /* mid-size kernel: partial sums joined with a == +-b */
#define EGES_DIAG_HANDOFF 10  /* a wave hand-off timed out: the workgroup's items got EGES_ENGINE_FAULT */
#define EGES_DIAG_LAT_TRI 11  /* latency kernels: launches that ran the three-wave form */
#define EGES_DIAG_RESIDENT 12 /* resident single-call server: jobs served */
#define EGES_DIAG_COUNT 16
/* Copies min(n, EGES_DIAG_COUNT) counters of `device` (summed over the engine's instances of
 * it) into out; reset != 0 zeroes them afterwards. Synchronises the device. */
int eges_diag_counters(int device, uint64_t *out, size_t n, int reset);
/* 1 while the resident single-call server of `device` is running (its persistent launch has not
 * ended: it serves jobs, or polls for one until its idle window runs out), 0 when it is not,
 * EGES_E_INVALID_ARG for a device the engine does not manage. Does not synchronise anything
 * (bench.py and tests use it to record whether the server was alive at a given moment). */
int eges_diag_resident_running(int device);

/* Engine knobs. Read from the environment once, at the first eges_init (EGES_LAT_MAX,
 * EGES_LAT_WIDE_MAX, EGES_MID_MAX, EGES_TXROWS_WAVE_MAX, EGES_TEST_ROOT_HELPERS, EGES_OVERLAP,
 * EGES_TEST_FORCE_REDO, EGES_TEST_SKIP_FLAG, ...); no call path reads the environment after that.
 * A call reads the routing knobs once, at its start: a change takes effect from the next call. These two entries
 * change / read one by its environment name while the engine runs (tests and A/B tools; the
 * product defaults need neither). Return EGES_E_INVALID_ARG for an unknown name. */
int eges_test_set_knob(const char *name, long long value);
int eges_test_get_knob(const char *name, long long *value);

#ifdef __cplusplus
}
#endif

#endif /* EGES_H */
