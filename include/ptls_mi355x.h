/*
 * ptls_mi355x.h -- MI355X (gfx950) AES-GCM engine behind picotls' AEAD slot.
 *
 * Drop-in boundary: the picotls crypto-binding ABI, include/picotls.h:308-400 of the
 * reference (mpiraux/rapido @ 2024-08-07).  The engine exports the same kind of objects
 * as the x86 "fusion" engine (include/picotls/fusion.h:87-88, lib/fusion.c:974-1005):
 *
 *     ptls_aead_algorithm_t   ptls_mi355x_aes128gcm, ptls_mi355x_aes256gcm;
 *     ptls_cipher_algorithm_t ptls_mi355x_aes128ctr, ptls_mi355x_aes256ctr;
 *
 * so the TLS 1.3 record layer (lib/picotls.c:630-654) and through it rapido's TCPLS
 * send/receive path (lib/rapido.c:2083-2113, 1929-2026) call it unchanged via
 * ptls_aead_new_direct()/ptls_aead_encrypt()/ptls_aead_decrypt() and the streaming
 * init/update/final trio.  All slot entry points are synchronous and leave nothing
 * retained after return, as the slot contract requires.
 *
 * Throughput comes from the batch extension (ptls_mi355x_seal_batch/open_batch) which
 * seals or opens a whole array of independent records resident in GPU memory with one
 * kernel launch; it is called only by new code (a batched record layer), never by picotls.
 *
 * Include picotls.h BEFORE this header when both are used; otherwise this header declares
 * layout-identical copies of the five picotls types it needs.
 */
#ifndef PTLS_MI355X_H
#define PTLS_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef picotls_h
/* ---- picotls crypto-binding ABI (field order and types of include/picotls.h:311-400) ---- */
typedef struct st_ptls_cipher_context_t {
    const struct st_ptls_cipher_algorithm_t *algo;
    void (*do_dispose)(struct st_ptls_cipher_context_t *ctx);
    void (*do_init)(struct st_ptls_cipher_context_t *ctx, const void *iv);
    void (*do_transform)(struct st_ptls_cipher_context_t *ctx, void *output, const void *input, size_t len);
} ptls_cipher_context_t;

typedef const struct st_ptls_cipher_algorithm_t {
    const char *name;
    size_t key_size;
    size_t block_size;
    size_t iv_size;
    size_t context_size;
    int (*setup_crypto)(ptls_cipher_context_t *ctx, int is_enc, const void *key);
} ptls_cipher_algorithm_t;

typedef struct st_ptls_aead_supplementary_encryption_t {
    ptls_cipher_context_t *ctx;
    const void *input;
    uint8_t output[16];
} ptls_aead_supplementary_encryption_t;

typedef struct st_ptls_aead_context_t {
    const struct st_ptls_aead_algorithm_t *algo;
    void (*dispose_crypto)(struct st_ptls_aead_context_t *ctx);
    void (*do_xor_iv)(struct st_ptls_aead_context_t *ctx, const void *bytes, size_t len);
    void (*do_encrypt_init)(struct st_ptls_aead_context_t *ctx, uint64_t seq, const void *aad, size_t aadlen);
    size_t (*do_encrypt_update)(struct st_ptls_aead_context_t *ctx, void *output, const void *input, size_t inlen);
    size_t (*do_encrypt_final)(struct st_ptls_aead_context_t *ctx, void *output);
    void (*do_encrypt)(struct st_ptls_aead_context_t *ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                       const void *aad, size_t aadlen, ptls_aead_supplementary_encryption_t *supp);
    size_t (*do_decrypt)(struct st_ptls_aead_context_t *ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                         const void *aad, size_t aadlen);
} ptls_aead_context_t;

typedef const struct st_ptls_aead_algorithm_t {
    const char *name;
    const uint64_t confidentiality_limit;
    const uint64_t integrity_limit;
    ptls_cipher_algorithm_t *ctr_cipher;
    ptls_cipher_algorithm_t *ecb_cipher;
    size_t key_size;
    size_t iv_size;
    size_t tag_size;
    size_t context_size;
    int (*setup_crypto)(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv);
} ptls_aead_algorithm_t;
#endif /* picotls_h */

/* ======================================================================================
 * 1. AEAD slot objects -- replace ptls_fusion_aes{128,256}gcm (lib/fusion.c:986-1005) and
 *    ptls_fusion_aes{128,256}ctr (lib/fusion.c:974-985).
 *    - setup_crypto(ctx, is_enc, key, iv): like aesgcm_setup (lib/fusion.c:942-962): key == NULL
 *      only (re)loads the static IV; both the encrypt and decrypt halves are populated.
 *    - do_encrypt writes inlen + 16 bytes (output == input allowed); supp, when given, receives
 *      AES-ECB(supp->ctx key, 16 bytes at supp->input) computed after the record is written
 *      (lib/fusion.c:472-487).
 *    - do_decrypt returns inlen - 16, or SIZE_MAX for a bad tag or inlen < 16
 *      (lib/fusion.c:917-932).  Unlike fusion, a failed open leaves the output zeroed.
 *    - do_encrypt_init/update/final are implemented (fusion asserts, lib/fusion.c:881-896):
 *      update buffers the plaintext and returns 0, final emits ciphertext || tag and returns
 *      inlen + 16, as picotls' record layer (lib/picotls.c:637-640) permits.
 *    - do_xor_iv XORs persistently into the leading static-IV bytes (lib/fusion.c:934-940).
 * ====================================================================================== */
extern ptls_cipher_algorithm_t ptls_mi355x_aes128ctr, ptls_mi355x_aes256ctr;
extern ptls_aead_algorithm_t ptls_mi355x_aes128gcm, ptls_mi355x_aes256gcm;
/*
 * AES-ECB cipher objects, the aead->ecb_cipher of both AEAD objects (fusion leaves ecb_cipher NULL,
 * lib/fusion.c:990,1000; the generic suite t/picotls.c:266-307 needs it).  Like ptls_openssl_aes{128,256}ecb
 * (lib/openssl.c:1580-1597): block_size 16, iv_size 0, no do_init; setup_crypto(ctx, is_enc, key) picks the
 * AES cipher (is_enc != 0) or the inverse cipher (is_enc == 0); do_transform processes len / 16 whole blocks
 * (len must be a multiple of 16).
 */
extern ptls_cipher_algorithm_t ptls_mi355x_aes128ecb, ptls_mi355x_aes256ecb;

/* Capability probe -- replaces ptls_fusion_is_supported_by_cpu (lib/fusion.c:1041-1065):
 * 1 when the calling thread's current HIP device is a gfx950, else 0 (contexts bind to that device). */
int ptls_mi355x_is_supported(void);

/* ======================================================================================
 * 2. Direct engine API -- mirrors ptls_fusion_aesgcm_new/_free/_encrypt/_decrypt
 *    (include/picotls/fusion.h:48-88).  A context owns the device-resident key image
 *    (round keys + GHASH tables) on the device that was current at creation time.
 *    The x86 __m128i counter argument is replaced by the 12-byte nonce.
 * ====================================================================================== */
typedef struct st_ptls_mi355x_aesgcm_context ptls_mi355x_aesgcm_context_t;

/* capacity is accepted for API parity (lib/fusion.c:775); tables do not depend on it. */
ptls_mi355x_aesgcm_context_t *ptls_mi355x_aesgcm_new(const void *key, size_t key_size, size_t capacity);
/* waits for the context's launches (any stream), clears the key image and frees it (ptls_fusion_aesgcm_free,
 * lib/fusion.c:814-820).  An error met there -- an asynchronous fault of earlier GPU work surfaces at the
 * synchronisation -- is printed and reported by the next ptls_mi355x_device_check. */
void ptls_mi355x_aesgcm_free(ptls_mi355x_aesgcm_context_t *ctx);
/* the same, returning 0, or -1 with the first error in ptls_mi355x_last_error (the context is freed either way) */
int ptls_mi355x_aesgcm_release(ptls_mi355x_aesgcm_context_t *ctx);
/* diagnostics: synchronises the current device; 0, or -1 with ptls_mi355x_last_error naming the first error seen
 * since the previous check -- a fault of queued work, or one a free path met (which return nothing) */
int ptls_mi355x_device_check(void);
/* the same on HIP device `device` (one thread serving several GPUs: a context per GPU, records sharded across them,
 * SURVEY.md 8(e)); the caller's current device is left as it was.  NULL, with ptls_mi355x_last_error naming the
 * ordinal, if that device is not present. */
ptls_mi355x_aesgcm_context_t *ptls_mi355x_aesgcm_new_on(int device, const void *key, size_t key_size, size_t capacity);
/* HIP device ordinal the context lives on */
int ptls_mi355x_aesgcm_device(const ptls_mi355x_aesgcm_context_t *ctx);

/* Host-memory, synchronous, one record: output = ciphertext || tag (inlen + 16 bytes). */
int ptls_mi355x_aesgcm_encrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                               const void *nonce12, const void *aad, size_t aadlen);
/* returns 1 if the tag verified (plaintext written), 0 if not (output zeroed), <0 on error */
int ptls_mi355x_aesgcm_decrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                               const void *nonce12, const void *aad, size_t aadlen, const void *tag);

/* AES-ECB encryption of nblocks 16-byte blocks in host memory with the context's key
 * (ptls_fusion_aesecb_encrypt, lib/fusion.c:747-752). */
int ptls_mi355x_aesecb_encrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t nblocks);

/*
 * Round-keys-only AES context: the ECB and CTR cipher objects and header protection (the analogue of
 * ptls_fusion_aesecb_context_t, include/picotls/fusion.h:36-39 / ptls_fusion_aesecb_init, lib/fusion.c:692-740).
 * Holds the encryption schedule and the equivalent-inverse-cipher schedule (FIPS-197 5.3.5) on the device
 * that is current at creation -- 480 bytes, no GHASH tables.
 *   ptls_mi355x_aes_ecb:       host buffers, synchronous (is_enc 0 = decrypt)
 *   ptls_mi355x_aes_ecb_batch: device buffers, asynchronous on `stream`
 */
typedef struct st_ptls_mi355x_aes_context ptls_mi355x_aes_context_t;
ptls_mi355x_aes_context_t *ptls_mi355x_aes_new(const void *key, size_t key_size);
void ptls_mi355x_aes_free(ptls_mi355x_aes_context_t *ctx);
int ptls_mi355x_aes_ecb(ptls_mi355x_aes_context_t *ctx, int is_enc, void *output, const void *input, size_t nblocks);
int ptls_mi355x_aes_ecb_batch(ptls_mi355x_aes_context_t *ctx, int is_enc, uint8_t *dst, const uint8_t *src,
                              size_t nblocks, void *stream);

/* ======================================================================================
 * 3. Batch extension (the hot path).  Seals or opens n independent records in ONE launch.
 *    All buffers are DEVICE pointers on the context's device; `stream` is a hipStream_t
 *    (NULL = the null stream).  The call is asynchronous.
 *
 *    Record i: nonce = static_iv XOR (0^32 || BE64(recs[i].seq))   (lib/picotls.c:5291-5305)
 *      seal: reads src[recs[i].src .. +len), aad[recs[i].aad .. +aadlen);
 *            writes dst[recs[i].dst .. +len+16) = ciphertext || tag
 *      open: reads src[recs[i].src .. +len+16) = ciphertext || tag;
 *            writes dst[recs[i].dst .. +len) = plaintext (zeroed on failure) and
 *            status[i] = len, or 0xffffffff when the tag does not verify
 *    In-place (dst == src with equal offsets) is allowed.  Records may start at any byte
 *    offset; 16-byte aligned starts are the fast path.
 * ====================================================================================== */
typedef struct st_ptls_mi355x_record_t {
    uint64_t src;    /* byte offset of the record's input in the src arena */
    uint64_t dst;    /* byte offset of the record's output in the dst arena */
    uint64_t aad;    /* byte offset of the AAD in the aad arena */
    uint64_t seq;    /* record sequence number */
    uint32_t len;    /* payload bytes (open: ciphertext bytes, tag excluded) */
    uint32_t aadlen; /* AAD bytes */
} ptls_mi355x_record_t;

int ptls_mi355x_seal_batch(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12, const ptls_mi355x_record_t *recs,
                           size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad, void *stream);
int ptls_mi355x_open_batch(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12, const ptls_mi355x_record_t *recs,
                           size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *status, void *stream);

/* Ragged batches: same as above, but record i of the launch is recs[order[i]] (status is still
 * indexed by descriptor).  ptls_mi355x_order_by_length() fills `order` (n device uint32) with the
 * descriptor indices sorted by decreasing work (device radix sort on the stream), so each wave's
 * records have similar lengths and the longest go first (the kernels hand out record groups
 * dynamically).  The order can be reused for the matching open batch. */
int ptls_mi355x_order_by_length(ptls_mi355x_aesgcm_context_t *ctx, const ptls_mi355x_record_t *recs, size_t n,
                                uint32_t *order, void *stream);
int ptls_mi355x_seal_batch_ordered(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                   const ptls_mi355x_record_t *recs, const uint32_t *order, size_t n, const uint8_t *src,
                                   uint8_t *dst, const uint8_t *aad, void *stream);
int ptls_mi355x_open_batch_ordered(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                   const ptls_mi355x_record_t *recs, const uint32_t *order, size_t n, const uint8_t *src,
                                   uint8_t *dst, const uint8_t *aad, uint32_t *status, void *stream);

/*
 * Multi-key batches: the records of many sessions -- each with its own traffic key and static IV (a rapido server's
 * connections, include/rapido.h:147, lib/rapido.c:135-200) -- in ONE launch.  ctxs[k] (k < nkeys) is the context of key
 * k and static_ivs its 12-byte IV at static_ivs + 12 k (host memory); key_idx (n device uint32) the key of each record.
 * Every context must live on ctxs[0]'s device and have its key size; ctxs[0] leads the launch (its scratch holds the key
 * table and the by-key sort, which run on `stream` before the kernel).  Results are those of one single-key call per
 * key.  A record whose key index is >= nkeys is not processed: seal writes nothing, open reports status 0xffffffff with
 * its output untouched (never a record under another key).  Up to a fifth of the CUs' records run on the split window
 * kernels, up to one record per CU on the 16-lane window kernels (each workgroup on its record's key), larger batches
 * on the batch kernels, whose workgroups take one key at a time and move between keys as their groups run out (DESIGN.md
 * section 3, "Multi-key batches").  The context's (and the key table's) upload is skipped when the keys repeat.
 */
int ptls_mi355x_seal_batch_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys,
                                    const ptls_mi355x_record_t *recs, const uint32_t *key_idx, size_t n,
                                    const uint8_t *src, uint8_t *dst, const uint8_t *aad, void *stream);
int ptls_mi355x_open_batch_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys,
                                    const ptls_mi355x_record_t *recs, const uint32_t *key_idx, size_t n,
                                    const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *status, void *stream);
/* The by-key sort once for several launches over the same records (a batch's seal and open): ptls_mi355x_order_by_key
 * fills `order` (n device uint32) with the descriptor indices grouped by key index, keys ascending, out-of-range
 * indices last (within a key the order is unspecified: a device counting sort), on ctx's scratch and `stream`; the
 * _ordered launches take it instead of grouping.  The order must be one of ptls_mi355x_order_by_key's for these key
 * indices. */
int ptls_mi355x_order_by_key(ptls_mi355x_aesgcm_context_t *ctx, const uint32_t *key_idx, size_t n, size_t nkeys,
                             uint32_t *order, void *stream);
int ptls_mi355x_seal_batch_multikey_ordered(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs,
                                            size_t nkeys, const ptls_mi355x_record_t *recs, const uint32_t *key_idx,
                                            const uint32_t *order, size_t n, const uint8_t *src, uint8_t *dst,
                                            const uint8_t *aad, void *stream);
int ptls_mi355x_open_batch_multikey_ordered(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs,
                                            size_t nkeys, const ptls_mi355x_record_t *recs, const uint32_t *key_idx,
                                            const uint32_t *order, size_t n, const uint8_t *src, uint8_t *dst,
                                            const uint8_t *aad, uint32_t *status, void *stream);

/* ======================================================================================
 * 4. TLS 1.3 record framing in the batch.  The framing of picotls's
 *    record layer done by the kernel, so a send window / recv() window of records is ONE launch
 *    instead of per-record ptls_aead_encrypt/decrypt slot calls.
 *
 *    seal -- replaces buffer_push_encrypted_records + aead_encrypt + build_aad
 *            (lib/picotls.c:621-643,658-684) for one record per descriptor:
 *        reads  src[recs[i].src .. +len)                      (the fragment, len <= 16384)
 *        writes dst[recs[i].dst .. +len+22) = 17 03 03 BE16(len+17) || ciphertext(fragment ||
 *               (uint8)type) || tag, AAD = the 5 header bytes, nonce from recs[i].seq
 *    open -- replaces aead_decrypt + the padding strip / content-type pop of handle_input_tls13
 *            (lib/picotls.c:645-654,4779-4791) for one header-framed record per descriptor:
 *        reads  src[recs[i].src .. +5+len) = header || ciphertext || tag, len = the header's
 *               length field (AAD rebuilt as 17 03 03 BE16(len), as build_aad does)
 *        writes dst[recs[i].dst .. +len-16) = plaintext with padding and type, then
 *               status[i] = inner plaintext length and types[i] = content type, or
 *               status[i] = PTLS_MI355X_TLS_BAD_RECORD_MAC (tag, or len < 16; plaintext zeroed)
 *                           PTLS_MI355X_TLS_UNEXPECTED_MESSAGE (no non-zero byte)
 *    A context is used by one host thread at a time (as picotls contexts are); launches may go to any
 *    streams.
 *    Device pointers, asynchronous on `stream`, like section 3.  Headers are parsed and
 *    descriptors planned on the host (ptls_mi355x_tls_plan_send / _parse_records below).
 * ====================================================================================== */
typedef struct st_ptls_mi355x_tls_record_t {
    uint64_t src;  /* seal: fragment offset in src;     open: record (header) offset in src */
    uint64_t dst;  /* seal: record (header) offset in dst; open: plaintext offset in dst */
    uint64_t seq;  /* record sequence number */
    uint32_t len;  /* seal: fragment bytes (<= 16384; a longer one is skipped, nothing written); open: the header's length field */
    uint32_t type; /* seal: inner content type (23 = application_data); open: unused */
} ptls_mi355x_tls_record_t;

#define PTLS_MI355X_TLS_HEADER_SIZE 5
#define PTLS_MI355X_TLS_MAX_FRAGMENT 16384              /* PTLS_MAX_PLAINTEXT_RECORD_SIZE, lib/picotls.c:38 */
#define PTLS_MI355X_TLS_MAX_RECORD (16384 + 256)        /* PTLS_MAX_ENCRYPTED_RECORD_SIZE, lib/picotls.c:39 */
#define PTLS_MI355X_TLS_OVERHEAD (5 + 1 + 16)           /* header + content type + tag */
#define PTLS_MI355X_TLS_BAD_RECORD_MAC 0xffffffffu      /* -> PTLS_ALERT_BAD_RECORD_MAC (20) */
#define PTLS_MI355X_TLS_UNEXPECTED_MESSAGE 0xfffffffeu  /* -> PTLS_ALERT_UNEXPECTED_MESSAGE (10) */
#define PTLS_MI355X_TLS_NOT_PROCESSED 0xfffffffdu       /* behind a failed record (PTLS_MI355X_OPEN_STOP_AT_FAILURE) */

int ptls_mi355x_tls_seal_records(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                 const ptls_mi355x_tls_record_t *recs, size_t n, const uint8_t *src, uint8_t *dst,
                                 void *stream);
int ptls_mi355x_tls_open_records(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                 const ptls_mi355x_tls_record_t *recs, size_t n, const uint8_t *src, uint8_t *dst,
                                 uint32_t *status, uint8_t *types, void *stream);
/* Windows of several TCPLS connections of one session in one launch.  rapido gives every connection
 * the session's key and its own IV: IV bytes 0..3 ^= BE32(connection_id) (derive_connection_aead_iv,
 * lib/rapido.c:127-133; setup_connection_crypto_context :135-200), with a seq per connection.
 * conn_ids[i] (device memory, one per descriptor) is that connection_id for record i; conn_ids == NULL
 * is the single-connection call above. */
int ptls_mi355x_tls_seal_records_multi(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                       const ptls_mi355x_tls_record_t *recs, const uint32_t *conn_ids, size_t n,
                                       const uint8_t *src, uint8_t *dst, void *stream);
int ptls_mi355x_tls_open_records_multi(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                       const ptls_mi355x_tls_record_t *recs, const uint32_t *conn_ids, size_t n,
                                       const uint8_t *src, uint8_t *dst, uint32_t *status, uint8_t *types,
                                       void *stream);

/*
 * picotls stops at the first record that fails and never advances seq past it (aead_decrypt returns
 * PTLS_ALERT_BAD_RECORD_MAC, lib/picotls.c:650-652; an all-zero inner plaintext PTLS_ALERT_UNEXPECTED_MESSAGE,
 * :4790).  The batch open above verifies every record independently.  With PTLS_MI355X_OPEN_STOP_AT_FAILURE,
 * every record behind a failed record OF THE SAME CONNECTION gets status PTLS_MI355X_TLS_NOT_PROCESSED, type 0
 * and a zeroed plaintext slot, so the accepted records are exactly the ones ptls_receive would have delivered
 * before raising the alert.  Connections are runs of equal conn_ids (conn_ids == NULL: one connection); a
 * connection's records must be contiguous and in seq order, as tls_parse_records lays out a recv window.
 * Without the flag the caller must discard the statuses after a connection's first failure itself.
 */
#define PTLS_MI355X_OPEN_STOP_AT_FAILURE 1
int ptls_mi355x_tls_open_records_ex(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                    const ptls_mi355x_tls_record_t *recs, const uint32_t *conn_ids, size_t n,
                                    const uint8_t *src, uint8_t *dst, uint32_t *status, uint8_t *types, int flags,
                                    void *stream);

/*
 * Delivery of opened records: the receive loop of handle_input (lib/picotls.c:4757-4842) over a batch the open kernels
 * verified, on the device.  For each part (one connection's records recs[k0 .. k0 + n) of that launch), the records
 * are taken in order up to the first one whose status is a failure (BAD_RECORD_MAC, UNEXPECTED_MESSAGE,
 * NOT_PROCESSED), whose type is not application_data (23) -- unless any_type, which takes exactly one record of any
 * type -- or whose plaintext would overflow `capacity`; their plaintexts (status[i] bytes at slots + recs[i].dst)
 * are copied back to back to out.  The host reproduces the counts from status / types (the same walk).  Device
 * pointers (out may be a registered host range's device address); asynchronous on stream.  A part may hold at most
 * 4096 records (max_records: the largest n of the parts).  0 or -1.
 */
#define PTLS_MI355X_DELIVER_MAX 4096
typedef struct st_ptls_mi355x_tls_deliver_t {
    const uint8_t *slots;
    uint8_t *out;
    uint64_t capacity;
    uint32_t k0, n, any_type, reserved;
} ptls_mi355x_tls_deliver_t;
int ptls_mi355x_tls_deliver_records(ptls_mi355x_aesgcm_context_t *ctx, const ptls_mi355x_tls_record_t *recs,
                                    const uint32_t *status, const uint8_t *types, const ptls_mi355x_tls_deliver_t *parts,
                                    size_t nparts, size_t max_records, void *stream);

/* Host-side planning (no device access), the loops of the reference record layer:
 *  plan_send: splits len bytes at src_off into <= 16384-byte fragments with consecutive seq
 *    from *seq, records laid out back to back from dst_off (buffer_push_encrypted_records,
 *    lib/picotls.c:664-684).  Returns the number of records (recs may be NULL to count);
 *    *wire_len = bytes the records occupy; *seq advanced past them (unchanged when counting).  Writes at most max.
 *  parse_records: walks the complete records at the start of wire[0..len) (parse_record +
 *    parse_record_header fast path, lib/picotls.c:4243-4268): type 23 records only, one
 *    descriptor each (src = src_off + offset, plaintext slots back to back from dst_off,
 *    consecutive seq from *seq).  Stops before an incomplete record, a record of another
 *    type (left to the caller's slot path) or after max.  *consumed = bytes parsed,
 *    *nrecs = descriptors written.  Returns 0, or PTLS_ALERT_DECODE_ERROR (50) for a length
 *    field above PTLS_MI355X_TLS_MAX_RECORD (parse_record_header :4249-4251). */
size_t ptls_mi355x_tls_plan_send(size_t len, uint32_t type, uint64_t *seq, uint64_t src_off, uint64_t dst_off,
                                 ptls_mi355x_tls_record_t *recs, size_t max, size_t *wire_len);
int ptls_mi355x_tls_parse_records(const uint8_t *wire, size_t len, uint64_t src_off, uint64_t *seq, uint64_t dst_off,
                                  ptls_mi355x_tls_record_t *recs, size_t max, size_t *nrecs, size_t *consumed);

/* ---- 5. batched record layer over host buffers (csrc/record_layer.c) ----
 * One traffic direction of one connection, for an application with its own record layer: picotls hands such an
 * application the traffic secret through its update_traffic_key callback (lib/picotls.c:1206-1211), and rapido
 * derives each connection's key and IV from it (ptls_hkdf_expand_label "key"/"iv", then derive_connection_aead_iv,
 * lib/rapido.c:127-150); INTEGRATION.md section 4 shows the callback.  Each call seals or opens all the records of
 * a whole window in one launch; it returns when the results are in the caller's buffer.  A layer is used by one host
 * thread at a time. */
typedef struct st_ptls_mi355x_record_layer_t ptls_mi355x_record_layer_t;
typedef struct st_ptls_mi355x_iovec_t { /* layout of ptls_iovec_t (include/picotls.h) */
    const uint8_t *base;
    size_t len;
} ptls_mi355x_iovec_t;
/* a layer for key (16 or 32 bytes) and the 12-byte static IV, starting at record sequence number seq; NULL on error
 * (ptls_mi355x_record_layer_last_error) */
ptls_mi355x_record_layer_t *ptls_mi355x_record_layer_new(const void *key, size_t key_size, const void *iv12, uint64_t seq);
void ptls_mi355x_record_layer_free(ptls_mi355x_record_layer_t *rl);
uint64_t ptls_mi355x_record_layer_get_seq(const ptls_mi355x_record_layer_t *rl);
void ptls_mi355x_record_layer_set_seq(ptls_mi355x_record_layer_t *rl, uint64_t seq);
/* ptls_send (lib/picotls.c:4969-4988) for a window: every fragment is framed as records of <= 16384 bytes of inner
 * content type `type` (buffer_push_encrypted_records, :664-684), all sealed in one launch; the records go to out
 * back to back (*outlen bytes, *nrecords records; each record is fragment + 22 bytes) and seq advances past them.
 * A fragment is one ptls_send call: ptls_send forces a key update once seq >= 2^24 (:4976-4977), so an application
 * data fragment (type 23) is sealed only if seq is below PTLS_MI355X_RECORD_LAYER_SEQ_LIMIT when it starts.  The
 * window stops before the first fragment at or past the limit and the call returns
 * PTLS_MI355X_RECORD_LAYER_KEY_UPDATE: the records of the fragments before it are written (*outlen, *nrecords; a
 * fragment of n bytes is max(1, ceil(n / 16384)) records, none when empty), nothing after it.  The caller then sends
 * the KeyUpdate message (type 22, sealed past the limit under the old key, as update_send_key does, :4949-4962),
 * installs the next traffic key (ptls_mi355x_record_layer_rekey: seq restarts at 0) and seals the rest.
 * Returns 0, PTLS_MI355X_RECORD_LAYER_KEY_UPDATE, or -1: a capacity below the wire size (nothing written, seq
 * unchanged), or an engine error (seq unchanged if the launch failed; if the launch was accepted and the wait failed,
 * records may be partly written and seq stays past them, so no nonce is ever used twice). */
#define PTLS_MI355X_RECORD_LAYER_SEQ_LIMIT (1ull << 24)
#define PTLS_MI355X_RECORD_LAYER_KEY_UPDATE 1
int ptls_mi355x_record_layer_seal(ptls_mi355x_record_layer_t *rl, const ptls_mi355x_iovec_t *frags, size_t nfrags,
                                  uint8_t type, void *out, size_t capacity, size_t *outlen, size_t *nrecords);
/* The send windows of several connections -- of one session or of many -- in ONE launch: layers[l] seals
 * frags[l][0..nfrags[l]) into out[l] (capacity[l]) exactly as ptls_mi355x_record_layer_seal would, outlen[l] /
 * nrecords[l] its results, each layer's seq advanced.  Layers sharing the key and IV bytes 4..11 are the connections of
 * one session, whose IVs differ by the connection id in bytes 0..3 (derive_connection_aead_iv, lib/rapido.c:123-133);
 * the kernel applies each record's difference (ptls_mi355x_tls_seal_records_multi).  Layers of different sessions (a
 * server's many connections, each session with its own traffic key, include/rapido.h:147) go into the same launch as
 * a multi-key batch (ptls_mi355x_tls_seal_records_multikey): a session's key is the context of its first layer.  All
 * layers must have one key size.  Runs on layers[0]'s stream and staging; direct when every fragment and output lies
 * in a range registered with any of the layers.  0, or -1: a capacity or another key size (nothing written, no seq
 * advanced), or an engine error (as for ptls_mi355x_record_layer_seal: seq stays past records whose launch was
 * accepted). */
int ptls_mi355x_record_layer_seal_multi(ptls_mi355x_record_layer_t *const *layers, size_t nlayers,
                                        const ptls_mi355x_iovec_t *const *frags, const size_t *nfrags, uint8_t type,
                                        void *const *out, const size_t *capacity, size_t *outlen, size_t *nrecords);
/* ptls_receive / handle_input (lib/picotls.c:4757-4842, 4913-4947) for a window: the complete application_data
 * records at the start of in are opened in one launch; their plaintexts (padding and content type removed) go to out
 * back to back, in order, up to the first record that fails (its alert is returned: 20 BAD_RECORD_MAC, 10
 * UNEXPECTED_MESSAGE; 50 DECODE_ERROR for a bad length field), the first record of another inner content type, an
 * incomplete record or a record of another outer type -- those are left for the caller's picotls path.
 * *consumed = wire bytes of the delivered records, seq advances by *nrecords.  -1: engine error or out too small
 * for the first record. */
int ptls_mi355x_record_layer_open(ptls_mi355x_record_layer_t *rl, const void *in, size_t inlen, size_t *consumed,
                                  void *out, size_t capacity, size_t *outlen, size_t *nrecords);
/* The receive windows of several connections of one session in ONE launch: layers[l] opens in[l][0..inlen[l]) into
 * out[l] (capacity[l]) exactly as ptls_mi355x_record_layer_open would; alerts[l] is what that call would have
 * returned (0, a TLS alert, or -1 for out[l] too small for its first record), consumed[l] / outlen[l] / nrecords[l]
 * its results.  Layers of one or of many sessions, grouped and launched as in ptls_mi355x_record_layer_seal_multi, on
 * the same stream.  0, or -1 (engine error: nothing consumed, no seq advanced). */
int ptls_mi355x_record_layer_open_multi(ptls_mi355x_record_layer_t *const *layers, size_t nlayers, const void *const *in,
                                        const size_t *inlen, size_t *consumed, void *const *out, const size_t *capacity,
                                        size_t *outlen, size_t *nrecords, int *alerts);
/* ptls_receive for ONE record of any inner content type at the start of in (the handshake / alert record a window
 * open stopped at, e.g. a KeyUpdate): its plaintext (padding and type removed) to out, its inner type to
 * *content_type, seq advanced by one.  Returns 0 (*consumed == 0: no complete application_data-framed record), a TLS
 * alert, or -1. */
int ptls_mi355x_record_layer_open_record(ptls_mi355x_record_layer_t *rl, const void *in, size_t inlen, size_t *consumed,
                                         void *out, size_t capacity, size_t *outlen, uint8_t *content_type);
/* a new traffic key for this direction (the update_traffic_key callback of a KeyUpdate epoch change,
 * INTEGRATION.md section 5): key and static IV replaced, seq restarts at 0 (setup_traffic_protection,
 * lib/picotls.c:1217).  No window may be outstanding.  0 or -1. */
int ptls_mi355x_record_layer_rekey(ptls_mi355x_record_layer_t *rl, const void *key, size_t key_size, const void *iv12);
/*
 * Asynchronous windows: a submit plans and stages the window and launches it on the next of the layer's (layers[0]'s)
 * 4 launch slots -- each its own stream, staging and engine context -- and returns at once; so consecutive windows of
 * one connection, and windows of several connections, overlap their PCIe transfers and kernels.  Windows complete in
 * submission order: ptls_mi355x_record_layer_wait(rl, ticket, ...) for the oldest ticket of rl, then the next.  At
 * most 32 windows per layer are outstanding (a 33rd submit returns -1), in at most 4 launches.
 *
 * Coalescing (a single-layer submit, the default): a connection's windows are queued and go out together, ONE launch
 * for a group (as if the layer had been given once per window in one submit), the group being the layer's outstanding
 * windows spread over its 4 launch slots: ceil(outstanding / 4).  So up to 4 windows outstanding every window launches
 * at its submit, as without coalescing; at 16 outstanding, 4 windows per launch, 4 launches in flight.  A queue goes
 * out when its group is complete and a launch slot is free (checked at each submit and wait), when nothing of its
 * layer runs on the GPU, at the first wait for one of its windows, when 16 are queued
 * (ptls_mi355x_record_layer_set_coalesce), or at ptls_mi355x_record_layer_flush.  Tickets, seq and results are those
 * of separate launches.  A synchronous call or a rekey on a layer
 * with windows outstanding -- its own, or another layer's windows that name it -- returns -1.  Buffers (fragments,
 * inputs, outputs) must stay untouched until the window's wait.  Freeing or unregistering a layer that another
 * layer's outstanding window names first waits for the device; that window then completes with alerts[l] =
 * PTLS_MI355X_RECORD_LAYER_STALE for it and delivers nothing to it.
 *
 * A layer may appear several times in one submit: its windows in that order, each behind the one before (one
 * connection's consecutive windows in one launch).
 *  seal_submit: the records take their seq at submit (get_seq includes them).  Its wait gives per layer outlen[l],
 *               nrecords[l], consumed[l] = fragments sealed, alerts[l] = 0 or PTLS_MI355X_RECORD_LAYER_KEY_UPDATE.
 *  open_submit: parsed[l] = the wire bytes of the complete records taken from in[l] (the next window starts behind
 *               them).  The records take the seq that follows the windows in flight before them; their wait gives
 *               what ptls_mi355x_record_layer_open_multi would (consumed[l], outlen[l], nrecords[l], alerts[l]).  When a
 *               window stops before its last parsed record (an alert, another content type, a full output), seq
 *               stays at the stop and every window submitted behind it completes with alerts[l] =
 *               PTLS_MI355X_RECORD_LAYER_STALE, nothing consumed: resubmit from the stop.
 * Returns 0 or -1 (ptls_mi355x_record_layer_last_error).
 */
#define PTLS_MI355X_RECORD_LAYER_STALE (-2)
int ptls_mi355x_record_layer_seal_submit(ptls_mi355x_record_layer_t *const *layers, size_t nlayers,
                                         const ptls_mi355x_iovec_t *const *frags, const size_t *nfrags, uint8_t type,
                                         void *const *out, const size_t *capacity, uint64_t *ticket);
int ptls_mi355x_record_layer_open_submit(ptls_mi355x_record_layer_t *const *layers, size_t nlayers, const void *const *in,
                                         const size_t *inlen, void *const *out, const size_t *capacity, size_t *parsed,
                                         uint64_t *ticket);
int ptls_mi355x_record_layer_wait(ptls_mi355x_record_layer_t *rl, uint64_t ticket, size_t *outlen, size_t *nrecords,
                                  size_t *consumed, int *alerts);
/* windows submitted and not yet waited for (queued or launched) */
size_t ptls_mi355x_record_layer_pending(const ptls_mi355x_record_layer_t *rl);
/* launches the layer's queued windows now (when one of its 4 launch slots is free; else at the next wait); 0 or -1 */
int ptls_mi355x_record_layer_flush(ptls_mi355x_record_layer_t *rl);
/* at most `windows` (<= 16) of a connection's queued windows per launch; 0 or 1: every single-layer window launches at
 * its submit.  Flushes the queue; returns the previous value (default 16). */
size_t ptls_mi355x_record_layer_set_coalesce(ptls_mi355x_record_layer_t *rl, size_t windows);
/* on != 0: single-layer windows queue even while nothing of the layer runs, until the queue holds `coalesce` windows,
 * the first wait for one of them, or cork(rl, 0), which launches them (TCP_CORK for a burst of windows known to
 * follow each other).  0 or -1 (the launch on uncorking failed). */
int ptls_mi355x_record_layer_cork(ptls_mi355x_record_layer_t *rl, int on);
/* launches this layer has led so far (diagnostics: coalesced windows share one) */
uint64_t ptls_mi355x_record_layer_launches(const ptls_mi355x_record_layer_t *rl);
const char *ptls_mi355x_record_layer_last_error(void);
/* How the bytes travel (record_layer.c): a call whose fragments and output (seal), or input and output (open; out
 * at least as large as the records' ciphertexts), all lie in ranges registered below runs DIRECT: read and written in
 * place by the kernels (default; an open's plaintexts are written once, back to back, by the delivery kernel), or by
 * DMA to and from device memory (ptls_mi355x_record_layer_set_direct_dma), no staging copy either way.  Otherwise a window of at most `zero copy bytes` (descriptors, input and
 * output) is copied into the layer's pinned, mapped staging, which the kernel reads and writes over PCIe (one
 * launch, one synchronisation); larger windows move by one H2D and one D2H DMA copy.  Results are identical. */
/* registers host memory [base, base+len) that stays allocated (a connection's socket buffers) for direct calls
 * (hipHostRegister, mapped); up to 8 ranges per layer.  Layers share registrations process-wide: a range inside one
 * a layer registered (the other direction of the connection sharing a buffer, or a part of it) is counted on that
 * mapping, which is unmapped only when the last layer holding it unregisters it or is freed; a range that overlaps a
 * registered one without lying inside it is refused (register the enclosing range first).  A range the application
 * registered itself is used as it is and never unregistered here; it must stay registered while a layer uses it.  0,
 * or -1 (ptls_mi355x_record_layer_last_error). */
int ptls_mi355x_record_layer_register(ptls_mi355x_record_layer_t *rl, void *base, size_t len);
/* unregisters a range given to ptls_mi355x_record_layer_register (by its base); 0 or -1.  The layer unregisters
 * its ranges when freed. */
int ptls_mi355x_record_layer_unregister(ptls_mi355x_record_layer_t *rl, void *base);
/* windows whose buffers are all registered: 0 (default) has the kernels read the inputs in place over PCIe and write
 * the outputs into the registered ranges (a sealed window whose fragments overlap its output goes through the
 * staging instead); 1 moves them by DMA copies between the registered ranges and device memory around a
 * device-resident launch (measured slower: DESIGN.md section 2); PTLS_MI355X_RECORD_LAYER_DMA_IN (2) moves only the
 * inputs (fragments, wire records) to device memory by DMA and writes the outputs in place as 0 does (the fastest
 * open: DESIGN.md section 2).  Results are identical.  Returns the previous value. */
#define PTLS_MI355X_RECORD_LAYER_DMA_IN 2
int ptls_mi355x_record_layer_set_direct_dma(ptls_mi355x_record_layer_t *rl, int on);
/* Once per process and device (the current one): has the HIP runtime set up its copy machinery now -- its first
 * copy of 64 KiB or more, its first copies on four streams at once and each new high of copies in flight stalled
 * that copy 8-30 ms -- instead of inside a later window.  A record layer calls it before its first copy (DMA transports and
 * staged copy windows); a caller may call it at startup.  0, or -1 (ptls_mi355x_last_error). */
int ptls_mi355x_prepare_copies(void);
/* Sets up, now, everything a layer's windows would otherwise create at their first use: the stream and engine context
 * of each of its 4 launch slots (a key setup each), their pinned staging and device buffers sized for
 * `windows_per_launch` windows of up to `window_bytes` each (the wire or fragment bytes of one window), and the HIP
 * copy path (ptls_mi355x_prepare_copies).  A fresh layer's first window on each slot otherwise costs ~3 ms of setup
 * (DESIGN.md section 2); a connection calls this once, after creating its layers.  0, or -1 (windows outstanding, or
 * an allocation failed).  The staging's per-record space (descriptors, statuses, types, 128 B a record) is sized for
 * windows of full-size records (16 KiB fragments, as rapido sends them); the descriptor arrays for the most records
 * an open can parse (window_bytes / 5 + 1).  A window of many small records -- more than window_bytes / 16384 + 2 --
 * still grows a slot's staging once, at its first such window (a one-time stall of ~1-3 ms). */
int ptls_mi355x_record_layer_reserve(ptls_mi355x_record_layer_t *rl, size_t window_bytes, size_t windows_per_launch);
/* zero-copy limit in bytes (default 4 MiB; 0 = always DMA copies); returns the previous value */
size_t ptls_mi355x_record_layer_set_zero_copy_bytes(ptls_mi355x_record_layer_t *rl, size_t n);

/*
 * Multi-key framing (section 3's multi-key batches over section 4's records): the windows of many sessions in one launch,
 * key_idx[i] selecting record i's key and IV, conn_ids[i] (may be NULL) its rapido connection id within that session.
 * With PTLS_MI355X_OPEN_STOP_AT_FAILURE a connection is a (key, connection id) pair: consecutive records of one.
 */
int ptls_mi355x_tls_seal_records_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys,
                                          const ptls_mi355x_tls_record_t *recs, const uint32_t *key_idx,
                                          const uint32_t *conn_ids, size_t n, const uint8_t *src, uint8_t *dst,
                                          void *stream);
int ptls_mi355x_tls_open_records_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys,
                                          const ptls_mi355x_tls_record_t *recs, const uint32_t *key_idx,
                                          const uint32_t *conn_ids, size_t n, const uint8_t *src, uint8_t *dst,
                                          uint32_t *status, uint8_t *types, int flags, void *stream);

/* ---- tuning / introspection ---- */
/* lanes per record used by the batch kernels (1, 2, 4 or 8; default 4); returns the previous value, or -1 */
int ptls_mi355x_set_lanes_per_record(int k);
int ptls_mi355x_get_lanes_per_record(void);
/* framing batches (section 4) of at most n records run on the window kernels, which cut every record into
 * 64-block GHASH segments walked in parallel (latency of rapido-sized windows); larger batches run on the
 * batch kernels (throughput).  Default 16384; returns the previous value.  Results are identical. */
size_t ptls_mi355x_set_tls_window_records(size_t n);
/* the same for the AEAD batch calls (section 3) and the single-record slot calls, which are batches of
 * one: up to n records run on the window kernels.  Default 2048 (1400-B records break even there; 16 KiB
 * records gain up to 16384); returns the previous value. */
size_t ptls_mi355x_set_aead_window_records(size_t n);
/*
 * Single-record slot calls (ptls_mi355x_aesgcm_encrypt/decrypt, the ptls_aead slot) whose staged bytes
 * (64 + AAD + record + tag, 16-byte rounded) are at most n run zero-copy: the kernel reads the record from
 * the context's pinned staging buffer and writes the result back into it over PCIe, with no DMA copies.
 * Larger ones are copied in and out.  Returns the previous value (default 1 MiB).  Process-wide.
 */
size_t ptls_mi355x_set_slot_zero_copy_bytes(size_t n);
/*
 * Window batches (see above) of at most n records -- the slot calls and a few connections' windows -- cut
 * records into 32-position GHASH segments (4 steps of 8 lanes, one record per workgroup) instead of 64:
 * half the walk latency, for a slightly longer join.  SIZE_MAX (the default) means the device's CU count,
 * 0 disables.  Returns the previous value.  Results are identical.
 */
size_t ptls_mi355x_set_seg32_records(size_t n);
/*
 * Window batches of at most n records use the 16-lane single-record kernels instead: 32-position segments
 * walked by 16 lanes in 2 steps, one record per 576-thread workgroup -- the latency
 * kernels of a rapido send window.  Takes precedence over ptls_mi355x_set_seg32_records.
 * SIZE_MAX (the default) means the device's CU count, 0 disables.  Returns the previous value.  Results are
 * identical.
 */
size_t ptls_mi355x_set_win16_records(size_t n);
/*
 * Window batches of at most n records use the split kernels: every record's segments are cut into runs of 8, each
 * walked by its own 128-thread workgroup on its own CU (5 per TLS record), the runs' partial GHASH sums joined by the
 * last to arrive.  The lowest-latency family for a few records (a rapido send window).  Takes precedence over
 * ptls_mi355x_set_win16_records.  SIZE_MAX (the default) means a fifth of the device's CU count, 0 disables.
 * Returns the previous value.  Results are identical.
 */
size_t ptls_mi355x_set_split_records(size_t n);
/*
 * Diagnostics: the batch kernels' work counters are never reset (each launch starts where the previous one
 * on its slot ended, modulo 2^32).  Contexts created after this call start their counters at `origin`
 * instead of 0, so a test can place the 2^32 wrap inside its first launches.  Returns the previous value.
 */
uint32_t ptls_mi355x_set_work_ticket_origin(uint32_t origin);
/* name of the kernel symbol a launch of n records with these parameters uses on the current device (framing:
 * the section-4 entry points) -- the same selection launch_batch makes (for profiling and reports) */
const char *ptls_mi355x_kernel_name(int is_seal, size_t key_size, size_t n, int framing);
/* the same for a multi-key launch (the ptls_mi355x_*_multikey entry points) */
const char *ptls_mi355x_kernel_name_multikey(int is_seal, size_t key_size, size_t n, int framing);
/* LDS table reads (ds_read_b128) per 16-byte block of the batch kernels' GHASH Horner multiply at k lanes per record:
 * 16 with the 8-bit latin tables (k = 4), 32 with the nibble tables; -1 for an invalid k
 * (for the LDS roofline in reports) */
int ptls_mi355x_batch_ghash_reads(int k);
/* last HIP error string seen by the engine ("" if none) */
const char *ptls_mi355x_last_error(void);

/* ---- fault attribution (rapido_amd/csrc/fault_journal.c) ---- */
/*
 * Registers an observer for the GPU's memory-fault events (hsa_amd_register_system_event_handler) and keeps a journal
 * of the engine's last 256 device events: every launch (kernel, stream, grid, pointer arguments with their extents
 * where known), every device allocation and free, every host registration, every device check.  On a fault the
 * handler writes the faulting virtual address, the fault reasons and the journal (ranges holding the address marked)
 * to stderr and appends it to `path` (NULL: stderr only).  It only observes: HIP's own handling of the fault (the
 * sticky hipErrorIllegalAddress) is unchanged.  Call it before the first HIP call where possible.  Returns 0, or the
 * HSA status of hsa_init / the registration (e.g. no GPU).  Calling it again only changes `path`.
 */
int ptls_mi355x_fault_journal_install(const char *path);
int ptls_mi355x_fault_journal_installed(void);
/* memory-fault events the handler has received */
unsigned long ptls_mi355x_fault_journal_faults(void);
/* writes the report the handler writes, for a fault at `va` (diagnostics: a report on demand, and its test) */
void ptls_mi355x_fault_journal_report(uint64_t va, uint32_t reason_mask);
/* records a device memory event over [p, p + len) in the journal (the engine's own allocations are recorded) */
void ptls_mi355x_fault_journal_note(const char *what, const void *p, size_t len);

/* ---- slot error accounting and test hooks ---- */
/* engine errors the AEAD slot's do_decrypt failed closed on: the record was refused as a bad MAC (SIZE_MAX) and its
 * output zeroed, the process kept running (aead_slot.c; do_encrypt has no error return and aborts) */
unsigned long ptls_mi355x_slot_engine_errors(void);
/* test hook: AEAD slot contexts set up while `on` get no engine context, so every engine call of theirs fails (the
 * engine-error path without a GPU).  Returns the previous setting.  Not for production use. */
int ptls_mi355x_test_slot_without_engine(int on);
/* test hook: the next n single-record engine calls (the slot's encrypt / decrypt) fail as a GPU error would.  Returns
 * the previous count.  Not for production use. */
unsigned ptls_mi355x_test_inject_engine_errors(unsigned n);
/*
 * Build provenance: the first 16 hex digits of SHA-256 over the library's sources (rapido_amd/csrc/ and this header,
 * in name order, each as "<name>\0<bytes>"), fixed when the library was built (rapido_amd/build.py).  Equal to
 * rapido_amd.source_build_id() of the tree iff the library was built from that tree's sources.
 */
const char *ptls_mi355x_build_id(void);

#ifdef __cplusplus
}
#endif

#endif /* PTLS_MI355X_H */
