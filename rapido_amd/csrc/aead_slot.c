/*
 * aead_slot.c -- picotls AEAD / cipher slot adapter for the MI355X engine (host C).
 *
 * Counterpart of the fusion adapter, lib/fusion.c:822-1005 of the reference:
 *   struct aesgcm_context (lib/fusion.c:68-75)    -> struct mi355x_aead
 *   aesgcm_setup          (lib/fusion.c:942-962)  -> aesgcm_setup
 *   aead_do_encrypt/decrypt (lib/fusion.c:907-932) -> aead_do_encrypt/decrypt
 *   aesgcm_xor_iv         (lib/fusion.c:934-940)  -> aesgcm_xor_iv
 *   streaming stubs       (lib/fusion.c:881-896)  -> implemented (buffering)
 *   ctr cipher            (lib/fusion.c:822-872)  -> struct mi355x_ctr
 *   ecb cipher            (NULL in fusion, lib/fusion.c:990) -> struct mi355x_ecb (t/picotls.c:266-307)
 * Every AES/GHASH computation is done by the HIP engine (gcm_engine.hip); this file only
 * keeps per-context state (static IV, streaming buffer) and maps picotls' arguments onto
 * the engine's record descriptor.  A GPU failure inside a void slot entry point (do_encrypt,
 * the streaming trio, the ciphers) aborts with a message: those ABI entries have no error
 * return, and silently emitting wrong ciphertext is not an option.  do_decrypt has one: an
 * engine error there fails closed -- the output is zeroed and SIZE_MAX returned, which picotls
 * turns into PTLS_ALERT_BAD_RECORD_MAC (lib/picotls.c:645-654) -- so one GPU fault ends the
 * connection it hit, not the process serving every connection.
 */
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../include/ptls_mi355x.h"

#ifndef PTLS_ERROR_NO_MEMORY
#define PTLS_ERROR_NO_MEMORY 0x201 /* include/picotls.h:183 */
#endif
#ifndef PTLS_ERROR_LIBRARY
#define PTLS_ERROR_LIBRARY 0x203 /* include/picotls.h:185 */
#endif
#ifndef PTLS_AESGCM_CONFIDENTIALITY_LIMIT
#define PTLS_AESGCM_CONFIDENTIALITY_LIMIT 0x2000000 /* 2^25, include/picotls.h:80 */
#endif
#ifndef PTLS_AESGCM_INTEGRITY_LIMIT
#define PTLS_AESGCM_INTEGRITY_LIMIT UINT64_C(0x40000000000000) /* 2^54, include/picotls.h:81 */
#endif

#define MI355X_IV_SIZE 12
#define MI355X_TAG_SIZE 16

static void engine_abort(const char *what)
{
    fprintf(stderr, "ptls_mi355x: %s failed: %s\n", what, ptls_mi355x_last_error());
    abort();
}

/* engine errors the slot's decrypt failed closed on (ptls_mi355x_slot_engine_errors) */
static atomic_ulong g_slot_errors;
/* test hook (ptls_mi355x_test_slot_without_engine): slot contexts set up while it is on get no engine context */
static atomic_int g_test_no_engine;

unsigned long ptls_mi355x_slot_engine_errors(void)
{
    return atomic_load(&g_slot_errors);
}

int ptls_mi355x_test_slot_without_engine(int on)
{
    return atomic_exchange(&g_test_no_engine, on != 0);
}

/* ------------------------------------------------------------------------ AES-CTR ------ */

/* both ciphers hold a round-keys-only device context (ptls_mi355x_aes_new), no GHASH tables */
struct mi355x_ctr {
    ptls_cipher_context_t super;
    ptls_mi355x_aes_context_t *aes;
    uint8_t bits[16];
    int is_ready;
};

static void ctr_dispose(ptls_cipher_context_t *_ctx)
{
    struct mi355x_ctr *ctx = (struct mi355x_ctr *)_ctx;
    ptls_mi355x_aes_free(ctx->aes);
    ctx->aes = NULL;
    memset(ctx->bits, 0, sizeof(ctx->bits));
}

/* bits = E_K(iv): one AES-ECB block on the device (lib/fusion.c:843-848) */
static void ctr_init(ptls_cipher_context_t *_ctx, const void *iv)
{
    struct mi355x_ctr *ctx = (struct mi355x_ctr *)_ctx;
    if (ptls_mi355x_aes_ecb(ctx->aes, 1, ctx->bits, iv, 1) != 0)
        engine_abort("aes-ecb");
    ctx->is_ready = 1;
}

/* at most 16 bytes once per init, like fusion (lib/fusion.c:850-862) */
static void ctr_transform(ptls_cipher_context_t *_ctx, void *output, const void *input, size_t len)
{
    struct mi355x_ctr *ctx = (struct mi355x_ctr *)_ctx;
    if (!ctx->is_ready || len > 16) {
        fprintf(stderr, "ptls_mi355x: CTR transform is supported once per init, up to 16 bytes\n");
        abort();
    }
    ctx->is_ready = 0;
    for (size_t i = 0; i < len; ++i)
        ((uint8_t *)output)[i] = ((const uint8_t *)input)[i] ^ ctx->bits[i];
}

static int aesctr_setup(ptls_cipher_context_t *_ctx, const void *key, size_t key_size)
{
    struct mi355x_ctr *ctx = (struct mi355x_ctr *)_ctx;
    ctx->super.do_dispose = ctr_dispose;
    ctx->super.do_init = ctr_init;
    ctx->super.do_transform = ctr_transform;
    ctx->is_ready = 0;
    if ((ctx->aes = ptls_mi355x_aes_new(key, key_size)) == NULL)
        return PTLS_ERROR_LIBRARY;
    return 0;
}

static int aes128ctr_setup(ptls_cipher_context_t *ctx, int is_enc, const void *key)
{
    (void)is_enc;
    return aesctr_setup(ctx, key, 16);
}

static int aes256ctr_setup(ptls_cipher_context_t *ctx, int is_enc, const void *key)
{
    (void)is_enc;
    return aesctr_setup(ctx, key, 32);
}

/* ------------------------------------------------------------------------ AES-ECB ------ */

/*
 * The ECB cipher of the generic suite (t/picotls.c:266-307; ptls_openssl_aes{128,256}ecb, lib/openssl.c:831-838,
 * 1580-1597; cifra's aesecb_setup_crypto, lib/cifra/aes-common.h:55-63): is_enc selects the AES cipher or the
 * inverse cipher, there is no IV, and every transform is len / 16 independent blocks.
 */
struct mi355x_ecb {
    ptls_cipher_context_t super;
    ptls_mi355x_aes_context_t *aes;
    int is_enc;
};

static void ecb_dispose(ptls_cipher_context_t *_ctx)
{
    struct mi355x_ecb *ctx = (struct mi355x_ecb *)_ctx;
    ptls_mi355x_aes_free(ctx->aes);
    ctx->aes = NULL;
}

static void ecb_transform(ptls_cipher_context_t *_ctx, void *output, const void *input, size_t len)
{
    struct mi355x_ecb *ctx = (struct mi355x_ecb *)_ctx;
    if (len % 16 != 0) {
        fprintf(stderr, "ptls_mi355x: ECB transform of %zu bytes (not a multiple of the block size)\n", len);
        abort();
    }
    if (ptls_mi355x_aes_ecb(ctx->aes, ctx->is_enc, output, input, len / 16) != 0)
        engine_abort(ctx->is_enc ? "aes-ecb encrypt" : "aes-ecb decrypt");
}

static int aesecb_setup(ptls_cipher_context_t *_ctx, int is_enc, const void *key, size_t key_size)
{
    struct mi355x_ecb *ctx = (struct mi355x_ecb *)_ctx;
    ctx->super.do_dispose = ecb_dispose;
    ctx->super.do_init = NULL;
    ctx->super.do_transform = ecb_transform;
    ctx->is_enc = is_enc != 0;
    if ((ctx->aes = ptls_mi355x_aes_new(key, key_size)) == NULL)
        return PTLS_ERROR_LIBRARY;
    return 0;
}

static int aes128ecb_setup(ptls_cipher_context_t *ctx, int is_enc, const void *key)
{
    return aesecb_setup(ctx, is_enc, key, 16);
}

static int aes256ecb_setup(ptls_cipher_context_t *ctx, int is_enc, const void *key)
{
    return aesecb_setup(ctx, is_enc, key, 32);
}

/* ------------------------------------------------------------------------ AES-GCM ------ */

struct mi355x_aead {
    ptls_aead_context_t super;
    ptls_mi355x_aesgcm_context_t *engine;
    uint8_t static_iv[MI355X_IV_SIZE];
    /* streaming encryption state (init/update/final) */
    uint64_t s_seq;
    uint8_t *s_aad, *s_buf;
    size_t s_aadlen, s_aadcap, s_len, s_cap;
};

/* nonce = static_iv XOR (0^32 || BE64(seq))   -- ptls_aead__build_iv, lib/picotls.c:5291-5305 */
static void build_nonce(const struct mi355x_aead *ctx, uint64_t seq, uint8_t nonce[MI355X_IV_SIZE])
{
    memcpy(nonce, ctx->static_iv, MI355X_IV_SIZE);
    for (int i = 0; i < 8; ++i)
        nonce[4 + i] ^= (uint8_t)(seq >> (56 - 8 * i));
}

static int reserve(uint8_t **buf, size_t *cap, size_t need)
{
    if (need <= *cap)
        return 0;
    size_t c = *cap ? *cap : 256;
    while (c < need)
        c *= 2;
    uint8_t *p = realloc(*buf, c);
    if (p == NULL)
        return -1;
    *buf = p;
    *cap = c;
    return 0;
}

static void aesgcm_dispose_crypto(ptls_aead_context_t *_ctx)
{
    struct mi355x_aead *ctx = (struct mi355x_aead *)_ctx;
    ptls_mi355x_aesgcm_free(ctx->engine);
    ctx->engine = NULL;
    if (ctx->s_buf) {
        memset(ctx->s_buf, 0, ctx->s_cap);
        free(ctx->s_buf);
    }
    free(ctx->s_aad);
    ctx->s_buf = ctx->s_aad = NULL;
    ctx->s_cap = ctx->s_aadcap = 0;
}

static void aead_do_encrypt(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                            const void *aad, size_t aadlen, ptls_aead_supplementary_encryption_t *supp)
{
    struct mi355x_aead *ctx = (struct mi355x_aead *)_ctx;
    uint8_t nonce[MI355X_IV_SIZE];
    build_nonce(ctx, seq, nonce);
    if (ptls_mi355x_aesgcm_encrypt(ctx->engine, output, input, inlen, nonce, aad, aadlen) != 0)
        engine_abort("seal");
    if (supp != NULL) {
        /* header-protection mask over the written record (lib/fusion.c:472-487) */
        supp->ctx->do_init(supp->ctx, supp->input);
        memset(supp->output, 0, sizeof(supp->output));
        supp->ctx->do_transform(supp->ctx, supp->output, supp->output, sizeof(supp->output));
    }
}

static size_t aead_do_decrypt(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                              const void *aad, size_t aadlen)
{
    struct mi355x_aead *ctx = (struct mi355x_aead *)_ctx;
    uint8_t nonce[MI355X_IV_SIZE];
    if (inlen < MI355X_TAG_SIZE)
        return SIZE_MAX;
    size_t enclen = inlen - MI355X_TAG_SIZE;
    build_nonce(ctx, seq, nonce);
    int ok = ctx->engine != NULL ? ptls_mi355x_aesgcm_decrypt(ctx->engine, output, input, enclen, nonce, aad, aadlen,
                                                              (const uint8_t *)input + enclen)
                                 : -1;
    if (ok < 0) {
        /*
         * Fail closed: nothing of the record is released (the output is zeroed, in place or not) and the record is
         * refused as a bad MAC.  picotls raises PTLS_ALERT_BAD_RECORD_MAC for it and does not advance the receive
         * sequence (lib/picotls.c:645-654, include/picotls.h:1354-1358); the error is printed and counted.
         */
        if (enclen != 0)
            memset(output, 0, enclen);
        atomic_fetch_add(&g_slot_errors, 1);
        fprintf(stderr, "ptls_mi355x: open failed closed (record refused as a bad MAC): %s\n",
                ctx->engine != NULL ? ptls_mi355x_last_error() : "no engine context");
        return SIZE_MAX;
    }
    return ok ? enclen : SIZE_MAX;
}

static void aead_do_encrypt_init(ptls_aead_context_t *_ctx, uint64_t seq, const void *aad, size_t aadlen)
{
    struct mi355x_aead *ctx = (struct mi355x_aead *)_ctx;
    ctx->s_seq = seq;
    ctx->s_len = 0;
    ctx->s_aadlen = 0;
    if (aadlen != 0) {
        if (reserve(&ctx->s_aad, &ctx->s_aadcap, aadlen) != 0)
            engine_abort("streaming init (out of memory)");
        memcpy(ctx->s_aad, aad, aadlen);
        ctx->s_aadlen = aadlen;
    }
}

/* buffers the plaintext; nothing is emitted before final (include/picotls.h:1331-1339 allows it) */
static size_t aead_do_encrypt_update(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen)
{
    struct mi355x_aead *ctx = (struct mi355x_aead *)_ctx;
    (void)output;
    if (inlen == 0)
        return 0;
    if (reserve(&ctx->s_buf, &ctx->s_cap, ctx->s_len + inlen) != 0)
        engine_abort("streaming update (out of memory)");
    memcpy(ctx->s_buf + ctx->s_len, input, inlen);
    ctx->s_len += inlen;
    return 0;
}

/* emits ciphertext || tag for everything buffered since init */
static size_t aead_do_encrypt_final(ptls_aead_context_t *_ctx, void *output)
{
    struct mi355x_aead *ctx = (struct mi355x_aead *)_ctx;
    size_t n = ctx->s_len;
    aead_do_encrypt(_ctx, output, ctx->s_buf, n, ctx->s_seq, ctx->s_aadlen ? ctx->s_aad : NULL, ctx->s_aadlen, NULL);
    if (n)
        memset(ctx->s_buf, 0, n);
    ctx->s_len = 0;
    return n + MI355X_TAG_SIZE;
}

static void aesgcm_xor_iv(ptls_aead_context_t *_ctx, const void *_bytes, size_t len)
{
    struct mi355x_aead *ctx = (struct mi355x_aead *)_ctx;
    const uint8_t *bytes = _bytes;
    if (len > MI355X_IV_SIZE)
        len = MI355X_IV_SIZE;
    for (size_t i = 0; i < len; ++i)
        ctx->static_iv[i] ^= bytes[i];
}

static int aesgcm_setup(ptls_aead_context_t *_ctx, int is_enc, const void *key, const void *iv, size_t key_size)
{
    struct mi355x_aead *ctx = (struct mi355x_aead *)_ctx;
    (void)is_enc; /* both halves are populated, as fusion does (lib/fusion.c:951-957) */

    memcpy(ctx->static_iv, iv, MI355X_IV_SIZE);
    if (key == NULL)
        return 0;

    ctx->super.dispose_crypto = aesgcm_dispose_crypto;
    ctx->super.do_xor_iv = aesgcm_xor_iv;
    ctx->super.do_encrypt_init = aead_do_encrypt_init;
    ctx->super.do_encrypt_update = aead_do_encrypt_update;
    ctx->super.do_encrypt_final = aead_do_encrypt_final;
    ctx->super.do_encrypt = aead_do_encrypt;
    ctx->super.do_decrypt = aead_do_decrypt;
    ctx->s_buf = ctx->s_aad = NULL;
    ctx->s_len = ctx->s_cap = ctx->s_aadlen = ctx->s_aadcap = 0;

    if (atomic_load(&g_test_no_engine)) { /* test hook: a context whose every engine call fails */
        ctx->engine = NULL;
        return 0;
    }
    if ((ctx->engine = ptls_mi355x_aesgcm_new(key, key_size, 1500)) == NULL)
        return PTLS_ERROR_LIBRARY;
    return 0;
}

static int aes128gcm_setup(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv)
{
    return aesgcm_setup(ctx, is_enc, key, iv, 16);
}

static int aes256gcm_setup(ptls_aead_context_t *ctx, int is_enc, const void *key, const void *iv)
{
    return aesgcm_setup(ctx, is_enc, key, iv, 32);
}

/* ------------------------------------------------------------------------ objects ------ */

ptls_cipher_algorithm_t ptls_mi355x_aes128ctr = {"AES128-CTR", 16, 1, 16, sizeof(struct mi355x_ctr), aes128ctr_setup};
ptls_cipher_algorithm_t ptls_mi355x_aes256ctr = {"AES256-CTR", 32, 1, 16, sizeof(struct mi355x_ctr), aes256ctr_setup};
ptls_cipher_algorithm_t ptls_mi355x_aes128ecb = {"AES128-ECB", 16, 16, 0, sizeof(struct mi355x_ecb), aes128ecb_setup};
ptls_cipher_algorithm_t ptls_mi355x_aes256ecb = {"AES256-ECB", 32, 16, 0, sizeof(struct mi355x_ecb), aes256ecb_setup};

ptls_aead_algorithm_t ptls_mi355x_aes128gcm = {"AES128-GCM",
                                               PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                               PTLS_AESGCM_INTEGRITY_LIMIT,
                                               &ptls_mi355x_aes128ctr,
                                               &ptls_mi355x_aes128ecb, /* fusion: NULL (lib/fusion.c:990) */
                                               16,
                                               MI355X_IV_SIZE,
                                               MI355X_TAG_SIZE,
                                               sizeof(struct mi355x_aead),
                                               aes128gcm_setup};

ptls_aead_algorithm_t ptls_mi355x_aes256gcm = {"AES256-GCM",
                                               PTLS_AESGCM_CONFIDENTIALITY_LIMIT,
                                               PTLS_AESGCM_INTEGRITY_LIMIT,
                                               &ptls_mi355x_aes256ctr,
                                               &ptls_mi355x_aes256ecb,
                                               32,
                                               MI355X_IV_SIZE,
                                               MI355X_TAG_SIZE,
                                               sizeof(struct mi355x_aead),
                                               aes256gcm_setup};
