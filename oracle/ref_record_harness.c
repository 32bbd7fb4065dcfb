/*
 * oracle/ref_record_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the engine).
 *
 * Drives the REFERENCE TLS record layer -- picotls.c's ptls_send() / ptls_receive(), compiled
 * unmodified from /root/reference/lib/picotls.c by including it into this translation unit
 * (no source is copied into the repository) -- to produce golden wire records for the batched
 * framing kernels:
 *
 *   send:    buffer_push_encrypted_records (lib/picotls.c:664-684): <= 16384-byte fragments,
 *            header 17 03 03 BE16(len + 17), aead_encrypt (:630-643) appends the content type,
 *            AAD = the header (build_aad :621-628), one seq per record
 *   receive: handle_input_tls13 (:4760-4799): parse_record, aead_decrypt (:645-654), padding
 *            strip + content-type pop, PTLS_ALERT_BAD_RECORD_MAC / PTLS_ALERT_UNEXPECTED_MESSAGE
 *
 * The record layer needs a streaming AEAD (encrypt_init/update/final).  fusion's slot adapter
 * stubs streaming (lib/fusion.c:881-896) and its tags are wrong above ~1500 B,
 * so the AEAD here buffers the record and seals it with the fusion CORE
 * (ptls_fusion_aesgcm_new with capacity = record + AAD, ptls_fusion_aesgcm_encrypt/decrypt),
 * which SURVEY.md 8(c).2 verifies equals standard AES-GCM.
 */
#include "picotls.c" /* -I$(REF)/lib: the reference record layer itself (static functions, struct st_ptls_t) */
#include "picotls/fusion.h"
#include <immintrin.h>

struct rec_aead {
    ptls_aead_context_t super;
    uint8_t key[32];
    uint8_t static_iv[12];
    uint64_t seq;
    uint8_t aad[64];
    size_t aadlen;
    uint8_t *buf;
    size_t len, cap;
};

/* picotls nonce (lib/picotls.c:5291-5305) as the fusion counter block, like calc_counter (lib/fusion.c:898-905) */
static __m128i rec_ctr(const uint8_t static_iv[12], uint64_t seq)
{
    uint8_t iv[16];
    memcpy(iv, static_iv, 12);
    for (int i = 0; i < 8; ++i)
        iv[4 + i] ^= (uint8_t)(seq >> (56 - 8 * i));
    iv[12] = iv[13] = iv[14] = iv[15] = 0; /* low word 0, as calc_counter leaves it */
    __m128i v = _mm_loadu_si128((const __m128i *)iv);
    return _mm_shuffle_epi8(v, _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15));
}

static void rec_encrypt_init(ptls_aead_context_t *_ctx, uint64_t seq, const void *aad, size_t aadlen)
{
    struct rec_aead *ctx = (struct rec_aead *)_ctx;
    assert(aadlen <= sizeof(ctx->aad));
    ctx->seq = seq;
    memcpy(ctx->aad, aad, aadlen);
    ctx->aadlen = aadlen;
    ctx->len = 0;
}

static size_t rec_encrypt_update(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen)
{
    struct rec_aead *ctx = (struct rec_aead *)_ctx;
    (void)output;
    if (ctx->len + inlen > ctx->cap) {
        ctx->cap = (ctx->len + inlen) * 2 + 64;
        ctx->buf = realloc(ctx->buf, ctx->cap);
        assert(ctx->buf != NULL);
    }
    memcpy(ctx->buf + ctx->len, input, inlen);
    ctx->len += inlen;
    return 0; /* everything is emitted by final */
}

static size_t rec_encrypt_final(ptls_aead_context_t *_ctx, void *output)
{
    struct rec_aead *ctx = (struct rec_aead *)_ctx;
    size_t keylen = ctx->super.algo->key_size;
    ptls_fusion_aesgcm_context_t *f = ptls_fusion_aesgcm_new(ctx->key, keylen, ctx->len + ctx->aadlen);
    ptls_fusion_aesgcm_encrypt(f, output, ctx->buf, ctx->len, rec_ctr(ctx->static_iv, ctx->seq), ctx->aad, ctx->aadlen,
                               NULL);
    ptls_fusion_aesgcm_free(f);
    return ctx->len + 16;
}

static size_t rec_decrypt(ptls_aead_context_t *_ctx, void *output, const void *input, size_t inlen, uint64_t seq,
                          const void *aad, size_t aadlen)
{
    struct rec_aead *ctx = (struct rec_aead *)_ctx;
    if (inlen < 16)
        return SIZE_MAX;
    size_t keylen = ctx->super.algo->key_size, len = inlen - 16;
    ptls_fusion_aesgcm_context_t *f = ptls_fusion_aesgcm_new(ctx->key, keylen, len + aadlen);
    int ok = ptls_fusion_aesgcm_decrypt(f, output, input, len, rec_ctr(ctx->static_iv, seq), aad, aadlen,
                                        (const uint8_t *)input + len);
    ptls_fusion_aesgcm_free(f);
    return ok ? len : SIZE_MAX;
}

static void rec_dispose(ptls_aead_context_t *_ctx)
{
    free(((struct rec_aead *)_ctx)->buf);
}

static int rec_setup(ptls_aead_context_t *_ctx, int is_enc, const void *key, const void *iv)
{
    struct rec_aead *ctx = (struct rec_aead *)_ctx;
    (void)is_enc;
    memcpy(ctx->key, key, ctx->super.algo->key_size);
    memcpy(ctx->static_iv, iv, 12);
    ctx->buf = NULL;
    ctx->len = ctx->cap = 0;
    ctx->super.dispose_crypto = rec_dispose;
    ctx->super.do_encrypt_init = rec_encrypt_init;
    ctx->super.do_encrypt_update = rec_encrypt_update;
    ctx->super.do_encrypt_final = rec_encrypt_final;
    ctx->super.do_decrypt = rec_decrypt;
    return 0;
}

static ptls_aead_algorithm_t rec_aes128gcm = {"AES128-GCM", PTLS_AESGCM_CONFIDENTIALITY_LIMIT, PTLS_AESGCM_INTEGRITY_LIMIT,
                                              NULL, NULL, 16, 12, 16, sizeof(struct rec_aead), rec_setup};
static ptls_aead_algorithm_t rec_aes256gcm = {"AES256-GCM", PTLS_AESGCM_CONFIDENTIALITY_LIMIT, PTLS_AESGCM_INTEGRITY_LIMIT,
                                              NULL, NULL, 32, 12, 16, sizeof(struct rec_aead), rec_setup};

static void rec_random(void *buf, size_t len) { memset(buf, 0x5a, len); }
static ptls_context_t rec_context = {rec_random, &ptls_get_time};

static ptls_t *rec_tls(size_t keylen, int is_dec, const uint8_t *key, const uint8_t iv[12], uint64_t seq0)
{
    ptls_t *tls = ptls_server_new(&rec_context);
    tls->state = PTLS_STATE_SERVER_POST_HANDSHAKE; /* keys installed directly, as rapido does per connection */
    struct st_ptls_traffic_protection_t prot = {{0}};
    prot.aead = ptls_aead_new_direct(keylen == 32 ? &rec_aes256gcm : &rec_aes128gcm, !is_dec, key, iv);
    prot.seq = seq0;
    ptls_set_traffic_protection(tls, &prot, is_dec);
    return tls;
}

/*
 * ptls_send(): `len` bytes of application data -> wire records into out[cap].
 * Returns 0 or a picotls error; *outlen = wire bytes, *seq_after = the next sequence number.
 */
int ref_tls_send(const uint8_t *key, size_t keylen, const uint8_t iv[12], uint64_t seq0, const uint8_t *in, size_t len,
                 uint8_t *out, size_t cap, size_t *outlen, uint64_t *seq_after)
{
    ptls_t *tls = rec_tls(keylen, 0, key, iv, seq0);
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, out, cap);
    int ret = ptls_send(tls, &buf, in, len);
    if (ret == 0 && buf.is_allocated)
        ret = PTLS_ERROR_NO_MEMORY; /* caller's buffer too small */
    *outlen = buf.off;
    *seq_after = tls->traffic_protection.enc.seq;
    if (buf.is_allocated) /* dispose also zeroes a caller-owned buffer: only on the error path */
        ptls_buffer_dispose(&buf);
    ptls_free(tls);
    return ret;
}

/*
 * ptls_receive() over a whole wire buffer: every record is decrypted, padding-stripped and
 * appended to out[cap].  Returns 0 or the first error (e.g. PTLS_ALERT_BAD_RECORD_MAC,
 * PTLS_ALERT_UNEXPECTED_MESSAGE); *outlen = plaintext bytes, *consumed = wire bytes consumed
 * before the error, *seq_after = the next sequence number.
 */
int ref_tls_receive(const uint8_t *key, size_t keylen, const uint8_t iv[12], uint64_t seq0, const uint8_t *wire,
                    size_t wirelen, uint8_t *out, size_t cap, size_t *outlen, size_t *consumed, uint64_t *seq_after)
{
    ptls_t *tls = rec_tls(keylen, 1, key, iv, seq0);
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, out, cap);
    size_t off = 0;
    int ret = 0;
    while (off < wirelen) {
        size_t n = wirelen - off;
        if ((ret = ptls_receive(tls, &buf, wire + off, &n)) != 0)
            break;
        off += n;
    }
    if (ret == 0 && buf.is_allocated)
        ret = PTLS_ERROR_NO_MEMORY;
    *outlen = buf.off;
    *consumed = off;
    *seq_after = tls->traffic_protection.dec.seq;
    if (buf.is_allocated) /* dispose also zeroes a caller-owned buffer: only on the error path */
        ptls_buffer_dispose(&buf);
    ptls_free(tls);
    return ret;
}
