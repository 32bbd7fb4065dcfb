/*
 * oracle/ref_fusion_harness.c -- thin C driver around the REFERENCE engine.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY.  oracle/Makefile compiles this file
 * together with the unmodified reference sources /root/reference/lib/fusion.c
 * and /root/reference/lib/picotls.c (exactly as they lie there, built with the
 * flags of CMakeLists.txt:158: -mavx2 -maes -mpclmul) into oracle/_ref/, which
 * is git-ignored.  It is used
 *   - by tests/golden/gen_golden.py to produce golden vectors from the
 *     reference itself (run in the container that has /root/reference);
 *   - by tests/ to cross-check the CPU oracle against the reference;
 *   - by bench.py's cpu_baseline leg (cpu_baseline.kind = "reference"), which
 *     times lib/fusion.c with the t/ptlsbench.c methodology (t/ptlsbench.c:80-175).
 * Nothing in rapido_amd/ links or loads it.
 *
 * Counter construction follows calc_counter (lib/fusion.c:898-905): the 12-byte
 * nonce is byte-swapped into the upper 96 bits of an __m128i; the engine inserts
 * the 32-bit block counter itself (lib/fusion.c:312-314).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <pthread.h>
#include <immintrin.h>
#include "picotls.h"
#include "picotls/fusion.h"
#include "aes.h" /* deps/cifra/src/aes.h: the reference's minicrypto AES (ECB decrypt, lib/cifra/aes-common.h:48-53) */

static __m128i nonce_to_ctr(const uint8_t iv[12])
{
    uint8_t buf[16] = {0};
    memcpy(buf, iv, 12);
    const __m128i bswap = _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    return _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)buf), bswap);
}

int ref_supported(void) { return ptls_fusion_is_supported_by_cpu(); }

/* direct core API with capacity >= record (SURVEY sec. 8(c) finding 2): standard AES-GCM */
int ref_seal(const uint8_t *key, size_t keylen, const uint8_t iv[12], const uint8_t *aad, size_t aadlen, const uint8_t *in,
             size_t len, uint8_t *out)
{
    ptls_fusion_aesgcm_context_t *ctx = ptls_fusion_aesgcm_new(key, keylen, len + aadlen);
    if (ctx == NULL)
        return -1;
    ptls_fusion_aesgcm_encrypt(ctx, out, in, len, nonce_to_ctr(iv), aad, aadlen, NULL);
    ptls_fusion_aesgcm_free(ctx);
    return 0;
}

/* returns 1 when the tag verifies (plaintext written either way, lib/fusion.c:497-679) */
int ref_open(const uint8_t *key, size_t keylen, const uint8_t iv[12], const uint8_t *aad, size_t aadlen, const uint8_t *in,
             size_t len, const uint8_t *tag, uint8_t *out)
{
    ptls_fusion_aesgcm_context_t *ctx = ptls_fusion_aesgcm_new(key, keylen, len + aadlen);
    if (ctx == NULL)
        return -1;
    int ok = ptls_fusion_aesgcm_decrypt(ctx, out, in, len, nonce_to_ctr(iv), aad, aadlen, tag);
    ptls_fusion_aesgcm_free(ctx);
    return ok;
}

/* seal with a supplementary AES-CTR context keyed by supp_key (QUIC header protection sample) */
int ref_seal_supp(const uint8_t *key, size_t keylen, const uint8_t iv[12], const uint8_t *aad, size_t aadlen,
                  const uint8_t *in, size_t len, uint8_t *out, const uint8_t *supp_key, size_t supp_off, uint8_t supp_out[16])
{
    ptls_fusion_aesgcm_context_t *ctx = ptls_fusion_aesgcm_new(key, keylen, len + aadlen);
    ptls_aead_supplementary_encryption_t supp;
    supp.ctx = ptls_cipher_new(keylen == 32 ? &ptls_fusion_aes256ctr : &ptls_fusion_aes128ctr, 1, supp_key);
    supp.input = out + supp_off;
    ptls_fusion_aesgcm_encrypt(ctx, out, in, len, nonce_to_ctr(iv), aad, aadlen, &supp);
    memcpy(supp_out, supp.output, 16);
    ptls_cipher_free(supp.ctx);
    ptls_fusion_aesgcm_free(ctx);
    return 0;
}

/* through the AEAD slot exactly as ptlsbench / the record layer call it (valid below the 96-entry capacity) */
int ref_slot_seal(const uint8_t *key, size_t keylen, const uint8_t static_iv[12], const uint8_t *xor_iv, size_t xor_len,
                  uint64_t seq, const uint8_t *aad, size_t aadlen, const uint8_t *in, size_t len, uint8_t *out)
{
    ptls_aead_context_t *c = ptls_aead_new_direct(keylen == 32 ? &ptls_fusion_aes256gcm : &ptls_fusion_aes128gcm, 1, key, static_iv);
    if (c == NULL)
        return -1;
    if (xor_len != 0)
        ptls_aead_xor_iv(c, xor_iv, xor_len);
    ptls_aead_encrypt(c, out, in, len, seq, aad, aadlen);
    ptls_aead_free(c);
    return 0;
}

size_t ref_slot_open(const uint8_t *key, size_t keylen, const uint8_t static_iv[12], const uint8_t *xor_iv, size_t xor_len,
                     uint64_t seq, const uint8_t *aad, size_t aadlen, const uint8_t *in, size_t inlen, uint8_t *out)
{
    ptls_aead_context_t *c = ptls_aead_new_direct(keylen == 32 ? &ptls_fusion_aes256gcm : &ptls_fusion_aes128gcm, 0, key, static_iv);
    if (c == NULL)
        return SIZE_MAX;
    if (xor_len != 0)
        ptls_aead_xor_iv(c, xor_iv, xor_len);
    size_t r = ptls_aead_decrypt(c, out, in, inlen, seq, aad, aadlen);
    ptls_aead_free(c);
    return r;
}

int ref_ecb(const uint8_t *key, size_t keylen, const uint8_t in[16], uint8_t out[16])
{
    ptls_fusion_aesecb_context_t ecb;
    ptls_fusion_aesecb_init(&ecb, 1, key, keylen);
    ptls_fusion_aesecb_encrypt(&ecb, out, in);
    ptls_fusion_aesecb_dispose(&ecb);
    return 0;
}

/*
 * AES-ECB decryption of the reference's minicrypto binding (aesecb_decrypt, lib/cifra/aes-common.h:48-53:
 * cf_aes_init + cf_aes_decrypt of the vendored deps/cifra/src/aes.c, compiled from where it lies) -- fusion
 * has no decryption; this pins the oracle's InvCipher to reference code.
 */
int ref_ecb_decrypt(const uint8_t *key, size_t keylen, const uint8_t in[16], uint8_t out[16])
{
    cf_aes_context aes;
    cf_aes_init(&aes, key, keylen);
    cf_aes_decrypt(&aes, in, out);
    cf_aes_finish(&aes);
    return 0;
}

/* ------------------------------------------------------------------------------------------------
 * CPU baseline: t/ptlsbench.c methodology (t/ptlsbench.c:80-175) on N threads.
 * Each thread owns its contexts (fusion contexts are not thread-safe), seals
 * batches of 1000 records (seq = record counter, the AAD carries the seq as ptlsbench's h[] does)
 * and then opens them.  Output buffers are pre-faulted (ptlsbench times first-touch faults,
 * t/ptlsbench.c:101-106).  For records above fusion's slot capacity (lib/fusion.c:808, SURVEY
 * sec. 8(c).1) the direct core API is used with capacity = len + aad so the tags are valid.
 * ---------------------------------------------------------------------------------------------- */
#define BENCH_BATCH 1000

typedef struct {
    size_t keylen, len, aadlen, nrec;
    double seal_s, open_s;
    uint64_t checksum;
    int failed;
} bench_job_t;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *bench_worker(void *arg)
{
    bench_job_t *j = arg;
    uint8_t key[32], iv[12];
    memset(key, 'z', sizeof(key));
    memset(iv, 'y', sizeof(iv));
    ptls_fusion_aesgcm_context_t *ctx = ptls_fusion_aesgcm_new(key, j->keylen, j->len + j->aadlen);
    __m128i ctr0 = nonce_to_ctr(iv);
    uint8_t *v_in = calloc(1, j->len + 16), *v_dec = calloc(1, j->len + 16);
    uint8_t **v_enc = calloc(BENCH_BATCH, sizeof(*v_enc));
    uint8_t aad[64] = {0};
    for (int i = 0; i < BENCH_BATCH; ++i) {
        v_enc[i] = malloc(j->len + 16);
        memset(v_enc[i], 0, j->len + 16);
    }
    for (size_t k = 0; k < j->nrec;) {
        size_t imax = j->nrec - k < BENCH_BATCH ? j->nrec - k : BENCH_BATCH;
        double t0 = now_s();
        for (size_t i = 0; i < imax; ++i) {
            uint64_t seq = k + i + 1;
            memcpy(aad, &seq, sizeof(seq));
            __m128i ctr = _mm_xor_si128(ctr0, _mm_slli_si128(_mm_insert_epi64(_mm_setzero_si128(), (long long)seq, 0), 4));
            ptls_fusion_aesgcm_encrypt(ctx, v_enc[i], v_in, j->len, ctr, aad, j->aadlen, NULL);
            j->checksum += v_enc[i][j->len];
        }
        double t1 = now_s();
        for (size_t i = 0; i < imax; ++i) {
            uint64_t seq = k + i + 1;
            memcpy(aad, &seq, sizeof(seq));
            __m128i ctr = _mm_xor_si128(ctr0, _mm_slli_si128(_mm_insert_epi64(_mm_setzero_si128(), (long long)seq, 0), 4));
            if (!ptls_fusion_aesgcm_decrypt(ctx, v_dec, v_enc[i], j->len, ctr, aad, j->aadlen, v_enc[i] + j->len))
                j->failed = 1;
            j->checksum += v_dec[0];
        }
        double t2 = now_s();
        j->seal_s += t1 - t0;
        j->open_s += t2 - t1;
        k += imax;
    }
    for (int i = 0; i < BENCH_BATCH; ++i)
        free(v_enc[i]);
    free(v_enc);
    free(v_in);
    free(v_dec);
    ptls_fusion_aesgcm_free(ctx);
    return NULL;
}

/*
 * Runs nthreads workers, each sealing+opening nrec_per_thread records of len bytes.
 * out[0] = aggregate seal bytes/s, out[1] = aggregate open bytes/s (each = sum over threads of
 * payload / that thread's own seal (resp. open) time), out[2] = wall seconds, out[3] = failures.
 */
int ref_bench(size_t keylen, size_t len, size_t aadlen, size_t nrec_per_thread, int nthreads, double out[4])
{
    if (nthreads < 1 || nthreads > 256 || aadlen > 64)
        return -1;
    pthread_t th[256];
    bench_job_t jobs[256];
    double t0 = now_s();
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (bench_job_t){keylen, len, aadlen, nrec_per_thread, 0, 0, 0, 0};
        pthread_create(&th[t], NULL, bench_worker, &jobs[t]);
    }
    double seal_bps = 0, open_bps = 0;
    int failed = 0;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        seal_bps += (double)len * nrec_per_thread / jobs[t].seal_s;
        open_bps += (double)len * nrec_per_thread / jobs[t].open_s;
        failed |= jobs[t].failed;
    }
    out[0] = seal_bps;
    out[1] = open_bps;
    out[2] = now_s() - t0;
    out[3] = failed;
    return 0;
}
