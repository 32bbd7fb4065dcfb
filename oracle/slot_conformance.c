/*
 * oracle/slot_conformance.c -- the MI355X engine driven through the REFERENCE picotls code.
 *
 * TEST INFRASTRUCTURE.  oracle/Makefile links this file with the unmodified reference sources
 * /root/reference/lib/picotls.c (ptls_aead_new_direct, ptls_aead_free) and lib/fusion.c, and with
 * rapido_amd/_lib/libptls_mi355x.so, into oracle/_ref/slot_conformance.  The inline dispatchers
 * (ptls_aead_encrypt, _decrypt, _xor_iv, _encrypt_init/_update/_final, include/picotls.h:1513-1564)
 * are the reference's own.  tests/test_gpu_conformance.py runs it on the GPU box.
 *
 * Checks, TAP style, modelled on the reference's tests:
 *   1. t/fusion.c:99-125  gcm_basic vector through the AEAD slot
 *   2. t/fusion.c:197-231 gcm_iv96 (persistent xor_iv, wrong-IV rejection)
 *   3. t/fusion.c:233-321 test_generated, both directions: engine seal -> fusion open, fusion seal ->
 *      engine open, for AES-128/256 x {plain, iv96}, random key/iv/seq/aad/text < 256 B
 *   4. lib/picotls.c:630-654 record-layer sequence (build_aad, init, update(data), update(type),
 *      final) on the engine, equal to fusion's one-shot encryption of data||type, for TLS lengths
 *   5. t/picotls.c:161-198 test_ciphersuite streaming + tamper detection
 *   6. t/picotls.c:266-321 test_ecb (encrypt, then decrypt with an is_enc = 0 context) for aead->ecb_cipher of
 *      both AEADs, and test_ctr for aead->ctr_cipher
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "picotls.h"
#include "picotls/fusion.h"
#include "ptls_mi355x.h"

static int n_ok, n_fail;
#define CHECK(cond, ...)                                                                                               \
    do {                                                                                                               \
        if (cond) {                                                                                                    \
            ++n_ok;                                                                                                    \
        } else {                                                                                                       \
            ++n_fail;                                                                                                  \
            printf("not ok - ");                                                                                       \
            printf(__VA_ARGS__);                                                                                       \
            printf(" (%s:%d)\n", __FILE__, __LINE__);                                                                  \
        }                                                                                                              \
    } while (0)

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint64_t rnd(void)
{
    rng_state ^= rng_state >> 12;
    rng_state ^= rng_state << 25;
    rng_state ^= rng_state >> 27;
    return rng_state * 0x2545f4914f6cdd1dull;
}
static void rnd_bytes(uint8_t *p, size_t n)
{
    for (size_t i = 0; i < n; ++i)
        p[i] = (uint8_t)rnd();
}

static const uint8_t hello_key[16] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x77,
                                      0x88, 0x99, 0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff};
static const uint8_t hello_text[] = "hello world\nhello world\nhello world\nhello world\nhello world\nhello world\nhello world\n";

static void test_gcm_basic_and_iv96(void)
{
    uint8_t aad[20], iv[12], enc[sizeof(hello_text) + 16], dec[sizeof(hello_text)];
    for (int i = 0; i < 20; ++i)
        aad[i] = (uint8_t)i;
    for (int i = 0; i < 12; ++i)
        iv[i] = (uint8_t)(20 + i);
    /* reference answer computed by fusion in the same process */
    uint8_t want[sizeof(enc)];
    ptls_aead_context_t *f = ptls_aead_new_direct(&ptls_fusion_aes128gcm, 1, hello_key, iv);
    ptls_aead_encrypt(f, want, hello_text, sizeof(hello_text), 0, aad, sizeof(aad));
    ptls_aead_free(f);
    CHECK(want[0] == 0xd3 && want[sizeof(want) - 1] == 0x2f, "fusion reproduces t/fusion.c:110-116");

    ptls_aead_context_t *g = ptls_aead_new_direct(&ptls_mi355x_aes128gcm, 0, hello_key, iv);
    CHECK(g != NULL, "ptls_aead_new_direct(mi355x)");
    ptls_aead_encrypt(g, enc, hello_text, sizeof(hello_text), 0, aad, sizeof(aad));
    CHECK(memcmp(enc, want, sizeof(enc)) == 0, "gcm_basic ciphertext+tag");
    CHECK(ptls_aead_decrypt(g, dec, enc, sizeof(enc), 0, aad, sizeof(aad)) == sizeof(hello_text), "gcm_basic open");
    CHECK(memcmp(dec, hello_text, sizeof(hello_text)) == 0, "gcm_basic plaintext");
    ptls_aead_free(g);

    uint8_t iv2[12] = {20, 20, 20, 20, 24, 25, 26, 27, 28, 29, 30, 31}, seq32[4] = {0, 1, 2, 3}, bad32[4] = {0x89, 0xab, 0xcd, 0xef};
    g = ptls_aead_new_direct(&ptls_mi355x_aes128gcm, 0, hello_key, iv2);
    ptls_aead_xor_iv(g, seq32, sizeof(seq32));
    ptls_aead_encrypt(g, enc, hello_text, sizeof(hello_text), 0, aad, sizeof(aad));
    CHECK(memcmp(enc, want, sizeof(enc)) == 0, "iv96 ciphertext+tag");
    CHECK(ptls_aead_decrypt(g, dec, enc, sizeof(enc), 0, aad, sizeof(aad)) == sizeof(hello_text), "iv96 open");
    ptls_aead_xor_iv(g, seq32, sizeof(seq32));
    ptls_aead_xor_iv(g, bad32, sizeof(bad32));
    CHECK(ptls_aead_decrypt(g, dec, enc, sizeof(enc), 0, aad, sizeof(aad)) == SIZE_MAX, "iv96 wrong IV rejected");
    ptls_aead_xor_iv(g, bad32, sizeof(bad32));
    ptls_aead_xor_iv(g, seq32, sizeof(seq32));
    CHECK(ptls_aead_decrypt(g, dec, enc, sizeof(enc), 0, aad, sizeof(aad)) == sizeof(hello_text), "iv96 no side effect");
    ptls_aead_free(g);
}

static void test_generated(int aes256, int iv96, int runs)
{
    ptls_aead_algorithm_t *ours = aes256 ? &ptls_mi355x_aes256gcm : &ptls_mi355x_aes128gcm;
    ptls_aead_algorithm_t *theirs = aes256 ? &ptls_fusion_aes256gcm : &ptls_fusion_aes128gcm;
    int bad = 0;
    for (int i = 0; i < runs && bad < 5; ++i) {
        uint8_t key[32], iv[12], seq32[4], aad[256], text[256], e1[272], e2[272], d[256];
        rnd_bytes(key, sizeof(key));
        rnd_bytes(iv, sizeof(iv));
        rnd_bytes(seq32, sizeof(seq32));
        size_t aadlen = rnd() % 256, textlen = rnd() % 256;
        uint64_t seq = rnd();
        rnd_bytes(aad, sizeof(aad));
        rnd_bytes(text, sizeof(text));
        ptls_aead_context_t *g = ptls_aead_new_direct(ours, 1, key, iv), *f = ptls_aead_new_direct(theirs, 1, key, iv);
        if (iv96) {
            ptls_aead_xor_iv(g, seq32, sizeof(seq32));
            ptls_aead_xor_iv(f, seq32, sizeof(seq32));
        }
        ptls_aead_encrypt(g, e1, text, textlen, seq, aad, aadlen);
        ptls_aead_encrypt(f, e2, text, textlen, seq, aad, aadlen);
        int ok = memcmp(e1, e2, textlen + 16) == 0;
        ok &= ptls_aead_decrypt(f, d, e1, textlen + 16, seq, aad, aadlen) == textlen && memcmp(d, text, textlen) == 0;
        ok &= ptls_aead_decrypt(g, d, e2, textlen + 16, seq, aad, aadlen) == textlen && memcmp(d, text, textlen) == 0;
        e2[rnd() % (textlen + 16)] ^= (uint8_t)(1u << (rnd() % 8));
        ok &= ptls_aead_decrypt(g, d, e2, textlen + 16, seq, aad, aadlen) == SIZE_MAX;
        ptls_aead_free(g);
        ptls_aead_free(f);
        if (!ok)
            ++bad;
        CHECK(ok, "generated aes%d iv96=%d case %d (aad %zu, text %zu)", aes256 ? 256 : 128, iv96, i, aadlen, textlen);
    }
}

/* lib/picotls.c:621-643 build_aad + aead_encrypt, against fusion sealing data||type in one call */
static void test_record_layer_sequence(int aes256)
{
    ptls_aead_algorithm_t *ours = aes256 ? &ptls_mi355x_aes256gcm : &ptls_mi355x_aes128gcm;
    ptls_aead_algorithm_t *theirs = aes256 ? &ptls_fusion_aes256gcm : &ptls_fusion_aes128gcm;
    static const size_t lens[] = {0, 1, 15, 16, 17, 100, 1000, 1400};
    uint8_t key[32], iv[12];
    rnd_bytes(key, sizeof(key));
    rnd_bytes(iv, sizeof(iv));
    ptls_aead_context_t *g = ptls_aead_new_direct(ours, 1, key, iv), *f = ptls_aead_new_direct(theirs, 1, key, iv);
    static uint8_t data[1401], inner[1402], out[1500], want[1500], dec[1500];
    for (size_t k = 0; k < sizeof(lens) / sizeof(lens[0]); ++k) {
        size_t inlen = lens[k];
        uint64_t seq = 1000 + k;
        uint8_t type = 0x17, aad[5];
        size_t reclen = inlen + 1 + 16;
        aad[0] = 0x17, aad[1] = 0x03, aad[2] = 0x03, aad[3] = (uint8_t)(reclen >> 8), aad[4] = (uint8_t)reclen;
        rnd_bytes(data, inlen);
        size_t off = 0;
        ptls_aead_encrypt_init(g, seq, aad, sizeof(aad));
        off += ptls_aead_encrypt_update(g, out + off, data, inlen);
        off += ptls_aead_encrypt_update(g, out + off, &type, 1);
        off += ptls_aead_encrypt_final(g, out + off);
        memcpy(inner, data, inlen);
        inner[inlen] = type;
        ptls_aead_encrypt(f, want, inner, inlen + 1, seq, aad, sizeof(aad));
        CHECK(off == reclen && memcmp(out, want, reclen) == 0, "record layer seal, aes%d, %zu B", aes256 ? 256 : 128, inlen);
        CHECK(ptls_aead_decrypt(f, dec, out, reclen, seq, aad, sizeof(aad)) == inlen + 1, "fusion opens engine record");
        CHECK(ptls_aead_decrypt(g, dec, want, reclen, seq, aad, sizeof(aad)) == inlen + 1 && memcmp(dec, inner, inlen + 1) == 0,
              "engine opens fusion record");
    }
    ptls_aead_free(g);
    ptls_aead_free(f);
}

/* t/picotls.c:161-198 test_ciphersuite (with a direct key instead of HKDF from a traffic secret) */
static void test_ciphersuite_streaming(ptls_aead_algorithm_t *algo)
{
    const char *src1 = "hello world", *src2 = "good bye, all";
    uint8_t key[32], iv[12];
    char enc1[256], enc2[256], dec1[256], dec2[256];
    size_t enc1len, enc2len, dec1len, dec2len;
    rnd_bytes(key, sizeof(key));
    rnd_bytes(iv, sizeof(iv));
    ptls_aead_context_t *c = ptls_aead_new_direct(algo, 1, key, iv);
    ptls_aead_encrypt_init(c, 0, NULL, 0);
    enc1len = ptls_aead_encrypt_update(c, enc1, src1, strlen(src1));
    enc1len += ptls_aead_encrypt_final(c, enc1 + enc1len);
    ptls_aead_encrypt_init(c, 1, NULL, 0);
    enc2len = ptls_aead_encrypt_update(c, enc2, src2, strlen(src2));
    enc2len += ptls_aead_encrypt_final(c, enc2 + enc2len);
    ptls_aead_free(c);
    c = ptls_aead_new_direct(algo, 0, key, iv);
    dec1len = ptls_aead_decrypt(c, dec1, enc1, enc1len, 0, NULL, 0);
    CHECK(dec1len == strlen(src1) && memcmp(src1, dec1, dec1len) == 0, "ciphersuite 1");
    dec2len = ptls_aead_decrypt(c, dec2, enc2, enc2len, 1, NULL, 0);
    CHECK(dec2len == strlen(src2) && memcmp(src2, dec2, dec2len) == 0, "ciphersuite 2");
    enc1[0] ^= 1;
    CHECK(ptls_aead_decrypt(c, dec1, enc1, enc1len, 0, NULL, 0) == SIZE_MAX, "ciphersuite tamper");
    ptls_aead_free(c);
}

/*
 * t/picotls.c:266-307 test_ecb through aead->ecb_cipher, with the reference's ptls_cipher_new / ptls_cipher_free
 * (lib/picotls.c) and ptls_cipher_encrypt dispatcher: FIPS-197 C.1 / C.3 encryption, then decryption in place with
 * a context made with is_enc = 0.  Plus a 64-block buffer against fusion's ECB encryption, and back.
 */
static void test_ecb_cipher(ptls_aead_algorithm_t *aead, const char *expected_hex)
{
    static const uint8_t fips_pt[16] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x66, 0x77,
                                        0x88, 0x99, 0xaa, 0xbb, 0xcc, 0xdd, 0xee, 0xff};
    uint8_t key[32], expected[16], actual[16];
    for (int i = 0; i < 32; ++i)
        key[i] = (uint8_t)i;
    for (int i = 0; i < 16; ++i)
        sscanf(expected_hex + 2 * i, "%2hhx", &expected[i]);
    ptls_cipher_algorithm_t *algo = aead->ecb_cipher;
    CHECK(algo != NULL, "%s has an ecb_cipher", aead->name);
    if (algo == NULL)
        return;
    ptls_cipher_context_t *c = ptls_cipher_new(algo, 1, key);
    CHECK(c != NULL, "ptls_cipher_new(ecb, enc)");
    memset(actual, 0, sizeof(actual));
    ptls_cipher_encrypt(c, actual, fips_pt, sizeof(actual));
    ptls_cipher_free(c);
    CHECK(memcmp(actual, expected, 16) == 0, "%s ecb encrypt (FIPS-197)", algo->name);
    c = ptls_cipher_new(algo, 0, key);
    ptls_cipher_encrypt(c, actual, actual, sizeof(actual));
    ptls_cipher_free(c);
    CHECK(memcmp(actual, fips_pt, 16) == 0, "%s ecb decrypt back to the plaintext", algo->name);

    uint8_t buf[64 * 16], enc[64 * 16], want[64 * 16];
    rnd_bytes(key, sizeof(key));
    rnd_bytes(buf, sizeof(buf));
    ptls_fusion_aesecb_context_t f;
    ptls_fusion_aesecb_init(&f, 1, key, algo->key_size);
    for (int b = 0; b < 64; ++b)
        ptls_fusion_aesecb_encrypt(&f, want + 16 * b, buf + 16 * b);
    ptls_fusion_aesecb_dispose(&f);
    c = ptls_cipher_new(algo, 1, key);
    ptls_cipher_encrypt(c, enc, buf, sizeof(buf));
    ptls_cipher_free(c);
    CHECK(memcmp(enc, want, sizeof(enc)) == 0, "%s ecb 64 blocks vs fusion", algo->name);
    c = ptls_cipher_new(algo, 0, key);
    ptls_cipher_encrypt(c, enc, enc, sizeof(enc));
    ptls_cipher_free(c);
    CHECK(memcmp(enc, buf, sizeof(enc)) == 0, "%s ecb 64 blocks decrypt", algo->name);
}

/* t/picotls.c:309-321 test_ctr through aead->ctr_cipher: AES128-CTR keystream of 16 zero bytes */
static void test_ctr_cipher(void)
{
    static const uint8_t key[16] = {0x2b, 0x7e, 0x15, 0x16, 0x28, 0xae, 0xd2, 0xa6, 0xab, 0xf7, 0x15, 0x88, 0x09, 0xcf, 0x4f, 0x3c},
                         iv[16] = {0x6b, 0xc1, 0xbe, 0xe2, 0x2e, 0x40, 0x9f, 0x96, 0xe9, 0x3d, 0x7e, 0x11, 0x73, 0x93, 0x17, 0x2a},
                         expected[16] = {0x3a, 0xd7, 0x7b, 0xb4, 0x0d, 0x7a, 0x36, 0x60,
                                         0xa8, 0x9e, 0xca, 0xf3, 0x24, 0x66, 0xef, 0x97};
    static const uint8_t zeroes[16] = {0};
    uint8_t buf[16];
    ptls_cipher_algorithm_t *algo = ptls_mi355x_aes128gcm.ctr_cipher;
    CHECK(algo->key_size == 16 && algo->iv_size == 16, "ctr cipher sizes");
    ptls_cipher_context_t *c = ptls_cipher_new(algo, 1, key);
    ptls_cipher_init(c, iv);
    ptls_cipher_encrypt(c, buf, zeroes, sizeof(buf));
    ptls_cipher_free(c);
    CHECK(memcmp(buf, expected, 16) == 0, "aes128ctr KAT");
}

int main(int argc, char **argv)
{
    int runs = argc > 1 ? atoi(argv[1]) : 1000;
    if (!ptls_mi355x_is_supported()) {
        printf("Bail out! no gfx950 device\n");
        return 2;
    }
    if (!ptls_fusion_is_supported_by_cpu()) {
        printf("Bail out! host CPU lacks AES-NI/PCLMUL/AVX2 (fusion cannot run)\n");
        return 3;
    }
    test_gcm_basic_and_iv96();
    for (int a = 0; a < 2; ++a)
        for (int v = 0; v < 2; ++v)
            test_generated(a, v, runs);
    test_record_layer_sequence(0);
    test_record_layer_sequence(1);
    test_ciphersuite_streaming(&ptls_mi355x_aes128gcm);
    test_ciphersuite_streaming(&ptls_mi355x_aes256gcm);
    test_ecb_cipher(&ptls_mi355x_aes128gcm, "69c4e0d86a7b0430d8cdb78070b4c55a");
    test_ecb_cipher(&ptls_mi355x_aes256gcm, "8ea2b7ca516745bfeafc49904b496089");
    test_ctr_cipher();
    printf("%d ok, %d failed\n", n_ok, n_fail);
    return n_fail ? 1 : 0;
}
