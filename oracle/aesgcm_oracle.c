/*
 * oracle/aesgcm_oracle.c -- CPU restatement of AES-GCM for the parity tests.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in rapido_amd/ links, loads or calls this
 * file: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * use it, and only as the checker.  The product path is the HIP engine.
 *
 * What it restates (reference = mpiraux/rapido @ 2024-08-07):
 *   - AES-128/256 block encryption and key expansion; the reference computes the
 *     same function with AES-NI in lib/fusion.c:187-197 (aesecb_encrypt) and
 *     lib/fusion.c:681-740 (ptls_fusion_aesecb_init / expand_key).  Written here
 *     from FIPS-197 sec. 5.1-5.2 (byte oriented, no tables except the S-box,
 *     which is itself derived from the GF(2^8) inverse + affine map).
 *   - AES-128/256 block decryption (FIPS-197 sec. 5.3 InvCipher), the inverse of the
 *     ECB cipher the generic suite needs (t/picotls.c:266-307: encrypt, then decrypt back).
 *   - GHASH and GCM with a 96-bit IV; reference: ptls_fusion_aesgcm_encrypt /
 *     _decrypt (lib/fusion.c:239-679), structured as in NIST SP 800-38D
 *     (Algorithm 1 for the multiply, Algorithm 4/5 for seal/open) -- the same
 *     structure as deps/cifra/src/gcm.c:105-249 and deps/cifra/src/gf128.c:82-114.
 *   - The picotls nonce rule nonce = static_iv XOR (0^32 || BE64(seq))
 *     (lib/picotls.c:5291-5305, ptls_aead__build_iv), the fusion counter block
 *     built by calc_counter (lib/fusion.c:898-905) and the persistent XOR of
 *     leading IV bytes (aesgcm_xor_iv, lib/fusion.c:934-940).
 *   - The AEAD slot conventions: seal writes len+16 bytes with the tag last
 *     (lib/fusion.c:470); open returns the plaintext length or SIZE_MAX on a bad
 *     tag or inlen < 16 (lib/fusion.c:917-932, include/picotls.h:1354-1358).
 *
 * Parity status: pinned.  tests/test_oracle.py checks this file against every
 * known-answer vector of t/fusion.c (ECB, gcm_basic, gcm_capacity, the 18
 * gcm_test_vectors tags + supp outputs, gcm_iv96), the McGrew-Viega GCM cases
 * 1-4 of deps/cifra/src/testmodes.c:395-505, the ECB/CTR KATs of
 * t/picotls.c:266-330, and random vectors produced by the reference's own
 * lib/fusion.c built from /root/reference (tests/golden/gen_golden.py).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

/* ---------------------------------------------------------------- AES ----- */

static uint8_t sbox[256];
static int sbox_ready;

static uint8_t gf8_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1)
            r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

static uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }

static void build_sbox(void)
{
    /* FIPS-197 sec. 5.1.1: multiplicative inverse in GF(2^8), then the affine map */
    for (int x = 0; x < 256; ++x) {
        uint8_t inv = 0;
        if (x != 0)
            for (int y = 1; y < 256; ++y)
                if (gf8_mul((uint8_t)x, (uint8_t)y) == 1) {
                    inv = (uint8_t)y;
                    break;
                }
        sbox[x] = (uint8_t)(inv ^ rotl8(inv, 1) ^ rotl8(inv, 2) ^ rotl8(inv, 3) ^ rotl8(inv, 4) ^ 0x63);
    }
    sbox_ready = 1;
}

typedef struct {
    uint8_t rk[15][16];
    int rounds;
} oracle_aes_t;

/* FIPS-197 sec. 5.2 KeyExpansion (Nk = 4 or 8). */
static int aes_expand(oracle_aes_t *a, const uint8_t *key, size_t keylen)
{
    if (!sbox_ready)
        build_sbox();
    int nk = (int)(keylen / 4);
    if (keylen != 16 && keylen != 32)
        return -1;
    a->rounds = nk + 6;
    int total = 4 * (a->rounds + 1);
    uint8_t w[60][4];
    uint8_t rcon = 1;
    for (int i = 0; i < total; ++i) {
        if (i < nk) {
            memcpy(w[i], key + 4 * i, 4);
            continue;
        }
        uint8_t t[4];
        memcpy(t, w[i - 1], 4);
        if (i % nk == 0) {
            uint8_t t0 = t[0];
            t[0] = (uint8_t)(sbox[t[1]] ^ rcon);
            t[1] = sbox[t[2]];
            t[2] = sbox[t[3]];
            t[3] = sbox[t0];
            rcon = gf8_mul(rcon, 2);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; ++k)
                t[k] = sbox[t[k]];
        }
        for (int k = 0; k < 4; ++k)
            w[i][k] = (uint8_t)(w[i - nk][k] ^ t[k]);
    }
    for (int r = 0; r <= a->rounds; ++r)
        for (int c = 0; c < 4; ++c)
            memcpy(&a->rk[r][4 * c], w[4 * r + c], 4);
    return 0;
}

/* FIPS-197 sec. 5.1 Cipher(); state byte s[r + 4c] is row r, column c. */
static void aes_encrypt(const oracle_aes_t *a, const uint8_t in[16], uint8_t out[16])
{
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; ++i)
        s[i] = in[i] ^ a->rk[0][i];
    for (int r = 1; r <= a->rounds; ++r) {
        /* SubBytes + ShiftRows: row r of column c takes column (c + r) mod 4 */
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row)
                t[row + 4 * c] = sbox[s[row + 4 * ((c + row) & 3)]];
        if (r != a->rounds) {
            /* MixColumns */
            for (int c = 0; c < 4; ++c) {
                uint8_t *col = t + 4 * c, a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3];
                s[4 * c + 0] = (uint8_t)(gf8_mul(a0, 2) ^ gf8_mul(a1, 3) ^ a2 ^ a3);
                s[4 * c + 1] = (uint8_t)(a0 ^ gf8_mul(a1, 2) ^ gf8_mul(a2, 3) ^ a3);
                s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ gf8_mul(a2, 2) ^ gf8_mul(a3, 3));
                s[4 * c + 3] = (uint8_t)(gf8_mul(a0, 3) ^ a1 ^ a2 ^ gf8_mul(a3, 2));
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; ++i)
            s[i] ^= a->rk[r][i];
    }
    memcpy(out, s, 16);
}

/*
 * FIPS-197 sec. 5.3 InvCipher() (the straightforward inverse, not the equivalent inverse cipher the
 * engine uses): AddRoundKey with the last round key, then per round InvShiftRows, InvSubBytes,
 * AddRoundKey, InvMixColumns.  Reference counterpart: AES-ECB decryption of the generic suite's
 * ecb_cipher (t/picotls.c:266-307; OpenSSL EVP_aes_*_ecb, lib/openssl.c:831-838).
 */
static void aes_decrypt(const oracle_aes_t *a, const uint8_t in[16], uint8_t out[16])
{
    uint8_t inv[256], s[16], t[16];
    for (int x = 0; x < 256; ++x)
        inv[sbox[x]] = (uint8_t)x;
    for (int i = 0; i < 16; ++i)
        s[i] = in[i] ^ a->rk[a->rounds][i];
    for (int r = a->rounds - 1; r >= 0; --r) {
        /* InvShiftRows + InvSubBytes: row r of column c comes from column (c - r) mod 4 */
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row)
                t[row + 4 * c] = inv[s[row + 4 * ((c - row + 4) & 3)]];
        for (int i = 0; i < 16; ++i)
            t[i] ^= a->rk[r][i];
        if (r != 0) {
            /* InvMixColumns */
            for (int c = 0; c < 4; ++c) {
                uint8_t *col = t + 4 * c, a0 = col[0], a1 = col[1], a2 = col[2], a3 = col[3];
                s[4 * c + 0] = (uint8_t)(gf8_mul(a0, 14) ^ gf8_mul(a1, 11) ^ gf8_mul(a2, 13) ^ gf8_mul(a3, 9));
                s[4 * c + 1] = (uint8_t)(gf8_mul(a0, 9) ^ gf8_mul(a1, 14) ^ gf8_mul(a2, 11) ^ gf8_mul(a3, 13));
                s[4 * c + 2] = (uint8_t)(gf8_mul(a0, 13) ^ gf8_mul(a1, 9) ^ gf8_mul(a2, 14) ^ gf8_mul(a3, 11));
                s[4 * c + 3] = (uint8_t)(gf8_mul(a0, 11) ^ gf8_mul(a1, 13) ^ gf8_mul(a2, 9) ^ gf8_mul(a3, 14));
            }
        } else {
            memcpy(s, t, 16);
        }
    }
    memcpy(out, s, 16);
}

/* -------------------------------------------------------------- GHASH ----- */

/* SP 800-38D Algorithm 1: Z = X * Y in GF(2^128), bit 0 = MSB of byte 0. */
static void gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t z[16])
{
    uint8_t Z[16] = {0}, V[16];
    memcpy(V, y, 16);
    for (int i = 0; i < 128; ++i) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1)
            for (int k = 0; k < 16; ++k)
                Z[k] ^= V[k];
        int lsb = V[15] & 1;
        for (int k = 15; k > 0; --k)
            V[k] = (uint8_t)((V[k] >> 1) | (V[k - 1] << 7));
        V[0] >>= 1;
        if (lsb)
            V[0] ^= 0xe1;
    }
    memcpy(z, Z, 16);
}

/* absorbs data (zero-padded to a block multiple) into Y */
static void ghash_absorb(uint8_t Y[16], const uint8_t H[16], const uint8_t *p, size_t n)
{
    while (n != 0) {
        size_t take = n < 16 ? n : 16;
        for (size_t k = 0; k < take; ++k)
            Y[k] ^= p[k];
        gf128_mul(Y, H, Y);
        p += take;
        n -= take;
    }
}

static void be64(uint8_t *p, uint64_t v)
{
    for (int i = 7; i >= 0; --i) {
        p[i] = (uint8_t)v;
        v >>= 8;
    }
}

/* inc32 of SP 800-38D: increments only the trailing 32 bits, big endian */
static void inc32(uint8_t cb[16])
{
    for (int i = 15; i >= 12; --i)
        if (++cb[i] != 0)
            break;
}

/* tag (16 B) over (aad, ciphertext) and the CTR pass over data; J0 = iv || 0^31 || 1 */
static void gcm_core(const oracle_aes_t *a, const uint8_t iv[12], const uint8_t *aad, size_t aadlen, const uint8_t *in,
                     uint8_t *out, size_t len, int is_seal, uint8_t tag[16])
{
    uint8_t H[16] = {0}, J0[16], cb[16], ks[16], Y[16] = {0}, lens[16];
    aes_encrypt(a, H, H);
    memcpy(J0, iv, 12);
    J0[12] = J0[13] = J0[14] = 0;
    J0[15] = 1;

    ghash_absorb(Y, H, aad, aadlen);

    memcpy(cb, J0, 16);
    for (size_t off = 0; off < len; off += 16) {
        size_t take = len - off < 16 ? len - off : 16;
        uint8_t ctblk[16] = {0};
        inc32(cb);
        aes_encrypt(a, cb, ks);
        for (size_t k = 0; k < take; ++k) {
            uint8_t c_in = in[off + k];
            uint8_t o = (uint8_t)(c_in ^ ks[k]);
            ctblk[k] = is_seal ? o : c_in;
            out[off + k] = o;
        }
        for (size_t k = 0; k < 16; ++k)
            Y[k] ^= ctblk[k];
        gf128_mul(Y, H, Y);
    }

    be64(lens, (uint64_t)aadlen * 8);
    be64(lens + 8, (uint64_t)len * 8);
    for (int k = 0; k < 16; ++k)
        Y[k] ^= lens[k];
    gf128_mul(Y, H, Y);

    aes_encrypt(a, J0, ks);
    for (int k = 0; k < 16; ++k)
        tag[k] = (uint8_t)(Y[k] ^ ks[k]);
}

/* ------------------------------------------------------------ exports ----- */

/* nonce = static_iv XOR (0^32 || BE64(seq))   -- lib/picotls.c:5291-5305 */
void oracle_build_iv(const uint8_t static_iv[12], uint64_t seq, uint8_t out[12])
{
    memcpy(out, static_iv, 12);
    for (int i = 0; i < 8; ++i)
        out[4 + i] ^= (uint8_t)(seq >> (56 - 8 * i));
}

/* AES-ECB, one block.  Returns 0 or -1 on a bad key size. */
int oracle_aes_ecb_encrypt(const uint8_t *key, size_t keylen, const uint8_t in[16], uint8_t out[16])
{
    oracle_aes_t a;
    if (aes_expand(&a, key, keylen) != 0)
        return -1;
    aes_encrypt(&a, in, out);
    return 0;
}

/* nblocks of AES-ECB decryption (FIPS-197 InvCipher) */
int oracle_aes_ecb_decrypt(const uint8_t *key, size_t keylen, const uint8_t *in, uint8_t *out, size_t nblocks)
{
    oracle_aes_t a;
    if (aes_expand(&a, key, keylen) != 0)
        return -1;
    for (size_t b = 0; b < nblocks; ++b)
        aes_decrypt(&a, in + 16 * b, out + 16 * b);
    return 0;
}

/* nblocks of AES-ECB encryption */
int oracle_aes_ecb_encrypt_n(const uint8_t *key, size_t keylen, const uint8_t *in, uint8_t *out, size_t nblocks)
{
    oracle_aes_t a;
    if (aes_expand(&a, key, keylen) != 0)
        return -1;
    for (size_t b = 0; b < nblocks; ++b)
        aes_encrypt(&a, in + 16 * b, out + 16 * b);
    return 0;
}

/* out must hold len + 16; tag is written at out + len.  out == in is allowed. */
int oracle_gcm_seal(const uint8_t *key, size_t keylen, const uint8_t iv[12], const uint8_t *aad, size_t aadlen,
                    const uint8_t *in, size_t len, uint8_t *out)
{
    oracle_aes_t a;
    uint8_t tag[16];
    if (aes_expand(&a, key, keylen) != 0)
        return -1;
    gcm_core(&a, iv, aad, aadlen, in, out, len, 1, tag);
    memcpy(out + len, tag, 16);
    return 0;
}

/* in holds inlen bytes = ciphertext || tag.  Returns plaintext length or SIZE_MAX. */
size_t oracle_gcm_open(const uint8_t *key, size_t keylen, const uint8_t iv[12], const uint8_t *aad, size_t aadlen,
                       const uint8_t *in, size_t inlen, uint8_t *out)
{
    oracle_aes_t a;
    uint8_t tag[16], diff = 0;
    if (inlen < 16 || aes_expand(&a, key, keylen) != 0)
        return SIZE_MAX;
    size_t len = inlen - 16;
    uint8_t rx[16];
    memcpy(rx, in + len, 16); /* in == out is allowed */
    gcm_core(&a, iv, aad, aadlen, in, out, len, 0, tag);
    for (int k = 0; k < 16; ++k)
        diff |= (uint8_t)(tag[k] ^ rx[k]);
    return diff ? SIZE_MAX : len;
}

/* Multiplication in GF(2^128) exposed for the table tests. */
void oracle_gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t z[16]) { gf128_mul(x, y, z); }

/*
 * Batch form over the engine's record descriptor layout (include/ptls_mi355x.h,
 * ptls_mi355x_record_t): {src, dst, aad, seq (u64); len, aadlen (u32)}.
 * Seal writes len + 16 at dst; open writes len at dst and status[i] = len or
 * 0xffffffff.  Threads split the records; used only to check the GPU engine.
 */
typedef struct {
    uint64_t src, dst, aad, seq;
    uint32_t len, aadlen;
} oracle_record_t;

typedef struct {
    const oracle_aes_t *aes;
    const uint8_t *static_iv;
    const oracle_record_t *recs;
    size_t begin, end;
    const uint8_t *src, *aad;
    uint8_t *dst;
    uint32_t *status;
    int is_seal;
} batch_job_t;

static void *batch_worker(void *arg)
{
    batch_job_t *j = (batch_job_t *)arg;
    for (size_t i = j->begin; i < j->end; ++i) {
        const oracle_record_t *r = &j->recs[i];
        uint8_t iv[12], tag[16];
        oracle_build_iv(j->static_iv, r->seq, iv);
        const uint8_t *in = j->src + r->src;
        uint8_t *out = j->dst + r->dst;
        if (j->is_seal) {
            gcm_core(j->aes, iv, j->aad + r->aad, r->aadlen, in, out, r->len, 1, tag);
            memcpy(out + r->len, tag, 16);
        } else {
            uint8_t rx[16], diff = 0;
            memcpy(rx, in + r->len, 16);
            gcm_core(j->aes, iv, j->aad + r->aad, r->aadlen, in, out, r->len, 0, tag);
            for (int k = 0; k < 16; ++k)
                diff |= (uint8_t)(tag[k] ^ rx[k]);
            j->status[i] = diff ? 0xffffffffu : r->len;
        }
    }
    return NULL;
}

int oracle_gcm_batch(int is_seal, const uint8_t *key, size_t keylen, const uint8_t static_iv[12],
                     const oracle_record_t *recs, size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad,
                     uint32_t *status, int nthreads)
{
    oracle_aes_t a;
    if (aes_expand(&a, key, keylen) != 0)
        return -1;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 64)
        nthreads = 64;
    pthread_t th[64];
    int joinable[64] = {0};
    batch_job_t jobs[64];
    size_t per = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int t = 0; t < nthreads; ++t) {
        size_t b = (size_t)t * per, e = b + per;
        if (b >= n)
            break;
        if (e > n)
            e = n;
        jobs[t] = (batch_job_t){&a, static_iv, recs, b, e, src, aad, dst, status, is_seal};
        if (pthread_create(&th[t], NULL, batch_worker, &jobs[t]) == 0)
            joinable[t] = 1;
        else
            batch_worker(&jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t)
        if (joinable[t])
            pthread_join(th[t], NULL);
    return 0;
}

/* ------------------------------------------------------- TLS 1.3 records ----- */

/*
 * TLS 1.3 record framing over the AEAD, restated from picotls's record layer:
 *   header = 17 03 03 BE16(length)          build_aad (lib/picotls.c:621-628) + buffer_push_record (:658-662)
 *   body   = seal(fragment || type || 0^pad, aad = header, seq)
 *                                           aead_encrypt (:630-643), length = fraglen + 1 + pad + 16
 *   one record per <= 16384-byte fragment, seq + 1 per record   buffer_push_encrypted_records (:664-684)
 * pad != 0 produces the zero padding picotls never sends but must strip on receive (RFC 8446 5.4).
 * Writes 5 + fraglen + 1 + pad + 16 bytes to out (returned).  out must not overlap frag.
 */
size_t oracle_tls_seal_record(const uint8_t *key, size_t keylen, const uint8_t static_iv[12], uint64_t seq, uint8_t type,
                              const uint8_t *frag, size_t fraglen, size_t pad, uint8_t *out)
{
    size_t body = fraglen + 1 + pad;
    uint8_t iv[12];
    out[0] = 23; /* PTLS_CONTENT_TYPE_APPDATA */
    out[1] = 3;
    out[2] = 3;
    out[3] = (uint8_t)((body + 16) >> 8);
    out[4] = (uint8_t)(body + 16);
    memcpy(out + 5, frag, fraglen);
    out[5 + fraglen] = type;
    memset(out + 5 + fraglen + 1, 0, pad);
    oracle_build_iv(static_iv, seq, iv);
    if (oracle_gcm_seal(key, keylen, iv, out, 5, out + 5, body, out + 5) != 0)
        return 0;
    return 5 + body + 16;
}

/*
 * Receive side of one record whose header is at wire[0..5) (length field L = ciphertext + tag):
 * aead_decrypt (lib/picotls.c:645-654) with the AAD rebuilt from L (build_aad), then the padding
 * strip and content-type pop of handle_input_tls13 (:4784-4791).  Returns the inner plaintext
 * length with *type set; SIZE_MAX for a bad tag or L < 16 (-> PTLS_ALERT_BAD_RECORD_MAC),
 * SIZE_MAX - 1 for an all-zero plaintext (-> PTLS_ALERT_UNEXPECTED_MESSAGE).  out holds L - 16 bytes.
 */
size_t oracle_tls_open_record(const uint8_t *key, size_t keylen, const uint8_t static_iv[12], uint64_t seq,
                              const uint8_t *wire, uint8_t *out, uint8_t *type)
{
    size_t L = ((size_t)wire[3] << 8) | wire[4];
    uint8_t aad[5] = {23, 3, 3, wire[3], wire[4]}, iv[12];
    oracle_build_iv(static_iv, seq, iv);
    size_t n = oracle_gcm_open(key, keylen, iv, aad, 5, wire + 5, L, out);
    if (n == SIZE_MAX)
        return SIZE_MAX;
    while (n != 0 && out[n - 1] == 0)
        --n;
    if (n == 0)
        return SIZE_MAX - 1;
    *type = out[--n];
    return n;
}
