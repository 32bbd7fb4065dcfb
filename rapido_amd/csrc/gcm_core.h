/*
 * gcm_core.h -- AES-GCM building blocks of the MI355X engine, shared by the HIP
 * kernels (gcm_engine.hip) and by the host-side kernel model used in tests
 * (tests/cpp/kernel_model.cpp).  Every function here is the exact code the
 * kernels run; on the host the two gfx950 builtins it uses (v_perm_b32 and the
 * LDS loads) are emulated bit-for-bit.
 *
 * Semantics follow the reference engine lib/fusion.c:
 *   - AES-128/256 encryption (aesecb_encrypt, lib/fusion.c:187-197);
 *   - GCM counter blocks J0 = nonce || BE32(1), payload block c uses
 *     nonce || BE32(c + 2) (lib/fusion.c:245-257, 312-314 build the same blocks);
 *   - GHASH over A || pad || C || pad || BE64(8|A|) || BE64(8|C|)
 *     (lib/fusion.c:303, 459-470).
 *
 * Layout conventions (all little-endian dwords, byte 0 of a 16-B block in bits
 * 0-7 of dword 0, exactly the byte order in HBM):
 *   - AES state column j = dword j; T0[x] = (2S, S, S, 3S) packed LE.
 *   - GHASH field elements are kept in stream byte order.  Multiplication by a
 *     constant c uses 32 nibble tables Tab_c[t][v] (t = 8*d + n is nibble n of
 *     dword d, v its value) so that X*c = XOR_t Tab_c[t][nibble_t(X)].
 *
 * LDS map used by the batch kernels (one workgroup per CU):
 *   [0x00000, 0x10000)  AES T-table image: row x (256 B) = T0[x] replicated in
 *                       32 banks, then T1[x] = rotl8(T0[x]) replicated in 32
 *                       banks.  Lane l reads bank (l & 31): conflict-free
 *                       ds_read_b32 for any mix of indices.
 *   [0x10000, ...)      GHASH nibble tables, 8 KiB each; slot j holds
 *                       Tab_{H^(K-j)} (slot 0 = H^K is also the Horner factor).
 *                       A table is 32 rows of 256 B (one bank row per nibble
 *                       position), so a ds_read_b128 of any 64 nibbles from one
 *                       table is conflict-free.
 */
#pragma once
#include <stdint.h>
#include <stddef.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GCM_HD __host__ __device__ __forceinline__
#define GCM_HDC __host__ __device__ constexpr
#else
#define GCM_HD static inline
#define GCM_HDC constexpr
#endif

namespace mi355x {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));

enum : uint32_t {
    LDS_AES_BASE = 0x00000u,
    LDS_AES_BYTES = 0x10000u,
    LDS_GH_BASE = 0x10000u,
    GH_TABLE_BYTES = 32u * 16u * 16u, /* 8 KiB */
    MAX_K = 8,                        /* lanes per record, upper bound */
};

/* ------------------------------------------------------------------ constant tables ------ */

GCM_HDC uint8_t gf8_xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

struct AesTables {
    uint8_t sbox[256];
    uint32_t t0[256];
    constexpr AesTables() : sbox{}, t0{}
    {
        /* S-box from log/antilog tables of generator 3 (FIPS-197 sec. 5.1.1) */
        uint8_t exp_[256] = {}, log_[256] = {};
        uint8_t x = 1;
        for (int i = 0; i < 255; ++i) {
            exp_[i] = x;
            log_[x] = (uint8_t)i;
            x = (uint8_t)(x ^ gf8_xtime(x)); /* x *= 3 */
        }
        for (int v = 0; v < 256; ++v) {
            uint8_t inv = v == 0 ? 0 : exp_[(255 - log_[v]) % 255];
            uint8_t s = inv;
            for (int r = 1; r <= 4; ++r)
                s ^= (uint8_t)((inv << r) | (inv >> (8 - r)));
            sbox[v] = (uint8_t)(s ^ 0x63);
        }
        for (int v = 0; v < 256; ++v) {
            uint8_t s = sbox[v], s2 = gf8_xtime(s), s3 = (uint8_t)(s2 ^ s);
            t0[v] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
        }
    }
};

/* ------------------------------------------------------------------ primitives ----------- */

GCM_HD uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

GCM_HD uint32_t bswap32(uint32_t x)
{
    return (x >> 24) | ((x >> 8) & 0xff00u) | ((x << 8) & 0xff0000u) | (x << 24);
}

/* v_perm_b32: byte i of the result = byte sel_i of the 8-byte value {hi, lo} (lo = bytes 0-3);
 * selector 12 gives 0x00, >= 13 gives 0xff (the sign-replicating selectors 8-11 are unused). */
GCM_HD uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    uint64_t v = ((uint64_t)hi << 32) | lo;
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        uint32_t s = (sel >> (8 * i)) & 0xffu, b;
        if (s < 8)
            b = (uint32_t)(v >> (8 * s)) & 0xffu;
        else if (s == 12)
            b = 0;
        else
            b = 0xffu;
        r |= b << (8 * i);
    }
    return r;
#endif
}

GCM_HD uint32_t lds_u32(const uint8_t *lds, uint32_t addr) { return *(const uint32_t *)(lds + addr); }
GCM_HD u32x4 lds_u32x4(const uint8_t *lds, uint32_t addr) { return *(const u32x4 *)(lds + addr); }

/*
 * One AES encryption of w[4] with the replicated T-table image at lds[0, 64K).
 * lanesel = 4 * (lane & 31): each lane reads its own bank.  rk = 4*(NR+1) round-key dwords.
 * Per column and round: 4 v_perm (address), 4 ds_read_b32, 2 rotates, 2 xor3.
 */
template <int NR>
GCM_HD void aes_encrypt_tt(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, uint32_t w[4])
{
    /* address of byte k of word x: (x.b_k << 8) | lanesel */
#define GCM_TADDR(x, k) perm((x), lanesel, 0x0c0c0400u | ((4u + (k)) << 8))
    uint32_t s0 = w[0] ^ rk[0], s1 = w[1] ^ rk[1], s2 = w[2] ^ rk[2], s3 = w[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        const uint32_t *k = rk + 4 * r;
        uint32_t a0 = GCM_TADDR(s0, 0), a1 = GCM_TADDR(s1, 1), a2 = GCM_TADDR(s2, 2), a3 = GCM_TADDR(s3, 3);
        uint32_t b0 = GCM_TADDR(s1, 0), b1 = GCM_TADDR(s2, 1), b2 = GCM_TADDR(s3, 2), b3 = GCM_TADDR(s0, 3);
        uint32_t c0 = GCM_TADDR(s2, 0), c1 = GCM_TADDR(s3, 1), c2 = GCM_TADDR(s0, 2), c3 = GCM_TADDR(s1, 3);
        uint32_t d0 = GCM_TADDR(s3, 0), d1 = GCM_TADDR(s0, 1), d2 = GCM_TADDR(s1, 2), d3 = GCM_TADDR(s2, 3);
        /* T0 at +0, T1 at +128 within a row; T2 = rotl16(T0), T3 = rotl16(T1) */
        uint32_t n0 = lds_u32(lds, a0) ^ lds_u32(lds, a1 + 128) ^ rotl32(lds_u32(lds, a2), 16) ^
                      rotl32(lds_u32(lds, a3 + 128), 16) ^ k[0];
        uint32_t n1 = lds_u32(lds, b0) ^ lds_u32(lds, b1 + 128) ^ rotl32(lds_u32(lds, b2), 16) ^
                      rotl32(lds_u32(lds, b3 + 128), 16) ^ k[1];
        uint32_t n2 = lds_u32(lds, c0) ^ lds_u32(lds, c1 + 128) ^ rotl32(lds_u32(lds, c2), 16) ^
                      rotl32(lds_u32(lds, c3 + 128), 16) ^ k[2];
        uint32_t n3 = lds_u32(lds, d0) ^ lds_u32(lds, d1 + 128) ^ rotl32(lds_u32(lds, d2), 16) ^
                      rotl32(lds_u32(lds, d3 + 128), 16) ^ k[3];
        s0 = n0;
        s1 = n1;
        s2 = n2;
        s3 = n3;
    }
    /* last round: SubBytes + ShiftRows + AddRoundKey; S[x] is byte 1 (and 2) of T0[x] */
    {
        const uint32_t *k = rk + 4 * NR;
        uint32_t x[4] = {s0, s1, s2, s3};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t ra = lds_u32(lds, GCM_TADDR(x[j], 0));
            uint32_t rb = lds_u32(lds, GCM_TADDR(x[(j + 1) & 3], 1));
            uint32_t rc = lds_u32(lds, GCM_TADDR(x[(j + 2) & 3], 2));
            uint32_t rd = lds_u32(lds, GCM_TADDR(x[(j + 3) & 3], 3));
            uint32_t lo = perm(rb, ra, 0x0c0c0501u); /* S_a -> byte 0, S_b -> byte 1 */
            uint32_t hi = perm(rd, rc, 0x06020c0cu); /* S_c -> byte 2, S_d -> byte 3 */
            w[j] = lo ^ hi ^ k[j];
        }
    }
#undef GCM_TADDR
}

/*
 * r = x * c with the nibble tables of c at LDS byte offset (base: bytes 1..2 of basereg, a multiple of
 * 256 in [64K, 128K)).  32 conflict-free ds_read_b128 + ~110 VALU.
 */
GCM_HD u32x4 ghash_mul_lds(const uint8_t *lds, uint32_t basereg, u32x4 x)
{
    u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        uint32_t w = x[d];
        uint32_t lo = (w << 4) & 0xf0f0f0f0u; /* byte m = 16 * nibble (8d + 2m)     */
        uint32_t hi = w & 0xf0f0f0f0u;        /* byte m = 16 * nibble (8d + 2m + 1) */
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            uint32_t sel = 0x0c020100u | (4u + (uint32_t)m);
            uint32_t alo = perm(lo, basereg, sel), ahi = perm(hi, basereg, sel);
            r ^= lds_u32x4(lds, alo + (uint32_t)(8 * d + 2 * m) * 256u);
            r ^= lds_u32x4(lds, ahi + (uint32_t)(8 * d + 2 * m + 1) * 256u);
        }
    }
    return r;
}

/* --------------------------------------------------------- GF(2^128) on byte strings ---- */

/* SP 800-38D Algorithm 1 on stream-order bytes (used only by the key setup). */
GCM_HD void gf128_mul_bytes(const uint8_t x[16], const uint8_t y[16], uint8_t z[16])
{
    uint8_t Z[16] = {0}, V[16];
    for (int k = 0; k < 16; ++k)
        V[k] = y[k];
    for (int i = 0; i < 128; ++i) {
        if ((x[i >> 3] >> (7 - (i & 7))) & 1)
            for (int k = 0; k < 16; ++k)
                Z[k] ^= V[k];
        uint8_t lsb = V[15] & 1;
        for (int k = 15; k > 0; --k)
            V[k] = (uint8_t)((V[k] >> 1) | (V[k - 1] << 7));
        V[0] >>= 1;
        if (lsb)
            V[0] ^= 0xe1;
    }
    for (int k = 0; k < 16; ++k)
        z[k] = Z[k];
}

/* v <- v * x (one step of Algorithm 1's V update) */
GCM_HD void gf128_mulx_bytes(uint8_t v[16])
{
    uint8_t lsb = v[15] & 1;
    for (int k = 15; k > 0; --k)
        v[k] = (uint8_t)((v[k] >> 1) | (v[k - 1] << 7));
    v[0] >>= 1;
    if (lsb)
        v[0] ^= 0xe1;
}

/* GCM bit index (0 = MSB of byte 0) of bit s (0..3) of nibble t (t = 8*d + n, nibble n of LE dword d) */
GCM_HD int nibble_bit_index(int t, int s)
{
    int byte = 4 * (t >> 3) + ((t & 7) >> 1);
    int q = ((t & 1) ? 4 : 0) + s; /* bit position inside the byte, 0 = LSB */
    return 8 * byte + (7 - q);
}

/* ------------------------------------------------------------------ key image ------------- */

/*
 * Device-resident per-key state, built once per context by the setup kernel (the analogue of
 * ptls_fusion_aesgcm_new, lib/fusion.c:775-795, which precomputes H powers for a capacity;
 * here the table set is fixed and independent of the record size).
 */
struct KeyImage {
    uint32_t rk[60];    /* round keys, LE dwords of the FIPS-197 key schedule */
    uint32_t rounds;    /* 10 or 14 */
    uint32_t key_size;  /* 16 or 32 */
    uint32_t pad_[2];
    uint8_t H[16];      /* E_K(0^128) */
    uint8_t gh[MAX_K][32][16][16]; /* gh[p-1] = nibble tables of H^p, p = 1..MAX_K */
};

/* ------------------------------------------------------------------ record walk ----------- */

/* The batch descriptor (include/ptls_mi355x.h, ptls_mi355x_record_t). */
struct Record {
    uint64_t src, dst, aad, seq;
    uint32_t len, aadlen;
};

/*
 * Work split of one record over K lanes.  GHASH consumes g = A + C + 1 blocks (AAD blocks,
 * ciphertext blocks, length block); the sequence is front-padded with zero blocks to K*T
 * (zero blocks do not change a Horner evaluation started from 0).  Lane j handles padded
 * positions j, j+K, ... and Horner-accumulates with factor H^K; afterwards its sum is scaled
 * by H^(K-j) and the K partial sums are XOR-reduced.  The same lane runs the AES block of the
 * ciphertext position it hashes; the lane holding the length block computes E_K(J0).
 */
struct Walk {
    uint32_t A, C, T, pad;
};

GCM_HD Walk make_walk(uint32_t len, uint32_t aadlen, uint32_t K)
{
    Walk w;
    w.A = (aadlen + 15u) >> 4;
    w.C = (len + 15u) >> 4;
    uint32_t g = w.A + w.C + 1u;
    w.T = (g + K - 1u) / K;
    w.pad = w.T * K - g;
    return w;
}


/* ------------------------------------------------------------------ key setup ------------- */

/* FIPS-197 sec. 5.2 key expansion into LE dwords (rk[4r + c] = column c of round key r). */
GCM_HD uint32_t aes_expand_key(const uint8_t *sbox, const uint8_t *key, uint32_t keylen, uint32_t *rk)
{
    const uint32_t nk = keylen / 4, nr = nk + 6, total = 4 * (nr + 1);
    uint8_t rcon = 1;
    for (uint32_t i = 0; i < nk; ++i)
        rk[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
                ((uint32_t)key[4 * i + 3] << 24);
    for (uint32_t i = nk; i < total; ++i) {
        uint32_t t = rk[i - 1];
        if (i % nk == 0) {
            t = (t >> 8) | (t << 24); /* RotWord on LE bytes */
            t = (uint32_t)sbox[t & 0xff] | ((uint32_t)sbox[(t >> 8) & 0xff] << 8) | ((uint32_t)sbox[(t >> 16) & 0xff] << 16) |
                ((uint32_t)sbox[t >> 24] << 24);
            t ^= rcon;
            rcon = gf8_xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            t = (uint32_t)sbox[t & 0xff] | ((uint32_t)sbox[(t >> 8) & 0xff] << 8) | ((uint32_t)sbox[(t >> 16) & 0xff] << 16) |
                ((uint32_t)sbox[t >> 24] << 24);
        }
        rk[i] = rk[i - nk] ^ t;
    }
    return nr;
}

/* Plain (table-free except the S-box) AES of one block; used by the cold paths only. */
GCM_HD void aes_encrypt_bytes(const uint8_t *sbox, const uint32_t *rk, uint32_t nr, const uint8_t in[16], uint8_t out[16])
{
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; ++i)
        s[i] = (uint8_t)(in[i] ^ (uint8_t)(rk[i >> 2] >> (8 * (i & 3))));
    for (uint32_t r = 1; r <= nr; ++r) {
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row)
                t[row + 4 * c] = sbox[s[row + 4 * ((c + row) & 3)]];
        if (r != nr) {
            for (int c = 0; c < 4; ++c) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                uint8_t e = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
                s[4 * c + 0] = (uint8_t)(a0 ^ e ^ gf8_xtime((uint8_t)(a0 ^ a1)));
                s[4 * c + 1] = (uint8_t)(a1 ^ e ^ gf8_xtime((uint8_t)(a1 ^ a2)));
                s[4 * c + 2] = (uint8_t)(a2 ^ e ^ gf8_xtime((uint8_t)(a2 ^ a3)));
                s[4 * c + 3] = (uint8_t)(a3 ^ e ^ gf8_xtime((uint8_t)(a3 ^ a0)));
            }
        } else {
            for (int i = 0; i < 16; ++i)
                s[i] = t[i];
        }
        for (int i = 0; i < 16; ++i)
            s[i] ^= (uint8_t)(rk[4 * r + (i >> 2)] >> (8 * (i & 3)));
    }
    for (int i = 0; i < 16; ++i)
        out[i] = s[i];
}

/* Builds the whole KeyImage (round keys, H, nibble tables of H^1..H^MAX_K) sequentially. */
GCM_HD int build_key_image(const uint8_t *sbox, const uint8_t *key, uint32_t keylen, KeyImage *ki)
{
    if (keylen != 16 && keylen != 32)
        return -1;
    for (int i = 0; i < 60; ++i)
        ki->rk[i] = 0;
    ki->rounds = aes_expand_key(sbox, key, keylen, ki->rk);
    ki->key_size = keylen;
    ki->pad_[0] = ki->pad_[1] = 0;
    uint8_t zero[16] = {0};
    aes_encrypt_bytes(sbox, ki->rk, ki->rounds, zero, ki->H);

    uint8_t hp[16];
    for (int k = 0; k < 16; ++k)
        hp[k] = ki->H[k];
    for (int p = 1; p <= MAX_K; ++p) {
        if (p > 1)
            gf128_mul_bytes(hp, ki->H, hp);
        uint8_t(*tab)[16][16] = ki->gh[p - 1];
        for (int t = 0; t < 32; ++t)
            for (int k = 0; k < 16; ++k)
                tab[t][0][k] = 0;
        /* single-bit entries: the element with GCM bit k set, times H^p, is H^p * x^k */
        uint8_t v[16];
        for (int k = 0; k < 16; ++k)
            v[k] = hp[k];
        for (int bit = 0; bit < 128; ++bit) {
            int byte = bit >> 3, q = 7 - (bit & 7);
            int t = 8 * (byte >> 2) + 2 * (byte & 3) + (q >= 4 ? 1 : 0), s = q & 3;
            for (int k = 0; k < 16; ++k)
                tab[t][1 << s][k] = v[k];
            gf128_mulx_bytes(v);
        }
        for (int t = 0; t < 32; ++t)
            for (int e = 3; e < 16; ++e)
                if (e & (e - 1))
                    for (int k = 0; k < 16; ++k)
                        tab[t][e][k] = (uint8_t)(tab[t][e & (e - 1)][k] ^ tab[t][e & -e][k]);
    }
    return 0;
}

/*
 * LDS image fill, split over nthr threads: AES T-table replicas and the K GHASH tables
 * (slot j = tables of H^(K-j)).  Called by every thread of a workgroup before the barrier.
 */
GCM_HD void fill_lds(uint8_t *lds, const uint32_t *t0, const KeyImage *ki, uint32_t K, uint32_t tid, uint32_t nthr)
{
    for (uint32_t i = tid; i < LDS_AES_BYTES / 16; i += nthr) {
        uint32_t off = i * 16, x = off >> 8;
        uint32_t v = t0[x];
        if (off & 128)
            v = rotl32(v, 8);
        u32x4 q = {v, v, v, v};
        *(u32x4 *)(lds + LDS_AES_BASE + off) = q;
    }
    const uint32_t nvec = K * (GH_TABLE_BYTES / 16);
    for (uint32_t i = tid; i < nvec; i += nthr) {
        uint32_t slot = i / (GH_TABLE_BYTES / 16), within = i % (GH_TABLE_BYTES / 16);
        const u32x4 *srcv = (const u32x4 *)ki->gh[K - slot - 1];
        *(u32x4 *)(lds + LDS_GH_BASE + slot * GH_TABLE_BYTES + within * 16) = srcv[within];
    }
}

/* ------------------------------------------------------------------ per-lane record walk -- */

/* loads n (< 16) bytes zero-extended */
GCM_HD u32x4 load_partial(const uint8_t *p, uint32_t n)
{
    u32x4 v = {0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < n; ++i)
        v[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
    return v;
}

GCM_HD void store_partial(uint8_t *p, uint32_t n, u32x4 v)
{
    for (uint32_t i = 0; i < n; ++i)
        p[i] = (uint8_t)(v[i >> 2] >> (8 * (i & 3)));
}

/* bytes of a block at and beyond n zeroed (n < 16) */
GCM_HD u32x4 mask_tail(u32x4 v, uint32_t n)
{
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        int keep = (int)n - 4 * d;
        uint32_t m = keep >= 4 ? 0xffffffffu : keep <= 0 ? 0u : (0xffffffffu >> (32 - 8 * keep));
        v[d] &= m;
    }
    return v;
}

/*
 * One lane's share of one record (see struct Walk).  Returns the lane's partial GHASH already
 * scaled by H^(K-j); the lane holding the length block has E_K(J0) folded in, so the XOR of the
 * K returned values is the tag.  Lanes with valid == false run the same instruction stream
 * without touching memory (Tmax is the wave-wide trip count).
 * iv0..iv2: the record's 96-bit nonce as LE dwords.
 */
template <int NR, int K, bool SEAL>
GCM_HD u32x4 lane_walk(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, uint32_t j, const Record &rec, bool valid,
                       uint32_t Tmax, uint32_t iv0, uint32_t iv1, uint32_t iv2, const uint8_t *src, uint8_t *dst,
                       const uint8_t *aad)
{
    const Walk wk = make_walk(rec.len, rec.aadlen, K);
    const uint8_t *in = src + rec.src;
    uint8_t *out = dst + rec.dst;
    const uint8_t *ad = aad + rec.aad;
    u32x4 acc = {0u, 0u, 0u, 0u}, ek0 = {0u, 0u, 0u, 0u};

    for (uint32_t t = 0; t < Tmax; ++t) {
        const bool active = valid && t < wk.T;
        const int32_t p = (int32_t)(j + K * t) - (int32_t)wk.pad;
        const bool is_aad = active && p >= 0 && (uint32_t)p < wk.A;
        const bool is_pay = active && (uint32_t)p >= wk.A && (uint32_t)p < wk.A + wk.C && p >= 0;
        const bool is_len = active && (uint32_t)p == wk.A + wk.C;
        const uint32_t c = (uint32_t)p - wk.A;
        const uint32_t clen = rec.len - 16u * c; /* bytes of this payload block if < 16 */

        u32x4 X = {0u, 0u, 0u, 0u}, data = {0u, 0u, 0u, 0u};
        if (is_pay) {
            if (clen >= 16)
                data = *(const u32x4_u *)(in + 16u * c);
            else
                data = load_partial(in + 16u * c, clen);
        } else if (is_aad) {
            uint32_t alen = rec.aadlen - 16u * (uint32_t)p;
            if (alen >= 16)
                X = *(const u32x4_u *)(ad + 16u * (uint32_t)p);
            else
                X = load_partial(ad + 16u * (uint32_t)p, alen);
        }

        /* one AES per lane per step: payload counter c + 2, otherwise J0 (counter 1) */
        uint32_t ctr = is_pay ? c + 2u : 1u;
        uint32_t w[4] = {iv0, iv1, iv2, bswap32(ctr)};
        aes_encrypt_tt<NR>(lds, lanesel, rk, w);
        u32x4 ks = {w[0], w[1], w[2], w[3]};

        if (is_pay) {
            u32x4 o = data ^ ks;
            if (clen >= 16) {
                *(u32x4_u *)(out + 16u * c) = o;
                X = SEAL ? o : data;
            } else {
                store_partial(out + 16u * c, clen, o);
                X = SEAL ? mask_tail(o, clen) : data;
            }
        } else if (is_len) {
            uint64_t abits = (uint64_t)rec.aadlen * 8u, cbits = (uint64_t)rec.len * 8u;
            X[0] = bswap32((uint32_t)(abits >> 32));
            X[1] = bswap32((uint32_t)abits);
            X[2] = bswap32((uint32_t)(cbits >> 32));
            X[3] = bswap32((uint32_t)cbits);
            ek0 = ks;
        }
        if (active) {
            acc ^= X;
            if (t + 1 < wk.T)
                acc = ghash_mul_lds(lds, LDS_GH_BASE, acc);
        }
    }
    /* scale by H^(K-j): table slot j */
    acc = ghash_mul_lds(lds, LDS_GH_BASE + j * GH_TABLE_BYTES, acc);
    return acc ^ ek0;
}

} // namespace mi355x
