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
 * LDS map used by the batch kernels (one workgroup per CU; struct Layout<K>):
 *   K <= 4 ("four tables", 128 KiB AES + K x 8 KiB = 160 KiB at K = 4):
 *   [0x00000, 0x10000)  AES T-table image A: row x (256 B) = T0[x] replicated in 32
 *                       banks, then T1[x] = rotl8(T0[x]) replicated in 32 banks.
 *   [0x10000, 0x20000)  image B: the same rows for T2 = rotl16(T0) and T3 = rotl24(T0).
 *                       Lane l reads bank (l & 31): conflict-free ds_read_b32 for any
 *                       mix of indices, and no rotates in the round function.
 *   [0x20000, ...)      GHASH nibble tables, 8 KiB each; slot j holds
 *                       Tab_{H^(K-j)} (slot 0 = H^K is also the Horner factor).
 *   K = 8 ("two tables", 64 KiB AES + 8 x 8 KiB = 128 KiB): only image A; T2 and T3 are
 *                       rotl16 of the T0/T1 reads (one XOR + one rotate per column), and
 *                       the GHASH tables start at 0x10000.  K = 8 makes every wave-wide
 *                       load/store cover whole 128-byte lines of 8 records.
 *                       A table is 32 rows of 256 B (one bank row per nibble
 *                       position), so a ds_read_b128 of any 64 nibbles from one
 *                       table is conflict-free.
 */
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <type_traits>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define GCM_HD __host__ __device__ __forceinline__
#define GCM_HDC __host__ __device__ constexpr
#else
#define GCM_HD static inline
#define GCM_HDC constexpr
#endif

/*
 * Profiling ablations (scripts/ablate.py builds them as separate libraries; the product
 * build never defines these): GCM_ABLATE_GHASH skips the GHASH multiplies, GCM_ABLATE_AES
 * skips the AES rounds.  Outputs are wrong in those builds; only their timings are used.
 */
#ifndef GCM_ABLATE_GHASH
#define GCM_ABLATE_GHASH 0
#endif
#ifndef GCM_SCALE_W
#define GCM_SCALE_W 0 /* the closing scaling multiply (lane_walk): 0 compiler-paired reads, 1 two batches of 16, 2 all 32 */
#endif
#ifndef GCM_ABLATE_SCALE
#define GCM_ABLATE_SCALE 0 /* measurement builds: no closing scaling multiply (wrong tags) */
#endif
#ifndef GCM_ABLATE_AES
#define GCM_ABLATE_AES 0
#endif

#ifndef GCM_WALK_STAMP
#define GCM_WALK_STAMP(i) ((void)0) /* timestamps inside lane_walk (measurement builds only, gcm_engine.hip) */
#endif

namespace mi355x {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef uint32_t uint32_t_u __attribute__((aligned(1)));

enum : uint32_t {
    LDS_AES_BASE = 0x00000u,
    LDS_AES_BYTES = 0x20000u,         /* two 64 KiB images: (T0|T1) and (T2|T3) */
    LDS_GH_BASE = 0x20000u,
    GH_TABLE_BYTES = 32u * 16u * 16u, /* 8 KiB */
    MAX_K = 8,                        /* tables kept in the key image: H^1..H^8 */
    MAX_KERNEL_K = 8,
    GH5_CHUNKS = 26u,                 /* 5-bit tables: chunk c = bits [5c, 5c + 5) of the 128-bit X */
    GH5_BYTES = GH5_CHUNKS * 512u,    /* per chunk a 256-B row of low halves, then one of high halves */
    GH8_BYTES = 256u * 256u,          /* 8-bit latin tables: 256 rows (byte value) x 16 slots (byte position) */
};

#ifndef GCM_GH5
#define GCM_GH5 0
#endif
/*
 * GCM_GH5 (an evaluated layout, OFF): K = 4 with the Horner factor H^4 as 5-bit tables of 8-byte halves at
 * [0, GH5_BYTES) -- 26 chunks x 2 ds_read_b64 = 104 nominal LDS cycles per multiply instead of 32
 * ds_read_b128 = 128, since a b64 read costs the same 2 cycles as a b32 one and 32 entries x 8 B fill one
 * bank row -- the AES images after them, and nibble tables of H^2 | H^1 for the closing scaling (H^e, e in
 * 1..4, as two multiplies).  Bit-exact, but measured 33% SLOWER (scripts/ablate.py nogh5 vs gh5, 1400 B):
 * SQ_LDS_BANK_CONFLICT rose from 6 to 201 cycles per block.  Unlike ds_read_b128 on the nibble tables,
 * ds_read_b64 does not broadcast lanes that read the same address, and random 5-bit indices put 2-4 lanes
 * on each entry.
 */
#ifndef GCM_GH8
#define GCM_GH8 1
#endif
#ifndef GCM_GH8_KR_SALU
#define GCM_GH8_KR_SALU 1 /* GH8 rounds: rotl16 of the round keys by two SALU per key, in the round */
#endif
/*
 * GCM_GH8: K = 4 with the Horner factor H^4 as 8-bit "latin" tables (gh8_* below): 16 conflict-free ds_read_b128 per
 * multiply instead of the nibble tables' 32.  The 64 KiB table takes [0, 64K); the AES runs on the two-table image
 * (T0 | T1) at [64K, 128K), addressed through byte 2 of the lane selector (aes_b2); the nibble tables of H^4..H^1
 * for the closing lane scaling stay at [128K, 160K).
 */
template <int K>
struct Layout {
    static constexpr bool gh8 = GCM_GH8 && K == 4;
    static constexpr bool four_tables = K <= 4 && !gh8;
    static constexpr bool gh5 = GCM_GH5 && K == 4 && !gh8;
    static constexpr uint32_t aes_base = gh5 ? (uint32_t)GH5_BYTES : 0u;
    /* v_perm selector of an AES address's byte 2: 0x0c = zero (image at aes_base), 0x02 = lanesel byte 2 (+64K) */
    static constexpr uint32_t aes_b2 = gh8 ? 0x02u : 0x0cu;
    static constexpr uint32_t aes_bytes = four_tables ? 0x20000u : 0x10000u;
    /* nibble tables: slot s = H^(n_nibble - s) */
    static constexpr uint32_t gh_base = gh8 ? 0x20000u : aes_base + aes_bytes;
    static constexpr uint32_t n_nibble = gh5 ? 2u : (uint32_t)K;
    static constexpr uint32_t total = gh_base + n_nibble * GH_TABLE_BYTES;
    static constexpr bool split_scale = false; /* lane scaling by one table H^(K - slot) (lane_walk) */
    static constexpr bool x2_walk = false;
    static_assert(total <= 160u * 1024u, "LDS budget");
};

/* ------------------------------------------------------------------ constant tables ------ */

GCM_HDC uint8_t gf8_xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

GCM_HDC uint8_t gf8_mul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    for (int i = 0; i < 8; ++i) {
        if (b & 1)
            r = (uint8_t)(r ^ a);
        a = gf8_xtime(a);
        b = (uint8_t)(b >> 1);
    }
    return r;
}

struct AesTables {
    uint8_t sbox[256];
    uint32_t t0[256];
    uint8_t inv_sbox[256]; /* FIPS-197 5.3.2 */
    uint32_t td0[256];     /* InvMixColumns column 0 times InvS[x]: (e, 9, d, b) * InvS[x], packed LE */
    constexpr AesTables() : sbox{}, t0{}, inv_sbox{}, td0{}
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
        for (int v = 0; v < 256; ++v)
            inv_sbox[sbox[v]] = (uint8_t)v;
        for (int v = 0; v < 256; ++v) {
            uint8_t s = inv_sbox[v];
            td0[v] = (uint32_t)gf8_mul(s, 0x0e) | ((uint32_t)gf8_mul(s, 0x09) << 8) | ((uint32_t)gf8_mul(s, 0x0d) << 16) |
                     ((uint32_t)gf8_mul(s, 0x0b) << 24);
        }
    }
};

/* ------------------------------------------------------------------ primitives ----------- */

GCM_HD uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

/* a ^ b ^ c in one v_bitop3_b32 (gfx950 has no v_xor3_b32) */
GCM_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
    return a ^ b ^ c;
#endif
}

/* xor3 that the optimizer may not move: pins a GHASH accumulation step right behind its
 * LDS reads (the IR passes otherwise sink the chain past the AES rounds and spill) */
GCM_HD uint32_t xor3_pinned(uint32_t a, uint32_t b, uint32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    uint32_t r;
    asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return a ^ b ^ c;
#endif
}

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

/* scheduling fence: keeps the compiler from hoisting one round's independent LDS reads into
 * another (which it otherwise does, spilling registers at 16 waves per CU) */
#if defined(__HIP_DEVICE_COMPILE__)
#define GCM_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define GCM_SCHED_FENCE() ((void)0)
#endif
/* value the optimiser cannot see through (blocks hoisting of rare-path work out of the loop) */
#if defined(__HIP_DEVICE_COMPILE__)
#define GCM_OPAQUE(x) asm volatile("" : "+v"(x))
#else
#define GCM_OPAQUE(x) ((void)0)
#endif
/* x as a wave-uniform (scalar) value: lane 0's copy; the host kernel model runs one lane at a time */
GCM_HD uint32_t wave_uniform(uint32_t x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_readfirstlane(x);
#else
    return x;
#endif
}

GCM_HD uint32_t lds_u32(const uint8_t *lds, uint32_t addr) { return *(const uint32_t *)(lds + addr); }
GCM_HD u32x4 lds_u32x4(const uint8_t *lds, uint32_t addr) { return *(const u32x4 *)(lds + addr); }
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
GCM_HD u32x2 lds_u32x2(const uint8_t *lds, uint32_t addr) { return *(const u32x2 *)(lds + addr); }

/* bits [s, s + 32) of the 64-bit value {hi, lo} (v_alignbit_b32), 0 <= s < 32 */
GCM_HD uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, s);
#else
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
#endif
}

/*
 * One AES encryption of w[4] with the replicated T-table images at lds[0, 128K).
 * lanesel = 4 * (lane & 31) | 0x10000: bits 0-7 pick the lane's bank, byte 2 selects image B.
 * rk = 4*(NR+1) round-key dwords (wave-uniform: SGPRs).
 * Per column and round: 4 v_perm (addresses), 4 ds_read_b32, 2 v_bitop3 (xor3).
 */
/* one full AES round column: T0[a] ^ T1[b] ^ T2[c] ^ T3[d] ^ k, from 4 or 2 tables */
template <bool FOUR>
GCM_HD uint32_t aes_col(const uint8_t *lds, uint32_t lanesel, uint32_t sa, uint32_t sb, uint32_t sc, uint32_t sd, uint32_t k)
{
#define GCM_TA(x, kk) perm((x), lanesel, 0x0c0c0400u | ((4u + (kk)) << 8))
#define GCM_TB(x, kk) perm((x), lanesel, 0x0c020400u | ((4u + (kk)) << 8))
    if (FOUR)
        return xor3(xor3(lds_u32(lds, GCM_TA(sa, 0)), lds_u32(lds, GCM_TA(sb, 1) + 128), k), lds_u32(lds, GCM_TB(sc, 2)),
                    lds_u32(lds, GCM_TB(sd, 3) + 128));
    /* T2 = rotl16(T0), T3 = rotl16(T1): rotate the XOR of the two reads once */
    return xor3(lds_u32(lds, GCM_TA(sa, 0)), lds_u32(lds, GCM_TA(sb, 1) + 128),
                k ^ rotl32(lds_u32(lds, GCM_TA(sc, 2)) ^ lds_u32(lds, GCM_TA(sd, 3) + 128), 16));
#undef GCM_TA
#undef GCM_TB
}

template <int NR, bool FOUR = true>
GCM_HD void aes_encrypt_tt(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, uint32_t w[4])
{
    /* address of byte k of word x in image A: (x.b_k << 8) | lane bank; image B adds byte 2 of lanesel */
#define GCM_TA(x, k) perm((x), lanesel, 0x0c0c0400u | ((4u + (k)) << 8))
#define GCM_TB(x, k) perm((x), lanesel, 0x0c020400u | ((4u + (k)) << 8))
    uint32_t s0 = w[0] ^ rk[0], s1 = w[1] ^ rk[1], s2 = w[2] ^ rk[2], s3 = w[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        const uint32_t *k = rk + 4 * r;
        /* column j: T0[s_j.b0] ^ T1[s_{j+1}.b1] ^ T2[s_{j+2}.b2] ^ T3[s_{j+3}.b3] ^ rk */
        uint32_t n0 = aes_col<FOUR>(lds, lanesel, s0, s1, s2, s3, k[0]);
        uint32_t n1 = aes_col<FOUR>(lds, lanesel, s1, s2, s3, s0, k[1]);
        uint32_t n2 = aes_col<FOUR>(lds, lanesel, s2, s3, s0, s1, k[2]);
        uint32_t n3 = aes_col<FOUR>(lds, lanesel, s3, s0, s1, s2, k[3]);
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
            uint32_t ra = lds_u32(lds, GCM_TA(x[j], 0));
            uint32_t rb = lds_u32(lds, GCM_TA(x[(j + 1) & 3], 1));
            uint32_t rc = lds_u32(lds, GCM_TA(x[(j + 2) & 3], 2));
            uint32_t rd = lds_u32(lds, GCM_TA(x[(j + 3) & 3], 3));
            uint32_t lo = perm(rb, ra, 0x0c0c0501u); /* S_a -> byte 0, S_b -> byte 1 */
            uint32_t hi = perm(rd, rc, 0x06020c0cu); /* S_c -> byte 2, S_d -> byte 3 */
            w[j] = xor3(lo, hi, k[j]);
        }
    }
#undef GCM_TA
#undef GCM_TB
}

/*
 * Four of the 32 nibble-table reads of a GHASH multiply (dword d, nibble pairs m0, m0+1):
 * P ^= Tab[8d+2m][lo.b_m] ^ Tab[8d+2m+1][hi.b_m].  Used to spread one multiply over the
 * AES rounds so a wave always has independent LDS reads in flight.
 */
GCM_HD void ghash_quarter(const uint8_t *lds, uint32_t basereg, uint32_t w, int d, int m0, u32x4 &P)
{
    uint32_t lo = (w << 4) & 0xf0f0f0f0u, hi = w & 0xf0f0f0f0u;
#pragma unroll
    for (int m = m0; m < m0 + 2; ++m) {
        uint32_t sel = 0x0c020100u | (4u + (uint32_t)m);
        u32x4 e = lds_u32x4(lds, perm(lo, basereg, sel) + (uint32_t)(8 * d + 2 * m) * 256u);
        u32x4 f = lds_u32x4(lds, perm(hi, basereg, sel) + (uint32_t)(8 * d + 2 * m + 1) * 256u);
        P[0] = xor3_pinned(P[0], e[0], f[0]);
        P[1] = xor3_pinned(P[1], e[1], f[1]);
        P[2] = xor3_pinned(P[2], e[2], f[2]);
        P[3] = xor3_pinned(P[3], e[3], f[3]);
    }
}

/* ghash_quarter split in two: the four table reads, and their accumulation into P */
GCM_HD void ghash_quarter_issue(const uint8_t *lds, uint32_t basereg, uint32_t w, int d, int m0, u32x4 g[4])
{
    uint32_t lo = (w << 4) & 0xf0f0f0f0u, hi = w & 0xf0f0f0f0u;
#pragma unroll
    for (int m = m0; m < m0 + 2; ++m) {
        uint32_t sel = 0x0c020100u | (4u + (uint32_t)m);
        g[2 * (m - m0)] = lds_u32x4(lds, perm(lo, basereg, sel) + (uint32_t)(8 * d + 2 * m) * 256u);
        g[2 * (m - m0) + 1] = lds_u32x4(lds, perm(hi, basereg, sel) + (uint32_t)(8 * d + 2 * m + 1) * 256u);
    }
}

GCM_HD void ghash_quarter_acc(const u32x4 g[4], u32x4 &P)
{
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
        P[0] = xor3_pinned(P[0], g[i][0], g[i + 1][0]);
        P[1] = xor3_pinned(P[1], g[i][1], g[i + 1][1]);
        P[2] = xor3_pinned(P[2], g[i][2], g[i + 1][2]);
        P[3] = xor3_pinned(P[3], g[i][3], g[i + 1][3]);
    }
}

/*
 * 5-bit GHASH tables (Layout<4>::gh5, built by fill_lds from the key image's nibble tables): chunk c of X
 * is bits [5c, 5c + 5) (bit 32d + i = bit i of dword d; chunk 25 has 3 bits).  Row c*512 holds the low
 * 8 bytes of (chunk value v placed at bit 5c) * H^4 for v = 0..31, row c*512 + 256 the high 8 bytes.
 * The row offset of v, 8v, comes from one shift (or v_alignbit across dwords) and one AND: the tables
 * sit at LDS address 0, so the chunk's row is the read's immediate offset.
 */
GCM_HD uint32_t gh5_off(const u32x4 &X, int c)
{
    const int b = 5 * c, d = b >> 5, o = b & 31;
    uint32_t t;
    if (o + 5 <= 32 || d == 3)
        t = o >= 3 ? X[d] >> (o - 3) : X[d] << (3 - o);
    else
        t = alignbit(X[d + 1], X[d], (uint32_t)(o - 3));
    return t & 0xf8u;
}

/* the 2n reads of chunks c0 .. c0+n-1 (n <= 4) */
GCM_HD void gh5_issue(const uint8_t *lds, const u32x4 &X, int c0, int n, u32x2 g[8])
{
#pragma unroll
    for (int i = 0; i < n; ++i) {
        const uint32_t a = gh5_off(X, c0 + i) + (uint32_t)(c0 + i) * 512u;
        g[2 * i] = lds_u32x2(lds, a);
        g[2 * i + 1] = lds_u32x2(lds, a + 256u);
    }
}

GCM_HD void gh5_acc(const u32x2 g[8], int n, u32x4 &P)
{
#pragma unroll
    for (int i = 0; i + 1 < n; i += 2) {
        P[0] = xor3_pinned(P[0], g[2 * i][0], g[2 * i + 2][0]);
        P[1] = xor3_pinned(P[1], g[2 * i][1], g[2 * i + 2][1]);
        P[2] = xor3_pinned(P[2], g[2 * i + 1][0], g[2 * i + 3][0]);
        P[3] = xor3_pinned(P[3], g[2 * i + 1][1], g[2 * i + 3][1]);
    }
    if (n & 1) {
        P[0] ^= g[2 * (n - 1)][0];
        P[1] ^= g[2 * (n - 1)][1];
        P[2] ^= g[2 * (n - 1) + 1][0];
        P[3] ^= g[2 * (n - 1) + 1][1];
    }
}

/* chunks of GHASH slot s (0..7) of a fused multiply: 3,3,3,3,3,3,4,4 */
GCM_HDC int gh5_slot_first(int s) { return s < 6 ? 3 * s : 18 + 4 * (s - 6); }
GCM_HDC int gh5_slot_count(int s) { return s < 6 ? 3 : 4; }

/* X * H^4 from the 5-bit tables, not fused */
GCM_HD u32x4 ghash5_mul_lds(const uint8_t *lds, u32x4 X)
{
    u32x4 P = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int s = 0; s < 8; ++s) {
        u32x2 g[8];
        gh5_issue(lds, X, gh5_slot_first(s), gh5_slot_count(s), g);
        gh5_acc(g, gh5_slot_count(s), P);
    }
    return P;
}

#ifndef GCM_ROUND_PRIO
#define GCM_ROUND_PRIO 1 /* GH8 middle rounds: wave priority raised while a round issues its 16 LDS reads (measured) */
#endif
#ifndef GCM_PRIO_LEVEL
#define GCM_PRIO_LEVEL 2
#endif
#ifndef GCM_PRIO_LAST
#define GCM_PRIO_LAST 0 /* 1: raised through the last round's 16 S-box reads too */
#endif
#ifndef GCM_PRIO_GH8
#define GCM_PRIO_GH8 1 /* 1: raised already before the round's two GH8 reads */
#endif
#define GCM_STR2(x) #x
#define GCM_STR(x) GCM_STR2(x)
#if GCM_ROUND_PRIO
#define GCM_PRIO_HI "s_setprio " GCM_STR(GCM_PRIO_LEVEL) "\n\t"
#define GCM_PRIO_LO "s_setprio 0\n\t"
#else
#define GCM_PRIO_HI ""
#define GCM_PRIO_LO ""
#endif
#ifndef GCM_ROUND_ASM
#define GCM_ROUND_ASM 1
#endif
#ifndef GCM_R2CACHE
#define GCM_R2CACHE 1
#endif
#if defined(__HIP_DEVICE_COMPILE__)
/*
 * One full AES round on the four-table image (aes_col x 4) as a single instruction block:
 * 16 address perms, the 16 ds_read_b32 back to back, then counted waits feeding the column
 * XORs, so every wave keeps 16 (+ the GHASH quarter's 4, issued just before) LDS reads in
 * flight regardless of the compiler's scheduling heuristics.  The block ends with
 * lgkmcnt(0): no read of it is outstanding afterwards, so the compiler's own counted waits
 * stay exact (DS reads complete in order).  Bit-identical to the aes_col sequence.
 */
/* BASE: LDS address of the AES images (Layout::aes_base), folded into the reads' immediate offsets */
template <uint32_t BASE = 0u>
__device__ __forceinline__ void aes_round_tt4_asm(uint32_t ls, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                                  const uint32_t *k, uint32_t &n0, uint32_t &n1, uint32_t &n2,
                                                  uint32_t &n3)
{
    uint32_t t1, t2, t3, t5, t6, t7, t9, t10, t11, t13, t14, t15;
    asm volatile(
        /* column c reads T0[s_c.b0], T1[s_(c+1).b1] (+128), T2[s_(c+2).b2], T3[s_(c+3).b3] (+128) */
        "v_perm_b32 %[n0], %[s0], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t1], %[s1], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t2], %[s2], %[ls], %[b2]\n\t"
        "v_perm_b32 %[t3], %[s3], %[ls], %[b3]\n\t"
        "ds_read_b32 %[n0], %[n0] offset:%[o0]\n\t"
        "ds_read_b32 %[t1], %[t1] offset:%[o1]\n\t"
        "ds_read_b32 %[t2], %[t2] offset:%[o0]\n\t"
        "ds_read_b32 %[t3], %[t3] offset:%[o1]\n\t"
        "v_perm_b32 %[n1], %[s1], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t5], %[s2], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t6], %[s3], %[ls], %[b2]\n\t"
        "v_perm_b32 %[t7], %[s0], %[ls], %[b3]\n\t"
        "ds_read_b32 %[n1], %[n1] offset:%[o0]\n\t"
        "ds_read_b32 %[t5], %[t5] offset:%[o1]\n\t"
        "ds_read_b32 %[t6], %[t6] offset:%[o0]\n\t"
        "ds_read_b32 %[t7], %[t7] offset:%[o1]\n\t"
        "v_perm_b32 %[n2], %[s2], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t9], %[s3], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t10], %[s0], %[ls], %[b2]\n\t"
        "v_perm_b32 %[t11], %[s1], %[ls], %[b3]\n\t"
        "ds_read_b32 %[n2], %[n2] offset:%[o0]\n\t"
        "ds_read_b32 %[t9], %[t9] offset:%[o1]\n\t"
        "ds_read_b32 %[t10], %[t10] offset:%[o0]\n\t"
        "ds_read_b32 %[t11], %[t11] offset:%[o1]\n\t"
        "v_perm_b32 %[n3], %[s3], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t13], %[s0], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t14], %[s1], %[ls], %[b2]\n\t"
        "v_perm_b32 %[t15], %[s2], %[ls], %[b3]\n\t"
        "ds_read_b32 %[n3], %[n3] offset:%[o0]\n\t"
        "ds_read_b32 %[t13], %[t13] offset:%[o1]\n\t"
        "ds_read_b32 %[t14], %[t14] offset:%[o0]\n\t"
        "ds_read_b32 %[t15], %[t15] offset:%[o1]\n\t"
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_bitop3_b32 %[n0], %[n0], %[t1], %[k0] bitop3:0x96\n\t"
        "v_bitop3_b32 %[n0], %[n0], %[t2], %[t3] bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(8)\n\t"
        "v_bitop3_b32 %[n1], %[n1], %[t5], %[k1] bitop3:0x96\n\t"
        "v_bitop3_b32 %[n1], %[n1], %[t6], %[t7] bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        "v_bitop3_b32 %[n2], %[n2], %[t9], %[k2] bitop3:0x96\n\t"
        "v_bitop3_b32 %[n2], %[n2], %[t10], %[t11] bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_bitop3_b32 %[n3], %[n3], %[t13], %[k3] bitop3:0x96\n\t"
        "v_bitop3_b32 %[n3], %[n3], %[t14], %[t15] bitop3:0x96"
        : [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2), [n3] "=&v"(n3), [t1] "=&v"(t1), [t2] "=&v"(t2),
          [t3] "=&v"(t3), [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7), [t9] "=&v"(t9), [t10] "=&v"(t10),
          [t11] "=&v"(t11), [t13] "=&v"(t13), [t14] "=&v"(t14), [t15] "=&v"(t15)
        : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [ls] "v"(ls), [k0] "s"(k[0]), [k1] "s"(k[1]),
          [k2] "s"(k[2]), [k3] "s"(k[3]), [a0] "s"(0x0c0c0400u), [a1] "s"(0x0c0c0500u), [b2] "s"(0x0c020600u),
          [b3] "s"(0x0c020700u), [o0] "i"(BASE), [o1] "i"(BASE + 128u)
        : "memory");
}

/*
 * The same for the two-table image (T0 | T1 rows only: K = 8 batch kernels, window kernels): column c is
 * T0[a] ^ T1[b] ^ k ^ rotl16(T0[c'] ^ T1[d']) (T2 = rotl16(T0), T3 = rotl16(T1)).  All 16 reads are issued
 * before the first wait; at one wave per SIMD (window kernels) the compiler's grouped waits otherwise
 * expose an LDS latency per group.
 */
template <uint32_t BASE = 0u>
__device__ __forceinline__ void aes_round_tt2_asm(uint32_t ls, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                                  const uint32_t *k, uint32_t &n0, uint32_t &n1, uint32_t &n2,
                                                  uint32_t &n3)
{
    uint32_t t1, t2, t3, t5, t6, t7, t9, t10, t11, t13, t14, t15;
    asm volatile(
        "v_perm_b32 %[n0], %[s0], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t1], %[s1], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t2], %[s2], %[ls], %[a2]\n\t"
        "v_perm_b32 %[t3], %[s3], %[ls], %[a3]\n\t"
        "ds_read_b32 %[n0], %[n0] offset:%[o0]\n\t"
        "ds_read_b32 %[t1], %[t1] offset:%[o1]\n\t"
        "ds_read_b32 %[t2], %[t2] offset:%[o0]\n\t"
        "ds_read_b32 %[t3], %[t3] offset:%[o1]\n\t"
        "v_perm_b32 %[n1], %[s1], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t5], %[s2], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t6], %[s3], %[ls], %[a2]\n\t"
        "v_perm_b32 %[t7], %[s0], %[ls], %[a3]\n\t"
        "ds_read_b32 %[n1], %[n1] offset:%[o0]\n\t"
        "ds_read_b32 %[t5], %[t5] offset:%[o1]\n\t"
        "ds_read_b32 %[t6], %[t6] offset:%[o0]\n\t"
        "ds_read_b32 %[t7], %[t7] offset:%[o1]\n\t"
        "v_perm_b32 %[n2], %[s2], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t9], %[s3], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t10], %[s0], %[ls], %[a2]\n\t"
        "v_perm_b32 %[t11], %[s1], %[ls], %[a3]\n\t"
        "ds_read_b32 %[n2], %[n2] offset:%[o0]\n\t"
        "ds_read_b32 %[t9], %[t9] offset:%[o1]\n\t"
        "ds_read_b32 %[t10], %[t10] offset:%[o0]\n\t"
        "ds_read_b32 %[t11], %[t11] offset:%[o1]\n\t"
        "v_perm_b32 %[n3], %[s3], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t13], %[s0], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t14], %[s1], %[ls], %[a2]\n\t"
        "v_perm_b32 %[t15], %[s2], %[ls], %[a3]\n\t"
        "ds_read_b32 %[n3], %[n3] offset:%[o0]\n\t"
        "ds_read_b32 %[t13], %[t13] offset:%[o1]\n\t"
        "ds_read_b32 %[t14], %[t14] offset:%[o0]\n\t"
        "ds_read_b32 %[t15], %[t15] offset:%[o1]\n\t"
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_xor_b32 %[t2], %[t2], %[t3]\n\t"
        "v_bitop3_b32 %[n0], %[n0], %[t1], %[k0] bitop3:0x96\n\t"
        "v_alignbit_b32 %[t2], %[t2], %[t2], 16\n\t"
        "v_xor_b32 %[n0], %[n0], %[t2]\n\t"
        "s_waitcnt lgkmcnt(8)\n\t"
        "v_xor_b32 %[t6], %[t6], %[t7]\n\t"
        "v_bitop3_b32 %[n1], %[n1], %[t5], %[k1] bitop3:0x96\n\t"
        "v_alignbit_b32 %[t6], %[t6], %[t6], 16\n\t"
        "v_xor_b32 %[n1], %[n1], %[t6]\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        "v_xor_b32 %[t10], %[t10], %[t11]\n\t"
        "v_bitop3_b32 %[n2], %[n2], %[t9], %[k2] bitop3:0x96\n\t"
        "v_alignbit_b32 %[t10], %[t10], %[t10], 16\n\t"
        "v_xor_b32 %[n2], %[n2], %[t10]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_xor_b32 %[t14], %[t14], %[t15]\n\t"
        "v_bitop3_b32 %[n3], %[n3], %[t13], %[k3] bitop3:0x96\n\t"
        "v_alignbit_b32 %[t14], %[t14], %[t14], 16\n\t"
        "v_xor_b32 %[n3], %[n3], %[t14]"
        : [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2), [n3] "=&v"(n3), [t1] "=&v"(t1), [t2] "=&v"(t2),
          [t3] "=&v"(t3), [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7), [t9] "=&v"(t9), [t10] "=&v"(t10),
          [t11] "=&v"(t11), [t13] "=&v"(t13), [t14] "=&v"(t14), [t15] "=&v"(t15)
        : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [ls] "v"(ls), [k0] "s"(k[0]), [k1] "s"(k[1]),
          [k2] "s"(k[2]), [k3] "s"(k[3]), [a0] "s"(0x0c0c0400u), [a1] "s"(0x0c0c0500u), [a2] "s"(0x0c0c0600u),
          [a3] "s"(0x0c0c0700u), [o0] "i"(BASE), [o1] "i"(BASE + 128u)
        : "memory");
}
/*
 * One middle round of the two-table layout (aes_round_tt2_asm) for TWO independent states A and B, as one asm block:
 * A's 16 reads go out first, B's 16 addresses are formed while they are in flight, and each of A's columns is
 * finished as its reads return, followed by one column of B's reads, so at most 16 reads are outstanding (the LDS
 * counter's reach) and B's reads overlap A's XORs.  For the latency-bound split walk, where one wave per SIMD has
 * nothing else to hide an LDS round trip behind: two counter blocks per lane per step instead of one.
 */
template <uint32_t BASE>
__device__ __forceinline__ void aes_round_tt2_asm_x2(uint32_t ls, const uint32_t sA[4], const uint32_t sB[4],
                                                     const uint32_t *k, uint32_t nA[4], uint32_t nB[4])
{
    uint32_t tA1, tA2, tA3, tA5, tA6, tA7, tA9, tA10, tA11, tA13, tA14, tA15, tB1, tB2, tB3, tB5, tB6, tB7, tB9, tB10, tB11, tB13, tB14, tB15;
    asm volatile(
        "v_perm_b32 %[nA0], %[sA0], %[ls], %[a0]\n\t"
        "v_perm_b32 %[tA1], %[sA1], %[ls], %[a1]\n\t"
        "v_perm_b32 %[tA2], %[sA2], %[ls], %[a2]\n\t"
        "v_perm_b32 %[tA3], %[sA3], %[ls], %[a3]\n\t"
        "ds_read_b32 %[nA0], %[nA0] offset:%[o0]\n\t"
        "ds_read_b32 %[tA1], %[tA1] offset:%[o1]\n\t"
        "ds_read_b32 %[tA2], %[tA2] offset:%[o0]\n\t"
        "ds_read_b32 %[tA3], %[tA3] offset:%[o1]\n\t"
        "v_perm_b32 %[nA1], %[sA1], %[ls], %[a0]\n\t"
        "v_perm_b32 %[tA5], %[sA2], %[ls], %[a1]\n\t"
        "v_perm_b32 %[tA6], %[sA3], %[ls], %[a2]\n\t"
        "v_perm_b32 %[tA7], %[sA0], %[ls], %[a3]\n\t"
        "ds_read_b32 %[nA1], %[nA1] offset:%[o0]\n\t"
        "ds_read_b32 %[tA5], %[tA5] offset:%[o1]\n\t"
        "ds_read_b32 %[tA6], %[tA6] offset:%[o0]\n\t"
        "ds_read_b32 %[tA7], %[tA7] offset:%[o1]\n\t"
        "v_perm_b32 %[nA2], %[sA2], %[ls], %[a0]\n\t"
        "v_perm_b32 %[tA9], %[sA3], %[ls], %[a1]\n\t"
        "v_perm_b32 %[tA10], %[sA0], %[ls], %[a2]\n\t"
        "v_perm_b32 %[tA11], %[sA1], %[ls], %[a3]\n\t"
        "ds_read_b32 %[nA2], %[nA2] offset:%[o0]\n\t"
        "ds_read_b32 %[tA9], %[tA9] offset:%[o1]\n\t"
        "ds_read_b32 %[tA10], %[tA10] offset:%[o0]\n\t"
        "ds_read_b32 %[tA11], %[tA11] offset:%[o1]\n\t"
        "v_perm_b32 %[nA3], %[sA3], %[ls], %[a0]\n\t"
        "v_perm_b32 %[tA13], %[sA0], %[ls], %[a1]\n\t"
        "v_perm_b32 %[tA14], %[sA1], %[ls], %[a2]\n\t"
        "v_perm_b32 %[tA15], %[sA2], %[ls], %[a3]\n\t"
        "ds_read_b32 %[nA3], %[nA3] offset:%[o0]\n\t"
        "ds_read_b32 %[tA13], %[tA13] offset:%[o1]\n\t"
        "ds_read_b32 %[tA14], %[tA14] offset:%[o0]\n\t"
        "ds_read_b32 %[tA15], %[tA15] offset:%[o1]\n\t"
        "v_perm_b32 %[nB0], %[sB0], %[ls], %[a0]\n\t"
        "v_perm_b32 %[tB1], %[sB1], %[ls], %[a1]\n\t"
        "v_perm_b32 %[tB2], %[sB2], %[ls], %[a2]\n\t"
        "v_perm_b32 %[tB3], %[sB3], %[ls], %[a3]\n\t"
        "v_perm_b32 %[nB1], %[sB1], %[ls], %[a0]\n\t"
        "v_perm_b32 %[tB5], %[sB2], %[ls], %[a1]\n\t"
        "v_perm_b32 %[tB6], %[sB3], %[ls], %[a2]\n\t"
        "v_perm_b32 %[tB7], %[sB0], %[ls], %[a3]\n\t"
        "v_perm_b32 %[nB2], %[sB2], %[ls], %[a0]\n\t"
        "v_perm_b32 %[tB9], %[sB3], %[ls], %[a1]\n\t"
        "v_perm_b32 %[tB10], %[sB0], %[ls], %[a2]\n\t"
        "v_perm_b32 %[tB11], %[sB1], %[ls], %[a3]\n\t"
        "v_perm_b32 %[nB3], %[sB3], %[ls], %[a0]\n\t"
        "v_perm_b32 %[tB13], %[sB0], %[ls], %[a1]\n\t"
        "v_perm_b32 %[tB14], %[sB1], %[ls], %[a2]\n\t"
        "v_perm_b32 %[tB15], %[sB2], %[ls], %[a3]\n\t"
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_xor_b32 %[tA2], %[tA2], %[tA3]\n\t"
        "v_bitop3_b32 %[nA0], %[nA0], %[tA1], %[k0] bitop3:0x96\n\t"
        "v_alignbit_b32 %[tA2], %[tA2], %[tA2], 16\n\t"
        "v_xor_b32 %[nA0], %[nA0], %[tA2]\n\t"
        "ds_read_b32 %[nB0], %[nB0] offset:%[o0]\n\t"
        "ds_read_b32 %[tB1], %[tB1] offset:%[o1]\n\t"
        "ds_read_b32 %[tB2], %[tB2] offset:%[o0]\n\t"
        "ds_read_b32 %[tB3], %[tB3] offset:%[o1]\n\t"
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_xor_b32 %[tA6], %[tA6], %[tA7]\n\t"
        "v_bitop3_b32 %[nA1], %[nA1], %[tA5], %[k1] bitop3:0x96\n\t"
        "v_alignbit_b32 %[tA6], %[tA6], %[tA6], 16\n\t"
        "v_xor_b32 %[nA1], %[nA1], %[tA6]\n\t"
        "ds_read_b32 %[nB1], %[nB1] offset:%[o0]\n\t"
        "ds_read_b32 %[tB5], %[tB5] offset:%[o1]\n\t"
        "ds_read_b32 %[tB6], %[tB6] offset:%[o0]\n\t"
        "ds_read_b32 %[tB7], %[tB7] offset:%[o1]\n\t"
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_xor_b32 %[tA10], %[tA10], %[tA11]\n\t"
        "v_bitop3_b32 %[nA2], %[nA2], %[tA9], %[k2] bitop3:0x96\n\t"
        "v_alignbit_b32 %[tA10], %[tA10], %[tA10], 16\n\t"
        "v_xor_b32 %[nA2], %[nA2], %[tA10]\n\t"
        "ds_read_b32 %[nB2], %[nB2] offset:%[o0]\n\t"
        "ds_read_b32 %[tB9], %[tB9] offset:%[o1]\n\t"
        "ds_read_b32 %[tB10], %[tB10] offset:%[o0]\n\t"
        "ds_read_b32 %[tB11], %[tB11] offset:%[o1]\n\t"
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_xor_b32 %[tA14], %[tA14], %[tA15]\n\t"
        "v_bitop3_b32 %[nA3], %[nA3], %[tA13], %[k3] bitop3:0x96\n\t"
        "v_alignbit_b32 %[tA14], %[tA14], %[tA14], 16\n\t"
        "v_xor_b32 %[nA3], %[nA3], %[tA14]\n\t"
        "ds_read_b32 %[nB3], %[nB3] offset:%[o0]\n\t"
        "ds_read_b32 %[tB13], %[tB13] offset:%[o1]\n\t"
        "ds_read_b32 %[tB14], %[tB14] offset:%[o0]\n\t"
        "ds_read_b32 %[tB15], %[tB15] offset:%[o1]\n\t"
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_xor_b32 %[tB2], %[tB2], %[tB3]\n\t"
        "v_bitop3_b32 %[nB0], %[nB0], %[tB1], %[k0] bitop3:0x96\n\t"
        "v_alignbit_b32 %[tB2], %[tB2], %[tB2], 16\n\t"
        "v_xor_b32 %[nB0], %[nB0], %[tB2]\n\t"
        "s_waitcnt lgkmcnt(8)\n\t"
        "v_xor_b32 %[tB6], %[tB6], %[tB7]\n\t"
        "v_bitop3_b32 %[nB1], %[nB1], %[tB5], %[k1] bitop3:0x96\n\t"
        "v_alignbit_b32 %[tB6], %[tB6], %[tB6], 16\n\t"
        "v_xor_b32 %[nB1], %[nB1], %[tB6]\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        "v_xor_b32 %[tB10], %[tB10], %[tB11]\n\t"
        "v_bitop3_b32 %[nB2], %[nB2], %[tB9], %[k2] bitop3:0x96\n\t"
        "v_alignbit_b32 %[tB10], %[tB10], %[tB10], 16\n\t"
        "v_xor_b32 %[nB2], %[nB2], %[tB10]\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_xor_b32 %[tB14], %[tB14], %[tB15]\n\t"
        "v_bitop3_b32 %[nB3], %[nB3], %[tB13], %[k3] bitop3:0x96\n\t"
        "v_alignbit_b32 %[tB14], %[tB14], %[tB14], 16\n\t"
        "v_xor_b32 %[nB3], %[nB3], %[tB14]"
        : [nA0] "=&v"(nA[0]), [nA1] "=&v"(nA[1]), [nA2] "=&v"(nA[2]), [nA3] "=&v"(nA[3]), [nB0] "=&v"(nB[0]),
          [nB1] "=&v"(nB[1]), [nB2] "=&v"(nB[2]), [nB3] "=&v"(nB[3]), [tA1] "=&v"(tA1), [tA2] "=&v"(tA2),
          [tA3] "=&v"(tA3), [tA5] "=&v"(tA5), [tA6] "=&v"(tA6), [tA7] "=&v"(tA7), [tA9] "=&v"(tA9),
          [tA10] "=&v"(tA10), [tA11] "=&v"(tA11), [tA13] "=&v"(tA13), [tA14] "=&v"(tA14), [tA15] "=&v"(tA15),
          [tB1] "=&v"(tB1), [tB2] "=&v"(tB2), [tB3] "=&v"(tB3), [tB5] "=&v"(tB5), [tB6] "=&v"(tB6), [tB7] "=&v"(tB7),
          [tB9] "=&v"(tB9), [tB10] "=&v"(tB10), [tB11] "=&v"(tB11), [tB13] "=&v"(tB13), [tB14] "=&v"(tB14),
          [tB15] "=&v"(tB15)
        : [sA0] "v"(sA[0]), [sA1] "v"(sA[1]), [sA2] "v"(sA[2]), [sA3] "v"(sA[3]), [sB0] "v"(sB[0]), [sB1] "v"(sB[1]),
          [sB2] "v"(sB[2]), [sB3] "v"(sB[3]), [ls] "v"(ls), [k0] "s"(k[0]), [k1] "s"(k[1]), [k2] "s"(k[2]),
          [k3] "s"(k[3]), [a0] "s"(0x0c0c0400u), [a1] "s"(0x0c0c0500u), [a2] "s"(0x0c0c0600u), [a3] "s"(0x0c0c0700u),
          [o0] "i"(BASE), [o1] "i"(BASE + 128u)
        : "memory");
}

/*
 * A middle round on the two-table image for the GH8 layout: the image is reached through byte 2 of the lane selector
 * (selectors 0x0c02....), and the round key enters before the rotation, kr = rotl16(k) (wave-uniform):
 *     column = T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d] ^ kr)
 * three VALU per column (xor3, rotate, xor3) instead of aes_round_tt2_asm's four.
 */
__device__ __forceinline__ void aes_round_tt2k_asm(uint32_t ls, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3,
                                                   const uint32_t *kr, uint32_t &n0, uint32_t &n1, uint32_t &n2,
                                                   uint32_t &n3)
{
    uint32_t t1, t2, t3, t5, t6, t7, t9, t10, t11, t13, t14, t15;
    asm volatile(
        GCM_PRIO_HI
        "v_perm_b32 %[n0], %[s0], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t1], %[s1], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t2], %[s2], %[ls], %[a2]\n\t"
        "v_perm_b32 %[t3], %[s3], %[ls], %[a3]\n\t"
        "ds_read_b32 %[n0], %[n0]\n\t"
        "ds_read_b32 %[t1], %[t1] offset:128\n\t"
        "ds_read_b32 %[t2], %[t2]\n\t"
        "ds_read_b32 %[t3], %[t3] offset:128\n\t"
        "v_perm_b32 %[n1], %[s1], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t5], %[s2], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t6], %[s3], %[ls], %[a2]\n\t"
        "v_perm_b32 %[t7], %[s0], %[ls], %[a3]\n\t"
        "ds_read_b32 %[n1], %[n1]\n\t"
        "ds_read_b32 %[t5], %[t5] offset:128\n\t"
        "ds_read_b32 %[t6], %[t6]\n\t"
        "ds_read_b32 %[t7], %[t7] offset:128\n\t"
        "v_perm_b32 %[n2], %[s2], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t9], %[s3], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t10], %[s0], %[ls], %[a2]\n\t"
        "v_perm_b32 %[t11], %[s1], %[ls], %[a3]\n\t"
        "ds_read_b32 %[n2], %[n2]\n\t"
        "ds_read_b32 %[t9], %[t9] offset:128\n\t"
        "ds_read_b32 %[t10], %[t10]\n\t"
        "ds_read_b32 %[t11], %[t11] offset:128\n\t"
        "v_perm_b32 %[n3], %[s3], %[ls], %[a0]\n\t"
        "v_perm_b32 %[t13], %[s0], %[ls], %[a1]\n\t"
        "v_perm_b32 %[t14], %[s1], %[ls], %[a2]\n\t"
        "v_perm_b32 %[t15], %[s2], %[ls], %[a3]\n\t"
        "ds_read_b32 %[n3], %[n3]\n\t"
        "ds_read_b32 %[t13], %[t13] offset:128\n\t"
        "ds_read_b32 %[t14], %[t14]\n\t"
        "ds_read_b32 %[t15], %[t15] offset:128\n\t"
        GCM_PRIO_LO
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_bitop3_b32 %[t2], %[t2], %[t3], %[r0] bitop3:0x96\n\t"
        "v_alignbit_b32 %[t2], %[t2], %[t2], 16\n\t"
        "v_bitop3_b32 %[n0], %[n0], %[t1], %[t2] bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(8)\n\t"
        "v_bitop3_b32 %[t6], %[t6], %[t7], %[r1] bitop3:0x96\n\t"
        "v_alignbit_b32 %[t6], %[t6], %[t6], 16\n\t"
        "v_bitop3_b32 %[n1], %[n1], %[t5], %[t6] bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        "v_bitop3_b32 %[t10], %[t10], %[t11], %[r2] bitop3:0x96\n\t"
        "v_alignbit_b32 %[t10], %[t10], %[t10], 16\n\t"
        "v_bitop3_b32 %[n2], %[n2], %[t9], %[t10] bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_bitop3_b32 %[t14], %[t14], %[t15], %[r3] bitop3:0x96\n\t"
        "v_alignbit_b32 %[t14], %[t14], %[t14], 16\n\t"
        "v_bitop3_b32 %[n3], %[n3], %[t13], %[t14] bitop3:0x96"
        : [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2), [n3] "=&v"(n3), [t1] "=&v"(t1), [t2] "=&v"(t2),
          [t3] "=&v"(t3), [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7), [t9] "=&v"(t9), [t10] "=&v"(t10),
          [t11] "=&v"(t11), [t13] "=&v"(t13), [t14] "=&v"(t14), [t15] "=&v"(t15)
        : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [ls] "v"(ls), [r0] "s"(kr[0]), [r1] "s"(kr[1]),
          [r2] "s"(kr[2]), [r3] "s"(kr[3]), [a0] "s"(0x0c020400u), [a1] "s"(0x0c020500u), [a2] "s"(0x0c020600u),
          [a3] "s"(0x0c020700u)
        : "memory");
}

#endif

/*
 * 8-bit latin GHASH tables (Layout<4>::gh8).  Multiplication by a constant c is GF(2)-linear, so
 * X * c = XOR over the 16 byte positions p of T_p[X_p], T_p[e] = (e at byte p of X) * c.  The 64 KiB table at LDS 0 has
 * T_p[e] at row e (256 B, one full bank row of the 64 banks), slot p: bank group p.  A ds_read_b128 is served 16
 * consecutive lanes at a time; lane i (= lane & 15) takes, at read r (0..15), byte position r ^ i of its X, so the 16
 * lanes of a pass always hit 16 distinct bank groups, whatever their bytes: conflict-free, 16 reads per multiply
 * against the nibble tables' 32 (whose rows are per nibble position, so 16 lanes on one row conflict only through
 * equal entries, which broadcast).  The lane multiplies X with its bytes permuted by i (gh8_rotate: byte r of Xr =
 * byte r ^ i of X; 8 v_cndmask swap the dwords, 4 v_perm with a lane selector swap the bytes); read r's address is one
 * v_perm of byte r & 3 of dword r >> 2 and of byte r & 3 of C_q = Ci ^ K_q (q = r >> 2, one v_xor per four reads),
 * ((r ^ i) << 4).  The product is the same for every i (measured bit-exact against the nibble tables by
 * scripts/probe_gh8.py, and through every batch-kernel suite).
 */
#ifndef GCM_GH8_LANESEL
#define GCM_GH8_LANESEL 0 /* 1: the byte part of the permutation in per-lane address selectors (4 VGPRs, 4 VALU less) */
#endif
struct Gh8Lane {
    uint32_t selL; /* v_perm selector: byte b <- byte b ^ (i & 3) */
    uint32_t Ci;   /* (i << 4) in every byte */
    bool q1, q2;   /* bits 2 and 3 of i: the dword swaps */
#if GCM_GH8_LANESEL
    uint32_t selv[4]; /* read 4q + s: address byte 1 <- byte s ^ (i & 3) of dword q, byte 0 <- byte s of C_q */
#endif
};

GCM_HD Gh8Lane gh8_lane(uint32_t i)
{
    Gh8Lane L;
    i &= 15u;
    L.selL = 0x03020100u ^ ((i & 3u) * 0x01010101u);
    L.Ci = (i << 4) * 0x01010101u;
    L.q1 = (i & 4u) != 0u;
    L.q2 = (i & 8u) != 0u;
#if GCM_GH8_LANESEL
    for (uint32_t t = 0; t < 4u; ++t)
        L.selv[t] = 0x0c0c0000u | ((t ^ (i & 3u)) << 8) | (4u + t);
#endif
    return L;
}

/* byte r of the result = byte r ^ i of X (GCM_GH8_LANESEL: only the dwords; the bytes by the address selectors) */
GCM_HD u32x4 gh8_rotate(const u32x4 &X, const Gh8Lane &L)
{
    const uint32_t v0 = L.q1 ? X[1] : X[0], v1 = L.q1 ? X[0] : X[1], v2 = L.q1 ? X[3] : X[2], v3 = L.q1 ? X[2] : X[3];
    const uint32_t w0 = L.q2 ? v2 : v0, w1 = L.q2 ? v3 : v1, w2 = L.q2 ? v0 : v2, w3 = L.q2 ? v1 : v3;
#if GCM_GH8_LANESEL
    return u32x4{w0, w1, w2, w3};
#else
    return u32x4{perm(w0, w0, L.selL), perm(w1, w1, L.selL), perm(w2, w2, L.selL), perm(w3, w3, L.selL)};
#endif
}

/* byte s of K_q = (4q + s) << 4 */
GCM_HDC uint32_t gh8_kq(int q)
{
    return ((uint32_t)(4 * q) << 4) * 0x01010101u + 0x30201000u;
}

/* reads r, r + 1 of the multiply of the rotated Xr */
GCM_HD void gh8_issue2(const uint8_t *lds, const u32x4 &Xr, const Gh8Lane &L, int r, u32x4 g[2])
{
    const uint32_t C = L.Ci ^ gh8_kq(r >> 2); /* r even: both reads in dword r >> 2 */
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int rr = r + t;
#if GCM_GH8_LANESEL
        const uint32_t sel = L.selv[rr & 3];
#else
        const uint32_t sel = 0x0c0c0000u | ((uint32_t)(rr & 3) << 8) | (4u + (uint32_t)(rr & 3));
#endif
        g[t] = lds_u32x4(lds, perm(C, Xr[rr >> 2], sel));
    }
}

GCM_HD void gh8_acc2(const u32x4 g[2], u32x4 &P)
{
    P[0] = xor3_pinned(P[0], g[0][0], g[1][0]);
    P[1] = xor3_pinned(P[1], g[0][1], g[1][1]);
    P[2] = xor3_pinned(P[2], g[0][2], g[1][2]);
    P[3] = xor3_pinned(P[3], g[0][3], g[1][3]);
}

/* X * H^4 from the GH8 table, not fused */
GCM_HD u32x4 gh8_mul_lds(const uint8_t *lds, const u32x4 &X, const Gh8Lane &L)
{
    const u32x4 Xr = gh8_rotate(X, L);
    u32x4 P = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
        u32x4 g[2];
        gh8_issue2(lds, Xr, L, r, g);
        gh8_acc2(g, P);
    }
    return P;
}

/*
 * AES of w (in place) fused with P = A * c (nibble tables of c at basereg): the GHASH reads are
 * independent of the AES chain and are issued in rounds 1..8, four per round, so each wave keeps
 * ~20 LDS reads in flight per round instead of 16.  Bit-identical to aes_encrypt_tt + ghash_mul_lds.
 */
template <int NR, bool FOUR = true>
GCM_HD u32x4 aes_ghash_fused(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, uint32_t w[4], uint32_t basereg, u32x4 A)
{
#define GCM_TA(x, k) perm((x), lanesel, 0x0c0c0400u | ((4u + (k)) << 8))
#define GCM_TB(x, k) perm((x), lanesel, 0x0c020400u | ((4u + (k)) << 8))
    u32x4 P = {0u, 0u, 0u, 0u};
    uint32_t s0 = w[0] ^ rk[0], s1 = w[1] ^ rk[1], s2 = w[2] ^ rk[2], s3 = w[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        const uint32_t *k = rk + 4 * r;
        uint32_t n0 = aes_col<FOUR>(lds, lanesel, s0, s1, s2, s3, k[0]);
        uint32_t n1 = aes_col<FOUR>(lds, lanesel, s1, s2, s3, s0, k[1]);
        uint32_t n2 = aes_col<FOUR>(lds, lanesel, s2, s3, s0, s1, k[2]);
        uint32_t n3 = aes_col<FOUR>(lds, lanesel, s3, s0, s1, s2, k[3]);
        if (r <= 8)
            ghash_quarter(lds, basereg, A[(r - 1) >> 1], (r - 1) >> 1, ((r - 1) & 1) * 2, P);
        GCM_SCHED_FENCE();
        s0 = n0;
        s1 = n1;
        s2 = n2;
        s3 = n3;
    }
    {
        const uint32_t *k = rk + 4 * NR;
        uint32_t x[4] = {s0, s1, s2, s3};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t ra = lds_u32(lds, GCM_TA(x[j], 0));
            uint32_t rb = lds_u32(lds, GCM_TA(x[(j + 1) & 3], 1));
            uint32_t rc = lds_u32(lds, GCM_TA(x[(j + 2) & 3], 2));
            uint32_t rd = lds_u32(lds, GCM_TA(x[(j + 3) & 3], 3));
            w[j] = xor3(perm(rb, ra, 0x0c0c0501u), perm(rd, rc, 0x06020c0cu), k[j]);
        }
    }
    return P;
#undef GCM_TA
#undef GCM_TB
}

/* T_t[byte kk of x] from the 4-table or the 2-table image; B2: selector of the address's byte 2 (Layout::aes_b2) */
template <bool FOUR, uint32_t B2 = 0x0cu>
GCM_HD uint32_t tlook(const uint8_t *lds, uint32_t lanesel, uint32_t x, uint32_t kk, int t)
{
    const uint32_t a = perm(x, lanesel, 0x0c000400u | (B2 << 16) | ((4u + kk) << 8));
    if (t == 0)
        return lds_u32(lds, a);
    if (t == 1)
        return lds_u32(lds, a + 128);
    if (FOUR) {
        const uint32_t b = perm(x, lanesel, 0x0c020400u | ((4u + kk) << 8));
        return lds_u32(lds, t == 2 ? b : b + 128);
    }
    return rotl32(lds_u32(lds, t == 2 ? a : a + 128), 16);
}

/*
 * CTR-mode round-1 hoisting.  The AES input of every block of a record is nonce || BE32(ctr): the
 * first 12 bytes never change, and inside a 2^16-block window neither do ctr's two high bytes
 * (every TLS record lies in the first window).  Round 1 then has only two table reads that depend
 * on the block (T3 of the counter's low byte for column 0, T2 of its next byte for column 1);
 * everything else of round 1 is folded into four constants c[0..3], recomputed when the window
 * changes.
 */
template <bool FOUR>
GCM_HD void aes_round1_consts(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, uint32_t iv0, uint32_t iv1,
                              uint32_t iv2, uint32_t ctr_hi, uint32_t c[4])
{
    /* ctr_hi = ctr & 0xffff0000: the two counter bytes that are constant inside a 2^16-block window */
    const uint32_t s0 = iv0 ^ rk[0], s1 = iv1 ^ rk[1], s2 = iv2 ^ rk[2], s3 = bswap32(ctr_hi) ^ rk[3];
    const uint32_t *k = rk + 4;
    c[0] = xor3(tlook<FOUR>(lds, lanesel, s0, 0, 0), tlook<FOUR>(lds, lanesel, s1, 1, 1),
                tlook<FOUR>(lds, lanesel, s2, 2, 2) ^ k[0]);
    c[1] = xor3(tlook<FOUR>(lds, lanesel, s1, 0, 0), tlook<FOUR>(lds, lanesel, s2, 1, 1),
                tlook<FOUR>(lds, lanesel, s0, 3, 3) ^ k[1]);
    c[2] = xor3(xor3(tlook<FOUR>(lds, lanesel, s2, 0, 0), tlook<FOUR>(lds, lanesel, s3, 1, 1), k[2]),
                tlook<FOUR>(lds, lanesel, s0, 2, 2), tlook<FOUR>(lds, lanesel, s1, 3, 3));
    c[3] = xor3(xor3(tlook<FOUR>(lds, lanesel, s3, 0, 0), tlook<FOUR>(lds, lanesel, s0, 1, 1), k[3]),
                tlook<FOUR>(lds, lanesel, s1, 2, 2), tlook<FOUR>(lds, lanesel, s2, 3, 3));
}

/*
 * CTR caching over rounds 1 AND 2 (GCM_R2CACHE): inside a 2^8-block window only the counter's low
 * byte (state byte 15: row 3 of column 3) changes.  ShiftRows moves it to column 0, so after round 1
 * only column 0 varies (n0 = c[0] ^ T3[x]); in round 2 every output column takes exactly one byte of
 * that column (m0 <- n0.b0 via T0, m3 <- n0.b1 via T1, m2 <- n0.b2 via T2, m1 <- n0.b3 via T3), and
 * its three other terms plus the round key are constants c[4..7].  Per block: 1 + 4 table reads for
 * rounds 1-2 instead of 2 + 16.  c[0..7] are recomputed when ctr & 0xffffff00 changes.
 */
template <bool FOUR, uint32_t B2 = 0x0cu>
GCM_HD void aes_round12_consts(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, uint32_t iv0, uint32_t iv1,
                               uint32_t iv2, uint32_t ctr_hi, uint32_t c[8])
{
#define GCM_TL(x, kk, t) tlook<FOUR, B2>(lds, lanesel, (x), (kk), (t))
    /* ctr_hi = ctr & 0xffffff00 */
    const uint32_t s0 = iv0 ^ rk[0], s1 = iv1 ^ rk[1], s2 = iv2 ^ rk[2], s3 = bswap32(ctr_hi) ^ rk[3];
    const uint32_t *k = rk + 4;
    c[0] = xor3(GCM_TL(s0, 0, 0), GCM_TL(s1, 1, 1), GCM_TL(s2, 2, 2) ^ k[0]); /* + T3[s3.b3] per block */
    const uint32_t n1 = xor3(xor3(GCM_TL(s1, 0, 0), GCM_TL(s2, 1, 1), k[1]), GCM_TL(s3, 2, 2), GCM_TL(s0, 3, 3));
    const uint32_t n2 = xor3(xor3(GCM_TL(s2, 0, 0), GCM_TL(s3, 1, 1), k[2]), GCM_TL(s0, 2, 2), GCM_TL(s1, 3, 3));
    const uint32_t n3 = xor3(xor3(GCM_TL(s3, 0, 0), GCM_TL(s0, 1, 1), k[3]), GCM_TL(s1, 2, 2), GCM_TL(s2, 3, 3));
    c[1] = n1;
    c[2] = n2;
    c[3] = n3;
    const uint32_t *k2 = rk + 8;
    c[4] = xor3(GCM_TL(n1, 1, 1), GCM_TL(n2, 2, 2), GCM_TL(n3, 3, 3) ^ k2[0]); /* + T0[n0.b0] */
    c[5] = xor3(GCM_TL(n1, 0, 0), GCM_TL(n2, 1, 1), GCM_TL(n3, 2, 2) ^ k2[1]); /* + T3[n0.b3] */
    c[6] = xor3(GCM_TL(n2, 0, 0), GCM_TL(n3, 1, 1), GCM_TL(n1, 3, 3) ^ k2[2]); /* + T2[n0.b2] */
    c[7] = xor3(GCM_TL(n3, 0, 0), GCM_TL(n1, 2, 2), GCM_TL(n2, 3, 3) ^ k2[3]); /* + T1[n0.b1] */
#undef GCM_TL
}

/*
 * aes_ghash_fused for a block whose round 1 is hoisted (c from the block's 2^16 window): 2 table reads in round 1
 * instead of 16; the GHASH reads go to rounds 2..9.  Writes the keystream to w[4].
 * GH5: P = A * H^4 from the 5-bit tables at LDS 0 (eight slots of 3-4 chunks); otherwise from the nibble
 * tables at basereg (eight quarters).  AES_BASE: LDS address of the AES images.
 */
template <int NR, bool FOUR = true, bool GH5 = false, uint32_t AES_BASE = 0u>
GCM_HD u32x4 aes_ghash_fused_h(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, const uint32_t *c,
                               uint32_t ctr, uint32_t w[4], uint32_t basereg, u32x4 A)
{
#define GCM_TA(x, k) perm((x), lanesel, 0x0c0c0400u | ((4u + (k)) << 8))
    const uint8_t *la = lds + AES_BASE;
    u32x4 P = {0u, 0u, 0u, 0u};
    const uint32_t s3 = bswap32(ctr) ^ rk[3];
#if GCM_R2CACHE
    /* rounds 1 and 2 from the window constants c[0..7] (aes_round12_consts): 5 reads */
    const uint32_t n0 = c[0] ^ tlook<FOUR>(la, lanesel, s3, 3, 3);
    uint32_t s0 = c[4] ^ tlook<FOUR>(la, lanesel, n0, 0, 0), s1 = c[5] ^ tlook<FOUR>(la, lanesel, n0, 3, 3);
    uint32_t s2 = c[6] ^ tlook<FOUR>(la, lanesel, n0, 2, 2), s3r = c[7] ^ tlook<FOUR>(la, lanesel, n0, 1, 1);
    if (GH5) {
        u32x2 g5[8];
        gh5_issue(lds, A, gh5_slot_first(0), gh5_slot_count(0), g5);
        gh5_acc(g5, gh5_slot_count(0), P);
    } else {
        ghash_quarter(lds, basereg, A[0], 0, 0, P);
    }
    GCM_SCHED_FENCE();
    constexpr int R0 = 3;
#else
    uint32_t s0 = c[0] ^ tlook<FOUR>(la, lanesel, s3, 3, 3), s1 = c[1] ^ tlook<FOUR>(la, lanesel, s3, 2, 2);
    uint32_t s2 = c[2], s3r = c[3];
    constexpr int R0 = 2;
#endif
#pragma unroll
    for (int r = R0; r < NR; ++r) {
        const uint32_t *k = rk + 4 * r;
        uint32_t n0, n1, n2, n3;
#if defined(__HIP_DEVICE_COMPILE__) && GCM_ROUND_ASM
        if (true) {
            /* GHASH slot: reads issued ahead of the round, accumulated after it */
            if (GH5 && FOUR) {
                u32x2 g5[8];
                if (r <= 9)
                    gh5_issue(lds, A, gh5_slot_first(r - 2), gh5_slot_count(r - 2), g5);
                aes_round_tt4_asm<AES_BASE>(lanesel, s0, s1, s2, s3r, k, n0, n1, n2, n3);
                if (r <= 9)
                    gh5_acc(g5, gh5_slot_count(r - 2), P);
            } else {
                u32x4 g[4];
                if (r <= 9)
                    ghash_quarter_issue(lds, basereg, A[(r - 2) >> 1], (r - 2) >> 1, ((r - 2) & 1) * 2, g);
                if (FOUR)
                    aes_round_tt4_asm<AES_BASE>(lanesel, s0, s1, s2, s3r, k, n0, n1, n2, n3);
                else
                    aes_round_tt2_asm<AES_BASE>(lanesel, s0, s1, s2, s3r, k, n0, n1, n2, n3);
                if (r <= 9)
                    ghash_quarter_acc(g, P);
            }
        } else
#endif
        {
            n0 = aes_col<FOUR>(la, lanesel, s0, s1, s2, s3r, k[0]);
            n1 = aes_col<FOUR>(la, lanesel, s1, s2, s3r, s0, k[1]);
            n2 = aes_col<FOUR>(la, lanesel, s2, s3r, s0, s1, k[2]);
            n3 = aes_col<FOUR>(la, lanesel, s3r, s0, s1, s2, k[3]);
            if (r <= 9) {
                if (GH5) {
                    u32x2 g5[8];
                    gh5_issue(lds, A, gh5_slot_first(r - 2), gh5_slot_count(r - 2), g5);
                    gh5_acc(g5, gh5_slot_count(r - 2), P);
                } else {
                    ghash_quarter(lds, basereg, A[(r - 2) >> 1], (r - 2) >> 1, ((r - 2) & 1) * 2, P);
                }
            }
        }
        GCM_SCHED_FENCE();
        s0 = n0;
        s1 = n1;
        s2 = n2;
        s3r = n3;
    }
    {
        const uint32_t *k = rk + 4 * NR;
        uint32_t x[4] = {s0, s1, s2, s3r};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint32_t ra = lds_u32(la, GCM_TA(x[j], 0));
            uint32_t rb = lds_u32(la, GCM_TA(x[(j + 1) & 3], 1));
            uint32_t rc = lds_u32(la, GCM_TA(x[(j + 2) & 3], 2));
            uint32_t rd = lds_u32(la, GCM_TA(x[(j + 3) & 3], 3));
            w[j] = xor3(perm(rb, ra, 0x0c0c0501u), perm(rd, rc, 0x06020c0cu), k[j]);
        }
    }
    return P;
#undef GCM_TA
}

/*
 * aes_ghash_fused_h for the GH8 layout (Layout<4>::gh8): the AES on the two-table image at 64K (selectors take byte 2
 * of lanesel; middle rounds aes_round_tt2k_asm with kr = rotl16 of the round keys), P = A * H^4 from the GH8 table:
 * A rotated once (gh8_rotate), its 16 reads issued two per slot -- rounds 1-2, then rounds 3..9 -- ahead of the
 * round's asm block and accumulated after it.  Writes the keystream to w[4].
 */
template <int NR>
GCM_HD u32x4 aes_gh8_fused_h(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, const uint32_t *kr, const uint32_t *c,
                             uint32_t ctr, uint32_t w[4], const u32x4 &A, const Gh8Lane &L)
{
#define GCM_TL(x, kk, t) tlook<false, 0x02u>(lds, lanesel, (x), (kk), (t))
    const u32x4 Ar = gh8_rotate(A, L);
    u32x4 P = {0u, 0u, 0u, 0u};
    const uint32_t s3 = bswap32(ctr) ^ rk[3];
    /* rounds 1 and 2 from the window constants c[0..7] (aes_round12_consts): 5 reads */
    const uint32_t n0 = c[0] ^ GCM_TL(s3, 3, 3);
    uint32_t s0 = c[4] ^ GCM_TL(n0, 0, 0), s1 = c[5] ^ GCM_TL(n0, 3, 3);
    uint32_t s2 = c[6] ^ GCM_TL(n0, 2, 2), s3r = c[7] ^ GCM_TL(n0, 1, 1);
    {
        u32x4 g[2];
        gh8_issue2(lds, Ar, L, 0, g);
        gh8_acc2(g, P);
    }
    GCM_SCHED_FENCE();
#pragma unroll
    for (int r = 3; r < NR; ++r) {
        uint32_t n[4];
        u32x4 g[2];
#if defined(__HIP_DEVICE_COMPILE__) && GCM_ROUND_PRIO && GCM_PRIO_GH8
        asm volatile(GCM_PRIO_HI ::: "memory");
        GCM_SCHED_FENCE();
#endif
        if (r <= 9)
            gh8_issue2(lds, Ar, L, 2 * (r - 2), g);
#if defined(__HIP_DEVICE_COMPILE__) && GCM_ROUND_ASM
#if GCM_GH8_KR_SALU
        /* rotl16 of the round keys on the scalar unit, here, rather than 44-60 more live SGPRs */
        uint32_t krr[4];
        for (int col = 0; col < 4; ++col) {
            uint32_t t;
            asm("s_lshl_b32 %0, %2, 16\n\ts_pack_hh_b32_b16 %1, %2, %0" : "=&s"(t), "=s"(krr[col]) : "s"(rk[4 * r + col]));
        }
        aes_round_tt2k_asm(lanesel, s0, s1, s2, s3r, krr, n[0], n[1], n[2], n[3]);
#else
        aes_round_tt2k_asm(lanesel, s0, s1, s2, s3r, kr + 4 * r, n[0], n[1], n[2], n[3]);
#endif
#else
        {
            const uint32_t s[4] = {s0, s1, s2, s3r}, *k = rk + 4 * r;
            for (int col = 0; col < 4; ++col)
                n[col] = xor3(GCM_TL(s[col], 0, 0), GCM_TL(s[(col + 1) & 3], 1, 1), GCM_TL(s[(col + 2) & 3], 2, 2)) ^
                         GCM_TL(s[(col + 3) & 3], 3, 3) ^ k[col];
            (void)kr;
        }
#endif
        if (r <= 9)
            gh8_acc2(g, P);
        GCM_SCHED_FENCE();
        s0 = n[0];
        s1 = n[1];
        s2 = n[2];
        s3r = n[3];
    }
    {
#if defined(__HIP_DEVICE_COMPILE__) && GCM_ROUND_PRIO && GCM_PRIO_LAST
        asm volatile(GCM_PRIO_HI ::: "memory");
        GCM_SCHED_FENCE();
#endif
        const uint32_t *k = rk + 4 * NR;
        const uint32_t x[4] = {s0, s1, s2, s3r};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            /* S[x] is byte 1 (and 2) of T0[x]: all four reads from T0 */
            const uint32_t ra = lds_u32(lds, perm(x[j], lanesel, 0x0c020400u));
            const uint32_t rb = lds_u32(lds, perm(x[(j + 1) & 3], lanesel, 0x0c020500u));
            const uint32_t rc = lds_u32(lds, perm(x[(j + 2) & 3], lanesel, 0x0c020600u));
            const uint32_t rd = lds_u32(lds, perm(x[(j + 3) & 3], lanesel, 0x0c020700u));
            w[j] = xor3(perm(rb, ra, 0x0c0c0501u), perm(rd, rc, 0x06020c0cu), k[j]);
        }
#if defined(__HIP_DEVICE_COMPILE__) && GCM_ROUND_PRIO && GCM_PRIO_LAST
        GCM_SCHED_FENCE();
        asm volatile(GCM_PRIO_LO ::: "memory");
#endif
    }
    return P;
#undef GCM_TL
}

/*
 * Keystreams of two counter blocks of one record (ctrA, ctrB) with the two-table layout, their rounds interleaved
 * (aes_round_tt2_asm_x2): rounds 1-2 from the window constants cA / cB (aes_round12_consts of each block's window),
 * rounds 3..NR-1 two states per asm block, the last round for both.  Bit-identical to two aes_ghash_fused_h calls'
 * keystreams; no GHASH.
 */
template <int NR, uint32_t AES_BASE = 0u>
GCM_HD void aes_ctr_x2_h(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, const uint32_t *cA, const uint32_t *cB,
                         uint32_t ctrA, uint32_t ctrB, uint32_t wA[4], uint32_t wB[4])
{
#define GCM_TA(x, k) perm((x), lanesel, 0x0c0c0400u | ((4u + (k)) << 8))
    const uint8_t *la = lds + AES_BASE;
    uint32_t sA[4], sB[4];
    {
        const uint32_t a3 = bswap32(ctrA) ^ rk[3], b3 = bswap32(ctrB) ^ rk[3];
        const uint32_t a0 = cA[0] ^ tlook<false>(la, lanesel, a3, 3, 3), b0 = cB[0] ^ tlook<false>(la, lanesel, b3, 3, 3);
        sA[0] = cA[4] ^ tlook<false>(la, lanesel, a0, 0, 0);
        sB[0] = cB[4] ^ tlook<false>(la, lanesel, b0, 0, 0);
        sA[1] = cA[5] ^ tlook<false>(la, lanesel, a0, 3, 3);
        sB[1] = cB[5] ^ tlook<false>(la, lanesel, b0, 3, 3);
        sA[2] = cA[6] ^ tlook<false>(la, lanesel, a0, 2, 2);
        sB[2] = cB[6] ^ tlook<false>(la, lanesel, b0, 2, 2);
        sA[3] = cA[7] ^ tlook<false>(la, lanesel, a0, 1, 1);
        sB[3] = cB[7] ^ tlook<false>(la, lanesel, b0, 1, 1);
    }
#pragma unroll
    for (int r = 3; r < NR; ++r) {
        uint32_t nA[4], nB[4];
#if defined(__HIP_DEVICE_COMPILE__) && GCM_ROUND_ASM
        aes_round_tt2_asm_x2<AES_BASE>(lanesel, sA, sB, rk + 4 * r, nA, nB);
#else
        const uint32_t *k = rk + 4 * r;
        for (int c = 0; c < 4; ++c) {
            nA[c] = aes_col<false>(la, lanesel, sA[c], sA[(c + 1) & 3], sA[(c + 2) & 3], sA[(c + 3) & 3], k[c]);
            nB[c] = aes_col<false>(la, lanesel, sB[c], sB[(c + 1) & 3], sB[(c + 2) & 3], sB[(c + 3) & 3], k[c]);
        }
#endif
        GCM_SCHED_FENCE();
        for (int c = 0; c < 4; ++c) {
            sA[c] = nA[c];
            sB[c] = nB[c];
        }
    }
    const uint32_t *k = rk + 4 * NR;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t ra = lds_u32(la, GCM_TA(sA[j], 0)), rb = lds_u32(la, GCM_TA(sA[(j + 1) & 3], 1));
        const uint32_t rc = lds_u32(la, GCM_TA(sA[(j + 2) & 3], 2)), rd = lds_u32(la, GCM_TA(sA[(j + 3) & 3], 3));
        const uint32_t qa = lds_u32(la, GCM_TA(sB[j], 0)), qb = lds_u32(la, GCM_TA(sB[(j + 1) & 3], 1));
        const uint32_t qc = lds_u32(la, GCM_TA(sB[(j + 2) & 3], 2)), qd = lds_u32(la, GCM_TA(sB[(j + 3) & 3], 3));
        wA[j] = xor3(perm(rb, ra, 0x0c0c0501u), perm(rd, rc, 0x06020c0cu), k[j]);
        wB[j] = xor3(perm(qb, qa, 0x0c0c0501u), perm(qd, qc, 0x06020c0cu), k[j]);
    }
#undef GCM_TA
}

/*
 * r = x * c with the nibble tables of c at LDS byte offset (base: bytes 1..2 of basereg, a multiple of
 * 256 in [128K, 160K)).  32 conflict-free ds_read_b128 + ~108 VALU.
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
            u32x4 e = lds_u32x4(lds, alo + (uint32_t)(8 * d + 2 * m) * 256u);
            u32x4 f = lds_u32x4(lds, ahi + (uint32_t)(8 * d + 2 * m + 1) * 256u);
            r[0] = xor3(r[0], e[0], f[0]);
            r[1] = xor3(r[1], e[1], f[1]);
            r[2] = xor3(r[2], e[2], f[2]);
            r[3] = xor3(r[3], e[3], f[3]);
        }
    }
    return r;
}

/*
 * ghash_mul_lds with all 32 table reads issued before the first XOR: for latency-bound chains (the window
 * kernels' segment join), where the compiler otherwise waits on the reads in small groups.  128 VGPRs of
 * reads in flight, so only for kernels with registers to spare (one wave per SIMD).
 */
GCM_HD u32x4 ghash_mul_lds_wide(const uint8_t *lds, uint32_t basereg, u32x4 x)
{
    u32x4 e[32];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t lo = (x[d] << 4) & 0xf0f0f0f0u, hi = x[d] & 0xf0f0f0f0u;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const uint32_t sel = 0x0c020100u | (4u + (uint32_t)m);
            e[8 * d + 2 * m] = lds_u32x4(lds, perm(lo, basereg, sel) + (uint32_t)(8 * d + 2 * m) * 256u);
            e[8 * d + 2 * m + 1] = lds_u32x4(lds, perm(hi, basereg, sel) + (uint32_t)(8 * d + 2 * m + 1) * 256u);
        }
    }
    GCM_SCHED_FENCE();
    u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 32; i += 2) {
        r[0] = xor3(r[0], e[i][0], e[i + 1][0]);
        r[1] = xor3(r[1], e[i][1], e[i + 1][1]);
        r[2] = xor3(r[2], e[i][2], e[i + 1][2]);
        r[3] = xor3(r[3], e[i][3], e[i + 1][3]);
    }
    return r;
}

/* ghash_mul_lds_wide in two halves of 16 reads (64 VGPRs in flight): kernels at three waves per SIMD */
GCM_HD u32x4 ghash_mul_lds_half(const uint8_t *lds, uint32_t basereg, u32x4 x)
{
    u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        u32x4 e[16];
#pragma unroll
        for (int d = 2 * h; d < 2 * h + 2; ++d) {
            const uint32_t lo = (x[d] << 4) & 0xf0f0f0f0u, hi = x[d] & 0xf0f0f0f0u;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const uint32_t sel = 0x0c020100u | (4u + (uint32_t)m);
                e[8 * (d - 2 * h) + 2 * m] = lds_u32x4(lds, perm(lo, basereg, sel) + (uint32_t)(8 * d + 2 * m) * 256u);
                e[8 * (d - 2 * h) + 2 * m + 1] =
                    lds_u32x4(lds, perm(hi, basereg, sel) + (uint32_t)(8 * d + 2 * m + 1) * 256u);
            }
        }
        GCM_SCHED_FENCE();
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
            r[0] = xor3(r[0], e[i][0], e[i + 1][0]);
            r[1] = xor3(r[1], e[i][1], e[i + 1][1]);
            r[2] = xor3(r[2], e[i][2], e[i + 1][2]);
            r[3] = xor3(r[3], e[i][3], e[i + 1][3]);
        }
    }
    return r;
}

/* the window join's multiply: W = 2 all 32 reads in flight, 1 two halves of 16, 0 compiler-scheduled */
template <int W>
GCM_HD u32x4 ghash_mul_join(const uint8_t *lds, uint32_t basereg, u32x4 x)
{
    if constexpr (W == 2)
        return ghash_mul_lds_wide(lds, basereg, x);
    else if constexpr (W == 1)
        return ghash_mul_lds_half(lds, basereg, x);
    else
        return ghash_mul_lds(lds, basereg, x);
}

/* the closing lane scaling of split_scale layouts: all 32 reads in flight when the kernel has the registers */
template <bool WIDE>
GCM_HD u32x4 ghash_mul_scale(const uint8_t *lds, uint32_t basereg, u32x4 x)
{
    if constexpr (WIDE)
        return ghash_mul_lds_wide(lds, basereg, x);
    else
        return ghash_mul_lds(lds, basereg, x);
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
    /*
     * gh .. gh256 are contiguous, in this order: the 16-lane latency kernels copy them into LDS as one 96 KiB block
     * behind the AES image (LayoutWin16).
     */
    uint8_t gh[MAX_K][32][16][16]; /* gh[p-1] = nibble tables of H^p, p = 1..MAX_K */
    uint8_t gh16[32][16][16];      /* H^16: the Horner factor of 16 lanes per segment (LayoutWin16) */
    uint8_t gh32[32][16][16];      /* H^32 and H^128: the joins of the 32-position segments of the */
    uint8_t gh128[32][16][16];     /* single-record latency kernels (window_body SEG = 32) */
    uint8_t gh256[32][16][16];     /* nibble tables of H^256: joins groups of 4 segments (window_join) */
    uint8_t gh64[32][16][16];      /* nibble tables of H^64: joins the 64-position segments of the window kernels */
    uint8_t gh512[32][16][16];     /* H^256 m, m = 1..4 (gh256, gh512, gh768, gh1024): scale a run of 8 segments */
    uint8_t gh1024[32][16][16];    /* to the record's end, m runs after it (the split window kernels, LayoutSplit) */
    uint8_t gh768[32][16][16];
};
static_assert(offsetof(KeyImage, gh16) == offsetof(KeyImage, gh) + MAX_K * 8192 &&
                  offsetof(KeyImage, gh256) == offsetof(KeyImage, gh16) + 3 * 8192 && offsetof(KeyImage, gh) % 16 == 0,
              "LayoutWin16 / LayoutSplit copy gh .. gh256 (gh128) as one block");

/* ------------------------------------------------------------------ record walk ----------- */

/* The batch descriptor (include/ptls_mi355x.h, ptls_mi355x_record_t). */
struct Record {
    uint64_t src, dst, aad, seq;
    uint32_t len, aadlen;
};

/*
 * Work split of one record over K lanes.  GHASH consumes g = A + C + 1 blocks (AAD blocks,
 * ciphertext blocks, length block) at positions q = pad .. pad + g - 1 of a K x T grid; lane j
 * handles positions j, j+K, ... and Horner-accumulates with factor H^K.  Positions before pad
 * are zero blocks (they do not change a Horner evaluation started from 0); positions from
 * pad + g on are skipped, so lane j's chain ends at its last real position q_last(j) and the
 * chain is scaled by H^(pad + g - q_last(j)), an exponent in [1, K] (GHASH degree of block i is
 * g - i).  The K partial sums are then XOR-reduced.  The same lane runs the AES block of the
 * ciphertext position it hashes; the lane holding the length block computes E_K(J0).
 *
 * pad is free in [0, K): make_walk picks it so that every step's K payload blocks start at a
 * multiple of K blocks of the OUTPUT address (out16 = address / 16), i.e. a step's stores of a
 * record form one aligned 16K-byte piece (64 B at K = 4).  Misaligned pieces straddle two
 * 64-byte segments and measured 1.5-1.6x the algorithmic write traffic and 6-15% lower
 * throughput (scripts/pmc_lengths.py).  Alignment can cost one step; short records
 * (T < GCM_ALIGN_MIN_T) only take it when it is free.
 *
 * AAD hoisting (A <= K, e.g. every TLS record): the AAD blocks sit right before payload block 0, so
 * aligning the payload used to push them into an extra step (1400-B records: 24 steps instead of 23,
 * so alignment was skipped and the stores straddled).  Horner allows a block at lane j's position
 * BEFORE step 0 (grid position j - K): it is simply the lane's starting accumulator, and step 0's
 * fused multiply -- otherwise a multiply of 0 -- raises it by H^K.  So the AAD blocks may sit at
 * negative grid positions (pad = q0 - A < 0, two's complement in the uint32) and lane_walk seeds the
 * lanes that hold them; payload block 0 goes to its aligned grid position q0 = out16 mod K at the
 * minimal step count ceil((q0 + C + 1) / K).
 */
#ifndef GCM_PAIR_STORES
#define GCM_PAIR_STORES 0 /* 1: K = 4 walks store whole 128-byte lines (lane_walk; measured slower) */
#endif
#ifndef GCM_ALIGN_MIN_T
#define GCM_ALIGN_MIN_T 32u
#endif
#ifndef GCM_ALIGN_OUTPUT
#define GCM_ALIGN_OUTPUT 1
#endif
#ifndef GCM_HOIST_AAD
#define GCM_HOIST_AAD 1
#endif
struct Walk {
    uint32_t A, C, T, pad; /* pad: int32 in two's complement (negative: hoisted AAD, or a later window segment) */
};

GCM_HD Walk make_walk(uint32_t len, uint32_t aadlen, uint32_t K, uint32_t out16 = 0xffffffffu)
{
    Walk w;
    w.A = (aadlen + 15u) >> 4;
    w.C = (len + 15u) >> 4;
    /* q0: grid position of payload block 0 (pad = q0 - A); the AAD blocks precede it */
    const uint32_t q0_min = GCM_HOIST_AAD && w.A <= K ? 0u : w.A;
    const uint32_t n = q0_min + w.C + 1u;
    uint32_t q0 = q0_min + (K - n % K) % K; /* minimal step count, the grid ending on a step boundary */
    w.T = (q0 + w.C + 1u) / K;
    if (GCM_ALIGN_OUTPUT && out16 != 0xffffffffu) {
        const uint32_t qa = q0_min + ((out16 - q0_min) & (K - 1u)); /* q0 = out16 (mod K) */
        const uint32_t Ta = (qa + w.C + 1u + K - 1u) / K;
        if (Ta == w.T || w.T >= GCM_ALIGN_MIN_T) {
            q0 = qa;
            w.T = Ta;
        }
    }
    w.pad = q0 - w.A;
    return w;
}

/*
 * table slot (H^(K - slot)) that scales lane j's chain: exponent pad + g - q_last(j).  end_cap bounds the
 * chain to the first end_cap padded positions (a segment of the window kernels, see lane_walk).  Lane j
 * holds grid positions j + K m for m >= -1 (m = -1: a hoisted AAD block, make_walk).
 */
GCM_HD uint32_t walk_scale_slot(const Walk &w, uint32_t j, uint32_t K, uint32_t end_cap = 0xffffffffu)
{
    int32_t end = (int32_t)(w.pad + w.A + w.C + 1u); /* one past the last real position (> 0) */
    if (end_cap != 0xffffffffu && end > (int32_t)end_cap)
        end = (int32_t)end_cap;
    const int32_t e = end - 1 - (int32_t)j;
    if (e < -(int32_t)K)
        return 0u; /* no real position: the chain is 0 */
    const int32_t q_last = (int32_t)j + (e >= 0 ? (int32_t)K * (e / (int32_t)K) : -(int32_t)K);
    return K - (uint32_t)(end - q_last);
}

/*
 * Interior steps of lane j's walk: [lo, hi), the steps t whose position holds a whole payload block read from the
 * input, 0 <= c < len / 16 with c = j + K t - pad - A (len: the payload bytes taken from the input; a FRAME seal's
 * content-type byte is not one).  In those steps lane_walk's step is: counter c + 2, load at in + 16 c, store at
 * out + 16 c, chain ^= ciphertext -- nothing else.  The batch kernels intersect the lanes' ranges over the wave
 * (gcm_batch_body) and pass it to lane_walk, which then takes that path by a scalar branch.
 */
GCM_HD void walk_interior(const Walk &w, uint32_t j, uint32_t K, uint32_t len, uint32_t &lo, uint32_t &hi)
{
    const int32_t cb = (int32_t)j - (int32_t)w.pad - (int32_t)w.A; /* c(t) = cb + K t */
    const int32_t nfull = (int32_t)(len >> 4), k = (int32_t)K;
    lo = cb >= 0 ? 0u : (uint32_t)((k - 1 - cb) / k);          /* ceil(-cb / K): c >= 0 */
    hi = nfull > cb ? (uint32_t)((nfull - cb + k - 1) / k) : 0u; /* K t < nfull - cb: c < nfull */
}

/* the walk's output alignment key: the payload output address in 16-byte units */
GCM_HD uint32_t walk_out16(const uint8_t *out) { return (uint32_t)((uintptr_t)out >> 4); }


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

/* ------------------------------------------------------------------ AES-ECB cipher (cold) -- */

/* InvMixColumns of one column (FIPS-197 5.3.3), LE dword: byte r = row r */
GCM_HD uint32_t aes_inv_mix_column(uint32_t c)
{
    const uint8_t a0 = (uint8_t)c, a1 = (uint8_t)(c >> 8), a2 = (uint8_t)(c >> 16), a3 = (uint8_t)(c >> 24);
    const uint8_t b0 = (uint8_t)(gf8_mul(a0, 14) ^ gf8_mul(a1, 11) ^ gf8_mul(a2, 13) ^ gf8_mul(a3, 9));
    const uint8_t b1 = (uint8_t)(gf8_mul(a0, 9) ^ gf8_mul(a1, 14) ^ gf8_mul(a2, 11) ^ gf8_mul(a3, 13));
    const uint8_t b2 = (uint8_t)(gf8_mul(a0, 13) ^ gf8_mul(a1, 9) ^ gf8_mul(a2, 14) ^ gf8_mul(a3, 11));
    const uint8_t b3 = (uint8_t)(gf8_mul(a0, 11) ^ gf8_mul(a1, 13) ^ gf8_mul(a2, 9) ^ gf8_mul(a3, 14));
    return (uint32_t)b0 | ((uint32_t)b1 << 8) | ((uint32_t)b2 << 16) | ((uint32_t)b3 << 24);
}

/*
 * Round keys of the equivalent inverse cipher (FIPS-197 5.3.5): dk_0 = rk_nr, dk_r = InvMixColumns(rk_(nr-r))
 * for 0 < r < nr, dk_nr = rk_0, so decryption runs the same table-round shape as encryption.
 */
GCM_HD void aes_decrypt_key_schedule(const uint32_t *rk, uint32_t nr, uint32_t *dk)
{
    for (uint32_t c = 0; c < 4; ++c) {
        dk[c] = rk[4 * nr + c];
        dk[4 * nr + c] = rk[c];
    }
    for (uint32_t r = 1; r < nr; ++r)
        for (uint32_t c = 0; c < 4; ++c)
            dk[4 * r + c] = aes_inv_mix_column(rk[4 * (nr - r) + c]);
}

/*
 * One AES block, encryption (T = T0, S = S-box, k = the FIPS-197 schedule) or decryption (T = Td0,
 * S = InvS-box, k = aes_decrypt_key_schedule), from a single 1 KiB table and its byte rotations
 * (T_i = rotl(T, 8 i)).  Encryption: column c of a round takes row r from column c + r (ShiftRows);
 * decryption from column c - r (InvShiftRows).  T and S may live in LDS (the ECB kernels) or host
 * memory (the kernel model).
 */
template <bool DEC>
GCM_HD void aes_ecb_block(const uint32_t *T, const uint8_t *S, const uint32_t *k, uint32_t nr, uint32_t w[4])
{
    uint32_t s[4] = {w[0] ^ k[0], w[1] ^ k[1], w[2] ^ k[2], w[3] ^ k[3]};
    for (uint32_t r = 1; r < nr; ++r) {
        uint32_t n[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int c1 = DEC ? (c + 3) & 3 : (c + 1) & 3, c2 = (c + 2) & 3, c3 = DEC ? (c + 1) & 3 : (c + 3) & 3;
            n[c] = T[s[c] & 0xffu] ^ rotl32(T[(s[c1] >> 8) & 0xffu], 8) ^ rotl32(T[(s[c2] >> 16) & 0xffu], 16) ^
                   rotl32(T[s[c3] >> 24], 24) ^ k[4 * r + (uint32_t)c];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
            s[c] = n[c];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int c1 = DEC ? (c + 3) & 3 : (c + 1) & 3, c2 = (c + 2) & 3, c3 = DEC ? (c + 1) & 3 : (c + 3) & 3;
        w[c] = ((uint32_t)S[s[c] & 0xffu] | ((uint32_t)S[(s[c1] >> 8) & 0xffu] << 8) |
                ((uint32_t)S[(s[c2] >> 16) & 0xffu] << 16) | ((uint32_t)S[s[c3] >> 24] << 24)) ^
               k[4 * nr + (uint32_t)c];
    }
}

/* Round keys only: the context of the ECB/CTR ciphers (no GHASH tables) */
struct AesKeys {
    uint32_t rk[60]; /* encryption schedule */
    uint32_t dk[60]; /* equivalent-inverse-cipher schedule */
    uint32_t rounds;
    uint32_t key_size;
    uint32_t pad_[2];
};

GCM_HD int build_aes_keys(const uint8_t *sbox, const uint8_t *key, uint32_t keylen, AesKeys *k)
{
    if (keylen != 16 && keylen != 32)
        return -1;
    for (int i = 0; i < 60; ++i)
        k->rk[i] = k->dk[i] = 0;
    k->rounds = aes_expand_key(sbox, key, keylen, k->rk);
    aes_decrypt_key_schedule(k->rk, k->rounds, k->dk);
    k->key_size = keylen;
    k->pad_[0] = k->pad_[1] = 0;
    return 0;
}

/* ------------------------------------------------------------------ parallel key image -- */

/*
 * GF(2^128) elements as a big-endian 128-bit integer {hi, lo}: GCM bit k (x^k, bit 7 - k % 8 of
 * stream byte k / 8) is bit 127 - k.  Multiplying by x is a right shift, and x^128 = 1 + x + x^2 + x^7.
 */
struct Gf128 {
    uint64_t hi, lo;
};

GCM_HD Gf128 gf_from_bytes(const uint8_t b[16])
{
    Gf128 r = {0u, 0u};
    for (int i = 0; i < 8; ++i) {
        r.hi = (r.hi << 8) | b[i];
        r.lo = (r.lo << 8) | b[8 + i];
    }
    return r;
}

GCM_HD void gf_to_bytes(Gf128 v, uint8_t b[16])
{
    for (int i = 0; i < 8; ++i) {
        b[i] = (uint8_t)(v.hi >> (56 - 8 * i));
        b[8 + i] = (uint8_t)(v.lo >> (56 - 8 * i));
    }
}

GCM_HD Gf128 gf_shr(Gf128 v, uint32_t n) /* n < 128 */
{
    if (n == 0)
        return v;
    if (n >= 64)
        return Gf128{0u, v.hi >> (n - 64)};
    return Gf128{v.hi >> n, (v.lo >> n) | (v.hi << (64 - n))};
}

GCM_HD Gf128 gf_shl(Gf128 v, uint32_t n) /* n < 128 */
{
    if (n == 0)
        return v;
    if (n >= 64)
        return Gf128{v.lo << (n - 64), 0u};
    return Gf128{(v.hi << n) | (v.lo >> (64 - n)), v.lo << n};
}

GCM_HD Gf128 gf_xor(Gf128 a, Gf128 b) { return Gf128{a.hi ^ b.hi, a.lo ^ b.lo}; }

/*
 * v * x^i for i <= 64, branch-light: the i bits shifted out below x^127 come back as
 * T * (1 + x + x^2 + x^7), T = those bits placed at x^0 .. x^(i-1) (bit positions >= 64 of {hi, lo}),
 * so one reduction pass suffices (T x^7 stays below x^71).
 */
GCM_HD Gf128 gf_mul_xpow64(Gf128 v, uint32_t i)
{
    if (i == 0)
        return v;
    const Gf128 t = gf_shl(v, 128u - i);
    return gf_xor(gf_xor(gf_shr(v, i), t), gf_xor(gf_xor(gf_shr(t, 1), gf_shr(t, 2)), gf_shr(t, 7)));
}

/* v * x^i, 0 <= i < 128 */
GCM_HD Gf128 gf_mul_xpow(Gf128 v, uint32_t i) { return i > 64u ? gf_mul_xpow64(gf_mul_xpow64(v, 64u), i - 64u) : gf_mul_xpow64(v, i); }

/* the element's GCM bit k (coefficient of x^k) */
GCM_HD uint32_t gf_bit(Gf128 v, uint32_t k) { return (uint32_t)((k < 64 ? v.hi >> (63 - k) : v.lo >> (127 - k)) & 1u); }

/*
 * Lane `lane` (0..63)'s share of X * Y in the wave-parallel multiply of the key setup: Y x^lane and
 * Y x^(lane + 64), masked by X's bits lane and lane + 64.  X * Y is the XOR of the 64 shares.
 */
GCM_HD Gf128 gf_mul_lane_share(Gf128 X, Gf128 Y, uint32_t lane)
{
    const Gf128 a = gf_mul_xpow64(Y, lane), b = gf_mul_xpow64(gf_mul_xpow64(Y, 64u), lane);
    Gf128 acc = {0u, 0u};
    if (gf_bit(X, lane))
        acc = a;
    if (gf_bit(X, lane + 64u))
        acc = gf_xor(acc, b);
    return acc;
}

/* The 16 multipliers of the key image, by index s: H^1..H^8, then H^64, H^256, H^32, H^128, H^16, H^512, H^1024,
 * H^768. */
enum : uint32_t { KEY_IMAGE_TABLES = MAX_K + 8 };

GCM_HD uint8_t (*key_image_table(KeyImage *ki, uint32_t s))[16][16]
{
    return s < (uint32_t)MAX_K      ? ki->gh[s]
           : s == (uint32_t)MAX_K   ? ki->gh64
           : s == MAX_K + 1u        ? ki->gh256
           : s == MAX_K + 2u        ? ki->gh32
           : s == MAX_K + 3u        ? ki->gh128
           : s == MAX_K + 4u        ? ki->gh16
           : s == MAX_K + 5u        ? ki->gh512
           : s == MAX_K + 6u        ? ki->gh1024
                                    : ki->gh768;
}

/*
 * Entry i of the KEY_IMAGE_TABLES x 32 x 16 nibble-table entries: table s = i / 512, nibble t, value v; the XOR of the
 * single-bit products bits[s][k] = P_s x^k of v's set bits (bit b of nibble t is GCM bit nibble_bit_index(t, b)),
 * stored as its 16 stream bytes in LE dwords.
 */
GCM_HD void key_image_store_entry(KeyImage *ki, const Gf128 (*bits)[128], uint32_t i)
{
    const uint32_t s = i >> 9, t = (i >> 4) & 31u, v = i & 15u;
    Gf128 e = {0u, 0u};
    for (int b = 0; b < 4; ++b)
        if ((v >> b) & 1u)
            e = gf_xor(e, bits[s][nibble_bit_index((int)t, b)]);
    *(u32x4 *)key_image_table(ki, s)[t][v] = u32x4{bswap32((uint32_t)(e.hi >> 32)), bswap32((uint32_t)e.hi),
                                                    bswap32((uint32_t)(e.lo >> 32)), bswap32((uint32_t)e.lo)};
}

/* the 32 nibble tables of multiplication by c: tab[t][v] = (nibble t of the element = v) * c */
GCM_HD void nibble_tables(const uint8_t c[16], uint8_t (*tab)[16][16])
{
    for (int t = 0; t < 32; ++t)
        for (int k = 0; k < 16; ++k)
            tab[t][0][k] = 0;
    /* single-bit entries: the element with GCM bit k set, times c, is c * x^k */
    uint8_t v[16];
    for (int k = 0; k < 16; ++k)
        v[k] = c[k];
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

/* Builds the whole KeyImage (round keys, H, nibble tables of H^1..H^MAX_K and H^64) sequentially. */
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
        nibble_tables(hp, ki->gh[p - 1]);
    }
    /* H^16 = (H^8)^2, H^32 = (H^16)^2, ... H^1024 = (H^512)^2 */
    gf128_mul_bytes(hp, hp, hp);
    nibble_tables(hp, ki->gh16);
    gf128_mul_bytes(hp, hp, hp);
    nibble_tables(hp, ki->gh32);
    gf128_mul_bytes(hp, hp, hp);
    nibble_tables(hp, ki->gh64);
    gf128_mul_bytes(hp, hp, hp);
    nibble_tables(hp, ki->gh128);
    gf128_mul_bytes(hp, hp, hp);
    nibble_tables(hp, ki->gh256);
    uint8_t h256[16], h768[16];
    for (int k = 0; k < 16; ++k)
        h256[k] = hp[k];
    gf128_mul_bytes(hp, hp, hp);
    nibble_tables(hp, ki->gh512);
    gf128_mul_bytes(hp, h256, h768); /* H^768 = H^512 H^256 */
    nibble_tables(h768, ki->gh768);
    gf128_mul_bytes(hp, hp, hp);
    nibble_tables(hp, ki->gh1024);
    return 0;
}

/*
 * LDS image fill, split over nthr threads: AES T-table replicas and the K GHASH tables
 * (slot j = tables of H^(K-j)).  Called by every thread of a workgroup before the barrier.
 */
/*
 * 8-byte half `half` of entry v of chunk c of the 5-bit tables of H^4: XOR of the single-bit products
 * (bit 5c + q set) * H^4, q in v, read from the nibble tables of H^4 (bit i of dword d is bit k = i % 8 of
 * byte m = i / 8: nibble table 8d + 2m + k / 4, entry 1 << (k % 4)).
 */
GCM_HD u32x2 gh5_entry(const KeyImage *ki, uint32_t c, uint32_t half, uint32_t v)
{
    u32x2 r = {0u, 0u};
    for (uint32_t q = 0; q < 5u; ++q) {
        const uint32_t b = 5u * c + q;
        if (((v >> q) & 1u) == 0u || b >= 128u)
            continue;
        const uint32_t d = b >> 5, i = b & 31u, m = i >> 3, k = i & 7u;
        const uint32_t *e = (const uint32_t *)ki->gh[3][8u * d + 2u * m + (k >> 2)][1u << (k & 3u)];
        r[0] ^= e[2u * half];
        r[1] ^= e[2u * half + 1u];
    }
    return r;
}

GCM_HD void fill_lds(uint8_t *lds, const uint32_t *t0, const KeyImage *ki, uint32_t K, uint32_t tid, uint32_t nthr)
{
    /* mirrors struct Layout<K> */
    const bool gh8 = GCM_GH8 && K == 4u;
    const bool gh5 = GCM_GH5 && K == 4u && !gh8;
    /* gh8: the two-table image at [64K, 128K), the GH8 table at [0, 64K) */
    const uint32_t aes_base = gh5 ? (uint32_t)GH5_BYTES : gh8 ? 0x10000u : 0u;
    const uint32_t aes_bytes = K <= 4 && !gh8 ? 0x20000u : 0x10000u, gh_base = gh8 ? 0x20000u : aes_base + aes_bytes;
    const uint32_t n_nibble = gh5 ? 2u : K;
    if (gh8) {
        /* row e, slot p: (e at byte p) * H^4 = nibble tables 2p (low nibble of e) ^ 2p + 1 (high nibble) */
        for (uint32_t i = tid; i < GH8_BYTES / 16u; i += nthr) {
            const uint32_t e = i >> 4, p = i & 15u;
            const u32x4 lo = *(const u32x4 *)ki->gh[3][2u * p][e & 15u];
            const u32x4 hi = *(const u32x4 *)ki->gh[3][2u * p + 1u][e >> 4];
            *(u32x4 *)(lds + 16u * i) = lo ^ hi;
        }
    }
    for (uint32_t i = tid; i < aes_bytes / 16; i += nthr) {
        uint32_t off = i * 16, x = (off >> 8) & 0xffu;
        uint32_t v = t0[x];
        /* image A: T0 | T1, image B: T2 | T3;  T_i = rotl(T0, 8 i) */
        uint32_t rot = ((off & 0x10000u) ? 16u : 0u) + ((off & 128u) ? 8u : 0u);
        if (rot)
            v = rotl32(v, (int)rot);
        u32x4 q = {v, v, v, v};
        *(u32x4 *)(lds + aes_base + off) = q;
    }
    const uint32_t nvec = n_nibble * (GH_TABLE_BYTES / 16);
    for (uint32_t i = tid; i < nvec; i += nthr) {
        uint32_t slot = i / (GH_TABLE_BYTES / 16), within = i % (GH_TABLE_BYTES / 16);
        const u32x4 *srcv = (const u32x4 *)ki->gh[n_nibble - slot - 1];
        *(u32x4 *)(lds + gh_base + slot * GH_TABLE_BYTES + within * 16) = srcv[within];
    }
    if (gh5) {
        /* entry e: chunk e / 64, half (e / 32) & 1, value e & 31 -> byte 8e */
        for (uint32_t e = tid; e < GH5_BYTES / 8u; e += nthr)
            *(u32x2 *)(lds + 8u * e) = gh5_entry(ki, e >> 6, (e >> 5) & 1u, e & 31u);
    }
}

/*
 * fill_lds split for the multi-key batch kernels (the GH8 layout, Layout<4>): the key-independent AES image once per
 * workgroup, and a key's GHASH tables (the GH8 table of H^4, the nibble tables of H^4..H^1) at every key change.
 */
GCM_HD void fill_lds_aes(uint8_t *lds, const uint32_t *t0, uint32_t K, uint32_t tid, uint32_t nthr)
{
    const uint32_t aes_base = 0x10000u, aes_bytes = 0x10000u;
    (void)K;
    for (uint32_t i = tid; i < aes_bytes / 16; i += nthr) {
        const uint32_t off = i * 16, x = (off >> 8) & 0xffu;
        uint32_t v = t0[x];
        if (off & 128u)
            v = rotl32(v, 8); /* image A: T0 | T1 */
        *(u32x4 *)(lds + aes_base + off) = u32x4{v, v, v, v};
    }
}

GCM_HD void fill_lds_key(uint8_t *lds, const KeyImage *ki, uint32_t tid, uint32_t nthr)
{
    for (uint32_t i = tid; i < GH8_BYTES / 16u; i += nthr) {
        const uint32_t e = i >> 4, p = i & 15u;
        const u32x4 lo = *(const u32x4 *)ki->gh[3][2u * p][e & 15u];
        const u32x4 hi = *(const u32x4 *)ki->gh[3][2u * p + 1u][e >> 4];
        *(u32x4 *)(lds + 16u * i) = lo ^ hi;
    }
    const uint32_t gh_base = 0x20000u, nvec = 4u * (GH_TABLE_BYTES / 16);
    for (uint32_t i = tid; i < nvec; i += nthr) {
        const uint32_t slot = i / (GH_TABLE_BYTES / 16), within = i % (GH_TABLE_BYTES / 16);
        const u32x4 *srcv = (const u32x4 *)ki->gh[3u - slot];
        *(u32x4 *)(lds + gh_base + slot * GH_TABLE_BYTES + within * 16) = srcv[within];
    }
}

/* ------------------------------------------------------------------ window kernels --------- */

/*
 * LDS map of the window kernels (small framing / AEAD batches, gcm_engine.hip window_body), KW lanes per
 * segment: the two-table AES image, the tables of H^KW..H^1 (slot j = H^(KW-j), the lane scaling of a
 * KW-lane walk), the tables of H^64 (joining 64-position segments), then the segment sums.
 */
template <int KW = 4, int SEG = 64>
struct LayoutWin {
    static constexpr bool four_tables = false;
    static constexpr bool gh5 = false;
    static constexpr bool gh8 = false;
    static constexpr uint32_t aes_b2 = 0x0cu;
    static constexpr uint32_t aes_base = 0u;
    static constexpr uint32_t gh_base = 0x10000u;
    /* join tables: H^SEG (within groups of 4 segments), H^(4 SEG) (across groups); SEG = 32 adds H^256
     * (across pairs of groups, window_pair_*) */
    static constexpr uint32_t gh64 = gh_base + (uint32_t)KW * GH_TABLE_BYTES;
    static constexpr uint32_t gh256 = gh64 + GH_TABLE_BYTES;
    static constexpr uint32_t ghpair = gh256 + GH_TABLE_BYTES;
    static constexpr uint32_t parts = ghpair + (SEG == 32 ? GH_TABLE_BYTES : 0u);
    static constexpr bool split_scale = false;
    static constexpr bool x2_walk = false;
    static constexpr bool parts_alias = false; /* the segment sums have their own LDS (after the tables) */
};

/*
 * LDS map of the 16-lane single-record latency kernels (window_body KW = 16, SEG = 32: two steps per segment).
 * 160 KiB, filled in one pass as two copies: the two-table AES image (the same rows as LayoutWin, kept once per
 * device) and the key image's contiguous tables H^1..H^8, H^16, H^32, H^128, H^256.
 *   [0, 64K)       AES image T0 | T1
 *   [64K, 128K)    H^e at 64K + 8K (e - 1), e = 1..8 (lane scaling)
 *   [128K, 136K)   H^16: the Horner factor (gh_base)
 *   [136K, 160K)   H^32 (groups of 4 segments), H^128 (pairs of groups), H^256 (the chain of pairs)
 * A lane's scaling H^e, e in 1..16, is one multiply for e <= 8 or e = 16, else H^8 then H^(e - 8) (split_scale).
 * The segment sums alias the scaling tables: they are written after a barrier that ends every walk.
 */
struct LayoutWin16 {
    static constexpr bool four_tables = false;
    static constexpr bool gh5 = false;
    static constexpr bool gh8 = false;
    static constexpr uint32_t aes_b2 = 0x0cu;
    static constexpr uint32_t aes_base = 0u;
    static constexpr uint32_t gh_pow1 = 0x10000u; /* H^1; H^e at gh_pow1 + (e - 1) GH_TABLE_BYTES */
    static constexpr uint32_t gh_base = 0x20000u; /* H^16 */
    static constexpr uint32_t gh64 = 0x22000u;    /* window_body's within-group join table: H^32 */
    static constexpr uint32_t gh256 = 0x24000u;   /* pairs of groups: H^128 */
    static constexpr uint32_t ghpair = 0x26000u;  /* the chain of pairs: H^256 */
    static constexpr uint32_t parts = 0x10000u;
    static constexpr uint32_t bytes = 0x28000u;
    static constexpr bool split_scale = true;
    static constexpr bool x2_walk = false;
    static constexpr bool wide_scale = false; /* 3 waves per SIMD: no registers for 32 reads in flight */
    static constexpr bool parts_alias = true;
};
enum : uint32_t {
    WIN_SEG = 64,    /* GHASH positions per segment: 4 lanes x 16 steps */
    WIN_MAXSEG = 17, /* segments of the largest TLS record (16640-byte record: 1 + 1039 + 1 positions) */
    WIN_SEG32_MAXSEG = 33, /* the same in 32-position segments (single-record latency kernels) */
};

/* vector v of the window image: AES image A (T0 | T1 rows) for v < 4096, then the kw + 2 GHASH tables */
GCM_HD u32x4 window_image_vec(const uint32_t *t0, const KeyImage *ki, uint32_t v, uint32_t kw, uint32_t seglen = 64u)
{
    if (v < 0x10000u / 16u) {
        const uint32_t off = v * 16u, x = (off >> 8) & 0xffu;
        const uint32_t w = (off & 128u) ? rotl32(t0[x], 8) : t0[x];
        return u32x4{w, w, w, w};
    }
    const uint32_t i = v - 0x10000u / 16u, slot = i / (GH_TABLE_BYTES / 16u), within = i % (GH_TABLE_BYTES / 16u);
    /* the two join tables: H^seglen (groups of 4 segments) and H^(4 seglen) (chaining the groups) */
    const u32x4 *srcv = slot < kw           ? (const u32x4 *)ki->gh[kw - 1u - slot]
                        : slot == kw        ? (const u32x4 *)(seglen == 32u ? ki->gh32 : ki->gh64)
                        : slot == kw + 1u   ? (const u32x4 *)(seglen == 32u ? ki->gh128 : ki->gh256)
                                            : (const u32x4 *)ki->gh256; /* seglen 32: H^256 joins pairs of groups */
    return srcv[within];
}

/*
 * Fills the window image, split over nthr threads.  Eight vectors per thread are loaded before any is
 * stored: a fill pass is one memory latency, and with 256 threads the image takes 26 vectors per thread.
 */
#ifndef GCM_SPLIT_X2
#define GCM_SPLIT_X2 1 /* split kernels: a segment's two steps as one interleaved two-block AES (lane_walk) */
#endif
#ifndef GCM_WIN_FILL
#define GCM_WIN_FILL 8u /* vectors loaded per thread before any is stored (one memory latency per pass) */
#endif
GCM_HD void fill_lds_window(uint8_t *lds, const uint32_t *t0, const KeyImage *ki, uint32_t tid, uint32_t nthr,
                            uint32_t kw = 4u, uint32_t seglen = 64u)
{
    const uint32_t total = 0x10000u / 16u + (kw + (seglen == 32u ? 3u : 2u)) * GH_TABLE_BYTES / 16u;
    for (uint32_t base = tid; base < total; base += GCM_WIN_FILL * nthr) {
        u32x4 v[GCM_WIN_FILL];
#pragma unroll
        for (uint32_t k = 0; k < GCM_WIN_FILL; ++k)
            if (base + k * nthr < total)
                v[k] = window_image_vec(t0, ki, base + k * nthr, kw, seglen);
#pragma unroll
        for (uint32_t k = 0; k < GCM_WIN_FILL; ++k)
            if (base + k * nthr < total)
                *(u32x4 *)(lds + 16u * (base + k * nthr)) = v[k];
    }
}

/*
 * LDS map of the split window kernels (gcm_engine.hip split_body): a record's 32-position segments are cut into runs
 * of 8, each run walked by its own 128-thread workgroup (16 lanes per segment, one two-block trip) on its own CU.  As
 * LayoutWin16 up to 152K; the last table scales the run's sum to the record's end, H^(256 m) for the m runs after it.
 *   [0, 64K) AES image; [64K, 128K) H^1..H^8; [128K) H^16 (Horner); [136K) H^32 (groups of 4 segments);
 *   [144K) H^128 (the chain of groups); [152K) H^256, H^512, H^768 or H^1024 (gh_run)
 */
struct LayoutSplit {
    static constexpr bool four_tables = false;
    static constexpr bool gh5 = false;
    static constexpr bool gh8 = false;
    static constexpr uint32_t aes_b2 = 0x0cu;
    static constexpr uint32_t aes_base = 0u;
    static constexpr uint32_t gh_pow1 = 0x10000u;
    static constexpr uint32_t gh_base = 0x20000u;  /* H^16 */
    static constexpr uint32_t gh_group = 0x22000u; /* H^32 */
    static constexpr uint32_t gh_chain = 0x24000u; /* H^128 */
    static constexpr uint32_t gh_run = 0x26000u;   /* H^(512 m) */
    static constexpr uint32_t parts = 0x10000u;    /* segment sums, after the walk (aliases H^1) */
    static constexpr uint32_t bytes = 0x28000u;
    static constexpr bool split_scale = true;
    static constexpr bool x2_walk = true; /* a segment's two steps in one trip (lane_walk) */
    static constexpr bool wide_scale = true; /* one wave per SIMD: registers for 32 reads in flight */
    static constexpr bool parts_alias = true;
};
enum : uint32_t {
    SPLIT_RUNSEG = 8,   /* segments per run (one workgroup) */
    SPLIT_MAXRUN = 5,   /* runs of a TLS record (33 segments); larger records are walked whole by run 0 */
    SPLIT_THREADS = 128,
    SPLIT_PSLOTS = SPLIT_MAXRUN,     /* u32x4 slots per record in the split buffer: the runs' partials */
};

/* H^(256 m): scales a run of SPLIT_RUNSEG 32-position segments over the m runs after it (m = 1..4; any for m = 0) */
GCM_HD const u32x4 *split_run_table(const KeyImage *ki, uint32_t m)
{
    return (const u32x4 *)(m <= 1u ? &ki->gh256[0][0][0] : m == 2u ? &ki->gh512[0][0][0]
                                                         : m == 3u ? &ki->gh768[0][0][0] : &ki->gh1024[0][0][0]);
}

/* vector v of the LayoutSplit image for a run followed by m (0..4) runs: AES rows, gh[0] .. gh128, H^(256 m) */
GCM_HD u32x4 split_image_vec(const uint32_t *t0, const KeyImage *ki, uint32_t v, uint32_t m)
{
    if (v < 0x10000u / 16u)
        return window_image_vec(t0, ki, v, 8u, 32u);
    if (v < LayoutSplit::gh_run / 16u)
        return ((const u32x4 *)ki->gh)[v - 0x10000u / 16u];
    return split_run_table(ki, m)[v - LayoutSplit::gh_run / 16u];
}

/* vector v (16 B) of the LayoutWin16 image: the AES rows of window_image_vec, then the key image from gh[0] on */
GCM_HD u32x4 win16_image_vec(const uint32_t *t0, const KeyImage *ki, uint32_t v)
{
    if (v < 0x10000u / 16u)
        return window_image_vec(t0, ki, v, 8u, 32u);
    return ((const u32x4 *)ki->gh)[v - 0x10000u / 16u];
}

/* the whole LayoutWin16 image, split over nthr threads (the host model; the kernels copy it, window_body) */
GCM_HD void fill_lds_win16(uint8_t *lds, const uint32_t *t0, const KeyImage *ki, uint32_t tid, uint32_t nthr)
{
    for (uint32_t v = tid; v < LayoutWin16::bytes / 16u; v += nthr)
        *(u32x4 *)(lds + 16u * v) = win16_image_vec(t0, ki, v);
}

/*
 * Segment seg of a record of A AAD blocks and C payload blocks: its g = A + C + 1 GHASH positions are
 * front-padded to nseg * seglen; the returned walk covers padded positions [seglen seg, seglen (seg + 1)) (its pad is
 * negative as int32 after the first segment).  Framed records have A = 1 (the 5-byte header).
 */
GCM_HD Walk window_segment(uint32_t A, uint32_t C, uint32_t seg, uint32_t *nseg, uint32_t kw = 4u,
                           uint32_t seglen = WIN_SEG)
{
    const uint32_t g = A + C + 1u;
    *nseg = (g + seglen - 1u) / seglen;
    Walk w;
    w.A = A;
    w.C = C;
    w.T = seglen / kw; /* kw lanes per segment */
    w.pad = seglen * *nseg - g - seglen * seg;
    return w;
}

/*
 * Joining a record's segment sums P_0..P_{ns-1}: GHASH = sum_s P_s * H^(64 (ns-1-s)).  The segments are
 * grouped in fours aligned to the record's END (the first group holds the ns mod 4 leftovers), so every group
 * after the first spans exactly 4 segments: phase A folds each group with H^64 (<= 3 multiplies, all groups
 * in parallel), phase B chains the groups with H^256 (<= 4 multiplies for 17 segments) -- 7 dependent
 * multiplies instead of 16.  window_group_end(s) is one past the last segment of the group led by s.
 */
GCM_HD uint32_t window_group_offset(uint32_t ns) { return (4u - ns % 4u) % 4u; }
GCM_HD bool window_group_leader(uint32_t s, uint32_t ns) { return s < ns && (s == 0u || (s + window_group_offset(ns)) % 4u == 0u); }
GCM_HD uint32_t window_group_end(uint32_t s, uint32_t ns)
{
    const uint32_t o = window_group_offset(ns), e = ((s + o) & ~3u) + 4u - o;
    return e < ns ? e : ns;
}
/*
 * 32-position segments (up to 33 per record, 9 groups): a middle level joins the groups in pairs, also
 * aligned to the record's end, before the chain -- G_a H^128 + G_b per pair in parallel, then the pairs
 * (8 segments = 256 positions apart) chained with H^256: 3 + 1 + 4 dependent multiplies instead of 3 + 8.
 * Group g (0-based) leads a pair when ng - g is even; the first group stands alone when ng is odd.
 * window_group_start(g, ns) is the leading segment of group g.
 */
GCM_HD uint32_t window_group_count(uint32_t ns) { return (ns + window_group_offset(ns) + 3u) / 4u; }
GCM_HD uint32_t window_group_start(uint32_t g, uint32_t ns) { return g == 0u ? 0u : 4u * g - window_group_offset(ns); }

/* ------------------------------------------------------------------ per-lane record walk -- */

/*
 * GCM_READ(p, n): the walk is about to read bytes [p, p + n) of a record (or its AAD / descriptor).  Nothing in the
 * kernels; the CPU test suite's host model (tests/cpp/kernel_model.cpp, GCM_HOST_READ_CHECK) checks every such range
 * against the records' own bytes, so a read outside them -- a fault wherever a record ends at an unmapped page --
 * fails on the CPU, deterministically.  GCM_WRITE(p, n), likewise for every store of the walk, against the records'
 * output ranges: a stray store -- which need not stop its wave, and faults late, if at all -- fails there too.
 */
#if defined(GCM_HOST_READ_CHECK) && !defined(__HIP_DEVICE_COMPILE__)
extern "C" void gcm_host_read_check(const void *p, size_t n);
extern "C" void gcm_host_write_check(const void *p, size_t n);
#define GCM_READ(p, n) gcm_host_read_check((const void *)(p), (size_t)(n))
#define GCM_WRITE(p, n) gcm_host_write_check((const void *)(p), (size_t)(n))
#else
#define GCM_READ(p, n) ((void)0)
#define GCM_WRITE(p, n) ((void)0)
#endif

/* loads n (< 16) bytes zero-extended */
GCM_HD u32x4 load_partial(const uint8_t *p, uint32_t n)
{
    GCM_READ(p, n);
    /* loop-free (n < 16): whole dwords, then up to 3 bytes of dword q = n / 4 */
    u32x4 v = {0u, 0u, 0u, 0u};
    const uint32_t q = n >> 2, rem = n & 3u;
#pragma unroll
    for (uint32_t d = 0; d < 3; ++d)
        if (d < q)
            v[d] = *(const uint32_t_u *)(p + 4u * d);
    uint32_t t = 0u;
    if (rem > 0u)
        t = p[4u * q];
    if (rem > 1u)
        t |= (uint32_t)p[4u * q + 1u] << 8;
    if (rem > 2u)
        t |= (uint32_t)p[4u * q + 2u] << 16;
    v[0] = q == 0u ? t : v[0];
    v[1] = q == 1u ? t : v[1];
    v[2] = q == 2u ? t : v[2];
    v[3] = q == 3u ? t : v[3];
    return v;
}

GCM_HD void store_partial(uint8_t *p, uint32_t n, u32x4 v)
{
    /* loop-free (n < 16), mirror of load_partial */
    GCM_WRITE(p, n);
    const uint32_t q = n >> 2, rem = n & 3u;
#pragma unroll
    for (uint32_t d = 0; d < 3; ++d)
        if (d < q)
            *(uint32_t_u *)(p + 4u * d) = v[d];
    const uint32_t t = q == 0u ? v[0] : q == 1u ? v[1] : q == 2u ? v[2] : v[3];
    if (rem > 0u)
        p[4u * q] = (uint8_t)t;
    if (rem > 1u)
        p[4u * q + 1u] = (uint8_t)(t >> 8);
    if (rem > 2u)
        p[4u * q + 2u] = (uint8_t)(t >> 16);
}

/* byte n (< 16) of the block set to b; the block's bytes at and beyond n are zero */
GCM_HD u32x4 insert_byte(u32x4 v, uint32_t n, uint32_t b)
{
    const uint32_t bits = (b & 0xffu) << (8u * (n & 3u));
    v[0] |= (n >> 2) == 0u ? bits : 0u;
    v[1] |= (n >> 2) == 1u ? bits : 0u;
    v[2] |= (n >> 2) == 2u ? bits : 0u;
    v[3] |= (n >> 2) == 3u ? bits : 0u;
    return v;
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

/* byte shift of a 16-byte block towards byte 0: out.b_i = v.b_(i+n), zero-filled; 0 <= n < 16 */
GCM_HD u32x4 shr_bytes(u32x4 v, uint32_t n)
{
    const uint32_t q = n >> 2, r = n & 3u;
    uint32_t w0 = q == 0 ? v[0] : q == 1 ? v[1] : q == 2 ? v[2] : v[3];
    uint32_t w1 = q == 0 ? v[1] : q == 1 ? v[2] : q == 2 ? v[3] : 0u;
    uint32_t w2 = q == 0 ? v[2] : q == 1 ? v[3] : 0u;
    uint32_t w3 = q == 0 ? v[3] : 0u;
#if defined(__HIP_DEVICE_COMPILE__)
    u32x4 o = {__builtin_amdgcn_alignbyte(w1, w0, r), __builtin_amdgcn_alignbyte(w2, w1, r),
               __builtin_amdgcn_alignbyte(w3, w2, r), __builtin_amdgcn_alignbyte(0u, w3, r)};
#else
    auto ab = [](uint32_t hi, uint32_t lo, uint32_t rr) {
        return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * rr));
    };
    u32x4 o = {ab(w1, w0, r), ab(w2, w1, r), ab(w3, w2, r), ab(0u, w3, r)};
#endif
    return o;
}

#ifndef GCM_NT_LOADS
#define GCM_NT_LOADS 0
#endif
#ifndef GCM_NT_STORES
#define GCM_NT_STORES 1 /* the walk's whole-block stores marked non-temporal (measured: scripts/ablate.py ntstore) */
#endif
/* a record block's 16-byte load (GCM_NT_LOADS: marked non-temporal, so the streamed input does not displace the
 * half-written output lines from L2) */
GCM_HD u32x4 walk_load(const uint8_t *p)
{
    GCM_READ(p, 16);
#if defined(__HIP_DEVICE_COMPILE__) && GCM_NT_LOADS
    return __builtin_nontemporal_load((const u32x4_u *)p);
#else
    return *(const u32x4_u *)p;
#endif
}

/*
 * Address of lane j's 16-byte load in step t of walk wk (lane_walk): the AAD or payload block at the lane's grid
 * position, the received tag for the length block of an open, or `dummy` (steps with nothing to read).  A partial
 * last AAD block is read as the AAD's last 16 bytes, a sealed partial payload block as the payload's last 16.
 * in = src + rec.src, ad = aad + rec.aad, plen the GCM payload length.
 */
template <int K, bool SEAL, bool FRAME>
GCM_HD const uint8_t *walk_fetch_ptr(uint32_t t, uint32_t j, const Walk &wk, const Record &rec, bool valid, uint32_t plen,
                                     const uint8_t *in, const uint8_t *ad, const uint8_t *dummy)
{
    if (!valid || t >= wk.T)
        return dummy;
    const int32_t p = (int32_t)(j + K * t) - (int32_t)wk.pad;
    if (p < 0)
        return dummy;
    if ((uint32_t)p < wk.A) {
        if (FRAME)
            return dummy;
        if (16u * (uint32_t)p + 16u <= rec.aadlen)
            return ad + 16u * (uint32_t)p;
        return rec.aadlen >= 16u ? ad + rec.aadlen - 16u : dummy;
    }
    const uint32_t c = (uint32_t)p - wk.A;
    if (c >= wk.C) /* the length block; open fetches the received tag into its slot */
        return !SEAL && c == wk.C ? in + plen : dummy;
    if (!SEAL || 16u * c + 16u <= rec.len)
        return in + 16u * c;
    return rec.len >= 16u ? in + rec.len - 16u : dummy;
}

/*
 * One lane's share of one record (see struct Walk).  Returns the lane's partial GHASH already
 * scaled by H^(K-j); the lane holding the length block has E_K(J0) folded in, so the XOR of the
 * K returned values is the tag (seal), or the tag XOR the received tag (open: the length
 * lane fetches the received tag through its prefetch slot, so the record verifies iff the XOR
 * is zero and nothing has to be read after the walk).  Lanes with valid == false run the same instruction stream
 * without touching memory (Tmax is the wave-wide trip count).
 * iv0..iv2: the record's 96-bit nonce as LE dwords.
 *
 * Memory pipeline: every step issues at most ONE full 16-byte load (the block of the NEXT
 * step, so its latency hides under this step's AES + GHASH) and at most one 16-byte store.
 * Byte-granular reads happen only for an AAD shorter than 16 bytes (at setup, into the first
 * buffer) and a sealed payload shorter than 16 bytes (in its step).  A partial last AAD block
 * or payload block of a longer AAD/record is read as its last 16 bytes and shifted in
 * registers (seal), or read directly since the tag follows it (open) -- nothing is ever
 * read outside [aad, aad + aadlen) and [src, src + len (+16 for open)).
 */
/*
 * seg (window kernels): walk only one 64-position segment of the record.  The record's GHASH positions are
 * front-padded to a multiple of K*T (T = seg->T) and seg->pad is that padding minus the segment's first
 * padded position (negative as int32 for later segments); the lane's chain is scaled to the segment's end.
 * LY: the LDS layout (T-table image count and GHASH table base).
 */
template <int NR, int K, bool SEAL, bool FRAME = false, class LY = Layout<K>, int PF = 1>
GCM_HD u32x4 lane_walk_seg(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, uint32_t j, const Record &rec,
                           bool valid, uint32_t Tmax, uint32_t iv0, uint32_t iv1, uint32_t iv2, const uint8_t *src,
                           uint8_t *dst, const uint8_t *aad, const uint8_t *dummy, uint32_t ctype, bool use_seg,
                           Walk segw, uint32_t t0, const uint32_t *kr = nullptr, uint32_t f_lo = 0u, uint32_t f_hi = 0u)
{
    /* kr (LY::gh8): rotl16 of the round keys, wave-uniform (aes_round_tt2k_asm) */
    /* [f_lo, f_hi): interior steps of every lane of the wave (walk_interior; none by default), taken on a fast path */
    const Gh8Lane L8 = gh8_lane(lanesel >> 2); /* lane & 15: the GH8 read order (LY::gh8) */
    /* use_seg: walk the segment segw (window kernels); otherwise the whole record (make_walk) */
    /*
     * FRAME (TLS 1.3 record framing, lib/picotls.c:621-684 and :4779-4791): the AAD is the 5-byte
     * record header 17 03 03 BE16(plen + 16), built here in registers (build_aad), never read;
     * seal's GCM payload is the fragment (rec.len bytes at src) followed by the content-type byte
     * ctype, so plen = rec.len + 1 and the block holding the type byte is assembled in registers.
     */
    const uint32_t plen = FRAME && SEAL ? rec.len + 1u : rec.len;
    const uint32_t aadlen = FRAME ? 5u : rec.aadlen;
    const Walk wk = use_seg ? segw : make_walk(plen, aadlen, K, walk_out16(dst + rec.dst));
    const uint32_t end_cap = use_seg ? (uint32_t)K * segw.T : 0xffffffffu;
    const uint32_t gend = wk.A + wk.C + 1u; /* positions p >= gend are trailing pads */
    const uint8_t *in = src + rec.src;
    uint8_t *out = dst + rec.dst;
    const uint8_t *ad = aad + rec.aad;
    const uint32_t arem = rec.aadlen & 15u;
    u32x4 acc = {0u, 0u, 0u, 0u}, ek0 = {0u, 0u, 0u, 0u};
    if (!use_seg && valid) {
        /* hoisted AAD (make_walk): an AAD block at lane j's position before step 0 seeds its chain */
        const int32_t pv = (int32_t)j - (int32_t)K - (int32_t)wk.pad; /* record position of grid slot j - K */
        if (pv >= 0 && (uint32_t)pv < wk.A) {
            if (FRAME) { /* 17 03 03 BE16(plen + 16) */
                const uint32_t reclen = plen + 16u;
                acc[0] = 0x00030317u | ((reclen >> 8) & 0xffu) << 24;
                acc[1] = reclen & 0xffu;
            } else if (rec.aadlen < 16u) {
                acc = load_partial(ad, rec.aadlen);
            } else if (16u * (uint32_t)pv + 16u <= rec.aadlen) {
                GCM_READ(ad + 16u * (uint32_t)pv, 16);
                acc = *(const u32x4_u *)(ad + 16u * (uint32_t)pv);
            } else { /* partial last block: its last 16 bytes, shifted */
                GCM_READ(ad + rec.aadlen - 16u, 16);
                acc = shr_bytes(*(const u32x4_u *)(ad + rec.aadlen - 16u), 16u - arem);
            }
        }
    }
    /* hoisted round-1 (and round-2, GCM_R2CACHE) constants of the current counter window */
#if GCM_R2CACHE
    constexpr uint32_t WIN = 0xffffff00u; /* 2^8-block windows (aes_round12_consts) */
    uint32_t c1[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}, c1_hi = 0u;
    aes_round12_consts<LY::four_tables, LY::aes_b2>(lds + LY::aes_base, lanesel, rk, iv0, iv1, iv2, 0u, c1);
#else
    constexpr uint32_t WIN = 0xffff0000u; /* 2^16-block windows (aes_round1_consts) */
    uint32_t c1[4] = {0u, 0u, 0u, 0u}, c1_hi = 0u;
    aes_round1_consts<LY::four_tables>(lds + LY::aes_base, lanesel, rk, iv0, iv1, iv2, 0u, c1);
#endif

    /*
     * Address of the 16-byte load of step t (walk_fetch_ptr).  The load is issued unconditionally (steps with
     * nothing to read load 16 harmless bytes at `dummy`): with a load in every step the compiler can wait with
     * vmcnt(1) for the current block while the next one is in flight, instead of vmcnt(0).
     */
    const uint32_t cb = j - wk.pad - wk.A; /* payload block of step t: c = cb + K t (two's complement) */
    auto fetch_ptr = [&](uint32_t t) -> const uint8_t * {
        GCM_OPAQUE(t); /* recompute from t: no strength-reduced induction variables (VGPRs) */
        const uint32_t tu = wave_uniform(t);
        if (tu >= f_lo && tu < f_hi) /* interior step: every lane reads its whole payload block */
            return in + 16u * (cb + (uint32_t)K * tu);
        return walk_fetch_ptr<K, SEAL, FRAME>(t, j, wk, rec, valid, plen, in, ad, dummy);
    };

    /*
     * Horner with factor H^K, software-pipelined: in step t the multiply of the previous
     * value, P = A_(t-1) * H^K, runs inside the AES of step t (aes_ghash_fused), then
     * A_t = P ^ X_t.  A_(-1) = 0, and A_(T-1) is the lane's sum.
     */
    /*
     * Paired stores (K = 4): a step writes a 64-byte piece of a record, half of a 128-byte line.  Lines left half
     * written are written back as two partial requests, which measured 1.12-1.20x the algorithmic write traffic
     * (scripts/pmc_lengths.py; K = 8, whole lines per step, 1.00x).  A lane therefore holds a block that falls in the
     * first half of a line and stores it together with the next step's block, the second half (its address + 64).
     */
    constexpr bool PAIRST = GCM_PAIR_STORES && K == 4;
    /* batch kernels (LY = Layout<K>): streamed output stores non-temporal; the window kernels keep plain stores (their
     * last arrival reads a record's stored bytes back) */
    constexpr bool NTST = GCM_NT_STORES && std::is_same<LY, Layout<K>>::value;
    u32x4 pend_v = {0u, 0u, 0u, 0u};
    uint32_t pend_c = 0xffffffffu; /* payload block of the held store (none: ~0) */
    /*
     * The schedule is static: blocks of even steps are held, odd steps store the held block and their own.  t is
     * wave-uniform, so this is a scalar branch; walks start on even steps (t0), and a record whose payload is 128-byte
     * aligned (every 256-byte record slot) then pairs exactly the two halves of each line.
     */
    auto put = [&](uint32_t t, uint32_t c, u32x4 o) {
        if constexpr (PAIRST) {
            if ((t & 1u) == 0u) {
                if (pend_c != 0xffffffffu) /* (a lane's payload blocks are consecutive steps: not reached) */
                    GCM_WRITE(out + 16u * pend_c, 16), *(u32x4_u *)(out + 16u * pend_c) = pend_v;
                pend_v = o;
                pend_c = c;
                return;
            }
            if (pend_c != 0xffffffffu) {
                GCM_WRITE(out + 16u * pend_c, 16), *(u32x4_u *)(out + 16u * pend_c) = pend_v;
                pend_c = 0xffffffffu;
            }
        }
        GCM_WRITE(out + 16u * c, 16);
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (NTST)
            __builtin_nontemporal_store(o, (u32x4_u *)(out + 16u * c));
        else
#endif
            *(u32x4_u *)(out + 16u * c) = o;
    };
    /*
     * step_ctr and finish: step() below cut at its keystream, for the split kernels' two-step trip (x2 walk).  step()
     * keeps its own copy of both halves: expressed through these two lambdas it measured 2-3% slower in the batch
     * kernels at 1400 B (codegen), so the same logic is written twice; tests/test_kernel_model.py and the GPU suites
     * check both against the oracle.
     */
    auto step_ctr = [&](uint32_t t) -> uint32_t {
        const int32_t p = (int32_t)(j + K * t) - (int32_t)wk.pad;
        const bool is_pay = valid && t < wk.T && p < (int32_t)gend && p >= 0 && (uint32_t)p >= wk.A &&
                            (uint32_t)p < wk.A + wk.C;
        return is_pay ? (uint32_t)p - wk.A + 2u : 1u;
    };
    /* everything of step t after its keystream ks and its Horner product P = A_(t-1) * H^K */
    auto finish = [&](uint32_t t, u32x4 cur, u32x4 ks, u32x4 P) {
        const int32_t p = (int32_t)(j + K * t) - (int32_t)wk.pad;
        const bool active = valid && t < wk.T && p < (int32_t)gend;
        const bool is_aad = active && p >= 0 && (uint32_t)p < wk.A;
        const bool is_pay = active && (uint32_t)p >= wk.A && (uint32_t)p < wk.A + wk.C && p >= 0;
        const bool is_len = active && (uint32_t)p == wk.A + wk.C;
        const uint32_t c = (uint32_t)p - wk.A;
        const uint32_t clen = plen - 16u * c;    /* bytes of this payload block if < 16 */
        const uint32_t flen = rec.len - 16u * c; /* of them from the input (FRAME seal: all but the type byte) */
        u32x4 X = {0u, 0u, 0u, 0u};
        if (is_pay) {
            u32x4 data = cur;
            if (FRAME && SEAL && flen < 16u) {
                /* the last block: fb = flen fragment bytes (0..15), then the content type */
                if (flen == 0u)
                    data = u32x4{0u, 0u, 0u, 0u};
                else if (rec.len >= 16u)
                    data = shr_bytes(data, 16u - flen);
                else /* rare: a fragment under 16 bytes, read in place */
                    data = load_partial(in, rec.len);
                data = insert_byte(data, flen, ctype);
                const u32x4 o = data ^ ks;
                if (clen == 16u)
                    put(t, c, o);
                else
                    store_partial(out + 16u * c, clen, o);
                X = mask_tail(o, clen);
            } else if (clen >= 16u) {
                const u32x4 o = data ^ ks;
                put(t, c, o);
                X = SEAL ? o : data;
            } else {
                if (SEAL) {
                    if (rec.len >= 16u)
                        data = shr_bytes(data, 16u - clen);
                    else /* rare: a whole payload under 16 bytes, read in place */
                        data = load_partial(in, rec.len);
                }
                const u32x4 o = data ^ ks;
                store_partial(out + 16u * c, clen, o);
                X = mask_tail(SEAL ? o : data, clen);
            }
        } else if (is_aad) {
            if (FRAME) { /* 17 03 03 BE16(plen + 16) */
                const uint32_t reclen = plen + 16u;
                X[0] = 0x00030317u | ((reclen >> 8) & 0xffu) << 24;
                X[1] = reclen & 0xffu;
            } else if (use_seg && rec.aadlen < 16u) {
                X = load_partial(ad, rec.aadlen); /* segment walks: the short AAD may sit in any step */
            } else {
                X = 16u * (uint32_t)p + 16u <= rec.aadlen || rec.aadlen < 16u ? cur : shr_bytes(cur, 16u - arem);
            }
        } else if (is_len) {
            uint64_t abits = (uint64_t)aadlen * 8u, cbits = (uint64_t)plen * 8u;
            X[0] = bswap32((uint32_t)(abits >> 32));
            X[1] = bswap32((uint32_t)abits);
            X[2] = bswap32((uint32_t)(cbits >> 32));
            X[3] = bswap32((uint32_t)cbits);
            ek0 = SEAL ? ks : ks ^ cur; /* open: E(J0) ^ received tag */
        }
        if (active)
            acc = P ^ X;
    };
    auto step = [&](uint32_t t, u32x4 cur) {
        GCM_OPAQUE(t);
        /*
         * Interior step (f_lo <= t < f_hi, wave-uniform: a scalar branch): every lane seals / opens a whole payload
         * block c, so the flags below are not evaluated; the rare cases stay on the general path.
         */
        const uint32_t tu = wave_uniform(t);
        const bool fast = tu >= f_lo && tu < f_hi;
        int32_t p = 0;
        bool active = false, is_aad = false, is_pay = false, is_len = false;
        uint32_t c, ctr;
        if (fast) {
            c = cb + (uint32_t)K * tu;
            ctr = c + 2u;
        } else {
            p = (int32_t)(j + K * t) - (int32_t)wk.pad;
            active = valid && t < wk.T && p < (int32_t)gend;
            is_aad = active && p >= 0 && (uint32_t)p < wk.A;
            is_pay = active && (uint32_t)p >= wk.A && (uint32_t)p < wk.A + wk.C && p >= 0;
            is_len = active && (uint32_t)p == wk.A + wk.C;
            c = (uint32_t)p - wk.A;
            /* one AES per lane per step: payload counter c + 2, otherwise J0 (counter 1) */
            ctr = is_pay ? c + 2u : 1u;
        }
        const uint32_t clen = plen - 16u * c;    /* bytes of this payload block if < 16 */
        const uint32_t flen = rec.len - 16u * c; /* of them from the input (FRAME seal: all but the type byte) */

        uint32_t w[4] = {iv0, iv1, iv2, bswap32(ctr)};
#if GCM_ABLATE_AES && GCM_ABLATE_GHASH
        const u32x4 P = acc;
#elif GCM_ABLATE_AES
        const u32x4 P = LY::gh5 ? ghash5_mul_lds(lds, acc) : ghash_mul_lds(lds, LY::gh_base, acc);
#elif GCM_ABLATE_GHASH
        aes_encrypt_tt<NR, LY::four_tables>(lds + LY::aes_base, lanesel, rk, w);
        const u32x4 P = acc;
#else
        if ((ctr & WIN) != c1_hi) { /* a record crossing a counter window (>= 2^8 blocks with GCM_R2CACHE) */
            c1_hi = ctr & WIN;
            /* opaque inputs: keeps LICM from parking this rare path's 16 LDS addresses in VGPRs */
            uint32_t o0 = iv0, o1 = iv1, o2 = iv2, ol = lanesel;
            GCM_OPAQUE(o0);
            GCM_OPAQUE(o1);
            GCM_OPAQUE(o2);
            GCM_OPAQUE(ol);
#if GCM_R2CACHE
            aes_round12_consts<LY::four_tables, LY::aes_b2>(lds + LY::aes_base, ol, rk, o0, o1, o2, c1_hi, c1);
#else
            aes_round1_consts<LY::four_tables>(lds + LY::aes_base, ol, rk, o0, o1, o2, c1_hi, c1);
#endif
        }
        u32x4 P;
        if constexpr (LY::gh8)
            P = aes_gh8_fused_h<NR>(lds, lanesel, rk, kr, c1, ctr, w, acc, L8);
        else
            P = aes_ghash_fused_h<NR, LY::four_tables, LY::gh5, LY::aes_base>(lds, lanesel, rk, c1, ctr, w, LY::gh_base, acc);
#endif
        const u32x4 ks = {w[0], w[1], w[2], w[3]};
        if (fast) {
            const u32x4 o = cur ^ ks;
            put(t, c, o);
            acc = P ^ (SEAL ? o : cur);
            return;
        }

        u32x4 X = {0u, 0u, 0u, 0u};
        if (is_pay) {
            u32x4 data = cur;
            if (FRAME && SEAL && flen < 16u) {
                /* the last block: fb = flen fragment bytes (0..15), then the content type */
                if (flen == 0u)
                    data = u32x4{0u, 0u, 0u, 0u};
                else if (rec.len >= 16u)
                    data = shr_bytes(data, 16u - flen);
                else /* rare: a fragment under 16 bytes, read in place */
                    data = load_partial(in, rec.len);
                data = insert_byte(data, flen, ctype);
                const u32x4 o = data ^ ks;
                if (clen == 16u)
                    put(t, c, o);
                else
                    store_partial(out + 16u * c, clen, o);
                X = mask_tail(o, clen);
            } else if (clen >= 16u) {
                const u32x4 o = data ^ ks;
                put(t, c, o);
                X = SEAL ? o : data;
            } else {
                if (SEAL) {
                    if (rec.len >= 16u)
                        data = shr_bytes(data, 16u - clen);
                    else /* rare: a whole payload under 16 bytes, read in place */
                        data = load_partial(in, rec.len);
                }
                const u32x4 o = data ^ ks;
                store_partial(out + 16u * c, clen, o);
                X = mask_tail(SEAL ? o : data, clen);
            }
        } else if (is_aad) {
            if (FRAME) { /* 17 03 03 BE16(plen + 16) */
                const uint32_t reclen = plen + 16u;
                X[0] = 0x00030317u | ((reclen >> 8) & 0xffu) << 24;
                X[1] = reclen & 0xffu;
            } else if (use_seg && rec.aadlen < 16u) {
                X = load_partial(ad, rec.aadlen); /* segment walks: the short AAD may sit in any step */
            } else {
                X = 16u * (uint32_t)p + 16u <= rec.aadlen || rec.aadlen < 16u ? cur : shr_bytes(cur, 16u - arem);
            }
        } else if (is_len) {
            uint64_t abits = (uint64_t)aadlen * 8u, cbits = (uint64_t)plen * 8u;
            X[0] = bswap32((uint32_t)(abits >> 32));
            X[1] = bswap32((uint32_t)abits);
            X[2] = bswap32((uint32_t)(cbits >> 32));
            X[3] = bswap32((uint32_t)cbits);
            ek0 = SEAL ? ks : ks ^ cur; /* open: E(J0) ^ received tag */
        }
        if (active)
            acc = P ^ X;
    };

    /*
     * Two steps per trip with two load buffers: the block of step t+1 is in flight during step
     * t and the load of step t+2 reuses the registers step t has just consumed, so no register
     * copy (and no vmcnt(0) behind the step's own store) sits on the loop back-edge.
     */
    /*
     * An AAD shorter than 16 bytes (TLS: the 5-byte record header) is position 0, which lies in
     * step 0 (front padding < K): its lane reads it byte-exact into the first buffer.
     */
    /*
     * t0 (even, segment walks): the first step with a real position in any lane of the wave.  Steps before
     * it hold only front padding, and a Horner chain stays 0 through leading zero blocks.
     */
    GCM_WALK_STAMP(8);
    u32x4 bufA;
    if (!FRAME && !use_seg && valid && rec.aadlen != 0u && rec.aadlen < 16u && j == wk.pad)
        bufA = load_partial(ad, rec.aadlen);
    else
        bufA = walk_load(fetch_ptr(t0));
#if GCM_SPLIT_X2 && !GCM_ABLATE_AES && !GCM_ABLATE_GHASH
    if constexpr (LY::x2_walk) {
        static_assert(GCM_R2CACHE && !LY::four_tables, "the x2 walk runs the two-table rounds with round-2 caching");
        if (use_seg && Tmax == t0 + 2u) { /* wave-uniform: a whole segment in one trip */
            /*
             * Both steps' counter blocks in one interleaved AES (aes_ctr_x2_h): the walk's two dependent AES chains
             * become one, at the price of exposing the one Horner multiply (the chain is 0 before the segment's
             * first step, so that step's product is 0 and only the second one multiplies).
             */
            const u32x4 bufB = walk_load(fetch_ptr(t0 + 1u));
            const uint32_t ctrA = step_ctr(t0), ctrB = step_ctr(t0 + 1u);
            uint32_t o0 = iv0, o1 = iv1, o2 = iv2, ol = lanesel;
            if ((ctrA & WIN) != c1_hi) {
                c1_hi = ctrA & WIN;
                aes_round12_consts<false>(lds + LY::aes_base, ol, rk, o0, o1, o2, c1_hi, c1);
            }
            uint32_t c2[8];
            for (int i = 0; i < 8; ++i)
                c2[i] = c1[i];
            if ((ctrB & WIN) != c1_hi) /* the two blocks straddle a counter window */
                aes_round12_consts<false>(lds + LY::aes_base, ol, rk, o0, o1, o2, ctrB & WIN, c2);
            uint32_t wA[4] = {iv0, iv1, iv2, bswap32(ctrA)}, wB[4] = {iv0, iv1, iv2, bswap32(ctrB)};
            aes_ctr_x2_h<NR, LY::aes_base>(lds, lanesel, rk, c1, c2, ctrA, ctrB, wA, wB);
            finish(t0, bufA, u32x4{wA[0], wA[1], wA[2], wA[3]}, u32x4{0u, 0u, 0u, 0u});
            const u32x4 P = ghash_mul_scale<LY::wide_scale>(lds, LY::gh_base, acc);
            finish(t0 + 1u, bufB, u32x4{wB[0], wB[1], wB[2], wB[3]}, P);
            goto Scale;
        }
    }
#endif
    if (PF >= 3) {
        /*
         * Prefetch three steps ahead (window kernels at one wave per SIMD, where nothing else hides a load's
         * latency behind a step): four buffers, four steps per trip.
         */
        u32x4 b1 = walk_load(fetch_ptr(t0 + 1u)), b2 = walk_load(fetch_ptr(t0 + 2u));
        for (uint32_t t = t0; t < Tmax; t += 4u) {
            const u32x4 b3 = walk_load(fetch_ptr(t + 3u));
            step(t, bufA);
            bufA = walk_load(fetch_ptr(t + 4u));
            if (t + 1u < Tmax)
                step(t + 1u, b1);
            b1 = walk_load(fetch_ptr(t + 5u));
            if (t + 2u < Tmax)
                step(t + 2u, b2);
            b2 = walk_load(fetch_ptr(t + 6u));
            if (t + 3u < Tmax)
                step(t + 3u, b3);
        }
    } else {
        for (uint32_t t = t0; t < Tmax; t += 2u) {
            const u32x4 bufB = walk_load(fetch_ptr(t + 1u));
            GCM_WALK_STAMP(9);
            step(t, bufA);
            GCM_WALK_STAMP(10);
            bufA = walk_load(fetch_ptr(t + 2u));
            if (t + 1u < Tmax)
                step(t + 1u, bufB);
            GCM_WALK_STAMP(11);
        }
    }
#if GCM_SPLIT_X2 && !GCM_ABLATE_AES && !GCM_ABLATE_GHASH
Scale:
#endif
    GCM_WALK_STAMP(12);
    if constexpr (PAIRST) {
        if (pend_c != 0xffffffffu) /* a first half with no second half in this walk */
            GCM_WRITE(out + 16u * pend_c, 16), *(u32x4_u *)(out + 16u * pend_c) = pend_v;
    }
    /* scale the chain by H^(pad + g - q_last(j)) (make_walk) */
    if (LY::gh5) {
        /* H^e, e = 4 - slot in 1..4, from the nibble tables of H^2 (slot 0) and H^1 (slot 1) */
        const uint32_t e = (uint32_t)K - walk_scale_slot(wk, j, K, end_cap);
        acc = ghash_mul_lds(lds, LY::gh_base + (e >= 2u ? 0u : GH_TABLE_BYTES), acc);
        const u32x4 y = ghash_mul_lds(lds, LY::gh_base + (e == 4u ? 0u : GH_TABLE_BYTES), acc);
        if (e >= 3u)
            acc = y;
    } else if constexpr (LY::split_scale) {
        /* H^e, e = K - slot in 1..16: H^16 (gh_base) or H^e directly, else H^8 then H^(e - 8) (LayoutWin16) */
        uint32_t e = (uint32_t)K - walk_scale_slot(wk, j, K, end_cap);
        if (e > 8u && e < 16u) {
            acc = ghash_mul_scale<LY::wide_scale>(lds, LY::gh_pow1 + 7u * GH_TABLE_BYTES, acc);
            e -= 8u;
        }
        acc = ghash_mul_scale<LY::wide_scale>(lds, e == 16u ? LY::gh_base : LY::gh_pow1 + (e - 1u) * GH_TABLE_BYTES, acc);
    } else if (!GCM_ABLATE_SCALE) {
        /* GCM_SCALE_W: the reads issued in two batches of 16 (1) or all 32 (2) rather than as the compiler pairs them */
        acc = ghash_mul_join<GCM_SCALE_W>(lds, LY::gh_base + walk_scale_slot(wk, j, K, end_cap) * GH_TABLE_BYTES, acc);
    }
    GCM_WALK_STAMP(13);
    return acc ^ ek0;
}

template <int NR, int K, bool SEAL, bool FRAME = false, class LY = Layout<K>, int PF = 1>
GCM_HD u32x4 lane_walk(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, uint32_t j, const Record &rec, bool valid,
                       uint32_t Tmax, uint32_t iv0, uint32_t iv1, uint32_t iv2, const uint8_t *src, uint8_t *dst,
                       const uint8_t *aad, const uint8_t *dummy, uint32_t ctype = 0u, const Walk *seg = nullptr,
                       uint32_t t0 = 0u, const uint32_t *kr = nullptr, uint32_t f_lo = 0u, uint32_t f_hi = 0u)
{
    return lane_walk_seg<NR, K, SEAL, FRAME, LY, PF>(lds, lanesel, rk, j, rec, valid, Tmax, iv0, iv1, iv2, src, dst, aad,
                                                     dummy, ctype, seg != nullptr, seg != nullptr ? *seg : Walk{0, 0, 0, 0},
                                                     t0, kr, f_lo, f_hi);
}

} // namespace mi355x
