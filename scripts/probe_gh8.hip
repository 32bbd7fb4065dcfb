/*
 * scripts/probe_gh8.hip -- measurement probe (not part of the product library): GHASH from 8-bit "latin" tables
 * against the nibble tables, inside the batch kernels' AES-CTR, compute-only (each keystream block is hashed as if it
 * were the data, as scripts/probe_gf2.hip does).
 *
 * The 8-bit latin tables.  Multiplication by a constant c is linear, so X * c = XOR over the 16 byte positions p of
 * T_p[X_p] with T_p[e] = (e at byte p) * c.  A 64 KiB table holds all of them: row e (256 B, one full bank row of the
 * 64 banks) has T_p[e] in slot p, i.e. in bank group p.  A ds_read_b128 is served 16 lanes at a time; lane i
 * (= lane & 15) reads, at read r (0..15), byte position (r + i) & 15 of its X, so the 16 lanes of a pass hit 16
 * distinct bank groups whatever their bytes are: conflict-free, 16 reads per multiply instead of the nibble tables' 32.
 * (This probe first ran a rotate-by-i read order, lane i reading position (r + i) & 15 at read r; it now runs the
 * product's XOR order, position r ^ i, from gcm_core.h.)
 *
 * 64 KiB does not fit beside the four bank-replicated T-table images (128 KiB), so the AES runs on two of them
 * (T2 = rotl16(T0), T3 = rotl16(T1), as the K = 8 and window kernels do).  The rotated column costs one VALU more than
 * the four-table column when the round key is folded in before the rotation (rotl16(k) precomputed, wave-uniform):
 *     T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d] ^ rotl16(k)).
 *
 * LDS map: [0, 64K) GH8 table of H^4, [64K, 128K) the two-table AES image (T0 | T1, addressed through byte 2 of the
 * lane selector), [128K, 136K) the nibble tables of H^4 (modes that use them).  Four-table modes use [0, 128K) for the
 * AES images as the batch kernels do.
 *
 *   probe_gh8_run<NR, MODE>  persistent 1024-thread groups, units of 16 wave steps of 2 blocks per lane:
 *       0  AES (4 tables) only                         1  AES (2 tables, k folded) only
 *       2  AES (4 tables) + nibble GHASH (shipped)     3  AES (2 tables, k folded) + nibble GHASH
 *       4  AES (2 tables, k folded) + GH8 GHASH        5  AES (2 tables, plain tt2 column) + GH8 GHASH
 *   probe_gh8_check  one wave: Horner chains of X * H^4 by GH8 and by the nibble tables, both written out
 *
 * Driven by scripts/probe_gh8.py.
 */
#include <hip/hip_runtime.h>
#include "../rapido_amd/csrc/gcm_core.h"

using namespace mi355x;

__constant__ AesTables c_tabs = AesTables();

namespace {
constexpr uint32_t GH8_BASE = 0x00000u;
constexpr uint32_t AESB_BASE = 0x10000u; /* two-table image, reached with lanesel byte 2 = 1 */
constexpr uint32_t NIB_BASE = 0x20000u;
constexpr uint32_t LDS_BYTES = 0x28000u;

__device__ void fill(uint8_t *lds, const KeyImage *ki, int mode)
{
    const bool four = mode == 0 || mode == 2;
    for (uint32_t i = threadIdx.x; i < 0x20000u / 16u; i += blockDim.x) {
        const uint32_t off = i * 16u, x = (off >> 8) & 0xffu;
        if (!four && off < 0x10000u) {
            /* GH8 row e = off >> 8, slot p = (off >> 4) & 15: nibble tables 2p (low nibble) and 2p + 1 (high) */
            const uint32_t e = off >> 8, p = (off >> 4) & 15u;
            const u32x4 lo = *(const u32x4 *)ki->gh[3][2u * p][e & 15u];
            const u32x4 hi = *(const u32x4 *)ki->gh[3][2u * p + 1u][e >> 4];
            *(u32x4 *)(lds + off) = lo ^ hi;
            continue;
        }
        uint32_t v = c_tabs.t0[x];
        const uint32_t rot = ((four && (off & 0x10000u)) ? 16u : 0u) + ((off & 128u) ? 8u : 0u);
        if (rot)
            v = rotl32(v, (int)rot);
        *(u32x4 *)(lds + off) = u32x4{v, v, v, v};
    }
    if (mode == 2 || mode == 3)
        for (uint32_t i = threadIdx.x; i < GH_TABLE_BYTES / 16u; i += blockDim.x)
            *(u32x4 *)(lds + NIB_BASE + 16u * i) = ((const u32x4 *)ki->gh[3])[i];
}

/* T_t[byte kk of x] from the two-table image at AESB_BASE (lanesel byte 2 = 1) */
__device__ __forceinline__ uint32_t tlook_b(const uint8_t *lds, uint32_t lanesel, uint32_t x, uint32_t kk, int t)
{
    const uint32_t a = perm(x, lanesel, 0x0c020400u | ((4u + kk) << 8));
    const uint32_t v = lds_u32(lds, (t & 1) ? a + 128u : a);
    return t >= 2 ? rotl32(v, 16) : v;
}

/* one middle round on the two-table image B; KROT: column = T0a ^ T1b ^ rotl16(T0c ^ T1d ^ kr) (3 VALU),
 * else the tt2 column (xor, xor3 with k, rotate, xor: 4 VALU) */
template <bool KROT>
__device__ __forceinline__ void round_tt2b(uint32_t ls, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, const uint32_t *k,
                                           const uint32_t *kr, uint32_t &n0, uint32_t &n1, uint32_t &n2, uint32_t &n3)
{
    uint32_t t1, t2, t3, t5, t6, t7, t9, t10, t11, t13, t14, t15;
#define RB_READS                                                                                                       \
    "v_perm_b32 %[n0], %[s0], %[ls], %[a0]\n\t"                                                                        \
    "v_perm_b32 %[t1], %[s1], %[ls], %[a1]\n\t"                                                                        \
    "v_perm_b32 %[t2], %[s2], %[ls], %[a2]\n\t"                                                                        \
    "v_perm_b32 %[t3], %[s3], %[ls], %[a3]\n\t"                                                                        \
    "ds_read_b32 %[n0], %[n0]\n\t"                                                                                     \
    "ds_read_b32 %[t1], %[t1] offset:128\n\t"                                                                          \
    "ds_read_b32 %[t2], %[t2]\n\t"                                                                                     \
    "ds_read_b32 %[t3], %[t3] offset:128\n\t"                                                                          \
    "v_perm_b32 %[n1], %[s1], %[ls], %[a0]\n\t"                                                                        \
    "v_perm_b32 %[t5], %[s2], %[ls], %[a1]\n\t"                                                                        \
    "v_perm_b32 %[t6], %[s3], %[ls], %[a2]\n\t"                                                                        \
    "v_perm_b32 %[t7], %[s0], %[ls], %[a3]\n\t"                                                                        \
    "ds_read_b32 %[n1], %[n1]\n\t"                                                                                     \
    "ds_read_b32 %[t5], %[t5] offset:128\n\t"                                                                          \
    "ds_read_b32 %[t6], %[t6]\n\t"                                                                                     \
    "ds_read_b32 %[t7], %[t7] offset:128\n\t"                                                                          \
    "v_perm_b32 %[n2], %[s2], %[ls], %[a0]\n\t"                                                                        \
    "v_perm_b32 %[t9], %[s3], %[ls], %[a1]\n\t"                                                                        \
    "v_perm_b32 %[t10], %[s0], %[ls], %[a2]\n\t"                                                                       \
    "v_perm_b32 %[t11], %[s1], %[ls], %[a3]\n\t"                                                                       \
    "ds_read_b32 %[n2], %[n2]\n\t"                                                                                     \
    "ds_read_b32 %[t9], %[t9] offset:128\n\t"                                                                          \
    "ds_read_b32 %[t10], %[t10]\n\t"                                                                                   \
    "ds_read_b32 %[t11], %[t11] offset:128\n\t"                                                                        \
    "v_perm_b32 %[n3], %[s3], %[ls], %[a0]\n\t"                                                                        \
    "v_perm_b32 %[t13], %[s0], %[ls], %[a1]\n\t"                                                                       \
    "v_perm_b32 %[t14], %[s1], %[ls], %[a2]\n\t"                                                                       \
    "v_perm_b32 %[t15], %[s2], %[ls], %[a3]\n\t"                                                                       \
    "ds_read_b32 %[n3], %[n3]\n\t"                                                                                     \
    "ds_read_b32 %[t13], %[t13] offset:128\n\t"                                                                        \
    "ds_read_b32 %[t14], %[t14]\n\t"                                                                                   \
    "ds_read_b32 %[t15], %[t15] offset:128\n\t"
#define RB_OUTS                                                                                                        \
    : [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2), [n3] "=&v"(n3), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), \
      [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7), [t9] "=&v"(t9), [t10] "=&v"(t10), [t11] "=&v"(t11),              \
      [t13] "=&v"(t13), [t14] "=&v"(t14), [t15] "=&v"(t15)
#define RB_INS                                                                                                         \
    [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [ls] "v"(ls), [a0] "s"(0x0c020400u),                       \
        [a1] "s"(0x0c020500u), [a2] "s"(0x0c020600u), [a3] "s"(0x0c020700u)
    if (KROT) {
        asm volatile(RB_READS
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
                     RB_OUTS
                     : RB_INS, [r0] "s"(kr[0]), [r1] "s"(kr[1]), [r2] "s"(kr[2]), [r3] "s"(kr[3])
                     : "memory");
    } else {
        asm volatile(RB_READS
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
                     RB_OUTS
                     : RB_INS, [k0] "s"(k[0]), [k1] "s"(k[1]), [k2] "s"(k[2]), [k3] "s"(k[3])
                     : "memory");
    }
#undef RB_READS
#undef RB_OUTS
#undef RB_INS
}

/* the GH8 read order, rotation and reads are the product's own (gcm_core.h: Gh8Lane, gh8_lane, gh8_rotate,
 * gh8_issue2, gh8_acc2, gh8_mul_lds; round 3's first probe used a rotate-by-i variant with 4 lane constants) */

/*
 * AES-CTR on the two-table image B fused with P = A * H^4 (GH: 0 none, 1 nibble tables at NIB_BASE, 2 GH8):
 * rounds 1-2 from the window constants (5 reads), rounds 3..NR-1 as asm blocks with the GHASH reads of the round
 * issued ahead of them and accumulated after, the last round from T0's S-box bytes.
 */
template <int NR, bool KROT, int GH>
__device__ __forceinline__ u32x4 fused_b(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, const uint32_t *kr,
                                         const uint32_t *c, uint32_t ctr, uint32_t w[4], const u32x4 &A, const Gh8Lane &L)
{
    u32x4 P = {0u, 0u, 0u, 0u};
    u32x4 Ar = {0u, 0u, 0u, 0u};
    if (GH == 2)
        Ar = gh8_rotate(A, L);
    const uint32_t s3 = bswap32(ctr) ^ rk[3];
    const uint32_t n0 = c[0] ^ tlook_b(lds, lanesel, s3, 3, 3);
    uint32_t s0 = c[4] ^ tlook_b(lds, lanesel, n0, 0, 0), s1 = c[5] ^ tlook_b(lds, lanesel, n0, 3, 3);
    uint32_t s2 = c[6] ^ tlook_b(lds, lanesel, n0, 2, 2), s3r = c[7] ^ tlook_b(lds, lanesel, n0, 1, 1);
    if (GH == 1)
        ghash_quarter(lds, (NIB_BASE >> 8) << 8, A[0], 0, 0, P);
    if (GH == 2) {
        u32x4 g[2];
        gh8_issue2(lds, Ar, L, 0, g);
        gh8_acc2(g, P);
    }
    GCM_SCHED_FENCE();
#pragma unroll
    for (int r = 3; r < NR; ++r) {
        uint32_t m0, m1, m2, m3;
        u32x4 g[4];
        const bool gh = r <= 9;
        if (GH == 1 && gh)
            ghash_quarter_issue(lds, (NIB_BASE >> 8) << 8, A[(r - 2) >> 1], (r - 2) >> 1, ((r - 2) & 1) * 2, g);
        if (GH == 2 && gh)
            gh8_issue2(lds, Ar, L, 2 * (r - 2), g);
#if defined(__HIP_DEVICE_COMPILE__)
        round_tt2b<KROT>(lanesel, s0, s1, s2, s3r, rk + 4 * r, kr + 4 * r, m0, m1, m2, m3);
#else
        m0 = m1 = m2 = m3 = 0u;
#endif
        if (GH == 1 && gh)
            ghash_quarter_acc(g, P);
        if (GH == 2 && gh)
            gh8_acc2(g, P);
        GCM_SCHED_FENCE();
        s0 = m0;
        s1 = m1;
        s2 = m2;
        s3r = m3;
    }
    const uint32_t *k = rk + 4 * NR;
    const uint32_t x[4] = {s0, s1, s2, s3r};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t ra = lds_u32(lds, perm(x[j], lanesel, 0x0c020400u));
        const uint32_t rb = lds_u32(lds, perm(x[(j + 1) & 3], lanesel, 0x0c020500u));
        const uint32_t rc = lds_u32(lds, perm(x[(j + 2) & 3], lanesel, 0x0c020600u));
        const uint32_t rd = lds_u32(lds, perm(x[(j + 3) & 3], lanesel, 0x0c020700u));
        w[j] = xor3(perm(rb, ra, 0x0c0c0501u), perm(rd, rc, 0x06020c0cu), k[j]);
    }
    return P;
}

/* one AES-CTR keystream block on the four-table image (the batch kernels' rounds without GHASH) */
template <int NR>
__device__ __forceinline__ u32x4 aes_ctr_tt4(const uint8_t *lds, uint32_t lanesel, const uint32_t *rk, const uint32_t *c,
                                             uint32_t ctr)
{
    const uint32_t s3 = bswap32(ctr) ^ rk[3];
    const uint32_t n0 = c[0] ^ tlook<true>(lds, lanesel, s3, 3, 3);
    uint32_t s0 = c[4] ^ tlook<true>(lds, lanesel, n0, 0, 0), s1 = c[5] ^ tlook<true>(lds, lanesel, n0, 3, 3);
    uint32_t s2 = c[6] ^ tlook<true>(lds, lanesel, n0, 2, 2), s3r = c[7] ^ tlook<true>(lds, lanesel, n0, 1, 1);
    GCM_SCHED_FENCE();
#pragma unroll
    for (int r = 3; r < NR; ++r) {
        uint32_t m0, m1, m2, m3;
#if defined(__HIP_DEVICE_COMPILE__)
        aes_round_tt4_asm<0u>(lanesel, s0, s1, s2, s3r, rk + 4 * r, m0, m1, m2, m3);
#else
        m0 = m1 = m2 = m3 = 0u;
#endif
        GCM_SCHED_FENCE();
        s0 = m0;
        s1 = m1;
        s2 = m2;
        s3r = m3;
    }
    const uint32_t *k = rk + 4 * NR;
    const uint32_t x[4] = {s0, s1, s2, s3r};
    u32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t ra = lds_u32(lds, perm(x[j], lanesel, 0x0c0c0400u));
        const uint32_t rb = lds_u32(lds, perm(x[(j + 1) & 3], lanesel, 0x0c0c0500u));
        const uint32_t rc = lds_u32(lds, perm(x[(j + 2) & 3], lanesel, 0x0c0c0600u));
        const uint32_t rd = lds_u32(lds, perm(x[(j + 3) & 3], lanesel, 0x0c0c0700u));
        w[j] = xor3(perm(rb, ra, 0x0c0c0501u), perm(rd, rc, 0x06020c0cu), k[j]);
    }
    return w;
}

template <int NR, int MODE>
__device__ void run_body(const KeyImage *ki, uint32_t nunits, uint32_t *work, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    fill(lds, ki, MODE);
    uint32_t rk[4 * (NR + 1)], kr[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); ++i) {
        rk[i] = ki->rk[i];
        kr[i] = rotl32(rk[i], 16);
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const bool four = MODE == 0 || MODE == 2;
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u;
    const Gh8Lane L = gh8_lane(lane & 15u);
    const uint32_t iv0 = 0x03020100u ^ lane, iv1 = 0x07060504u ^ blockIdx.x, iv2 = 0x0b0a0908u ^ (threadIdx.x >> 6);
    uint32_t c1[8];
    if (four)
        aes_round12_consts<true>(lds, lanesel, rk, iv0, iv1, iv2, 0u, c1);
    else
        aes_round12_consts<false>(lds + AESB_BASE, lanesel & 0xffffu, rk, iv0, iv1, iv2, 0u, c1);
    u32x4 acc = {lane, threadIdx.x >> 6, 0u, 0u};
    uint32_t ctr = 2u;
    for (;;) {
        uint32_t g = 0;
        if (lane == 0)
            g = atomicAdd(work, 1u);
        g = (uint32_t)__shfl((int)g, 0, 64);
        if (g >= nunits)
            break;
        for (uint32_t s = 0; s < 16u; ++s) {
            if (MODE == 0) {
                acc ^= aes_ctr_tt4<NR>(lds, lanesel, rk, c1, ctr) ^ aes_ctr_tt4<NR>(lds, lanesel, rk, c1, ctr + 1u);
            } else if (MODE == 2) {
                uint32_t k0[4], k1[4];
                u32x4 P = aes_ghash_fused_h<NR, true, false, 0u>(lds, lanesel, rk, c1, ctr, k0, NIB_BASE, acc);
                acc = P ^ u32x4{k0[0], k0[1], k0[2], k0[3]};
                P = aes_ghash_fused_h<NR, true, false, 0u>(lds, lanesel, rk, c1, ctr + 1u, k1, NIB_BASE, acc);
                acc = P ^ u32x4{k1[0], k1[1], k1[2], k1[3]};
            } else {
                constexpr bool KROT = MODE != 5;
                constexpr int GH = MODE == 1 ? 0 : MODE == 3 ? 1 : 2;
                uint32_t k0[4], k1[4];
                u32x4 P = fused_b<NR, KROT, GH>(lds, lanesel, rk, kr, c1, ctr, k0, acc, L);
                acc = (GH ? P : acc) ^ u32x4{k0[0], k0[1], k0[2], k0[3]};
                P = fused_b<NR, KROT, GH>(lds, lanesel, rk, kr, c1, ctr + 1u, k1, acc, L);
                acc = (GH ? P : acc) ^ u32x4{k1[0], k1[1], k1[2], k1[3]};
            }
            ctr = 2u + ((ctr + 2u) & 127u);
        }
    }
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    out[gid] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
}
} // namespace

#define RUN(NR, MODE)                                                                                                  \
    extern "C" __global__ __launch_bounds__(1024) void probe_gh8_run_##NR##_##MODE(const KeyImage *ki, uint32_t nunits, \
                                                                                   uint32_t *work, uint32_t *out)      \
    {                                                                                                                  \
        run_body<NR, MODE>(ki, nunits, work, out);                                                                     \
    }
RUN(10, 0)
RUN(10, 1)
RUN(10, 2)
RUN(10, 3)
RUN(10, 4)
RUN(10, 5)
RUN(14, 0)
RUN(14, 1)
RUN(14, 2)
RUN(14, 3)
RUN(14, 4)
RUN(14, 5)

/* one wave: S chained Horner steps A = (A ^ data[s][lane]) * H^4 by GH8 (out[lane]) and by the nibble tables
 * (out[64 + lane]) */
extern "C" __global__ __launch_bounds__(64) void probe_gh8_check(const KeyImage *ki, const u32x4 *data, uint32_t S, u32x4 *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    fill(lds, ki, 3);
    __syncthreads();
    const uint32_t lane = threadIdx.x;
    const Gh8Lane L = gh8_lane(lane & 15u);
    u32x4 A = {0u, 0u, 0u, 0u}, B = {0u, 0u, 0u, 0u};
    for (uint32_t s = 0; s < S; ++s) {
        const u32x4 d = data[s * 64u + lane];
        A = gh8_mul_lds(lds, A ^ d, L);
        B = ghash_mul_lds(lds, (NIB_BASE >> 8) << 8, B ^ d);
    }
    out[lane] = A;
    out[64u + lane] = B;
}

extern "C" __global__ void probe_gh8_setup(const uint8_t *key, uint32_t keylen, KeyImage *ki, int *rc)
{
    if (threadIdx.x == 0 && blockIdx.x == 0)
        *rc = build_key_image(c_tabs.sbox, key, keylen, ki);
}

/* ------------------------------------------------------------------ host entry points ---- */
extern "C" size_t probe_key_image_size(void) { return sizeof(KeyImage); }

extern "C" int probe_key(const void *d_key, uint32_t keylen, void *d_ki, int *d_rc, void *stream)
{
    hipLaunchKernelGGL(probe_gh8_setup, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint8_t *)d_key, keylen,
                       (KeyImage *)d_ki, d_rc);
    return (int)hipGetLastError();
}

extern "C" int probe_run(int nr, int mode, const void *d_ki, uint32_t nunits, uint32_t nblocks, void *d_work, void *d_out,
                         void *stream)
{
    typedef void (*kern_t)(const KeyImage *, uint32_t, uint32_t *, uint32_t *);
    static const kern_t k10[6] = {probe_gh8_run_10_0, probe_gh8_run_10_1, probe_gh8_run_10_2,
                                  probe_gh8_run_10_3, probe_gh8_run_10_4, probe_gh8_run_10_5};
    static const kern_t k14[6] = {probe_gh8_run_14_0, probe_gh8_run_14_1, probe_gh8_run_14_2,
                                  probe_gh8_run_14_3, probe_gh8_run_14_4, probe_gh8_run_14_5};
    if (mode < 0 || mode > 5)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(nr == 10 ? k10[mode] : k14[mode], dim3(nblocks), dim3(1024), 0, (hipStream_t)stream,
                       (const KeyImage *)d_ki, nunits, (uint32_t *)d_work, (uint32_t *)d_out);
    return (int)hipGetLastError();
}

extern "C" int probe_check(const void *d_ki, const void *d_data, uint32_t S, void *d_out, void *stream)
{
    hipLaunchKernelGGL(probe_gh8_check, dim3(1), dim3(64), 0, (hipStream_t)stream, (const KeyImage *)d_ki,
                       (const u32x4 *)d_data, S, (u32x4 *)d_out);
    return (int)hipGetLastError();
}

extern "C" const char *probe_err(int e) { return hipGetErrorString((hipError_t)e); }
