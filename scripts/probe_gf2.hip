/*
 * scripts/probe_gf2.hip -- measurement probe (not part of the product library): GHASH on the matrix cores, against
 * the nibble tables, inside the batch kernels' AES-CTR, compute-only (no HBM traffic: each keystream block is hashed
 * as if it were the data, as scripts/probe_bs.hip does).
 *
 * The GF(2) GEMM.  Four blocks X0..X3 of a record fold into its GHASH state as
 *     Y' = M(H^4)(Y ^ X0) ^ M(H^3) X1 ^ M(H^2) X2 ^ M(H) X3          (fusion's aggregated form, lib/fusion.c:151-185)
 * with M(c) the 128 x 128 GF(2) matrix of multiplication by c: one 128 x 512 bit matrix W times the 512 data bits.
 * On v_mfma_scale_f32_32x32x64_f8f6f4 with e2m1 (FP4) operands, 32 records per N tile:
 *   - data bits -> FP4 by AND masks alone: d & 0x11111111 puts bits 4m at nibble bit 0 (e2m1 0.5 b), & 0x22222222
 *     bits 4m+1 at nibble bit 1 (1.0 b), & 0x44444444 bits 4m+2 at nibble bit 2 (2.0 b), (d >> 3) & 0x11111111 bits
 *     4m+3 (0.5 b); W's entries are 2.0 / 1.0 / 0.5 / 2.0 for those, so every product is exactly 0 or 1;
 *   - the accumulator starts at 2^23: the f32 sum 2^23 + popcount keeps the parity in the mantissa's bit 0;
 *   - 4 M tiles x 8 K tiles = 32 MFMAs per 128 blocks (a wave step: lane (h, n) holds blocks 2h, 2h+1 of record n);
 *     W (32 KiB of FP4 fragments) is read from LDS per MFMA (ds_read_b128, linear, conflict-free);
 *   - the 64 parities of a lane half are packed with v_perm gathers (1.25 VALU per bit) and the upper half's two
 *     dwords cross to the lower half (Y is folded into block 0 there).
 *
 *   probe_gf2_run<MODE>  persistent 1024-thread groups, work in units of 16 wave steps of 128 blocks:
 *                        MODE 0 AES-CTR only (2 blocks per lane and step), 1 AES + MFMA GHASH (v_perm gather pack),
 *                        2 AES + nibble-table GHASH (the batch kernels' fused rounds, aes_ghash_fused_h, H^4 Horner per
 *                        lane), 3 AES + MFMA GHASH with the v_alignbit pack (W rows in its bit order)
 *   probe_gf2_check      one wave: the MFMA GHASH of given data (S chunks of 32 records x 4 blocks) -> Y per record
 *
 * Driven by scripts/probe_gf2.py.
 */
#include <hip/hip_runtime.h>
#include "../rapido_amd/csrc/gcm_core.h"

using namespace mi355x;

__constant__ AesTables c_tabs = AesTables();

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

namespace {
constexpr uint32_t W_BASE = 0x20000u; /* MODE 1: 32 KiB of W fragments; MODE 2: the nibble tables of H^4 (8 KiB) */
constexpr uint32_t LDS_BYTES = 0x28000u;

__device__ void fill(uint8_t *lds, const KeyImage *ki, const u32x4 *w, int mode)
{
    for (uint32_t i = threadIdx.x; i < 0x20000u / 16u; i += blockDim.x) { /* T0|T1 and T2|T3, bank-replicated */
        const uint32_t off = i * 16u, x = (off >> 8) & 0xffu;
        uint32_t v = c_tabs.t0[x];
        const uint32_t rot = ((off & 0x10000u) ? 16u : 0u) + ((off & 128u) ? 8u : 0u);
        if (rot)
            v = rotl32(v, (int)rot);
        *(u32x4 *)(lds + off) = u32x4{v, v, v, v};
    }
    if (mode == 1)
        for (uint32_t i = threadIdx.x; i < 0x8000u / 16u; i += blockDim.x)
            *(u32x4 *)(lds + W_BASE + 16u * i) = w[i];
    if (mode == 2)
        for (uint32_t i = threadIdx.x; i < GH_TABLE_BYTES / 16u; i += blockDim.x)
            *(u32x4 *)(lds + W_BASE + 16u * i) = ((const u32x4 *)ki->gh[3])[i];
}

/* one AES-CTR keystream block, the batch kernels' rounds without the fused GHASH reads (aes_ghash_fused_h) */
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
        m0 = m1 = m2 = m3 = 0u; /* (host pass of hipcc only) */
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

/* bytes 0 of a, b, c, d -> bytes 0..3 */
__device__ __forceinline__ uint32_t gather4(float a, float b, float c, float d)
{
    const uint32_t ab = perm(__float_as_uint(b), __float_as_uint(a), 0x0c0c0400u);
    const uint32_t cd = perm(__float_as_uint(d), __float_as_uint(c), 0x0c0c0400u);
    return perm(cd, ab, 0x05040100u);
}

/*
 * One chunk of 4 blocks of each of the wave's 32 records: lane (h, n) = (lane >> 5, lane & 31) holds blocks 2h and
 * 2h + 1 of record n, Y already folded into block 0.  Returns the lane half's 64 bits of Y': y0 = Y' dword 2h,
 * y1 = dword 2h + 1.  K tile t takes dword t & 3 of block 2h + (t >> 2) of the half; element j = 8q + m of a
 * fragment is nibble m of VGPR q (the hardware's K order is the same for A and B, so W's columns follow it).
 * Value i of M tile mt in lane half h is W row 32 mt + (i & 3) + 8 (i >> 2) + 4 h and Y' bit
 * 64 h + 32 (mt >> 1) + 4 (mt & 1) + 8 (i & 3) + (i >> 2) (scripts/probe_gf2.py builds W to that map).
 */
template <int PACK>
__device__ __forceinline__ void gf2_chunk(const uint8_t *lds, uint32_t lane, const u32x4 &b0, const u32x4 &b1,
                                          uint32_t &y0, uint32_t &y1)
{
    v8i B[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        const uint32_t d = t < 4 ? b0[t] : b1[t - 4];
        B[t] = v8i{(int)(d & 0x11111111u), (int)(d & 0x22222222u), (int)(d & 0x44444444u), (int)((d >> 3) & 0x11111111u),
                   0, 0, 0, 0};
    }
    uint32_t y[2] = {0u, 0u};
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        v16f acc;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            acc[i] = 8388608.0f; /* 2^23: the popcount's parity lands in the mantissa's bit 0 */
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const u32x4 a = lds_u32x4(lds, W_BASE + (uint32_t)(mt * 8 + t) * 1024u + lane * 16u);
            const v8i A = {(int)a[0], (int)a[1], (int)a[2], (int)a[3], 0, 0, 0, 0};
            /* immediate zero scales: the unscaled v_mfma_f32_32x32x64_f8f6f4 (holds the SIMD's issue ~17 cycles
             * instead of ~19, profiles/r03a_mfma_isa.json) */
            acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, B[t], acc, 4, 4, 0, 0, 0, 0);
        }
        if (PACK == 0) {
            uint32_t bits = 0u;
#pragma unroll
            for (int g = 0; g < 4; ++g) /* values 4g .. 4g + 3 -> bits 8k + g (k = value & 3) */
                bits |= (gather4(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]) & 0x01010101u) << g;
            y[mt >> 1] |= bits << (4 * (mt & 1));
        } else {
            /* v_alignbit: y = (y >> 1) | (parity << 31), one VALU per bit, no masking (W rows ordered to match) */
#pragma unroll
            for (int i = 0; i < 16; ++i)
                y[mt >> 1] = alignbit(__float_as_uint(acc[i]), y[mt >> 1], 1u);
        }
    }
    y0 = y[0];
    y1 = y[1];
}

/* Y' of the chunk, crossed so that the lower half holds all four dwords (and folds them into its block 0) */
__device__ __forceinline__ u32x4 gf2_fold(uint32_t lane, uint32_t y0, uint32_t y1)
{
    const uint32_t z0 = (uint32_t)__shfl_xor((int)y0, 32, 64), z1 = (uint32_t)__shfl_xor((int)y1, 32, 64);
    return lane < 32u ? u32x4{y0, y1, z0, z1} : u32x4{0u, 0u, 0u, 0u};
}

template <int NR, int MODE>
__device__ void run_body(const KeyImage *ki, const u32x4 *w, uint32_t nunits, uint32_t *work, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    fill(lds, ki, w, MODE);
    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); ++i)
        rk[i] = ki->rk[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u;
    const uint32_t iv0 = 0x03020100u ^ lane, iv1 = 0x07060504u ^ blockIdx.x, iv2 = 0x0b0a0908u ^ (threadIdx.x >> 6);
    uint32_t c1[8];
    aes_round12_consts<true>(lds, lanesel, rk, iv0, iv1, iv2, 0u, c1);
    u32x4 acc = {lane, threadIdx.x >> 6, 0u, 0u}, Y = {0u, 0u, 0u, 0u};
    uint32_t ctr = 2u;
    for (;;) {
        uint32_t g = 0;
        if (lane == 0)
            g = atomicAdd(work, 1u);
        g = (uint32_t)__shfl((int)g, 0, 64);
        if (g >= nunits)
            break;
        for (uint32_t s = 0; s < 16u; ++s) {
            if (MODE == 2) { /* two fused AES + nibble-table multiplies, one H^4 Horner chain per lane */
                uint32_t k0[4], k1[4];
                u32x4 P = aes_ghash_fused_h<NR, true, false, 0u>(lds, lanesel, rk, c1, ctr, k0, W_BASE, acc);
                acc = P ^ u32x4{k0[0], k0[1], k0[2], k0[3]};
                P = aes_ghash_fused_h<NR, true, false, 0u>(lds, lanesel, rk, c1, ctr + 1u, k1, W_BASE, acc);
                acc = P ^ u32x4{k1[0], k1[1], k1[2], k1[3]};
            } else {
                u32x4 x0 = aes_ctr_tt4<NR>(lds, lanesel, rk, c1, ctr);
                const u32x4 x1 = aes_ctr_tt4<NR>(lds, lanesel, rk, c1, ctr + 1u);
                if (MODE == 0) {
                    acc ^= x0 ^ x1;
                } else {
                    x0 ^= Y;
                    uint32_t y0, y1;
                    gf2_chunk<MODE == 3>(lds, lane, x0, x1, y0, y1);
                    Y = gf2_fold(lane, y0, y1);
                }
            }
            ctr = 2u + ((ctr + 2u) & 127u);
        }
    }
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    out[gid] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3] ^ Y[0] ^ Y[1] ^ Y[2] ^ Y[3];
}
} // namespace

#define RUN(NR, MODE)                                                                                                  \
    extern "C" __global__ __launch_bounds__(1024) void probe_gf2_run_##NR##_##MODE(const KeyImage *ki, const u32x4 *w,  \
                                                                                   uint32_t nunits, uint32_t *work,     \
                                                                                   uint32_t *out)                        \
    {                                                                                                                  \
        run_body<NR, MODE>(ki, w, nunits, work, out);                                                                  \
    }
RUN(10, 0)
RUN(10, 1)
RUN(10, 2)
RUN(10, 3)
RUN(14, 3)
RUN(14, 0)
RUN(14, 1)
RUN(14, 2)

/* one wave: Y of each of 32 records after S chunks (data[((s * 32 + n) * 4 + j) * 16], block j of record n) */
extern "C" __global__ __launch_bounds__(64) void probe_gf2_check(const u32x4 *w, const u32x4 *data, uint32_t S, u32x4 *y_out,
                                                                 uint32_t pack)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    for (uint32_t i = threadIdx.x; i < 0x8000u / 16u; i += blockDim.x)
        *(u32x4 *)(lds + W_BASE + 16u * i) = w[i];
    __syncthreads();
    const uint32_t lane = threadIdx.x, h = lane >> 5, n = lane & 31u;
    u32x4 Y = {0u, 0u, 0u, 0u};
    for (uint32_t s = 0; s < S; ++s) {
        u32x4 x0 = data[(s * 32u + n) * 4u + 2u * h], x1 = data[(s * 32u + n) * 4u + 2u * h + 1u];
        x0 ^= Y;
        uint32_t y0, y1;
        if (pack)
            gf2_chunk<1>(lds, lane, x0, x1, y0, y1);
        else
            gf2_chunk<0>(lds, lane, x0, x1, y0, y1);
        Y = gf2_fold(lane, y0, y1);
    }
    if (lane < 32u)
        y_out[n] = Y;
}

extern "C" __global__ void probe_gf2_setup(const uint8_t *key, uint32_t keylen, KeyImage *ki, int *rc)
{
    if (threadIdx.x == 0 && blockIdx.x == 0)
        *rc = build_key_image(c_tabs.sbox, key, keylen, ki);
}

/* ------------------------------------------------------------------ host entry points ---- */
extern "C" size_t probe_key_image_size(void) { return sizeof(KeyImage); }

extern "C" int probe_key(const void *d_key, uint32_t keylen, void *d_ki, int *d_rc, void *stream)
{
    hipLaunchKernelGGL(probe_gf2_setup, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint8_t *)d_key, keylen,
                       (KeyImage *)d_ki, d_rc);
    return (int)hipGetLastError();
}

extern "C" int probe_run(int nr, int mode, const void *d_ki, const void *d_w, uint32_t nunits, uint32_t nblocks,
                         void *d_work, void *d_out, void *stream)
{
    typedef void (*kern_t)(const KeyImage *, const u32x4 *, uint32_t, uint32_t *, uint32_t *);
    kern_t k = nr == 10 ? (mode == 0 ? probe_gf2_run_10_0 : mode == 1 ? probe_gf2_run_10_1 : mode == 2 ? probe_gf2_run_10_2 : probe_gf2_run_10_3)
                        : (mode == 0 ? probe_gf2_run_14_0 : mode == 1 ? probe_gf2_run_14_1 : mode == 2 ? probe_gf2_run_14_2 : probe_gf2_run_14_3);
    hipLaunchKernelGGL(k, dim3(nblocks), dim3(1024), 0, (hipStream_t)stream, (const KeyImage *)d_ki, (const u32x4 *)d_w,
                       nunits, (uint32_t *)d_work, (uint32_t *)d_out);
    return (int)hipGetLastError();
}

extern "C" int probe_check(const void *d_w, const void *d_data, uint32_t S, void *d_y, void *stream, uint32_t pack)
{
    hipLaunchKernelGGL(probe_gf2_check, dim3(1), dim3(64), 0, (hipStream_t)stream, (const u32x4 *)d_w,
                       (const u32x4 *)d_data, S, (u32x4 *)d_y, pack);
    return (int)hipGetLastError();
}

extern "C" const char *probe_err(int e) { return hipGetErrorString((hipError_t)e); }
