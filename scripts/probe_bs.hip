/*
 * scripts/probe_bs.hip -- measurement probe (not part of the product library): how much AES-CTR +
 * GHASH throughput a CU delivers when some of its 16 waves run the LDS T-table AES (gcm_core.h)
 * and the others the VALU bitsliced AES (gcm_bitslice.h).  No HBM traffic: each step's keystream is
 * hashed as if it were the data, so the probe isolates the compute mix the batch kernels run.
 *
 *   probe_mix    persistent 1024-thread workgroups; waves < n_tt run T-table steps (64 blocks per
 *                wave step), the rest bitsliced steps (128 blocks per wave step); work is taken in
 *                chunks of 16 "units" of 64 blocks from an atomic counter.
 *   probe_check  keystream of the bitsliced path for 128 counter blocks (correctness on the GPU).
 *
 * Built and driven by scripts/probe_bs.py.
 */
#include <hip/hip_runtime.h>
#include "../rapido_amd/csrc/gcm_core.h"
#include "gcm_bitslice.h"

using namespace mi355x;

__constant__ AesTables c_tabs = AesTables();

namespace {
constexpr uint32_t GH = 0x20000u;           /* nibble tables of H^4 */
constexpr uint32_t KP = 0x20000u + 0x2000u; /* key planes */
constexpr uint32_t LDS_BYTES = KP + KEYPLANE_BYTES;

__device__ void fill(uint8_t *lds, const KeyImage *ki)
{
    for (uint32_t i = threadIdx.x; i < 0x20000u / 16u; i += blockDim.x) {
        const uint32_t off = i * 16u, x = (off >> 8) & 0xffu;
        uint32_t v = c_tabs.t0[x];
        const uint32_t rot = ((off & 0x10000u) ? 16u : 0u) + ((off & 128u) ? 8u : 0u);
        if (rot)
            v = rotl32(v, (int)rot);
        *(u32x4 *)(lds + off) = u32x4{v, v, v, v};
    }
    for (uint32_t i = threadIdx.x; i < GH_TABLE_BYTES / 16u; i += blockDim.x)
        *(u32x4 *)(lds + GH + 16u * i) = ((const u32x4 *)ki->gh[3])[i];
    fill_keyplanes(lds + KP, ki->rk, ki->rounds, threadIdx.x, blockDim.x);
}

template <int NR>
__device__ void mix_body(const KeyImage *ki, uint32_t n_tt, uint32_t nunits, uint32_t *work, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    fill(lds, ki);
    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); ++i)
        rk[i] = ki->rk[i];
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t iv0 = 0x03020100u ^ lane, iv1 = 0x07060504u ^ blockIdx.x, iv2 = 0x0b0a0908u;
    u32x4 acc = {lane, wave, 0u, 0u};
    if (wave < n_tt) {
        const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u;
        uint32_t c1[8];
        aes_round12_consts<true>(lds, lanesel, rk, iv0, iv1, iv2, 0u, c1);
        uint32_t ctr = 2u;
        for (;;) {
            uint32_t g = 0;
            if (lane == 0)
                g = atomicAdd(work, 16u);
            g = (uint32_t)__shfl((int)g, 0, 64);
            if (g >= nunits)
                break;
            for (uint32_t s = 0; s < 16u; ++s) {
                uint32_t w[4] = {iv0, iv1, iv2, bswap32(ctr)};
                const u32x4 P = aes_ghash_fused_h<NR, true>(lds, lanesel, rk, c1, ctr, w, GH, acc);
                acc = P ^ u32x4{w[0], w[1], w[2], w[3]};
                ctr = 2u + ((ctr + 1u) & 127u);
            }
        }
    } else {
        QuadOpsDev o(lane);
        uint32_t ctr0 = 8u * (lane >> 2);
        for (;;) {
            uint32_t g = 0;
            if (lane == 0)
                g = atomicAdd(work, 16u);
            g = (uint32_t)__shfl((int)g, 0, 64);
            if (g >= nunits)
                break;
#if PROBE_ILP2
            for (uint32_t s = 0; s < 4u; ++s) {
                uint32_t ks[4][4];
                ctr_keystream_bs2<NR>(o, lds, KP, iv0, iv1, iv2, ctr0, ctr0 + 128u, ks);
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc = ghash_mul_lds(lds, GH, acc ^ u32x4{ks[b][0], ks[b][1], ks[b][2], ks[b][3]});
                ctr0 += 256u;
            }
#else
            for (uint32_t s = 0; s < 8u; ++s) {
                uint32_t ka[4], kb[4];
                ctr_keystream_bs<NR>(o, lds, KP, iv0, iv1, iv2, ctr0, ka, kb);
                acc = ghash_mul_lds(lds, GH, acc ^ u32x4{ka[0], ka[1], ka[2], ka[3]});
                acc = ghash_mul_lds(lds, GH, acc ^ u32x4{kb[0], kb[1], kb[2], kb[3]});
                ctr0 += 128u;
            }
#endif
        }
    }
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    out[gid] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
}
} // namespace

extern "C" __global__ __launch_bounds__(1024) void probe_mix128(const KeyImage *ki, uint32_t n_tt, uint32_t nunits,
                                                                 uint32_t *work, uint32_t *out)
{
    mix_body<10>(ki, n_tt, nunits, work, out);
}

extern "C" __global__ __launch_bounds__(1024) void probe_mix256(const KeyImage *ki, uint32_t n_tt, uint32_t nunits,
                                                                 uint32_t *work, uint32_t *out)
{
    mix_body<14>(ki, n_tt, nunits, work, out);
}

/* one wave: quad m encrypts counters ctr0 + 8m .. ctr0 + 8m + 7; out = 128 blocks in counter order */
extern "C" __global__ __launch_bounds__(64) void probe_check(const KeyImage *ki, uint32_t n0, uint32_t n1, uint32_t n2,
                                                             uint32_t ctr0, uint8_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t kp[KEYPLANE_BYTES];
    fill_keyplanes(kp, ki->rk, ki->rounds, threadIdx.x, blockDim.x);
    __syncthreads();
    const uint32_t lane = threadIdx.x, quad = lane >> 2, t = lane & 3u;
    QuadOpsDev o(lane);
    uint32_t ka[4], kb[4];
    if (ki->rounds == 10)
        ctr_keystream_bs<10>(o, kp, 0u, n0, n1, n2, ctr0 + 8u * quad, ka, kb);
    else
        ctr_keystream_bs<14>(o, kp, 0u, n0, n1, n2, ctr0 + 8u * quad, ka, kb);
    uint32_t *oa = (uint32_t *)(out + 16u * (8u * quad + t)), *ob = (uint32_t *)(out + 16u * (8u * quad + t + 4u));
    for (int d = 0; d < 4; ++d) {
        oa[d] = ka[d];
        ob[d] = kb[d];
    }
}

extern "C" __global__ void probe_setup(const uint8_t *key, uint32_t keylen, KeyImage *ki, int *rc)
{
    if (threadIdx.x == 0 && blockIdx.x == 0)
        *rc = build_key_image(c_tabs.sbox, key, keylen, ki);
}

/* ------------------------------------------------------------------ host entry points ---- */
extern "C" int probe_key(const void *d_key, uint32_t keylen, void *d_ki, int *d_rc, void *stream)
{
    hipLaunchKernelGGL(probe_setup, dim3(1), dim3(64), 0, (hipStream_t)stream, (const uint8_t *)d_key, keylen,
                       (KeyImage *)d_ki, d_rc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" size_t probe_key_image_size(void) { return sizeof(KeyImage); }

extern "C" int probe_run(const void *d_ki, int nr, uint32_t n_tt, uint32_t nunits, uint32_t nblocks, void *d_work,
                         void *d_out, void *stream, uint32_t threads)
{
    if (nr == 10)
        hipLaunchKernelGGL(probe_mix128, dim3(nblocks), dim3(threads), 0, (hipStream_t)stream, (const KeyImage *)d_ki, n_tt,
                           nunits, (uint32_t *)d_work, (uint32_t *)d_out);
    else
        hipLaunchKernelGGL(probe_mix256, dim3(nblocks), dim3(threads), 0, (hipStream_t)stream, (const KeyImage *)d_ki, n_tt,
                           nunits, (uint32_t *)d_work, (uint32_t *)d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int probe_check_run(const void *d_ki, uint32_t n0, uint32_t n1, uint32_t n2, uint32_t ctr0, void *d_out,
                               void *stream)
{
    hipLaunchKernelGGL(probe_check, dim3(1), dim3(64), 0, (hipStream_t)stream, (const KeyImage *)d_ki, n0, n1, n2, ctr0,
                       (uint8_t *)d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
