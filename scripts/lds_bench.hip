/*
 * scripts/lds_bench.hip -- LDS read-rate microbenchmark (measurement only, not the product).
 *
 * Measures how many wave-level LDS reads per clock a CU sustains with the access patterns of the
 * batch kernels: bank-replicated T-table lookups (ds_read_b32, lane l reads bank l & 31 of a random
 * 256-byte row) and nibble-table GHASH lookups (ds_read_b128, one 256-byte row per table).
 * 16 waves per CU, each keeping a batch of independent reads in flight (XOR-accumulated so
 * nothing is dead), one workgroup per CU.
 *   mode 0: b32 only   mode 1: b128 only   mode 2: 133 b32 : 32 b128 (an AES-128-GCM block)
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__device__ void body(uint32_t iters, uint32_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[0x20000 + 0x8000];
    for (uint32_t i = threadIdx.x; i < (0x28000u / 16u); i += blockDim.x)
        *(u32x4 *)(lds + 16u * i) = u32x4{i, i * 3u, i * 5u, i * 7u};
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    /* four state words as in the AES kernels; one v_perm per address (row byte -> bits 8-15, bank -> bits 0-7) */
    uint32_t s0 = 0x9e3779b9u * (threadIdx.x + 1u) ^ blockIdx.x, s1 = s0 * 3u + 1u, s2 = s0 * 5u + 7u, s3 = s0 * 7u + 3u;
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u;
    uint32_t acc = 0;
    u32x4 acc4 = {0u, 0u, 0u, 0u};
    for (uint32_t it = 0; it < iters; ++it) {
        if (MODE == 0 || MODE == 2) {
            uint32_t v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t w = (k & 3) == 0 ? s0 : (k & 3) == 1 ? s1 : (k & 3) == 2 ? s2 : s3;
                const uint32_t sel = ((k & 2) ? 0x0c020400u : 0x0c0c0400u) | ((4u + (uint32_t)(k >> 2)) << 8);
                v[k] = *(const uint32_t *)(lds + __builtin_amdgcn_perm(w, lanesel, sel) + ((k & 1) ? 128u : 0u));
            }
#pragma unroll
            for (int k = 0; k < 16; k += 2)
                acc = __builtin_amdgcn_bitop3_b32(acc, v[k], v[k + 1], 0x96);
        }
        if (MODE == 3 || MODE == 4) {
            /* 16 T-table style reads as ds_read_b64: lane l reads the 8-byte slot l & 31 of a random row */
            const uint32_t lanesel8 = (lane & 31u) * 8u | 0x10000u;
            uint32_t v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t w = (k & 3) == 0 ? s0 : (k & 3) == 1 ? s1 : (k & 3) == 2 ? s2 : s3;
                const uint32_t sel = ((k & 2) ? 0x0c020400u : 0x0c0c0400u) | ((4u + (uint32_t)(k >> 2)) << 8);
                const uint32_t a = __builtin_amdgcn_perm(w, lanesel8, sel);
                typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
                const u32x2 d = *(const u32x2 *)(lds + a);
                v[k] = (k & 1) ? d[1] : d[0];
            }
#pragma unroll
            for (int k = 0; k < 16; k += 2)
                acc = __builtin_amdgcn_bitop3_b32(acc, v[k], v[k + 1], 0x96);
        }
        if (MODE == 1 || ((MODE == 2 || MODE == 4) && (it & 3u) == 0u)) {
            u32x4 g[16];
            const uint32_t lo = (s0 << 4) & 0xf0f0f0f0u, hi = s0 & 0xf0f0f0f0u;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const uint32_t sel = 0x0c020100u | (4u + (uint32_t)(k & 3));
                g[k] = *(const u32x4 *)(lds + __builtin_amdgcn_perm((k & 4) ? hi : lo, 0x20000u, sel) + ((uint32_t)k << 8));
            }
#pragma unroll
            for (int k = 0; k < 16; k += 2)
                acc4 = u32x4{(uint32_t)__builtin_amdgcn_bitop3_b32(acc4[0], g[k][0], g[k + 1][0], 0x96),
                             (uint32_t)__builtin_amdgcn_bitop3_b32(acc4[1], g[k][1], g[k + 1][1], 0x96),
                             (uint32_t)__builtin_amdgcn_bitop3_b32(acc4[2], g[k][2], g[k + 1][2], 0x96),
                             (uint32_t)__builtin_amdgcn_bitop3_b32(acc4[3], g[k][3], g[k + 1][3], 0x96)};
        }
        /* next state: independent of the loaded values (no latency chain), one op per word */
        s0 = __builtin_amdgcn_alignbit(s0, s0, 7u) + 0x9e3779b9u;
        s1 = __builtin_amdgcn_alignbit(s1, s1, 11u) + 0x7f4a7c15u;
        s2 = __builtin_amdgcn_alignbit(s2, s2, 13u) + 0x94d049bbu;
        s3 = __builtin_amdgcn_alignbit(s3, s3, 17u) + 0x2545f491u;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ acc4[0] ^ acc4[1] ^ acc4[2] ^ acc4[3];
}

extern "C" __global__ __launch_bounds__(1024) void lds_b32(uint32_t iters, uint32_t *out) { body<0>(iters, out); }
extern "C" __global__ __launch_bounds__(1024) void lds_b128(uint32_t iters, uint32_t *out) { body<1>(iters, out); }
extern "C" __global__ __launch_bounds__(1024) void lds_mix(uint32_t iters, uint32_t *out) { body<2>(iters, out); }
extern "C" __global__ __launch_bounds__(1024) void lds_b64(uint32_t iters, uint32_t *out) { body<3>(iters, out); }
extern "C" __global__ __launch_bounds__(1024) void lds_mix64(uint32_t iters, uint32_t *out) { body<4>(iters, out); }

extern "C" int lds_bench_run(int mode, uint32_t iters, uint32_t nblocks, uint32_t threads, void *out, void *stream)
{
    void (*k)(uint32_t, uint32_t *) = mode == 0 ? lds_b32 : mode == 1 ? lds_b128 : mode == 2 ? lds_mix : mode == 3 ? lds_b64 : lds_mix64;
    hipLaunchKernelGGL(k, dim3(nblocks), dim3(threads), 0, (hipStream_t)stream, iters, (uint32_t *)out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
