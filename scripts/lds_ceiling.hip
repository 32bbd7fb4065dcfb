/*
 * scripts/lds_ceiling.hip -- the LDS ceiling of the batch kernels' exact read mix (measurement only, not the product).
 *
 * One 16-B block of the GH8 batch kernels (gcm_core.h aes_gh8_fused_h) costs, per lane:
 *   AES-128: 133 ds_read_b32 (bank-replicated T-table lookups: lane l reads bank l & 31 of a random 256-B row of the
 *            two-table image at LDS 64K, address = one v_perm of a state byte, as the kernels form it)
 *   AES-256: 197 ds_read_b32
 *   GHASH:   16 ds_read_b128 from the 8-bit latin table at LDS 0 (row e = a random byte, 256 B; read r of lane i takes
 *            slot r ^ (i & 15): 16 distinct bank groups per pass, conflict-free)
 * This probe issues exactly that mix per block -- 8 rounds of 16 b32 + 2 b128, then the remaining 5 (or 69) b32 --
 * with 16 waves per CU, addresses from a hash chain independent of the loaded values (nothing waits on a load but its
 * XOR), and no HBM traffic.  Blocks per second per CU at the measured clock give the LDS cycles one block really
 * costs: the measured ceiling the bench line's lds_roofline is priced against (the nominal 2 / 4 clk per b32 / b128
 * read model gives 330 / 458 clk per 64 blocks).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int EXTRA_B32, bool B32, bool B128>
__device__ void body(uint32_t blocks, uint32_t *out, uint64_t *stamps)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[0x20000];
    for (uint32_t i = threadIdx.x; i < (0x20000u / 16u); i += blockDim.x)
        *(u32x4 *)(lds + 16u * i) = u32x4{i, i * 3u, i * 5u, i * 7u};
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, gi = lane & 15u;
    uint32_t s0 = 0x9e3779b9u * (threadIdx.x + 1u) ^ blockIdx.x, s1 = s0 * 3u + 1u, s2 = s0 * 5u + 7u, s3 = s0 * 7u + 3u;
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u; /* bank + the two-table image at 64K */
    uint32_t acc = 0;
    u32x4 acc4 = {0u, 0u, 0u, 0u};
    /* the in-kernel clock (MI355X_MICROARCH.md, DVFS item 6): shader cycles and 100 MHz ticks around the loop */
    __syncthreads();
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t b = 0; b < blocks; ++b) {
#pragma unroll
        for (int round = 0; round < 8; ++round) {
            if (B32) {
                uint32_t v[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    const uint32_t w = (k & 3) == 0 ? s0 : (k & 3) == 1 ? s1 : (k & 3) == 2 ? s2 : s3;
                    const uint32_t sel = 0x0c020400u | ((4u + (uint32_t)(k >> 2)) << 8); /* 64K | row << 8 | bank */
                    v[k] = *(const uint32_t *)(lds + (__builtin_amdgcn_perm(w, lanesel, sel) | ((k & 1) ? 0x80u : 0u)));
                }
#pragma unroll
                for (int k = 0; k < 16; k += 2)
                    acc = __builtin_amdgcn_bitop3_b32(acc, v[k], v[k + 1], 0x96);
            }
            if (B128) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const uint32_t r = 2u * (uint32_t)round + (uint32_t)q, p = r ^ gi;
                    const uint32_t w = q ? s2 : s1;
                    const uint32_t e = (w >> (8u * (r & 3u))) & 0xffu;
                    const u32x4 g = *(const u32x4 *)(lds + (e << 8) + (p << 4));
                    acc4 ^= g;
                }
            }
            s0 = __builtin_amdgcn_alignbit(s0, s0, 7u) + 0x9e3779b9u;
            s1 = __builtin_amdgcn_alignbit(s1, s1, 11u) + 0x7f4a7c15u;
            s2 = __builtin_amdgcn_alignbit(s2, s2, 13u) + 0x94d049bbu;
            s3 = __builtin_amdgcn_alignbit(s3, s3, 17u) + 0x2545f491u;
            __builtin_amdgcn_sched_barrier(0); /* a round's reads stay in its round, as in the kernels (no spills) */
        }
        if (B32 && EXTRA_B32 > 0) {
#pragma unroll
            for (int k = 0; k < EXTRA_B32; ++k) {
                const uint32_t w = (k & 3) == 0 ? s0 : (k & 3) == 1 ? s1 : (k & 3) == 2 ? s2 : s3;
                const uint32_t sel = 0x0c020400u | ((4u + (uint32_t)((k >> 2) & 3)) << 8);
                acc ^= *(const uint32_t *)(lds + (__builtin_amdgcn_perm(w + (uint32_t)k, lanesel, sel)));
            }
            s0 = __builtin_amdgcn_alignbit(s0, s0, 5u) + 0x2545f491u;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ acc4[0] ^ acc4[1] ^ acc4[2] ^ acc4[3];
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

/* an AES-128-GCM block: 133 b32 + 16 b128; AES-256: 197 + 16; and each read kind alone */
#define CEIL_KERNEL(NAME, X, A, B)                                                                                     \
    extern "C" __global__ __launch_bounds__(1024) void NAME(uint32_t n, uint32_t *o, uint64_t *st)                      \
    {                                                                                                                  \
        body<X, A, B>(n, o, st);                                                                                       \
    }
CEIL_KERNEL(ceil_aes128, 5, true, true)
CEIL_KERNEL(ceil_aes256, 69, true, true)
CEIL_KERNEL(ceil_b32, 5, true, false)
CEIL_KERNEL(ceil_b128, 0, false, true)

/* stamps: 2 x ngroups u64 (shader cycles, 100 MHz ticks of each workgroup's loop) */
extern "C" int lds_ceiling_run(int mode, uint32_t blocks, uint32_t ngroups, void *out, void *stamps, void *stream)
{
    void (*k)(uint32_t, uint32_t *, uint64_t *) =
        mode == 0 ? ceil_aes128 : mode == 1 ? ceil_aes256 : mode == 2 ? ceil_b32 : ceil_b128;
    hipLaunchKernelGGL(k, dim3(ngroups), dim3(1024), 0, (hipStream_t)stream, blocks, (uint32_t *)out, (uint64_t *)stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
