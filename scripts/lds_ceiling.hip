/*
 * scripts/lds_ceiling.hip -- the LDS ceiling of the batch kernels' exact read mix (measurement only, not the product).
 *
 * One 16-B block of the GH8 batch kernels (gcm_core.h aes_gh8_fused_h) costs, per lane:
 *   AES-128: 133 ds_read_b32 (bank-replicated T-table lookups: lane l reads bank l & 31 of a random 256-B row of the
 *            two-table image at LDS 64K, address = one v_perm of a state byte, as the kernels form it)
 *   AES-256: 197 ds_read_b32
 *   GHASH:   16 ds_read_b128 from the 8-bit latin table at LDS 0 (row e = a random byte, 256 B; read r of lane i takes
 *            slot r ^ (i & 15): 16 distinct bank groups per pass, conflict-free)
 * This probe issues exactly that mix per block -- rounds of 16 b32 (+ 2 b128 in the first 8), software-pipelined --
 * with 16 waves per CU, addresses from a hash chain independent of the loaded values (nothing waits on a load but its
 * XOR), and no HBM traffic.  Blocks per second per CU at the measured clock give the LDS cycles one block really
 * costs: the measured ceiling the bench line's lds_roofline is priced against (the nominal 2 / 4 clk per b32 / b128
 * read model gives 330 / 458 clk per 64 blocks).
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

/*
 * N32 ds_read_b32 and N128 ds_read_b128 per block, issued in rounds of up to 16 b32 (+ 2 b128 in the first N128 / 2
 * rounds) as the kernels issue a middle AES round (aes_round_tt2k_asm) with its GH8 reads; software-pipelined two
 * rounds deep (the reads of round R are issued before round R - 1's are consumed), so a wave keeps ~36 reads in flight
 * and the probe measures the LDS, not its latency.
 */
template <int N32, int N128>
__device__ void body(uint32_t blocks, uint32_t *out, uint64_t *stamps)
{
    constexpr int NR = (N32 + 15) / 16 > N128 / 2 ? (N32 + 15) / 16 : N128 / 2;
    __shared__ __attribute__((aligned(16))) uint8_t lds[0x20000];
    for (uint32_t i = threadIdx.x; i < (0x20000u / 16u); i += blockDim.x)
        *(u32x4 *)(lds + 16u * i) = u32x4{i, i * 3u, i * 5u, i * 7u};
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, gi = lane & 15u;
    uint32_t s0 = 0x9e3779b9u * (threadIdx.x + 1u) ^ blockIdx.x, s1 = s0 * 3u + 1u, s2 = s0 * 5u + 7u, s3 = s0 * 7u + 3u;
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u; /* bank + the two-table image at 64K */
    uint32_t acc = 0;
    u32x4 acc4 = {0u, 0u, 0u, 0u};
    uint32_t v[2][16];
    u32x4 g[2][2];
    /* the in-kernel clock (MI355X_MICROARCH.md, DVFS item 6): shader cycles and 100 MHz ticks around the loop */
    __syncthreads();
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t b = 0; b < blocks; ++b) {
#pragma unroll
        for (int R = 0; R <= NR; ++R) {
            if (R < NR) { /* issue round R */
                const int n32 = N32 - 16 * R < 16 ? N32 - 16 * R : 16, n128 = 2 * R < N128 ? 2 : 0;
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    if (k < n32) {
                        const uint32_t w = (k & 3) == 0 ? s0 : (k & 3) == 1 ? s1 : (k & 3) == 2 ? s2 : s3;
                        const uint32_t sel = 0x0c020400u | ((4u + (uint32_t)(k >> 2)) << 8); /* 64K | row << 8 | bank */
                        v[R & 1][k] = *(const uint32_t *)(lds + (__builtin_amdgcn_perm(w, lanesel, sel) | ((k & 1) ? 0x80u : 0u)));
                    }
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    if (q < n128) {
                        const uint32_t r = (2u * (uint32_t)R + (uint32_t)q) & 15u, p = r ^ gi; /* latin read order */
                        const uint32_t e = ((q ? s2 : s1) >> (8u * (r & 3u))) & 0xffu;
                        g[R & 1][q] = *(const u32x4 *)(lds + (e << 8) + (p << 4));
                    }
                }
                s0 = __builtin_amdgcn_alignbit(s0, s0, 7u) + 0x9e3779b9u;
                s1 = __builtin_amdgcn_alignbit(s1, s1, 11u) + 0x7f4a7c15u;
                s2 = __builtin_amdgcn_alignbit(s2, s2, 13u) + 0x94d049bbu;
                s3 = __builtin_amdgcn_alignbit(s3, s3, 17u) + 0x2545f491u;
            }
            if (R > 0) { /* consume round R - 1 */
                const int P = R - 1;
                const int n32 = N32 - 16 * P < 16 ? N32 - 16 * P : 16, n128 = 2 * P < N128 ? 2 : 0;
#pragma unroll
                for (int k = 0; k < 16; k += 2) {
                    if (k + 1 < n32)
                        acc = __builtin_amdgcn_bitop3_b32(acc, v[P & 1][k], v[P & 1][k + 1], 0x96);
                    else if (k < n32)
                        acc ^= v[P & 1][k];
                }
#pragma unroll
                for (int q = 0; q < 2; ++q)
                    if (q < n128)
                        acc4 ^= g[P & 1][q];
            }
            __builtin_amdgcn_sched_barrier(0); /* the pipeline as written (no hoisting of every read: spills) */
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc ^ acc4[0] ^ acc4[1] ^ acc4[2] ^ acc4[3];
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

#define CEIL_KERNEL(NAME, N32, N128)                                                                                   \
    extern "C" __global__ __launch_bounds__(1024) void NAME(uint32_t n, uint32_t *o, uint64_t *st)                      \
    {                                                                                                                  \
        body<N32, N128>(n, o, st);                                                                                     \
    }
CEIL_KERNEL(ceil_aes128, 133, 16)
CEIL_KERNEL(ceil_aes256, 197, 16)
CEIL_KERNEL(ceil_b32, 133, 0)
CEIL_KERNEL(ceil_b128, 0, 16)

/* stamps: 2 x ngroups u64 (shader cycles, 100 MHz ticks of each workgroup's loop) */
extern "C" int lds_ceiling_run(int mode, uint32_t blocks, uint32_t ngroups, void *out, void *stamps, void *stream)
{
    void (*k)(uint32_t, uint32_t *, uint64_t *) =
        mode == 0 ? ceil_aes128 : mode == 1 ? ceil_aes256 : mode == 2 ? ceil_b32 : ceil_b128;
    hipLaunchKernelGGL(k, dim3(ngroups), dim3(1024), 0, (hipStream_t)stream, blocks, (uint32_t *)out, (uint64_t *)stamps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
