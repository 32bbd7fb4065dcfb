/*
 * scripts/valu_bench.hip -- VALU issue-rate microbenchmark (measurement only): wave64 instructions per
 * clock per SIMD for the opcodes the AES engines are made of, 16 waves per CU, 8 independent chains
 * per lane (no dependency stalls), 64 instructions per chain per iteration.
 */
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CHAINS 8
template <int OP>
__device__ __forceinline__ uint32_t op(uint32_t a, uint32_t b, uint32_t c)
{
    if (OP == 0)
        return a ^ b;  /* v_xor_b32 (VOP2) */
    if (OP == 1)
        return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); /* v_bitop3_b32 (VOP3, 3 VGPR sources) */
    if (OP == 2)
        return __builtin_amdgcn_perm(a, b, c);             /* v_perm_b32 (VOP3, 3 VGPR sources) */
    if (OP == 3)
        return __builtin_amdgcn_alignbit(a, b, 7u);        /* v_alignbit_b32 */
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x39, 0xf, 0xf, false) ^ b; /* v_xor_b32_dpp */
}

template <int OP>
__device__ void body(uint32_t iters, uint32_t *out)
{
    uint32_t x[CHAINS], y = threadIdx.x * 0x9e3779b9u, z = blockIdx.x * 0x7f4a7c15u + 0x01020304u;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
        x[c] = threadIdx.x * (c + 1) + 12345u * c;
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 64; ++k)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c)
                x[c] = op<OP>(x[c], y + (uint32_t)k, z ^ (uint32_t)c);
        asm volatile("" : "+v"(y)); /* the loop-invariant operands stay opaque (no folding) */
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c)
        r ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

extern "C" __global__ __launch_bounds__(1024) void valu_xor(uint32_t n, uint32_t *o) { body<0>(n, o); }
extern "C" __global__ __launch_bounds__(1024) void valu_bitop3(uint32_t n, uint32_t *o) { body<1>(n, o); }
extern "C" __global__ __launch_bounds__(1024) void valu_perm(uint32_t n, uint32_t *o) { body<2>(n, o); }
extern "C" __global__ __launch_bounds__(1024) void valu_alignbit(uint32_t n, uint32_t *o) { body<3>(n, o); }
extern "C" __global__ __launch_bounds__(1024) void valu_xor_dpp(uint32_t n, uint32_t *o) { body<4>(n, o); }

extern "C" int valu_bench_run(int op, uint32_t iters, uint32_t nblocks, uint32_t threads, void *out, void *stream)
{
    void (*k)(uint32_t, uint32_t *) =
        op == 0 ? valu_xor : op == 1 ? valu_bitop3 : op == 2 ? valu_perm : op == 3 ? valu_alignbit : valu_xor_dpp;
    hipLaunchKernelGGL(k, dim3(nblocks), dim3(threads), 0, (hipStream_t)stream, iters, (uint32_t *)out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
