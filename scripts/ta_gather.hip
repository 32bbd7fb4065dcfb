/*
 * scripts/ta_gather.hip -- can the vector-memory path (TA/TD + L1) serve T-table lookups beside the LDS?
 * (measurement only).  16 waves per CU on every CU; each lane runs 8 independent lookup chains
 * x = T[byte(x)] ^ c, the address of every lookup taken from the previous result of its chain (as in an AES
 * round).  Variants:
 *   lds     ds_read_b32 from a bank-replicated 1 KiB table (row x = T[x] x 32 banks), the engine's pattern
 *   buf1k   buffer_load_dword from a 1 KiB table in global memory (L1-resident)
 *   buf4k   the same from four 1 KiB tables (4 KiB)
 *   mix3    3 LDS chains : 1 buffer chain per 4 chains (the two paths side by side)
 *   mix1    7 LDS chains : 1 buffer chain
 * Prints ms and lookups per clock per CU (at 2.4 GHz, relative only).
 *   hipcc --offload-arch=gfx950 -O3 scripts/ta_gather.hip -o scripts/_bin/ta_gather && scripts/_bin/ta_gather
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

template <int MODE>
__global__ __launch_bounds__(1024) void gather(uint32_t iters, const uint32_t *__restrict__ gtab, uint32_t *out)
{
    __shared__ uint32_t lds[256 * 32];
    for (uint32_t i = threadIdx.x; i < 256u * 32u; i += blockDim.x)
        lds[i] = gtab[(i >> 5) & 255u] ;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)gtab, (short)0, 4096, 0x00020000);
    const uint32_t lane = threadIdx.x & 31u;
    uint32_t x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
        x[c] = (threadIdx.x * 0x9e3779b9u) ^ (0x01020304u * (c + 1));
    for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const bool use_buf = MODE == 1 || MODE == 2 || (MODE == 3 && (c & 3) == 3) || (MODE == 4 && c == 7);
                const uint32_t b = (x[c] >> (8 * (k & 3))) & 0xffu;
                if (use_buf) {
                    const uint32_t off = (MODE == 2 ? ((uint32_t)(c & 3) << 10) : 0u) + b * 4u;
                    x[c] ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0) + (uint32_t)k;
                } else {
                    x[c] ^= lds[b * 32u + lane] + (uint32_t)k;
                }
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c)
        r ^= x[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main()
{
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t h[1024];
    for (int i = 0; i < 1024; ++i)
        h[i] = (uint32_t)i * 2654435761u;
    uint32_t *gtab = nullptr, *out = nullptr;
    if (hipMalloc(&gtab, 4096) != hipSuccess || hipMalloc(&out, (size_t)ncu * 1024 * 4) != hipSuccess)
        return 1;
    (void)hipMemcpy(gtab, h, 4096, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *names[] = {"lds", "buf1k", "buf4k", "mix3lds1buf", "mix7lds1buf"};
    void (*ks[])(uint32_t, const uint32_t *, uint32_t *) = {gather<0>, gather<1>, gather<2>, gather<3>, gather<4>};
    const uint32_t iters = 256;
    printf("{\"what\": \"scripts/ta_gather.hip: 8 chains x 16 lookups per trip per lane, 16 waves/CU\", \"rows\": [\n");
    for (int v = 0; v < 5; ++v) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(ks[v], dim3(ncu), dim3(1024), 0, 0, iters, gtab, out);
            (void)hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess)
                return 2;
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best)
                best = ms;
        }
        const double lookups_per_cu = 1024.0 * 8.0 * 16.0 * iters; /* 1024 threads x 8 chains x 16 x iters */
        const double per_clk = lookups_per_cu / (best * 1e-3 * 2.4e9);
        printf("  {\"mode\": \"%s\", \"ms\": %.3f, \"lookups_per_clk_per_cu\": %.2f, \"wave_instr_clk\": %.2f}%s\n", names[v],
               best, per_clk, 64.0 / per_clk, v < 4 ? "," : "");
        fflush(stdout);
    }
    printf("]}\n");
    return 0;
}
