/*
 * scripts/lat_probe.hip -- single-wave latencies on gfx950 (measurement only), for the window kernels, which run
 * at one wave per SIMD where every dependent round trip is exposed.  One workgroup of 64 threads on one CU;
 * s_memrealtime (100 MHz) brackets N repetitions of each pattern; prints ns per repetition:
 *   lds_chase_b32    dependent ds_read_b32 (the address is the previous value)
 *   lds_chase_b128   dependent ds_read_b128
 *   lds_16_b32       16 independent ds_read_b32, then one wait (an AES round's reads)
 *   lds_32_b128      32 independent ds_read_b128, then one wait (a GHASH multiply's reads)
 *   valu_perm_dep    dependent v_perm_b32 chain
 *   valu_xor_dep     dependent v_xor_b32 chain
 *   valu_perm_ind16  16 independent v_perm_b32 (an AES round's address perms)
 *   round_tt2        one window-kernel AES round: 16 perms, 16 reads, counted waits, 8 XOR (aes_round_tt2_asm shape)
 *   gmem_chase       dependent global_load_dword (L2-resident 4 KiB)
 *   barrier          s_barrier in a 64-thread group (one wave)
 *   hipcc --offload-arch=gfx950 -O3 scripts/lat_probe.hip -o scripts/_bin/lat_probe && scripts/_bin/lat_probe
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define REPS 256
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

__global__ __launch_bounds__(64) void probe(uint32_t *gtab, uint64_t *out, uint32_t seed)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[16384];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 16384u; i += 64u)
        lds[i] = ((i * 2654435761u) & 0x3ff0u) | (t * 4u & 0xcu); /* an in-range byte address, 16-B aligned-ish */
    __syncthreads();
    uint32_t a = (seed + t * 64u) & 0x3ff0u, x = seed ^ t, y = t * 3u;
    uint64_t t0, t1;
    int k = 0;

    /* lds_chase_b32 */
    t0 = now();
    for (int r = 0; r < REPS; ++r)
        asm volatile("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)" : "+v"(a));
    t1 = now();
    out[k++] = t1 - t0;

    /* lds_chase_b128 */
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        uint32_t v0, v1, v2, v3;
        asm volatile("ds_read_b128 v[100:103], %4\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 %0, v100\n\tv_mov_b32 %1, v101\n\t"
                     "v_mov_b32 %2, v102\n\tv_mov_b32 %3, v103"
                     : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3)
                     : "v"(a)
                     : "v100", "v101", "v102", "v103");
        a = (v0 ^ v1 ^ v2 ^ v3) & 0x3ff0u;
    }
    t1 = now();
    out[k++] = t1 - t0;

    /* lds_16_b32 */
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        uint32_t v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
            asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v[i]) : "v"(a), "i"(i * 256));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            s ^= v[i];
        a = s & 0x3ff0u;
    }
    t1 = now();
    out[k++] = t1 - t0;

    /* lds_32_b128 */
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        uint32_t s = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t v[16][4];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                u32x4 q;
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(q) : "v"(a), "i"(i * 256 + h * 4096));
                v[i][0] = q[0], v[i][3] = q[3];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < 16; ++i)
                s ^= v[i][0] ^ v[i][3];
        }
        a = s & 0x3ff0u;
    }
    t1 = now();
    out[k++] = t1 - t0;

    /* valu_perm_dep */
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "s"(0x05040706u));
    }
    t1 = now();
    out[k++] = (t1 - t0) / 16;

    /* valu_xor_dep */
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(y));
    }
    t1 = now();
    out[k++] = (t1 - t0) / 16;

    /* valu_perm_ind16 */
    t0 = now();
    for (int r = 0; r < REPS; ++r) {
        uint32_t v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
            asm volatile("v_perm_b32 %0, %1, %2, %3" : "=v"(v[i]) : "v"(x), "v"(y + i), "s"(0x05040706u));
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
            s ^= v[i];
        x = s;
    }
    t1 = now();
    out[k++] = t1 - t0;

    /* round_tt2: 16 perms -> 16 reads -> counted waits -> XORs, dependent across rounds */
    {
        uint32_t s0 = x & 0x3f3f3f3fu, s1 = y & 0x3f3f3f3fu, s2 = (x ^ y) & 0x3f3f3f3fu, s3 = (x + y) & 0x3f3f3f3fu;
        const uint32_t ls = (t & 31u) * 4u;
        t0 = now();
        for (int r = 0; r < REPS; ++r) {
            uint32_t n[4], tt[12];
            asm volatile(
                "v_perm_b32 %0, %16, %20, %21\n\tv_perm_b32 %4, %17, %20, %22\n\t"
                "v_perm_b32 %5, %18, %20, %23\n\tv_perm_b32 %6, %19, %20, %24\n\t"
                "ds_read_b32 %0, %0\n\tds_read_b32 %4, %4 offset:128\n\tds_read_b32 %5, %5\n\tds_read_b32 %6, %6 offset:128\n\t"
                "v_perm_b32 %1, %17, %20, %21\n\tv_perm_b32 %7, %18, %20, %22\n\t"
                "v_perm_b32 %8, %19, %20, %23\n\tv_perm_b32 %9, %16, %20, %24\n\t"
                "ds_read_b32 %1, %1\n\tds_read_b32 %7, %7 offset:128\n\tds_read_b32 %8, %8\n\tds_read_b32 %9, %9 offset:128\n\t"
                "v_perm_b32 %2, %18, %20, %21\n\tv_perm_b32 %10, %19, %20, %22\n\t"
                "v_perm_b32 %11, %16, %20, %23\n\tv_perm_b32 %12, %17, %20, %24\n\t"
                "ds_read_b32 %2, %2\n\tds_read_b32 %10, %10 offset:128\n\tds_read_b32 %11, %11\n\tds_read_b32 %12, %12 offset:128\n\t"
                "v_perm_b32 %3, %19, %20, %21\n\tv_perm_b32 %13, %16, %20, %22\n\t"
                "v_perm_b32 %14, %17, %20, %23\n\tv_perm_b32 %15, %18, %20, %24\n\t"
                "ds_read_b32 %3, %3\n\tds_read_b32 %13, %13 offset:128\n\tds_read_b32 %14, %14\n\tds_read_b32 %15, %15 offset:128\n\t"
                "s_waitcnt lgkmcnt(12)\n\tv_xor_b32 %5, %5, %6\n\tv_bitop3_b32 %0, %0, %4, %5 bitop3:0x96\n\t"
                "s_waitcnt lgkmcnt(8)\n\tv_xor_b32 %8, %8, %9\n\tv_bitop3_b32 %1, %1, %7, %8 bitop3:0x96\n\t"
                "s_waitcnt lgkmcnt(4)\n\tv_xor_b32 %11, %11, %12\n\tv_bitop3_b32 %2, %2, %10, %11 bitop3:0x96\n\t"
                "s_waitcnt lgkmcnt(0)\n\tv_xor_b32 %14, %14, %15\n\tv_bitop3_b32 %3, %3, %13, %14 bitop3:0x96"
                : "=&v"(n[0]), "=&v"(n[1]), "=&v"(n[2]), "=&v"(n[3]), "=&v"(tt[0]), "=&v"(tt[1]), "=&v"(tt[2]),
                  "=&v"(tt[3]), "=&v"(tt[4]), "=&v"(tt[5]), "=&v"(tt[6]), "=&v"(tt[7]), "=&v"(tt[8]), "=&v"(tt[9]),
                  "=&v"(tt[10]), "=&v"(tt[11])
                : "v"(s0), "v"(s1), "v"(s2), "v"(s3), "v"(ls), "s"(0x0c0c0400u), "s"(0x0c0c0500u), "s"(0x0c0c0600u),
                  "s"(0x0c0c0700u));
            s0 = n[0] & 0x3f3f3f3fu, s1 = n[1] & 0x3f3f3f3fu, s2 = n[2] & 0x3f3f3f3fu, s3 = n[3] & 0x3f3f3f3fu;
        }
        t1 = now();
        out[k++] = t1 - t0;
        x ^= s0 ^ s1 ^ s2 ^ s3;
    }

    /* gmem_chase */
    {
        uint32_t g = (t * 4u) & 1023u;
        t0 = now();
        for (int r = 0; r < REPS; ++r)
            g = __builtin_nontemporal_load(gtab + g) & 1023u;
        t1 = now();
        out[k++] = t1 - t0;
        x ^= g;
    }

    /* barrier */
    t0 = now();
    for (int r = 0; r < REPS; ++r)
        __syncthreads();
    t1 = now();
    out[k++] = t1 - t0;

    if (t == 0)
        out[15] = a ^ x;
}

int main()
{
    uint32_t h[1024];
    for (int i = 0; i < 1024; ++i)
        h[i] = (uint32_t)(i * 37 + 11) & 1023u;
    uint32_t *gtab = nullptr;
    uint64_t *out = nullptr;
    if (hipMalloc(&gtab, sizeof(h)) != hipSuccess || hipMalloc(&out, 16 * sizeof(uint64_t)) != hipSuccess)
        return 1;
    (void)hipMemcpy(gtab, h, sizeof(h), hipMemcpyHostToDevice);
    const char *names[] = {"lds_chase_b32", "lds_chase_b128", "lds_16_b32", "lds_32_b128", "valu_perm_dep",
                           "valu_xor_dep", "valu_perm_ind16", "round_tt2", "gmem_chase", "barrier"};
    const int n = 10;
    uint64_t best[16];
    for (int i = 0; i < 16; ++i)
        best[i] = ~0ull;
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, gtab, out, (uint32_t)rep);
        uint64_t o[16];
        if (hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost) != hipSuccess)
            return 2;
        for (int i = 0; i < n; ++i)
            if (rep && o[i] < best[i])
                best[i] = o[i];
    }
    printf("{\"what\": \"scripts/lat_probe.hip: one wave on one CU, ns per repetition (s_memrealtime 100 MHz, best of 4)\",\n");
    for (int i = 0; i < n; ++i)
        printf(" \"%s\": %.1f%s\n", names[i], best[i] * 10.0 / REPS, i + 1 < n ? "," : "}");
    return 0;
}
