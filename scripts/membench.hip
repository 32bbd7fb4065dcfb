// scripts/membench.hip -- access-pattern micro-benchmark for the record walk (profiling tool).
//
// Streams n records of `len` bytes (256-B aligned slots) through a load -> xor -> store loop
// with the batch kernels' lane mapping: K lanes per record, 64/K records per wave step,
// lane j touching 16-byte blocks j, j+K, ...  Variants: K, prefetch depth D (blocks in
// flight per lane besides the one being consumed), waves per workgroup.  Prints GB/s of
// HBM traffic (read + write).
//
//   hipcc --offload-arch=gfx950 -O3 -o membench scripts/membench.hip && ./membench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int K, int D>
__global__ __launch_bounds__(1024) void walk(const uint8_t *src, uint8_t *dst, uint32_t nrec, uint32_t len, uint32_t slot)
{
    constexpr uint32_t R = 64 / K;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    const uint32_t j = lane % K, s = lane / K;
    const uint32_t nblk = (len + 15) / 16, T = (nblk + K - 1) / K;
    const uint64_t ngroups = (nrec + R - 1) / R;
    for (uint64_t g = (uint64_t)blockIdx.x * wpb + wave; g < ngroups; g += (uint64_t)gridDim.x * wpb) {
        const uint64_t r = g * R + s;
        const uint8_t *in = src + r * slot;
        uint8_t *out = dst + r * slot;
        u32x4 buf[D + 1];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            uint32_t b = j + K * d;
            buf[d] = *(const u32x4 *)(in + 16u * (b < nblk ? b : 0));
        }
        for (uint32_t t = 0; t < T; t += D + 1) {
#pragma unroll
            for (int d = 0; d <= D; ++d) {
                uint32_t tt = t + d;
                // issue the load D steps ahead into the slot consumed D+1 steps ago
                uint32_t bn = j + K * (tt + D);
                buf[(d + D) % (D + 1)] = *(const u32x4 *)(in + 16u * (bn < nblk ? bn : 0));
                uint32_t b = j + K * tt;
                if (tt < T && b < nblk)
                    *(u32x4 *)(out + 16u * b) = buf[d] ^ (u32x4){0x5a5a5a5au, tt, b, 7u};
            }
        }
    }
}

template <int K, int D>
static void run(const char *name, uint8_t *src, uint8_t *dst, uint32_t nrec, uint32_t len, uint32_t slot, int threads)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int blocks = 256;
    for (int w = 0; w < 2; ++w)
        hipLaunchKernelGGL((walk<K, D>), dim3(blocks), dim3(threads), 0, 0, src, dst, nrec, len, slot);
    hipEventRecord(a);
    const int reps = 5;
    for (int w = 0; w < reps; ++w)
        hipLaunchKernelGGL((walk<K, D>), dim3(blocks), dim3(threads), 0, 0, src, dst, nrec, len, slot);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    double bytes = 2.0 * (double)nrec * len;
    printf("%-10s len=%5u K=%2d D=%d threads=%4d  %8.3f ms  %7.1f GB/s  payload %7.1f GiB/s\n", name, len, K, D, threads, ms,
           bytes / ms / 1e6, (double)nrec * len / (ms * 1e-3) / (1 << 30));
}

int main()
{
    struct Cfg { uint32_t nrec, len; } cfgs[] = {{1u << 20, 1400}, {1u << 18, 16384}};
    for (auto c : cfgs) {
        uint32_t slot = ((c.len + 16 + 255) / 256) * 256;
        size_t bytes = (size_t)c.nrec * slot;
        uint8_t *src, *dst;
        hipMalloc(&src, bytes);
        hipMalloc(&dst, bytes);
        hipMemset(src, 1, bytes);
        run<4, 1>("k4d1", src, dst, c.nrec, c.len, slot, 1024);
        run<4, 2>("k4d2", src, dst, c.nrec, c.len, slot, 1024);
        run<4, 3>("k4d3", src, dst, c.nrec, c.len, slot, 1024);
        run<2, 1>("k2d1", src, dst, c.nrec, c.len, slot, 1024);
        run<2, 3>("k2d3", src, dst, c.nrec, c.len, slot, 1024);
        run<8, 1>("k8d1", src, dst, c.nrec, c.len, slot, 1024);
        run<8, 3>("k8d3", src, dst, c.nrec, c.len, slot, 1024);
        run<16, 1>("k16d1", src, dst, c.nrec, c.len, slot, 1024);
        run<16, 3>("k16d3", src, dst, c.nrec, c.len, slot, 1024);
        run<64, 1>("k64d1", src, dst, c.nrec, c.len, slot, 1024);
        run<64, 3>("k64d3", src, dst, c.nrec, c.len, slot, 1024);
        run<4, 1>("k4d1w8", src, dst, c.nrec, c.len, slot, 512);
        run<4, 3>("k4d3w8", src, dst, c.nrec, c.len, slot, 512);
        hipFree(src);
        hipFree(dst);
    }
    return 0;
}
