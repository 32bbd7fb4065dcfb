// scripts/energy_probe.hip -- energy per HBM byte of the record walk's access pattern (measurement only).
//
// The batch kernels run at the package power limit, so the energy each byte costs sets the clock
// they hold.  This probe streams 256 K records of 16 KiB (256-B aligned slots, 16 640 B apart) through load -> xor ->
// store with the batch walk's lane mapping -- K lanes per record, 64 / K records per wave step, lane j on 16-B blocks
// j, j + K, ..., three steps of loads in flight -- so one wave instruction touches 64 / K pieces of 16 K bytes each:
// K = 4 is the shipped walk (16 pieces of 64 B, half lines), K = 8 whole 128-B lines, K = 64 one 1-KiB piece.
// `filler` dependent v_bitop3 per lane and step stand in for the AES + GHASH work and bring the stream down to the
// kernels' rate.  Runs each launch back to back for `seconds`; scripts/gpu_energy_probe.sh samples amd-smi meanwhile.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/_bin/energy_probe scripts/energy_probe.hip
//   scripts/_bin/energy_probe K filler seconds        -> one JSON line
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <chrono>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHK(x)                                                                                                         \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                                    \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

template <int K>
__global__ __launch_bounds__(1024) void walk(const uint8_t *src, uint8_t *dst, uint32_t nrec, uint32_t len, uint32_t slot,
                                             uint32_t filler, uint32_t *work)
{
    constexpr uint32_t R = 64 / K;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t j = lane % K, s = lane / K;
    const uint32_t nblk = len / 16u, T = (nblk + K - 1) / K;
    const uint32_t ngroups = (nrec + R - 1) / R;
    uint32_t x = lane, y = lane * 7u + 1u, z = lane * 13u + 5u;
    for (;;) {
        uint32_t g = 0;
        if (lane == 0)
            g = atomicAdd(work, 1u);
        g = (uint32_t)__shfl((int)g, 0, 64);
        if (g >= ngroups)
            break;
        const uint64_t r = (uint64_t)g * R + s;
        const uint8_t *in = src + r * slot;
        uint8_t *out = dst + r * slot;
        auto ld = [&](uint32_t t) {
            const uint32_t b = j + K * t;
            return *(const u32x4 *)(in + 16u * (b < nblk ? b : 0u)); /* plain loads, as the batch kernels */
        };
        u32x4 b0 = ld(0), b1 = ld(1), b2 = ld(2);
        for (uint32_t t = 0; t < T; ++t) {
            const u32x4 b3 = ld(t + 3u);
            for (uint32_t i = 0; i < filler; ++i) /* the AES + GHASH stand-in: a dependent chain */
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "v"(z));
            const uint32_t b = j + K * t;
            if (b < nblk)
                __builtin_nontemporal_store(b0 ^ u32x4{x, t, b, 7u}, (u32x4 *)(out + 16u * b));
            b0 = b1;
            b1 = b2;
            b2 = b3;
        }
    }
    if (x == 0xdeadbeefu) /* keep the chain */
        dst[0] = 1;
}

template <int K>
static void run(uint32_t filler, double seconds)
{
    const uint32_t nrec = 1u << 18, len = 16384, slot = 16640;
    const size_t bytes = (size_t)nrec * slot;
    uint8_t *src, *dst;
    uint32_t *work;
    CHK(hipMalloc(&src, bytes));
    CHK(hipMalloc(&dst, bytes));
    CHK(hipMalloc(&work, 4096 * sizeof(uint32_t)));
    CHK(hipMemset(src, 1, bytes));
    CHK(hipMemset(work, 0, 4096 * sizeof(uint32_t)));
    int ncu = 0;
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    uint32_t launches = 0;
    double ms_sum = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL((walk<K>), dim3(ncu), dim3(1024), 0, 0, src, dst, nrec, len, slot, filler, work + (launches % 4096));
        CHK(hipGetLastError());
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (++launches > 3)
            ms_sum += ms;
        if (launches % 4096 == 0)
            CHK(hipMemset(work, 0, 4096 * sizeof(uint32_t)));
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds)
            break;
    }
    const double ms = ms_sum / (launches - 3);
    printf("{\"K\": %d, \"filler\": %u, \"launches\": %u, \"ms_per_launch\": %.4f, \"traffic_gbps\": %.1f, "
           "\"payload_gibps\": %.1f}\n",
           K, filler, launches, ms, 2.0 * nrec * len / (ms * 1e-3) / 1e9, (double)nrec * len / (ms * 1e-3) / (1u << 30));
    fflush(stdout);
    CHK(hipFree(src));
    CHK(hipFree(dst));
    CHK(hipFree(work));
}

int main(int argc, char **argv)
{
    if (argc < 4) {
        fprintf(stderr, "usage: energy_probe K filler seconds\n");
        return 2;
    }
    const int K = atoi(argv[1]);
    const uint32_t filler = (uint32_t)atoi(argv[2]);
    const double seconds = atof(argv[3]);
    switch (K) {
    case 4: run<4>(filler, seconds); break;
    case 8: run<8>(filler, seconds); break;
    case 16: run<16>(filler, seconds); break;
    case 64: run<64>(filler, seconds); break;
    default: fprintf(stderr, "K in 4, 8, 16, 64\n"); return 2;
    }
    return 0;
}
