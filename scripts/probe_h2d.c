/* Host time of hipMemcpyAsync host -> device calls from hipHostRegister'ed memory, by size and stream: which first
 * copies stall (coalesced dma_in windows).  Measurement only.
 *   hipcc -O2 -o scripts/_build/probe_h2d scripts/probe_h2d.c && scripts/_build/probe_h2d */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

__global__ void touch(unsigned *p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1; }

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

#define CHK(x)                                                                                                             \
    do {                                                                                                                   \
        hipError_t e_ = (x);                                                                                               \
        if (e_ != hipSuccess) {                                                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                                       \
            return 1;                                                                                                      \
        }                                                                                                                  \
    } while (0)

int main(void)
{
    const size_t max = 64u << 20;
    void *host = NULL, *dev = NULL;
    if (posix_memalign(&host, 4096, max) != 0)
        return 1;
    for (size_t i = 0; i < max; i += 4096)
        ((char *)host)[i] = (char)i;
    CHK(hipMalloc(&dev, max));
    CHK(hipHostRegister(host, max, hipHostRegisterMapped));
    hipStream_t st[4];
    for (int i = 0; i < 4; ++i)
        CHK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    for (int round = 0; round < 2; ++round)
        for (int s = 0; s < 4; ++s)
            for (size_t n = 4096; n <= max; n *= 4) {
                const double t0 = now();
                CHK(hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, st[s]));
                const double t1 = now();
                CHK(hipStreamSynchronize(st[s]));
                const double t2 = now();
                if (t1 - t0 > 1e-3 || round == 0)
                    printf("round %d stream %d %9zu B: call %8.3f ms, sync %8.3f ms\n", round, s, n, (t1 - t0) * 1e3,
                           (t2 - t1) * 1e3);
            }
    /* unsynchronised: several copies in flight on one stream, then on all four */
    for (int s = 0; s < 4; ++s) {
        const double t0 = now();
        for (int k = 0; k < 8; ++k)
            CHK(hipMemcpyAsync((char *)dev + k * (1 << 20), (char *)host + k * (1 << 20), 1 << 20, hipMemcpyHostToDevice,
                               st[s]));
        printf("stream %d: 8 x 1 MiB queued in %.3f ms\n", s, (now() - t0) * 1e3);
    }
    for (int s = 0; s < 4; ++s)
        CHK(hipStreamSynchronize(st[s]));
    /* more registered ranges: the first large copy from each */
    for (int r = 0; r < 3; ++r) {
        void *h2 = NULL;
        if (posix_memalign(&h2, 4096, 16u << 20) != 0)
            return 1;
        for (size_t i = 0; i < (16u << 20); i += 4096)
            ((char *)h2)[i] = (char)i;
        CHK(hipHostRegister(h2, 16u << 20, hipHostRegisterMapped));
        for (size_t n = 4096; n <= (16u << 20); n *= 4) {
            const double t0 = now();
            CHK(hipMemcpyAsync(dev, h2, n, hipMemcpyHostToDevice, st[r]));
            const double t1 = now();
            CHK(hipStreamSynchronize(st[r]));
            if (t1 - t0 > 1e-3)
                printf("range %d %9zu B: call %8.3f ms\n", r, n, (t1 - t0) * 1e3);
        }
        /* device -> host into it */
        for (size_t n = 4096; n <= (16u << 20); n *= 4) {
            const double t0 = now();
            CHK(hipMemcpyAsync(h2, dev, n, hipMemcpyDeviceToHost, st[r]));
            const double t1 = now();
            CHK(hipStreamSynchronize(st[r]));
            if (t1 - t0 > 1e-3)
                printf("range %d d2h %9zu B: call %8.3f ms\n", r, n, (t1 - t0) * 1e3);
        }
    }
    /* a range written by D2H first, then read by H2D (a sealed wire buffer, opened next) */
    for (int r = 0; r < 2; ++r) {
        void *h3 = NULL;
        if (posix_memalign(&h3, 4096, 16u << 20) != 0)
            return 1;
        for (size_t i = 0; i < (16u << 20); i += 4096)
            ((char *)h3)[i] = (char)i;
        CHK(hipHostRegister(h3, 16u << 20, hipHostRegisterMapped));
        for (int dir = 0; dir < 2; ++dir)
            for (size_t n = 4096; n <= (16u << 20); n *= 4) {
                const double t0 = now();
                CHK(dir == 0 ? hipMemcpyAsync(h3, dev, n, hipMemcpyDeviceToHost, st[r])
                             : hipMemcpyAsync(dev, h3, n, hipMemcpyHostToDevice, st[r]));
                const double t1 = now();
                CHK(hipStreamSynchronize(st[r]));
                if (t1 - t0 > 1e-3)
                    printf("d2h-first range %d %s %9zu B: call %8.3f ms\n", r, dir ? "h2d" : "d2h", n, (t1 - t0) * 1e3);
            }
        /* and with a kernel in flight on another stream */
        hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, st[3], (unsigned *)dev);
        const double t0 = now();
        CHK(hipMemcpyAsync(dev, (char *)h3 + (8u << 20), 1u << 20, hipMemcpyHostToDevice, st[r]));
        if (now() - t0 > 1e-3)
            printf("range %d h2d beside a kernel: %.3f ms\n", r, (now() - t0) * 1e3);
        CHK(hipDeviceSynchronize());
    }
    /* copies and kernels interleaved on the four streams, more in flight each time */
    for (int d = 1; d <= 64; d *= 2) {
        const double t0 = now();
        for (int k = 0; k < d; ++k)
            for (int s = 0; s < 4; ++s) {
                const double c0 = now();
                CHK(hipMemcpyAsync((char *)dev + (s << 22), (char *)host + (k << 18), 1 << 18, hipMemcpyHostToDevice, st[s]));
                const double c1 = now();
                hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, st[s], (unsigned *)dev + s * 1024);
                const double c2 = now();
                if (c1 - c0 > 1e-3 || c2 - c1 > 1e-3)
                    printf("depth %d k %d stream %d: copy call %.3f ms, launch %.3f ms\n", d, k, s, (c1 - c0) * 1e3,
                           (c2 - c1) * 1e3);
            }
        for (int s = 0; s < 4; ++s)
            CHK(hipStreamSynchronize(st[s]));
        printf("depth %d: %.3f ms\n", d, (now() - t0) * 1e3);
    }
    printf("done\n");
    return 0;
}
