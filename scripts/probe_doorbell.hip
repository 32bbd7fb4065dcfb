/*
 * scripts/probe_doorbell.hip -- measurement only: what a resident, doorbell-driven kernel saves over a launch per window.
 *
 * A persistent grid: one dispatcher lane polls a job ring in pinned, mapped, coherent host memory and copies new
 * jobs into device memory; P 128-thread worker workgroups poll that copy (L2, not PCIe).  The host writes a job (units
 * of work, source and destination) and bumps `tail`; a worker claims a unit with a CAS on the job's claim word
 * (epoch << 32 | count: never over-claimed, so no reset race), does it, fences at system scope, and counts it done; the
 * last unit's worker resets the job's words and writes fin[job] into host memory, which the host polls.  The
 * dispatcher leaves after IDLE_MS with every job finished, on `stop`, or after MAX_S, and the workers follow it: every
 * wave reaches the exit whatever the host does.
 *
 * Prints one JSON line per measurement (host-timed, clock_gettime):
 *   launch_sync        an empty kernel launch + hipStreamSynchronize (the floor of a launch-per-call design)
 *   doorbell_empty     post one empty job, poll its fin
 *   copy_launch        a 256 KiB window copied host -> host by a kernel launch (64 x 4 KiB units), + sync
 *   copy_doorbell_dD   the same window as a doorbell job, D jobs outstanding: latency and GB/s
 *
 *   hipcc --offload-arch=gfx950 -O3 scripts/probe_doorbell.hip -o scripts/_bin/probe_doorbell && scripts/_bin/probe_doorbell
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <algorithm>
#include <vector>

#define RING 64
#define IDLE_MS 50
#define MAX_S 30
#define UNIT_THREADS 128

struct Job {
    uint64_t id;
    uint32_t nunits, unit_bytes;
    uint32_t base, pad; /* static mode: unit u goes to worker (base + u) % P */
    const uint8_t *src;
    uint8_t *dst;
};

struct Ring {
    uint64_t tail;
    uint32_t stop;
    uint32_t pad0[13];
    Job jobs[RING];
    uint64_t fin[RING];
};

#define CHK(x)                                                                                                         \
    do {                                                                                                               \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess) {                                                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                                                    \
            exit(1);                                                                                                   \
        }                                                                                                              \
    } while (0)

/* relaxed polls only: an acquire per poll invalidates caches every time (MI355X_MICROARCH.md, inter-workgroup
 * visibility: "polling with ACQUIRE loads ... 255 pollers cut chip bandwidth 37-71 %") */
__device__ __forceinline__ uint64_t ld_sys64(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_dev64(const unsigned long long *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_dev32(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
/* a 16-byte store at system scope (sc0 sc1: written through, not kept in L2) */
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_sys16(uint4 *p, uint4 v)
{
    const u32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(x) : "memory");
}
template <typename T> __device__ __forceinline__ void st_dev(T *p, T v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sys32(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

/*
 * Device-side state of the resident grid: the dispatcher's copy of the ring (workers never touch host memory to find
 * work: polling PCIe from every workgroup saturates the link with small reads), the claim and done words.
 */
struct DevJob {
    unsigned long long src, dst;
    uint32_t nunits, unit_bytes, base, pad;
};
struct DevState {
    unsigned long long tail; /* jobs published to the workers */
    uint32_t stop;           /* set by the dispatcher when it leaves (idle, host stop, lifetime): the workers follow */
    uint32_t pad[13];
    DevJob jobs[RING];
    unsigned long long claim[RING];
    uint32_t done[RING];
};

/* mode bit 0: units claimed by CAS (else statically: worker (base + u) % P); bit 1: a system release per unit */
__global__ __launch_bounds__(UNIT_THREADS) void resident(Ring *ring, DevState *ds, uint64_t first, uint64_t idle_ticks,
                                                         uint64_t max_ticks, uint32_t mode)
{
    __shared__ uint64_t s_job, s_src, s_dst;
    __shared__ uint32_t s_unit, s_state, s_ub; /* state: 0 work, 1 idle, 2 exit */
    const uint64_t born = wall_clock64();
    if (blockIdx.x == 0) {
        /* the dispatcher: one lane polls the host ring and publishes new jobs in device memory */
        if (threadIdx.x != 0)
            return;
        uint64_t pub = __hip_atomic_load(&ds->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t idle_since = born;
        for (;;) {
            const uint64_t now = wall_clock64();
            if (ld_sys32(&ring->stop) != 0u || now - born > max_ticks)
                break;
            const uint64_t tail = ld_sys64(&ring->tail);
            if (tail > pub) {
                /* job fields: sc0 sc1 loads (uncached, issued after the tail load returned); published with sc1 stores,
                 * drained, then an sc1 tail store (the guide's sc1 hand-off: workers read them with sc1 loads) */
                for (; pub < tail; ++pub) {
                    const uint32_t slot = (uint32_t)(pub % RING);
                    st_dev(&ds->jobs[slot].nunits, ld_sys32(&ring->jobs[slot].nunits));
                    st_dev(&ds->jobs[slot].unit_bytes, ld_sys32(&ring->jobs[slot].unit_bytes));
                    st_dev(&ds->jobs[slot].base, ld_sys32(&ring->jobs[slot].base));
                    st_dev(&ds->jobs[slot].src, (unsigned long long)ld_sys64((const uint64_t *)&ring->jobs[slot].src));
                    st_dev(&ds->jobs[slot].dst, (unsigned long long)ld_sys64((const uint64_t *)&ring->jobs[slot].dst));
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_dev(&ds->tail, (unsigned long long)pub);
                idle_since = now;
            } else {
                /* idle only once every published job is finished */
                bool busy = false;
                if (pub > 0) {
                    const uint32_t slot = (uint32_t)((pub - 1) % RING);
                    busy = ld_sys64(&ring->fin[slot]) != pub;
                }
                if (busy)
                    idle_since = now;
                else if (now - idle_since > idle_ticks)
                    break;
                __builtin_amdgcn_s_sleep(32);
            }
        }
        __hip_atomic_store(&ds->stop, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const uint32_t P = gridDim.x - 1u, w = blockIdx.x - 1u;
    uint64_t cur = first;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t state = 1;
            if (ld_dev32(&ds->stop) != 0u || wall_clock64() - born > max_ticks + idle_ticks)
                state = 2;
            else {
                const uint64_t tail = ld_dev64(&ds->tail);
                while (cur < tail) {
                    const uint32_t slot = (uint32_t)(cur % RING);
                    const uint32_t n = ld_dev32(&ds->jobs[slot].nunits);
                    if (!(mode & 1u)) {
                        /* static: this worker's first unit of the job, if any (the next ones are P apart) */
                        const uint32_t u0 = (w + P - ld_dev32(&ds->jobs[slot].base) % P) % P;
                        if (u0 >= n) {
                            ++cur;
                            continue;
                        }
                        s_src = ld_dev64(&ds->jobs[slot].src);
                        s_dst = ld_dev64(&ds->jobs[slot].dst);
                        s_ub = ld_dev32(&ds->jobs[slot].unit_bytes);
                        s_job = cur;
                        s_unit = u0;
                        state = 0;
                        ++cur;
                        break;
                    }
                    const unsigned long long epoch = cur / RING;
                    unsigned long long c = ld_dev64(&ds->claim[slot]);
                    if ((c >> 32) > epoch || (uint32_t)c >= n) {
                        ++cur; /* done, or every unit claimed */
                        continue;
                    }
                    if ((c >> 32) < epoch)
                        break; /* the slot's previous job is still being reset (host posts at most RING ahead) */
                    if (atomicCAS(&ds->claim[slot], c, c + 1ull) == c) {
                        s_src = ld_dev64(&ds->jobs[slot].src);
                        s_dst = ld_dev64(&ds->jobs[slot].dst);
                        s_ub = ld_dev32(&ds->jobs[slot].unit_bytes);
                        s_job = cur;
                        s_unit = (uint32_t)c;
                        state = 0;
                        break;
                    }
                }
            }
            s_state = state;
        }
        __syncthreads();
        const uint32_t state = s_state;
        if (state == 2)
            return;
        if (state == 1) {
            __syncthreads(); /* everyone has read s_state before thread 0 rewrites it */
            __builtin_amdgcn_s_sleep(4);
            continue;
        }
        const uint64_t j = s_job;
        const uint32_t slot = (uint32_t)(j % RING);
        const uint32_t ub = s_ub, n = ld_dev32(&ds->jobs[slot].nunits);
        uint32_t mine = 0;
        for (uint32_t u = s_unit; u < n; u += (mode & 1u) ? n : P) {
            const uint4 *src = (const uint4 *)((const uint8_t *)s_src + (size_t)u * ub);
            uint4 *dst = (uint4 *)((uint8_t *)s_dst + (size_t)u * ub);
            if (mode & 4u) {
                for (uint32_t i = threadIdx.x; i < ub / 16u; i += UNIT_THREADS)
                    st_sys16(dst + i, src[i]);
            } else {
                for (uint32_t i = threadIdx.x; i < ub / 16u; i += UNIT_THREADS)
                    dst[i] = src[i];
            }
            ++mine;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            if (mode & 2u) {
                /* one system-scope release per unit, by one lane, behind every wave's drained stores */
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const uint32_t old = atomicAdd(&ds->done[slot], mine);
            if (old + mine == n) {
                st_dev(&ds->done[slot], 0u);
                __hip_atomic_store(&ds->claim[slot], (unsigned long long)(j / RING + 1ull) << 32, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&ring->fin[slot], j + 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        __syncthreads();
    }
}

__global__ void empty_kernel() {}

__global__ __launch_bounds__(UNIT_THREADS) void copy_kernel(const uint8_t *src, uint8_t *dst, uint32_t ub)
{
    const uint4 *s = (const uint4 *)(src + (size_t)blockIdx.x * ub);
    uint4 *d = (uint4 *)(dst + (size_t)blockIdx.x * ub);
    for (uint32_t i = threadIdx.x; i < ub / 16u; i += UNIT_THREADS)
        d[i] = s[i];
}

static double now_us()
{
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static volatile Ring *g_ring;
static uint64_t g_next, g_units;
static uint32_t g_P;

static uint64_t post(uint32_t nunits, uint32_t ub, const uint8_t *src, uint8_t *dst)
{
    const uint64_t j = g_next++;
    volatile Job *jb = &g_ring->jobs[j % RING];
    jb->id = j;
    jb->nunits = nunits;
    jb->unit_bytes = ub;
    jb->base = (uint32_t)(g_units % g_P);
    g_units += nunits;
    jb->src = src;
    jb->dst = dst;
    __atomic_thread_fence(__ATOMIC_RELEASE);
    g_ring->tail = j + 1;
    return j;
}

static int wait_job(uint64_t j)
{
    const double t0 = now_us();
    while (g_ring->fin[j % RING] != j + 1) {
        if (now_us() - t0 > 2e6) {
            fprintf(stderr, "job %llu: no completion after 2 s\n", (unsigned long long)j);
            g_ring->stop = 1;
            return -1;
        }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return 0;
}

int main(int argc, char **argv)
{
    const int P = argc > 1 ? atoi(argv[1]) : 256;
    const uint32_t mode = argc > 2 ? (uint32_t)atoi(argv[2]) : 0u;
    g_P = (uint32_t)P;
    int wclk_khz = 0;
    CHK(hipDeviceGetAttribute(&wclk_khz, hipDeviceAttributeWallClockRate, 0));
    const uint64_t ticks_ms = (uint64_t)wclk_khz;
    hipStream_t st;
    CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

    Ring *ring_h = nullptr, *ring_d = nullptr;
    CHK(hipHostMalloc((void **)&ring_h, sizeof(Ring), hipHostMallocMapped | hipHostMallocCoherent));
    memset(ring_h, 0, sizeof(Ring));
    CHK(hipHostGetDevicePointer((void **)&ring_d, ring_h, 0));
    g_ring = ring_h;
    DevState *ds = nullptr;
    CHK(hipMalloc(&ds, sizeof(DevState)));
    CHK(hipMemset(ds, 0, sizeof(DevState)));

    const size_t WIN = 256 << 10, UB = 4096, NWIN = 32;
    uint8_t *hsrc, *hdst, *dsrc, *ddst;
    CHK(hipHostMalloc((void **)&hsrc, WIN * NWIN, hipHostMallocMapped | hipHostMallocCoherent));
    CHK(hipHostMalloc((void **)&hdst, WIN * NWIN, hipHostMallocMapped | hipHostMallocCoherent));
    for (size_t i = 0; i < WIN * NWIN; ++i)
        hsrc[i] = (uint8_t)(i * 2654435761u >> 13);
    CHK(hipHostGetDevicePointer((void **)&dsrc, hsrc, 0));
    CHK(hipHostGetDevicePointer((void **)&ddst, hdst, 0));

    /* 1: launch + sync floor */
    std::vector<double> v;
    for (int i = 0; i < 2200; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st);
        CHK(hipStreamSynchronize(st));
        if (i >= 200)
            v.push_back(now_us() - t0);
    }
    printf("{\"what\": \"launch_sync\", \"median_us\": %.2f}\n", median(v));

    /* 2: copy window by a launch per window */
    v.clear();
    for (int i = 0; i < 600; ++i) {
        const double t0 = now_us();
        hipLaunchKernelGGL(copy_kernel, dim3(WIN / UB), dim3(UNIT_THREADS), 0, st, dsrc + (i % NWIN) * WIN,
                           ddst + (i % NWIN) * WIN, (uint32_t)UB);
        CHK(hipStreamSynchronize(st));
        if (i >= 100)
            v.push_back(now_us() - t0);
    }
    printf("{\"what\": \"copy_launch\", \"window_bytes\": %zu, \"median_us\": %.2f}\n", WIN, median(v));
    fflush(stdout);

    /* the resident grid */
    hipLaunchKernelGGL(resident, dim3(P + 1), dim3(UNIT_THREADS), 0, st, ring_d, ds, (uint64_t)0,
                       (uint64_t)IDLE_MS * ticks_ms, (uint64_t)MAX_S * 1000ull * ticks_ms, mode);
    CHK(hipGetLastError());
    int rc = 0;

    /* 3: empty doorbell job */
    v.clear();
    for (int i = 0; i < 2200 && rc == 0; ++i) {
        const double t0 = now_us();
        rc = wait_job(post(1, 0, dsrc, ddst));
        if (i >= 200)
            v.push_back(now_us() - t0);
    }
    if (rc == 0)
        printf("{\"what\": \"doorbell_empty\", \"grid\": %d, \"mode\": %u, \"median_us\": %.2f}\n", P, mode, median(v));

    /* 4: copy window as doorbell jobs, D outstanding */
    const int depths[] = {1, 2, 4, 8, 16};
    for (int d : depths) {
        if (rc != 0)
            break;
        memset(hdst, 0, WIN * NWIN);
        const int N = 800;
        std::vector<uint64_t> ids;
        std::vector<double> post_t(N);
        v.clear();
        const double t0 = now_us();
        for (int i = 0; i < N && rc == 0; ++i) {
            if (i >= d) {
                rc = wait_job(ids[i - d]);
                v.push_back(now_us() - post_t[i - d]);
            }
            post_t[i] = now_us();
            ids.push_back(post((uint32_t)(WIN / UB), (uint32_t)UB, dsrc + (i % NWIN) * WIN, ddst + (i % NWIN) * WIN));
        }
        for (int i = N - d; i < N && rc == 0; ++i) {
            rc = wait_job(ids[i]);
            v.push_back(now_us() - post_t[i]);
        }
        const double el = now_us() - t0;
        if (rc == 0) {
            const int ok = memcmp(hsrc, hdst, WIN * NWIN) == 0;
            printf("{\"what\": \"copy_doorbell_d%d\", \"grid\": %d, \"mode\": %u, \"window_bytes\": %zu, "
                   "\"latency_median_us\": %.2f, \"gbps_each_way\": %.2f, \"us_per_window\": %.2f, \"verified\": %d}\n",
                   d, P, mode, WIN, median(v), (double)N * WIN / el / 1e3, el / N, ok);
            fflush(stdout);
        }
    }
    g_ring->stop = 1;
    CHK(hipStreamSynchronize(st));
    printf("{\"what\": \"resident_exit\", \"ok\": %d}\n", rc == 0);
    return rc == 0 ? 0 : 2;
}
