/*
 * tests/cpp/guard_alloc.c -- device memory with unmapped guard ranges on both sides (test only).
 *
 * A virtual range of 3 x `bytes` (granularity-rounded) is reserved and only its middle third is mapped, read-write,
 * on the current device.  A kernel that reads or writes past either end of the middle third touches an address with
 * no mapping behind it: a GPU page fault, which the test's device check reports.  tests/test_gpu_read_bounds.py places
 * records, descriptors and outputs flush against both ends and runs every kernel family over them: the deterministic
 * form of "nothing is read outside a record" (a record that ends at a page edge of a torch allocation faulted only
 * when the allocator happened to put it there).  Not part of the product.
 */
#include <stdint.h>
#include <string.h>
#include <hip/hip_runtime_api.h>

typedef struct {
    void *reserved;
    size_t reserved_len;
    void *data; /* the mapped middle */
    size_t len;
    hipMemGenericAllocationHandle_t handle;
} guard_t;

static hipMemAllocationProp prop_for(int dev)
{
    hipMemAllocationProp p;
    memset(&p, 0, sizeof(p));
    p.type = hipMemAllocationTypePinned;
    p.location.type = hipMemLocationTypeDevice;
    p.location.id = dev;
    return p;
}

/* 0 and *out filled, or the HIP error code; *data_len receives the mapped length (>= bytes) */
int guard_alloc(size_t bytes, guard_t *out)
{
    memset(out, 0, sizeof(*out));
    int dev = 0, vmm = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess)
        e = hipDeviceGetAttribute(&vmm, hipDeviceAttributeVirtualMemoryManagementSupported, dev);
    if (e != hipSuccess)
        return (int)e;
    if (!vmm)
        return -1;
    hipMemAllocationProp p = prop_for(dev);
    size_t g = 0;
    if ((e = hipMemGetAllocationGranularity(&g, &p, hipMemAllocationGranularityMinimum)) != hipSuccess)
        return (int)e;
    const size_t len = (bytes + g - 1) / g * g;
    if ((e = hipMemAddressReserve(&out->reserved, 3 * len, g, NULL, 0)) != hipSuccess)
        return (int)e;
    out->reserved_len = 3 * len;
    out->data = (uint8_t *)out->reserved + len;
    out->len = len;
    if ((e = hipMemCreate(&out->handle, len, &p, 0)) != hipSuccess)
        goto Fail;
    if ((e = hipMemMap(out->data, len, 0, out->handle, 0)) != hipSuccess)
        goto Fail;
    hipMemAccessDesc a;
    memset(&a, 0, sizeof(a));
    a.location = p.location;
    a.flags = hipMemAccessFlagsProtReadWrite;
    if ((e = hipMemSetAccess(out->data, len, &a, 1)) != hipSuccess)
        goto Fail;
    return 0;
Fail:
    if (out->handle != NULL) {
        (void)hipMemUnmap(out->data, len);
        (void)hipMemRelease(out->handle);
    }
    (void)hipMemAddressFree(out->reserved, out->reserved_len);
    memset(out, 0, sizeof(*out));
    return (int)e;
}

int guard_free(guard_t *g)
{
    hipError_t e = hipDeviceSynchronize();
    if (g->handle != NULL) {
        const hipError_t e1 = hipMemUnmap(g->data, g->len);
        const hipError_t e2 = hipMemRelease(g->handle);
        e = e != hipSuccess ? e : e1 != hipSuccess ? e1 : e2;
    }
    if (g->reserved != NULL) {
        const hipError_t e3 = hipMemAddressFree(g->reserved, g->reserved_len);
        e = e != hipSuccess ? e : e3;
    }
    memset(g, 0, sizeof(*g));
    return (int)e;
}

size_t guard_struct_size(void) { return sizeof(guard_t); }

/* blocking copies in and out of guarded memory (hipMemcpy): 0 or the HIP error code */
int guard_h2d(void *dst, const void *src, size_t n) { return n ? (int)hipMemcpy(dst, src, n, hipMemcpyHostToDevice) : 0; }
int guard_d2h(void *dst, const void *src, size_t n) { return n ? (int)hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) : 0; }
int guard_memset(void *dst, int v, size_t n) { return n ? (int)hipMemset(dst, v, n) : 0; }
