/*
 * fault_journal.c -- attribution of GPU memory faults.
 *
 * A page fault of a kernel reaches the process asynchronously: the faulting wave does not stop, the KFD signals the
 * fault, and the ROCr event thread hands it to every handler registered with hsa_amd_register_system_event_handler
 * (HIP registers one, which turns the fault into the sticky hipErrorIllegalAddress and prints nothing).  The address
 * and the cause are then lost: the next HIP call of whatever code runs next reports "an illegal memory access".
 *
 * This file keeps a ring of the engine's last 256 device events -- every kernel launch with its stream, grid and
 * pointer arguments (with their extents where the engine knows them), every device allocation, free, host
 * registration and device check -- and registers a handler of its own that, on HSA_AMD_GPU_MEMORY_FAULT_EVENT,
 * writes the faulting virtual address, the fault reasons and the journal (each range that holds the address marked)
 * to stderr and to the file given at install.  The handler only observes: it returns HSA_STATUS_ERROR, so the
 * runtime's handling (HIP's) is what decides the outcome, as without it.
 *
 * The report also says what the faulting address IS at the moment of the fault: what the runtime knows of it and of
 * the byte before its page (hsa_amd_pointer_info: an HSA allocation, a locked / registered host range and its extent,
 * or unknown), the /proc/self/maps line that holds it (device memory, the heap, an anonymous mapping, nothing), and
 * the tables other parts of the library keep (the record layer's host registrations, via
 * ptls_mi355x_fault_journal_add_dumper) -- so a fault on memory the engine never launched on still names its owner.
 */
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include "fault_journal.h"

#define RING 256

enum { EV_LAUNCH = 1, EV_MEM = 2 };

struct event {
    uint64_t seq, t_ns;
    int kind;
    const char *what; /* kernel name or memory event (static strings) */
    const void *stream;
    uint32_t blocks, threads;
    uint64_t n;
    size_t nargs;
    ptls_mi355x_journal_arg_t a[PTLS_MI355X_JOURNAL_ARGS];
};

static struct event g_ring[RING];
static uint64_t g_next; /* events recorded (under g_mu) */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static char g_path[512];
#define DUMPERS 4
static ptls_mi355x_journal_dumper_t g_dumpers[DUMPERS];
static atomic_int g_ndumpers;
static atomic_ulong g_faults;
static atomic_int g_installed;

static uint64_t now_ns(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static void record(const struct event *e)
{
    pthread_mutex_lock(&g_mu);
    struct event *slot = &g_ring[g_next % RING];
    *slot = *e;
    slot->seq = g_next++;
    slot->t_ns = now_ns();
    pthread_mutex_unlock(&g_mu);
}

void ptls_mi355x_journal_launch(const char *kernel, const void *stream, uint32_t blocks, uint32_t threads, uint64_t n,
                                const ptls_mi355x_journal_arg_t *args, size_t nargs)
{
    struct event e;
    memset(&e, 0, sizeof(e));
    e.kind = EV_LAUNCH;
    e.what = kernel;
    e.stream = stream;
    e.blocks = blocks;
    e.threads = threads;
    e.n = n;
    e.nargs = nargs < PTLS_MI355X_JOURNAL_ARGS ? nargs : PTLS_MI355X_JOURNAL_ARGS;
    memcpy(e.a, args, e.nargs * sizeof(*args));
    record(&e);
}

void ptls_mi355x_fault_journal_note(const char *what, const void *p, size_t len)
{
    struct event e;
    memset(&e, 0, sizeof(e));
    e.kind = EV_MEM;
    e.what = what;
    e.nargs = 1;
    e.a[0].name = "range";
    e.a[0].p = p;
    e.a[0].len = len;
    record(&e);
}

static const char *reasons(uint32_t m, char *buf, size_t cap)
{
    static const struct {
        uint32_t bit;
        const char *name;
    } names[] = {{HSA_AMD_MEMORY_FAULT_PAGE_NOT_PRESENT, "page not present or supervisor privilege"},
                 {HSA_AMD_MEMORY_FAULT_READ_ONLY, "write to a read-only page"},
                 {HSA_AMD_MEMORY_FAULT_NX, "execute on a no-execute page"},
                 {HSA_AMD_MEMORY_FAULT_HOST_ONLY, "host-only memory"},
                 {HSA_AMD_MEMORY_FAULT_DRAMECC, "DRAM ECC"},
                 {HSA_AMD_MEMORY_FAULT_IMPRECISE, "imprecise"},
                 {HSA_AMD_MEMORY_FAULT_SRAMECC, "SRAM ECC"},
                 {HSA_AMD_MEMORY_FAULT_HANG, "hang"}};
    buf[0] = 0;
    for (size_t i = 0; i < sizeof(names) / sizeof(names[0]); ++i)
        if (m & names[i].bit) {
            size_t l = strlen(buf);
            snprintf(buf + l, cap - l, "%s%s", l ? ", " : "", names[i].name);
        }
    return buf[0] ? buf : "none given";
}

/* where va lies relative to an argument: inside its known extent, or (extent unknown) at most 1 GiB past its base */
static const char *hit(const ptls_mi355x_journal_arg_t *a, uint64_t va)
{
    const uint64_t p = (uint64_t)(uintptr_t)a->p;
    if (a->p == NULL)
        return "";
    if (a->len != 0)
        return va >= p && va - p < a->len ? "   <== HOLDS THE FAULTING ADDRESS" : "";
    return va >= p && va - p < (1ull << 30) ? "   <== faulting address within 1 GiB past this base" : "";
}

static const char *pointer_type(hsa_amd_pointer_type_t t)
{
    switch (t) {
    case HSA_EXT_POINTER_TYPE_UNKNOWN: return "unknown to the runtime";
    case HSA_EXT_POINTER_TYPE_HSA: return "HSA allocation (device memory or hipHostMalloc)";
    case HSA_EXT_POINTER_TYPE_LOCKED: return "locked host range (hipHostRegister, or a runtime pin of pageable memory)";
    case HSA_EXT_POINTER_TYPE_GRAPHICS: return "graphics interop";
    case HSA_EXT_POINTER_TYPE_IPC: return "IPC import";
    case HSA_EXT_POINTER_TYPE_RESERVED_ADDR: return "reserved address range (virtual memory API)";
    case HSA_EXT_POINTER_TYPE_HSA_VMEM: return "virtual memory API allocation";
    default: return "?";
    }
}

/* what the runtime knows of an address now */
static void describe_pointer(FILE *f, const char *label, uint64_t a)
{
    hsa_amd_pointer_info_t info;
    memset(&info, 0, sizeof(info));
    info.size = sizeof(info);
    const hsa_status_t st = hsa_amd_pointer_info((const void *)(uintptr_t)a, &info, NULL, NULL, NULL);
    if (st != HSA_STATUS_SUCCESS) {
        fprintf(f, "  %s 0x%llx: hsa_amd_pointer_info status %d\n", label, (unsigned long long)a, (int)st);
        return;
    }
    if (info.type == HSA_EXT_POINTER_TYPE_UNKNOWN) {
        fprintf(f, "  %s 0x%llx: %s\n", label, (unsigned long long)a, pointer_type(info.type));
        return;
    }
    fprintf(f, "  %s 0x%llx: %s, host base %p, agent base %p, %llu bytes (ends at 0x%llx)\n", label,
            (unsigned long long)a, pointer_type(info.type), info.hostBaseAddress, info.agentBaseAddress,
            (unsigned long long)info.sizeInBytes,
            (unsigned long long)((uintptr_t)info.hostBaseAddress + info.sizeInBytes));
}

/* the process mappings around an address (/proc/self/maps: the line holding it, and the one before) */
static void describe_mapping(FILE *f, uint64_t va)
{
    FILE *m = fopen("/proc/self/maps", "r");
    if (m == NULL) {
        fprintf(f, "  /proc/self/maps: unreadable\n");
        return;
    }
    char line[512], prev[512] = "";
    int found = 0;
    while (fgets(line, sizeof(line), m) != NULL) {
        unsigned long long lo = 0, hi = 0;
        if (sscanf(line, "%llx-%llx", &lo, &hi) != 2)
            continue;
        if (va < lo) {
            fprintf(f, "  maps: 0x%llx is in no mapping; around it:\n    %s    %s", (unsigned long long)va,
                    prev[0] ? prev : "(none)\n", line);
            found = 1;
            break;
        }
        if (va < hi) {
            fprintf(f, "  maps: %s", line);
            found = 1;
            break;
        }
        snprintf(prev, sizeof(prev), "%s", line);
    }
    if (!found)
        fprintf(f, "  maps: 0x%llx is above every mapping\n", (unsigned long long)va);
    fclose(m);
}

static void write_report(FILE *f, uint64_t va, uint32_t mask, uint64_t agent, uint64_t t_fault)
{
    char rbuf[256];
    fprintf(f, "=== ptls_mi355x fault journal: GPU memory fault at VA 0x%016llx, reasons 0x%x (%s), agent 0x%llx, pid %d,"
               " t=%llu ns ===\n",
            (unsigned long long)va, mask, reasons(mask, rbuf, sizeof(rbuf)), (unsigned long long)agent, (int)getpid(),
            (unsigned long long)t_fault);
    fprintf(f, "the faulting address now:\n");
    describe_pointer(f, "fault VA", va);
    describe_pointer(f, "byte before its page", (va & ~4095ull) - 1);
    describe_mapping(f, va);
    const int nd = atomic_load(&g_ndumpers);
    for (int i = 0; i < nd && i < DUMPERS; ++i)
        if (g_dumpers[i] != NULL)
            g_dumpers[i](f, va);
    /* a snapshot under the lock when it can be had (the faulting thread may hold it: then read as it is) */
    const int locked = pthread_mutex_trylock(&g_mu) == 0;
    const uint64_t end = g_next, start = end > RING ? end - RING : 0;
    fprintf(f, "journal: events %llu..%llu (oldest first; t = ms before the fault)\n", (unsigned long long)start,
            (unsigned long long)(end ? end - 1 : 0));
    for (uint64_t s = start; s < end; ++s) {
        const struct event *e = &g_ring[s % RING];
        const double ago = t_fault >= e->t_ns ? (double)(t_fault - e->t_ns) / 1e6 : -(double)(e->t_ns - t_fault) / 1e6;
        if (e->kind == EV_LAUNCH) {
            fprintf(f, "#%llu t-%.3f launch %s stream %p grid %ux%u n %llu\n", (unsigned long long)e->seq, ago,
                    e->what ? e->what : "?", e->stream, e->blocks, e->threads, (unsigned long long)e->n);
            for (size_t i = 0; i < e->nargs; ++i)
                fprintf(f, "      %-8s %p + %llu%s\n", e->a[i].name ? e->a[i].name : "?", e->a[i].p,
                        (unsigned long long)e->a[i].len, hit(&e->a[i], va));
        } else {
            fprintf(f, "#%llu t-%.3f %s %p + %llu%s\n", (unsigned long long)e->seq, ago, e->what ? e->what : "?",
                    e->a[0].p, (unsigned long long)e->a[0].len, hit(&e->a[0], va));
        }
    }
    if (locked)
        pthread_mutex_unlock(&g_mu);
    fprintf(f, "=== end of fault journal ===\n");
    fflush(f);
}

static void report(uint64_t va, uint32_t mask, uint64_t agent)
{
    const uint64_t t = now_ns();
    write_report(stderr, va, mask, agent, t);
    if (g_path[0] != 0) {
        FILE *f = fopen(g_path, "a");
        if (f != NULL) {
            write_report(f, va, mask, agent, t);
            fclose(f);
        }
    }
}

static hsa_status_t on_system_event(const hsa_amd_event_t *event, void *data)
{
    (void)data;
    if (event != NULL && event->event_type == HSA_AMD_GPU_MEMORY_FAULT_EVENT) {
        atomic_fetch_add(&g_faults, 1);
        report(event->memory_fault.virtual_address, event->memory_fault.fault_reason_mask,
               event->memory_fault.agent.handle);
    }
    return HSA_STATUS_ERROR; /* observe only: the runtime's own handling (HIP's handler) decides the outcome */
}

int ptls_mi355x_fault_journal_install(const char *path)
{
    pthread_mutex_lock(&g_mu);
    if (path != NULL)
        snprintf(g_path, sizeof(g_path), "%s", path);
    else
        g_path[0] = 0;
    pthread_mutex_unlock(&g_mu);
    if (atomic_load(&g_installed))
        return 0;
    /* the runtime stays initialised for the process (HIP initialises it too; the reference count only grows) */
    hsa_status_t st = hsa_init();
    if (st != HSA_STATUS_SUCCESS)
        return (int)st;
    st = hsa_amd_register_system_event_handler(on_system_event, NULL);
    if (st != HSA_STATUS_SUCCESS)
        return (int)st;
    atomic_store(&g_installed, 1);
    return 0;
}

void ptls_mi355x_fault_journal_add_dumper(ptls_mi355x_journal_dumper_t fn)
{
    pthread_mutex_lock(&g_mu);
    const int n = atomic_load(&g_ndumpers);
    int have = 0;
    for (int i = 0; i < n; ++i)
        have |= g_dumpers[i] == fn;
    if (!have && n < DUMPERS) {
        g_dumpers[n] = fn;
        atomic_store(&g_ndumpers, n + 1);
    }
    pthread_mutex_unlock(&g_mu);
}

int ptls_mi355x_fault_journal_installed(void)
{
    return atomic_load(&g_installed);
}

unsigned long ptls_mi355x_fault_journal_faults(void)
{
    return atomic_load(&g_faults);
}

void ptls_mi355x_fault_journal_report(uint64_t va, uint32_t reason_mask)
{
    report(va, reason_mask, 0);
}
