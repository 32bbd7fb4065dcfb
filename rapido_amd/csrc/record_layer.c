/*
 * record_layer.c -- a batched TLS 1.3 record layer over HOST buffers (include/ptls_mi355x.h section 5).
 *
 * The reference hands each record to the AEAD one at a time: rapido_prepare_data loops ptls_send over its send
 * window (lib/rapido.c:2083-2111), and picotls frames one record per call (buffer_push_encrypted_records,
 * lib/picotls.c:664-684; handle_input, lib/picotls.c:4757-4842).  An application with its own record layer gets the
 * traffic secrets from picotls' update_traffic_key callback (lib/picotls.c:1206-1211) instead.  This file is that
 * record layer for one traffic direction of one connection, on the GPU: a whole window of records is framed and
 * sealed (or opened and unframed) in one launch.
 *
 *   seal: the fragments are planned into records (ptls_mi355x_tls_plan_send, <= 16384 bytes each, consecutive
 *         seq), sealed by ptls_mi355x_tls_seal_records; seq advances by the record count, as ptls_send's does.
 *         A fragment is one ptls_send call: it is sealed only if seq is below 2^24 when it starts (ptls_send forces a
 *         key update there, lib/picotls.c:4976-4977); the window stops before the first fragment at or past the
 *         limit and reports PTLS_MI355X_RECORD_LAYER_KEY_UPDATE.  Records of other content types (the KeyUpdate
 *         message itself, update_send_key :4949-4962) are sealed past it.
 *   open: the complete application_data records at the start of the input are parsed (ptls_mi355x_tls_parse_
 *         records) and opened by ptls_mi355x_tls_open_records.  Records are then delivered in order until the first
 *         failure (its alert is returned, as ptls_receive returns it, lib/picotls.c:650-652) or the first record
 *         whose inner type is not application_data (left unconsumed, seq not advanced, for open_record below).
 *         Every record is verified independently by the kernel; the stop at the first failure is this host loop,
 *         and nothing behind it reaches the caller (slots are zeroed).
 *
 * Windows are asynchronous: a submit plans, stages and launches a window on one of the layer's RL_SLOTS slots and
 * returns; wait (in submission order) completes it.  Each slot has its own stream, staging, device buffer and engine
 * context (the split kernels' arrival tickets and the batch kernels' work counters are per context, so windows on
 * different slots never wait for each other).  A send window's records take their seq at submit.  A receive window
 * takes the seq that follows the windows before it (speculatively: they are not verified yet); if one of them stops
 * early (a failure, a non-application_data record, a full output), the windows submitted behind it are stale and
 * their wait reports PTLS_MI355X_RECORD_LAYER_STALE with nothing delivered.  The synchronous calls are a submit and
 * its wait.
 *
 * Where the bytes travel, per window (the first that applies):
 *   direct     -- the fragments and the output (seal), or the input and the output (open), all lie in host ranges
 *                 the caller registered (ptls_mi355x_record_layer_register: long-lived socket buffers): the kernel
 *                 reads the input in place over PCIe.  Seal writes the wire records in place (inputs overlapping the
 *                 outputs go through the staging instead); open leaves the plaintext slots in device memory and the
 *                 delivery kernel (ptls_mi355x_tls_deliver_records) writes the delivered plaintexts once, back to
 *                 back, into the caller's buffer.  Only descriptors and statuses pass through the slot's staging.
 *                 ptls_mi355x_record_layer_set_direct_dma(rl, 1) moves registered windows by DMA copies to and from
 *                 device memory instead (measured slower); (rl, 2) moves only the inputs by DMA (the copy
 *                 engine reads host memory faster than kernel loads do) and keeps the in-place writes: seal's wire
 *                 records, an open's delivery kernel.
 *   zero-copy  -- the window fits the zero-copy limit: fragments / input are copied into the slot's pinned,
 *                 mapped, coherent staging and the kernel works on it over PCIe.
 *   copy       -- larger windows: staging -> one H2D copy -> launch -> one D2H copy (DMA at the link rate).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <stdio.h>
#include <pthread.h>
#include <hip/hip_runtime_api.h>
#include "../../include/ptls_mi355x.h"
#include "fault_journal.h"

#define RL_MAX_REGIONS 8
#define RL_ZERO_COPY_DEFAULT ((size_t)4 << 20)
#define RL_SLOTS 4    /* launches in flight per layer */
#define RL_TICKETS 32 /* windows outstanding per layer (submitted and not yet waited for) */
#define RL_COALESCE_DEFAULT 16 /* a connection's queued windows per launch (ptls_mi355x_record_layer_set_coalesce) */
/* a coalescing slot's staging grows with headroom for larger groups of the same windows (no allocation stall
 * mid-stream), but never more than this beyond what the op needs: pinned memory per connection stays bounded for
 * servers with hundreds of connections (4 slots x (need + 2 MiB) at most) */
#define RL_STAGE_HEADROOM ((size_t)2 << 20)

typedef struct {
    uint8_t *base;   /* host address as registered */
    uint8_t *dev;    /* its device address */
    size_t len;
    int owned;       /* holds a reference on the process-wide entry (g_reg) of the range that contains it */
    uint8_t *shared; /* that entry's base */
} rl_region_t;

/* one layer's part of a window */
typedef struct {
    /* seal */
    size_t nfrags, wire; /* fragments taken (before the key-update limit), their wire bytes */
    int stopped;         /* stopped at the limit */
    /* open */
    size_t k0, n, cons, ptbytes; /* descriptors recs[k0 .. k0 + n), wire bytes parsed, plaintext slot bytes */
    size_t slots16;              /* the slot bytes with every slot 16-aligned (delivery kernel) */
    uint64_t src_add, dst_add;   /* added to its descriptors' offsets (its position in the launch's src / dst) */
    int perr;
    /* both */
    uint64_t seq0; /* seq of its first record */
    size_t nrec;   /* records in the launch */
} rl_part_t;

typedef struct {
    void *dst;
    const void *src;
    size_t n;
} rl_copy_t;

typedef struct {
    int busy, is_seal, any_type; /* any_type: open_record (one record of any inner content type) */
    uint64_t ticket;             /* the first window's ticket */
    size_t nwin, waited;         /* windows (tickets) in the launch, and how many of them have been waited for */
    int coalesced;               /* one single-layer window per part (the layer's queued windows) */
    int done, failed;            /* completed (results below), or its launch / synchronisation failed */
    size_t *r_outlen, *r_nrec, *r_cons; /* per part, once done */
    int *r_alert;
    size_t nlayers;
    ptls_mi355x_record_layer_t **layers;
    void **out;
    size_t *capacity;
    rl_part_t *part;
    int direct, zero_copy, dma; /* direct: the results land in the caller's buffers (mapped or dma) */
    int deliver;                /* mapped open: slots in device memory, the delivery kernel writes the plaintexts */
    int dma_in;                 /* direct, the inputs moved to device memory by DMA first (set_direct_dma 2) */
    size_t nrec, off_src, srcbytes, off_dst, dstbytes, off_st, off_ty, off_dp, max_part;
    rl_copy_t *h2d, *d2h; /* dma: registered host ranges <-> the slot's device buffer */
    size_t nh2d, nd2h;
    /*
     * Sessions (op_sessions): the op's layers grouped by session -- key and IV bytes 4..11 (a rapido session's
     * connections differ only in IV bytes 0..3, lib/rapido.c:127-133).  One session: the single-key launch, each record
     * carrying its connection's IV difference.  Several: a multi-key launch (ptls_mi355x_tls_*_records_multikey), each
     * record also carrying its session's index, the key of session k being its first layer's context.
     */
    size_t nsess;
    ptls_mi355x_aesgcm_context_t **sess_ctx; /* per session */
    uint8_t *sess_iv;                        /* per session: its first layer's IV */
    uint32_t *sess_of;                       /* per layer: its session */
    size_t off_kidx;                         /* nsess > 1: the per-record session indices in the staging layout */
} rl_op_t;

typedef struct {
    hipStream_t stream;
    ptls_mi355x_aesgcm_context_t *ctx;
    uint8_t *h_buf; /* pinned, mapped, coherent staging: [descriptors | conn ids | input | output | status | types] */
    uint8_t *h_dev; /* the staging's device address (zero-copy and direct windows) */
    size_t cap;
    uint8_t *d_buf; /* device copy of the staging layout (copy windows), allocated on first use */
    size_t d_cap;
    ptls_mi355x_tls_record_t *recs; /* host descriptors */
    size_t recs_cap;
    size_t grow; /* a coalesced op of n windows: its staging grows to this many times its need (cap / n), so a later,
                  * larger group of the same windows finds room (no allocation, and no stall, mid-stream) */
    int copies_prepared; /* ptls_mi355x_prepare_copies called for its first copy */
    rl_op_t op;
} rl_slot_t;

struct st_ptls_mi355x_record_layer_t {
    uint8_t key[32]; /* the key, for the slots' contexts and to check that the layers of a _multi call share it */
    size_t key_size;
    uint8_t iv[12];
    uint64_t seq;      /* seal: the next record's seq; open: the seq of the next record to deliver */
    uint64_t spec_seq; /* open: the seq of the next record to submit (ahead of seq while windows are in flight) */
    size_t zero_copy_bytes;
    int direct_dma; /* registered windows move by DMA to and from device memory (1), are read in place (0, default), or
                     * the inputs move by DMA and the outputs are written in place (2) */
    rl_region_t reg[RL_MAX_REGIONS];
    size_t nreg;
    rl_slot_t slot[RL_SLOTS];
    uint64_t next_ticket, oldest; /* tickets [oldest, next_ticket) are outstanding */
    /* launches in flight that name this layer, on its own slots or on another layer's (a multi-layer submit): counted
     * once per launch when it goes out, dropped when it completes (a wait, or its lead layer's free) */
    size_t inflight;
    int zombie; /* freed while windows of other layers still name it: its memory goes with the last of them */
    uint64_t launches;                /* launches so far (slot = launches % RL_SLOTS) */
    int8_t ticket_slot[RL_TICKETS];   /* ticket % RL_TICKETS -> slot of the launch holding it */
    /*
     * Coalescing: single-layer windows submitted while a launch of this layer is still running are queued here and go
     * out together, one launch for all of them, when the layer's launches are done (checked at the next submit), at
     * the first wait for one of them, when `coalesce` windows are queued, or at ptls_mi355x_record_layer_flush.
     */
    size_t coalesce;                  /* windows per launch at most; <= 1: every window launched at its submit */
    int corked;                       /* windows queue even while nothing runs (ptls_mi355x_record_layer_cork) */
    struct rl_queued *queue;          /* coalesce entries */
    size_t nqueued;
    uint64_t queue_ticket;            /* ticket of queue[0] */
};

/* a window queued for coalescing: its submit arguments (the iovec array copied) and the seq it takes */
struct rl_queued {
    ptls_mi355x_iovec_t *frags; /* seal */
    size_t nfrags;
    const void *in; /* open */
    size_t inlen;
    void *out;
    size_t capacity;
    uint64_t seq0; /* seal: seq of its first record; open: the speculative seq its records take */
    int is_seal;
    uint8_t type; /* seal: the content type its records carry (a group never mixes types: rl_flush_n) */
};

static _Thread_local char rl_err[160]; /* per thread, as the engine's (layers on different threads) */

/* gcm_engine.hip: an error met where nothing can be returned (a free path) -- printed and kept for
 * ptls_mi355x_device_check, never dropped */
void ptls_mi355x_defer_error(const char *what, int err);
#define RL_DEFER(what, call) ptls_mi355x_defer_error("record layer: " what, (int)(call))

static void op_discard(rl_op_t *op);
static void op_release_layers(rl_op_t *op);
static int rl_flush_n(ptls_mi355x_record_layer_t *rl, size_t n);
static int overlaps(const void *a, size_t alen, const void *b, size_t blen);

static size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

static int rl_fail(const char *what, hipError_t e)
{
    snprintf(rl_err, sizeof(rl_err), "record layer: %s: %s", what, hipGetErrorString(e));
    (void)hipGetLastError(); /* reported here: not left for the next unrelated call to find */
    return -1;
}

static int rl_msg(const char *msg)
{
    snprintf(rl_err, sizeof(rl_err), "record layer: %s", msg);
    return -1;
}

const char *ptls_mi355x_record_layer_last_error(void) { return rl_err; }

static int reserve_recs(rl_slot_t *s, size_t nrecs)
{
    if (nrecs <= s->recs_cap)
        return 0;
    size_t c = s->recs_cap ? s->recs_cap : 64;
    while (c < nrecs)
        c *= 2;
    ptls_mi355x_tls_record_t *r = realloc(s->recs, c * sizeof(*r));
    if (r == NULL)
        return rl_msg("out of memory");
    s->recs = r;
    s->recs_cap = c;
    return 0;
}

/* PTLS_MI355X_RL_TRACE set: every allocation a window triggers (staging growth, slot creation) to stderr, with its
 * slot -- they synchronise or stall, and belong at setup rather than mid-stream */
static int rl_trace_on(void)
{
    static int on = -1;
    if (on < 0)
        on = getenv("PTLS_MI355X_RL_TRACE") != NULL;
    return on;
}

static double rl_now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

/* traced: a call of op_launch that took over 1 ms */
static void rl_slow(const char *what, double t0)
{
    const double dt = rl_now() - t0;
    if (dt > 1e-3)
        fprintf(stderr, "record layer: %s took %.3f ms\n", what, dt * 1e3);
}

static int reserve_stage(rl_slot_t *s, size_t bytes)
{
    if (bytes <= s->cap)
        return 0;
    size_t c = s->cap ? s->cap : 1 << 16;
    if (s->grow > 1) { /* headroom for a larger group later, at most RL_STAGE_HEADROOM beyond the need */
        const size_t want = bytes * s->grow, most = bytes + RL_STAGE_HEADROOM;
        bytes = want < most ? want : most;
    }
    while (c < bytes)
        c *= 2;
    hipError_t e;
    if (s->h_buf != NULL) {
        memset(s->h_buf, 0, s->cap);
        ptls_mi355x_fault_journal_note("record layer: hipHostFree staging (device view)", s->h_dev, s->cap);
        const hipError_t ef = hipHostFree(s->h_buf);
        s->h_buf = s->h_dev = NULL;
        s->cap = 0;
        if (ef != hipSuccess)
            return rl_fail("hipHostFree (staging growth)", ef);
    }
    s->h_buf = s->h_dev = NULL;
    s->cap = 0;
    /* coherent: the kernel's zero-copy reads never see stale lines of an earlier window */
    if ((e = hipHostMalloc((void **)&s->h_buf, c, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
        return rl_fail("hipHostMalloc", e);
    if ((e = hipHostGetDevicePointer((void **)&s->h_dev, s->h_buf, 0)) != hipSuccess)
        return rl_fail("hipHostGetDevicePointer", e);
    ptls_mi355x_fault_journal_note("record layer: hipHostMalloc staging (device view)", s->h_dev, c);
    s->cap = c;
    if (rl_trace_on())
        fprintf(stderr, "record layer: slot %p staging grown to %zu B\n", (void *)s, c);
    return 0;
}

static int reserve_device(rl_slot_t *s)
{
    if (s->cap <= s->d_cap)
        return 0;
    hipError_t e;
    if (s->d_buf != NULL) {
        hipError_t ef = hipMemsetAsync(s->d_buf, 0, s->d_cap, s->stream);
        if (ef == hipSuccess)
            ef = hipStreamSynchronize(s->stream);
        ptls_mi355x_fault_journal_note("record layer: hipFree device buffer", s->d_buf, s->d_cap);
        const hipError_t ef2 = hipFree(s->d_buf);
        s->d_buf = NULL;
        s->d_cap = 0;
        if (ef != hipSuccess || ef2 != hipSuccess)
            return rl_fail("clearing and freeing the device buffer (growth)", ef != hipSuccess ? ef : ef2);
    }
    s->d_buf = NULL;
    s->d_cap = 0;
    if ((e = hipMalloc((void **)&s->d_buf, s->cap)) != hipSuccess)
        return rl_fail("hipMalloc", e);
    ptls_mi355x_fault_journal_note("record layer: hipMalloc device buffer", s->d_buf, s->cap);
    s->d_cap = s->cap;
    if (rl_trace_on())
        fprintf(stderr, "record layer: slot %p device buffer grown to %zu B\n", (void *)s, s->cap);
    return 0;
}

/* the slot's stream and engine context, created on first use (a synchronous layer only ever uses slot 0) */
static int slot_ready(ptls_mi355x_record_layer_t *rl, rl_slot_t *s)
{
    hipError_t e;
    if (rl_trace_on() && (s->stream == NULL || s->ctx == NULL))
        fprintf(stderr, "record layer: slot %p created\n", (void *)s);
    if (s->stream == NULL && (e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess) {
        s->stream = NULL;
        return rl_fail("hipStreamCreateWithFlags", e);
    }
    if (s->ctx == NULL && (s->ctx = ptls_mi355x_aesgcm_new(rl->key, rl->key_size, 0)) == NULL)
        return rl_msg(ptls_mi355x_last_error());
    return 0;
}

/* the slot's launches are done */
static void slot_sync(rl_slot_t *s)
{
    if (s->stream != NULL)
        RL_DEFER("slot synchronisation", hipStreamSynchronize(s->stream));
}

static void slot_release(rl_slot_t *s)
{
    slot_sync(s);
    if (s->d_buf != NULL) { /* cleared on the slot's stream, before that stream goes */
        RL_DEFER("clearing the device buffer", hipMemsetAsync(s->d_buf, 0, s->d_cap, s->stream));
        RL_DEFER("slot synchronisation", hipStreamSynchronize(s->stream));
        ptls_mi355x_fault_journal_note("record layer: hipFree device buffer", s->d_buf, s->d_cap);
        RL_DEFER("hipFree (device buffer)", hipFree(s->d_buf));
    }
    if (s->stream != NULL)
        RL_DEFER("hipStreamDestroy", hipStreamDestroy(s->stream));
    if (s->h_buf != NULL) {
        memset(s->h_buf, 0, s->cap); /* plaintexts passed through the staging */
        ptls_mi355x_fault_journal_note("record layer: hipHostFree staging (device view)", s->h_dev, s->cap);
        RL_DEFER("hipHostFree (staging)", hipHostFree(s->h_buf));
    }
    free(s->recs);
    ptls_mi355x_aesgcm_free(s->ctx);
    memset(s, 0, sizeof(*s));
}

/* device address of host range [p, p+len) if it lies inside one registered range, else NULL */
static uint8_t *dev_addr(const ptls_mi355x_record_layer_t *rl, const void *p, size_t len)
{
    const uint8_t *b = p;
    for (size_t i = 0; i < rl->nreg; ++i) {
        const rl_region_t *r = rl->reg + i;
        if (b >= r->base && (size_t)(b - r->base) <= r->len && len <= r->len - (size_t)(b - r->base))
            return r->dev + (b - r->base);
    }
    return NULL;
}

ptls_mi355x_record_layer_t *ptls_mi355x_record_layer_new(const void *key, size_t key_size, const void *iv12, uint64_t seq)
{
    if (key_size != 16 && key_size != 32) {
        rl_msg("key size must be 16 or 32");
        return NULL;
    }
    ptls_mi355x_record_layer_t *rl = calloc(1, sizeof(*rl));
    if (rl == NULL)
        return NULL;
    memcpy(rl->key, key, key_size);
    rl->key_size = key_size;
    memcpy(rl->iv, iv12, 12);
    rl->seq = rl->spec_seq = seq;
    rl->zero_copy_bytes = RL_ZERO_COPY_DEFAULT;
    rl->direct_dma = 0;
    rl->coalesce = RL_COALESCE_DEFAULT;
    if ((rl->queue = calloc(RL_TICKETS, sizeof(*rl->queue))) == NULL || slot_ready(rl, &rl->slot[0]) != 0) {
        /* the key is set up now: errors surface here, not at the first window */
        slot_release(&rl->slot[0]);
        memset(rl->key, 0, sizeof(rl->key));
        free(rl->queue);
        free(rl);
        return NULL;
    }
    return rl;
}

/* drops the queued (not yet launched) windows */
static void queue_clear(ptls_mi355x_record_layer_t *rl)
{
    for (size_t i = 0; i < rl->nqueued; ++i)
        free(rl->queue[i].frags);
    memset(rl->queue, 0, RL_TICKETS * sizeof(*rl->queue));
    rl->nqueued = 0;
}

static void layer_dispose(ptls_mi355x_record_layer_t *rl)
{
    memset(rl->key, 0, sizeof(rl->key));
    memset(rl->iv, 0, sizeof(rl->iv));
    free(rl->queue);
    free(rl);
}

void ptls_mi355x_record_layer_free(ptls_mi355x_record_layer_t *rl)
{
    if (rl == NULL)
        return;
    queue_clear(rl); /* queued windows never launched: dropped */
    for (int i = 0; i < RL_SLOTS; ++i) {
        rl_op_t *op = &rl->slot[i].op;
        slot_sync(&rl->slot[i]); /* its own windows finish before their buffers and ranges go */
        if (op->busy) { /* never waited (or not for all its windows): completes here, its results dropped */
            if (!op->done)
                op_release_layers(op);
            op_discard(op);
        }
    }
    while (rl->nreg != 0) /* waits for other layers' windows that still read or write its ranges */
        (void)ptls_mi355x_record_layer_unregister(rl, rl->reg[rl->nreg - 1].base);
    for (int i = 0; i < RL_SLOTS; ++i)
        slot_release(&rl->slot[i]);
    rl->next_ticket = rl->oldest;
    if (rl->inflight != 0) { /* named by windows of other layers: they drop it at their completion */
        rl->zombie = 1;
        return;
    }
    layer_dispose(rl);
}

uint64_t ptls_mi355x_record_layer_get_seq(const ptls_mi355x_record_layer_t *rl) { return rl->seq; }

void ptls_mi355x_record_layer_set_seq(ptls_mi355x_record_layer_t *rl, uint64_t seq) { rl->seq = rl->spec_seq = seq; }

size_t ptls_mi355x_record_layer_pending(const ptls_mi355x_record_layer_t *rl) { return (size_t)(rl->next_ticket - rl->oldest); }

int ptls_mi355x_record_layer_rekey(ptls_mi355x_record_layer_t *rl, const void *key, size_t key_size, const void *iv12)
{
    if (key_size != 16 && key_size != 32)
        return rl_msg("key size must be 16 or 32");
    if (rl->next_ticket != rl->oldest || rl->inflight != 0)
        return rl_msg("rekey with windows outstanding (wait for them first)");
    uint8_t k[32];
    memcpy(k, key, key_size);
    ptls_mi355x_aesgcm_context_t *ctx = ptls_mi355x_aesgcm_new(k, key_size, 0);
    if (ctx == NULL) {
        memset(k, 0, sizeof(k));
        return rl_msg(ptls_mi355x_last_error());
    }
    /* every slot's context holds the old key: slot 0 gets the new one, and the other slots that had a context get one
     * too, now (a rekey keeps the layer's setup, ptls_mi355x_record_layer_reserve, instead of moving a key setup into
     * each slot's next window) */
    int had[RL_SLOTS];
    for (int i = 0; i < RL_SLOTS; ++i) {
        rl_slot_t *s = &rl->slot[i];
        had[i] = s->ctx != NULL;
        if (s->ctx != NULL) {
            if (s->stream != NULL)
                RL_DEFER("rekey: slot synchronisation", hipStreamSynchronize(s->stream));
            ptls_mi355x_aesgcm_free(s->ctx);
            s->ctx = NULL;
        }
    }
    rl->slot[0].ctx = ctx;
    for (int i = 1; i < RL_SLOTS; ++i)
        if (had[i])
            rl->slot[i].ctx = ptls_mi355x_aesgcm_new(k, key_size, 0); /* (NULL: created at the slot's next use) */
    memcpy(rl->key, k, key_size);
    memset(k, 0, sizeof(k));
    rl->key_size = key_size;
    memcpy(rl->iv, iv12, 12);
    rl->seq = rl->spec_seq = 0; /* a new traffic key starts at record 0 (setup_traffic_protection, lib/picotls.c:1217) */
    return 0;
}

int ptls_mi355x_record_layer_reserve(ptls_mi355x_record_layer_t *rl, size_t window_bytes, size_t windows_per_launch)
{
    if (window_bytes == 0 || windows_per_launch == 0 || windows_per_launch > RL_TICKETS)
        return rl_msg("reserve: window bytes and 1..32 windows per launch");
    /* the largest layout a launch of such windows of full-size records takes (copy transport: descriptors, inputs,
     * outputs, statuses, types, delivery parts, every piece 16-aligned), and its descriptors (an open parses up to
     * inlen / 5 + 1).  Staging for the per-record pieces of windows of many small records is not reserved: 128 B a
     * record at the parse bound would be ~6x the window bytes (include/ptls_mi355x.h) */
    const size_t recs = window_bytes / 16384u + 2u;
    const size_t need = windows_per_launch * (2u * window_bytes + recs * 128u) + 4096u;
    for (int i = 0; i < RL_SLOTS; ++i) {
        rl_slot_t *s = &rl->slot[i];
        if (s->op.busy)
            return rl_msg("reserve with windows outstanding");
        if (slot_ready(rl, s) != 0 || reserve_stage(s, need) != 0 || reserve_device(s) != 0 ||
            reserve_recs(s, windows_per_launch * (window_bytes / PTLS_MI355X_TLS_HEADER_SIZE + 1u)) != 0)
            return -1;
        s->copies_prepared = 1;
    }
    return ptls_mi355x_prepare_copies() == 0 ? 0 : rl_msg(ptls_mi355x_last_error());
}

int ptls_mi355x_record_layer_set_direct_dma(ptls_mi355x_record_layer_t *rl, int on)
{
    const int prev = rl->direct_dma;
    rl->direct_dma = on == PTLS_MI355X_RECORD_LAYER_DMA_IN ? on : on != 0;
    return prev;
}

size_t ptls_mi355x_record_layer_set_zero_copy_bytes(ptls_mi355x_record_layer_t *rl, size_t n)
{
    const size_t prev = rl->zero_copy_bytes;
    rl->zero_copy_bytes = n;
    return prev;
}

/*
 * Host ranges registered through the layers, process-wide and counted: the first layer to register a range maps it
 * (hipHostRegister), the others share that mapping, and it is unmapped when the LAST of them lets go.  Two layers
 * share ranges whenever the two directions of a connection use the same socket buffers; with a per-layer "first one
 * owns it" rule the owner's free unmapped a range the other layer still ran windows on, and those kernels then
 * faulted on the unmapped host addresses.  A range inside one mapped here shares that mapping (and counts on it); a
 * range that overlaps one mapped here without lying inside it is refused, since only the mapped part would be reachable
 * and the rest would fault.  A range the application registered itself (hipHostRegister answers already-registered and
 * the table holds nothing over it) is used and never unregistered here.
 */
typedef struct {
    uint8_t *base, *dev; /* mapped here (hipHostRegister) */
    size_t len;
    int refs; /* layer registrations inside it */
} rl_shared_range_t;

#define RL_MAX_SHARED 1024
static pthread_mutex_t g_reg_mu = PTHREAD_MUTEX_INITIALIZER;
static rl_shared_range_t g_reg[RL_MAX_SHARED];
static size_t g_nreg;

/* the table entry of the range starting at base, or NULL (g_reg_mu held) */
static rl_shared_range_t *shared_range(const void *base)
{
    for (size_t i = 0; i < g_nreg; ++i)
        if (g_reg[i].base == base)
            return &g_reg[i];
    return NULL;
}

/* a table entry overlapping [base, base + len) -- one containing it if there is one -- or NULL (g_reg_mu held) */
static rl_shared_range_t *shared_overlap(const uint8_t *base, size_t len)
{
    rl_shared_range_t *any = NULL;
    for (size_t i = 0; i < g_nreg; ++i) {
        rl_shared_range_t *r = &g_reg[i];
        if (!overlaps(r->base, r->len, base, len))
            continue;
        if (base >= r->base && len <= r->len - (size_t)(base - r->base))
            return r;
        any = r;
    }
    return any;
}

/* the fault report's view of the table (fault_journal.c): never blocks, since a thread may hold g_reg_mu */
static void rl_dump_registrations(FILE *f, uint64_t va)
{
    if (pthread_mutex_trylock(&g_reg_mu) != 0) {
        fprintf(f, "  record layer registrations: table busy (held by another thread)\n");
        return;
    }
    fprintf(f, "  record layer registrations: %zu range(s) mapped by the layers\n", g_nreg);
    for (size_t i = 0; i < g_nreg; ++i) {
        const uint64_t b = (uint64_t)(uintptr_t)g_reg[i].base, d = (uint64_t)(uintptr_t)g_reg[i].dev;
        const int in = (va >= b && va - b < g_reg[i].len) || (va >= d && va - d < g_reg[i].len);
        const int next = va >= b + g_reg[i].len && va - (b + g_reg[i].len) < 4096;
        fprintf(f, "    host %p dev %p + %zu, %d ref(s)%s\n", (void *)g_reg[i].base, (void *)g_reg[i].dev, g_reg[i].len,
                g_reg[i].refs, in ? "   <== HOLDS THE FAULTING ADDRESS" : next ? "   <== the fault is the page after it" : "");
    }
    pthread_mutex_unlock(&g_reg_mu);
}

int ptls_mi355x_record_layer_register(ptls_mi355x_record_layer_t *rl, void *base, size_t len)
{
    ptls_mi355x_fault_journal_add_dumper(rl_dump_registrations);
    if (rl->nreg == RL_MAX_REGIONS || base == NULL || len == 0)
        return rl_msg(base == NULL || len == 0 ? "empty range" : "too many ranges");
    for (size_t i = 0; i < rl->nreg; ++i)
        if (rl->reg[i].base == base)
            return rl_msg("range already registered with this layer");
    pthread_mutex_lock(&g_reg_mu);
    rl_shared_range_t *sr = shared_overlap((const uint8_t *)base, len);
    if (sr != NULL) {
        const size_t off = (size_t)((const uint8_t *)base - sr->base);
        if ((const uint8_t *)base < sr->base || len > sr->len - off) {
            pthread_mutex_unlock(&g_reg_mu);
            return rl_msg("range overlaps a registered range without lying inside it (register the enclosing range)");
        }
        ++sr->refs; /* inside a range mapped here (by this or another layer): shared and counted */
        rl->reg[rl->nreg++] = (rl_region_t){(uint8_t *)base, sr->dev + off, len, 1, sr->base};
        pthread_mutex_unlock(&g_reg_mu);
        return 0;
    }
    if (g_nreg == RL_MAX_SHARED) {
        pthread_mutex_unlock(&g_reg_mu);
        return rl_msg("too many registered ranges in the process");
    }
    hipError_t e;
    uint8_t *dev = NULL;
    int owned = 1;
    if ((e = hipHostRegister(base, len, hipHostRegisterMapped)) == hipErrorHostMemoryAlreadyRegistered) {
        (void)hipGetLastError();
        owned = 0; /* registered by the application (or overlapping a range mapped here): used, never unmapped here */
    } else if (e != hipSuccess) {
        pthread_mutex_unlock(&g_reg_mu);
        return rl_fail("hipHostRegister", e);
    }
    if ((e = hipHostGetDevicePointer((void **)&dev, base, 0)) != hipSuccess) {
        if (owned)
            RL_DEFER("hipHostUnregister (after a failed registration)", hipHostUnregister(base));
        pthread_mutex_unlock(&g_reg_mu);
        return rl_fail("hipHostGetDevicePointer", e);
    }
    ptls_mi355x_fault_journal_note(owned ? "record layer: hipHostRegister (device view)"
                                         : "record layer: application-registered range (device view)",
                                   dev, len);
    if (owned) {
        g_reg[g_nreg++] = (rl_shared_range_t){(uint8_t *)base, dev, len, 1};
        rl->reg[rl->nreg++] = (rl_region_t){(uint8_t *)base, dev, len, 1, (uint8_t *)base};
    } else { /* the application's registration: used, not counted, never unmapped here */
        rl->reg[rl->nreg++] = (rl_region_t){(uint8_t *)base, dev, len, 0, NULL};
    }
    pthread_mutex_unlock(&g_reg_mu);
    return 0;
}

int ptls_mi355x_record_layer_unregister(ptls_mi355x_record_layer_t *rl, void *base)
{
    for (size_t i = 0; i < rl->nreg; ++i) {
        if (rl->reg[i].base == base) {
            for (int k = 0; k < RL_SLOTS; ++k) /* no window of this layer still reads the range */
                if (rl->slot[k].stream != NULL)
                    slot_sync(&rl->slot[k]);
            /* nor a window of another layer that names this one (its kernels may address the range): the device */
            if (rl->inflight != 0)
                RL_DEFER("unregister: hipDeviceSynchronize", hipDeviceSynchronize());
            hipError_t e = hipSuccess;
            if (rl->reg[i].owned) { /* holds a reference on the shared entry */
                pthread_mutex_lock(&g_reg_mu);
                rl_shared_range_t *sr = shared_range(rl->reg[i].shared);
                if (sr != NULL && --sr->refs == 0) {
                    ptls_mi355x_fault_journal_note("record layer: hipHostUnregister (device view)", sr->dev, sr->len);
                    e = hipHostUnregister(sr->base);
                    *sr = g_reg[--g_nreg];
                }
                pthread_mutex_unlock(&g_reg_mu);
            }
            rl->reg[i] = rl->reg[--rl->nreg];
            return e == hipSuccess ? 0 : rl_fail("hipHostUnregister", e);
        }
    }
    return rl_msg("range not registered");
}

/* device address of [p, p+len) inside a range registered with any of the layers, else NULL */
static uint8_t *dev_addr_any(ptls_mi355x_record_layer_t *const *layers, size_t n, const void *p, size_t len)
{
    for (size_t i = 0; i < n; ++i) {
        uint8_t *d = dev_addr(layers[i], p, len);
        if (d != NULL)
            return d;
    }
    return NULL;
}

static int overlaps(const void *a, size_t alen, const void *b, size_t blen)
{
    const uint8_t *x = a, *y = b;
    return alen != 0 && blen != 0 && x < y + blen && y < x + alen;
}

static uint32_t be32(const uint8_t *b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; }

/* the layers of one launch share the key size (a launch runs the AES-128 or the AES-256 kernels) */
static int same_key_size(ptls_mi355x_record_layer_t *const *layers, size_t nlayers)
{
    for (size_t l = 1; l < nlayers; ++l)
        if (layers[l]->key_size != layers[0]->key_size) {
            snprintf(rl_err, sizeof(rl_err), "record layer: layer %zu has another key size", l);
            return 0;
        }
    return 1;
}

/* the connections of one session share the key and IV bytes 4..11 (lib/rapido.c:127-133) */
static int same_session(const ptls_mi355x_record_layer_t *a, const ptls_mi355x_record_layer_t *b)
{
    return a->key_size == b->key_size && memcmp(a->key, b->key, a->key_size) == 0 && memcmp(a->iv + 4, b->iv + 4, 8) == 0;
}

/*
 * Groups the op's layers by session (rl_op_t): session 0 is layers[0]'s, led by the launch slot's context; another
 * session's key is its first layer's own slot-0 context (created here if need be).  That layer counts the launch in
 * flight like every layer it names, so its context is not rekeyed or freed under it.
 */
static int op_sessions(rl_slot_t *s)
{
    rl_op_t *op = &s->op;
    const size_t n = op->nlayers;
    uint8_t *mem = calloc(1, n * (sizeof(void *) + 12 + sizeof(uint32_t) + sizeof(void *)));
    if (mem == NULL)
        return rl_msg("out of memory");
    op->sess_ctx = (ptls_mi355x_aesgcm_context_t **)mem;
    ptls_mi355x_record_layer_t **lead = (ptls_mi355x_record_layer_t **)(mem + n * sizeof(void *));
    op->sess_iv = mem + 2 * n * sizeof(void *);
    op->sess_of = (uint32_t *)(op->sess_iv + 12 * n);
    op->nsess = 0;
    for (size_t l = 0; l < n; ++l) {
        ptls_mi355x_record_layer_t *x = op->layers[l];
        size_t k = 0;
        while (k < op->nsess && !same_session(lead[k], x))
            ++k;
        if (k == op->nsess) {
            ptls_mi355x_aesgcm_context_t *c = s->ctx;
            if (k != 0) {
                rl_slot_t *xs = &x->slot[0];
                if (slot_ready(x, xs) != 0)
                    return -1;
                c = xs->ctx;
            }
            lead[k] = x;
            op->sess_ctx[k] = c;
            memcpy(op->sess_iv + 12 * k, x->iv, 12);
            ++op->nsess;
        }
        op->sess_of[l] = (uint32_t)k;
    }
    return 0;
}

/* a new op on layers[0]'s next launch slot: its arrays allocated, NULL when every slot is in flight or on error */
static rl_slot_t *op_begin(ptls_mi355x_record_layer_t *const *layers, size_t nlayers, int is_seal)
{
    ptls_mi355x_record_layer_t *rl = layers[0];
    rl_slot_t *s = &rl->slot[rl->launches % RL_SLOTS];
    if (s->op.busy) {
        rl_msg("all launch slots are in flight (wait for the oldest window first)");
        return NULL;
    }
    if (slot_ready(rl, s) != 0)
        return NULL;
    rl_op_t *op = &s->op;
    memset(op, 0, sizeof(*op));
    /* one allocation: layers | out | capacity | parts | results (outlen, nrec, consumed, alert) */
    const size_t bytes = nlayers * (2 * sizeof(void *) + sizeof(size_t) + sizeof(rl_part_t) + 3 * sizeof(size_t) +
                                    sizeof(int));
    uint8_t *mem = calloc(1, bytes);
    if (mem == NULL) {
        rl_msg("out of memory");
        return NULL;
    }
    op->layers = (ptls_mi355x_record_layer_t **)mem;
    op->out = (void **)(mem + nlayers * sizeof(void *));
    op->capacity = (size_t *)(mem + 2 * nlayers * sizeof(void *));
    op->part = (rl_part_t *)(mem + nlayers * (2 * sizeof(void *) + sizeof(size_t)));
    op->r_outlen = (size_t *)(mem + nlayers * (2 * sizeof(void *) + sizeof(size_t) + sizeof(rl_part_t)));
    op->r_nrec = op->r_outlen + nlayers;
    op->r_cons = op->r_nrec + nlayers;
    op->r_alert = (int *)(op->r_cons + nlayers);
    memcpy(op->layers, layers, nlayers * sizeof(void *));
    op->nlayers = nlayers;
    op->is_seal = is_seal;
    return s;
}

static void op_discard(rl_op_t *op)
{
    free(op->h2d);
    free(op->layers);
    free(op->sess_ctx);
    memset(op, 0, sizeof(*op));
}

/* 1 when layers[l] appeared earlier in the op (a layer given several times counts once) */
static int repeated(const rl_op_t *op, size_t l)
{
    for (size_t m = 0; m < l; ++m)
        if (op->layers[m] == op->layers[l])
            return 1;
    return 0;
}

/*
 * Launched: the op takes its lead layer's next launch slot and holds `nwin` windows from ticket0 on (a submit's one
 * window, or the layer's coalesced windows, whose tickets were handed out at their submits); every layer it names
 * counts it in flight.
 */
static void op_commit(ptls_mi355x_record_layer_t *rl, rl_slot_t *s, uint64_t ticket0, size_t nwin, int coalesced)
{
    s->op.busy = 1;
    s->op.ticket = ticket0;
    s->op.nwin = nwin;
    s->op.coalesced = coalesced;
    for (uint64_t t = ticket0; t < ticket0 + nwin; ++t)
        rl->ticket_slot[t % RL_TICKETS] = (int8_t)(s - rl->slot);
    ++rl->launches;
    for (size_t l = 0; l < s->op.nlayers; ++l)
        if (!repeated(&s->op, l))
            ++s->op.layers[l]->inflight;
}

/* a submit's window: the lead layer's next ticket */
static void op_commit_window(rl_slot_t *s, uint64_t *ticket)
{
    ptls_mi355x_record_layer_t *rl = s->op.layers[0];
    const uint64_t t = rl->next_ticket++;
    op_commit(rl, s, t, 1, 0);
    if (ticket != NULL)
        *ticket = t;
}

/*
 * The op is complete (waited, or dropped with its lead layer): every layer it names counts it out.  A layer with no
 * window left in flight has no speculative receive position ahead of its delivered one (spec_seq = seq: a window
 * that failed or came back STALE out of order leaves nothing to follow), and a layer freed meanwhile goes now.
 */
static void op_release_layers(rl_op_t *op)
{
    for (size_t l = 0; l < op->nlayers; ++l) {
        ptls_mi355x_record_layer_t *x = op->layers[l];
        if (repeated(op, l) || x->inflight == 0)
            continue;
        if (--x->inflight == 0) {
            if (x->nqueued == 0)
                x->spec_seq = x->seq;
            if (x->zombie && x != op->layers[0])
                layer_dispose(x);
        }
    }
}

/* a copy list of up to n entries (dma windows: one allocation for both directions) */
static int op_copies(rl_op_t *op, size_t n)
{
    if ((op->h2d = calloc(2 * n, sizeof(rl_copy_t))) == NULL)
        return rl_msg("out of memory");
    op->d2h = op->h2d + n;
    return 0;
}

/* host -> device copy of [src, src + n) to dst, merged with the previous one when both are contiguous */
static void op_h2d(rl_op_t *op, void *dst, const void *src, size_t n)
{
    rl_copy_t *c = op->nh2d != 0 ? &op->h2d[op->nh2d - 1] : NULL;
    if (c != NULL && (const uint8_t *)c->src + c->n == (const uint8_t *)src && (uint8_t *)c->dst + c->n == (uint8_t *)dst)
        c->n += n;
    else if (n != 0)
        op->h2d[op->nh2d++] = (rl_copy_t){dst, src, n};
}

/*
 * H2D, the launch, D2H, everything on the slot's stream.  zero-copy: the kernel works on the pinned staging; copy: the
 * staging moves to the device buffer and back; mapped: descriptors from the staging, data in place in registered host
 * memory; dma: descriptors and the registered inputs to the device buffer, the outputs back into the registered
 * ranges (statuses and types of an open into the staging).
 */
static int op_launch(rl_slot_t *s, const uint8_t *src_base, uint8_t *dst_base)
{
    rl_op_t *op = &s->op;
    uint8_t *base = op->zero_copy ? s->h_dev : s->d_buf;
    const int mapped = op->direct && !op->dma;
    const uint8_t *src = op->dma_in ? s->d_buf + op->off_src : mapped ? src_base : base + op->off_src;
    uint8_t *dst = op->deliver ? s->d_buf + op->off_dst : mapped ? dst_base : base + op->off_dst;
    const uint32_t *conn = op->nlayers > 1 ? (const uint32_t *)(base + up16(op->nrec * sizeof(ptls_mi355x_tls_record_t))) : NULL;
    const uint32_t *kidx = op->nsess > 1 ? (const uint32_t *)(base + op->off_kidx) : NULL;
    hipError_t e;
    int rc;
    /* the runtime's one-time copy setup, before the first copy rather than inside some later window's */
    if ((!op->zero_copy || op->nh2d != 0 || op->nd2h != 0) && !s->copies_prepared) {
        if (ptls_mi355x_prepare_copies() != 0)
            return rl_msg(ptls_mi355x_last_error());
        s->copies_prepared = 1;
    }
    const int tr = rl_trace_on();
    double t0 = tr ? rl_now() : 0;
    if (!op->zero_copy &&
        (e = hipMemcpyAsync(s->d_buf, s->h_buf, op->dma ? op->off_src : op->off_src + op->srcbytes, hipMemcpyHostToDevice,
                            s->stream)) != hipSuccess)
        return rl_fail("H2D", e);
    if (tr)
        rl_slow("the staging H2D", t0);
    for (size_t i = 0; i < op->nh2d; ++i) {
        t0 = tr ? rl_now() : 0;
        if ((e = hipMemcpyAsync(op->h2d[i].dst, op->h2d[i].src, op->h2d[i].n, hipMemcpyHostToDevice, s->stream)) != hipSuccess)
            return rl_fail("H2D", e);
        if (tr)
            rl_slow("an input H2D", t0);
    }
    t0 = tr ? rl_now() : 0;
    if (kidx != NULL && op->is_seal) /* several sessions: one multi-key launch */
        rc = ptls_mi355x_tls_seal_records_multikey(op->sess_ctx, op->sess_iv, op->nsess,
                                                   (const ptls_mi355x_tls_record_t *)base, kidx, conn, op->nrec, src, dst,
                                                   s->stream);
    else if (kidx != NULL)
        rc = ptls_mi355x_tls_open_records_multikey(op->sess_ctx, op->sess_iv, op->nsess,
                                                   (const ptls_mi355x_tls_record_t *)base, kidx, conn, op->nrec, src, dst,
                                                   (uint32_t *)(base + op->off_st), base + op->off_ty, 0, s->stream);
    else if (op->is_seal)
        rc = ptls_mi355x_tls_seal_records_multi(s->ctx, op->layers[0]->iv, (const ptls_mi355x_tls_record_t *)base, conn,
                                                op->nrec, src, dst, s->stream);
    else /* every record verified independently; the stop at a connection's first failure is the host loop in wait */
        rc = ptls_mi355x_tls_open_records_multi(s->ctx, op->layers[0]->iv, (const ptls_mi355x_tls_record_t *)base, conn,
                                                op->nrec, src, dst, (uint32_t *)(base + op->off_st), base + op->off_ty,
                                                s->stream);
    if (rc == 0 && op->deliver)
        rc = ptls_mi355x_tls_deliver_records(s->ctx, (const ptls_mi355x_tls_record_t *)base, (uint32_t *)(base + op->off_st),
                                             base + op->off_ty, (const ptls_mi355x_tls_deliver_t *)(base + op->off_dp),
                                             op->nlayers, op->max_part, s->stream);
    if (rc != 0)
        return rl_msg(ptls_mi355x_last_error());
    if (tr)
        rl_slow("the launch", t0);
    for (size_t i = 0; i < op->nd2h; ++i) {
        t0 = tr ? rl_now() : 0;
        if ((e = hipMemcpyAsync(op->d2h[i].dst, op->d2h[i].src, op->d2h[i].n, hipMemcpyDeviceToHost, s->stream)) != hipSuccess)
            return rl_fail("D2H", e);
        if (tr)
            rl_slow("an output D2H", t0);
    }
    t0 = tr ? rl_now() : 0;
    if (!op->zero_copy && !(op->dma && op->is_seal)) {
        const size_t from = op->dma ? op->off_st : op->off_dst;
        const size_t to = op->is_seal ? op->off_dst + op->dstbytes : op->off_ty + op->nrec;
        if (to > from &&
            (e = hipMemcpyAsync(s->h_buf + from, s->d_buf + from, to - from, hipMemcpyDeviceToHost, s->stream)) != hipSuccess)
            return rl_fail("D2H", e);
    }
    if (tr)
        rl_slow("the staging D2H", t0);
    return 0;
}

/* after a failed launch or wait: nothing of the window's plaintext stays in the staging */
static void op_scrub(rl_slot_t *s)
{
    rl_op_t *op = &s->op;
    slot_sync(s);
    if (!op->direct && s->h_buf != NULL) {
        const size_t end = op->is_seal ? op->off_dst + op->dstbytes : op->off_st;
        if (end > op->off_src && end <= s->cap)
            memset(s->h_buf + op->off_src, 0, end - op->off_src);
    }
}

/* ---------------------------------------------------------------------------------------------------- seal ---- */

/*
 * Plans, stages and launches a seal op on slot s (op_begin done): layers[l] seals frags[l] into out[l]; a layer given
 * again takes its next window behind the earlier one.  The layers' seq advance past their records.  -1: nothing
 * launched, the op discarded.
 */
static int seal_build(rl_slot_t *s, ptls_mi355x_record_layer_t *const *layers, size_t nlayers,
                      const ptls_mi355x_iovec_t *const *frags, const size_t *nfrags, uint8_t type, void *const *out,
                      const size_t *capacity)
{
    rl_op_t *op = &s->op;
    const int limited = type == 23; /* ptls_send's key-update check; handshake messages are pushed past it */
    size_t nrec = 0, srcbytes = 0, wire = 0;
    for (size_t l = 0; l < nlayers; ++l) {
        rl_part_t *p = &op->part[l];
        uint64_t sq = layers[l]->seq;
        for (size_t m = 0; m < l; ++m) /* a layer given again: its next window, behind the earlier one */
            if (layers[m] == layers[l])
                sq = op->part[m].seq0 + op->part[m].nrec;
        p->seq0 = sq;
        op->out[l] = out[l];
        op->capacity[l] = capacity[l];
        for (size_t f = 0; f < nfrags[l]; ++f) {
            if (limited && sq >= PTLS_MI355X_RECORD_LAYER_SEQ_LIMIT) {
                p->stopped = 1;
                break;
            }
            size_t w = 0;
            const size_t n = ptls_mi355x_tls_plan_send(frags[l][f].len, type, &sq, 0, 0, NULL, 0, &w);
            sq += n;
            p->nrec += n;
            p->wire += w;
            ++p->nfrags;
            srcbytes += frags[l][f].len;
        }
        if (p->wire > capacity[l]) {
            snprintf(rl_err, sizeof(rl_err), "record layer: %zu wire bytes exceed the output capacity %zu (layer %zu)",
                     p->wire, capacity[l], l);
            op_discard(op);
            return -1;
        }
        nrec += p->nrec;
        wire += p->wire;
    }
    op->nrec = nrec;
    if (nrec == 0) /* nothing to launch (empty or all at the limit): completes at its wait */
        return 0;
    if (reserve_recs(s, nrec) != 0)
        goto Fail;
    /* direct: every sealed fragment and every output in registered ranges; addressed from the lowest of each.  In
     * place (mapped) only when no fragment overlaps an output: the kernel would overwrite fragment bytes another
     * workgroup still reads.  dma windows copy the fragments to the device first, so overlap is harmless there. */
    uint8_t *src_base = NULL, *dst_base = NULL;
    int direct = 1, overlap = 0;
    size_t nfr = 0;
    for (size_t l = 0; direct && l < nlayers; ++l) {
        uint8_t *d = op->part[l].wire != 0 ? dev_addr_any(layers, nlayers, out[l], op->part[l].wire) : NULL;
        if (op->part[l].wire != 0 && d == NULL)
            direct = 0;
        else if (d != NULL && (dst_base == NULL || d < dst_base))
            dst_base = d;
        for (size_t f = 0; direct && f < op->part[l].nfrags; ++f) {
            ++nfr;
            if (frags[l][f].len == 0)
                continue;
            if ((d = dev_addr_any(layers, nlayers, frags[l][f].base, frags[l][f].len)) == NULL)
                direct = 0;
            else if (src_base == NULL || d < src_base)
                src_base = d;
            for (size_t m = 0; m < nlayers; ++m)
                overlap |= overlaps(frags[l][f].base, frags[l][f].len, out[m], op->part[m].wire);
        }
    }
    const int dma = direct && layers[0]->direct_dma == 1;
    /* DMA in: the fragments copied into device memory (one copy per contiguous run) first, the wire written in place */
    const int dma_in = direct && layers[0]->direct_dma == PTLS_MI355X_RECORD_LAYER_DMA_IN;
    if (direct && !dma && !dma_in && overlap)
        direct = 0;
    const int packed = !direct || dma; /* fragments and records back to back in the staging / device layout */
    op->direct = direct;
    op->dma = dma;
    op->dma_in = dma_in;
    if (op_sessions(s) != 0)
        goto Fail;
    const size_t off_conn = up16(nrec * sizeof(ptls_mi355x_tls_record_t));
    op->off_kidx = off_conn + (nlayers > 1 ? up16(nrec * 4) : 0);
    op->off_src = op->off_kidx + (op->nsess > 1 ? up16(nrec * 4) : 0);
    op->srcbytes = packed || dma_in ? srcbytes : 0;
    op->off_dst = op->off_src + up16(op->srcbytes);
    op->dstbytes = packed ? wire : 0;
    const size_t total = op->off_dst + up16(op->dstbytes);
    op->zero_copy = (direct && !dma) || (!direct && total <= layers[0]->zero_copy_bytes);
    if (reserve_stage(s, total) != 0 || ((!op->zero_copy || dma_in) && reserve_device(s) != 0) ||
        ((dma || dma_in) && op_copies(op, nfr + nlayers) != 0))
        goto Fail;
    /* descriptors (offsets relative to the src / dst bases), the per-record IV differences and, unless direct, the
     * fragments back to back */
    uint32_t *conn = (uint32_t *)(s->h_buf + off_conn), *kidx = (uint32_t *)(s->h_buf + op->off_kidx);
    size_t k = 0, src_off = 0, dst_off = 0;
    for (size_t l = 0; l < nlayers; ++l) {
        rl_part_t *p = &op->part[l];
        uint64_t sq = p->seq0;
        if (!packed && p->wire != 0)
            dst_off = (size_t)(dev_addr_any(layers, nlayers, out[l], p->wire) - dst_base);
        if (dma && p->wire != 0) /* the layer's wire records, back to the caller's output in one copy */
            op->d2h[op->nd2h++] = (rl_copy_t){out[l], s->d_buf + op->off_dst + dst_off, p->wire};
        /* BE32(cid) ^ IV[0..3] of its session's first layer = layer l's */
        const uint32_t sess = op->sess_of[l], cid = be32(layers[l]->iv) ^ be32(op->sess_iv + 12 * sess);
        const size_t k0 = k;
        for (size_t f = 0; f < p->nfrags; ++f) {
            const ptls_mi355x_iovec_t *fr = &frags[l][f];
            size_t w = 0;
            if (!packed && !dma_in && fr->len != 0)
                src_off = (size_t)(dev_addr_any(layers, nlayers, fr->base, fr->len) - src_base);
            k += ptls_mi355x_tls_plan_send(fr->len, type, &sq, src_off, dst_off, s->recs + k, nrec - k, &w);
            if (packed || dma_in) {
                if (dma || dma_in)
                    op_h2d(op, s->d_buf + op->off_src + src_off, fr->base, fr->len);
                else if (fr->len != 0)
                    memcpy(s->h_buf + op->off_src + src_off, fr->base, fr->len);
                src_off += fr->len;
            }
            dst_off += w;
        }
        if (nlayers > 1)
            for (size_t i = k0; i < k; ++i)
                conn[i] = cid;
        if (op->nsess > 1)
            for (size_t i = k0; i < k; ++i)
                kidx[i] = sess;
    }
    memcpy(s->h_buf, s->recs, nrec * sizeof(ptls_mi355x_tls_record_t));
    if (op_launch(s, src_base, dst_base) != 0) {
        op_scrub(s);
        goto Fail;
    }
    for (size_t l = 0; l < nlayers; ++l) /* the records have their seq: the next window continues behind them */
        layers[l]->seq = op->part[l].seq0 + op->part[l].nrec;
    return 0;
Fail:
    op_discard(op);
    return -1;
}

/* --------------------------------------------------------------------------------------------------- open ---- */

/*
 * Parses, stages and launches an open op on slot s (op_begin done): layers[l] opens the complete records at the start
 * of in[l] into out[l], from its speculative seq (a layer given again: behind its earlier window).  resync: a layer
 * with nothing in flight or queued first takes spec_seq = seq.  -1: nothing launched, the op discarded.
 */
static int open_build(rl_slot_t *s, ptls_mi355x_record_layer_t *const *layers, size_t nlayers, const void *const *in,
                      const size_t *inlen, void *const *out, const size_t *capacity, size_t *parsed, int any_type,
                      int resync)
{
    rl_op_t *op = &s->op;
    op->any_type = any_type;
    for (size_t l = 0; resync && l < nlayers; ++l) /* nothing in flight: the next record to submit is the next to deliver */
        if (layers[l]->inflight == 0 && layers[l]->nqueued == 0)
            layers[l]->spec_seq = layers[l]->seq;
    size_t max = 0, nrec = 0, srcbytes = 0, ptbytes = 0, slots16 = 0;
    for (size_t l = 0; l < nlayers; ++l) /* a record takes at least 5 wire bytes */
        max += any_type ? 1 : inlen[l] / PTLS_MI355X_TLS_HEADER_SIZE + 1;
    if (reserve_recs(s, max) != 0)
        goto Fail;
    /* the complete application_data records at the start of every input, offsets local to it for now */
    for (size_t l = 0; l < nlayers; ++l) {
        rl_part_t *p = &op->part[l];
        const size_t lmax = any_type ? 1 : inlen[l] / PTLS_MI355X_TLS_HEADER_SIZE + 1; /* its own budget */
        uint64_t seq = layers[l]->spec_seq;
        for (size_t m = 0; m < l; ++m) /* a layer given again: its next window, behind the earlier one */
            if (layers[m] == layers[l])
                seq = op->part[m].seq0 + op->part[m].n;
        p->seq0 = seq;
        p->k0 = nrec;
        op->out[l] = out[l];
        op->capacity[l] = capacity[l];
        p->perr = ptls_mi355x_tls_parse_records((const uint8_t *)in[l], inlen[l], 0, &seq, 0, s->recs + nrec, lmax, &p->n,
                                                &p->cons);
        if (p->n != 0) {
            const ptls_mi355x_tls_record_t *last = s->recs + nrec + p->n - 1;
            p->ptbytes = last->dst + (last->len >= 16u ? last->len - 16u : 0u);
        }
        for (size_t i = nrec; i < nrec + p->n; ++i)
            p->slots16 += up16(s->recs[i].len >= 16u ? s->recs[i].len - 16u : 0u);
        slots16 += p->slots16;
        p->nrec = p->n;
        nrec += p->n;
        srcbytes += up16(p->cons);
        ptbytes += up16(p->ptbytes);
        if (parsed != NULL)
            parsed[l] = p->cons;
    }
    op->nrec = nrec;
    if (nrec == 0)
        return 0;
    /* direct: every input and every plaintext buffer (at least as large as its slots) in registered ranges, and no
     * input overlapping a plaintext buffer (slots are packed tighter than records: an in-place open would overwrite
     * ciphertext another workgroup still reads) */
    uint8_t *src_base = NULL, *dst_base = NULL;
    int direct = 1, overlap = 0;
    for (size_t l = 0; direct && l < nlayers; ++l) {
        const rl_part_t *p = &op->part[l];
        if (p->n == 0)
            continue;
        uint8_t *di = dev_addr_any(layers, nlayers, in[l], p->cons);
        uint8_t *dout = capacity[l] >= p->ptbytes ? dev_addr_any(layers, nlayers, out[l], p->ptbytes) : NULL;
        if (di == NULL || dout == NULL) {
            direct = 0;
            break;
        }
        for (size_t m = 0; m < nlayers; ++m)
            overlap |= overlaps(in[l], p->cons, out[m], op->part[m].ptbytes);
        if (src_base == NULL || di < src_base)
            src_base = di;
        if (dst_base == NULL || dout < dst_base)
            dst_base = dout;
    }
    /* (the input reaches the device before any output is written) */
    const int dma = direct && layers[0]->direct_dma == 1;
    size_t max_part = 0;
    for (size_t l = 0; l < nlayers; ++l)
        max_part = op->part[l].n > max_part ? op->part[l].n : max_part;
    /* mapped: the records read in place, their slots in device memory, the delivery kernel writes each plaintext once
     * to its final place in the caller's buffer; overlapping buffers are harmless then */
    const int deliver = direct && !dma && max_part <= PTLS_MI355X_DELIVER_MAX;
    if (direct && !dma && !deliver && overlap)
        direct = 0;
    /* DMA in: the records copied into device memory (one copy per contiguous run of inputs) before the launch */
    const int dma_in = deliver && layers[0]->direct_dma == PTLS_MI355X_RECORD_LAYER_DMA_IN;
    const int packed = !direct || dma;
    op->direct = direct;
    op->dma = dma;
    op->deliver = deliver;
    op->dma_in = dma_in;
    op->max_part = max_part;
    if (op_sessions(s) != 0)
        goto Fail;
    const size_t off_conn = up16(nrec * sizeof(ptls_mi355x_tls_record_t));
    op->off_kidx = off_conn + (nlayers > 1 ? up16(nrec * 4) : 0);
    op->off_src = op->off_kidx + (op->nsess > 1 ? up16(nrec * 4) : 0);
    op->srcbytes = packed || dma_in ? srcbytes : 0;
    op->off_dst = op->off_src + op->srcbytes;
    op->dstbytes = packed ? ptbytes : deliver ? slots16 : 0;
    op->off_st = op->off_dst + op->dstbytes;
    op->off_ty = op->off_st + up16(nrec * 4);
    op->off_dp = op->off_ty + up16(nrec);
    const size_t total = op->off_dp + (deliver ? nlayers * sizeof(ptls_mi355x_tls_deliver_t) : 0);
    op->zero_copy = (direct && !dma) || (!direct && total <= layers[0]->zero_copy_bytes);
    if (reserve_stage(s, total) != 0 || ((!op->zero_copy || deliver) && reserve_device(s) != 0) ||
        ((dma || dma_in) && op_copies(op, nlayers) != 0))
        goto Fail;
    ptls_mi355x_tls_deliver_t *dp = (ptls_mi355x_tls_deliver_t *)(s->h_buf + op->off_dp);
    uint32_t *conn = (uint32_t *)(s->h_buf + off_conn), *kidx = (uint32_t *)(s->h_buf + op->off_kidx);
    for (size_t l = 0, so = 0, dso = 0; l < nlayers; ++l) {
        rl_part_t *p = &op->part[l];
        if (deliver)
            dp[l] = (ptls_mi355x_tls_deliver_t){s->d_buf + op->off_dst, NULL, 0u, (uint32_t)p->k0, 0u, 0u, 0u};
        if (p->n == 0)
            continue;
        if (deliver) {
            if (dma_in) { /* the input's packed place in device memory */
                p->src_add = so;
                op_h2d(op, s->d_buf + op->off_src + so, in[l], p->cons);
                so += up16(p->cons);
            } else {
                p->src_add = (uint64_t)(dev_addr_any(layers, nlayers, in[l], p->cons) - src_base);
            }
            p->dst_add = dso;
            /* every slot 16-aligned in the device buffer (parse_records packed them): the delivery kernel's copies
             * of whole-block plaintexts then run on 16-byte accesses */
            uint64_t at = 0;
            for (size_t i = p->k0; i < p->k0 + p->n; ++i) {
                s->recs[i].dst = at;
                at += up16(s->recs[i].len >= 16u ? s->recs[i].len - 16u : 0u);
            }
            dp[l] = (ptls_mi355x_tls_deliver_t){s->d_buf + op->off_dst, dev_addr_any(layers, nlayers, out[l], p->ptbytes),
                                                 capacity[l], (uint32_t)p->k0, (uint32_t)p->n, (uint32_t)any_type, 0u};
            dso += p->slots16;
        } else if (!packed) {
            p->src_add = (uint64_t)(dev_addr_any(layers, nlayers, in[l], p->cons) - src_base);
            p->dst_add = (uint64_t)(dev_addr_any(layers, nlayers, out[l], p->ptbytes) - dst_base);
        } else {
            p->src_add = so;
            p->dst_add = dso;
            if (dma) { /* the records in, the plaintext slots straight back into the caller's buffer */
                op_h2d(op, s->d_buf + op->off_src + so, in[l], p->cons);
                op->d2h[op->nd2h++] = (rl_copy_t){out[l], s->d_buf + op->off_dst + dso, p->ptbytes};
            } else {
                memcpy(s->h_buf + op->off_src + so, in[l], p->cons);
            }
            so += up16(p->cons);
            dso += up16(p->ptbytes);
        }
        const uint32_t sess = op->sess_of[l], cid = be32(layers[l]->iv) ^ be32(op->sess_iv + 12 * sess);
        for (size_t i = p->k0; i < p->k0 + p->n; ++i) {
            s->recs[i].src += p->src_add;
            s->recs[i].dst += p->dst_add;
            if (nlayers > 1)
                conn[i] = cid;
            if (op->nsess > 1)
                kidx[i] = sess;
        }
    }
    memcpy(s->h_buf, s->recs, nrec * sizeof(ptls_mi355x_tls_record_t));
    if (op_launch(s, src_base, dst_base) != 0) {
        op_scrub(s);
        goto Fail;
    }
    for (size_t l = 0; l < nlayers; ++l) /* speculative: the next window's records follow these */
        layers[l]->spec_seq = op->part[l].seq0 + op->part[l].n;
    return 0;
Fail:
    op_discard(op);
    return -1;
}

/* ------------------------------------------------------------------------------------------- coalescing ---- */

/* 1 while a launch of this layer's own slots is still running on the GPU */
static int rl_busy(ptls_mi355x_record_layer_t *rl)
{
    int busy = 0;
    for (int i = 0; i < RL_SLOTS && !busy; ++i) {
        const rl_slot_t *s = &rl->slot[i];
        busy = s->op.busy && !s->op.done && s->op.nrec != 0 && hipStreamQuery(s->stream) == hipErrorNotReady;
    }
    (void)hipGetLastError(); /* (hipErrorNotReady is an answer, not an error to leave behind) */
    return busy;
}

/*
 * How many queued windows go out now (0: none): the layer's outstanding windows spread over its RL_SLOTS launch
 * slots, so a connection that keeps w windows outstanding launches groups of ceil(w / 4) -- one window per launch up
 * to 4 outstanding, as without coalescing, 4 per launch at 16 -- with up to 4 launches in flight; a queue whose layer
 * has nothing running goes at once (no window waits for company that may not come); a corked one only when full.
 */
static size_t queue_due(ptls_mi355x_record_layer_t *rl)
{
    if (rl->nqueued == 0)
        return 0;
    const size_t cap = rl->coalesce > 1 ? rl->coalesce : 1;
    if (rl->corked)
        return rl->nqueued >= cap ? cap : 0;
    const size_t outstanding = (size_t)(rl->next_ticket - rl->oldest);
    size_t group = (outstanding + RL_SLOTS - 1) / RL_SLOTS;
    group = group < 1 ? 1 : group > cap ? cap : group;
    if (rl->nqueued >= group)
        return group;
    return rl_busy(rl) ? 0 : rl->nqueued;
}

/* the queue's due groups, while launch slots are free */
static int queue_drain(ptls_mi355x_record_layer_t *rl)
{
    int rc = 0;
    size_t n;
    while (!rl->slot[rl->launches % RL_SLOTS].op.busy && (n = queue_due(rl)) != 0)
        rc |= rl_flush_n(rl, n);
    return rc;
}

/* windows whose launch failed: their waits report -1 (seq stays past them: no nonce is used twice) */
static void op_fail_windows(ptls_mi355x_record_layer_t *rl, rl_slot_t *s, uint64_t ticket0, size_t n, int is_seal)
{
    rl_op_t *op = &s->op;
    memset(op, 0, sizeof(*op)); /* names no layer: nothing counted in flight, nothing to finish */
    op->is_seal = is_seal;
    op->done = op->failed = 1;
    op_commit(rl, s, ticket0, n, 1);
}

/*
 * Launches the first `n` of the layer's queued windows (all: n = 0) as ONE op (each window a part of the layer given
 * again), when a launch slot is free (else they stay queued: every slot is in flight, and the next wait frees one).
 * The seq / spec_seq the windows took at their submit is kept: the build re-derives the same values from the first
 * window's.  0: launched or left queued; -1: the launch failed (its windows' waits report it).
 */
static int rl_flush_n(ptls_mi355x_record_layer_t *rl, size_t n)
{
    if (n == 0 || n > rl->nqueued)
        n = rl->nqueued;
    if (n == 0 || rl->slot[rl->launches % RL_SLOTS].op.busy)
        return 0;
    /* one op seals one content type (one direction): the group ends where the queue's next window differs */
    const int is_seal = rl->queue[0].is_seal;
    const uint8_t type = rl->queue[0].type;
    for (size_t i = 1; i < n; ++i)
        if (rl->queue[i].is_seal != is_seal || rl->queue[i].type != type) {
            n = i;
            break;
        }
    ptls_mi355x_record_layer_t *layers[RL_TICKETS];
    const ptls_mi355x_iovec_t *frags[RL_TICKETS];
    size_t nfrags[RL_TICKETS], capacity[RL_TICKETS], inlen[RL_TICKETS], parsed[RL_TICKETS];
    void *out[RL_TICKETS];
    const void *in[RL_TICKETS];
    for (size_t i = 0; i < n; ++i) {
        const struct rl_queued *q = &rl->queue[i];
        layers[i] = rl;
        frags[i] = q->frags;
        nfrags[i] = q->nfrags;
        in[i] = q->in;
        inlen[i] = q->inlen;
        out[i] = q->out;
        capacity[i] = q->capacity;
    }
    const uint64_t ticket0 = rl->queue_ticket;
    rl_slot_t *s = op_begin(layers, n, is_seal);
    int rc = -1;
    if (s != NULL) {
        const size_t cap = rl->coalesce > 1 ? rl->coalesce : 1;
        s->grow = (cap + n - 1) / n;
        if (is_seal) {
            const uint64_t keep = rl->seq;
            rl->seq = rl->queue[0].seq0;
            rc = seal_build(s, layers, n, frags, nfrags, type, out, capacity);
            rl->seq = keep;
        } else {
            const uint64_t keep = rl->spec_seq; /* (a window stopped meanwhile may have reset it: kept as it is) */
            rl->spec_seq = rl->queue[0].seq0;
            rc = open_build(s, layers, n, in, inlen, out, capacity, parsed, 0, 0);
            rl->spec_seq = keep;
        }
        s->grow = 0;
    }
    for (size_t i = 0; i < n; ++i) /* the launched windows leave the queue */
        free(rl->queue[i].frags);
    memmove(rl->queue, rl->queue + n, (rl->nqueued - n) * sizeof(*rl->queue));
    memset(rl->queue + rl->nqueued - n, 0, n * sizeof(*rl->queue));
    rl->nqueued -= n;
    rl->queue_ticket += n;
    if (rc == 0) {
        op_commit(rl, s, ticket0, n, 1);
        return 0;
    }
    if (s == NULL)
        s = &rl->slot[rl->launches % RL_SLOTS]; /* (free: checked above) */
    op_fail_windows(rl, s, ticket0, n, is_seal);
    return -1;
}

static int rl_flush(ptls_mi355x_record_layer_t *rl)
{
    int rc = 0;
    while (rl->nqueued != 0 && !rl->slot[rl->launches % RL_SLOTS].op.busy)
        rc |= rl_flush_n(rl, rl->coalesce > 1 ? rl->coalesce : 1);
    return rc;
}

/* ptls_send's record count and wire bytes for frags from seq (stopping at the 2^24 limit for application data) */
static size_t plan_window(const ptls_mi355x_iovec_t *frags, size_t nfrags, uint8_t type, uint64_t *seq, size_t *wire)
{
    size_t nrec = 0;
    *wire = 0;
    for (size_t f = 0; f < nfrags; ++f) {
        if (type == 23 && *seq >= PTLS_MI355X_RECORD_LAYER_SEQ_LIMIT)
            break;
        size_t w = 0;
        const size_t k = ptls_mi355x_tls_plan_send(frags[f].len, type, seq, 0, 0, NULL, 0, &w);
        *seq += k;
        nrec += k;
        *wire += w;
    }
    return nrec;
}

/* the complete application_data records at the start of in (ptls_mi355x_tls_parse_records' walk, counting only) */
static size_t count_records(const uint8_t *in, size_t inlen, size_t *consumed)
{
    size_t off = 0, n = 0;
    while (inlen - off >= PTLS_MI355X_TLS_HEADER_SIZE) {
        const uint8_t *h = in + off;
        const uint32_t reclen = (uint32_t)h[3] << 8 | h[4];
        if (h[0] != 23 || reclen > PTLS_MI355X_TLS_MAX_RECORD || inlen - off < PTLS_MI355X_TLS_HEADER_SIZE + (size_t)reclen)
            break;
        off += PTLS_MI355X_TLS_HEADER_SIZE + reclen;
        ++n;
    }
    *consumed = off;
    return n;
}

/* a single-layer window into the layer's queue; launched at once when nothing of the layer is running */
static int queue_window(ptls_mi355x_record_layer_t *rl, int is_seal, uint8_t type, const ptls_mi355x_iovec_t *frags,
                        size_t nfrags, const void *in, size_t inlen, void *out, size_t capacity, size_t *parsed,
                        uint64_t *ticket)
{
    if (rl->next_ticket - rl->oldest >= RL_TICKETS)
        return rl_msg("all windows are outstanding (wait for the oldest first)");
    /* a window of another content type starts a group of its own (rl_flush_n); the queued ones go out first if they can */
    if (rl->nqueued != 0 && (rl->queue[rl->nqueued - 1].is_seal != is_seal || rl->queue[rl->nqueued - 1].type != type) &&
        rl_flush(rl) != 0)
        return -1;
    if (rl->nqueued != 0 && rl->queue[0].is_seal != is_seal) /* not launched (no free slot): cannot queue behind it */
        return rl_msg("windows of the other direction are queued and every launch slot is in flight");
    struct rl_queued *q = &rl->queue[rl->nqueued];
    memset(q, 0, sizeof(*q));
    if (is_seal) {
        uint64_t sq = rl->seq;
        size_t wire = 0;
        plan_window(frags, nfrags, type, &sq, &wire);
        if (wire > capacity) {
            snprintf(rl_err, sizeof(rl_err), "record layer: %zu wire bytes exceed the output capacity %zu (layer 0)", wire,
                     capacity);
            return -1;
        }
        if (nfrags != 0 && (q->frags = malloc(nfrags * sizeof(*frags))) == NULL)
            return rl_msg("out of memory");
        if (nfrags != 0)
            memcpy(q->frags, frags, nfrags * sizeof(*frags));
        q->nfrags = nfrags;
        q->seq0 = rl->seq;
        rl->seq = sq; /* the records take their seq at submit */
    } else {
        if (rl->inflight == 0 && rl->nqueued == 0)
            rl->spec_seq = rl->seq;
        size_t cons = 0;
        const size_t n = count_records((const uint8_t *)in, inlen, &cons);
        q->in = in;
        q->inlen = inlen;
        q->seq0 = rl->spec_seq;
        rl->spec_seq += n;
        if (parsed != NULL)
            *parsed = cons;
    }
    q->out = out;
    q->capacity = capacity;
    q->is_seal = is_seal;
    q->type = type;
    if (rl->nqueued++ == 0)
        rl->queue_ticket = rl->next_ticket;
    *ticket = rl->next_ticket++;
    return queue_drain(rl); /* (no free launch slot: stays queued; a failed launch: its windows' waits report it) */
}

int ptls_mi355x_record_layer_cork(ptls_mi355x_record_layer_t *rl, int on)
{
    rl->corked = on != 0;
    return on ? 0 : rl_flush(rl);
}

int ptls_mi355x_record_layer_flush(ptls_mi355x_record_layer_t *rl) { return rl_flush(rl); }

uint64_t ptls_mi355x_record_layer_launches(const ptls_mi355x_record_layer_t *rl) { return rl->launches; }

size_t ptls_mi355x_record_layer_set_coalesce(ptls_mi355x_record_layer_t *rl, size_t windows)
{
    const size_t prev = rl->coalesce;
    (void)rl_flush(rl);
    rl->coalesce = windows > RL_TICKETS ? RL_TICKETS : windows;
    return prev;
}

/* a multi-layer (or uncoalesced) window: the named layers' queued windows go out first */
static rl_slot_t *submit_begin(ptls_mi355x_record_layer_t *const *layers, size_t nlayers, int is_seal)
{
    if (nlayers == 0) {
        rl_msg("no layers");
        return NULL;
    }
    if (!same_key_size(layers, nlayers))
        return NULL;
    for (size_t l = 0; l < nlayers; ++l)
        if (layers[l]->nqueued != 0 && rl_flush(layers[l]) != 0)
            return NULL;
    if (layers[0]->next_ticket - layers[0]->oldest >= RL_TICKETS) {
        rl_msg("all windows are outstanding (wait for the oldest first)");
        return NULL;
    }
    return op_begin(layers, nlayers, is_seal);
}

int ptls_mi355x_record_layer_seal_submit(ptls_mi355x_record_layer_t *const *layers, size_t nlayers,
                                         const ptls_mi355x_iovec_t *const *frags, const size_t *nfrags, uint8_t type,
                                         void *const *out, const size_t *capacity, uint64_t *ticket)
{
    if (nlayers == 1 && layers[0]->coalesce > 1)
        return queue_window(layers[0], 1, type, frags[0], nfrags[0], NULL, 0, out[0], capacity[0], NULL, ticket);
    rl_slot_t *s = submit_begin(layers, nlayers, 1);
    if (s == NULL || seal_build(s, layers, nlayers, frags, nfrags, type, out, capacity) != 0)
        return -1;
    op_commit_window(s, ticket);
    return 0;
}

static int open_submit(ptls_mi355x_record_layer_t *const *layers, size_t nlayers, const void *const *in,
                       const size_t *inlen, void *const *out, const size_t *capacity, size_t *parsed, int any_type,
                       uint64_t *ticket)
{
    if (nlayers == 1 && layers[0]->coalesce > 1 && !any_type)
        return queue_window(layers[0], 0, 0, NULL, 0, in[0], inlen[0], out[0], capacity[0], parsed, ticket);
    rl_slot_t *s = submit_begin(layers, nlayers, 0);
    if (s == NULL || open_build(s, layers, nlayers, in, inlen, out, capacity, parsed, any_type, 1) != 0)
        return -1;
    op_commit_window(s, ticket);
    return 0;
}

int ptls_mi355x_record_layer_open_submit(ptls_mi355x_record_layer_t *const *layers, size_t nlayers, const void *const *in,
                                         const size_t *inlen, void *const *out, const size_t *capacity, size_t *parsed,
                                         uint64_t *ticket)
{
    return open_submit(layers, nlayers, in, inlen, out, capacity, parsed, 0, ticket);
}

/* ---------------------------------------------------------------------------------------------------- wait ---- */

/* results per part into the op (r_outlen, r_nrec, r_cons = fragments sealed, r_alert) */
static void finish_seal(rl_slot_t *s)
{
    rl_op_t *op = &s->op;
    for (size_t l = 0, off = 0; l < op->nlayers; ++l) {
        const rl_part_t *p = &op->part[l];
        if (op->layers[l]->zombie) { /* freed meanwhile: nothing is delivered to it */
            off += op->direct ? 0 : p->wire;
            op->r_outlen[l] = op->r_nrec[l] = op->r_cons[l] = 0;
            op->r_alert[l] = PTLS_MI355X_RECORD_LAYER_STALE;
            continue;
        }
        if (!op->direct && p->wire != 0) {
            memcpy(op->out[l], s->h_buf + op->off_dst + off, p->wire);
            off += p->wire;
        }
        op->r_outlen[l] = p->wire;
        op->r_nrec[l] = p->nrec;
        op->r_cons[l] = p->nfrags;
        op->r_alert[l] = p->stopped ? PTLS_MI355X_RECORD_LAYER_KEY_UPDATE : 0;
    }
    if (!op->direct && op->srcbytes != 0)
        memset(s->h_buf + op->off_src, 0, op->srcbytes); /* no plaintext left in the staging */
}

/* results per part into the op (r_outlen, r_nrec, r_cons = wire bytes delivered, r_alert); *type: the last delivered
 * record's inner content type (open_record) */
static void finish_open(rl_slot_t *s, uint8_t *type)
{
    rl_op_t *op = &s->op;
    const uint32_t *status = (const uint32_t *)(s->h_buf + op->off_st);
    const uint8_t *types = s->h_buf + op->off_ty;
    for (size_t l = 0; l < op->nlayers; ++l) {
        const rl_part_t *p = &op->part[l];
        ptls_mi355x_record_layer_t *x = op->layers[l];
        uint8_t *slots = op->direct ? (uint8_t *)op->out[l] : s->h_buf + op->off_dst + p->dst_add;
        size_t done = 0, wire_done = 0, olen = 0;
        int a = 0;
        if (x->zombie) { /* freed meanwhile: nothing is delivered to it */
            op->r_cons[l] = op->r_outlen[l] = op->r_nrec[l] = 0;
            op->r_alert[l] = PTLS_MI355X_RECORD_LAYER_STALE;
            if (p->n != 0 && !op->direct)
                memset(slots, 0, p->ptbytes);
            continue;
        }
        if (p->seq0 != x->seq) {
            a = PTLS_MI355X_RECORD_LAYER_STALE; /* a window before this one stopped early */
        } else if (p->n != 0) {
            /* slot i of this layer at its local plaintext offset: in out[l] (direct) or in the staging */
            for (size_t i = p->k0; i < p->k0 + p->n; ++i) {
                if (status[i] == PTLS_MI355X_TLS_BAD_RECORD_MAC) {
                    a = 20; /* PTLS_ALERT_BAD_RECORD_MAC */
                    break;
                }
                if (status[i] == PTLS_MI355X_TLS_UNEXPECTED_MESSAGE) {
                    a = 10; /* PTLS_ALERT_UNEXPECTED_MESSAGE: no content type */
                    break;
                }
                if (types[i] != 23 && !op->any_type) /* a handshake / alert record: open_record delivers it */
                    break;
                if (olen + status[i] > op->capacity[l]) {
                    if (done == 0) {
                        snprintf(rl_err, sizeof(rl_err), "record layer: %u plaintext bytes exceed the output capacity %zu",
                                 status[i], op->capacity[l]);
                        a = -1;
                    }
                    break;
                }
                /* delivered by the kernel; direct: slot i starts at or after olen, so the plaintexts close up in place */
                if (!op->deliver)
                    memmove((uint8_t *)op->out[l] + olen, slots + (s->recs[i].dst - p->dst_add), status[i]);
                olen += status[i];
                wire_done += PTLS_MI355X_TLS_HEADER_SIZE + s->recs[i].len;
                if (type != NULL)
                    *type = types[i];
                ++done;
            }
            x->seq += done;
        }
        if (p->n != 0 && !op->deliver) {
            if (op->direct)
                memset((uint8_t *)op->out[l] + olen, 0, p->ptbytes - olen); /* padding, types, records not delivered */
            else
                memset(slots, 0, p->ptbytes); /* no plaintext left in the staging */
        }
        if (a == 0 && done == p->n)
            a = p->perr; /* a DECODE_ERROR behind the parsed records */
        if (a != PTLS_MI355X_RECORD_LAYER_STALE && done < p->n)
            x->spec_seq = x->seq; /* stopped early: the windows behind this one are stale, new ones follow it */
        op->r_cons[l] = wire_done;
        op->r_outlen[l] = olen;
        op->r_nrec[l] = done;
        op->r_alert[l] = a;
    }
}

/* the op's launch is done (or failed): results into the op, its layers count it out */
static void op_complete(rl_slot_t *s, uint8_t *type)
{
    rl_op_t *op = &s->op;
    hipError_t e;
    if (op->nrec != 0 && (e = hipStreamSynchronize(s->stream)) != hipSuccess) {
        rl_fail("synchronize", e);
        op_scrub(s);
        if (!op->is_seal) /* nothing delivered: the next window starts at the delivered position */
            for (size_t l = 0; l < op->nlayers; ++l)
                if (!op->layers[l]->zombie)
                    op->layers[l]->spec_seq = op->layers[l]->seq;
        op->failed = 1;
    } else if (op->is_seal) {
        finish_seal(s);
    } else {
        finish_open(s, type);
    }
    op->done = 1;
    op_release_layers(op); /* (a failed window's open parts: spec_seq back to seq when nothing else is in flight) */
}

static int op_wait(ptls_mi355x_record_layer_t *rl, uint64_t ticket, size_t *outlen, size_t *nrecords, size_t *consumed,
                   int *alerts, uint8_t *type)
{
    if (ticket != rl->oldest || rl->oldest == rl->next_ticket)
        return rl_msg(rl->oldest == rl->next_ticket ? "no window outstanding" : "windows are completed in submission order");
    if (rl->nqueued != 0 && ticket >= rl->queue_ticket) { /* still queued: it goes out now (older windows are done) */
        (void)rl_flush(rl);
        if (rl->nqueued != 0 && ticket >= rl->queue_ticket)
            return rl_msg("a queued window found no free launch slot");
    }
    (void)queue_drain(rl);
    rl_slot_t *s = &rl->slot[rl->ticket_slot[ticket % RL_TICKETS]];
    rl_op_t *op = &s->op;
    if (!op->done)
        op_complete(s, type);
    int ret = op->failed ? -1 : 0;
    /* a coalesced launch: this ticket's window is part (ticket - first ticket); otherwise every part is this window */
    const size_t first = op->coalesced ? (size_t)(ticket - op->ticket) : 0, n = op->coalesced ? 1 : op->nlayers;
    for (size_t l = 0; l < n; ++l) {
        const int ok = !op->failed;
        outlen[l] = ok ? op->r_outlen[first + l] : 0;
        if (nrecords != NULL)
            nrecords[l] = ok ? op->r_nrec[first + l] : 0;
        if (consumed != NULL)
            consumed[l] = ok ? op->r_cons[first + l] : 0;
        alerts[l] = ok ? op->r_alert[first + l] : 0;
    }
    if (op->failed && op->nlayers == 0 && ret == -1 && rl_err[0] == 0)
        rl_msg("the window's launch failed");
    ++rl->oldest;
    if (++op->waited == op->nwin)
        op_discard(op);
    (void)queue_drain(rl); /* a launch slot may have come free: the queue goes out when due */
    return ret;
}

int ptls_mi355x_record_layer_wait(ptls_mi355x_record_layer_t *rl, uint64_t ticket, size_t *outlen, size_t *nrecords,
                                  size_t *consumed, int *alerts)
{
    return op_wait(rl, ticket, outlen, nrecords, consumed, alerts, NULL);
}

/* ------------------------------------------------------------------------------------- synchronous calls ---- */

/* 1 when no layer has an asynchronous window outstanding (a synchronous call is a submit and its wait) */
static int no_pending(ptls_mi355x_record_layer_t *const *layers, size_t nlayers)
{
    for (size_t l = 0; l < nlayers; ++l) {
        if (layers[l]->next_ticket != layers[l]->oldest || layers[l]->inflight != 0) {
            rl_msg("asynchronous windows outstanding (wait for them first)");
            return 0;
        }
    }
    return 1;
}

int ptls_mi355x_record_layer_seal_multi(ptls_mi355x_record_layer_t *const *layers, size_t nlayers,
                                        const ptls_mi355x_iovec_t *const *frags, const size_t *nfrags, uint8_t type,
                                        void *const *out, const size_t *capacity, size_t *outlen, size_t *nrecords)
{
    for (size_t l = 0; l < nlayers; ++l) {
        outlen[l] = 0;
        if (nrecords != NULL)
            nrecords[l] = 0;
    }
    if (nlayers == 0)
        return 0;
    if (!no_pending(layers, nlayers))
        return -1;
    int stack_alerts[8], *alerts = nlayers <= 8 ? stack_alerts : malloc(nlayers * sizeof(int));
    if (alerts == NULL)
        return rl_msg("out of memory");
    uint64_t t;
    int ret = ptls_mi355x_record_layer_seal_submit(layers, nlayers, frags, nfrags, type, out, capacity, &t);
    if (ret == 0)
        ret = op_wait(layers[0], t, outlen, nrecords, NULL, alerts, NULL);
    for (size_t l = 0; ret == 0 && l < nlayers; ++l)
        if (alerts[l] == PTLS_MI355X_RECORD_LAYER_KEY_UPDATE)
            ret = PTLS_MI355X_RECORD_LAYER_KEY_UPDATE;
    if (alerts != stack_alerts)
        free(alerts);
    return ret;
}

int ptls_mi355x_record_layer_seal(ptls_mi355x_record_layer_t *rl, const ptls_mi355x_iovec_t *frags, size_t nfrags,
                                  uint8_t type, void *out, size_t capacity, size_t *outlen, size_t *nrecords)
{
    return ptls_mi355x_record_layer_seal_multi(&rl, 1, &frags, &nfrags, type, &out, &capacity, outlen, nrecords);
}

int ptls_mi355x_record_layer_open_multi(ptls_mi355x_record_layer_t *const *layers, size_t nlayers, const void *const *in,
                                        const size_t *inlen, size_t *consumed, void *const *out, const size_t *capacity,
                                        size_t *outlen, size_t *nrecords, int *alerts)
{
    for (size_t l = 0; l < nlayers; ++l) {
        consumed[l] = outlen[l] = 0;
        alerts[l] = 0;
        if (nrecords != NULL)
            nrecords[l] = 0;
    }
    if (nlayers == 0)
        return 0;
    if (!no_pending(layers, nlayers))
        return -1;
    uint64_t t;
    if (open_submit(layers, nlayers, in, inlen, out, capacity, NULL, 0, &t) != 0)
        return -1;
    return op_wait(layers[0], t, outlen, nrecords, consumed, alerts, NULL);
}

int ptls_mi355x_record_layer_open(ptls_mi355x_record_layer_t *rl, const void *in, size_t inlen, size_t *consumed,
                                  void *out, size_t capacity, size_t *outlen, size_t *nrecords)
{
    int alert = 0;
    if (ptls_mi355x_record_layer_open_multi(&rl, 1, &in, &inlen, consumed, &out, &capacity, outlen, nrecords, &alert) != 0)
        return -1;
    return alert;
}

int ptls_mi355x_record_layer_open_record(ptls_mi355x_record_layer_t *rl, const void *in, size_t inlen, size_t *consumed,
                                         void *out, size_t capacity, size_t *outlen, uint8_t *content_type)
{
    *consumed = *outlen = 0;
    *content_type = 0;
    if (!no_pending(&rl, 1))
        return -1;
    uint64_t t;
    int alert = 0;
    if (open_submit(&rl, 1, &in, &inlen, &out, &capacity, NULL, 1, &t) != 0)
        return -1;
    if (op_wait(rl, t, outlen, NULL, consumed, &alert, content_type) != 0)
        return -1;
    if (*consumed == 0)
        *content_type = 0;
    return alert;
}
