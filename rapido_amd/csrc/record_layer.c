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
 *   open: the complete application_data records at the start of the input are parsed (ptls_mi355x_tls_parse_
 *         records) and opened by ptls_mi355x_tls_open_records.  Records are then delivered in order until the first
 *         failure (its alert is returned, as ptls_receive returns it, lib/picotls.c:650-652) or the first record
 *         whose inner type is not application_data (left unconsumed, seq not advanced, for the caller's picotls
 *         slot path).  Every record is verified independently by the kernel; the stop at the first failure is this
 *         host loop, and nothing behind it reaches the caller (slots are zeroed).
 *
 * Where the bytes travel, per call (the first that applies):
 *   direct     -- the fragments and the output (seal), or the input and the output (open), all lie in host ranges
 *                 the caller registered (ptls_mi355x_record_layer_register: long-lived socket buffers): the kernel
 *                 reads and writes them in place over PCIe.  Only the descriptors (and statuses) pass through the
 *                 layer's staging.  No copy at all.
 *   zero-copy  -- the window fits the zero-copy limit: fragments / input are copied into the layer's pinned,
 *                 mapped, coherent staging and the kernel works on it over PCIe; one launch, one synchronisation.
 *   copy       -- larger windows: staging -> one H2D copy -> launch -> one D2H copy (DMA at the link rate).
 * Everything runs on the layer's own stream and the call returns when the results are in the caller's buffer.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <hip/hip_runtime_api.h>
#include "../../include/ptls_mi355x.h"

#define RL_MAX_REGIONS 8
#define RL_ZERO_COPY_DEFAULT ((size_t)4 << 20)

typedef struct {
    uint8_t *base; /* host address as registered */
    uint8_t *dev;  /* its device address */
    size_t len;
    int owned;     /* registered by this layer (not already registered, e.g. by the other direction's layer) */
} rl_region_t;

struct st_ptls_mi355x_record_layer_t {
    ptls_mi355x_aesgcm_context_t *ctx;
    uint8_t iv[12];
    uint64_t seq;
    hipStream_t stream;
    uint8_t *h_buf; /* pinned, mapped, coherent staging: [descriptors | input | output | status | types] */
    uint8_t *h_dev; /* the staging's device address (zero-copy and direct calls) */
    size_t cap;
    uint8_t *d_buf; /* device copy of the staging layout (copy calls), allocated on first use */
    size_t d_cap;
    size_t zero_copy_bytes;
    rl_region_t reg[RL_MAX_REGIONS];
    size_t nreg;
    ptls_mi355x_tls_record_t *recs; /* host descriptors */
    size_t recs_cap;
};

static char rl_err[160];

static size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

static int rl_fail(const char *what, hipError_t e)
{
    snprintf(rl_err, sizeof(rl_err), "record layer: %s: %s", what, hipGetErrorString(e));
    (void)hipGetLastError(); /* reported here: not left for the next unrelated call to find */
    return -1;
}

const char *ptls_mi355x_record_layer_last_error(void) { return rl_err; }

static int reserve_recs(ptls_mi355x_record_layer_t *rl, size_t nrecs)
{
    if (nrecs <= rl->recs_cap)
        return 0;
    size_t c = rl->recs_cap ? rl->recs_cap : 64;
    while (c < nrecs)
        c *= 2;
    ptls_mi355x_tls_record_t *r = realloc(rl->recs, c * sizeof(*r));
    if (r == NULL) {
        snprintf(rl_err, sizeof(rl_err), "record layer: out of memory");
        return -1;
    }
    rl->recs = r;
    rl->recs_cap = c;
    return 0;
}

static int reserve_stage(ptls_mi355x_record_layer_t *rl, size_t bytes)
{
    if (bytes <= rl->cap)
        return 0;
    size_t c = rl->cap ? rl->cap : 1 << 16;
    while (c < bytes)
        c *= 2;
    hipError_t e;
    if (rl->h_buf != NULL)
        (void)hipHostFree(rl->h_buf);
    rl->h_buf = rl->h_dev = NULL;
    rl->cap = 0;
    /* coherent: the kernel's zero-copy reads never see stale lines of an earlier window */
    if ((e = hipHostMalloc((void **)&rl->h_buf, c, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
        return rl_fail("hipHostMalloc", e);
    if ((e = hipHostGetDevicePointer((void **)&rl->h_dev, rl->h_buf, 0)) != hipSuccess)
        return rl_fail("hipHostGetDevicePointer", e);
    rl->cap = c;
    return 0;
}

static int reserve_device(ptls_mi355x_record_layer_t *rl, size_t bytes)
{
    if (bytes <= rl->d_cap)
        return 0;
    hipError_t e;
    if (rl->d_buf != NULL)
        (void)hipFree(rl->d_buf);
    rl->d_buf = NULL;
    rl->d_cap = 0;
    if ((e = hipMalloc((void **)&rl->d_buf, rl->cap)) != hipSuccess)
        return rl_fail("hipMalloc", e);
    rl->d_cap = rl->cap;
    return 0;
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
    ptls_mi355x_record_layer_t *rl = calloc(1, sizeof(*rl));
    if (rl == NULL)
        return NULL;
    hipError_t e;
    if ((rl->ctx = ptls_mi355x_aesgcm_new(key, key_size, 0)) == NULL) {
        snprintf(rl_err, sizeof(rl_err), "record layer: %s", ptls_mi355x_last_error());
        free(rl);
        return NULL;
    }
    if ((e = hipStreamCreateWithFlags(&rl->stream, hipStreamNonBlocking)) != hipSuccess) {
        rl_fail("hipStreamCreateWithFlags", e);
        ptls_mi355x_aesgcm_free(rl->ctx);
        free(rl);
        return NULL;
    }
    memcpy(rl->iv, iv12, 12);
    rl->seq = seq;
    rl->zero_copy_bytes = RL_ZERO_COPY_DEFAULT;
    return rl;
}

void ptls_mi355x_record_layer_free(ptls_mi355x_record_layer_t *rl)
{
    if (rl == NULL)
        return;
    while (rl->nreg != 0)
        (void)ptls_mi355x_record_layer_unregister(rl, rl->reg[rl->nreg - 1].base);
    if (rl->stream != NULL) {
        (void)hipStreamSynchronize(rl->stream);
        (void)hipStreamDestroy(rl->stream);
    }
    if (rl->h_buf != NULL) {
        memset(rl->h_buf, 0, rl->cap); /* plaintexts passed through the staging */
        (void)hipHostFree(rl->h_buf);
    }
    if (rl->d_buf != NULL) {
        (void)hipMemset(rl->d_buf, 0, rl->d_cap);
        (void)hipFree(rl->d_buf);
    }
    free(rl->recs);
    ptls_mi355x_aesgcm_free(rl->ctx);
    memset(rl->iv, 0, sizeof(rl->iv));
    free(rl);
}

uint64_t ptls_mi355x_record_layer_get_seq(const ptls_mi355x_record_layer_t *rl) { return rl->seq; }

void ptls_mi355x_record_layer_set_seq(ptls_mi355x_record_layer_t *rl, uint64_t seq) { rl->seq = seq; }

size_t ptls_mi355x_record_layer_set_zero_copy_bytes(ptls_mi355x_record_layer_t *rl, size_t n)
{
    const size_t prev = rl->zero_copy_bytes;
    rl->zero_copy_bytes = n;
    return prev;
}

int ptls_mi355x_record_layer_register(ptls_mi355x_record_layer_t *rl, void *base, size_t len)
{
    if (rl->nreg == RL_MAX_REGIONS || base == NULL || len == 0) {
        snprintf(rl_err, sizeof(rl_err), "record layer: %s", base == NULL || len == 0 ? "empty range" : "too many ranges");
        return -1;
    }
    hipError_t e;
    uint8_t *dev = NULL;
    int owned = 1;
    if ((e = hipHostRegister(base, len, hipHostRegisterMapped)) == hipErrorHostMemoryAlreadyRegistered) {
        (void)hipGetLastError();
        owned = 0; /* a range the application (or another layer) registered: used, never unregistered here */
    } else if (e != hipSuccess) {
        return rl_fail("hipHostRegister", e);
    }
    if ((e = hipHostGetDevicePointer((void **)&dev, base, 0)) != hipSuccess) {
        if (owned)
            (void)hipHostUnregister(base);
        return rl_fail("hipHostGetDevicePointer", e);
    }
    rl->reg[rl->nreg++] = (rl_region_t){(uint8_t *)base, dev, len, owned};
    return 0;
}

int ptls_mi355x_record_layer_unregister(ptls_mi355x_record_layer_t *rl, void *base)
{
    for (size_t i = 0; i < rl->nreg; ++i) {
        if (rl->reg[i].base == base) {
            (void)hipStreamSynchronize(rl->stream); /* no launch of this layer still reads the range */
            hipError_t e = rl->reg[i].owned ? hipHostUnregister(base) : hipSuccess;
            if (e == hipErrorHostMemoryNotRegistered) { /* registered twice, already released by the other owner */
                (void)hipGetLastError();
                e = hipSuccess;
            }
            rl->reg[i] = rl->reg[--rl->nreg];
            return e == hipSuccess ? 0 : rl_fail("hipHostUnregister", e);
        }
    }
    snprintf(rl_err, sizeof(rl_err), "record layer: range not registered");
    return -1;
}

int ptls_mi355x_record_layer_seal(ptls_mi355x_record_layer_t *rl, const ptls_mi355x_iovec_t *frags, size_t nfrags,
                                  uint8_t type, void *out, size_t capacity, size_t *outlen, size_t *nrecords)
{
    size_t nrec = 0, srcbytes = 0, wire = 0;
    for (size_t f = 0; f < nfrags; ++f) {
        uint64_t s = 0;
        size_t w = 0;
        nrec += ptls_mi355x_tls_plan_send(frags[f].len, type, &s, 0, 0, NULL, 0, &w);
        srcbytes += frags[f].len;
        wire += w;
    }
    *outlen = 0;
    if (nrecords != NULL)
        *nrecords = 0;
    if (wire > capacity) {
        snprintf(rl_err, sizeof(rl_err), "record layer: %zu wire bytes exceed the output capacity %zu", wire, capacity);
        return -1;
    }
    if (nrec == 0)
        return 0;
    if (reserve_recs(rl, nrec) != 0)
        return -1;
    /* direct: every non-empty fragment and the output in registered ranges; fragments addressed from the lowest */
    uint8_t *out_dev = dev_addr(rl, out, wire), *src_base = NULL;
    int direct = out_dev != NULL;
    for (size_t f = 0; direct && f < nfrags; ++f) {
        if (frags[f].len == 0)
            continue;
        uint8_t *d = dev_addr(rl, frags[f].base, frags[f].len);
        if (d == NULL)
            direct = 0;
        else if (src_base == NULL || d < src_base)
            src_base = d;
    }
    const size_t off_src = up16(nrec * sizeof(ptls_mi355x_tls_record_t));
    const size_t off_dst = off_src + (direct ? 0 : up16(srcbytes)), total = off_dst + (direct ? 0 : up16(wire));
    const int zero_copy = direct || total <= rl->zero_copy_bytes;
    if (reserve_stage(rl, total) != 0 || (!zero_copy && reserve_device(rl, total) != 0))
        return -1;
    /* descriptors (offsets relative to the src / dst bases) and, unless direct, the fragments back to back */
    size_t k = 0, src_off = 0, dst_off = 0;
    uint64_t seq = rl->seq;
    for (size_t f = 0; f < nfrags; ++f) {
        size_t w = 0;
        if (direct && frags[f].len != 0)
            src_off = (size_t)(dev_addr(rl, frags[f].base, frags[f].len) - src_base);
        k += ptls_mi355x_tls_plan_send(frags[f].len, type, &seq, src_off, dst_off, rl->recs + k, nrec - k, &w);
        if (!direct) {
            if (frags[f].len != 0)
                memcpy(rl->h_buf + off_src + src_off, frags[f].base, frags[f].len);
            src_off += frags[f].len;
        }
        dst_off += w;
    }
    memcpy(rl->h_buf, rl->recs, nrec * sizeof(ptls_mi355x_tls_record_t));
    uint8_t *base = zero_copy ? rl->h_dev : rl->d_buf;
    hipError_t e;
    if (!zero_copy &&
        (e = hipMemcpyAsync(rl->d_buf, rl->h_buf, off_src + srcbytes, hipMemcpyHostToDevice, rl->stream)) != hipSuccess)
        return rl_fail("H2D", e);
    if (ptls_mi355x_tls_seal_records(rl->ctx, rl->iv, (const ptls_mi355x_tls_record_t *)base, nrec,
                                     direct ? src_base : base + off_src, direct ? out_dev : base + off_dst,
                                     rl->stream) != 0) {
        snprintf(rl_err, sizeof(rl_err), "record layer: %s", ptls_mi355x_last_error());
        return -1;
    }
    if (!zero_copy &&
        (e = hipMemcpyAsync(rl->h_buf + off_dst, rl->d_buf + off_dst, wire, hipMemcpyDeviceToHost, rl->stream)) !=
            hipSuccess)
        return rl_fail("D2H", e);
    if ((e = hipStreamSynchronize(rl->stream)) != hipSuccess)
        return rl_fail("synchronize", e);
    if (!direct) {
        memcpy(out, rl->h_buf + off_dst, wire);
        memset(rl->h_buf + off_src, 0, srcbytes); /* no plaintext left in the staging */
    }
    rl->seq = seq;
    *outlen = wire;
    if (nrecords != NULL)
        *nrecords = nrec;
    return 0;
}

int ptls_mi355x_record_layer_open(ptls_mi355x_record_layer_t *rl, const void *in, size_t inlen, size_t *consumed,
                                  void *out, size_t capacity, size_t *outlen, size_t *nrecords)
{
    *consumed = 0;
    *outlen = 0;
    if (nrecords != NULL)
        *nrecords = 0;
    const size_t max = inlen / (PTLS_MI355X_TLS_HEADER_SIZE + 16) + 1;
    if (reserve_recs(rl, max) != 0)
        return -1;
    uint64_t seq = rl->seq;
    size_t nrec = 0, cons = 0;
    const int perr = ptls_mi355x_tls_parse_records((const uint8_t *)in, inlen, 0, &seq, 0, rl->recs, max, &nrec, &cons);
    if (nrec == 0)
        return perr;
    const ptls_mi355x_tls_record_t *last = rl->recs + nrec - 1;
    const size_t ptbytes = last->dst + (last->len >= 16u ? last->len - 16u : 0u); /* the plaintext slots */
    /* direct: the input and the slots (capacity permitting) in registered ranges; the kernel writes the slots into out */
    uint8_t *in_dev = dev_addr(rl, in, cons), *out_dev = capacity >= ptbytes ? dev_addr(rl, out, ptbytes) : NULL;
    const int direct = in_dev != NULL && out_dev != NULL;
    const size_t off_src = up16(nrec * sizeof(ptls_mi355x_tls_record_t));
    const size_t off_dst = off_src + (direct ? 0 : up16(cons)), off_st = off_dst + (direct ? 0 : up16(ptbytes));
    const size_t off_ty = off_st + up16(nrec * 4), total = off_ty + up16(nrec);
    const int zero_copy = direct || total <= rl->zero_copy_bytes;
    if (reserve_stage(rl, total) != 0 || (!zero_copy && reserve_device(rl, total) != 0))
        return -1;
    memcpy(rl->h_buf, rl->recs, nrec * sizeof(ptls_mi355x_tls_record_t));
    if (!direct)
        memcpy(rl->h_buf + off_src, in, cons);
    uint8_t *base = zero_copy ? rl->h_dev : rl->d_buf;
    hipError_t e;
    if (!zero_copy && (e = hipMemcpyAsync(rl->d_buf, rl->h_buf, off_src + cons, hipMemcpyHostToDevice, rl->stream)) !=
                          hipSuccess)
        return rl_fail("H2D", e);
    if (ptls_mi355x_tls_open_records(rl->ctx, rl->iv, (const ptls_mi355x_tls_record_t *)base, nrec,
                                     direct ? in_dev : base + off_src, direct ? out_dev : base + off_dst,
                                     (uint32_t *)(base + off_st), base + off_ty, rl->stream) != 0) {
        snprintf(rl_err, sizeof(rl_err), "record layer: %s", ptls_mi355x_last_error());
        return -1;
    }
    if (!zero_copy && (e = hipMemcpyAsync(rl->h_buf + off_dst, rl->d_buf + off_dst, off_ty + nrec - off_dst,
                                          hipMemcpyDeviceToHost, rl->stream)) != hipSuccess)
        return rl_fail("D2H", e);
    if ((e = hipStreamSynchronize(rl->stream)) != hipSuccess)
        return rl_fail("synchronize", e);
    const uint32_t *status = (const uint32_t *)(rl->h_buf + off_st);
    const uint8_t *types = rl->h_buf + off_ty;
    uint8_t *slots = direct ? (uint8_t *)out : rl->h_buf + off_dst;
    size_t done = 0, wire_done = 0, olen = 0;
    int ret = 0;
    for (size_t i = 0; i < nrec; ++i) {
        if (status[i] == PTLS_MI355X_TLS_BAD_RECORD_MAC) {
            ret = 20; /* PTLS_ALERT_BAD_RECORD_MAC */
            break;
        }
        if (status[i] == PTLS_MI355X_TLS_UNEXPECTED_MESSAGE) {
            ret = 10; /* PTLS_ALERT_UNEXPECTED_MESSAGE: no content type */
            break;
        }
        if (types[i] != 23) /* a handshake / alert record inside: the caller's picotls path re-opens it */
            break;
        if (olen + status[i] > capacity) {
            if (done == 0) {
                snprintf(rl_err, sizeof(rl_err), "record layer: %u plaintext bytes exceed the output capacity %zu",
                         status[i], capacity);
                ret = -1;
            }
            break;
        }
        /* direct: slot i starts at or after olen, so the delivered plaintexts close up in place */
        memmove((uint8_t *)out + olen, slots + rl->recs[i].dst, status[i]);
        olen += status[i];
        wire_done += PTLS_MI355X_TLS_HEADER_SIZE + rl->recs[i].len;
        ++done;
    }
    if (direct)
        memset((uint8_t *)out + olen, 0, ptbytes - olen); /* padding, types and records not delivered */
    else
        memset(rl->h_buf + off_dst, 0, ptbytes); /* no plaintext left in the staging */
    rl->seq += done;
    *consumed = wire_done;
    *outlen = olen;
    if (nrecords != NULL)
        *nrecords = done;
    if (ret == 0 && done == nrec)
        ret = perr; /* a DECODE_ERROR behind the parsed records */
    return ret;
}
