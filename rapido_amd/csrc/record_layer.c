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
    uint8_t key[32]; /* the key, to check that the layers of a _multi call share it (zeroed on free) */
    size_t key_size;
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
    memcpy(rl->key, key, key_size);
    rl->key_size = key_size;
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
    memset(rl->key, 0, sizeof(rl->key));
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

static uint32_t be32(const uint8_t *b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; }

int ptls_mi355x_record_layer_seal_multi(ptls_mi355x_record_layer_t *const *layers, size_t nlayers,
                                        const ptls_mi355x_iovec_t *const *frags, const size_t *nfrags, uint8_t type,
                                        void *const *out, const size_t *capacity, size_t *outlen, size_t *nrecords)
{
    if (nlayers == 0)
        return 0;
    ptls_mi355x_record_layer_t *rl = layers[0];
    size_t nrec = 0, srcbytes = 0, wire = 0;
    for (size_t l = 0; l < nlayers; ++l) {
        const ptls_mi355x_record_layer_t *x = layers[l];
        outlen[l] = 0;
        if (nrecords != NULL)
            nrecords[l] = 0;
        /* one launch, one key image: the connections of one session (rapido: the session key, the IV differing in
         * bytes 0..3 only, derive_connection_aead_iv lib/rapido.c:123-133) */
        if (x->key_size != rl->key_size || memcmp(x->key, rl->key, rl->key_size) != 0 ||
            memcmp(x->iv + 4, rl->iv + 4, 8) != 0) {
            snprintf(rl_err, sizeof(rl_err), "record layer: layer %zu has another key or IV bytes 4..11", l);
            return -1;
        }
        size_t wl = 0;
        for (size_t f = 0; f < nfrags[l]; ++f) {
            uint64_t sq = 0;
            size_t w = 0;
            nrec += ptls_mi355x_tls_plan_send(frags[l][f].len, type, &sq, 0, 0, NULL, 0, &w);
            srcbytes += frags[l][f].len;
            wl += w;
        }
        if (wl > capacity[l]) {
            snprintf(rl_err, sizeof(rl_err), "record layer: %zu wire bytes exceed the output capacity %zu (layer %zu)",
                     wl, capacity[l], l);
            return -1;
        }
        outlen[l] = wl; /* provisional: reset below unless the call succeeds */
        wire += wl;
    }
    if (nrec == 0) {
        for (size_t l = 0; l < nlayers; ++l)
            outlen[l] = 0;
        return 0;
    }
    if (reserve_recs(rl, nrec) != 0)
        goto Fail;
    /* direct: every non-empty fragment and every output in registered ranges; addressed from the lowest of each */
    uint8_t *src_base = NULL, *dst_base = NULL;
    int direct = 1;
    for (size_t l = 0; direct && l < nlayers; ++l) {
        uint8_t *d = outlen[l] != 0 ? dev_addr_any(layers, nlayers, out[l], outlen[l]) : NULL;
        if (outlen[l] != 0 && d == NULL)
            direct = 0;
        else if (d != NULL && (dst_base == NULL || d < dst_base))
            dst_base = d;
        for (size_t f = 0; direct && f < nfrags[l]; ++f) {
            if (frags[l][f].len == 0)
                continue;
            if ((d = dev_addr_any(layers, nlayers, frags[l][f].base, frags[l][f].len)) == NULL)
                direct = 0;
            else if (src_base == NULL || d < src_base)
                src_base = d;
        }
    }
    const size_t off_conn = up16(nrec * sizeof(ptls_mi355x_tls_record_t));
    const size_t off_src = off_conn + (nlayers > 1 ? up16(nrec * 4) : 0);
    const size_t off_dst = off_src + (direct ? 0 : up16(srcbytes)), total = off_dst + (direct ? 0 : up16(wire));
    const int zero_copy = direct || total <= rl->zero_copy_bytes;
    if (reserve_stage(rl, total) != 0 || (!zero_copy && reserve_device(rl, total) != 0))
        goto Fail;
    /* descriptors (offsets relative to the src / dst bases), the per-record IV differences and, unless direct, the
     * fragments back to back */
    uint32_t *conn = (uint32_t *)(rl->h_buf + off_conn);
    uint64_t *seqs = (uint64_t *)malloc(nlayers * sizeof(uint64_t));
    if (seqs == NULL) {
        snprintf(rl_err, sizeof(rl_err), "record layer: out of memory");
        goto Fail;
    }
    size_t k = 0, src_off = 0, dst_off = 0;
    for (size_t l = 0; l < nlayers; ++l) {
        seqs[l] = layers[l]->seq;
        if (direct && outlen[l] != 0)
            dst_off = (size_t)(dev_addr_any(layers, nlayers, out[l], outlen[l]) - dst_base);
        const uint32_t cid = be32(layers[l]->iv) ^ be32(rl->iv); /* BE32(cid) ^ IV[0..3] of layer 0 = layer l's */
        const size_t k0 = k;
        for (size_t f = 0; f < nfrags[l]; ++f) {
            const ptls_mi355x_iovec_t *fr = &frags[l][f];
            size_t w = 0;
            if (direct && fr->len != 0)
                src_off = (size_t)(dev_addr_any(layers, nlayers, fr->base, fr->len) - src_base);
            k += ptls_mi355x_tls_plan_send(fr->len, type, &seqs[l], src_off, dst_off, rl->recs + k, nrec - k, &w);
            if (!direct) {
                if (fr->len != 0)
                    memcpy(rl->h_buf + off_src + src_off, fr->base, fr->len);
                src_off += fr->len;
            }
            dst_off += w;
        }
        if (nlayers > 1)
            for (size_t i = k0; i < k; ++i)
                conn[i] = cid;
    }
    memcpy(rl->h_buf, rl->recs, nrec * sizeof(ptls_mi355x_tls_record_t));
    uint8_t *base = zero_copy ? rl->h_dev : rl->d_buf;
    hipError_t e;
    int rc;
    if (!zero_copy &&
        (e = hipMemcpyAsync(rl->d_buf, rl->h_buf, off_src + srcbytes, hipMemcpyHostToDevice, rl->stream)) != hipSuccess) {
        free(seqs);
        rl_fail("H2D", e);
        goto Fail;
    }
    if (nlayers == 1)
        rc = ptls_mi355x_tls_seal_records(rl->ctx, rl->iv, (const ptls_mi355x_tls_record_t *)base, nrec,
                                          direct ? src_base : base + off_src, direct ? dst_base : base + off_dst,
                                          rl->stream);
    else
        rc = ptls_mi355x_tls_seal_records_multi(rl->ctx, rl->iv, (const ptls_mi355x_tls_record_t *)base,
                                                (const uint32_t *)(base + off_conn), nrec,
                                                direct ? src_base : base + off_src, direct ? dst_base : base + off_dst,
                                                rl->stream);
    if (rc != 0) {
        free(seqs);
        snprintf(rl_err, sizeof(rl_err), "record layer: %s", ptls_mi355x_last_error());
        goto Fail;
    }
    if ((!zero_copy && (e = hipMemcpyAsync(rl->h_buf + off_dst, rl->d_buf + off_dst, wire, hipMemcpyDeviceToHost,
                                           rl->stream)) != hipSuccess) ||
        (e = hipStreamSynchronize(rl->stream)) != hipSuccess) {
        free(seqs);
        rl_fail("synchronize", e);
        goto Fail;
    }
    for (size_t l = 0, off = 0; l < nlayers; ++l) {
        if (!direct) {
            memcpy(out[l], rl->h_buf + off_dst + off, outlen[l]);
            off += outlen[l];
        }
        if (nrecords != NULL)
            nrecords[l] = (size_t)(seqs[l] - layers[l]->seq);
        layers[l]->seq = seqs[l];
    }
    free(seqs);
    if (!direct)
        memset(rl->h_buf + off_src, 0, srcbytes); /* no plaintext left in the staging */
    return 0;
Fail:
    for (size_t l = 0; l < nlayers; ++l)
        outlen[l] = 0;
    return -1;
}

int ptls_mi355x_record_layer_seal(ptls_mi355x_record_layer_t *rl, const ptls_mi355x_iovec_t *frags, size_t nfrags,
                                  uint8_t type, void *out, size_t capacity, size_t *outlen, size_t *nrecords)
{
    return ptls_mi355x_record_layer_seal_multi(&rl, 1, &frags, &nfrags, type, &out, &capacity, outlen, nrecords);
}

/* the layers of one launch share the key and IV bytes 4..11 (the connections of a session) */
static int same_session(ptls_mi355x_record_layer_t *const *layers, size_t nlayers)
{
    const ptls_mi355x_record_layer_t *rl = layers[0];
    for (size_t l = 1; l < nlayers; ++l) {
        const ptls_mi355x_record_layer_t *x = layers[l];
        if (x->key_size != rl->key_size || memcmp(x->key, rl->key, rl->key_size) != 0 ||
            memcmp(x->iv + 4, rl->iv + 4, 8) != 0) {
            snprintf(rl_err, sizeof(rl_err), "record layer: layer %zu has another key or IV bytes 4..11", l);
            return 0;
        }
    }
    return 1;
}

typedef struct {
    size_t k0, n, cons, ptbytes; /* its descriptors rl->recs[k0 .. k0 + n), wire bytes parsed, plaintext slot bytes */
    uint64_t src_add, dst_add;   /* added to its descriptors' offsets (its position in the launch's src / dst) */
    int perr;
} rl_open_part_t;

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
    ptls_mi355x_record_layer_t *rl = layers[0];
    if (!same_session(layers, nlayers))
        return -1;
    rl_open_part_t *part = (rl_open_part_t *)calloc(nlayers, sizeof(*part));
    if (part == NULL) {
        snprintf(rl_err, sizeof(rl_err), "record layer: out of memory");
        return -1;
    }
    int ret = -1;
    size_t max = 0, nrec = 0, srcbytes = 0, ptbytes = 0;
    for (size_t l = 0; l < nlayers; ++l)
        max += inlen[l] / (PTLS_MI355X_TLS_HEADER_SIZE + 16) + 1;
    if (reserve_recs(rl, max) != 0)
        goto Exit;
    /* the complete application_data records at the start of every input, offsets local to it for now */
    for (size_t l = 0; l < nlayers; ++l) {
        uint64_t seq = layers[l]->seq;
        part[l].k0 = nrec;
        part[l].perr = ptls_mi355x_tls_parse_records((const uint8_t *)in[l], inlen[l], 0, &seq, 0, rl->recs + nrec,
                                                     max - nrec, &part[l].n, &part[l].cons);
        if (part[l].n != 0) {
            const ptls_mi355x_tls_record_t *last = rl->recs + nrec + part[l].n - 1;
            part[l].ptbytes = last->dst + (last->len >= 16u ? last->len - 16u : 0u);
        }
        nrec += part[l].n;
        srcbytes += up16(part[l].cons);
        ptbytes += up16(part[l].ptbytes);
    }
    if (nrec == 0) {
        for (size_t l = 0; l < nlayers; ++l)
            alerts[l] = part[l].perr;
        ret = 0;
        goto Exit;
    }
    /* direct: every input and every plaintext buffer (at least as large as its slots) in registered ranges */
    uint8_t *src_base = NULL, *dst_base = NULL;
    int direct = 1;
    for (size_t l = 0; direct && l < nlayers; ++l) {
        if (part[l].n == 0)
            continue;
        uint8_t *di = dev_addr_any(layers, nlayers, in[l], part[l].cons);
        uint8_t *dout = capacity[l] >= part[l].ptbytes ? dev_addr_any(layers, nlayers, out[l], part[l].ptbytes) : NULL;
        if (di == NULL || dout == NULL) {
            direct = 0;
            break;
        }
        if (src_base == NULL || di < src_base)
            src_base = di;
        if (dst_base == NULL || dout < dst_base)
            dst_base = dout;
    }
    const size_t off_conn = up16(nrec * sizeof(ptls_mi355x_tls_record_t));
    const size_t off_src = off_conn + (nlayers > 1 ? up16(nrec * 4) : 0);
    const size_t off_dst = off_src + (direct ? 0 : srcbytes), off_st = off_dst + (direct ? 0 : ptbytes);
    const size_t off_ty = off_st + up16(nrec * 4), total = off_ty + up16(nrec);
    const int zero_copy = direct || total <= rl->zero_copy_bytes;
    if (reserve_stage(rl, total) != 0 || (!zero_copy && reserve_device(rl, total) != 0))
        goto Exit;
    uint32_t *conn = (uint32_t *)(rl->h_buf + off_conn);
    for (size_t l = 0, so = 0, dso = 0; l < nlayers; ++l) {
        if (part[l].n == 0)
            continue;
        if (direct) {
            part[l].src_add = (uint64_t)(dev_addr_any(layers, nlayers, in[l], part[l].cons) - src_base);
            part[l].dst_add = (uint64_t)(dev_addr_any(layers, nlayers, out[l], part[l].ptbytes) - dst_base);
        } else {
            part[l].src_add = so;
            part[l].dst_add = dso;
            memcpy(rl->h_buf + off_src + so, in[l], part[l].cons);
            so += up16(part[l].cons);
            dso += up16(part[l].ptbytes);
        }
        const uint32_t cid = be32(layers[l]->iv) ^ be32(rl->iv);
        for (size_t i = part[l].k0; i < part[l].k0 + part[l].n; ++i) {
            rl->recs[i].src += part[l].src_add;
            rl->recs[i].dst += part[l].dst_add;
            if (nlayers > 1)
                conn[i] = cid;
        }
    }
    memcpy(rl->h_buf, rl->recs, nrec * sizeof(ptls_mi355x_tls_record_t));
    uint8_t *base = zero_copy ? rl->h_dev : rl->d_buf;
    hipError_t e;
    int rc;
    if (!zero_copy && (e = hipMemcpyAsync(rl->d_buf, rl->h_buf, off_src + srcbytes, hipMemcpyHostToDevice,
                                          rl->stream)) != hipSuccess) {
        rl_fail("H2D", e);
        goto Exit;
    }
    /* every record verified independently; the stop at a connection's first failure is the host loop below */
    if (nlayers == 1)
        rc = ptls_mi355x_tls_open_records(rl->ctx, rl->iv, (const ptls_mi355x_tls_record_t *)base, nrec,
                                          direct ? src_base : base + off_src, direct ? dst_base : base + off_dst,
                                          (uint32_t *)(base + off_st), base + off_ty, rl->stream);
    else
        rc = ptls_mi355x_tls_open_records_multi(rl->ctx, rl->iv, (const ptls_mi355x_tls_record_t *)base,
                                                (const uint32_t *)(base + off_conn), nrec,
                                                direct ? src_base : base + off_src, direct ? dst_base : base + off_dst,
                                                (uint32_t *)(base + off_st), base + off_ty, rl->stream);
    if (rc != 0) {
        snprintf(rl_err, sizeof(rl_err), "record layer: %s", ptls_mi355x_last_error());
        goto Exit;
    }
    if ((!zero_copy && (e = hipMemcpyAsync(rl->h_buf + off_dst, rl->d_buf + off_dst, off_ty + nrec - off_dst,
                                           hipMemcpyDeviceToHost, rl->stream)) != hipSuccess) ||
        (e = hipStreamSynchronize(rl->stream)) != hipSuccess) {
        rl_fail("synchronize", e);
        goto Exit;
    }
    const uint32_t *status = (const uint32_t *)(rl->h_buf + off_st);
    const uint8_t *types = rl->h_buf + off_ty;
    for (size_t l = 0; l < nlayers; ++l) {
        if (part[l].n == 0) {
            alerts[l] = part[l].perr;
            continue;
        }
        /* slot i of this layer at its local plaintext offset: in out[l] (direct) or in the staging */
        uint8_t *slots = direct ? (uint8_t *)out[l] : rl->h_buf + off_dst + part[l].dst_add;
        size_t done = 0, wire_done = 0, olen = 0;
        int a = 0;
        for (size_t i = part[l].k0; i < part[l].k0 + part[l].n; ++i) {
            if (status[i] == PTLS_MI355X_TLS_BAD_RECORD_MAC) {
                a = 20; /* PTLS_ALERT_BAD_RECORD_MAC */
                break;
            }
            if (status[i] == PTLS_MI355X_TLS_UNEXPECTED_MESSAGE) {
                a = 10; /* PTLS_ALERT_UNEXPECTED_MESSAGE: no content type */
                break;
            }
            if (types[i] != 23) /* a handshake / alert record inside: the caller's picotls path re-opens it */
                break;
            if (olen + status[i] > capacity[l]) {
                if (done == 0) {
                    snprintf(rl_err, sizeof(rl_err), "record layer: %u plaintext bytes exceed the output capacity %zu",
                             status[i], capacity[l]);
                    a = -1;
                }
                break;
            }
            /* direct: slot i starts at or after olen, so the delivered plaintexts close up in place */
            memmove((uint8_t *)out[l] + olen, slots + (rl->recs[i].dst - part[l].dst_add), status[i]);
            olen += status[i];
            wire_done += PTLS_MI355X_TLS_HEADER_SIZE + (rl->recs[i].len);
            ++done;
        }
        if (direct)
            memset((uint8_t *)out[l] + olen, 0, part[l].ptbytes - olen); /* padding, types, records not delivered */
        else
            memset(slots, 0, part[l].ptbytes); /* no plaintext left in the staging */
        layers[l]->seq += done;
        consumed[l] = wire_done;
        outlen[l] = olen;
        if (nrecords != NULL)
            nrecords[l] = done;
        alerts[l] = a == 0 && done == part[l].n ? part[l].perr : a; /* a DECODE_ERROR behind the parsed records */
    }
    ret = 0;
Exit:
    free(part);
    return ret;
}

int ptls_mi355x_record_layer_open(ptls_mi355x_record_layer_t *rl, const void *in, size_t inlen, size_t *consumed,
                                  void *out, size_t capacity, size_t *outlen, size_t *nrecords)
{
    int alert = 0;
    if (ptls_mi355x_record_layer_open_multi(&rl, 1, &in, &inlen, consumed, &out, &capacity, outlen, nrecords, &alert) != 0)
        return -1;
    return alert;
}
