/*
 * record_layer.c -- a batched TLS 1.3 record layer over HOST buffers (include/ptls_mi355x.h section 5).
 *
 * The reference hands each record to the AEAD one at a time: rapido_prepare_data loops ptls_send over its send
 * window (lib/rapido.c:2083-2111), and picotls frames one record per call (buffer_push_encrypted_records,
 * lib/picotls.c:664-684; handle_input, lib/picotls.c:4757-4842).  An application with its own record layer gets the
 * traffic secrets from picotls' update_traffic_key callback (lib/picotls.c:1206-1211) instead.  This file is that
 * record layer for one traffic direction of one connection, on the GPU: a whole window of records moves host ->
 * device in one copy, is framed and sealed (or opened and unframed) in one launch, and comes back in one copy.
 *
 *   seal: the fragments are planned into records (ptls_mi355x_tls_plan_send, <= 16384 bytes each, consecutive
 *         seq), copied with their descriptors into pinned staging, H2D, ptls_mi355x_tls_seal_records, D2H of the
 *         wire bytes; seq advances by the record count, as ptls_send's does.
 *   open: the complete application_data records at the start of the input are parsed (ptls_mi355x_tls_parse_
 *         records), H2D, opened with PTLS_MI355X_OPEN_STOP_AT_FAILURE, D2H of plaintexts, statuses and inner types.
 *         Records are then delivered in order until the first failure (its alert is returned, as ptls_receive
 *         returns it, lib/picotls.c:650-652) or the first record whose inner type is not application_data (left
 *         unconsumed, seq not advanced, for the caller's picotls slot path).
 *
 * Everything runs on the layer's own stream and the call returns when the results are in the caller's buffer.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <hip/hip_runtime_api.h>
#include "../../include/ptls_mi355x.h"

struct st_ptls_mi355x_record_layer_t {
    ptls_mi355x_aesgcm_context_t *ctx;
    uint8_t iv[12];
    uint64_t seq;
    hipStream_t stream;
    uint8_t *h_buf; /* pinned staging: [descriptors | input | output | status | types] */
    uint8_t *d_buf; /* the same layout on the device */
    size_t cap;
    ptls_mi355x_tls_record_t *recs; /* host descriptors */
    size_t recs_cap;
};

static char rl_err[160];

static size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

static int rl_fail(const char *what, hipError_t e)
{
    snprintf(rl_err, sizeof(rl_err), "record layer: %s: %s", what, hipGetErrorString(e));
    return -1;
}

const char *ptls_mi355x_record_layer_last_error(void) { return rl_err; }

static int reserve(ptls_mi355x_record_layer_t *rl, size_t bytes, size_t nrecs)
{
    if (nrecs > rl->recs_cap) {
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
    }
    if (bytes <= rl->cap)
        return 0;
    size_t c = rl->cap ? rl->cap : 1 << 16;
    while (c < bytes)
        c *= 2;
    hipError_t e;
    if (rl->h_buf != NULL)
        (void)hipHostFree(rl->h_buf);
    if (rl->d_buf != NULL)
        (void)hipFree(rl->d_buf);
    rl->h_buf = NULL;
    rl->d_buf = NULL;
    rl->cap = 0;
    if ((e = hipHostMalloc((void **)&rl->h_buf, c, hipHostMallocDefault)) != hipSuccess)
        return rl_fail("hipHostMalloc", e);
    if ((e = hipMalloc((void **)&rl->d_buf, c)) != hipSuccess)
        return rl_fail("hipMalloc", e);
    rl->cap = c;
    return 0;
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
    return rl;
}

void ptls_mi355x_record_layer_free(ptls_mi355x_record_layer_t *rl)
{
    if (rl == NULL)
        return;
    if (rl->stream != NULL) {
        (void)hipStreamSynchronize(rl->stream);
        (void)hipStreamDestroy(rl->stream);
    }
    if (rl->h_buf != NULL) {
        memset(rl->h_buf, 0, rl->cap); /* plaintexts passed through the staging */
        (void)hipHostFree(rl->h_buf);
    }
    if (rl->d_buf != NULL)
        (void)hipFree(rl->d_buf);
    free(rl->recs);
    ptls_mi355x_aesgcm_free(rl->ctx);
    memset(rl->iv, 0, sizeof(rl->iv));
    free(rl);
}

uint64_t ptls_mi355x_record_layer_get_seq(const ptls_mi355x_record_layer_t *rl) { return rl->seq; }

void ptls_mi355x_record_layer_set_seq(ptls_mi355x_record_layer_t *rl, uint64_t seq) { rl->seq = seq; }

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
    const size_t off_src = up16(nrec * sizeof(ptls_mi355x_tls_record_t)), off_dst = off_src + up16(srcbytes);
    if (reserve(rl, off_dst + up16(wire), nrec) != 0)
        return -1;
    /* descriptors (offsets relative to the src / dst regions) and the fragments, back to back */
    size_t k = 0, src_off = 0, dst_off = 0;
    uint64_t seq = rl->seq;
    for (size_t f = 0; f < nfrags; ++f) {
        size_t w = 0;
        k += ptls_mi355x_tls_plan_send(frags[f].len, type, &seq, src_off, dst_off, rl->recs + k, nrec - k, &w);
        if (frags[f].len != 0)
            memcpy(rl->h_buf + off_src + src_off, frags[f].base, frags[f].len);
        src_off += frags[f].len;
        dst_off += w;
    }
    memcpy(rl->h_buf, rl->recs, nrec * sizeof(ptls_mi355x_tls_record_t));
    hipError_t e;
    if ((e = hipMemcpyAsync(rl->d_buf, rl->h_buf, off_src + srcbytes, hipMemcpyHostToDevice, rl->stream)) != hipSuccess)
        return rl_fail("H2D", e);
    if (ptls_mi355x_tls_seal_records(rl->ctx, rl->iv, (const ptls_mi355x_tls_record_t *)rl->d_buf, nrec,
                                     rl->d_buf + off_src, rl->d_buf + off_dst, rl->stream) != 0) {
        snprintf(rl_err, sizeof(rl_err), "record layer: %s", ptls_mi355x_last_error());
        return -1;
    }
    if ((e = hipMemcpyAsync(rl->h_buf + off_dst, rl->d_buf + off_dst, wire, hipMemcpyDeviceToHost, rl->stream)) !=
            hipSuccess ||
        (e = hipStreamSynchronize(rl->stream)) != hipSuccess)
        return rl_fail("D2H", e);
    memcpy(out, rl->h_buf + off_dst, wire);
    memset(rl->h_buf + off_src, 0, srcbytes); /* no plaintext left in the staging */
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
    if (reserve(rl, 0, max) != 0)
        return -1;
    uint64_t seq = rl->seq;
    size_t nrec = 0, cons = 0;
    const int perr = ptls_mi355x_tls_parse_records((const uint8_t *)in, inlen, 0, &seq, 0, rl->recs, max, &nrec, &cons);
    if (nrec == 0)
        return perr;
    const ptls_mi355x_tls_record_t *last = rl->recs + nrec - 1;
    const size_t ptbytes = last->dst + (last->len >= 16u ? last->len - 16u : 0u);
    const size_t off_src = up16(nrec * sizeof(ptls_mi355x_tls_record_t)), off_dst = off_src + up16(cons);
    const size_t off_st = off_dst + up16(ptbytes), off_ty = off_st + up16(nrec * 4);
    if (reserve(rl, off_ty + up16(nrec), nrec) != 0)
        return -1;
    memcpy(rl->h_buf, rl->recs, nrec * sizeof(ptls_mi355x_tls_record_t));
    memcpy(rl->h_buf + off_src, in, cons);
    hipError_t e;
    if ((e = hipMemcpyAsync(rl->d_buf, rl->h_buf, off_src + cons, hipMemcpyHostToDevice, rl->stream)) != hipSuccess)
        return rl_fail("H2D", e);
    if (ptls_mi355x_tls_open_records_ex(rl->ctx, rl->iv, (const ptls_mi355x_tls_record_t *)rl->d_buf, NULL, nrec,
                                        rl->d_buf + off_src, rl->d_buf + off_dst, (uint32_t *)(rl->d_buf + off_st),
                                        rl->d_buf + off_ty, PTLS_MI355X_OPEN_STOP_AT_FAILURE, rl->stream) != 0) {
        snprintf(rl_err, sizeof(rl_err), "record layer: %s", ptls_mi355x_last_error());
        return -1;
    }
    if ((e = hipMemcpyAsync(rl->h_buf + off_dst, rl->d_buf + off_dst, off_ty + nrec - off_dst, hipMemcpyDeviceToHost,
                            rl->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(rl->stream)) != hipSuccess)
        return rl_fail("D2H", e);
    const uint32_t *status = (const uint32_t *)(rl->h_buf + off_st);
    const uint8_t *types = rl->h_buf + off_ty;
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
        memcpy((uint8_t *)out + olen, rl->h_buf + off_dst + rl->recs[i].dst, status[i]);
        olen += status[i];
        wire_done += PTLS_MI355X_TLS_HEADER_SIZE + rl->recs[i].len;
        ++done;
    }
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
