/*
 * tls_records.c -- host-side planning for the TLS 1.3 framing batch (include/ptls_mi355x.h
 * section 4): the sequential, byte-cheap parts of picotls's record layer that decide WHICH
 * records a send or receive window holds, so the kernels can frame or unframe all of them in
 * one launch.  No device access.
 */
#include <stddef.h>
#include <stdint.h>
#include "../../include/ptls_mi355x.h"

/* buffer_push_encrypted_records (lib/picotls.c:664-684): <= 16384-byte chunks, one seq each */
size_t ptls_mi355x_tls_plan_send(size_t len, uint32_t type, uint64_t *seq, uint64_t src_off, uint64_t dst_off,
                                 ptls_mi355x_tls_record_t *recs, size_t max, size_t *wire_len)
{
    size_t n = 0, wire = 0;
    uint64_t s = *seq;
    while (len != 0) {
        size_t chunk = len < PTLS_MI355X_TLS_MAX_FRAGMENT ? len : PTLS_MI355X_TLS_MAX_FRAGMENT;
        if (recs != NULL) {
            if (n == max)
                break;
            recs[n].src = src_off;
            recs[n].dst = dst_off + wire;
            recs[n].seq = s;
            recs[n].len = (uint32_t)chunk;
            recs[n].type = type;
        }
        ++n;
        ++s;
        wire += chunk + PTLS_MI355X_TLS_OVERHEAD;
        src_off += chunk;
        len -= chunk;
    }
    if (recs != NULL)
        *seq = s;
    if (wire_len != NULL)
        *wire_len = wire;
    return n;
}

/* parse_record fast path + parse_record_header (lib/picotls.c:4243-4268) over a receive window */
int ptls_mi355x_tls_parse_records(const uint8_t *wire, size_t len, uint64_t src_off, uint64_t *seq, uint64_t dst_off,
                                  ptls_mi355x_tls_record_t *recs, size_t max, size_t *nrecs, size_t *consumed)
{
    size_t off = 0, n = 0;
    uint64_t pt = dst_off;
    int ret = 0;
    while (n < max && len - off >= PTLS_MI355X_TLS_HEADER_SIZE) {
        const uint8_t *h = wire + off;
        const uint32_t reclen = (uint32_t)h[3] << 8 | h[4];
        if (h[0] != 23) /* not application_data: the caller's slot path (alerts, CCS, handshake) */
            break;
        if (reclen > PTLS_MI355X_TLS_MAX_RECORD) {
            ret = 50; /* PTLS_ALERT_DECODE_ERROR */
            break;
        }
        if (len - off < PTLS_MI355X_TLS_HEADER_SIZE + (size_t)reclen) /* incomplete: wait for more bytes */
            break;
        recs[n].src = src_off + off;
        recs[n].dst = pt;
        recs[n].seq = *seq + n;
        recs[n].len = reclen;
        recs[n].type = 0;
        pt += reclen >= 16u ? reclen - 16u : 0u;
        off += PTLS_MI355X_TLS_HEADER_SIZE + reclen;
        ++n;
    }
    *seq += n;
    *nrecs = n;
    *consumed = off;
    return ret;
}
