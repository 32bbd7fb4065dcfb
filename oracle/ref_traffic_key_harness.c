/*
 * oracle/ref_traffic_key_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the engine).
 *
 * The engine's record layer installed behind the REFERENCE picotls' own-record-layer hook and run against a
 * reference picotls peer.  picotls.c is compiled unmodified from /root/reference/lib (included into this unit for its
 * static functions and struct st_ptls_t); the peer's AEAD is the reference minicrypto AES-GCM (lib/cifra/aes{128,256}.c
 * over deps/cifra), an implementation independent of both the engine and fusion.
 *
 *   S  the GPU side: a ptls_t whose context sets update_traffic_key (lib/picotls.c:1206-1211), "the special path for
 *      applications having their own record layer".  Its callback (as C below) derives the
 *      key and IV from the secret as rapido does (ptls_hkdf_expand_label "key"/"iv", lib/rapido.c:135-150) and creates
 *      -- or, on a later epoch, rekeys -- a ptls_mi355x_record_layer for that direction.
 *   C  the peer: plain picotls, ptls_send / ptls_receive (lib/picotls.c:4913-4988) over minicrypto.
 *
 * Both hold the same application traffic secrets and key schedule (installed directly, as rapido installs its
 * connections' keys); setup_traffic_protection (lib/picotls.c:1190-1225) then invokes S's callback for both
 * directions.  The scenario, every byte checked:
 *   1. S seals send windows of 16 fragments with the layer; C's ptls_receive accepts them, the plaintext matches.
 *   2. C's ptls_send output (incl. a 40000-byte message) is opened by S's layer.
 *   3. C initiates a KeyUpdate (ptls_update_key; its next ptls_send emits KeyUpdate + data under the new key).  S's
 *      window open stops at the handshake record; open_record hands it over; ptls_handle_message processes it
 *      (handle_key_update -> update_traffic_key(tls, 0), whose setup_traffic_protection skips the callback:
 *      skip_notify), so the application re-invokes setup_traffic_protection for the new secret -> callback -> rekey;
 *      the rest of the window opens from seq 0.
 *   4. S initiates a KeyUpdate: the message sealed (type 22) under the old key, update_traffic_key(tls, 1), re-notify,
 *      and the next windows go out under the new key from seq 0; C's ptls_receive follows.
 *   5. The 2^24-record limit: both at seq 2^24 - 3, a 16-fragment window stops after 3 records
 *      (PTLS_MI355X_RECORD_LAYER_KEY_UPDATE); S runs step 4 and seals the other 13; C receives all 16 in order.
 *
 *   6. (argument "transfer") rapido's 1 MB stream (t/rapido_tests.c:290-340) both ways through the hook-installed
 *      layers: S -> C in rapido send windows of 16 x 16 KiB fragments (lib/rapido.c:2115-2126), C's ptls_receive
 *      checks every byte; C -> S by ptls_send, opened by S's layer in receive windows of at most 32 records
 *      (lib/rapido.c:2030).  Then the host-to-host rate of the same 1 MB, same key, IV and seq, three ways, each
 *      output compared byte for byte with the checked stream: the layer, one window at a time (rapido's loop); the
 *      layer with all four windows submitted at once; and the engine's AEAD slot as rapido uses it today -- ptls_send
 *      per 16 KiB record on a ptls_t whose traffic AEAD is ptls_mi355x_aes*gcm (ptls_set_traffic_protection,
 *      lib/rapido.c:135-200).  Receive the same way (the layer's windows; ptls_receive over the slot).
 *
 *   ref_traffic_key_harness <direct|dma|dma_in|zero_copy|copy> <16|32> [transfer]
 *       ->  prints "ok ..." (and with "transfer" a "rates ..." JSON line) and exits 0, or reports and exits 1
 */
#include <time.h>
#include "picotls.c" /* -I$(REF)/lib: the reference record layer and key schedule (static functions) */
#include "picotls/minicrypto.h"
#include "ptls_mi355x.h"

#define FAIL(...)                                                                                                      \
    do {                                                                                                               \
        fprintf(stderr, "traffic_key_harness: " __VA_ARGS__);                                                          \
        fprintf(stderr, " (line %d)\n", __LINE__);                                                                     \
        exit(1);                                                                                                       \
    } while (0)

static uint64_t rng_state = 0x243f6a8885a308d3ull;
static void fill_random(void *buf, size_t len)
{
    uint8_t *p = buf;
    for (size_t i = 0; i < len; ++i) {
        rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
        p[i] = (uint8_t)(rng_state >> 56);
    }
}

/* ---- the update_traffic_key callback of an application with its own record layer ---- */
struct gpu_record_layer_cb {
    ptls_update_traffic_key_t super;
    ptls_mi355x_record_layer_t *layer[2]; /* [is_enc] */
    uint32_t connection_id;               /* rapido: XORed into the IV's first four bytes */
    int direct_ranges;                    /* register the application's buffers below */
    void *ranges[4];
    size_t range_len[4], nranges;
    int zero_copy_off;
    int dma; /* registered ranges moved by DMA copies (1) or an open's input by DMA (2) instead of read in place */
    unsigned calls;
};

static int gpu_update_traffic_key(ptls_update_traffic_key_t *self, ptls_t *tls, int is_enc, size_t epoch, const void *secret)
{
    struct gpu_record_layer_cb *cb = (struct gpu_record_layer_cb *)self;
    ptls_cipher_suite_t *cs = ptls_get_cipher(tls);
    uint8_t key[PTLS_MAX_SECRET_SIZE], iv[PTLS_MAX_IV_SIZE];
    int ret;
    if (epoch != 3) /* handshake epochs stay on picotls' own path in this harness */
        return 0;
    if ((ret = ptls_hkdf_expand_label(cs->hash, key, cs->aead->key_size, ptls_iovec_init(secret, cs->hash->digest_size), "key",
                                      ptls_iovec_init(NULL, 0), tls->ctx->hkdf_label_prefix__obsolete)) != 0 ||
        (ret = ptls_hkdf_expand_label(cs->hash, iv, cs->aead->iv_size, ptls_iovec_init(secret, cs->hash->digest_size), "iv",
                                      ptls_iovec_init(NULL, 0), tls->ctx->hkdf_label_prefix__obsolete)) != 0)
        return ret;
    for (int i = 0; i < 4; ++i) /* derive_connection_aead_iv (lib/rapido.c:123-133) */
        iv[i] ^= (uint8_t)(cb->connection_id >> (24 - 8 * i));
    ptls_mi355x_record_layer_t **l = &cb->layer[is_enc != 0];
    if (*l == NULL) {
        if ((*l = ptls_mi355x_record_layer_new(key, cs->aead->key_size, iv, 0)) == NULL)
            ret = PTLS_ERROR_LIBRARY;
        for (size_t r = 0; ret == 0 && cb->direct_ranges && r < cb->nranges; ++r)
            if (ptls_mi355x_record_layer_register(*l, cb->ranges[r], cb->range_len[r]) != 0)
                ret = PTLS_ERROR_LIBRARY;
        if (ret == 0 && cb->zero_copy_off)
            ptls_mi355x_record_layer_set_zero_copy_bytes(*l, 0);
        if (ret == 0 && cb->dma)
            ptls_mi355x_record_layer_set_direct_dma(*l, cb->dma);
        /* every launch slot set up now, for rapido's windows: 16 send records, up to 32 received */
        if (ret == 0 && ptls_mi355x_record_layer_reserve(*l, (is_enc ? 16 : 32) * (16384 + PTLS_MI355X_TLS_OVERHEAD), 1) != 0)
            ret = PTLS_ERROR_LIBRARY;
    } else if (ptls_mi355x_record_layer_rekey(*l, key, cs->aead->key_size, iv) != 0) { /* a KeyUpdate epoch change */
        ret = PTLS_ERROR_LIBRARY;
    }
    ptls_clear_memory(key, sizeof(key));
    ptls_clear_memory(iv, sizeof(iv));
    ++cb->calls;
    return ret;
}
/* ---------------------------------------------------------------------------------------------------------------- */

static ptls_cipher_suite_t *suites128[] = {&ptls_minicrypto_aes128gcmsha256, NULL};
static ptls_cipher_suite_t *suites256[] = {&ptls_minicrypto_aes256gcmsha384, NULL};

/* a post-handshake ptls_t with the given application traffic secrets, its key schedule and cipher suite */
static ptls_t *session(ptls_context_t *ctx, int is_server, ptls_cipher_suite_t *cs, const uint8_t *enc_secret,
                       const uint8_t *dec_secret)
{
    ptls_t *tls = is_server ? ptls_server_new(ctx) : ptls_client_new(ctx);
    tls->cipher_suite = cs;
    tls->key_schedule = key_schedule_new(cs, NULL, ctx->hkdf_label_prefix__obsolete);
    tls->state = is_server ? PTLS_STATE_SERVER_POST_HANDSHAKE : PTLS_STATE_CLIENT_POST_HANDSHAKE;
    memcpy(tls->traffic_protection.enc.secret, enc_secret, cs->hash->digest_size);
    memcpy(tls->traffic_protection.dec.secret, dec_secret, cs->hash->digest_size);
    if (setup_traffic_protection(tls, 1, NULL, 3, 0) != 0 || setup_traffic_protection(tls, 0, NULL, 3, 0) != 0)
        FAIL("setup_traffic_protection");
    return tls;
}

static uint8_t *arena;
static size_t arena_off, arena_cap;
static uint8_t *take(size_t n)
{
    uint8_t *p = arena + arena_off;
    arena_off += (n + 63) & ~(size_t)63;
    if (arena_off > arena_cap)
        FAIL("arena exhausted");
    return p;
}

/* S seals frags through its enc layer; returns the wire bytes (in the arena) */
static int gpu_seal(struct gpu_record_layer_cb *cb, uint8_t **frag, size_t *len, size_t n, uint8_t type, uint8_t **wire,
                    size_t *wirelen, size_t *nrec)
{
    ptls_mi355x_iovec_t iov[32];
    size_t cap = 0;
    for (size_t i = 0; i < n; ++i) {
        iov[i] = (ptls_mi355x_iovec_t){frag[i], len[i]};
        cap += len[i] + (len[i] + 16383) / 16384 * PTLS_MI355X_TLS_OVERHEAD;
    }
    *wire = take(cap + 1);
    return ptls_mi355x_record_layer_seal(cb->layer[1], iov, n, type, *wire, cap, wirelen, nrec);
}

/* C receives wire with ptls_receive; the plaintext must equal the concatenation `want` */
static void peer_receive(ptls_t *c, const uint8_t *wire, size_t wirelen, const uint8_t *want, size_t wantlen)
{
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    size_t off = 0;
    while (off < wirelen) {
        size_t n = wirelen - off;
        int ret;
        if ((ret = ptls_receive(c, &buf, wire + off, &n)) != 0)
            FAIL("ptls_receive: %d at wire offset %zu", ret, off);
        off += n;
    }
    if (buf.off != wantlen || memcmp(buf.base, want, wantlen) != 0)
        FAIL("peer received %zu bytes, %zu expected, or other bytes", buf.off, wantlen);
    ptls_buffer_dispose(&buf);
}

/* S's application KeyUpdate (update_send_key, lib/picotls.c:4949-4962, for an own record layer) */
static void gpu_send_key_update(struct gpu_record_layer_cb *cb, ptls_t *s, ptls_t *c)
{
    static const uint8_t msg[5] = {PTLS_HANDSHAKE_TYPE_KEY_UPDATE, 0, 0, 1, 0};
    uint8_t *f = take(sizeof(msg)), *wire;
    memcpy(f, msg, sizeof(msg));
    size_t flen = sizeof(msg), wl, nr;
    unsigned calls = cb->calls;
    if (gpu_seal(cb, &f, &flen, 1, PTLS_CONTENT_TYPE_HANDSHAKE, &wire, &wl, &nr) != 0 || nr != 1)
        FAIL("seal of the KeyUpdate message: %s", ptls_mi355x_record_layer_last_error());
    /* the next application traffic secret; picotls skips the callback here (skip_notify), so the application
     * re-notifies itself through setup_traffic_protection, which hands the new secret to the callback */
    if (update_traffic_key(s, 1) != 0 || setup_traffic_protection(s, 1, NULL, 3, 0) != 0 || cb->calls != calls + 1)
        FAIL("send-side key update");
    if (ptls_mi355x_record_layer_get_seq(cb->layer[1]) != 0)
        FAIL("the new send key does not start at seq 0");
    peer_receive(c, wire, wl, NULL, 0); /* C: handle_key_update -> its new receive key */
    if (c->traffic_protection.dec.seq != 0)
        FAIL("peer did not switch its receive key");
}

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

#define XFER 1000000u /* t/rapido_tests.c:319: the 1 MB stream */
#define XWIN 16       /* fragments per send window (lib/rapido.c:2115-2126) */
#define XRECV 32      /* records per receive window (lib/rapido.c:2030) */

/* the stream's fragments: 16 KiB each (rapido's TCPLS records), the last one short */
static size_t xfer_frags(uint8_t *data, uint8_t **frag, size_t *len)
{
    size_t n = 0;
    for (size_t off = 0; off < XFER; off += 16384, ++n) {
        frag[n] = data + off;
        len[n] = XFER - off < 16384 ? XFER - off : 16384;
    }
    return n;
}

/* seal the stream through `rl` in windows of XWIN fragments into wire; depth 1: one window at a time (submit, wait),
 * else every window submitted, then waited.  Returns the wire bytes. */
static size_t layer_send(ptls_mi355x_record_layer_t *rl, uint8_t **frag, size_t *len, size_t nfrag, uint8_t *wire,
                         size_t cap, int all_at_once)
{
    ptls_mi355x_iovec_t iov[64];
    uint64_t ticket[8];
    void *out[8];
    size_t off = 0, nwin = 0, outcap[8], nf[8];
    for (size_t f = 0; f < nfrag; ++f)
        iov[f] = (ptls_mi355x_iovec_t){frag[f], len[f]};
    for (size_t f = 0; f < nfrag; f += XWIN, ++nwin) {
        nf[nwin] = nfrag - f < XWIN ? nfrag - f : XWIN;
        const ptls_mi355x_iovec_t *w = iov + f;
        size_t bytes = 0;
        for (size_t k = 0; k < nf[nwin]; ++k)
            bytes += len[f + k] + PTLS_MI355X_TLS_OVERHEAD;
        out[nwin] = wire + off;
        outcap[nwin] = bytes;
        off += bytes;
        if (off > cap || ptls_mi355x_record_layer_seal_submit(&rl, 1, &w, &nf[nwin], PTLS_CONTENT_TYPE_APPDATA, &out[nwin],
                                                              &outcap[nwin], &ticket[nwin]) != 0)
            FAIL("seal_submit: %s", ptls_mi355x_record_layer_last_error());
        if (!all_at_once) {
            size_t ol, nr, cons;
            int al;
            if (ptls_mi355x_record_layer_wait(rl, ticket[nwin], &ol, &nr, &cons, &al) != 0 || al != 0 || ol != outcap[nwin])
                FAIL("seal wait: %s", ptls_mi355x_record_layer_last_error());
        }
    }
    for (size_t w = 0; all_at_once && w < nwin; ++w) {
        size_t ol, nr, cons;
        int al;
        if (ptls_mi355x_record_layer_wait(rl, ticket[w], &ol, &nr, &cons, &al) != 0 || al != 0 || ol != outcap[w])
            FAIL("seal wait: %s", ptls_mi355x_record_layer_last_error());
    }
    return off;
}

/* open the wire through `rl` in receive windows of at most XRECV records into pt; returns the plaintext bytes */
static size_t layer_recv(ptls_mi355x_record_layer_t *rl, const uint8_t *wire, size_t wirelen, uint8_t *pt, size_t cap)
{
    size_t in = 0, got = 0;
    while (in < wirelen) {
        size_t win = 0, k = 0; /* XRECV complete records at most (a recv() of rapido's buffer) */
        while (k < XRECV && in + win + 5 <= wirelen) {
            const size_t rl_ = 5 + ((size_t)wire[in + win + 3] << 8 | wire[in + win + 4]);
            if (in + win + rl_ > wirelen)
                break;
            win += rl_;
            ++k;
        }
        size_t cons, olen, nrec;
        const double t0 = getenv("XFER_DEBUG") != NULL ? now() : 0;
        const int rc = ptls_mi355x_record_layer_open(rl, wire + in, win, &cons, pt + got, cap - got, &olen, &nrec);
        if (getenv("XFER_DEBUG") != NULL)
            fprintf(stderr, "open window of %zu records at +%zu: %.1f us\n", k, in, (now() - t0) * 1e6);
        if (rc != 0 || cons != win || nrec != k)
            FAIL("layer open: rc %d, %zu of %zu bytes: %s", rc, cons, win, ptls_mi355x_record_layer_last_error());
        in += cons;
        got += olen;
    }
    return got;
}

/* scenario 6: rapido's 1 MB stream through the hook-installed layers, then the rates (see the header) */
static void rapido_transfer(struct gpu_record_layer_cb *cb, ptls_t *s, ptls_t *c, ptls_cipher_suite_t *cs,
                            const char *transport, size_t keylen)
{
    uint8_t *data = take(XFER), *frag[64], *wire = take(XFER + 64 * PTLS_MI355X_TLS_OVERHEAD + 64), *pt = take(XFER + 64);
    size_t len[64];
    fill_random(data, XFER);
    const size_t nfrag = xfer_frags(data, frag, len);
    /* S -> C: the checked stream, from the send layer's current seq */
    const uint64_t seq0 = ptls_mi355x_record_layer_get_seq(cb->layer[1]);
    const size_t wl = layer_send(cb->layer[1], frag, len, nfrag, wire, XFER + 64 * PTLS_MI355X_TLS_OVERHEAD, 0);
    peer_receive(c, wire, wl, data, XFER);
    /* C -> S: ptls_send of the stream (rapido's per-record calls), the receive layer's windows */
    {
        ptls_buffer_t sb;
        ptls_buffer_init(&sb, "", 0);
        for (size_t f = 0; f < nfrag; ++f)
            if (ptls_send(c, &sb, frag[f], len[f]) != 0)
                FAIL("peer ptls_send");
        uint8_t *in = take(sb.off);
        memcpy(in, sb.base, sb.off);
        if (layer_recv(cb->layer[0], in, sb.off, pt, XFER + 64) != XFER || memcmp(pt, data, XFER) != 0)
            FAIL("the peer's 1 MB through the receive layer");
        ptls_buffer_dispose(&sb);
    }
    /* the rates: the same key, IV and seq as the checked stream; every output equal to it */
    uint8_t key[PTLS_MAX_SECRET_SIZE], iv[PTLS_MAX_IV_SIZE];
    if (ptls_hkdf_expand_label(cs->hash, key, cs->aead->key_size, ptls_iovec_init(s->traffic_protection.enc.secret,
                               cs->hash->digest_size), "key", ptls_iovec_init(NULL, 0), NULL) != 0 ||
        ptls_hkdf_expand_label(cs->hash, iv, cs->aead->iv_size, ptls_iovec_init(s->traffic_protection.enc.secret,
                               cs->hash->digest_size), "iv", ptls_iovec_init(NULL, 0), NULL) != 0)
        FAIL("key derivation");
    for (int i = 0; i < 4; ++i)
        iv[i] ^= (uint8_t)(cb->connection_id >> (24 - 8 * i));
    enum { REPS = 8 };
    double t_layer1 = 0, t_layer4 = 0, t_slot = 0, t_layer_recv = 0, t_slot_recv = 0;
    uint8_t *w2 = take(XFER + 64 * PTLS_MI355X_TLS_OVERHEAD + 64), *p2 = take(XFER + 64);
    /* long-lived layers and AEADs, as a connection's (set up by reserve; rep 0 untimed); every rep restarts them at
     * seq0, so each rep's output is the checked stream again */
    ptls_mi355x_record_layer_t *txs[2], *rxs[2];
    for (int mode = 0; mode < 2; ++mode) {
        ptls_mi355x_record_layer_t *tx = txs[mode] = ptls_mi355x_record_layer_new(key, keylen, iv, seq0),
                                   *rx = rxs[mode] = ptls_mi355x_record_layer_new(key, keylen, iv, seq0);
        if (tx == NULL || rx == NULL)
            FAIL("record_layer_new");
        if (cb->direct_ranges) {
            if (ptls_mi355x_record_layer_register(tx, arena, arena_cap) != 0 ||
                ptls_mi355x_record_layer_register(rx, arena, arena_cap) != 0)
                FAIL("register");
            if (cb->dma) {
                ptls_mi355x_record_layer_set_direct_dma(tx, cb->dma);
                ptls_mi355x_record_layer_set_direct_dma(rx, cb->dma);
            }
        }
        if (cb->zero_copy_off) {
            ptls_mi355x_record_layer_set_zero_copy_bytes(tx, 0);
            ptls_mi355x_record_layer_set_zero_copy_bytes(rx, 0);
        }
        /* a connection's layers set up once (without this, each slot's first window pays ~3 ms of setup) */
        if (ptls_mi355x_record_layer_reserve(tx, XWIN * (16384 + PTLS_MI355X_TLS_OVERHEAD), 1) != 0 ||
            ptls_mi355x_record_layer_reserve(rx, XRECV * (16384 + PTLS_MI355X_TLS_OVERHEAD), 1) != 0)
            FAIL("record_layer_reserve: %s", ptls_mi355x_record_layer_last_error());
    }
    /* the slot: ptls_send per record over a ptls_t whose traffic AEAD is the engine's (rapido today) */
    ptls_context_t ectx = {fill_random, &ptls_get_time};
    ptls_t *e = ptls_client_new(&ectx), *d = ptls_server_new(&ectx);
    {
        struct st_ptls_traffic_protection_t prot = {{0}}, dprot = {{0}};
        prot.aead = ptls_aead_new_direct(keylen == 32 ? &ptls_mi355x_aes256gcm : &ptls_mi355x_aes128gcm, 1, key, iv);
        dprot.aead = ptls_aead_new_direct(keylen == 32 ? &ptls_mi355x_aes256gcm : &ptls_mi355x_aes128gcm, 0, key, iv);
        if (prot.aead == NULL || dprot.aead == NULL)
            FAIL("ptls_aead_new_direct(engine)");
        ptls_set_traffic_protection(e, &prot, 0);
        ptls_set_traffic_protection(d, &dprot, 1);
        e->state = PTLS_STATE_CLIENT_POST_HANDSHAKE;
        d->state = PTLS_STATE_SERVER_POST_HANDSHAKE;
    }
    for (int rep = 0; rep < REPS + 1; ++rep) {
        for (int mode = 0; mode < 2; ++mode) {
            ptls_mi355x_record_layer_t *tx = txs[mode], *rx = rxs[mode];
            ptls_mi355x_record_layer_set_seq(tx, seq0);
            ptls_mi355x_record_layer_set_seq(rx, seq0);
            memset(w2, 0, wl);
            double t0 = now();
            const size_t n2 = layer_send(tx, frag, len, nfrag, w2, XFER + 64 * PTLS_MI355X_TLS_OVERHEAD, mode);
            const double dt = now() - t0;
            if (n2 != wl || memcmp(w2, wire, wl) != 0)
                FAIL("layer stream (mode %d) differs from the checked stream", mode);
            t0 = now();
            const size_t got = layer_recv(rx, w2, n2, p2, XFER + 64);
            const double dr = now() - t0;
            if (got != XFER || memcmp(p2, data, XFER) != 0)
                FAIL("layer receive of the stream");
            if (rep > 0) {
                *(mode ? &t_layer4 : &t_layer1) += dt;
                if (!mode)
                    t_layer_recv += dr;
            }
        }
        e->traffic_protection.enc.seq = seq0;
        d->traffic_protection.dec.seq = seq0;
        ptls_buffer_t sb;
        ptls_buffer_init(&sb, "", 0);
        double t0 = now();
        for (size_t f = 0; f < nfrag; ++f)
            if (ptls_send(e, &sb, frag[f], len[f]) != 0)
                FAIL("ptls_send over the engine slot");
        const double dt = now() - t0;
        if (sb.off != wl || memcmp(sb.base, wire, wl) != 0)
            FAIL("slot stream differs from the checked stream");
        ptls_buffer_t rb;
        ptls_buffer_init(&rb, "", 0);
        t0 = now();
        for (size_t off = 0; off < sb.off;) {
            size_t n = sb.off - off;
            if (ptls_receive(d, &rb, sb.base + off, &n) != 0)
                FAIL("ptls_receive over the engine slot");
            off += n;
        }
        const double dr = now() - t0;
        if (rb.off != XFER || memcmp(rb.base, data, XFER) != 0)
            FAIL("slot receive of the stream");
        if (rep > 0) {
            t_slot += dt;
            t_slot_recv += dr;
        }
        ptls_buffer_dispose(&sb);
        ptls_buffer_dispose(&rb);
    }
    ptls_free(e);
    ptls_free(d);
    for (int mode = 0; mode < 2; ++mode) {
        ptls_mi355x_record_layer_free(txs[mode]);
        ptls_mi355x_record_layer_free(rxs[mode]);
    }
    const double mb = XFER / 1e6 * REPS;
    printf("rates {\"transport\": \"%s\", \"key_bits\": %zu, \"stream_bytes\": %u, \"reps\": %d, "
           "\"layer_send_window_at_a_time_MBps\": %.1f, \"layer_send_all_windows_submitted_MBps\": %.1f, "
           "\"layer_recv_windows_of_32_MBps\": %.1f, \"slot_ptls_send_MBps\": %.1f, \"slot_ptls_receive_MBps\": %.1f}\n",
           transport, 8 * keylen, XFER, REPS, mb / t_layer1, mb / t_layer4, mb / t_layer_recv, mb / t_slot, mb / t_slot_recv);
    ptls_clear_memory(key, sizeof(key));
}

int main(int argc, char **argv)
{
    const char *transport = argc > 1 ? argv[1] : "zero_copy";
    const size_t keylen = argc > 2 ? (size_t)atoi(argv[2]) : 16;
    ptls_cipher_suite_t *cs = keylen == 32 ? suites256[0] : suites128[0];
    arena_cap = 48u << 20;
    if (posix_memalign((void **)&arena, 4096, arena_cap) != 0)
        return 1;
    memset(arena, 0, arena_cap);

    struct gpu_record_layer_cb cb = {{gpu_update_traffic_key}};
    cb.direct_ranges = strcmp(transport, "direct") == 0 || strcmp(transport, "dma") == 0 || strcmp(transport, "dma_in") == 0;
    cb.dma = strcmp(transport, "dma") == 0 ? 1 : strcmp(transport, "dma_in") == 0 ? PTLS_MI355X_RECORD_LAYER_DMA_IN : 0;
    cb.zero_copy_off = strcmp(transport, "copy") == 0;
    cb.ranges[0] = arena;
    cb.range_len[0] = arena_cap;
    cb.nranges = 1;
    ptls_context_t ctx_s = {fill_random, &ptls_get_time}, ctx_c = ctx_s;
    ctx_s.cipher_suites = ctx_c.cipher_suites = keylen == 32 ? suites256 : suites128;
    ctx_s.update_traffic_key = &cb.super;

    uint8_t c2s[PTLS_MAX_DIGEST_SIZE], s2c[PTLS_MAX_DIGEST_SIZE];
    fill_random(c2s, sizeof(c2s));
    fill_random(s2c, sizeof(s2c));
    ptls_t *s = session(&ctx_s, 1, cs, s2c, c2s), *c = session(&ctx_c, 0, cs, c2s, s2c);
    if (cb.calls != 2 || cb.layer[0] == NULL || cb.layer[1] == NULL)
        FAIL("setup_traffic_protection did not install both directions through the callback (%u calls)", cb.calls);
    size_t checks = 0;

    /* 1. S -> C: send windows of 16 fragments through the layer, ptls_receive on the peer */
    for (int w = 0; w < 3; ++w) {
        uint8_t *frag[16], *wire, *all = take(16 * 16384);
        size_t len[16], total = 0, wl, nr;
        for (int i = 0; i < 16; ++i) {
            uint32_t r;
            fill_random(&r, sizeof(r));
            len[i] = w == 0 ? 16384 : w == 2 && i == 5 ? 0 : 1 + r % 16384;
            frag[i] = take(len[i]);
            fill_random(frag[i], len[i]);
            memcpy(all + total, frag[i], len[i]);
            total += len[i];
        }
        if (gpu_seal(&cb, frag, len, 16, PTLS_CONTENT_TYPE_APPDATA, &wire, &wl, &nr) != 0 || nr != (w == 2 ? 15u : 16u))
            FAIL("seal window %d: %s", w, ptls_mi355x_record_layer_last_error());
        peer_receive(c, wire, wl, all, total);
        ++checks;
    }
    /* 2. C -> S: ptls_send output opened by the layer */
    {
        ptls_buffer_t sb;
        ptls_buffer_init(&sb, "", 0);
        uint8_t *msgs = take(40000 + 5000 + 1);
        fill_random(msgs, 45001);
        if (ptls_send(c, &sb, msgs, 40000) != 0 || ptls_send(c, &sb, msgs + 40000, 5000) != 0 ||
            ptls_send(c, &sb, msgs + 45000, 1) != 0)
            FAIL("peer ptls_send");
        uint8_t *in = take(sb.off), *out = take(sb.off);
        memcpy(in, sb.base, sb.off);
        size_t cons, olen, nrec;
        int rc = ptls_mi355x_record_layer_open(cb.layer[0], in, sb.off, &cons, out, sb.off, &olen, &nrec);
        if (rc != 0 || cons != sb.off || olen != 45001 || nrec != 5 || memcmp(out, msgs, 45001) != 0)
            FAIL("open of the peer's records: rc %d, %zu of %zu bytes, %zu records", rc, cons, sb.off, nrec);
        if (ptls_mi355x_record_layer_get_seq(cb.layer[0]) != c->traffic_protection.enc.seq)
            FAIL("receive seq differs from the peer's send seq");
        ptls_buffer_dispose(&sb);
        ++checks;
    }
    /* 3. C initiates a KeyUpdate: KeyUpdate record (old key) + data (new key, seq 0) in one flight */
    {
        if (ptls_update_key(c, 0) != 0)
            FAIL("ptls_update_key");
        ptls_buffer_t sb;
        ptls_buffer_init(&sb, "", 0);
        uint8_t *msg = take(20000);
        fill_random(msg, 20000);
        if (ptls_send(c, &sb, msg, 20000) != 0 || c->traffic_protection.enc.seq != 2)
            FAIL("peer ptls_send after ptls_update_key");
        uint8_t *in = take(sb.off), *out = take(sb.off);
        memcpy(in, sb.base, sb.off);
        size_t cons, olen, nrec;
        int rc = ptls_mi355x_record_layer_open(cb.layer[0], in, sb.off, &cons, out, sb.off, &olen, &nrec);
        if (rc != 0 || cons != 0 || nrec != 0)
            FAIL("window open did not stop at the KeyUpdate record (rc %d, %zu consumed)", rc, cons);
        uint8_t type = 0;
        rc = ptls_mi355x_record_layer_open_record(cb.layer[0], in, sb.off, &cons, out, sb.off, &olen, &type);
        if (rc != 0 || type != PTLS_CONTENT_TYPE_HANDSHAKE || olen != 5 || out[0] != PTLS_HANDSHAKE_TYPE_KEY_UPDATE)
            FAIL("open_record of the KeyUpdate: rc %d, type %u, %zu bytes", rc, type, olen);
        unsigned calls = cb.calls;
        size_t epoch_offsets[5] = {0};
        ptls_buffer_t hs;
        ptls_buffer_init(&hs, "", 0);
        if ((rc = ptls_handle_message(s, &hs, epoch_offsets, 3, out, olen, NULL)) != 0)
            FAIL("ptls_handle_message(KeyUpdate): %d", rc);
        ptls_buffer_dispose(&hs);
        if (cb.calls != calls || setup_traffic_protection(s, 0, NULL, 3, 0) != 0 || cb.calls != calls + 1)
            FAIL("receive-side re-notification");
        if (ptls_mi355x_record_layer_get_seq(cb.layer[0]) != 0)
            FAIL("the new receive key does not start at seq 0");
        size_t cons2;
        rc = ptls_mi355x_record_layer_open(cb.layer[0], in + cons, sb.off - cons, &cons2, out, sb.off, &olen, &nrec);
        if (rc != 0 || cons + cons2 != sb.off || olen != 20000 || nrec != 2 || memcmp(out, msg, 20000) != 0)
            FAIL("records under the peer's new key: rc %d, %zu bytes", rc, olen);
        ptls_buffer_dispose(&sb);
        ++checks;
    }
    /* 4. S initiates a KeyUpdate, then a window under the new key */
    {
        gpu_send_key_update(&cb, s, c);
        uint8_t *frag[4], *wire, *all = take(4 * 3000);
        size_t len[4], total = 0, wl, nr;
        for (int i = 0; i < 4; ++i) {
            len[i] = 3000 - 100 * i;
            frag[i] = take(len[i]);
            fill_random(frag[i], len[i]);
            memcpy(all + total, frag[i], len[i]);
            total += len[i];
        }
        if (gpu_seal(&cb, frag, len, 4, PTLS_CONTENT_TYPE_APPDATA, &wire, &wl, &nr) != 0 || nr != 4)
            FAIL("seal after the key update");
        peer_receive(c, wire, wl, all, total);
        ++checks;
    }
    /* 5. the 2^24-record limit: a window stops after 3 records; KeyUpdate; the other 13 under the next key */
    {
        ptls_mi355x_record_layer_set_seq(cb.layer[1], PTLS_MI355X_RECORD_LAYER_SEQ_LIMIT - 3);
        c->traffic_protection.dec.seq = PTLS_MI355X_RECORD_LAYER_SEQ_LIMIT - 3;
        uint8_t *frag[16], *wire, *all = take(16 * 2048);
        size_t len[16], total = 0, wl, nr;
        for (int i = 0; i < 16; ++i) {
            len[i] = 1000 + 50 * i;
            frag[i] = take(len[i]);
            fill_random(frag[i], len[i]);
            memcpy(all + total, frag[i], len[i]);
            total += len[i];
        }
        int rc = gpu_seal(&cb, frag, len, 16, PTLS_CONTENT_TYPE_APPDATA, &wire, &wl, &nr);
        if (rc != PTLS_MI355X_RECORD_LAYER_KEY_UPDATE || nr != 3 ||
            ptls_mi355x_record_layer_get_seq(cb.layer[1]) != PTLS_MI355X_RECORD_LAYER_SEQ_LIMIT)
            FAIL("window at the limit: rc %d, %zu records", rc, nr);
        size_t first = len[0] + len[1] + len[2];
        peer_receive(c, wire, wl, all, first);
        gpu_send_key_update(&cb, s, c);
        if (gpu_seal(&cb, frag + 3, len + 3, 13, PTLS_CONTENT_TYPE_APPDATA, &wire, &wl, &nr) != 0 || nr != 13)
            FAIL("rest of the window under the next key");
        peer_receive(c, wire, wl, all + first, total - first);
        ++checks;
    }
    if (argc > 3 && strcmp(argv[3], "transfer") == 0) {
        rapido_transfer(&cb, s, c, cs, transport, keylen);
        checks += 2;
    }
    printf("ok: %zu checks (%s scenarios), transport %s, AES-%zu, %u update_traffic_key callbacks\n", checks,
           argc > 3 && strcmp(argv[3], "transfer") == 0 ? "6" : "5", transport, 8 * keylen, cb.calls);
    ptls_free(s);
    ptls_free(c);
    ptls_mi355x_record_layer_free(cb.layer[0]);
    ptls_mi355x_record_layer_free(cb.layer[1]);
    free(arena);
    return 0;
}
