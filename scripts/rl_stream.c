/*
 * scripts/rl_stream.c -- measurement driver (not part of the product library): the host-to-host rate of the
 * asynchronous record layer (include/ptls_mi355x.h section 5) on a stream of rapido windows, driven from C as rapido
 * itself would drive it (its send loop, lib/rapido.c:2176-2301, keeps many windows moving; a window is 16 records of
 * 16 KiB, :2115-2126).
 *
 *   rl_stream [nwin] [depth] [key_bytes] [transport: direct|dma|dma_in|zero_copy|copy] [windows per launch]
 *             [one | sessions | sessions_apart]
 *   (windows per launch > 1: windows of that many connections of one session per launch; with "one" consecutive
 *   windows of one connection; with "sessions" windows of that many sessions -- each its own key and IV -- per launch
 *   (a multi-key launch); with "sessions_apart" the same sessions, each window submitted on its own, as a server
 *   without multi-key launches runs them)
 *
 * nwin windows are sealed from one host buffer into another with `depth` windows in flight (seal_submit, and the wait
 * of the oldest once `depth` are outstanding), then opened back the same way; the clock is CLOCK_MONOTONIC from the
 * first submit to the last wait, after one untimed pass.  Every opened window is compared with its fragments.  Prints
 * one JSON object.  Built by rapido_amd/build.py into scripts/_build/rl_stream; run by bench.py's record_layer_stream.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <signal.h>
#include <execinfo.h>
#include <unistd.h>
#include "../include/ptls_mi355x.h"

static void on_fault(int sig)
{
    void *bt[32];
    const int n = backtrace(bt, 32);
    fprintf(stderr, "rl_stream: signal %d\n", sig);
    backtrace_symbols_fd(bt, n, 2);
    _exit(128 + sig);
}

#define WIN 16
#define FRAG 16384
#define WIRE_WIN (WIN * (FRAG + PTLS_MI355X_TLS_OVERHEAD))
#define PT_WIN (WIN * (FRAG + 1))
#define MAXM 16 /* windows per launch */

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *page_alloc(size_t n)
{
    void *p = NULL;
    if (posix_memalign(&p, 4096, n) != 0)
        return NULL;
    memset(p, 0, n);
    return p;
}

static void die(const char *what)
{
    fprintf(stderr, "rl_stream: %s: %s\n", what, ptls_mi355x_record_layer_last_error());
    exit(1);
}

typedef struct {
    ptls_mi355x_record_layer_t *tx, *rx;
    ptls_mi355x_record_layer_t *txs[MAXM], *rxs[MAXM]; /* multi: the windows of `multi` connections per launch */
    size_t multi;
    int apart; /* sessions_apart: window w on layer w % multi, one window per submit */
    uint8_t *send, *wire, *pt;
    ptls_mi355x_iovec_t (*frags)[WIN];
    size_t nwin;
} stream_t;

/* one pass: seal every window (depth in flight), or open every window */
static double pass(stream_t *st, int seal, size_t depth, size_t max_inflight_seen[1])
{
    ptls_mi355x_record_layer_t *rl = seal ? st->tx : st->rx;
    ptls_mi355x_record_layer_t *tick_rl[64];
    uint64_t tickets[64], head = 0, tail = 0;
    ptls_mi355x_record_layer_set_seq(rl, 0);
    for (size_t c = 0; st->multi > 1 && c < st->multi; ++c) { /* each connection's windows: its own seq from 0 */
        ptls_mi355x_record_layer_set_seq(st->txs[c], 0);
        ptls_mi355x_record_layer_set_seq(st->rxs[c], 0);
    }
    const double t0 = now();
    /* RL_TRACE=<us>: every wait or submit over that many microseconds (default 1000), to stderr */
    const double trace = getenv("RL_TRACE") != NULL ? (atof(getenv("RL_TRACE")) > 0 ? atof(getenv("RL_TRACE")) : 1000) * 1e-6 : 0;
    for (size_t w = 0; w < st->nwin + depth; ++w) {
        if (tail - head == depth || (w >= st->nwin && tail != head)) {
            size_t outlen[MAXM], nrec[MAXM], cons[MAXM];
            int alert[MAXM];
            const double tw = now();
            if (ptls_mi355x_record_layer_wait(tick_rl[head % 64], tickets[head % 64], outlen, nrec, cons, alert) != 0)
                die("wait");
            if (trace > 0 && now() - tw > trace)
                fprintf(stderr, "rl_stream: %s wait for window %zu took %.3f ms (launches %llu)\n", seal ? "seal" : "open",
                        (size_t)head, (now() - tw) * 1e3,
                        (unsigned long long)ptls_mi355x_record_layer_launches(rl));
            for (size_t c = 0; c < (st->multi > 1 && !st->apart ? st->multi : 1); ++c)
                if (nrec[c] != WIN || alert[c] != 0 || outlen[c] != (seal ? (size_t)WIRE_WIN : (size_t)WIN * FRAG)) {
                    fprintf(stderr, "rl_stream: window %zu: %zu records, %zu bytes, alert %d\n", (size_t)head, nrec[c],
                            outlen[c], alert[c]);
                    exit(1);
                }
            ++head;
        }
        if (w >= st->nwin)
            continue;
        if (st->apart) { /* window w alone, on session w % multi */
            ptls_mi355x_record_layer_t *x = seal ? st->txs[w % st->multi] : st->rxs[w % st->multi];
            const ptls_mi355x_iovec_t *f = st->frags[w];
            const size_t nf = WIN, cap = seal ? WIRE_WIN : PT_WIN, inlen = WIRE_WIN;
            void *out = seal ? st->wire + w * WIRE_WIN : st->pt + w * PT_WIN;
            const void *in = st->wire + w * WIRE_WIN;
            size_t parsed;
            tick_rl[tail % 64] = x;
            if ((seal ? ptls_mi355x_record_layer_seal_submit(&x, 1, &f, &nf, 23, &out, &cap, &tickets[tail % 64])
                      : ptls_mi355x_record_layer_open_submit(&x, 1, &in, &inlen, &out, &cap, &parsed,
                                                             &tickets[tail % 64])) != 0)
                die("submit");
        } else if (st->multi > 1) { /* windows w .. w + multi - 1 as `multi` connections of one launch (_multi) */
            const ptls_mi355x_iovec_t *f[MAXM];
            size_t nf[MAXM], cap[MAXM], inlen[MAXM], parsed[MAXM];
            void *out[MAXM];
            const void *in[MAXM];
            for (size_t c = 0; c < st->multi; ++c) {
                f[c] = st->frags[w + c];
                nf[c] = WIN;
                cap[c] = seal ? WIRE_WIN : PT_WIN;
                out[c] = seal ? st->wire + (w + c) * WIRE_WIN : st->pt + (w + c) * PT_WIN;
                in[c] = st->wire + (w + c) * WIRE_WIN;
                inlen[c] = WIRE_WIN;
            }
            tick_rl[tail % 64] = seal ? st->txs[0] : st->rxs[0];
            if ((seal ? ptls_mi355x_record_layer_seal_submit(st->txs, st->multi, f, nf, 23, out, cap, &tickets[tail % 64])
                      : ptls_mi355x_record_layer_open_submit(st->rxs, st->multi, in, inlen, out, cap, parsed,
                                                             &tickets[tail % 64])) != 0)
                die("multi submit");
            w += st->multi - 1;
        } else if (seal) {
            const ptls_mi355x_iovec_t *f = st->frags[w];
            const size_t nf = WIN, cap = WIRE_WIN;
            void *out = st->wire + w * WIRE_WIN;
            const double ts = now();
            tick_rl[tail % 64] = rl;
            if (ptls_mi355x_record_layer_seal_submit(&st->tx, 1, &f, &nf, 23, &out, &cap, &tickets[tail % 64]) != 0)
                die("seal_submit");
            if (trace > 0 && now() - ts > trace)
                fprintf(stderr, "rl_stream: seal submit of window %zu took %.3f ms\n", w, (now() - ts) * 1e3);
        } else {
            const void *in = st->wire + w * WIRE_WIN;
            const size_t inlen = WIRE_WIN, cap = PT_WIN;
            void *out = st->pt + w * PT_WIN;
            size_t parsed;
            const double ts = now();
            tick_rl[tail % 64] = rl;
            if (ptls_mi355x_record_layer_open_submit(&st->rx, 1, &in, &inlen, &out, &cap, &parsed, &tickets[tail % 64]) != 0)
                die("open_submit");
            if (trace > 0 && now() - ts > trace)
                fprintf(stderr, "rl_stream: open submit of window %zu took %.3f ms\n", w, (now() - ts) * 1e3);
        }
        ++tail;
        if (tail - head > max_inflight_seen[0])
            max_inflight_seen[0] = tail - head;
    }
    return now() - t0;
}

int main(int argc, char **argv)
{
    const size_t nwin = argc > 1 ? (size_t)atoi(argv[1]) : 64, depth = argc > 2 ? (size_t)atoi(argv[2]) : 4;
    const size_t key_bytes = argc > 3 ? (size_t)atoi(argv[3]) : 16;
    const char *transport = argc > 4 ? argv[4] : "direct";
    const size_t multi = argc > 5 ? (size_t)atoi(argv[5]) : 1; /* windows per launch (_multi) */
    const int one_conn = argc > 6 && strcmp(argv[6], "one") == 0; /* ... of one connection instead of `multi` */
    const int sessions = argc > 6 && strncmp(argv[6], "sessions", 8) == 0; /* ... of `multi` sessions (own keys) */
    const int apart = argc > 6 && strcmp(argv[6], "sessions_apart") == 0;
    if (depth < 1 || depth > 32 || nwin < 1 || (key_bytes != 16 && key_bytes != 32) || multi < 1 || multi > MAXM ||
        nwin % multi != 0) {
        fprintf(stderr, "usage: rl_stream [nwin] [depth 1..32] [16|32] [direct|dma|dma_in|zero_copy|copy] "
                        "[windows per launch 1..16] [one|sessions|sessions_apart]\n");
        return 2;
    }
    signal(SIGSEGV, on_fault);
    stream_t st = {0};
    st.nwin = nwin;
    st.multi = multi;
    st.apart = apart && multi > 1;
    uint8_t key[32], iv[12];
    uint64_t x = 0x9e3779b97f4a7c15ull;
    for (size_t i = 0; i < 32; ++i)
        key[i] = (uint8_t)((x = x * 6364136223846793005ull + 1442695040888963407ull) >> 56);
    for (size_t i = 0; i < 12; ++i)
        iv[i] = (uint8_t)((x = x * 6364136223846793005ull + 1442695040888963407ull) >> 56);
    st.send = page_alloc(nwin * WIN * FRAG);
    st.wire = page_alloc(nwin * WIRE_WIN);
    st.pt = page_alloc(nwin * PT_WIN);
    st.frags = malloc(nwin * sizeof(*st.frags));
    if (st.send == NULL || st.wire == NULL || st.pt == NULL || st.frags == NULL)
        return 1;
    for (size_t i = 0; i < nwin * WIN * FRAG; i += 8) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        memcpy(st.send + i, &x, 8);
    }
    for (size_t w = 0; w < nwin; ++w)
        for (size_t i = 0; i < WIN; ++i)
            st.frags[w][i] = (ptls_mi355x_iovec_t){st.send + (w * WIN + i) * FRAG, FRAG};
    if ((st.tx = ptls_mi355x_record_layer_new(key, key_bytes, iv, 0)) == NULL ||
        (st.rx = ptls_mi355x_record_layer_new(key, key_bytes, iv, 0)) == NULL)
        die("record_layer_new");
    for (size_t c = 0; multi > 1 && c < multi; ++c) { /* connection c: IV bytes 0..3 ^ BE32(c) (lib/rapido.c:123-133) */
        uint8_t civ[12], ckey[32];
        memcpy(civ, iv, 12);
        memcpy(ckey, key, 32);
        civ[3] ^= (uint8_t)c;
        if (sessions && c > 0) { /* session c: its own traffic key and IV (lib/rapido.c:135-200) */
            ckey[0] ^= (uint8_t)(c * 37 + 1);
            civ[7] ^= (uint8_t)(c * 11 + 1);
        }
        if (one_conn && c > 0) { /* the same connection again: its next window in the same launch */
            st.txs[c] = st.txs[0];
            st.rxs[c] = st.rxs[0];
            continue;
        }
        if ((st.txs[c] = ptls_mi355x_record_layer_new(ckey, key_bytes, civ, 0)) == NULL ||
            (st.rxs[c] = ptls_mi355x_record_layer_new(ckey, key_bytes, civ, 0)) == NULL)
            die("record_layer_new");
    }
    ptls_mi355x_record_layer_t *all[2 + 2 * MAXM] = {st.tx, st.rx};
    size_t nall = 2;
    for (size_t c = 0; multi > 1 && c < (one_conn ? 1 : multi); ++c) {
        all[nall++] = st.txs[c];
        all[nall++] = st.rxs[c];
    }
    const char *co = getenv("RL_COALESCE"); /* windows per launch when coalescing (0/1: off; default 16) */
    for (size_t i = 0; co != NULL && i < nall; ++i)
        ptls_mi355x_record_layer_set_coalesce(all[i], (size_t)atoi(co));
    for (size_t i = 0; i < nall; ++i) {
        if (strcmp(transport, "direct") == 0 || strcmp(transport, "dma") == 0 || strcmp(transport, "dma_in") == 0) {
            if (ptls_mi355x_record_layer_register(all[i], st.send, nwin * WIN * FRAG) != 0 ||
                ptls_mi355x_record_layer_register(all[i], st.wire, nwin * WIRE_WIN) != 0 ||
                ptls_mi355x_record_layer_register(all[i], st.pt, nwin * PT_WIN) != 0)
                die("register");
            ptls_mi355x_record_layer_set_direct_dma(all[i], strcmp(transport, "dma") == 0      ? 1
                                                            : strcmp(transport, "dma_in") == 0 ? PTLS_MI355X_RECORD_LAYER_DMA_IN
                                                                                               : 0);
        } else if (strcmp(transport, "copy") == 0) {
            ptls_mi355x_record_layer_set_zero_copy_bytes(all[i], 0);
        }
    }
    size_t inflight = 0;
    double t_seal = 0, t_open = 0, t_seal1 = 0, t_open1 = 0;
    pass(&st, 1, depth, &inflight); /* untimed: every slot's stream, context and staging created */
    pass(&st, 0, depth, &inflight);
    /* launches: the lead layer's, or every session's own when they submit apart */
    uint64_t l0s = 0, l0o = 0, l1s = 0, l1o = 0;
    for (size_t c = 0; c < (st.apart ? multi : 1); ++c) {
        l0s += ptls_mi355x_record_layer_launches(multi > 1 ? st.txs[c] : st.tx);
        l0o += ptls_mi355x_record_layer_launches(multi > 1 ? st.rxs[c] : st.rx);
    }
    t_seal = pass(&st, 1, depth, &inflight);
    for (size_t c = 0; c < (st.apart ? multi : 1); ++c)
        l1s += ptls_mi355x_record_layer_launches(multi > 1 ? st.txs[c] : st.tx);
    t_open = pass(&st, 0, depth, &inflight);
    for (size_t c = 0; c < (st.apart ? multi : 1); ++c)
        l1o += ptls_mi355x_record_layer_launches(multi > 1 ? st.rxs[c] : st.rx);
    t_seal1 = pass(&st, 1, 1, &inflight);
    t_open1 = pass(&st, 0, 1, &inflight);
    for (size_t w = 0; w < nwin; ++w) {
        if (memcmp(st.pt + w * PT_WIN, st.send + w * WIN * FRAG, (size_t)WIN * FRAG) != 0) {
            fprintf(stderr, "rl_stream: window %zu opened to other bytes than its fragments\n", w);
            return 1;
        }
    }
    const double bytes = (double)nwin * WIN * FRAG, gib = (double)(1u << 30);
    printf("{\"seal_gibps\": %.2f, \"open_gibps\": %.2f, \"seal_us_per_window\": %.2f, \"open_us_per_window\": %.2f, "
           "\"seal_gibps_sync\": %.2f, \"open_gibps_sync\": %.2f, \"windows\": %zu, \"depth\": %zu, \"max_in_flight\": %zu, "
           "\"transport\": \"%s\", \"key_bits\": %zu, \"windows_per_launch\": %zu, \"connections_per_launch\": %zu, "
           "\"seal_launches\": %llu, \"open_launches\": %llu, \"sessions\": \"%s\"}\n",
           bytes / t_seal / gib, bytes / t_open / gib, t_seal / nwin * 1e6, t_open / nwin * 1e6, bytes / t_seal1 / gib,
           bytes / t_open1 / gib, nwin, depth, inflight, transport, 8 * key_bytes, multi, one_conn ? (size_t)1 : multi,
           (unsigned long long)(l1s - l0s), (unsigned long long)(l1o - l0o),
           apart ? "apart" : sessions ? "one launch" : "one session");
    for (size_t i = 0; i < nall; ++i)
        ptls_mi355x_record_layer_free(all[i]);
    free(st.send);
    free(st.wire);
    free(st.pt);
    free(st.frags);
    return 0;
}
