/*
 * oracle/ref_rapido_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the engine).
 *
 * rapido itself, unchanged, over the engine: lib/rapido.c and lib/picotls.c compiled unmodified from /root/reference,
 * driven through rapido's public API over loopback TCP.  The reference's own suite t/rapido_tests.c cannot be built
 * here (it needs deps/picotest, an un-vendored submodule whose directory is empty), so the scenarios below restate its
 * transfer tests (t/rapido_tests.c:290-340 test_large_transfer, :347-420 test_join) with this file's CHECK instead of
 * picotest's ok().
 *
 * The ptls_context_t the sessions run with is the only choice made here: its cipher_suites hold the engine,
 *
 *     {TLS_AES_128_GCM_SHA256, &ptls_mi355x_aes128gcm, &ptls_minicrypto_sha256}   (or the AES-256 / SHA-384 suite)
 *
 * so every TLS record picotls and rapido protect -- the handshake's, and every TCPLS record of every connection under
 * its connection's IV (derive_connection_aead_iv, lib/rapido.c:127-133; ptls_aead_new_direct(cipher->aead, ...),
 * lib/rapido.c:158-190) -- goes through the engine's slot.  Key exchange and the certificate are the reference
 * minicrypto's (x25519, the secp256r1 certificate of t/test.h).  In the mixed scenario one side runs the minicrypto
 * suite with the same id, an AES-GCM independent of the engine and of fusion.
 *
 *   ref_rapido_harness <16|32> [minicrypto]   -> "ok N checks ..." (exit 0) or "not ok ..." lines (exit 1);
 *   "minicrypto" runs the harness itself with minicrypto in place of the engine (CPU, no GPU)
 */
#include "picotls.h"
#include "picotls/minicrypto.h"
#include "ptls_mi355x.h"
#include "rapido.h"
#include "rapido_internals.h"
#include "test.h"
#include <netdb.h>
#include <resolv.h>

static int n_ok, n_fail;
#define CHECK(cond)                                                                                                    \
    do {                                                                                                               \
        if (cond) {                                                                                                    \
            ++n_ok;                                                                                                    \
        } else {                                                                                                       \
            ++n_fail;                                                                                                  \
            printf("not ok - %s (%s:%d)\n", #cond, __FILE__, __LINE__);                                                \
        }                                                                                                              \
    } while (0)

#define RUN_TIMEOUT 500 /* RUN_NETWORK_TIMEOUT_DEFAULT, t/rapido_tests.c:14 */

static ptls_cipher_suite_t mi355x_aes128gcmsha256 = {PTLS_CIPHER_SUITE_AES_128_GCM_SHA256, &ptls_mi355x_aes128gcm,
                                                     &ptls_minicrypto_sha256};
static ptls_cipher_suite_t mi355x_aes256gcmsha384 = {PTLS_CIPHER_SUITE_AES_256_GCM_SHA384, &ptls_mi355x_aes256gcm,
                                                     &ptls_minicrypto_sha384};

static int loopback(const char *port, struct sockaddr_in *a, socklen_t *len)
{
    struct addrinfo hints = {0}, *res;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    hints.ai_protocol = IPPROTO_TCP;
    if (getaddrinfo("127.0.0.1", port, &hints, &res) != 0)
        return -1;
    memcpy(a, res->ai_addr, res->ai_addrlen);
    *len = res->ai_addrlen;
    freeaddrinfo(res);
    return 0;
}

static void fill(uint8_t *p, size_t n, uint32_t seed)
{
    uint64_t s = 0x9e3779b97f4a7c15ull ^ seed;
    for (size_t i = 0; i < n; ++i) {
        s ^= s >> 12;
        s ^= s << 25;
        s ^= s >> 27;
        p[i] = (uint8_t)((s * 0x2545f4914f6cdd1dull) >> 56);
    }
}

/* every byte the receiver has for stream `sid`, in order (rapido_read_stream hands out contiguous runs) */
static size_t drain(rapido_session_t *s, rapido_stream_id_t sid, uint8_t *out, size_t cap)
{
    size_t got = 0;
    for (;;) {
        size_t len = cap - got;
        uint8_t *p = rapido_read_stream(s, sid, &len);
        if (p == NULL || len == 0)
            return got;
        memcpy(out + got, p, len);
        got += len;
    }
}

struct pair {
    rapido_session_t *client, *server;
    rapido_connection_id_t c_cid, s_cid;
    rapido_address_id_t c_aid_remote;
};

/* a session over one TCP connection, handshake done (t/rapido_tests.c:290-306) */
static int connect_pair(struct pair *p, ptls_context_t *cctx, ptls_context_t *sctx)
{
    p->client = rapido_new_session(cctx, false, "localhost", NULL);
    p->server = rapido_new_session(sctx, true, "localhost", NULL);
    struct sockaddr_in a;
    socklen_t len_a;
    if (loopback("4443", &a, &len_a) != 0)
        return -1;
    rapido_add_address(p->server, (struct sockaddr *)&a, len_a);
    p->c_aid_remote = rapido_add_remote_address(p->client, (struct sockaddr *)&a, len_a);
    p->c_cid = rapido_create_connection(p->client, 0, p->c_aid_remote);
    rapido_run_network(p->server, RUN_TIMEOUT);
    rapido_run_network(p->client, RUN_TIMEOUT);
    rapido_run_network(p->server, RUN_TIMEOUT);
    CHECK(ptls_handshake_is_complete(p->client->tls));
    CHECK(ptls_handshake_is_complete(p->server->tls));
    CHECK(p->server->pending_notifications.size > 0);
    if (p->server->pending_notifications.size == 0)
        return -1;
    rapido_application_notification_t *n = rapido_queue_pop(&p->server->pending_notifications);
    CHECK(n->notification_type == rapido_new_connection);
    p->s_cid = n->connection_id;
    while (p->server->pending_notifications.size > 0)
        rapido_queue_pop(&p->server->pending_notifications);
    return 0;
}

static void free_pair(struct pair *p)
{
    rapido_session_free(p->client);
    rapido_session_free(p->server);
    free(p->client);
    free(p->server);
}

static uint8_t sent[1000000], recv_buf[1100000];

/* `from` sends n bytes (1 MB at most) on a new stream over the connections `cids`; `to` must end up with exactly them */
static void transfer(rapido_session_t *from, rapido_session_t *to, const rapido_connection_id_t *cids, int ncid,
                     uint32_t seed, size_t n)
{
    fill(sent, n, seed);
    rapido_stream_id_t sid = rapido_open_stream(from);
    CHECK(rapido_add_to_stream(from, sid, sent, n) == 0);
    CHECK(rapido_close_stream(from, sid) == 0);
    for (int i = 0; i < ncid; ++i)
        CHECK(rapido_attach_stream(from, sid, cids[i]) == 0);
    size_t got = 0;
    for (int round = 0; round < 20 && got < n; ++round) {
        rapido_run_network(from, RUN_TIMEOUT);
        rapido_run_network(to, RUN_TIMEOUT);
        while (to->pending_notifications.size > 0)
            rapido_queue_pop(&to->pending_notifications);
        got += drain(to, sid, recv_buf + got, sizeof(recv_buf) - got);
    }
    CHECK(got == n);
    CHECK(memcmp(recv_buf, sent, n) == 0);
}

int main(int argc, char **argv)
{
    const int keylen = argc > 1 ? atoi(argv[1]) : 16;
    const int self_test = argc > 2 && strcmp(argv[2], "minicrypto") == 0; /* the harness alone: minicrypto everywhere */
    if (!self_test && !ptls_mi355x_is_supported()) {
        printf("not ok - no gfx950 device: the engine has no CPU fallback\n");
        return 1;
    }
    ptls_cipher_suite_t *eng[] = {keylen == 32 ? &mi355x_aes256gcmsha384 : &mi355x_aes128gcmsha256, NULL};
    ptls_cipher_suite_t *mc[] = {keylen == 32 ? &ptls_minicrypto_aes256gcmsha384 : &ptls_minicrypto_aes128gcmsha256, NULL};
    /* 1 MB per transfer between engines (t/rapido_tests.c:319); the minicrypto side of a mixed pair (bit-serial GHASH)
     * and the self-test move 256 KB */
    const size_t big = self_test ? 256000 : sizeof(sent), mixed = 256000;
    if (self_test)
        eng[0] = mc[0];
    ptls_iovec_t cert = ptls_iovec_init(SECP256R1_CERTIFICATE, sizeof(SECP256R1_CERTIFICATE) - 1);
    ptls_minicrypto_secp256r1sha256_sign_certificate_t sign_cert;
    if (ptls_minicrypto_init_secp256r1sha256_sign_certificate(
            &sign_cert, ptls_iovec_init(SECP256R1_PRIVATE_KEY, sizeof(SECP256R1_PRIVATE_KEY) - 1)) != 0)
        return 1;
    ptls_context_t engine_ctx = {ptls_minicrypto_random_bytes, &ptls_get_time, ptls_minicrypto_key_exchanges, eng,
                                 {&cert, 1}, NULL, NULL, NULL, &sign_cert.super};
    ptls_context_t minicrypto_ctx = engine_ctx;
    minicrypto_ctx.cipher_suites = mc;

    /* 1. test_large_transfer: 1 MB client -> server over one connection, then 1 MB back, both sides on the engine */
    {
        struct pair p;
        if (connect_pair(&p, &engine_ctx, &engine_ctx) == 0) {
            CHECK(ptls_get_cipher(p.client->tls)->aead == eng[0]->aead);
            CHECK(ptls_get_cipher(p.server->tls)->aead == eng[0]->aead);
            transfer(p.client, p.server, &p.c_cid, 1, 1, big);
            transfer(p.server, p.client, &p.s_cid, 1, 2, big);
        }
        free_pair(&p);
    }
    /* 2. test_join: a second connection (its own IV, lib/rapido.c:127-133) joins the session; 1 MB over both */
    {
        struct pair p;
        if (connect_pair(&p, &engine_ctx, &engine_ctx) == 0) {
            struct sockaddr_in c;
            socklen_t len_c;
            CHECK(loopback("14444", &c, &len_c) == 0);
            rapido_address_id_t c_aid_c = rapido_add_address(p.client, (struct sockaddr *)&c, len_c);
            rapido_run_network(p.client, RUN_TIMEOUT);
            rapido_run_network(p.server, RUN_TIMEOUT);
            rapido_run_network(p.client, RUN_TIMEOUT);
            rapido_connection_id_t c_cid2 = rapido_create_connection(p.client, c_aid_c, p.c_aid_remote);
            CHECK(c_cid2 != p.c_cid);
            rapido_run_network(p.server, RUN_TIMEOUT);
            rapido_run_network(p.client, RUN_TIMEOUT);
            rapido_run_network(p.server, RUN_TIMEOUT);
            size_t conns = 0;
            rapido_array_iter(&p.server->connections, i, rapido_connection_t * conn, { (void)conn; ++conns; });
            CHECK(conns == 2);
            while (p.server->pending_notifications.size > 0)
                rapido_queue_pop(&p.server->pending_notifications);
            rapido_connection_id_t both[2] = {p.c_cid, c_cid2};
            transfer(p.client, p.server, both, 2, 3, big);
        }
        free_pair(&p);
    }
    /* 3. the engine against an independent AES-GCM: engine client / minicrypto server, then the reverse */
    for (int side = 0; side < 2; ++side) {
        struct pair p;
        if (connect_pair(&p, side == 0 ? &engine_ctx : &minicrypto_ctx, side == 0 ? &minicrypto_ctx : &engine_ctx) == 0) {
            CHECK(ptls_get_cipher((side == 0 ? p.client : p.server)->tls)->aead == eng[0]->aead);
            CHECK(ptls_get_cipher((side == 0 ? p.server : p.client)->tls)->aead == mc[0]->aead);
            transfer(p.client, p.server, &p.c_cid, 1, 4 + side, mixed);
            transfer(p.server, p.client, &p.s_cid, 1, 6 + side, mixed);
        }
        free_pair(&p);
    }
    if (n_fail == 0)
        printf("ok %d checks, rapido over %s (%s)\n", n_ok, keylen == 32 ? "TLS_AES_256_GCM_SHA384" : "TLS_AES_128_GCM_SHA256",
               eng[0]->aead->name);
    return n_fail == 0 ? 0 : 1;
}
