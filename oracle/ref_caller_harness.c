/*
 * oracle/ref_caller_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the engine).
 *
 * The REFERENCE record layer calling the engine's AEAD objects unchanged.  picotls.c is compiled unmodified from
 * /root/reference/lib (included into this unit, as oracle/ref_record_harness.c does, for struct st_ptls_t and the
 * post-handshake state); the AEAD it calls is ptls_mi355x_aes128gcm / ptls_mi355x_aes256gcm itself, exported by
 * rapido_amd/_lib/libptls_mi355x.so, with no adapter in between.  The peer is the reference minicrypto AES-GCM
 * (lib/cifra/aes{128,256}.c over deps/cifra), independent of the engine and of fusion.
 *
 * Commands on stdin, one per line, results on stdout (tests/test_gpu_ref_caller.py):
 *
 *   send <engine|minicrypto> <keylen> <keyhex> <ivhex> <seq0> <datahex>
 *       ptls_send (lib/picotls.c:4969-4988) of the data on a ptls_t whose send traffic protection holds
 *       ptls_aead_new_direct(<aead>, 1, key, iv) at seq0, installed with ptls_set_traffic_protection exactly as
 *       rapido installs its connections' keys (lib/rapido.c:135-200)
 *       -> "ok <rc> <seq_after> <wirehex>"
 *   recv <engine|minicrypto> <keylen> <keyhex> <ivhex> <seq0> <wirehex>
 *       ptls_receive (lib/picotls.c:4913-4947) over the whole wire buffer, the receive protection installed the same
 *       way; stops at the first error as a picotls application would
 *       -> "ok <rc> <consumed> <seq_after> <plaintexthex>"
 *   handshake <engine-client|engine-server|engine-both|minicrypto-both> <16|32> <nbytes>
 *       a full TLS 1.3 handshake (ptls_handshake, minicrypto key exchange and secp256r1 certificate) between a client
 *       and a server, the engine's cipher suite {0x1301|0x1302, ptls_mi355x_aes*gcm, minicrypto sha256|384} on the
 *       named side(s) and the minicrypto suite with the same id on the other, so every handshake and application
 *       record the engine side writes is opened by minicrypto and vice versa; then nbytes of application data each
 *       way through ptls_send / ptls_receive, a KeyUpdate from each side (ptls_update_key) with more data under the
 *       new keys, and a record tampered in flight (-> PTLS_ALERT_BAD_RECORD_MAC)
 *       -> "ok <checks> <suite name> <engine aead name>"
 *
 * Any failure prints "fail ..." and exits 1.
 */
#include "picotls.c" /* -I$(REF)/lib: the reference record layer (static functions, struct st_ptls_t) */
#include "picotls/minicrypto.h"
#include "test.h"    /* -I$(REF)/t: SECP256R1_PRIVATE_KEY / SECP256R1_CERTIFICATE, the reference tests' own */
#include "ptls_mi355x.h"

#define FAIL(...)                                                                                                      \
    do {                                                                                                               \
        printf("fail ");                                                                                               \
        printf(__VA_ARGS__);                                                                                           \
        printf(" (line %d)\n", __LINE__);                                                                              \
        fflush(stdout);                                                                                                \
        exit(1);                                                                                                       \
    } while (0)

/* the engine as a TLS 1.3 cipher suite: only the AEAD is the engine's, the hash is the reference minicrypto's */
static ptls_cipher_suite_t mi355x_aes128gcmsha256 = {PTLS_CIPHER_SUITE_AES_128_GCM_SHA256, &ptls_mi355x_aes128gcm,
                                                     &ptls_minicrypto_sha256};
static ptls_cipher_suite_t mi355x_aes256gcmsha384 = {PTLS_CIPHER_SUITE_AES_256_GCM_SHA384, &ptls_mi355x_aes256gcm,
                                                     &ptls_minicrypto_sha384};

static void need_gpu(void)
{
    if (!ptls_mi355x_is_supported())
        FAIL("no gfx950 device: the engine has no CPU fallback");
}

static ptls_aead_algorithm_t *aead_of(const char *impl, size_t keylen)
{
    if (strcmp(impl, "engine") == 0 && (need_gpu(), 1))
        return keylen == 32 ? &ptls_mi355x_aes256gcm : &ptls_mi355x_aes128gcm;
    if (strcmp(impl, "minicrypto") == 0)
        return keylen == 32 ? &ptls_minicrypto_aes256gcm : &ptls_minicrypto_aes128gcm;
    FAIL("unknown aead %s", impl);
}

static uint64_t rng_state = 0x6a09e667f3bcc909ull;
static void fill_random(void *buf, size_t len)
{
    uint8_t *p = buf;
    for (size_t i = 0; i < len; ++i) {
        rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
        p[i] = (uint8_t)(rng_state >> 56);
    }
}

/* ------------------------------------------------------------------------------------------------ hex I/O ---- */
static size_t unhex(const char *s, uint8_t **out)
{
    size_t n = strlen(s) / 2;
    *out = malloc(n + 1);
    for (size_t i = 0; i < n; ++i) {
        unsigned v;
        if (sscanf(s + 2 * i, "%2x", &v) != 1)
            FAIL("bad hex");
        (*out)[i] = (uint8_t)v;
    }
    return n;
}

static void puthex(const uint8_t *p, size_t n)
{
    static const char d[] = "0123456789abcdef";
    for (size_t i = 0; i < n; ++i) {
        putchar(d[p[i] >> 4]);
        putchar(d[p[i] & 15]);
    }
    if (n == 0)
        putchar('-');
}

/* ----------------------------------------------------------- send / recv: keys installed as rapido does ---- */
static ptls_context_t direct_ctx = {fill_random, &ptls_get_time};

static ptls_t *direct_tls(ptls_aead_algorithm_t *aead, int is_dec, const uint8_t *key, const uint8_t *iv, uint64_t seq0)
{
    ptls_t *tls = ptls_server_new(&direct_ctx);
    tls->state = PTLS_STATE_SERVER_POST_HANDSHAKE; /* keys installed directly, as rapido does per connection */
    struct st_ptls_traffic_protection_t prot = {{0}};
    if ((prot.aead = ptls_aead_new_direct(aead, !is_dec, key, iv)) == NULL)
        FAIL("ptls_aead_new_direct(%s)", aead->name);
    prot.seq = seq0;
    ptls_set_traffic_protection(tls, &prot, is_dec);
    return tls;
}

static void cmd_send(const char *impl, size_t keylen, const char *khex, const char *ivhex, uint64_t seq0, const char *dhex)
{
    uint8_t *key, *iv, *data;
    if (unhex(khex, &key) != keylen || unhex(ivhex, &iv) != 12)
        FAIL("key or iv length");
    size_t len = strcmp(dhex, "-") == 0 ? (data = malloc(1), 0) : unhex(dhex, &data);
    ptls_t *tls = direct_tls(aead_of(impl, keylen), 0, key, iv, seq0);
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    int ret = ptls_send(tls, &buf, data, len);
    printf("ok %d %llu ", ret, (unsigned long long)tls->traffic_protection.enc.seq);
    puthex(buf.base, buf.off);
    putchar('\n');
    ptls_buffer_dispose(&buf);
    ptls_free(tls); /* frees the AEAD context too */
    free(key);
    free(iv);
    free(data);
}

static void cmd_recv(const char *impl, size_t keylen, const char *khex, const char *ivhex, uint64_t seq0, const char *whex)
{
    uint8_t *key, *iv, *wire;
    if (unhex(khex, &key) != keylen || unhex(ivhex, &iv) != 12)
        FAIL("key or iv length");
    size_t wirelen = unhex(whex, &wire), off = 0;
    ptls_t *tls = direct_tls(aead_of(impl, keylen), 1, key, iv, seq0);
    ptls_buffer_t buf;
    ptls_buffer_init(&buf, "", 0);
    int ret = 0;
    while (off < wirelen) {
        size_t n = wirelen - off;
        if ((ret = ptls_receive(tls, &buf, wire + off, &n)) != 0)
            break;
        off += n;
    }
    printf("ok %d %zu %llu ", ret, off, (unsigned long long)tls->traffic_protection.dec.seq);
    puthex(buf.base, buf.off);
    putchar('\n');
    ptls_buffer_dispose(&buf);
    ptls_free(tls);
    free(key);
    free(iv);
    free(wire);
}

/* ------------------------------------------------------------------------------- full handshake scenario ---- */
static ptls_iovec_t cert;
static ptls_minicrypto_secp256r1sha256_sign_certificate_t sign_cert;

static void init_ctx(ptls_context_t *c, ptls_cipher_suite_t **suites)
{
    memset(c, 0, sizeof(*c));
    c->random_bytes = fill_random;
    c->get_time = &ptls_get_time;
    c->key_exchanges = ptls_minicrypto_key_exchanges;
    c->cipher_suites = suites;
    c->certificates.list = &cert;
    c->certificates.count = 1;
    c->sign_certificate = &sign_cert.super;
}

/* moves everything `from` has to send into `to` (ptls_handshake / ptls_receive), collecting application data */
static int deliver(ptls_t *to, ptls_buffer_t *tosend, const uint8_t *wire, size_t len, ptls_buffer_t *appdata)
{
    size_t off = 0;
    while (off < len) {
        size_t n = len - off;
        int ret;
        if (!ptls_handshake_is_complete(to)) {
            ret = ptls_handshake(to, tosend, wire + off, &n, NULL);
            if (ret != 0 && ret != PTLS_ERROR_IN_PROGRESS)
                return ret;
        } else if ((ret = ptls_receive(to, appdata, wire + off, &n)) != 0) {
            return ret;
        }
        off += n;
    }
    return 0;
}

static size_t checks;

static void exchange(ptls_t *from, ptls_t *to, size_t nbytes, const char *what)
{
    uint8_t *msg = malloc(nbytes + 1);
    fill_random(msg, nbytes);
    ptls_buffer_t wire, app, back;
    ptls_buffer_init(&wire, "", 0);
    ptls_buffer_init(&app, "", 0);
    ptls_buffer_init(&back, "", 0);
    int ret;
    if ((ret = ptls_send(from, &wire, msg, nbytes)) != 0)
        FAIL("%s: ptls_send %d", what, ret);
    if ((ret = deliver(to, &back, wire.base, wire.off, &app)) != 0)
        FAIL("%s: receive %d", what, ret);
    if (app.off != nbytes || memcmp(app.base, msg, nbytes) != 0)
        FAIL("%s: %zu of %zu bytes arrived, or other bytes", what, app.off, nbytes);
    if (back.off != 0)
        FAIL("%s: the receiver produced %zu bytes to send back", what, back.off);
    ++checks;
    ptls_buffer_dispose(&wire);
    ptls_buffer_dispose(&app);
    ptls_buffer_dispose(&back);
    free(msg);
}

static void tamper(ptls_t *from, ptls_t *to, const char *what)
{
    uint8_t msg[3000];
    fill_random(msg, sizeof(msg));
    ptls_buffer_t wire, app;
    ptls_buffer_init(&wire, "", 0);
    ptls_buffer_init(&app, "", 0);
    if (ptls_send(from, &wire, msg, sizeof(msg)) != 0)
        FAIL("%s: ptls_send", what);
    wire.base[wire.off / 2] ^= 0x04; /* a ciphertext bit */
    size_t n = wire.off;
    int ret = ptls_receive(to, &app, wire.base, &n);
    if (ret != PTLS_ALERT_BAD_RECORD_MAC || app.off != 0)
        FAIL("%s: tampered record gave %d with %zu bytes delivered", what, ret, app.off);
    ++checks;
    ptls_buffer_dispose(&wire);
    ptls_buffer_dispose(&app);
}

static void cmd_handshake(const char *mode, size_t keylen, size_t nbytes)
{
    checks = 0;
    ptls_cipher_suite_t *eng[] = {keylen == 32 ? &mi355x_aes256gcmsha384 : &mi355x_aes128gcmsha256, NULL};
    ptls_cipher_suite_t *mc[] = {keylen == 32 ? &ptls_minicrypto_aes256gcmsha384 : &ptls_minicrypto_aes128gcmsha256, NULL};
    int eng_client = strcmp(mode, "engine-client") == 0 || strcmp(mode, "engine-both") == 0;
    int eng_server = strcmp(mode, "engine-server") == 0 || strcmp(mode, "engine-both") == 0;
    if (eng_client || eng_server)
        need_gpu();
    else if (strcmp(mode, "minicrypto-both") != 0) /* minicrypto-both: the harness itself, without the engine */
        FAIL("unknown handshake mode %s", mode);
    ptls_context_t cctx, sctx;
    init_ctx(&cctx, eng_client ? eng : mc);
    init_ctx(&sctx, eng_server ? eng : mc);
    ptls_t *client = ptls_client_new(&cctx), *server = ptls_server_new(&sctx);
    ptls_set_server_name(client, "test.example.com", 0);

    /* the handshake: flights back and forth until both sides complete */
    ptls_buffer_t cbuf, sbuf, app;
    ptls_buffer_init(&cbuf, "", 0);
    ptls_buffer_init(&sbuf, "", 0);
    ptls_buffer_init(&app, "", 0);
    size_t zero = 0;
    int ret = ptls_handshake(client, &cbuf, NULL, &zero, NULL);
    if (ret != PTLS_ERROR_IN_PROGRESS)
        FAIL("ClientHello: %d", ret);
    for (int round = 0; round < 8 && (cbuf.off != 0 || sbuf.off != 0); ++round) {
        if (cbuf.off != 0) {
            ret = deliver(server, &sbuf, cbuf.base, cbuf.off, &app);
            cbuf.off = 0;
            if (ret != 0)
                FAIL("server handshake: %d", ret);
        }
        if (sbuf.off != 0) {
            ret = deliver(client, &cbuf, sbuf.base, sbuf.off, &app);
            sbuf.off = 0;
            if (ret != 0)
                FAIL("client handshake: %d", ret);
        }
    }
    if (!ptls_handshake_is_complete(client) || !ptls_handshake_is_complete(server) || app.off != 0)
        FAIL("handshake did not complete");
    ptls_cipher_suite_t *cs_c = ptls_get_cipher(client), *cs_s = ptls_get_cipher(server);
    if (cs_c->id != cs_s->id || (eng_client && cs_c->aead != eng[0]->aead) || (eng_server && cs_s->aead != eng[0]->aead) ||
        (!eng_client && cs_c->aead == eng[0]->aead) || (!eng_server && cs_s->aead == eng[0]->aead))
        FAIL("negotiated suites: client %s (%s), server %s (%s)", cs_c->aead->name, cs_c == eng[0] ? "engine" : "minicrypto",
             cs_s->aead->name, cs_s == eng[0] ? "engine" : "minicrypto");
    ++checks;

    exchange(client, server, nbytes, "client -> server");
    exchange(server, client, nbytes, "server -> client");
    exchange(client, server, 1, "client -> server, 1 byte");
    /* KeyUpdate from each side: the next ptls_send carries KeyUpdate + data under the new key (lib/picotls.c:4949-4988) */
    if (ptls_update_key(client, 1) != 0)
        FAIL("ptls_update_key(client)");
    exchange(client, server, nbytes / 2 + 7, "client -> server after the client's KeyUpdate");
    exchange(server, client, 1000, "server -> client, answering the update request");
    if (ptls_update_key(server, 0) != 0)
        FAIL("ptls_update_key(server)");
    exchange(server, client, nbytes / 3 + 1, "server -> client after the server's KeyUpdate");
    exchange(client, server, 100, "client -> server");
    tamper(client, server, "client -> server, tampered");
    tamper(server, client, "server -> client, tampered");

    printf("ok %zu %s %s\n", checks, keylen == 32 ? "TLS_AES_256_GCM_SHA384" : "TLS_AES_128_GCM_SHA256",
           eng[0]->aead->name);
    ptls_buffer_dispose(&cbuf);
    ptls_buffer_dispose(&sbuf);
    ptls_buffer_dispose(&app);
    ptls_free(client);
    ptls_free(server);
}

int main(void)
{
    cert = ptls_iovec_init(SECP256R1_CERTIFICATE, sizeof(SECP256R1_CERTIFICATE) - 1);
    if (ptls_minicrypto_init_secp256r1sha256_sign_certificate(
            &sign_cert, ptls_iovec_init(SECP256R1_PRIVATE_KEY, sizeof(SECP256R1_PRIVATE_KEY) - 1)) != 0)
        FAIL("sign certificate");
    char *line = NULL;
    size_t cap = 0;
    ssize_t got;
    while ((got = getline(&line, &cap, stdin)) > 0) {
        char *argv[8] = {0};
        int argc = 0;
        for (char *tok = strtok(line, " \t\r\n"); tok != NULL && argc < 8; tok = strtok(NULL, " \t\r\n"))
            argv[argc++] = tok;
        if (argc == 0)
            continue;
        if (strcmp(argv[0], "send") == 0 && argc == 7)
            cmd_send(argv[1], (size_t)atoi(argv[2]), argv[3], argv[4], strtoull(argv[5], NULL, 10), argv[6]);
        else if (strcmp(argv[0], "recv") == 0 && argc == 7)
            cmd_recv(argv[1], (size_t)atoi(argv[2]), argv[3], argv[4], strtoull(argv[5], NULL, 10), argv[6]);
        else if (strcmp(argv[0], "handshake") == 0 && argc == 4)
            cmd_handshake(argv[1], (size_t)atoi(argv[2]), (size_t)atol(argv[3]));
        else
            FAIL("bad command %s (%d fields)", argv[0], argc);
        fflush(stdout);
    }
    free(line);
    return 0;
}
