/*
 * tests/cpp/model_sanitize.cpp -- the host kernel model under AddressSanitizer and UndefinedBehaviorSanitizer (test
 * only; tests/test_model_sanitizers.py builds it with -fsanitize=address,undefined and runs it as its own process).
 *
 * Every kernel family's code path of gcm_core.h (batch K = 1, 2, 4, 8 with the kernels' wave semantics; window 4/8
 * lanes with 64/32-position segments; 16-lane; split; TLS-framed batch and window) seals and opens records at the
 * lengths around block, segment and run edges, each call on exactly-sized heap buffers, so any access outside the
 * model's emulated LDS image, the key image, the tables, a stack array or the records' buffers -- or a shift, overflow
 * or misaligned access the C++ standard leaves undefined -- stops the run with a sanitizer report.  The walk's reads
 * and stores are also held to each record's own bytes (GCM_READ / GCM_WRITE), and every open must verify.
 */
#include "kernel_model.cpp"

#include <stdio.h>

static int g_fail = 0;
static unsigned long g_records = 0, g_calls = 0;

#define EXPECT(c, ...)                                                                                                 \
    do {                                                                                                               \
        if (!(c)) {                                                                                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);                                                       \
            fprintf(stderr, __VA_ARGS__);                                                                              \
            fprintf(stderr, "\n");                                                                                     \
            ++g_fail;                                                                                                  \
        }                                                                                                              \
    } while (0)

static uint64_t rng_state = 0x9e3779b97f4a7c15ull;
static uint8_t rnd8()
{
    rng_state ^= rng_state >> 12;
    rng_state ^= rng_state << 25;
    rng_state ^= rng_state >> 27;
    return (uint8_t)((rng_state * 0x2545F4914F6CDD1Dull) >> 56);
}

static const uint32_t LENS[] = {0, 1, 15, 16, 17, 31, 33, 63, 64, 65, 255, 256, 257, 1023, 1025, 1399, 1400, 4097,
                                8193, 16383, 16384, 16385};
static const uint32_t NL = sizeof(LENS) / sizeof(LENS[0]);
static const uint32_t AADS[] = {0, 5, 13, 16, 17, 33};
static const uint32_t GAP = 48;

static void ranges_check(const char *what)
{
    uint64_t rfirst[2], wfirst[2];
    const uint64_t r = model_read_violations(rfirst), w = model_write_violations(wfirst);
    EXPECT(r == 0 && w == 0, "%s: %llu reads / %llu writes outside the records", what, (unsigned long long)r,
           (unsigned long long)w);
}

/* fam: 1, 2, 4, 8 = batch K; 10 + kw (seglen 64), 20 + kw (seglen 32) = window; 30 = win16; 31 = split */
static int call_aead(int fam, int seal, const uint8_t *key, size_t keylen, const uint8_t *iv, const Record *recs,
                     size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *st)
{
    if (fam <= 8)
        return model_batch(seal, fam, key, keylen, iv, recs, n, src, dst, aad, st);
    if (fam >= 30)
        return model_batch_win16(seal, fam == 31, key, keylen, iv, recs, n, src, dst, aad, st);
    model_set_window_lanes(fam % 10);
    model_set_window_seglen(fam >= 20 ? 32 : 64);
    return model_batch_window(seal, key, keylen, iv, recs, n, src, dst, aad, st);
}

static void aead_family(int fam, size_t keylen)
{
    uint8_t key[32], iv[12];
    for (auto &b : key)
        b = rnd8();
    for (auto &b : iv)
        b = rnd8();
    std::vector<Record> recs(NL);
    uint64_t off = GAP, aoff = GAP;
    for (uint32_t i = 0; i < NL; ++i) {
        const uint32_t alen = AADS[i % (sizeof(AADS) / sizeof(AADS[0]))];
        recs[i] = Record{off, off, aoff, 100u + i, LENS[i], alen};
        off += LENS[i] + 16 + GAP;
        aoff += alen + GAP;
    }
    uint8_t *src = (uint8_t *)malloc(off), *ct = (uint8_t *)malloc(off), *pt = (uint8_t *)malloc(off);
    uint8_t *aad = (uint8_t *)malloc(aoff);
    uint32_t *st = (uint32_t *)malloc(NL * sizeof(uint32_t));
    for (uint64_t i = 0; i < off; ++i)
        src[i] = rnd8(), ct[i] = 0, pt[i] = 0;
    for (uint64_t i = 0; i < aoff; ++i)
        aad[i] = rnd8();
    std::vector<uint64_t> rd, wr;
    rd.push_back((uintptr_t)recs.data());
    rd.push_back((uintptr_t)(recs.data() + NL));
    for (const Record &r : recs) {
        rd.push_back((uintptr_t)(src + r.src));
        rd.push_back((uintptr_t)(src + r.src + r.len));
        rd.push_back((uintptr_t)(aad + r.aad));
        rd.push_back((uintptr_t)(aad + r.aad + r.aadlen));
        wr.push_back((uintptr_t)(ct + r.dst));
        wr.push_back((uintptr_t)(ct + r.dst + r.len + 16));
    }
    model_set_read_ranges(rd.data(), rd.size() / 2);
    model_set_write_ranges(wr.data(), wr.size() / 2);
    EXPECT(call_aead(fam, 1, key, keylen, iv, recs.data(), NL, src, ct, aad, st) == 0, "seal fam %d", fam);
    ranges_check("aead seal");
    rd.resize(2); /* the open's inputs: ciphertext + tag, and the AAD */
    wr.clear();
    for (const Record &r : recs) {
        rd.push_back((uintptr_t)(ct + r.src));
        rd.push_back((uintptr_t)(ct + r.src + r.len + 16));
        rd.push_back((uintptr_t)(aad + r.aad));
        rd.push_back((uintptr_t)(aad + r.aad + r.aadlen));
        wr.push_back((uintptr_t)(pt + r.dst));
        wr.push_back((uintptr_t)(pt + r.dst + r.len));
    }
    model_set_read_ranges(rd.data(), rd.size() / 2);
    model_set_write_ranges(wr.data(), wr.size() / 2);
    EXPECT(call_aead(fam, 0, key, keylen, iv, recs.data(), NL, ct, pt, aad, st) == 0, "open fam %d", fam);
    ranges_check("aead open");
    g_records += 2 * NL;
    g_calls += 2;
    model_set_read_ranges(nullptr, 0);
    model_set_write_ranges(nullptr, 0);
    for (uint32_t i = 0; i < NL; ++i) {
        EXPECT(st[i] == LENS[i], "fam %d key %zu len %u: status %u", fam, keylen, LENS[i], st[i]);
        EXPECT(memcmp(pt + recs[i].dst, src + recs[i].src, LENS[i]) == 0, "fam %d len %u: plaintext", fam, LENS[i]);
    }
    free(src), free(ct), free(pt), free(aad), free(st);
}

/* fam: 0 = TLS batch (K = 4); kw + 10 * (seglen == 32) = TLS window */
static void tls_family(int fam, size_t keylen)
{
    uint8_t key[32], iv[12];
    for (auto &b : key)
        b = rnd8();
    for (auto &b : iv)
        b = rnd8();
    std::vector<TlsRecord> t(NL), o(NL);
    uint64_t off = GAP, woff = GAP, poff = GAP;
    for (uint32_t i = 0; i < NL; ++i) {
        const uint32_t ln = LENS[i] > 16384 ? 16384 : LENS[i];
        t[i] = TlsRecord{off, woff, 7u + i, ln, i % 3 == 0 ? 22u : 23u};
        o[i] = TlsRecord{woff, poff, 7u + i, ln + 17, 0};
        off += ln + GAP;
        woff += ln + 22 + GAP;
        poff += ln + 1 + GAP;
    }
    uint8_t *src = (uint8_t *)malloc(off), *wire = (uint8_t *)calloc(woff, 1), *pt = (uint8_t *)calloc(poff, 1);
    uint32_t *st = (uint32_t *)malloc(NL * sizeof(uint32_t));
    uint8_t *ty = (uint8_t *)malloc(NL);
    for (uint64_t i = 0; i < off; ++i)
        src[i] = rnd8();
    auto call = [&](int seal, const TlsRecord *recs, const uint8_t *a, uint8_t *b) {
        if (fam == 0)
            return model_tls_batch(seal, key, keylen, iv, recs, NL, a, b, st, ty, nullptr);
        model_set_window_lanes(fam % 10);
        model_set_window_seglen(fam >= 10 ? 32 : 64);
        return model_tls_window(seal, key, keylen, iv, recs, NL, a, b, st, ty, nullptr);
    };
    std::vector<uint64_t> rd{(uintptr_t)t.data(), (uintptr_t)(t.data() + NL)}, wr;
    for (const TlsRecord &r : t) {
        rd.push_back((uintptr_t)(src + r.src));
        rd.push_back((uintptr_t)(src + r.src + r.len));
        wr.push_back((uintptr_t)(wire + r.dst));
        wr.push_back((uintptr_t)(wire + r.dst + r.len + 22));
    }
    model_set_read_ranges(rd.data(), rd.size() / 2);
    model_set_write_ranges(wr.data(), wr.size() / 2);
    EXPECT(call(1, t.data(), src, wire) == 0, "tls seal fam %d", fam);
    ranges_check("tls seal");
    rd.assign({(uintptr_t)o.data(), (uintptr_t)(o.data() + NL)});
    wr.clear();
    for (const TlsRecord &r : o) {
        rd.push_back((uintptr_t)(wire + r.src + 5));
        rd.push_back((uintptr_t)(wire + r.src + 5 + r.len));
        wr.push_back((uintptr_t)(pt + r.dst));
        wr.push_back((uintptr_t)(pt + r.dst + r.len - 16));
    }
    model_set_read_ranges(rd.data(), rd.size() / 2);
    model_set_write_ranges(wr.data(), wr.size() / 2);
    EXPECT(call(0, o.data(), wire, pt) == 0, "tls open fam %d", fam);
    ranges_check("tls open");
    g_records += 2 * NL;
    g_calls += 2;
    model_set_read_ranges(nullptr, 0);
    model_set_write_ranges(nullptr, 0);
    for (uint32_t i = 0; i < NL; ++i) {
        EXPECT(st[i] == t[i].len && ty[i] == t[i].type, "tls fam %d len %u: status %u type %u", fam, t[i].len, st[i],
               ty[i]);
        EXPECT(memcmp(pt + o[i].dst, src + t[i].src, t[i].len) == 0, "tls fam %d len %u: plaintext", fam, t[i].len);
    }
    free(src), free(wire), free(pt), free(st), free(ty);
}

int main()
{
    const int aead_fams[] = {1, 2, 4, 8, 14, 18, 28, 30, 31};
    const int tls_fams[] = {0, 4, 8, 18};
    for (size_t keylen : {16u, 32u}) {
        for (int f : aead_fams)
            aead_family(f, keylen);
        for (int f : tls_fams)
            tls_family(f, keylen);
    }
    printf("model_sanitize: %s (%d failures; %lu calls, %lu records sealed or opened)\n", g_fail ? "FAILED" : "ok",
           g_fail, g_calls, g_records);
    return g_fail ? 1 : 0;
}
