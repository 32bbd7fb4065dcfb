/*
 * tests/cpp/kernel_model.cpp -- host execution of the engine's kernel code (test only).
 *
 * Runs rapido_amd/csrc/gcm_core.h -- the very functions the HIP kernels are built from --
 * on the CPU, lane by lane, with v_perm_b32 and the LDS image emulated.  It lets the CPU test
 * suite check the algorithmic pieces of the kernels (T-table AES with bank-replicated
 * addressing, nibble-table GHASH, the K-lane record walk with front padding, the H^(K-j)
 * scaling) against the oracle without a GPU.  It is NOT part of the product library and the
 * product never calls it.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>
#include <vector>
#define GCM_HOST_READ_CHECK 1 /* every record read of the walk checked against the allowed ranges below */
#include "../../rapido_amd/csrc/gcm_core.h"
#include "../../scripts/gcm_bitslice.h"

using namespace mi355x;

/*
 * Read checking (GCM_READ in gcm_core.h): with ranges set, every byte range the walk reads must lie inside one of
 * them -- the records' own bytes (input, AAD, the received tag) and the descriptor array the idle loads point at.
 * Reads outside count as violations; the first one is kept.  No ranges set: nothing is checked.
 */
static std::vector<std::pair<uintptr_t, uintptr_t>> g_read_ok;
static uint64_t g_read_bad = 0, g_read_first[2] = {0, 0};

extern "C" void gcm_host_read_check(const void *p, size_t n)
{
    if (g_read_ok.empty() || n == 0)
        return;
    const uintptr_t a = (uintptr_t)p, b = a + n;
    for (const auto &r : g_read_ok)
        if (a >= r.first && b <= r.second)
            return;
    if (g_read_bad++ == 0) {
        g_read_first[0] = a;
        g_read_first[1] = n;
    }
}

/* the allowed ranges: n pairs (lo, hi) of host addresses; n = 0 stops checking.  Clears the violation count. */
extern "C" void model_set_read_ranges(const uint64_t *lohi, size_t n)
{
    g_read_ok.clear();
    for (size_t i = 0; i < n; ++i)
        g_read_ok.emplace_back((uintptr_t)lohi[2 * i], (uintptr_t)lohi[2 * i + 1]);
    g_read_bad = 0;
    g_read_first[0] = g_read_first[1] = 0;
}

/* violations since the ranges were set; first[0..1] = address and length of the first */
extern "C" uint64_t model_read_violations(uint64_t *first)
{
    first[0] = g_read_first[0];
    first[1] = g_read_first[1];
    return g_read_bad;
}

/* Write checking (GCM_WRITE): the same, for the walk's stores against the records' output ranges. */
static std::vector<std::pair<uintptr_t, uintptr_t>> g_write_ok;
static uint64_t g_write_bad = 0, g_write_first[2] = {0, 0};

extern "C" void gcm_host_write_check(const void *p, size_t n)
{
    if (g_write_ok.empty() || n == 0)
        return;
    const uintptr_t a = (uintptr_t)p, b = a + n;
    for (const auto &r : g_write_ok)
        if (a >= r.first && b <= r.second)
            return;
    if (g_write_bad++ == 0) {
        g_write_first[0] = a;
        g_write_first[1] = n;
    }
}

extern "C" void model_set_write_ranges(const uint64_t *lohi, size_t n)
{
    g_write_ok.clear();
    for (size_t i = 0; i < n; ++i)
        g_write_ok.emplace_back((uintptr_t)lohi[2 * i], (uintptr_t)lohi[2 * i + 1]);
    g_write_bad = 0;
    g_write_first[0] = g_write_first[1] = 0;
}

extern "C" uint64_t model_write_violations(uint64_t *first)
{
    first[0] = g_write_first[0];
    first[1] = g_write_first[1];
    return g_write_bad;
}

static constexpr AesTables kTabs{};

/* lanes per 64-position segment of the window math: 8 (latency kernels) or 4 (wide kernels) */
static int g_window_lanes = 8;
static uint32_t g_window_seglen = 64; /* 64, or 32 (the single-record latency kernels) */
extern "C" int model_set_window_seglen(int seglen)
{
    if (seglen != 64 && seglen != 32)
        return -1;
    const int prev = (int)g_window_seglen;
    g_window_seglen = (uint32_t)seglen;
    return prev;
}
extern "C" int model_set_window_lanes(int kw)
{
    if (kw != 4 && kw != 8)
        return -1;
    const int prev = g_window_lanes;
    g_window_lanes = kw;
    return prev;
}

/*
 * One wave of the batch kernels (batch_body, gcm_engine.hip): R = 64 / K records side by side, every lane walking to
 * the wave's longest walk (Tmax), the fast-path steps those every lane can take (an idle slot -- past the batch's
 * end, or a record the kernel does not walk -- leaves none), loads issued GCM_BATCH_PF = 3 steps ahead with the
 * descriptor array as the idle lanes' load address.  part[s] = the XOR of record s's K lane results.
 */
template <int NR, int K, bool SEAL, bool FRAME>
static void run_wave(const KeyImage *ki, const uint8_t *lds, const Record *rec, const bool *valid, const uint32_t (*iv)[3],
                     const uint32_t *ctype, const uint8_t *src, uint8_t *dst, const uint8_t *aad, const uint8_t *descs,
                     u32x4 *part)
{
    constexpr uint32_t R = 64u / (uint32_t)K;
    uint32_t Tmax = 0u, f_lo = 0xffffffffu, f_hi = 0u;
    for (uint32_t s = 0; s < R; ++s) {
        const uint32_t plen = FRAME && SEAL ? rec[s].len + 1u : rec[s].len;
        const Walk wk = make_walk(plen, FRAME ? 5u : rec[s].aadlen, K, walk_out16(dst + rec[s].dst));
        for (uint32_t j = 0; j < (uint32_t)K; ++j) {
            uint32_t lo = 0xffffffffu, hi = 0u;
            if (valid[s])
                walk_interior(wk, j, K, rec[s].len, lo, hi);
            f_lo = f_lo > lo ? f_lo : lo;
            f_hi = f_hi < hi ? f_hi : hi;
        }
        if (valid[s] && wk.T > Tmax)
            Tmax = wk.T;
    }
    for (uint32_t s = 0; s < R; ++s) {
        part[s] = u32x4{0, 0, 0, 0};
        for (uint32_t j = 0; j < (uint32_t)K; ++j)
            part[s] ^= lane_walk<NR, K, SEAL, FRAME, Layout<K>, 3>(lds, 4u * ((s * K + j) & 31u) | 0x10000u, ki->rk, j,
                                                                   rec[s], valid[s], Tmax, iv[s][0], iv[s][1], iv[s][2],
                                                                   src, dst, aad, descs, ctype[s], nullptr, 0u, nullptr,
                                                                   f_lo, f_hi);
    }
}

template <int NR, int K, bool SEAL>
static void run(const KeyImage *ki, const uint8_t *lds, const uint8_t *static_iv, const Record *recs, size_t n,
                const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *status)
{
    constexpr uint32_t R = 64u / (uint32_t)K;
    uint32_t iv0, iv1, iv2;
    memcpy(&iv0, static_iv, 4);
    memcpy(&iv1, static_iv + 4, 4);
    memcpy(&iv2, static_iv + 8, 4);
    for (size_t g = 0; g < n; g += R) {
        Record rec[R];
        bool valid[R];
        uint32_t iv[R][3], ctype[R];
        u32x4 part[R];
        for (uint32_t s = 0; s < R; ++s) {
            valid[s] = g + s < n;
            rec[s] = valid[s] ? recs[g + s] : Record{0, 0, 0, 0, 0, 0};
            iv[s][0] = iv0;
            iv[s][1] = iv1 ^ bswap32((uint32_t)(rec[s].seq >> 32));
            iv[s][2] = iv2 ^ bswap32((uint32_t)rec[s].seq);
            ctype[s] = 0u;
        }
        run_wave<NR, K, SEAL, false>(ki, lds, rec, valid, iv, ctype, src, dst, aad, (const uint8_t *)recs, part);
        for (uint32_t s = 0; s < R && g + s < n; ++s) {
            const Record &r = rec[s];
            if (SEAL) {
                memcpy(dst + r.dst + r.len, &part[s], 16);
            } else {
                const u32x4 d = part[s]; /* computed ^ received (lane_walk) */
                status[g + s] = (d[0] | d[1] | d[2] | d[3]) ? 0xffffffffu : r.len;
            }
        }
    }
}

/* ptls_mi355x_tls_record_t (include/ptls_mi355x.h section 4) */
struct TlsRecord {
    uint64_t src, dst, seq;
    uint32_t len, type;
};

/* the window kernels' two-phase join (window_group_*): groups of 4 folded with H^seglen, chained with H^(4 seglen)
 * (the LDS slots named gh64 / gh256 hold H^32 / H^128 when seglen is 32) */
template <int KW>
static u32x4 model_window_join(const uint8_t *lds, u32x4 *parts, uint32_t ns)
{
    for (uint32_t s = 0; s < ns; ++s) {
        if (!window_group_leader(s, ns))
            continue;
        u32x4 g = parts[s];
        for (uint32_t k = s + 1; k < window_group_end(s, ns); ++k)
            g = ghash_mul_lds_wide(lds, LayoutWin<KW>::gh64, g) ^ parts[k];
        parts[s] = g;
    }
    const uint32_t ng = window_group_count(ns);
    u32x4 acc = parts[0];
    if (g_window_seglen == 32u) { /* pairs of groups (H^128), then the pairs chained with H^256 */
        for (uint32_t g = 0; g + 1 < ng; ++g)
            if ((ng - g) % 2u == 0u)
                parts[window_group_start(g, ns)] = ghash_mul_lds_wide(lds, LayoutWin<KW, 32>::gh256,
                                                                      parts[window_group_start(g, ns)]) ^
                                                   parts[window_group_start(g + 1, ns)];
        acc = parts[0];
        for (uint32_t g = 2 - ng % 2; g < ng; g += 2)
            acc = ghash_mul_lds_wide(lds, LayoutWin<KW, 32>::ghpair, acc) ^ parts[window_group_start(g, ns)];
        return acc;
    }
    for (uint32_t k = window_group_end(0, ns); k < ns; k += 4)
        acc = ghash_mul_lds_wide(lds, LayoutWin<KW>::gh256, acc) ^ parts[k];
    return acc;
}

/* the FRAME walk (TLS 1.3 record framing) with the framing kernels' prologue/epilogue, K = 4, a wave of 16 records
 * at a time (run_wave) */
template <int NR, bool SEAL>
static void run_tls(const KeyImage *ki, const uint8_t *lds, const uint8_t *static_iv, const TlsRecord *trecs, size_t n,
                    const uint8_t *src, uint8_t *dst, uint32_t *status, uint8_t *types, const uint32_t *conn)
{
    constexpr int K = 4;
    constexpr uint32_t R = 64u / K;
    uint32_t iv0, iv1, iv2;
    memcpy(&iv0, static_iv, 4);
    memcpy(&iv1, static_iv + 4, 4);
    memcpy(&iv2, static_iv + 8, 4);
    for (size_t g = 0; g < n; g += R) {
        Record rec[R];
        bool valid[R];
        uint32_t iv[R][3], ctype[R];
        u32x4 part[R];
        for (uint32_t s = 0; s < R; ++s) {
            const bool in = g + s < n;
            const TlsRecord t = in ? trecs[g + s] : TlsRecord{0, 0, 0, 0, 0};
            Record r = {0, 0, 0, t.seq, 0, 5};
            if (SEAL) { /* header at t.dst, ciphertext after it; a fragment above 2^14 is not walked */
                r.src = t.src;
                r.dst = t.dst + 5;
                r.len = t.len;
                valid[s] = in && t.len <= 16384u;
            } else { /* shorter than a tag: bad_record_mac without a walk */
                r.src = t.src + 5;
                r.dst = t.dst;
                r.len = t.len >= 16u ? t.len - 16u : 0u;
                valid[s] = in && t.len >= 16u;
            }
            rec[s] = in ? r : Record{0, 0, 0, 0, 0, 0};
            iv[s][0] = conn != nullptr && in ? iv0 ^ bswap32(conn[g + s]) : iv0; /* rapido's per-connection IV */
            iv[s][1] = iv1 ^ bswap32((uint32_t)(rec[s].seq >> 32));
            iv[s][2] = iv2 ^ bswap32((uint32_t)rec[s].seq);
            ctype[s] = t.type;
        }
        run_wave<NR, K, SEAL, true>(ki, lds, rec, valid, iv, ctype, src, dst, nullptr, (const uint8_t *)trecs, part);
        for (uint32_t s = 0; s < R && g + s < n; ++s) {
            const size_t i = g + s;
            const Record &r = rec[s];
            const u32x4 tag = part[s];
            const uint32_t plen = SEAL ? r.len + 1 : r.len;
            if (SEAL) {
                if (!valid[s])
                    continue;
                memcpy(dst + r.dst + plen, &tag, 16);
                const uint32_t reclen = plen + 16;
                const uint8_t hdr[5] = {23, 3, 3, (uint8_t)(reclen >> 8), (uint8_t)reclen};
                memcpy(dst + trecs[i].dst, hdr, 5);
            } else if (!valid[s] || (tag[0] | tag[1] | tag[2] | tag[3])) {
                status[i] = 0xffffffffu;
                types[i] = 0;
                memset(dst + r.dst, 0, plen);
            } else {
                uint32_t m = plen;
                while (m != 0 && dst[r.dst + m - 1] == 0)
                    --m;
                status[i] = m ? m - 1 : 0xfffffffeu;
                types[i] = m ? dst[r.dst + m - 1] : 0;
            }
        }
    }
}

/* the window kernels' math (tls_window_body): per record, every 64-position segment walked by 4 lanes, sums
 * joined by Horner with H^64 (records above WIN_MAXSEG segments walked whole, as the kernel does) */
template <int NR, bool SEAL, int KW>
static void run_tls_window(const KeyImage *ki, const uint8_t *lds, const uint8_t *static_iv, const TlsRecord *trecs,
                           size_t n, const uint8_t *src, uint8_t *dst, uint32_t *status, uint8_t *types,
                           const uint32_t *conn)
{
    uint32_t iv0, iv1, iv2;
    memcpy(&iv0, static_iv, 4);
    memcpy(&iv1, static_iv + 4, 4);
    memcpy(&iv2, static_iv + 8, 4);
    for (size_t i = 0; i < n; ++i) {
        const TlsRecord &t = trecs[i];
        Record r = {0, 0, 0, t.seq, 0, 5};
        if (SEAL) {
            r.src = t.src;
            r.dst = t.dst + 5;
            r.len = t.len;
        } else {
            if (t.len < 16) {
                status[i] = 0xffffffffu;
                types[i] = 0;
                continue;
            }
            r.src = t.src + 5;
            r.dst = t.dst;
            r.len = t.len - 16;
        }
        const uint32_t plen = SEAL ? r.len + 1 : r.len;
        const uint32_t n1 = iv1 ^ bswap32((uint32_t)(r.seq >> 32)), n2 = iv2 ^ bswap32((uint32_t)r.seq);
        const uint32_t n0 = conn ? iv0 ^ bswap32(conn[i]) : iv0;
        uint32_t nseg;
        window_segment(1, (plen + 15) / 16, 0, &nseg, KW, g_window_seglen);
        u32x4 acc = {0, 0, 0, 0};
        if (nseg > (g_window_seglen == 32u ? (uint32_t)WIN_SEG32_MAXSEG : (uint32_t)WIN_MAXSEG)) {
            const Walk wk = make_walk(plen, 5, KW, walk_out16(dst + r.dst));
            for (uint32_t j = 0; j < (uint32_t)KW; ++j)
                acc ^= lane_walk<NR, KW, SEAL, true, LayoutWin<KW>, 3>(lds, 4u * j | 0x10000u, ki->rk, j, r, true, wk.T, n0, n1, n2,
                                                               src, dst, nullptr, (const uint8_t *)trecs, t.type);
        } else {
            u32x4 parts[WIN_SEG32_MAXSEG];
            for (uint32_t sg = 0; sg < nseg; ++sg) {
                const Walk sw = window_segment(1, (plen + 15) / 16, sg, &nseg, KW, g_window_seglen);
                u32x4 part = {0, 0, 0, 0};
                for (uint32_t j = 0; j < (uint32_t)KW; ++j)
                    part ^= lane_walk<NR, KW, SEAL, true, LayoutWin<KW>, 3>(lds, 4u * j | 0x10000u, ki->rk, j, r, true, sw.T, n0, n1,
                                                                    n2, src, dst, nullptr, (const uint8_t *)trecs, t.type,
                                                                    &sw);
                parts[sg] = part;
            }
            acc = model_window_join<KW>(lds, parts, nseg);
        }
        if (SEAL) {
            memcpy(dst + r.dst + plen, &acc, 16);
            const uint32_t reclen = plen + 16;
            const uint8_t hdr[5] = {23, 3, 3, (uint8_t)(reclen >> 8), (uint8_t)reclen};
            memcpy(dst + t.dst, hdr, 5);
        } else if (acc[0] | acc[1] | acc[2] | acc[3]) {
            status[i] = 0xffffffffu;
            types[i] = 0;
            memset(dst + r.dst, 0, plen);
        } else {
            uint32_t m = plen;
            while (m != 0 && dst[r.dst + m - 1] == 0)
                --m;
            status[i] = m ? m - 1 : 0xfffffffeu;
            types[i] = m ? dst[r.dst + m - 1] : 0;
        }
    }
}

/* the window kernels' math for AEAD records (any AAD length): segments joined with H^64, KW lanes per segment */
template <int NR, bool SEAL, int KW>
static void run_window(const KeyImage *ki, const uint8_t *lds, const uint8_t *static_iv, const Record *recs, size_t n,
                       const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *status)
{
    uint32_t iv0, iv1, iv2;
    memcpy(&iv0, static_iv, 4);
    memcpy(&iv1, static_iv + 4, 4);
    memcpy(&iv2, static_iv + 8, 4);
    for (size_t i = 0; i < n; ++i) {
        const Record &r = recs[i];
        const uint32_t n1 = iv1 ^ bswap32((uint32_t)(r.seq >> 32)), n2 = iv2 ^ bswap32((uint32_t)r.seq);
        const uint32_t A = (r.aadlen + 15) / 16, C = (r.len + 15) / 16;
        uint32_t nseg;
        window_segment(A, C, 0, &nseg, KW, g_window_seglen);
        u32x4 acc = {0, 0, 0, 0};
        if (nseg > (g_window_seglen == 32u ? (uint32_t)WIN_SEG32_MAXSEG : (uint32_t)WIN_MAXSEG)) {
            const Walk wk = make_walk(r.len, r.aadlen, KW, walk_out16(dst + r.dst));
            for (uint32_t j = 0; j < (uint32_t)KW; ++j)
                acc ^= lane_walk<NR, KW, SEAL, false, LayoutWin<KW>, 3>(lds, 4u * j | 0x10000u, ki->rk, j, r, true, wk.T, iv0, n1, n2,
                                                                src, dst, aad, (const uint8_t *)recs);
        } else {
            u32x4 parts[WIN_SEG32_MAXSEG];
            for (uint32_t sg = 0; sg < nseg; ++sg) {
                const Walk sw = window_segment(A, C, sg, &nseg, KW, g_window_seglen);
                u32x4 part = {0, 0, 0, 0};
                for (uint32_t j = 0; j < (uint32_t)KW; ++j)
                    part ^= lane_walk<NR, KW, SEAL, false, LayoutWin<KW>, 3>(lds, 4u * j | 0x10000u, ki->rk, j, r, true, sw.T, iv0,
                                                                     n1, n2, src, dst, aad, (const uint8_t *)recs, 0u, &sw);
                parts[sg] = part;
            }
            acc = model_window_join<KW>(lds, parts, nseg);
        }
        if (SEAL)
            memcpy(dst + r.dst + r.len, &acc, 16);
        else
            status[i] = (acc[0] | acc[1] | acc[2] | acc[3]) ? 0xffffffffu : r.len;
    }
}

extern "C" int model_batch_window(int is_seal, const uint8_t *key, size_t keylen, const uint8_t *static_iv,
                                  const Record *recs, size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad,
                                  uint32_t *status)
{
    KeyImage *ki = (KeyImage *)aligned_alloc(64, (sizeof(KeyImage) + 63) & ~(size_t)63) /* (a multiple of the alignment) */;
    uint8_t *lds = (uint8_t *)aligned_alloc(256, 160u * 1024u);
    if (build_key_image(kTabs.sbox, key, (uint32_t)keylen, ki) != 0) {
        free(ki);
        free(lds);
        return -1;
    }
    fill_lds_window(lds, kTabs.t0, ki, 0, 1, (uint32_t)g_window_lanes, g_window_seglen);
#define WIN_CASE(KWV)                                                                                                  \
    if (g_window_lanes == KWV) {                                                                                       \
        if (ki->rounds == 10)                                                                                          \
            is_seal ? run_window<10, true, KWV>(ki, lds, static_iv, recs, n, src, dst, aad, status)                    \
                    : run_window<10, false, KWV>(ki, lds, static_iv, recs, n, src, dst, aad, status);                  \
        else                                                                                                           \
            is_seal ? run_window<14, true, KWV>(ki, lds, static_iv, recs, n, src, dst, aad, status)                    \
                    : run_window<14, false, KWV>(ki, lds, static_iv, recs, n, src, dst, aad, status);                  \
    }
    WIN_CASE(4) WIN_CASE(8)
#undef WIN_CASE
    free(ki);
    free(lds);
    return 0;
}

/*
 * The 16-lane latency kernels (window_body with LayoutWin16) and the split kernels (split_body, LayoutSplit) for AEAD
 * records: 32-position segments walked by 16 lanes (2 steps; lane scaling H^(16 - j) as H^8 x H^(8 - j) for j < 8).
 * win16 joins the segments as window_body does with SEG = 32 (groups of 4 with H^32, pairs of groups with H^128, the
 * chain of pairs with H^256); split cuts them into runs of SPLIT_RUNSEG = 8 aligned to the record's end, joins each
 * run (groups of 4 with H^32, the two groups chained with H^128), scales it by H^(256 m) and XORs the runs.  Records
 * of more than 33 (win16) / 40 (split) segments are walked whole by 16 lanes.
 */
template <int NR, bool SEAL, bool SPLIT>
static void run_win16(const KeyImage *ki, uint8_t *lds, uint8_t *lds_m2, const uint8_t *static_iv, const Record *recs,
                      size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *status)
{
    constexpr int KW = 16;
    typedef typename std::conditional<SPLIT, LayoutSplit, LayoutWin16>::type LW;
    uint32_t iv0, iv1, iv2;
    memcpy(&iv0, static_iv, 4);
    memcpy(&iv1, static_iv + 4, 4);
    memcpy(&iv2, static_iv + 8, 4);
    const uint32_t maxseg = SPLIT ? SPLIT_RUNSEG * SPLIT_MAXRUN : WIN_SEG32_MAXSEG;
    for (size_t i = 0; i < n; ++i) {
        const Record &r = recs[i];
        const uint32_t n1 = iv1 ^ bswap32((uint32_t)(r.seq >> 32)), n2 = iv2 ^ bswap32((uint32_t)r.seq);
        const uint32_t A = (r.aadlen + 15) / 16, C = (r.len + 15) / 16;
        uint32_t nseg;
        window_segment(A, C, 0, &nseg, KW, 32);
        u32x4 acc = {0, 0, 0, 0};
        if (nseg > maxseg) {
            const Walk wk = make_walk(r.len, r.aadlen, KW, walk_out16(dst + r.dst));
            for (uint32_t j = 0; j < (uint32_t)KW; ++j)
                acc ^= lane_walk<NR, KW, SEAL, false, LW, 1>(lds, 4u * j | 0x10000u, ki->rk, j, r, true, wk.T, iv0, n1, n2, src,
                                                            dst, aad, (const uint8_t *)recs);
        } else {
            u32x4 parts[64];
            for (uint32_t sg = 0; sg < nseg; ++sg) {
                const Walk sw = window_segment(A, C, sg, &nseg, KW, 32);
                u32x4 part = {0, 0, 0, 0};
                for (uint32_t j = 0; j < (uint32_t)KW; ++j)
                    part ^= lane_walk<NR, KW, SEAL, false, LW, 1>(lds, 4u * j | 0x10000u, ki->rk, j, r, true, sw.T, iv0, n1,
                                                                 n2, src, dst, aad, (const uint8_t *)recs, 0u, &sw);
                parts[sg] = part;
            }
            if (!SPLIT) {
                /* window_body, SEG = 32: the LDS slots gh64 / gh256 / ghpair hold H^32 / H^128 / H^256 */
                for (uint32_t sg = 0; sg < nseg; ++sg)
                    if (window_group_leader(sg, nseg))
                        for (uint32_t k = sg + 1; k < window_group_end(sg, nseg); ++k)
                            parts[sg] = ghash_mul_lds_wide(lds, LayoutWin16::gh64, parts[sg]) ^ parts[k];
                const uint32_t ng = window_group_count(nseg);
                for (uint32_t g = 0; g + 1 < ng; ++g)
                    if ((ng - g) % 2u == 0u)
                        parts[window_group_start(g, nseg)] =
                            ghash_mul_lds_wide(lds, LayoutWin16::gh256, parts[window_group_start(g, nseg)]) ^
                            parts[window_group_start(g + 1, nseg)];
                acc = parts[0];
                for (uint32_t g = 2 - ng % 2; g < ng; g += 2)
                    acc = ghash_mul_lds_wide(lds, LayoutWin16::ghpair, acc) ^ parts[window_group_start(g, nseg)];
            } else {
                /* split_body: runs of SPLIT_RUNSEG aligned to the end, each joined, scaled by H^(256 m), XORed */
                const uint32_t R = (nseg + SPLIT_RUNSEG - 1) / SPLIT_RUNSEG;
                for (uint32_t k = 0; k < R; ++k) {
                    const int32_t first = (int32_t)nseg - (int32_t)(SPLIT_RUNSEG * (R - k));
                    const uint32_t lo = first < 0 ? 0u : (uint32_t)first, ns = (uint32_t)((int32_t)SPLIT_RUNSEG + (first < 0 ? first : 0));
                    u32x4 *p = parts + lo;
                    for (uint32_t li = 0; li < ns; ++li)
                        if (window_group_leader(li, ns))
                            for (uint32_t q = li + 1; q < window_group_end(li, ns); ++q)
                                p[li] = ghash_mul_lds_wide(lds, LayoutSplit::gh_group, p[li]) ^ p[q];
                    u32x4 run = p[0];
                    for (uint32_t q = window_group_end(0, ns); q < ns; q += 4)
                        run = ghash_mul_lds_wide(lds, LayoutSplit::gh_chain, run) ^ p[q];
                    const uint32_t m = R - 1 - k;
                    if (m != 0) { /* H^(256 m): the run's workgroup holds that table in its gh_run slot */
                        memcpy(lds_m2, lds, LayoutSplit::bytes);
                        memcpy(lds_m2 + LayoutSplit::gh_run, split_run_table(ki, m), GH_TABLE_BYTES);
                        run = ghash_mul_lds_wide(lds_m2, LayoutSplit::gh_run, run);
                    }
                    acc ^= run;
                }
            }
        }
        if (SEAL)
            memcpy(dst + r.dst + r.len, &acc, 16);
        else
            status[i] = (acc[0] | acc[1] | acc[2] | acc[3]) ? 0xffffffffu : r.len;
    }
}

/* the 16-lane (split = 0) or split (split = 1) window kernels' math for an AEAD batch */
extern "C" int model_batch_win16(int is_seal, int split, const uint8_t *key, size_t keylen, const uint8_t *static_iv,
                                 const Record *recs, size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad,
                                 uint32_t *status)
{
    KeyImage *ki = (KeyImage *)aligned_alloc(64, (sizeof(KeyImage) + 63) & ~(size_t)63) /* (a multiple of the alignment) */;
    uint8_t *lds = (uint8_t *)aligned_alloc(256, 160u * 1024u), *lds2 = (uint8_t *)aligned_alloc(256, 160u * 1024u);
    if (build_key_image(kTabs.sbox, key, (uint32_t)keylen, ki) != 0) {
        free(ki);
        free(lds);
        free(lds2);
        return -1;
    }
    if (split) { /* the image of a run followed by one run (H^256); run_win16 swaps the gh_run table per run */
        for (uint32_t v = 0; v < LayoutSplit::bytes / 16u; ++v)
            *(u32x4 *)(lds + 16u * v) = split_image_vec(kTabs.t0, ki, v, 1u);
    } else {
        fill_lds_win16(lds, kTabs.t0, ki, 0, 1);
    }
#define W16_CASE(NRV, SP)                                                                                              \
    if (ki->rounds == NRV && (split != 0) == SP) {                                                                     \
        if (is_seal)                                                                                                   \
            run_win16<NRV, true, SP>(ki, lds, lds2, static_iv, recs, n, src, dst, aad, status);                       \
        else                                                                                                           \
            run_win16<NRV, false, SP>(ki, lds, lds2, static_iv, recs, n, src, dst, aad, status);                      \
    }
    W16_CASE(10, false) W16_CASE(14, false) W16_CASE(10, true) W16_CASE(14, true)
#undef W16_CASE
    free(ki);
    free(lds);
    free(lds2);
    return 0;
}

extern "C" int model_tls_window(int is_seal, const uint8_t *key, size_t keylen, const uint8_t *static_iv,
                                const TlsRecord *trecs, size_t n, const uint8_t *src, uint8_t *dst, uint32_t *status,
                                uint8_t *types, const uint32_t *conn)
{
    KeyImage *ki = (KeyImage *)aligned_alloc(64, (sizeof(KeyImage) + 63) & ~(size_t)63) /* (a multiple of the alignment) */;
    uint8_t *lds = (uint8_t *)aligned_alloc(256, 160u * 1024u);
    if (build_key_image(kTabs.sbox, key, (uint32_t)keylen, ki) != 0) {
        free(ki);
        free(lds);
        return -1;
    }
    fill_lds_window(lds, kTabs.t0, ki, 0, 1, (uint32_t)g_window_lanes, g_window_seglen);
#define WIN_CASE(KWV)                                                                                                  \
    if (g_window_lanes == KWV) {                                                                                       \
        if (ki->rounds == 10)                                                                                          \
            is_seal ? run_tls_window<10, true, KWV>(ki, lds, static_iv, trecs, n, src, dst, status, types, conn)       \
                    : run_tls_window<10, false, KWV>(ki, lds, static_iv, trecs, n, src, dst, status, types, conn);     \
        else                                                                                                           \
            is_seal ? run_tls_window<14, true, KWV>(ki, lds, static_iv, trecs, n, src, dst, status, types, conn)       \
                    : run_tls_window<14, false, KWV>(ki, lds, static_iv, trecs, n, src, dst, status, types, conn);     \
    }
    WIN_CASE(4) WIN_CASE(8)
#undef WIN_CASE
    free(ki);
    free(lds);
    return 0;
}

extern "C" int model_tls_batch(int is_seal, const uint8_t *key, size_t keylen, const uint8_t *static_iv,
                               const TlsRecord *trecs, size_t n, const uint8_t *src, uint8_t *dst, uint32_t *status,
                               uint8_t *types, const uint32_t *conn)
{
    KeyImage *ki = (KeyImage *)aligned_alloc(64, (sizeof(KeyImage) + 63) & ~(size_t)63) /* (a multiple of the alignment) */;
    uint8_t *lds = (uint8_t *)aligned_alloc(256, 160u * 1024u);
    if (build_key_image(kTabs.sbox, key, (uint32_t)keylen, ki) != 0) {
        free(ki);
        free(lds);
        return -1;
    }
    fill_lds(lds, kTabs.t0, ki, 4u, 0, 1);
    if (ki->rounds == 10)
        is_seal ? run_tls<10, true>(ki, lds, static_iv, trecs, n, src, dst, status, types, conn)
                : run_tls<10, false>(ki, lds, static_iv, trecs, n, src, dst, status, types, conn);
    else
        is_seal ? run_tls<14, true>(ki, lds, static_iv, trecs, n, src, dst, status, types, conn)
                : run_tls<14, false>(ki, lds, static_iv, trecs, n, src, dst, status, types, conn);
    free(ki);
    free(lds);
    return 0;
}

extern "C" int model_batch(int is_seal, int K, const uint8_t *key, size_t keylen, const uint8_t *static_iv,
                           const Record *recs, size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad,
                           uint32_t *status)
{
    KeyImage *ki = (KeyImage *)aligned_alloc(64, (sizeof(KeyImage) + 63) & ~(size_t)63) /* (a multiple of the alignment) */;
    uint8_t *lds = (uint8_t *)aligned_alloc(256, 160u * 1024u);
    if (build_key_image(kTabs.sbox, key, (uint32_t)keylen, ki) != 0) {
        free(ki);
        free(lds);
        return -1;
    }
    fill_lds(lds, kTabs.t0, ki, (uint32_t)K, 0, 1);
    int nr = (int)ki->rounds, rc = 0;
#define MODEL_CASE(NRV, KV)                                                                                            \
    if (nr == NRV && K == KV) {                                                                                        \
        if (is_seal)                                                                                                   \
            run<NRV, KV, true>(ki, lds, static_iv, recs, n, src, dst, aad, status);                                    \
        else                                                                                                           \
            run<NRV, KV, false>(ki, lds, static_iv, recs, n, src, dst, aad, status);                                   \
    } else
    MODEL_CASE(10, 1) MODEL_CASE(10, 2) MODEL_CASE(10, 4) MODEL_CASE(10, 8) MODEL_CASE(14, 1) MODEL_CASE(14, 2)
        MODEL_CASE(14, 4) MODEL_CASE(14, 8) rc = -2;
#undef MODEL_CASE
    free(ki);
    free(lds);
    return rc;
}

/*
 * GH8 (gcm_core.h, Layout<4>::gh8): X * H^4 through the 8-bit latin table for every lane index i = 0..15 (the dword
 * swaps and byte permutations of all sixteen read orders), out[16 * (16 * n + i)] for input n, against the nibble
 * tables (out + 16 * 16 * nx).  Returns 0 when every i agrees with the nibble product, else 1 + the first bad i.
 */
extern "C" int model_gh8_mul(const uint8_t *key, size_t keylen, const uint8_t *x, size_t nx, uint8_t *out)
{
    KeyImage *ki = (KeyImage *)aligned_alloc(64, (sizeof(KeyImage) + 63) & ~(size_t)63) /* (a multiple of the alignment) */;
    uint8_t *lds = (uint8_t *)aligned_alloc(256, 160u * 1024u);
    if (build_key_image(kTabs.sbox, key, (uint32_t)keylen, ki) != 0) {
        free(ki);
        free(lds);
        return -1;
    }
    fill_lds(lds, kTabs.t0, ki, 4u, 0, 1);
    int rc = 0;
    for (size_t n = 0; n < nx; ++n) {
        u32x4 X;
        memcpy(&X, x + 16 * n, 16);
        const u32x4 want = ghash_mul_lds(lds, Layout<4>::gh_base, X); /* slot 0: H^4 */
        memcpy(out + 16 * (16 * nx + n), &want, 16);
        for (uint32_t i = 0; i < 16u; ++i) {
            const u32x4 got = gh8_mul_lds(lds, X, gh8_lane(i));
            memcpy(out + 16 * (16 * n + i), &got, 16);
            if (rc == 0 && memcmp(&got, &want, 16) != 0)
                rc = 1 + (int)i;
        }
    }
    free(ki);
    free(lds);
    return rc;
}

/* exposes the key image (round keys, H, tables) for table-level tests */
extern "C" int model_key_image(const uint8_t *key, size_t keylen, void *out, size_t outlen)
{
    if (outlen < sizeof(KeyImage))
        return -(int)sizeof(KeyImage);
    return build_key_image(kTabs.sbox, key, (uint32_t)keylen, (KeyImage *)out);
}

extern "C" size_t model_key_image_size(void) { return sizeof(KeyImage); }

/*
 * Bitsliced AES-CTR (gcm_bitslice.h) of one quad: blocks nonce || BE32(ctr0 + b), b = 0..7, written
 * to out[16 b ...] from the lanes that hold them (lane t: blocks t and t + 4).
 */
extern "C" int model_bs_keystream(const uint8_t *key, size_t keylen, const uint8_t *nonce12, uint32_t ctr0, uint8_t *out)
{
    KeyImage *ki = (KeyImage *)aligned_alloc(64, (sizeof(KeyImage) + 63) & ~(size_t)63) /* (a multiple of the alignment) */;
    uint8_t *kp = (uint8_t *)aligned_alloc(256, KEYPLANE_BYTES);
    if (build_key_image(kTabs.sbox, key, (uint32_t)keylen, ki) != 0) {
        free(ki);
        free(kp);
        return -1;
    }
    fill_keyplanes(kp, ki->rk, ki->rounds, 0, 1);
    uint32_t n[3];
    memcpy(n, nonce12, 12);
    QuadOpsHost o;
    Quad4 ka[4], kb[4];
    if (ki->rounds == 10)
        ctr_keystream_bs<10>(o, kp, 0u, q4(n[0]), q4(n[1]), q4(n[2]), q4(ctr0), ka, kb);
    else
        ctr_keystream_bs<14>(o, kp, 0u, q4(n[0]), q4(n[1]), q4(n[2]), q4(ctr0), ka, kb);
    for (int t = 0; t < 4; ++t)
        for (int d = 0; d < 4; ++d) {
            memcpy(out + 16 * t + 4 * d, &ka[d].v[t], 4);
            memcpy(out + 16 * (t + 4) + 4 * d, &kb[d].v[t], 4);
        }
    free(ki);
    free(kp);
    return 0;
}

/*
 * The parallel key setup of mi355x_gcm_setup, step by step on the host: the wave multiplies as the XOR of
 * the 64 lane shares (gf_mul_lane_share), the KEY_IMAGE_TABLES x 128 single-bit products, then every table entry
 * (key_image_store_entry).  Must equal build_key_image byte for byte.
 */
extern "C" int model_key_image_parallel(const uint8_t *key, size_t keylen, void *out, size_t outlen)
{
    if (outlen < sizeof(KeyImage) || (keylen != 16 && keylen != 32))
        return -1;
    KeyImage *ki = (KeyImage *)out;
    memset(ki, 0, sizeof(KeyImage));
    ki->rounds = aes_expand_key(kTabs.sbox, key, (uint32_t)keylen, ki->rk);
    ki->key_size = (uint32_t)keylen;
    const uint8_t zero[16] = {0};
    aes_encrypt_bytes(kTabs.sbox, ki->rk, ki->rounds, zero, ki->H);
    auto wave_mul = [](Gf128 x, Gf128 y) {
        Gf128 acc = {0u, 0u};
        for (uint32_t lane = 0; lane < 64; ++lane)
            acc = gf_xor(acc, gf_mul_lane_share(x, y, lane));
        return acc;
    };
    Gf128 pw[KEY_IMAGE_TABLES];
    const Gf128 h = gf_from_bytes(ki->H);
    pw[0] = h;
    Gf128 p = h;
    for (int e = 2; e <= MAX_K; ++e)
        pw[e - 1] = p = wave_mul(p, h);
    pw[MAX_K + 4] = p = wave_mul(p, p);    /* H^16 */
    pw[MAX_K + 2] = p = wave_mul(p, p);    /* H^32 */
    pw[MAX_K] = p = wave_mul(p, p);        /* H^64 */
    pw[MAX_K + 3] = p = wave_mul(p, p);    /* H^128 */
    pw[MAX_K + 1] = p = wave_mul(p, p);    /* H^256 */
    const Gf128 p256 = p;
    pw[MAX_K + 5] = p = wave_mul(p, p);    /* H^512 */
    pw[MAX_K + 7] = wave_mul(p, p256);     /* H^768 */
    pw[MAX_K + 6] = p = wave_mul(p, p);    /* H^1024 */
    static Gf128 bits[KEY_IMAGE_TABLES][128];
    for (uint32_t i = 0; i < KEY_IMAGE_TABLES * 128u; ++i)
        bits[i >> 7][i & 127u] = gf_mul_xpow(pw[i >> 7], i & 127u);
    for (uint32_t i = 0; i < KEY_IMAGE_TABLES * 32u * 16u; ++i)
        key_image_store_entry(ki, bits, i);
    return 0;
}

/* gf_mul_xpow (the monomial multiply of the key setup) on stream-order bytes */
extern "C" void model_gf_mul_xpow(const uint8_t *v, uint32_t i, uint8_t *out) { gf_to_bytes(gf_mul_xpow(gf_from_bytes(v), i), out); }

/* the ECB kernels' block function (aes_ecb_block) on the host: nblocks in place, encrypt or decrypt */
extern "C" int model_aes_ecb(const uint8_t *key, size_t keylen, int is_enc, uint8_t *buf, size_t nblocks)
{
    AesKeys k;
    if (build_aes_keys(kTabs.sbox, key, (uint32_t)keylen, &k) != 0)
        return -1;
    for (size_t b = 0; b < nblocks; ++b) {
        uint32_t w[4];
        memcpy(w, buf + 16 * b, 16);
        if (is_enc)
            aes_ecb_block<false>(kTabs.t0, kTabs.sbox, k.rk, k.rounds, w);
        else
            aes_ecb_block<true>(kTabs.td0, kTabs.inv_sbox, k.dk, k.rounds, w);
        memcpy(buf + 16 * b, w, 16);
    }
    return 0;
}

/* aes_last_round_bs2 on the host: two blocks' round-NR inputs a, b (LE words) -> outputs, with round key k */
extern "C" void model_last_round_bs2(uint32_t *a, uint32_t *b, const uint32_t *k) { aes_last_round_bs2(a, b, k); }

/* make_walk + walk_interior for one lane: out = {A, C, T, pad, lo, hi} (tests/test_kernel_model.py) */
extern "C" void model_walk_interior(uint32_t len, uint32_t aadlen, uint32_t K, uint32_t out16, uint32_t j, uint32_t in_len,
                                    uint32_t *out)
{
    const Walk w = make_walk(len, aadlen, K, out16);
    uint32_t lo, hi;
    walk_interior(w, j, K, in_len, lo, hi);
    out[0] = w.A;
    out[1] = w.C;
    out[2] = w.T;
    out[3] = w.pad;
    out[4] = lo;
    out[5] = hi;
}
