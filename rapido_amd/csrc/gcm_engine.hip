/*
 * gcm_engine.hip -- MI355X (gfx950) AES-GCM kernels and the engine half of the C ABI
 * declared in include/ptls_mi355x.h.
 *
 * Replaces, for the TLS/TCPLS record path, the x86 engine lib/fusion.c of the reference:
 *   ptls_fusion_aesgcm_new   (lib/fusion.c:775-795)  -> ptls_mi355x_aesgcm_new + mi355x_gcm_setup
 *   ptls_fusion_aesgcm_encrypt (lib/fusion.c:239-495) -> mi355x_gcm_seal_* batch kernels
 *   ptls_fusion_aesgcm_decrypt (lib/fusion.c:497-679) -> mi355x_gcm_open_* batch kernels
 *   ptls_fusion_aesecb_encrypt (lib/fusion.c:747-752) -> mi355x_aes_ecb
 *
 * Kernel design: one persistent workgroup of 16 waves per CU; LDS holds a
 * bank-replicated AES T-table image and the K nibble tables of H^K..H^1 (8 KiB each); K = 8
 * makes each wave-wide load/store cover whole 128-byte lines (K = 4, 64-byte pieces, is
 * the default: its four-table AES needs fewer VALU ops); round keys are wave-uniform and live in SGPRs.  A wave processes 64/K records at a
 * time, K lanes per record; lane j hashes padded GHASH positions j, j+K, ... (Horner with
 * H^K), runs the AES-CTR block of the ciphertext position it hashes, and the K partial sums
 * are scaled by H^(K-j) and XOR-reduced with cross-lane shuffles.  Every 16-byte block is
 * read once from HBM and written once.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <hipcub/hipcub.hpp>
#include "gcm_core.h"
#include "../../include/ptls_mi355x.h"

using namespace mi355x;

static_assert(sizeof(Record) == sizeof(ptls_mi355x_record_t), "descriptor layout");
static_assert(sizeof(Record) == 40, "descriptor layout");

__constant__ AesTables c_tabs = AesTables();

namespace {

#ifndef MI355X_WG_THREADS
#define MI355X_WG_THREADS 1024
#endif
constexpr int WG_THREADS = MI355X_WG_THREADS; /* 16 waves: 4 per SIMD */
#ifndef GCM_LANE_MAJOR
#define GCM_LANE_MAJOR 1
#endif
/*
 * Phase timestamps of the window kernels' first workgroup (measurement builds only, scripts/window_phases.py):
 * s_memrealtime (100 MHz) at entry, after the LDS fill, after the first pass's walk, after its barrier,
 * after its join and at the end of the pass.
 */
#ifndef GCM_WIN_TIMING
#define GCM_WIN_TIMING 0
#endif
#if GCM_WIN_TIMING
__device__ uint64_t g_win_times[8];
#define WIN_STAMP(i)                                                                                                   \
    do {                                                                                                               \
        if (blockIdx.x == 0 && threadIdx.x == 0 && grp == blockIdx.x)                                                  \
            g_win_times[i] = __builtin_amdgcn_s_memrealtime();                                                         \
    } while (0)
#else
#define WIN_STAMP(i) ((void)0)
#endif

__device__ __forceinline__ uint32_t shfl_xor_u32(uint32_t v, int mask) { return (uint32_t)__shfl_xor((int)v, mask, 64); }

__device__ __forceinline__ u32x4 shfl_xor_u32x4(u32x4 v, int mask)
{
    u32x4 r;
    r[0] = shfl_xor_u32(v[0], mask);
    r[1] = shfl_xor_u32(v[1], mask);
    r[2] = shfl_xor_u32(v[2], mask);
    r[3] = shfl_xor_u32(v[3], mask);
    return r;
}

/* TLS 1.3 record descriptor of the framing kernels (include/ptls_mi355x.h) */
struct TlsRecord {
    uint64_t src, dst, seq;
    uint32_t len, type;
};
static_assert(sizeof(TlsRecord) == sizeof(ptls_mi355x_tls_record_t), "descriptor layout");

/*
 * FRAME = false: descs are ptls_mi355x_record_t (the AEAD batch API).
 * FRAME = true:  descs are ptls_mi355x_tls_record_t; seal writes header || ciphertext(fragment ||
 * type) || tag at dst (lib/picotls.c:630-643,658-684), open verifies header-framed records and
 * strips padding / pops the content type (lib/picotls.c:4779-4791) into status / types.
 */
template <int NR, int K, bool SEAL, bool FRAME>
__device__ __forceinline__ void gcm_batch_body(const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2,
                                               const void *__restrict__ descs, const uint32_t *__restrict__ order,
                                               uint32_t nrecs, const uint8_t *src, uint8_t *dst,
                                               const uint8_t *__restrict__ aad, uint32_t *__restrict__ status,
                                               uint8_t *__restrict__ types, uint32_t *__restrict__ work,
                                               uint32_t work_base, const uint32_t *__restrict__ conn)
{
    static_assert(K <= MAX_KERNEL_K, "LDS holds at most MAX_KERNEL_K GHASH tables");
    __shared__ __attribute__((aligned(16))) uint8_t lds[Layout<K>::total];
    constexpr uint32_t R = 64 / K; /* records per wave step */
    const Record *__restrict__ recs = (const Record *)descs;
    const TlsRecord *__restrict__ trecs = (const TlsRecord *)descs;

    fill_lds(lds, c_tabs.t0, ki, K, threadIdx.x, blockDim.x);

    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); ++i)
        rk[i] = ki->rk[i];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
#if GCM_LANE_MAJOR
    /*
     * j-major lanes: lane = j * R + slot, so each 16-lane quarter of the wave (one ds_read_b128 pass)
     * holds one j.  The closing per-lane scaling multiply (table H^(K-j)) then reads ONE table per
     * pass -- conflict-free like the loop's H^K reads -- instead of K tables, whose same-bank entries
     * conflicted (~800 LDS cycles per record, 2% of a 1400-B record).
     */
    const uint32_t j = lane / R, slot = lane % R;
#else
    const uint32_t j = lane % K, slot = lane / K;
#endif
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u; /* bank + image-B select (gcm_core.h) */
    const uint32_t ngroups = (nrecs + R - 1) / R;

    /*
     * Record groups (64/K records) are handed out dynamically: one returning atomic per group
     * (MI355X_MICROARCH.md "dequeue": ~1 us under load, against ~100 us of work per group).
     * With `order` sorted by length (ptls_mi355x_order_by_length) this is longest-first
     * scheduling, and each group holds records of similar length.
     */
    for (;;) {
        uint32_t g = 0;
        if (lane == 0)
            g = atomicAdd(work, 1u) - work_base; /* tickets of this launch start at work_base (mod 2^32) */
        g = (uint32_t)__shfl((int)g, 0, 64);
        if (g >= ngroups)
            break;
        const uint32_t idx = g * R + slot;
        const bool in_batch = idx < nrecs;
        const uint32_t r = in_batch ? (order ? order[idx] : idx) : 0u;
        Record rec = {0, 0, 0, 0, 0, 0};
        uint32_t ctype = 0u;
        bool valid = in_batch;
        if (FRAME) {
            if (in_batch) {
                const TlsRecord t = trecs[r];
                rec.seq = t.seq;
                rec.aadlen = 5u;
                if (SEAL) { /* header at t.dst, ciphertext after it */
                    rec.src = t.src;
                    rec.dst = t.dst + 5u;
                    rec.len = t.len;
                    ctype = t.type;
                } else { /* header at t.src; length field = ciphertext + tag */
                    rec.src = t.src + 5u;
                    rec.dst = t.dst;
                    rec.len = t.len >= 16u ? t.len - 16u : 0u;
                    valid = t.len >= 16u; /* shorter: bad_record_mac without a walk (aead_do_decrypt) */
                }
            }
        } else if (in_batch) {
            rec = recs[r];
        }
        const uint32_t plen = FRAME && SEAL ? rec.len + 1u : rec.len;
        uint32_t T = valid ? make_walk(plen, rec.aadlen, K, walk_out16(dst + rec.dst)).T : 0u;
        uint32_t Tmax = T;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1)
            Tmax = max(Tmax, shfl_xor_u32(Tmax, o));

        const uint32_t n1 = iv1 ^ bswap32((uint32_t)(rec.seq >> 32)), n2 = iv2 ^ bswap32((uint32_t)rec.seq);
        /* per-connection IV (rapido derive_connection_aead_iv, lib/rapido.c:127-133): IV bytes 0..3 ^= BE32(id) */
        const uint32_t n0 = conn != nullptr && in_batch ? iv0 ^ bswap32(conn[r]) : iv0;
        /* 16 always-readable bytes for idle prefetch slots: the first descriptor (>= 32 B, nrecs >= 1) */
        const uint8_t *dummy = (const uint8_t *)descs;
        u32x4 part = lane_walk<NR, K, SEAL, FRAME>(lds, lanesel, rk, j, rec, valid, Tmax, n0, n1, n2, src, dst, aad,
                                                   dummy, ctype);
#pragma unroll
        for (int o = GCM_LANE_MAJOR ? (int)R : 1; o < (GCM_LANE_MAJOR ? 64 : K); o <<= 1)
            part ^= shfl_xor_u32x4(part, o);

        if (SEAL) {
            if (j == 0 && valid) {
                *(u32x4_u *)(dst + rec.dst + plen) = part;
                if (FRAME) { /* record header 17 03 03 BE16(plen + 16) (buffer_push_record, lib/picotls.c:658-662) */
                    const uint32_t reclen = plen + 16u;
                    store_partial(dst + rec.dst - 5u, 5u, u32x4{0x00030317u | ((reclen >> 8) & 0xffu) << 24, reclen & 0xffu,
                                                             0u, 0u});
                }
            }
        } else {
            /* part = computed tag ^ received tag (lane_walk) */
            const bool bad = in_batch && (!valid || (part[0] | part[1] | part[2] | part[3]) != 0u);
            if (j == 0 && in_batch && !FRAME)
                status[r] = bad ? 0xffffffffu : rec.len;
            if (bad) {
                /*
                 * Failed open: do not release plaintext (fusion leaves it, lib/fusion.c:656-679).
                 * Rare path: the descriptor is re-read through an opaque pointer so the walk does
                 * not keep dst/len alive in registers for it.
                 */
                uint64_t odst;
                uint32_t olen;
                if (FRAME) {
                    const TlsRecord *tp = trecs + r;
                    asm volatile("" : "+v"(tp));
                    const TlsRecord again = *tp;
                    odst = again.dst;
                    olen = again.len >= 16u ? again.len - 16u : 0u;
                    if (j == 0) {
                        status[r] = 0xffffffffu; /* PTLS_ALERT_BAD_RECORD_MAC */
                        types[r] = 0u;
                    }
                } else {
                    const Record *rp = recs + r;
                    asm volatile("" : "+v"(rp));
                    const Record again = *rp;
                    odst = again.dst;
                    olen = again.len;
                }
                uint8_t *out = dst + odst;
                for (uint32_t off = 16u * j; off < olen; off += 16u * K) {
                    uint32_t n = olen - off;
                    u32x4 z = {0u, 0u, 0u, 0u};
                    if (n >= 16)
                        *(u32x4_u *)(out + off) = z;
                    else
                        store_partial(out + off, n, z);
                }
            } else if (FRAME && in_batch && j == 0) {
                /*
                 * Verified record: skip the zero padding and pop the content type
                 * (handle_input_tls13, lib/picotls.c:4784-4791), reading back the plaintext the
                 * record's K lanes have just stored (made visible to this lane by the fence).
                 */
                __threadfence_block();
                const uint8_t *pt = dst + rec.dst;
                uint32_t n = plen, found = 0xfffffffeu; /* PTLS_ALERT_UNEXPECTED_MESSAGE if all zero */
                uint32_t ty = 0u;
                while (n != 0u && found == 0xfffffffeu) {
                    const uint32_t base = n >= 16u ? n - 16u : 0u;
                    const u32x4 v = n >= 16u ? *(const u32x4_u *)(pt + base) : load_partial(pt, n);
#pragma unroll
                    for (int d = 3; d >= 0; --d) {
                        if (found == 0xfffffffeu && v[d] != 0u) {
                            const uint32_t b = (31u - (uint32_t)__builtin_clz(v[d])) >> 3; /* highest nonzero byte */
                            found = base + 4u * (uint32_t)d + b;
                            ty = (v[d] >> (8u * b)) & 0xffu;
                        }
                    }
                    n = base;
                }
                status[r] = found;
                types[r] = (uint8_t)ty;
            }
        }
    }
}

/*
 * Window kernels for SMALL framing batches (rapido's 16-record send / 32-record recv windows, a few
 * connections' windows at once).  The batch kernels above give a record 4 lanes, so a 16-record window
 * is one wave walking 257 steps.  Here every record is cut into 64-position GHASH segments (its
 * positions front-padded to a multiple of 64 with zero blocks, which leaves GHASH unchanged), each
 * segment walked by its own 4-lane slot (16 steps), and the segment sums joined by Horner with H^64:
 *   GHASH = (..((P_0 H^64 + P_1) H^64 + P_2) ..) H^64 + P_{S-1}
 * (E_K(J0), folded into the length lane of the last segment, is added unmultiplied).  A 256-thread
 * workgroup holds WIN_RECS records x 17 segments; its LDS holds the two-table AES image, the tables of
 * H^4..H^1 (lane scaling) and of H^64.  A record of more than WIN_MAXSEG segments (larger than a TLS
 * record) is walked whole by its first slot instead.  Results are bit-identical to the batch kernels.
 */
template <int NR, bool SEAL, bool FRAME, int THREADS, int KW, int SEG = 64>
__device__ __forceinline__ void window_body(const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2,
                                            const void *__restrict__ descs, uint32_t nrecs, const uint8_t *src, uint8_t *dst,
                                            const uint8_t *__restrict__ aad, uint32_t *__restrict__ status,
                                            uint8_t *__restrict__ types, const uint32_t *__restrict__ conn)
{
    typedef LayoutWin<KW, SEG> LW;
    /* SEG = 32: half-length segments, twice as many, half the steps (single-record latency kernels) */
    static_assert(SEG == 64 || SEG == 32, "segment length");
    constexpr uint32_t MAXSEG = SEG == 64 ? WIN_MAXSEG : WIN_SEG32_MAXSEG;
    constexpr uint32_t SLOTS = THREADS / KW, RECS = SLOTS / MAXSEG; /* records per workgroup pass */
    static_assert(RECS >= 1, "a workgroup holds at least one record");
    constexpr bool LATENCY = THREADS <= 512;   /* few records: up to 2 waves per SIMD */
    constexpr int WIN_PF = LATENCY ? 3 : 1;    /* prefetch 3 steps ahead when little else hides a load (lane_walk) */
    __shared__ __attribute__((aligned(16))) uint8_t lds[LW::parts + RECS * MAXSEG * 16u];
    const Record *__restrict__ recs = (const Record *)descs;
    const TlsRecord *__restrict__ trecs = (const TlsRecord *)descs;
    {
        const uint32_t grp = blockIdx.x;
        (void)grp;
        WIN_STAMP(0);
    }
    fill_lds_window(lds, c_tabs.t0, ki, threadIdx.x, blockDim.x, (uint32_t)KW, (uint32_t)SEG);
    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); ++i)
        rk[i] = ki->rk[i];
    __syncthreads();
    {
        const uint32_t grp = blockIdx.x;
        (void)grp;
        WIN_STAMP(1);
    }

    const uint32_t lane = threadIdx.x & 63u, slot = threadIdx.x / KW, j = lane % KW;
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u;
    const uint32_t rl = slot / MAXSEG, seg = slot % MAXSEG;
    const uint32_t ngroups = (nrecs + RECS - 1u) / RECS;
    /* persistent: the workgroup fills its LDS once and takes record groups with a grid stride */
    for (uint32_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const uint32_t r = grp * RECS + rl;
        const bool in_batch = rl < RECS && r < nrecs;
        Record rec = {0, 0, 0, 0, 0, FRAME ? 5u : 0u};
        uint32_t ctype = 0u;
        bool valid = in_batch;
        if (FRAME) {
            if (in_batch) {
                const TlsRecord t = trecs[r];
                rec.seq = t.seq;
                if (SEAL) {
                    rec.src = t.src;
                    rec.dst = t.dst + 5u;
                    rec.len = t.len;
                    ctype = t.type;
                } else {
                    rec.src = t.src + 5u;
                    rec.dst = t.dst;
                    rec.len = t.len >= 16u ? t.len - 16u : 0u;
                    valid = t.len >= 16u;
                }
            }
        } else if (in_batch) {
            rec = recs[r];
        }
        const uint32_t plen = FRAME && SEAL ? rec.len + 1u : rec.len;
        const uint32_t A = FRAME ? 1u : (rec.aadlen + 15u) / 16u;
        uint32_t nseg;
        const Walk sw = window_segment(A, (plen + 15u) / 16u, seg, &nseg, (uint32_t)KW, (uint32_t)SEG);
        const bool whole = nseg > MAXSEG; /* larger than a TLS record: its first slot walks it all */
        const bool active = valid && (whole ? seg == 0u : seg < nseg);
        uint32_t Tw = active ? (whole ? make_walk(plen, rec.aadlen, (uint32_t)KW, walk_out16(dst + rec.dst)).T : sw.T) : 0u;
        /* first step holding a real position (segments that are mostly front padding start late) */
        uint32_t tf = active && !whole && (int32_t)sw.pad > 0 ? (uint32_t)(int32_t)sw.pad / (uint32_t)KW : (active ? 0u : ~0u);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            Tw = max(Tw, shfl_xor_u32(Tw, o));
            tf = min(tf, shfl_xor_u32(tf, o));
        }
        const uint32_t t0 = tf == ~0u ? 0u : tf & ~1u;
        const uint32_t n1 = iv1 ^ bswap32((uint32_t)(rec.seq >> 32)), n2 = iv2 ^ bswap32((uint32_t)rec.seq);
        const uint32_t n0 = conn != nullptr && in_batch ? iv0 ^ bswap32(conn[r]) : iv0;
        u32x4 part = lane_walk<NR, KW, SEAL, FRAME, LW, WIN_PF>(lds, lanesel, rk, j, rec, active, Tw, n0, n1, n2, src, dst,
                                                              aad, (const uint8_t *)descs, ctype, whole ? nullptr : &sw,
                                                              t0);
#pragma unroll
        for (int o = 1; o < KW; o <<= 1)
            part ^= shfl_xor_u32x4(part, o);
        WIN_STAMP(2);
        if (active && j == 0u)
            *(u32x4 *)(lds + LW::parts + (rl * MAXSEG + seg) * 16u) = part;
        __syncthreads();
        WIN_STAMP(3);
        /* join, phase A: each group leader folds its (up to 4) segments with H^64, in place (window_group_end) */
        const uint32_t ns = whole ? 1u : nseg;
        if (in_batch && valid && window_group_leader(seg, ns)) {
            u32x4 g = *(const u32x4 *)(lds + LW::parts + (rl * MAXSEG + seg) * 16u);
            const uint32_t gend = window_group_end(seg, ns);
            for (uint32_t k = seg + 1u; k < gend; ++k)
                g = (LATENCY ? ghash_mul_lds_wide(lds, LW::gh64, g) : ghash_mul_lds(lds, LW::gh64, g)) ^
                    *(const u32x4 *)(lds + LW::parts + (rl * MAXSEG + k) * 16u);
            *(u32x4 *)(lds + LW::parts + (rl * MAXSEG + seg) * 16u) = g;
        }
        __syncthreads();
        const uint32_t ng = window_group_count(ns);
        if constexpr (SEG == 32) {
            /* phase P (window_group_count): pair leaders fold the next group in with H^128 = H^(4 SEG), in place */
            if (in_batch && valid && window_group_leader(seg, ns)) {
                const uint32_t g = seg == 0u ? 0u : (seg + window_group_offset(ns)) / 4u;
                if ((ng - g) % 2u == 0u) {
                    const u32x4 a = *(const u32x4 *)(lds + LW::parts + (rl * MAXSEG + seg) * 16u);
                    const u32x4 b = *(const u32x4 *)(lds + LW::parts + (rl * MAXSEG + window_group_start(g + 1u, ns)) * 16u);
                    *(u32x4 *)(lds + LW::parts + (rl * MAXSEG + seg) * 16u) = ghash_mul_lds_wide(lds, LW::gh256, a) ^ b;
                }
            }
            __syncthreads();
        }
        if (in_batch && seg == 0u) {
            /*
             * phase B: the record's first slot chains the groups with H^(4 SEG) (SEG = 64), or the pairs of groups
             * with H^256 (SEG = 32): tag (seal) or tag ^ received tag (open)
             */
            u32x4 acc = {0u, 0u, 0u, 0u};
            if (valid) {
                acc = *(const u32x4 *)(lds + LW::parts + rl * MAXSEG * 16u);
                if constexpr (SEG == 32) {
                    for (uint32_t g = 2u - ng % 2u; g < ng; g += 2u)
                        acc = ghash_mul_lds_wide(lds, LW::ghpair, acc) ^
                              *(const u32x4 *)(lds + LW::parts + (rl * MAXSEG + window_group_start(g, ns)) * 16u);
                } else {
                    for (uint32_t k = window_group_end(0u, ns); k < ns; k += 4u)
                        acc = (LATENCY ? ghash_mul_lds_wide(lds, LW::gh256, acc) : ghash_mul_lds(lds, LW::gh256, acc)) ^
                              *(const u32x4 *)(lds + LW::parts + (rl * MAXSEG + k) * 16u);
                }
            }
            WIN_STAMP(4);
            if (SEAL) {
                if (j == 0u) {
                    *(u32x4_u *)(dst + rec.dst + plen) = acc;
                    if (FRAME) { /* 17 03 03 BE16(plen + 16) (lib/picotls.c:658-662) */
                        const uint32_t reclen = plen + 16u;
                        store_partial(dst + rec.dst - 5u, 5u,
                                      u32x4{0x00030317u | ((reclen >> 8) & 0xffu) << 24, reclen & 0xffu, 0u, 0u});
                    }
                }
            } else if (!valid || (acc[0] | acc[1] | acc[2] | acc[3]) != 0u) {
                /* no unverified plaintext is released (fusion leaves it, lib/fusion.c:656-679) */
                uint8_t *out = dst + rec.dst;
                for (uint32_t off = 16u * j; off < rec.len; off += 16u * KW) {
                    const uint32_t n = rec.len - off;
                    if (n >= 16u)
                        *(u32x4_u *)(out + off) = u32x4{0u, 0u, 0u, 0u};
                    else
                        store_partial(out + off, n, u32x4{0u, 0u, 0u, 0u});
                }
                if (j == 0u) {
                    status[r] = 0xffffffffu; /* SIZE_MAX / PTLS_ALERT_BAD_RECORD_MAC */
                    if (FRAME)
                        types[r] = 0u;
                }
            } else if (!FRAME) {
                if (j == 0u)
                    status[r] = rec.len;
            } else if (j == 0u) {
                /* padding strip + content-type pop (lib/picotls.c:4784-4791) over plaintext the other slots wrote */
                __threadfence();
                const uint8_t *pt = dst + rec.dst;
                uint32_t n = plen, found = 0xfffffffeu, ty = 0u; /* PTLS_ALERT_UNEXPECTED_MESSAGE if all zero */
                while (n != 0u && found == 0xfffffffeu) {
                    const uint32_t base = n >= 16u ? n - 16u : 0u;
                    const u32x4 v = n >= 16u ? *(const u32x4_u *)(pt + base) : load_partial(pt, n);
#pragma unroll
                    for (int d = 3; d >= 0; --d) {
                        if (found == 0xfffffffeu && v[d] != 0u) {
                            const uint32_t b = (31u - (uint32_t)__builtin_clz(v[d])) >> 3;
                            found = base + 4u * (uint32_t)d + b;
                            ty = (v[d] >> (8u * b)) & 0xffu;
                        }
                    }
                    n = base;
                }
                status[r] = found;
                types[r] = (uint8_t)ty;
            }
        }
        __syncthreads(); /* the segment sums of this pass are consumed before the next pass writes them */
        WIN_STAMP(5);
    }
}

} // namespace

/* Named kernel instances (readable in rocprofv3 traces). */
#define MI355X_GCM_KERNEL_F(NAME, NR, K, SEAL, FRAME)                                                                  \
    extern "C" __global__ __launch_bounds__(WG_THREADS) void NAME(                                                     \
        const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2, const void *__restrict__ descs,     \
        const uint32_t *__restrict__ order, uint32_t nrecs, const uint8_t *src, uint8_t *dst,                          \
        const uint8_t *__restrict__ aad, uint32_t *__restrict__ st, uint8_t *__restrict__ types,                       \
        uint32_t *__restrict__ work, uint32_t work_base, const uint32_t *__restrict__ conn)                            \
    {                                                                                                                  \
        gcm_batch_body<NR, K, SEAL, FRAME>(ki, iv0, iv1, iv2, descs, order, nrecs, src, dst, aad, st, types, work,     \
                                           work_base, conn);                                                           \
    }
#define MI355X_GCM_KERNEL(NAME, NR, K, SEAL) MI355X_GCM_KERNEL_F(NAME, NR, K, SEAL, false)

MI355X_GCM_KERNEL(mi355x_gcm_seal_aes128_k1, 10, 1, true)
MI355X_GCM_KERNEL(mi355x_gcm_seal_aes128_k2, 10, 2, true)
MI355X_GCM_KERNEL(mi355x_gcm_seal_aes128_k4, 10, 4, true)
MI355X_GCM_KERNEL(mi355x_gcm_seal_aes128_k8, 10, 8, true)
MI355X_GCM_KERNEL(mi355x_gcm_seal_aes256_k1, 14, 1, true)
MI355X_GCM_KERNEL(mi355x_gcm_seal_aes256_k2, 14, 2, true)
MI355X_GCM_KERNEL(mi355x_gcm_seal_aes256_k4, 14, 4, true)
MI355X_GCM_KERNEL(mi355x_gcm_seal_aes256_k8, 14, 8, true)
MI355X_GCM_KERNEL(mi355x_gcm_open_aes128_k1, 10, 1, false)
MI355X_GCM_KERNEL(mi355x_gcm_open_aes128_k2, 10, 2, false)
MI355X_GCM_KERNEL(mi355x_gcm_open_aes128_k4, 10, 4, false)
MI355X_GCM_KERNEL(mi355x_gcm_open_aes128_k8, 10, 8, false)
MI355X_GCM_KERNEL(mi355x_gcm_open_aes256_k1, 14, 1, false)
MI355X_GCM_KERNEL(mi355x_gcm_open_aes256_k2, 14, 2, false)
MI355X_GCM_KERNEL(mi355x_gcm_open_aes256_k4, 14, 4, false)
MI355X_GCM_KERNEL(mi355x_gcm_open_aes256_k8, 14, 8, false)
/* TLS 1.3 record framing (K = 4: the framing batches are window-sized, see ptls_mi355x_tls_seal_records) */
MI355X_GCM_KERNEL_F(mi355x_tls_seal_aes128_k4, 10, 4, true, true)
MI355X_GCM_KERNEL_F(mi355x_tls_seal_aes256_k4, 14, 4, true, true)
MI355X_GCM_KERNEL_F(mi355x_tls_open_aes128_k4, 10, 4, false, true)
MI355X_GCM_KERNEL_F(mi355x_tls_open_aes256_k4, 14, 4, false, true)

#define MI355X_WIN_KERNEL(NAME, NR, SEAL, FRAME, THREADS, KW)                                                              \
    extern "C" __global__ __launch_bounds__(THREADS) void NAME(                                                        \
        const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2, const void *__restrict__ descs,     \
        uint32_t nrecs, const uint8_t *src, uint8_t *dst, const uint8_t *__restrict__ aad, uint32_t *__restrict__ st,   \
        uint8_t *__restrict__ types, const uint32_t *__restrict__ conn)                                                \
    {                                                                                                                  \
        window_body<NR, SEAL, FRAME, THREADS, KW>(ki, iv0, iv1, iv2, descs, nrecs, src, dst, aad, st, types, conn);        \
    }
/* single-record latency kernels: 32-position segments (4 steps of 8 lanes), one record per 512-thread group */
#ifndef MI355X_WIN32_THREADS
#define MI355X_WIN32_THREADS 512
#endif
#define MI355X_WIN32_KERNEL(NAME, NR, SEAL, FRAME)                                                                     \
    extern "C" __global__ __launch_bounds__(MI355X_WIN32_THREADS) void NAME(                                           \
        const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2, const void *__restrict__ descs,     \
        uint32_t nrecs, const uint8_t *src, uint8_t *dst, const uint8_t *__restrict__ aad, uint32_t *__restrict__ st,   \
        uint8_t *__restrict__ types, const uint32_t *__restrict__ conn)                                                \
    {                                                                                                                  \
        window_body<NR, SEAL, FRAME, MI355X_WIN32_THREADS, 8, 32>(ki, iv0, iv1, iv2, descs, nrecs, src, dst, aad, st,  \
                                                                  types, conn);                                      \
    }
MI355X_WIN32_KERNEL(mi355x_tls_win32_seal_aes128, 10, true, true)
MI355X_WIN32_KERNEL(mi355x_tls_win32_seal_aes256, 14, true, true)
MI355X_WIN32_KERNEL(mi355x_tls_win32_open_aes128, 10, false, true)
MI355X_WIN32_KERNEL(mi355x_tls_win32_open_aes256, 14, false, true)
MI355X_WIN32_KERNEL(mi355x_gcm_win32_seal_aes128, 10, true, false)
MI355X_WIN32_KERNEL(mi355x_gcm_win32_seal_aes256, 14, true, false)
MI355X_WIN32_KERNEL(mi355x_gcm_win32_open_aes128, 10, false, false)
MI355X_WIN32_KERNEL(mi355x_gcm_win32_open_aes256, 14, false, false)
/* 256 threads (3 records per pass): a few records spread over many CUs; 1024 threads (15 records per pass,
 * persistent): hundreds of records */
MI355X_WIN_KERNEL(mi355x_tls_win_seal_aes128, 10, true, true, 512, 8)
MI355X_WIN_KERNEL(mi355x_tls_win_seal_aes256, 14, true, true, 512, 8)
MI355X_WIN_KERNEL(mi355x_tls_win_open_aes128, 10, false, true, 512, 8)
MI355X_WIN_KERNEL(mi355x_tls_win_open_aes256, 14, false, true, 512, 8)
MI355X_WIN_KERNEL(mi355x_tls_winw_seal_aes128, 10, true, true, 1024, 4)
MI355X_WIN_KERNEL(mi355x_tls_winw_seal_aes256, 14, true, true, 1024, 4)
MI355X_WIN_KERNEL(mi355x_tls_winw_open_aes128, 10, false, true, 1024, 4)
MI355X_WIN_KERNEL(mi355x_tls_winw_open_aes256, 14, false, true, 1024, 4)
MI355X_WIN_KERNEL(mi355x_gcm_win_seal_aes128, 10, true, false, 512, 8)
MI355X_WIN_KERNEL(mi355x_gcm_win_seal_aes256, 14, true, false, 512, 8)
MI355X_WIN_KERNEL(mi355x_gcm_win_open_aes128, 10, false, false, 512, 8)
MI355X_WIN_KERNEL(mi355x_gcm_win_open_aes256, 14, false, false, 512, 8)
MI355X_WIN_KERNEL(mi355x_gcm_winw_seal_aes128, 10, true, false, 1024, 4)
MI355X_WIN_KERNEL(mi355x_gcm_winw_seal_aes256, 14, true, false, 1024, 4)
MI355X_WIN_KERNEL(mi355x_gcm_winw_open_aes128, 10, false, false, 1024, 4)
MI355X_WIN_KERNEL(mi355x_gcm_winw_open_aes256, 14, false, false, 1024, 4)

/* key image: round keys, H and the nibble tables of H^1..H^8 and H^64 (cold path, one thread) */
extern "C" __global__ void mi355x_gcm_setup(const uint8_t *key, uint32_t keylen, KeyImage *ki, int *rc)
{
    if (threadIdx.x == 0 && blockIdx.x == 0)
        *rc = build_key_image(c_tabs.sbox, key, keylen, ki);
}

/* AES-ECB, one thread per block (cold path: header protection, ctr cipher) */
extern "C" __global__ void mi355x_aes_ecb(const KeyImage *__restrict__ ki, const uint8_t *in, uint8_t *out, uint32_t nblocks)
{
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nblocks)
        aes_encrypt_bytes(c_tabs.sbox, ki->rk, ki->rounds, in + 16u * i, out + 16u * i);
}

/* ================================================================== host side ============ */

typedef void (*batch_kernel_t)(const KeyImage *, uint32_t, uint32_t, uint32_t, const void *, const uint32_t *, uint32_t,
                               const uint8_t *, uint8_t *, const uint8_t *, uint32_t *, uint8_t *, uint32_t *,
                               uint32_t, const uint32_t *);

constexpr uint32_t WORK_SLOTS = 256; /* per-context ring of work counters: one per launch in flight */

struct st_ptls_mi355x_aesgcm_context {
    int device;
    int num_cu;
    uint32_t key_size;
    KeyImage *d_ki;
    hipStream_t stream;  /* private stream for the synchronous single-record calls */
    uint8_t *d_stage;    /* device staging for single-record calls */
    uint8_t *h_stage;    /* pinned host staging (mapped, coherent) */
    uint8_t *h_stage_dev; /* h_stage as the GPU addresses it: zero-copy slot calls read and write it directly */
    size_t stage_cap;
    uint32_t *d_work;    /* WORK_SLOTS dynamic-scheduling ticket counters, zeroed once at setup */
    uint32_t work_base[WORK_SLOTS]; /* each counter's value at the start of its next launch */
    uint32_t work_next;
    void *d_sort;        /* ptls_mi355x_order_by_length workspace */
    size_t sort_cap;
};

static thread_local char g_err[256];
static int g_lanes = 4;
/* framing batches of at most this many records go to the window kernels (ptls_mi355x_set_tls_window_records) */
static size_t g_window_records = 16384;
/* AEAD batches (section 3) of at most this many records go to the window kernels (ptls_mi355x_set_aead_window_records):
 * the single-record slot calls and small batches, where 4 lanes per record would leave the GPU idle */
static size_t g_aead_window_records = 2048; /* break-even of 1400-B records (scripts/window_bench.py aead_batches) */
/* single-record slot calls staging at most this many bytes run zero-copy (ptls_mi355x_set_slot_zero_copy_bytes) */
static size_t g_slot_zero_copy_bytes = 1u << 20;
/* starting value of new contexts' work counters (ptls_mi355x_set_work_ticket_origin; tests the 2^32 wrap) */
static uint32_t g_ticket_origin = 0u;
/* window batches of at most this many records use 32-position segments (ptls_mi355x_set_seg32_records;
 * SIZE_MAX = the device's CU count) */
static size_t g_seg32_records = SIZE_MAX;

static int fail(const char *what, hipError_t e)
{
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return -1;
}

#define HIPCHK(call)                                                                                                   \
    do {                                                                                                               \
        hipError_t e_ = (call);                                                                                        \
        if (e_ != hipSuccess)                                                                                          \
            return fail(#call, e_);                                                                                    \
    } while (0)

/* runs `body` with the context's device current, restoring the caller's device */
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev)
            (void)hipSetDevice(dev);
        else if (prev == dev)
            prev = -1;
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

static batch_kernel_t pick_kernel(bool seal, uint32_t rounds, int k, const char **name)
{
#define PICK(NAME)                                                                                                     \
    do {                                                                                                               \
        if (name)                                                                                                      \
            *name = #NAME;                                                                                             \
        return NAME;                                                                                                   \
    } while (0)
    if (seal && rounds == 10) {
        if (k == 1) PICK(mi355x_gcm_seal_aes128_k1);
        if (k == 2) PICK(mi355x_gcm_seal_aes128_k2);
        if (k == 4) PICK(mi355x_gcm_seal_aes128_k4);
        if (k == 8) PICK(mi355x_gcm_seal_aes128_k8);
    } else if (seal && rounds == 14) {
        if (k == 1) PICK(mi355x_gcm_seal_aes256_k1);
        if (k == 2) PICK(mi355x_gcm_seal_aes256_k2);
        if (k == 4) PICK(mi355x_gcm_seal_aes256_k4);
        if (k == 8) PICK(mi355x_gcm_seal_aes256_k8);
    } else if (!seal && rounds == 10) {
        if (k == 1) PICK(mi355x_gcm_open_aes128_k1);
        if (k == 2) PICK(mi355x_gcm_open_aes128_k2);
        if (k == 4) PICK(mi355x_gcm_open_aes128_k4);
        if (k == 8) PICK(mi355x_gcm_open_aes128_k8);
    } else if (!seal && rounds == 14) {
        if (k == 1) PICK(mi355x_gcm_open_aes256_k1);
        if (k == 2) PICK(mi355x_gcm_open_aes256_k2);
        if (k == 4) PICK(mi355x_gcm_open_aes256_k4);
        if (k == 8) PICK(mi355x_gcm_open_aes256_k8);
    }
#undef PICK
    if (name)
        *name = "";
    return nullptr;
}

static batch_kernel_t pick_tls_kernel(bool seal, uint32_t rounds)
{
    if (rounds == 10)
        return seal ? mi355x_tls_seal_aes128_k4 : mi355x_tls_open_aes128_k4;
    return seal ? mi355x_tls_seal_aes256_k4 : mi355x_tls_open_aes256_k4;
}

static inline uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

static int launch_batch(ptls_mi355x_aesgcm_context_t *ctx, bool seal, const void *static_iv12, const void *recs,
                        const uint32_t *order, size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad,
                        uint32_t *status, hipStream_t stream, bool frame = false, uint8_t *types = nullptr,
                        const uint32_t *conn = nullptr)
{
    if (n == 0)
        return 0;
    if (n > 0xffffffffull) {
        snprintf(g_err, sizeof(g_err), "batch of %zu records exceeds 2^32-1", n);
        return -1;
    }
    if (n <= (frame ? g_window_records : g_aead_window_records)) {
        /*
         * small batch: the window kernels (segments of 64 GHASH positions in parallel).  Up to 15 records per CU:
         * 512-thread groups of 3 records, 8 lanes (8 steps) per segment, so a few records spread over many CUs
         * with short chains; above that, when they fill every CU, persistent 1024-thread groups of 15 records,
         * 4 lanes per segment, one per CU.
         */
        typedef void (*win_kernel_t)(const KeyImage *, uint32_t, uint32_t, uint32_t, const void *, uint32_t,
                                     const uint8_t *, uint8_t *, const uint8_t *, uint32_t *, uint8_t *, const uint32_t *);
        static const win_kernel_t table[2][2][2][2] = {
            /* [frame][wide][seal][aes256] */
            {{{mi355x_gcm_win_open_aes128, mi355x_gcm_win_open_aes256}, {mi355x_gcm_win_seal_aes128, mi355x_gcm_win_seal_aes256}},
             {{mi355x_gcm_winw_open_aes128, mi355x_gcm_winw_open_aes256},
              {mi355x_gcm_winw_seal_aes128, mi355x_gcm_winw_seal_aes256}}},
            {{{mi355x_tls_win_open_aes128, mi355x_tls_win_open_aes256}, {mi355x_tls_win_seal_aes128, mi355x_tls_win_seal_aes256}},
             {{mi355x_tls_winw_open_aes128, mi355x_tls_winw_open_aes256},
              {mi355x_tls_winw_seal_aes128, mi355x_tls_winw_seal_aes256}}}};
        static const win_kernel_t table32[2][2][2] = {
            /* [frame][seal][aes256]: 32-position segments, one record per group */
            {{mi355x_gcm_win32_open_aes128, mi355x_gcm_win32_open_aes256},
             {mi355x_gcm_win32_seal_aes128, mi355x_gcm_win32_seal_aes256}},
            {{mi355x_tls_win32_open_aes128, mi355x_tls_win32_open_aes256},
             {mi355x_tls_win32_seal_aes128, mi355x_tls_win32_seal_aes256}}};
        const bool wide = n > 15u * (uint64_t)ctx->num_cu; /* the wide groups (15 records) fill every CU */
        /* at most g_seg32_records (default: one per CU): half-length segments, half the walk (4 steps) */
        constexpr uint32_t per32 = (MI355X_WIN32_THREADS / 8u) / WIN_SEG32_MAXSEG; /* records per 32-position group */
        const bool seg32 = !wide && n <= (g_seg32_records == SIZE_MAX ? (size_t)per32 * ctx->num_cu : g_seg32_records);
        const win_kernel_t wk = seg32 ? table32[frame][seal][ctx->key_size == 32]
                                      : table[frame][wide][seal][ctx->key_size == 32];
        /* latency kernels: 512 threads, 8 lanes per segment; wide: 1024 threads, 4 lanes (MI355X_WIN_KERNEL list) */
        const uint32_t threads = seg32 ? (uint32_t)MI355X_WIN32_THREADS : wide ? 1024u : 512u,
                       per = seg32 ? per32 : (threads / (wide ? 4u : 8u)) / WIN_MAXSEG;
        uint64_t blocks = (n + per - 1) / per;
        if (wide && blocks > (uint64_t)ctx->num_cu)
            blocks = (uint64_t)ctx->num_cu;
        const uint8_t *wiv = (const uint8_t *)static_iv12;
        DeviceGuard guard(ctx->device);
        hipLaunchKernelGGL(wk, dim3((unsigned)blocks), dim3(threads), 0, stream, ctx->d_ki, le32(wiv), le32(wiv + 4),
                           le32(wiv + 8), recs, (uint32_t)n, src, dst, aad, status, types, conn);
        HIPCHK(hipGetLastError());
        return 0;
    }
    const int k = frame ? 4 : g_lanes;
    batch_kernel_t kern = frame ? pick_tls_kernel(seal, ctx->key_size == 32 ? 14u : 10u)
                                : pick_kernel(seal, ctx->key_size == 32 ? 14u : 10u, k, nullptr);
    if (kern == nullptr) {
        snprintf(g_err, sizeof(g_err), "no kernel for lanes-per-record %d", k);
        return -1;
    }
    const uint8_t *iv = (const uint8_t *)static_iv12;
    const uint64_t ngroups = (n + (64 / k) - 1) / (64 / k);
    const uint64_t waves = WG_THREADS / 64;
    uint64_t blocks = (ngroups + waves - 1) / waves;
    if (blocks > (uint64_t)ctx->num_cu)
        blocks = (uint64_t)ctx->num_cu;
    DeviceGuard guard(ctx->device);
    /*
     * Work counters are never reset: every wave takes tickets until one is out of range, so a launch
     * consumes exactly ngroups + (its waves) tickets, and the next launch on the slot starts there.
     */
    const uint32_t wslot = ctx->work_next++ % WORK_SLOTS;
    uint32_t *work = ctx->d_work + wslot;
    const uint32_t work_base = ctx->work_base[wslot];
    ctx->work_base[wslot] = work_base + (uint32_t)ngroups + (uint32_t)(blocks * waves);
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(WG_THREADS), 0, stream, ctx->d_ki, le32(iv), le32(iv + 4),
                       le32(iv + 8), recs, order, (uint32_t)n, src, dst, aad, status, types, work, work_base,
                       conn);
    HIPCHK(hipGetLastError());
    return 0;
}

static int ensure_stage(ptls_mi355x_aesgcm_context_t *ctx, size_t need)
{
    if (need <= ctx->stage_cap)
        return 0;
    size_t cap = ctx->stage_cap ? ctx->stage_cap : 4096;
    while (cap < need)
        cap *= 2;
    if (ctx->d_stage)
        (void)hipFree(ctx->d_stage);
    if (ctx->h_stage)
        (void)hipHostFree(ctx->h_stage);
    ctx->d_stage = nullptr;
    ctx->h_stage = nullptr;
    ctx->h_stage_dev = nullptr;
    ctx->stage_cap = 0;
    HIPCHK(hipMalloc(&ctx->d_stage, cap));
    /* coherent: the GPU's zero-copy reads never see stale cache lines of a previous call */
    HIPCHK(hipHostMalloc(&ctx->h_stage, cap, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void **)&ctx->h_stage_dev, ctx->h_stage, 0));
    ctx->stage_cap = cap;
    return 0;
}

static inline size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

extern "C" {

const char *ptls_mi355x_last_error(void) { return g_err; }

int ptls_mi355x_is_supported(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess)
        return 0;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

int ptls_mi355x_set_lanes_per_record(int k)
{
    if (k != 1 && k != 2 && k != 4 && k != 8)
        return -1;
    int prev = g_lanes;
    g_lanes = k;
    return prev;
}

int ptls_mi355x_get_lanes_per_record(void) { return g_lanes; }

size_t ptls_mi355x_set_tls_window_records(size_t n)
{
    const size_t prev = g_window_records;
    g_window_records = n;
    return prev;
}

size_t ptls_mi355x_set_aead_window_records(size_t n)
{
    const size_t prev = g_aead_window_records;
    g_aead_window_records = n;
    return prev;
}

size_t ptls_mi355x_set_seg32_records(size_t n)
{
    const size_t prev = g_seg32_records;
    g_seg32_records = n;
    return prev;
}

uint32_t ptls_mi355x_set_work_ticket_origin(uint32_t origin)
{
    const uint32_t prev = g_ticket_origin;
    g_ticket_origin = origin;
    return prev;
}

size_t ptls_mi355x_set_slot_zero_copy_bytes(size_t n)
{
    const size_t prev = g_slot_zero_copy_bytes;
    g_slot_zero_copy_bytes = n;
    return prev;
}

const char *ptls_mi355x_kernel_name(int is_seal, size_t key_size)
{
    const char *name = "";
    pick_kernel(is_seal != 0, key_size == 32 ? 14u : 10u, g_lanes, &name);
    return name;
}

ptls_mi355x_aesgcm_context_t *ptls_mi355x_aesgcm_new(const void *key, size_t key_size, size_t capacity)
{
    (void)capacity;
    if (key_size != 16 && key_size != 32) {
        snprintf(g_err, sizeof(g_err), "unsupported key size %zu", key_size);
        return nullptr;
    }
    ptls_mi355x_aesgcm_context_t *ctx = (ptls_mi355x_aesgcm_context_t *)calloc(1, sizeof(*ctx));
    if (ctx == nullptr)
        return nullptr;
    ctx->key_size = (uint32_t)key_size;
    hipDeviceProp_t prop;
    int *d_rc = nullptr, rc = -1;
    if (hipGetDevice(&ctx->device) != hipSuccess || hipGetDeviceProperties(&prop, ctx->device) != hipSuccess)
        goto Fail;
    ctx->num_cu = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess)
        goto Fail;
    if (hipMalloc(&ctx->d_ki, sizeof(KeyImage)) != hipSuccess || ensure_stage(ctx, 4096) != 0 ||
        hipMalloc(&ctx->d_work, WORK_SLOTS * sizeof(uint32_t)) != hipSuccess ||
        hipMemsetD32Async((hipDeviceptr_t)ctx->d_work, (int)g_ticket_origin, WORK_SLOTS, ctx->stream) != hipSuccess)
        goto Fail;
    for (uint32_t i = 0; i < WORK_SLOTS; ++i)
        ctx->work_base[i] = g_ticket_origin;
    memcpy(ctx->h_stage, key, key_size);
    d_rc = (int *)(ctx->d_stage + 64);
    if (hipMemcpyAsync(ctx->d_stage, ctx->h_stage, key_size, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
        goto Fail;
    hipLaunchKernelGGL(mi355x_gcm_setup, dim3(1), dim3(64), 0, ctx->stream, ctx->d_stage, (uint32_t)key_size, ctx->d_ki, d_rc);
    if (hipGetLastError() != hipSuccess)
        goto Fail;
    if (hipMemcpyAsync(&rc, d_rc, sizeof(int), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess || rc != 0)
        goto Fail;
    memset(ctx->h_stage, 0, key_size);
    return ctx;
Fail:
    if (g_err[0] == 0)
        snprintf(g_err, sizeof(g_err), "context setup failed: %s", hipGetErrorString(hipGetLastError()));
    ptls_mi355x_aesgcm_free(ctx);
    return nullptr;
}

void ptls_mi355x_aesgcm_free(ptls_mi355x_aesgcm_context_t *ctx)
{
    if (ctx == nullptr)
        return;
    DeviceGuard guard(ctx->device);
    if (ctx->stream)
        (void)hipStreamSynchronize(ctx->stream);
    if (ctx->d_ki) {
        (void)hipMemset(ctx->d_ki, 0, sizeof(KeyImage)); /* clear key material, as ptls_fusion_aesgcm_free does */
        (void)hipFree(ctx->d_ki);
    }
    if (ctx->d_stage)
        (void)hipFree(ctx->d_stage);
    if (ctx->d_work)
        (void)hipFree(ctx->d_work);
    if (ctx->d_sort)
        (void)hipFree(ctx->d_sort);
    if (ctx->h_stage) {
        memset(ctx->h_stage, 0, ctx->stage_cap);
        (void)hipHostFree(ctx->h_stage);
    }
    if (ctx->stream)
        (void)hipStreamDestroy(ctx->stream);
    free(ctx);
}

int ptls_mi355x_aesgcm_device(const ptls_mi355x_aesgcm_context_t *ctx) { return ctx->device; }

int ptls_mi355x_seal_batch(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12, const ptls_mi355x_record_t *recs,
                           size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad, void *stream)
{
    return launch_batch(ctx, true, static_iv12, (const Record *)recs, nullptr, n, src, dst, aad, nullptr,
                        (hipStream_t)stream);
}

int ptls_mi355x_open_batch(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12, const ptls_mi355x_record_t *recs,
                           size_t n, const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *status, void *stream)
{
    return launch_batch(ctx, false, static_iv12, (const Record *)recs, nullptr, n, src, dst, aad, status,
                        (hipStream_t)stream);
}

int ptls_mi355x_seal_batch_ordered(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                   const ptls_mi355x_record_t *recs, const uint32_t *order, size_t n, const uint8_t *src,
                                   uint8_t *dst, const uint8_t *aad, void *stream)
{
    return launch_batch(ctx, true, static_iv12, (const Record *)recs, order, n, src, dst, aad, nullptr,
                        (hipStream_t)stream);
}

int ptls_mi355x_open_batch_ordered(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                   const ptls_mi355x_record_t *recs, const uint32_t *order, size_t n, const uint8_t *src,
                                   uint8_t *dst, const uint8_t *aad, uint32_t *status, void *stream)
{
    return launch_batch(ctx, false, static_iv12, (const Record *)recs, order, n, src, dst, aad, status,
                        (hipStream_t)stream);
}

int ptls_mi355x_tls_seal_records(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                 const ptls_mi355x_tls_record_t *recs, size_t n, const uint8_t *src, uint8_t *dst,
                                 void *stream)
{
    return ptls_mi355x_tls_seal_records_multi(ctx, static_iv12, recs, nullptr, n, src, dst, stream);
}

int ptls_mi355x_tls_open_records(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                 const ptls_mi355x_tls_record_t *recs, size_t n, const uint8_t *src, uint8_t *dst,
                                 uint32_t *status, uint8_t *types, void *stream)
{
    return ptls_mi355x_tls_open_records_multi(ctx, static_iv12, recs, nullptr, n, src, dst, status, types, stream);
}

int ptls_mi355x_tls_seal_records_multi(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                       const ptls_mi355x_tls_record_t *recs, const uint32_t *conn_ids, size_t n,
                                       const uint8_t *src, uint8_t *dst, void *stream)
{
    return launch_batch(ctx, true, static_iv12, recs, nullptr, n, src, dst, nullptr, nullptr, (hipStream_t)stream,
                        true, nullptr, conn_ids);
}

int ptls_mi355x_tls_open_records_multi(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                       const ptls_mi355x_tls_record_t *recs, const uint32_t *conn_ids, size_t n,
                                       const uint8_t *src, uint8_t *dst, uint32_t *status, uint8_t *types, void *stream)
{
    if (n != 0 && (status == nullptr || types == nullptr)) {
        snprintf(g_err, sizeof(g_err), "tls_open_records needs status and types");
        return -1;
    }
    return launch_batch(ctx, false, static_iv12, recs, nullptr, n, src, dst, nullptr, status, (hipStream_t)stream,
                        true, types, conn_ids);
}

/* keys = GHASH steps of each record (its work), values = record index */
extern "C" __global__ void mi355x_sort_keys(const Record *__restrict__ recs, uint32_t n, uint32_t *keys, uint32_t *vals)
{
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        Record r = recs[i];
        uint64_t blocks = ((uint64_t)r.len + 15) / 16 + ((uint64_t)r.aadlen + 15) / 16 + 1;
        keys[i] = blocks > 0xffffffu ? 0xffffffu : (uint32_t)blocks;
        vals[i] = i;
    }
}

int ptls_mi355x_order_by_length(ptls_mi355x_aesgcm_context_t *ctx, const ptls_mi355x_record_t *recs, size_t n,
                                uint32_t *order, void *stream_)
{
    if (n == 0)
        return 0;
    if (n > 0x7fffffffull) {
        snprintf(g_err, sizeof(g_err), "batch too large to order");
        return -1;
    }
    DeviceGuard guard(ctx->device);
    hipStream_t stream = (hipStream_t)stream_;
    size_t temp = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, temp, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                        (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n, 0, 24, stream));
    const size_t arr = ((n * sizeof(uint32_t)) + 255) & ~(size_t)255;
    const size_t need = 3 * arr + temp;
    if (need > ctx->sort_cap) {
        if (ctx->d_sort)
            (void)hipFree(ctx->d_sort);
        ctx->d_sort = nullptr;
        ctx->sort_cap = 0;
        HIPCHK(hipMalloc(&ctx->d_sort, need));
        ctx->sort_cap = need;
    }
    uint8_t *base = (uint8_t *)ctx->d_sort;
    uint32_t *keys_in = (uint32_t *)base, *keys_out = (uint32_t *)(base + arr), *vals_in = (uint32_t *)(base + 2 * arr);
    hipLaunchKernelGGL(mi355x_sort_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const Record *)recs,
                       (uint32_t)n, keys_in, vals_in);
    HIPCHK(hipGetLastError());
    HIPCHK(hipcub::DeviceRadixSort::SortPairsDescending(base + 3 * arr, temp, keys_in, keys_out, vals_in, order, (int)n, 0,
                                                        24, stream));
    return 0;
}

/*
 * Single record in host memory.  Stage layout (device and pinned host alike):
 *   [0, 64) descriptor | [64, 64 + A) aad | [D, D + inlen + 16) data (in place) | status
 */
static int single_record(ptls_mi355x_aesgcm_context_t *ctx, bool seal, void *output, const void *input, size_t inlen,
                         const void *nonce12, const void *aad, size_t aadlen, const void *tag)
{
    if (inlen > 0xffffffffu || aadlen > 0xffffffffu) {
        snprintf(g_err, sizeof(g_err), "record too large");
        return -1;
    }
    DeviceGuard guard(ctx->device);
    const size_t off_aad = 64, off_data = off_aad + up16(aadlen), off_status = off_data + up16(inlen + 16);
    const size_t total = off_status + 16;
    if (ensure_stage(ctx, total) != 0)
        return -1;
    Record rec = {off_data, off_data, off_aad, 0, (uint32_t)inlen, (uint32_t)aadlen};
    memcpy(ctx->h_stage, &rec, sizeof(rec));
    if (aadlen)
        memcpy(ctx->h_stage + off_aad, aad, aadlen);
    if (inlen)
        memcpy(ctx->h_stage + off_data, input, inlen);
    if (!seal)
        memcpy(ctx->h_stage + off_data + inlen, tag, 16);
    /*
     * Zero-copy up to g_slot_zero_copy_bytes staged bytes: the kernel reads the record from the pinned staging
     * buffer over PCIe and writes the result back into it, so a call is one launch and one synchronisation
     * instead of an H2D copy, the launch, a D2H copy and the synchronisation.  Larger records are copied.
     */
    const bool zc = total <= g_slot_zero_copy_bytes;
    uint8_t *base = zc ? ctx->h_stage_dev : ctx->d_stage;
    if (!zc)
        HIPCHK(hipMemcpyAsync(ctx->d_stage, ctx->h_stage, off_status, hipMemcpyHostToDevice, ctx->stream));
    /* one record: the window kernels (8-lane segments in parallel, leading pad steps skipped) are as fast as the
     * batch walk at 64 B and faster above it (scripts/slot_latency.py, profiles/r01f_slot_latency.txt) */
    if (launch_batch(ctx, seal, nonce12, (const Record *)base, nullptr, 1, base, base, base,
                     (uint32_t *)(base + off_status), ctx->stream, false, nullptr, nullptr) != 0)
        return -1;
    const size_t outlen = seal ? inlen + 16 : inlen;
    if (!zc) {
        HIPCHK(hipMemcpyAsync(ctx->h_stage + off_data, ctx->d_stage + off_data, outlen, hipMemcpyDeviceToHost, ctx->stream));
        if (!seal)
            HIPCHK(hipMemcpyAsync(ctx->h_stage + off_status, ctx->d_stage + off_status, 4, hipMemcpyDeviceToHost,
                                  ctx->stream));
    }
    HIPCHK(hipStreamSynchronize(ctx->stream));
    if (outlen)
        memcpy(output, ctx->h_stage + off_data, outlen);
    memset(ctx->h_stage + off_aad, 0, off_status - off_aad);
    if (seal)
        return 0;
    uint32_t st;
    memcpy(&st, ctx->h_stage + off_status, 4);
    return st == (uint32_t)inlen ? 1 : 0;
}

int ptls_mi355x_aesgcm_encrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                               const void *nonce12, const void *aad, size_t aadlen)
{
    return single_record(ctx, true, output, input, inlen, nonce12, aad, aadlen, nullptr);
}

int ptls_mi355x_aesgcm_decrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t inlen,
                               const void *nonce12, const void *aad, size_t aadlen, const void *tag)
{
    return single_record(ctx, false, output, input, inlen, nonce12, aad, aadlen, tag);
}

int ptls_mi355x_aesecb_encrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t nblocks)
{
    if (nblocks == 0)
        return 0;
    if (nblocks > 0xffffffffu / 16) {
        snprintf(g_err, sizeof(g_err), "too many blocks");
        return -1;
    }
    DeviceGuard guard(ctx->device);
    const size_t bytes = 16 * nblocks;
    if (ensure_stage(ctx, 2 * bytes) != 0)
        return -1;
    memcpy(ctx->h_stage, input, bytes);
    HIPCHK(hipMemcpyAsync(ctx->d_stage, ctx->h_stage, bytes, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(mi355x_aes_ecb, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, ctx->stream, ctx->d_ki,
                       ctx->d_stage, ctx->d_stage + bytes, (uint32_t)nblocks);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(ctx->h_stage + bytes, ctx->d_stage + bytes, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
    memcpy(output, ctx->h_stage + bytes, bytes);
    memset(ctx->h_stage, 0, 2 * bytes);
    return 0;
}

} /* extern "C" */

#if GCM_WIN_TIMING
/* measurement builds: the phase stamps of the last window launch (s_memrealtime ticks, 100 MHz) */
extern "C" int ptls_mi355x_debug_window_times(uint64_t *out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_win_times), sizeof(uint64_t) * 8) == hipSuccess ? 0 : -1;
}
#endif
