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
#include <rocprim/iterator/constant_iterator.hpp>
#include <time.h>
#include <atomic>
#include <mutex>
#include <new>
#if defined(GCM_WIN_TIMING) && GCM_WIN_TIMING
/* measurement build (scripts/window_phases.py): stamps inside the record walk of workgroup 0, thread 0 */
__device__ uint64_t g_win_times[32];
#ifndef GCM_STAMP_BLOCK
#define GCM_STAMP_BLOCK 0 /* the workgroup whose phases are stamped (split kernels: 3 r + k for run k of record r) */
#endif
#define GCM_WALK_STAMP(i)                                                                                              \
    do {                                                                                                               \
        if (blockIdx.x == GCM_STAMP_BLOCK && threadIdx.x == 0)                                                         \
            g_win_times[i] = __builtin_amdgcn_s_memrealtime();                                                         \
    } while (0)
/* split kernels: stamps of workgroup GCM_STAMP_BLOCK, and (6, 7) of the run that finishes record 0 */
#define SPLIT_STAMP(i) GCM_WALK_STAMP(i)
#define SPLIT_STAMP_LAST(i)                                                                                            \
    do {                                                                                                               \
        if (r == 0u && threadIdx.x == 0)                                                                               \
            g_win_times[i] = __builtin_amdgcn_s_memrealtime();                                                         \
    } while (0)
#else
#define SPLIT_STAMP(i) ((void)0)
#define SPLIT_STAMP_LAST(i) ((void)0)
#endif
#include "gcm_core.h"
#include "fault_journal.h"
#include "../../include/ptls_mi355x.h"

/* a device memory event in the fault journal (fault_journal.c) */
#define JNOTE(what, p, len) ptls_mi355x_fault_journal_note(what, (const void *)(p), (size_t)(len))

using namespace mi355x;

static_assert(sizeof(Record) == sizeof(ptls_mi355x_record_t), "descriptor layout");
static_assert(sizeof(Record) == 40, "descriptor layout");

__constant__ AesTables c_tabs = AesTables();

namespace {

#ifndef MI355X_WG_THREADS
#define MI355X_WG_THREADS 1024
#endif
constexpr int WG_THREADS = MI355X_WG_THREADS; /* 16 waves: 4 per SIMD */
#ifndef GCM_PASS_LANES
#define GCM_PASS_LANES 1 /* K = 4 batch kernels: a record's lane j is the lane's ds_read_b128 pass (gcm_batch_body) */
#endif
#ifndef GCM_LANE_MAJOR
#define GCM_LANE_MAJOR 1
#endif
#ifndef GCM_SPLIT_GLDS
#define GCM_SPLIT_GLDS 1 /* split window kernels fill their LDS image by LDS DMA (split_body) */
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
#define WIN_STAMP(i)                                                                                                   \
    do {                                                                                                               \
        if (blockIdx.x == 0 && threadIdx.x == 0 && grp == blockIdx.x)                                                  \
            g_win_times[i] = __builtin_amdgcn_s_memrealtime();                                                         \
    } while (0)
#else
#define WIN_STAMP(i) ((void)0)
#endif

__device__ __forceinline__ uint32_t shfl_xor_u32(uint32_t v, int mask) { return (uint32_t)__shfl_xor((int)v, mask, 64); }

/*
 * XOR of v over aligned groups of L lanes (L = 4, 8 or 16; a DPP row is 16 lanes), every lane receiving its group's
 * XOR: quad_perm [1,0,3,2] and [2,3,0,1], then row_half_mirror (lane i <- 7 - i) and row_mirror (i <- 15 - i), each
 * pairing lanes of the two halves of the previous level.  Register-to-register, unlike __shfl_xor (ds_bpermute).
 */
template <int L>
__device__ __forceinline__ uint32_t dpp_xor_reduce(uint32_t v)
{
    static_assert(L == 4 || L == 8 || L == 16, "group of 4, 8 or 16 lanes");
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
    v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);
    if constexpr (L >= 8)
        v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true);
    if constexpr (L >= 16)
        v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true);
    return v;
}

template <int L>
__device__ __forceinline__ u32x4 dpp_xor_reduce4(u32x4 v)
{
    return u32x4{dpp_xor_reduce<L>(v[0]), dpp_xor_reduce<L>(v[1]), dpp_xor_reduce<L>(v[2]), dpp_xor_reduce<L>(v[3])};
}

/*
 * x * c (nibble tables of c at basereg) computed by the L = 8 or 16 lanes of a window slot together, for the
 * latency-bound segment join where one slot multiplies while the others wait: lane j reads the 2 x 16 / L table
 * entries of byte pairs p = j, j + L (dword p / 4, byte p % 4: its low and high nibbles), then the group XOR-reduces
 * (dpp_xor_reduce).  Every lane of the group returns the product; bit-identical to ghash_mul_lds.
 */
template <int L>
__device__ __forceinline__ u32x4 ghash_mul_coop(const uint8_t *lds, uint32_t basereg, u32x4 x, uint32_t j)
{
    u32x4 r = {0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t q = 0; q < 16u / (uint32_t)L; ++q) {
        const uint32_t p = j + (uint32_t)L * q, d = p >> 2, m = p & 3u;
        const uint32_t w = d == 0u ? x[0] : d == 1u ? x[1] : d == 2u ? x[2] : x[3];
        const uint32_t lo = (w << 4) & 0xf0f0f0f0u, hi = w & 0xf0f0f0f0u, sel = 0x0c020100u | (4u + m);
        const uint32_t off = (8u * d + 2u * m) * 256u;
        const u32x4 e = lds_u32x4(lds, perm(lo, basereg, sel) + off);
        const u32x4 f = lds_u32x4(lds, perm(hi, basereg, sel) + off + 256u);
        r ^= e ^ f;
    }
    return dpp_xor_reduce4<L>(r);
}

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
#ifndef GCM_BATCH_PF
#define GCM_BATCH_PF 3 /* batch kernels: loads issued three steps ahead, four buffers (1: one step ahead, two buffers) */
#endif
#ifndef GCM_UNIFORM_TMAX
#define GCM_UNIFORM_TMAX 1
#endif
#ifndef GCM_STATIC_GROUPS
#define GCM_STATIC_GROUPS 0
#endif
#ifndef GCM_STAGGER
#define GCM_STAGGER 0 /* measurement builds: batch-kernel waves start in four phases (gcm_batch_body) */
#endif
#ifndef GCM_FAST_STEP
#define GCM_FAST_STEP 1 /* batch kernels: interior steps on lane_walk's fast path (scalar branch, no per-lane flags) */
#endif
/*
 * Multi-key batches (MK): one key of the launch (ptls_mi355x_seal_batch_multikey).  The prep kernels (mi355x_mk_*) fill
 * `first` / `end` -- the key's records are order[first .. end), order sorted by key -- and zero the key's group counter.
 */
struct MkKey {
    const KeyImage *ki;
    uint32_t iv0, iv1, iv2; /* the key's static IV (LE dwords) */
    uint32_t first, end, pad_;
};
static_assert(sizeof(MkKey) == 32, "multi-key table entry");
constexpr uint32_t MK_NONE = 0xffffffffu;

/* the launch's key table and the workgroups' phase state (MK kernels) */
struct MkLaunch {
    const MkKey *keys;
    uint32_t nkeys;
    uint32_t *ctr;    /* per key: record groups handed out (zeroed by the prep) */
    uint32_t *wg_key; /* per workgroup: the key of its current phase (the workgroup's broadcast slot) */
};

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

    uint32_t rk[4 * (NR + 1)], kr[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); ++i) {
        rk[i] = ki->rk[i];
        kr[i] = rotl32(rk[i], 16); /* GH8 layout: the round keys of aes_round_tt2k_asm (wave-uniform) */
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
#if GCM_LANE_MAJOR
    /*
     * j-major lanes: lane = j * R + slot, so each 16-lane quarter of the wave (one ds_read_b128 pass)
     * holds one j.  The closing per-lane scaling multiply (table H^(K-j)) then reads ONE table per
     * pass -- conflict-free like the loop's H^K reads -- instead of K tables, whose same-bank entries
     * conflicted (~800 LDS cycles per record, 2% of a 1400-B record).
     */
    /*
     * GCM_PASS_LANES (K = 4): a ds_read_b128 is served in four 16-lane passes that are NOT the wave's quarters but
     * {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32 (MI355X_MICROARCH.md, LDS table), so with
     * lane = j * 16 + slot a pass held two j's, two tables of the closing scaling multiply, whose equal nibbles
     * conflict (SQ_LDS_BANK_CONFLICT ~125 cycles per record group).  Here j is the lane's pass and slot its index in
     * it: quad q = (lane & 31) >> 2 belongs to pass (0x96 >> q) & 1 of its half, at slot 4 (q >> 1) + (lane & 3).
     * A record's lanes are then lane ^ {0, 4, 32, 36} (the closing reduce's shuffles).
     */
    const uint32_t q = (lane & 31u) >> 2;
    const uint32_t j = GCM_PASS_LANES && K == 4 ? 2u * (lane >> 5) + ((0x96u >> q) & 1u) : lane / R;
    const uint32_t slot = GCM_PASS_LANES && K == 4 ? 4u * (q >> 1) + (lane & 3u) : lane % R;
#else
    const uint32_t j = lane % K, slot = lane / K;
#endif
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u; /* bank + image-B select (gcm_core.h) */
    const uint32_t ngroups = (nrecs + R - 1) / R;
#if GCM_STAGGER
    /*
     * Measurement variant: the waves of a workgroup start their walks in four phases, GCM_STAGGER s_sleep 127 (~8K
     * cycles each) apart -- wave w in phase w >> 2, so each SIMD holds one wave of every phase.  With records of one
     * length every group takes the same time, so waves that start together stay in step, and their per-record phases
     * (the closing multiply, the next group's ticket, descriptors and first loads) coincide on the CU.
     */
    for (uint32_t i = 0, n = (threadIdx.x >> 8) * (uint32_t)GCM_STAGGER; i < n; ++i)
        __builtin_amdgcn_s_sleep(127);
#endif

    /*
     * Record groups (64/K records) are handed out dynamically: one returning atomic per group
     * (MI355X_MICROARCH.md "dequeue": ~1 us under load, against ~100 us of work per group).
     * With `order` sorted by length (ptls_mi355x_order_by_length) this is longest-first
     * scheduling, and each group holds records of similar length.
     */
#if GCM_STATIC_GROUPS /* measurement builds: group k of wave w is w + k * (waves in the grid), no atomic */
    const uint32_t wave_id = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), nwaves = gridDim.x * (blockDim.x >> 6);
    for (uint32_t gs = wave_id;; gs += nwaves) {
        const uint32_t g = __builtin_amdgcn_readfirstlane(gs);
        (void)work;
        (void)work_base;
#else
    for (;;) {
        uint32_t g = 0;
        if (lane == 0)
            g = atomicAdd(work, 1u) - work_base; /* tickets of this launch start at work_base (mod 2^32) */
        g = (uint32_t)__shfl((int)g, 0, 64);
#endif
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
                    valid = t.len <= PTLS_MI355X_TLS_MAX_FRAGMENT; /* larger: not a TLS record, nothing written */
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
        const Walk wk = make_walk(plen, rec.aadlen, K, walk_out16(dst + rec.dst));
        uint32_t Tmax = valid ? wk.T : 0u;
        /* the steps in which every lane of the wave holds a whole payload block (walk_interior): lane_walk's fast path */
        uint32_t f_lo = 0xffffffffu, f_hi = 0u;
        if (GCM_FAST_STEP && valid)
            walk_interior(wk, j, K, rec.len, f_lo, f_hi);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            Tmax = max(Tmax, shfl_xor_u32(Tmax, o));
            f_lo = max(f_lo, shfl_xor_u32(f_lo, o));
            f_hi = min(f_hi, shfl_xor_u32(f_hi, o));
        }
        f_lo = __builtin_amdgcn_readfirstlane(f_lo);
        f_hi = __builtin_amdgcn_readfirstlane(f_hi);
#if GCM_UNIFORM_TMAX
        Tmax = __builtin_amdgcn_readfirstlane(Tmax); /* the walk's trip tests on the scalar unit */
#endif

        const uint32_t n1 = iv1 ^ bswap32((uint32_t)(rec.seq >> 32)), n2 = iv2 ^ bswap32((uint32_t)rec.seq);
        /* per-connection IV (rapido derive_connection_aead_iv, lib/rapido.c:127-133): IV bytes 0..3 ^= BE32(id) */
        const uint32_t n0 = conn != nullptr && in_batch ? iv0 ^ bswap32(conn[r]) : iv0;
        /* 16 always-readable bytes for idle prefetch slots: the first descriptor (>= 32 B, nrecs >= 1) */
        const uint8_t *dummy = (const uint8_t *)descs;
        u32x4 part = lane_walk<NR, K, SEAL, FRAME, Layout<K>, GCM_BATCH_PF>(lds, lanesel, rk, j, rec, valid, Tmax, n0, n1,
                                                                           n2, src, dst, aad, dummy, ctype, nullptr, 0u, kr,
                                                                           f_lo, f_hi);
        if (GCM_LANE_MAJOR && GCM_PASS_LANES && K == 4) {
            part ^= shfl_xor_u32x4(part, 4);
            part ^= shfl_xor_u32x4(part, 32);
        } else {
#pragma unroll
            for (int o = GCM_LANE_MAJOR ? (int)R : 1; o < (GCM_LANE_MAJOR ? 64 : K); o <<= 1)
                part ^= shfl_xor_u32x4(part, o);
        }

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
 * Multi-key batch kernels: gcm_batch_body's record walk in key phases (below).  The single-key body above is kept as
 * it was -- expressed through the shared group lambda it compiled to a slightly different hot loop, 1% slower seal at
 * 1400 B on one box (profiles/r06c_ablate.txt) -- so the group body is written twice; tests/test_gpu_multikey.py
 * checks this one against the oracle and against single-key launches.
 */
template <int NR, int K, bool SEAL, bool FRAME>
__device__ __forceinline__ void gcm_batch_body_mk(const void *__restrict__ descs, const uint32_t *__restrict__ order,
                                                  uint32_t nrecs, const uint8_t *src, uint8_t *dst,
                                                  const uint8_t *__restrict__ aad, uint32_t *__restrict__ status,
                                                  uint8_t *__restrict__ types, const uint32_t *__restrict__ conn,
                                                  MkLaunch mk)
{
    static_assert(Layout<K>::gh8, "multi-key batches run the GH8 layout (K = 4)");
    __shared__ __attribute__((aligned(16))) uint8_t lds[Layout<K>::total];
    constexpr uint32_t R = 64 / K; /* records per wave step */
    const Record *__restrict__ recs = (const Record *)descs;
    const TlsRecord *__restrict__ trecs = (const TlsRecord *)descs;

    uint32_t rk[4 * (NR + 1)], kr[4 * (NR + 1)];
    fill_lds_aes(lds, c_tabs.t0, K, threadIdx.x, blockDim.x); /* the key-independent AES image, once */

    const uint32_t lane = threadIdx.x & 63u;
#if GCM_LANE_MAJOR /* the lanes of a record as in gcm_batch_body */
    const uint32_t q = (lane & 31u) >> 2;
    const uint32_t j = GCM_PASS_LANES && K == 4 ? 2u * (lane >> 5) + ((0x96u >> q) & 1u) : lane / R;
    const uint32_t slot = GCM_PASS_LANES && K == 4 ? 4u * (q >> 1) + (lane & 3u) : lane % R;
#else
    const uint32_t j = lane % K, slot = lane / K;
#endif
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u; /* bank + image-B select (gcm_core.h) */

    /* one record group: lane (j, slot) walks record order[idx] (idx itself without an order) if in_batch */
    auto run_group = [&](uint32_t idx, bool in_batch, uint32_t iv0, uint32_t iv1, uint32_t iv2) {
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
                    valid = t.len <= PTLS_MI355X_TLS_MAX_FRAGMENT; /* larger: not a TLS record, nothing written */
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
        const Walk wk = make_walk(plen, rec.aadlen, K, walk_out16(dst + rec.dst));
        uint32_t Tmax = valid ? wk.T : 0u;
        /* the steps in which every lane of the wave holds a whole payload block (walk_interior): lane_walk's fast path */
        uint32_t f_lo = 0xffffffffu, f_hi = 0u;
        if (GCM_FAST_STEP && valid)
            walk_interior(wk, j, K, rec.len, f_lo, f_hi);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            Tmax = max(Tmax, shfl_xor_u32(Tmax, o));
            f_lo = max(f_lo, shfl_xor_u32(f_lo, o));
            f_hi = min(f_hi, shfl_xor_u32(f_hi, o));
        }
        f_lo = __builtin_amdgcn_readfirstlane(f_lo);
        f_hi = __builtin_amdgcn_readfirstlane(f_hi);
#if GCM_UNIFORM_TMAX
        Tmax = __builtin_amdgcn_readfirstlane(Tmax); /* the walk's trip tests on the scalar unit */
#endif

        const uint32_t n1 = iv1 ^ bswap32((uint32_t)(rec.seq >> 32)), n2 = iv2 ^ bswap32((uint32_t)rec.seq);
        /* per-connection IV (rapido derive_connection_aead_iv, lib/rapido.c:127-133): IV bytes 0..3 ^= BE32(id) */
        const uint32_t n0 = conn != nullptr && in_batch ? iv0 ^ bswap32(conn[r]) : iv0;
        /* 16 always-readable bytes for idle prefetch slots: the first descriptor (>= 32 B, nrecs >= 1) */
        const uint8_t *dummy = (const uint8_t *)descs;
        u32x4 part = lane_walk<NR, K, SEAL, FRAME, Layout<K>, GCM_BATCH_PF>(lds, lanesel, rk, j, rec, valid, Tmax, n0, n1,
                                                                           n2, src, dst, aad, dummy, ctype, nullptr, 0u, kr,
                                                                           f_lo, f_hi);
        if (GCM_LANE_MAJOR && GCM_PASS_LANES && K == 4) {
            part ^= shfl_xor_u32x4(part, 4);
            part ^= shfl_xor_u32x4(part, 32);
        } else {
#pragma unroll
            for (int o = GCM_LANE_MAJOR ? (int)R : 1; o < (GCM_LANE_MAJOR ? 64 : K); o <<= 1)
                part ^= shfl_xor_u32x4(part, o);
        }

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
    };

    {
        /*
         * Multi-key phases.  The LDS holds one key's GHASH tables, shared by the workgroup's 16 waves, so a workgroup
         * works on one key at a time: its waves take that key's record groups from the key's counter, exactly as the
         * single-key kernels do from theirs, and when the key has none left the workgroup meets at a barrier, wave 0
         * picks the next key with groups left (starting from where this workgroup is, so the workgroups spread over the
         * keys), and the tables are refilled only if the key changed.  Barriers happen only at key changes: with 64
         * keys over 256 CUs a workgroup sees a handful.  The records of key k are order[first_k .. first_k + count_k).
         */
        uint32_t cur = MK_NONE, kk = (uint32_t)(((uint64_t)blockIdx.x * mk.nkeys) / gridDim.x);
        for (;;) {
            if (threadIdx.x < 64u) {
                uint32_t pick = MK_NONE;
                for (uint32_t b = 0; b < mk.nkeys && pick == MK_NONE; b += 64u) {
                    const uint32_t t = b + lane;
                    bool left = false;
                    uint32_t kx = 0u;
                    if (t < mk.nkeys) {
                        kx = kk + t < mk.nkeys ? kk + t : kk + t - mk.nkeys;
                        const uint32_t ng = (mk.keys[kx].end - mk.keys[kx].first + R - 1u) / R;
                        left = __hip_atomic_load(mk.ctr + kx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ng;
                    }
                    const uint64_t m = __ballot(left);
                    if (m != 0ull)
                        pick = (uint32_t)__shfl((int)kx, (int)__builtin_ctzll(m), 64);
                }
                if (lane == 0u)
                    __hip_atomic_store(mk.wg_key + blockIdx.x, pick, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            /*
             * The pick reaches L2 before the barrier (a workgroup fence: wave 0 waits for its store), and the other waves
             * read it from L2 (agent-scope atomic loads bypass the CU's L1).  An agent-scope __threadfence() here wrote
             * back and invalidated L2 (buffer_wbl2 / buffer_inv sc1) at every phase of every workgroup: a one-key batch
             * on these kernels ran 13% slower than on the single-key ones (profiles/r06e_mk_layout_probe.txt).
             */
            __threadfence_block();
            __syncthreads();
            const uint32_t k = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(mk.wg_key + blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (k == MK_NONE)
                break; /* uniform over the workgroup */
            /* the key's fields are wave-uniform: SGPRs, as the single-key kernels' arguments are (the round keys must be,
             * for the asm rounds) */
            const MkKey *kp = mk.keys + k;
            /* (readfirstlane returns int: each half widened as uint32_t, or a low half >= 2^31 would sign-extend over
             * the high half -- the first report of the fault journal) */
            const uint64_t ki_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)kp->ki),
                           ki_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)kp->ki >> 32));
            const KeyImage *kki = (const KeyImage *)(uintptr_t)(ki_hi << 32 | ki_lo);
            const uint32_t kfirst = __builtin_amdgcn_readfirstlane(kp->first),
                           count = __builtin_amdgcn_readfirstlane(kp->end) - kfirst;
            const uint32_t kiv0 = __builtin_amdgcn_readfirstlane(kp->iv0), kiv1 = __builtin_amdgcn_readfirstlane(kp->iv1),
                           kiv2 = __builtin_amdgcn_readfirstlane(kp->iv2);
            if (k != cur) { /* every wave is past the previous phase (the barrier at its end): the LDS is free */
                fill_lds_key(lds, kki, threadIdx.x, blockDim.x);
                cur = k;
            }
#pragma unroll
            for (int i = 0; i < 4 * (NR + 1); ++i) {
                rk[i] = __builtin_amdgcn_readfirstlane(kki->rk[i]);
                kr[i] = rotl32(rk[i], 16);
            }
            __syncthreads();
            const uint32_t ng = (count + R - 1u) / R;
            for (;;) {
                uint32_t g = 0;
                if (lane == 0)
                    g = atomicAdd(mk.ctr + k, 1u);
                g = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)g, 0, 64));
                if (g >= ng)
                    break;
                const uint32_t pos = g * R + slot;
                run_group(kfirst + pos, pos < count, kiv0, kiv1, kiv2);
            }
            kk = k;
            __syncthreads(); /* every wave is done with this key's tables */
        }
    }
}

/*
 * The TLS 1.3 padding strip (lib/picotls.c:4784-4791) over plaintext bytes [lo, n) of a record at pt: the position of
 * the last non-zero byte (the inner content type; the inner plaintext's length) and that byte, scanning back 16 bytes at
 * a time; found = 0xfffffffe if the bytes are all zero.
 */
__device__ __forceinline__ void strip_scan(const uint8_t *pt, uint32_t lo, uint32_t n, uint32_t &found, uint32_t &ty)
{
    found = 0xfffffffeu;
    ty = 0u;
    while (n > lo && found == 0xfffffffeu) {
        const uint32_t base = n - lo >= 16u ? n - 16u : lo;
        const u32x4 v = n - base == 16u ? *(const u32x4_u *)(pt + base) : load_partial(pt + base, n - base);
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
}

/*
 * The end of a record in the window kernels: seal writes the tag (and the TLS header), open verifies (acc = computed
 * tag ^ received tag), zeroes a failed record's plaintext and writes the status (and strips the TLS padding).  Run by
 * nt threads t = 0..nt-1 together; thread 0 does the single stores.
 * hint_found / hint_type: the strip's result if the caller already has it (split kernels), else 0xffffffff.
 */
template <bool SEAL, bool FRAME>
__device__ __forceinline__ void window_finish(u32x4 acc, bool valid, const Record &rec, uint32_t plen, uint32_t r, uint32_t t,
                                              uint32_t nt, uint8_t *dst, uint32_t *__restrict__ status,
                                              uint8_t *__restrict__ types, uint32_t hint_found = 0xffffffffu,
                                              uint32_t hint_type = 0u)
{
    if (SEAL) {
        if (t == 0u && valid) {
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
        for (uint32_t off = 16u * t; off < rec.len; off += 16u * nt) {
            const uint32_t n = rec.len - off;
            if (n >= 16u)
                *(u32x4_u *)(out + off) = u32x4{0u, 0u, 0u, 0u};
            else
                store_partial(out + off, n, u32x4{0u, 0u, 0u, 0u});
        }
        if (t == 0u) {
            status[r] = 0xffffffffu; /* SIZE_MAX / PTLS_ALERT_BAD_RECORD_MAC */
            if (FRAME)
                types[r] = 0u;
        }
    } else if (!FRAME) {
        if (t == 0u)
            status[r] = rec.len;
    } else if (t == 0u) {
        /* padding strip + content-type pop (lib/picotls.c:4784-4791) over plaintext the other slots (workgroups) wrote */
        uint32_t found = hint_found, ty = hint_type;
        if (found == 0xffffffffu) {
            __threadfence();
            strip_scan(dst + rec.dst, 0u, plen, found, ty); /* PTLS_ALERT_UNEXPECTED_MESSAGE (0xfffffffe) if all zero */
        }
        status[r] = found;
        types[r] = (uint8_t)ty;
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
template <int NR, bool SEAL, bool FRAME, int THREADS, int KW, int SEG = 64, class LW = LayoutWin<KW, SEG>>
__device__ __forceinline__ void window_body(const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2,
                                            const void *__restrict__ descs, uint32_t nrecs, const uint8_t *src, uint8_t *dst,
                                            const uint8_t *__restrict__ aad, uint32_t *__restrict__ status,
                                            uint8_t *__restrict__ types, const uint32_t *__restrict__ conn,
                                            const u32x4 *__restrict__ win_aes)
{
    /* SEG = 32: half-length segments, twice as many, half the steps (single-record latency kernels) */
    static_assert(SEG == 64 || SEG == 32, "segment length");
    constexpr uint32_t MAXSEG = SEG == 64 ? WIN_MAXSEG : WIN_SEG32_MAXSEG;
    constexpr uint32_t SLOTS = THREADS / KW, RECS = SLOTS / MAXSEG; /* records per workgroup pass */
    static_assert(RECS >= 1, "a workgroup holds at least one record");
    constexpr bool LATENCY = THREADS <= 576;   /* few records: up to 2-3 waves per SIMD */
    /*
     * join multiplies: the leader slot's KW lanes together (ghash_mul_coop) for 8 or 16 lanes per slot; otherwise
     * each lane alone, all reads in flight at 2 waves per SIMD (256 VGPRs), compiler-scheduled at 4
     */
    constexpr int JW = !LATENCY ? 0 : THREADS <= 512 ? 2 : 1;
    /* prefetch 3 steps ahead when little else hides a load (lane_walk); a 16-lane segment has only 2 steps */
    constexpr int WIN_PF = LATENCY && KW <= 8 ? 3 : 1;
    constexpr uint32_t LDS_BYTES = LW::parts_alias ? LayoutWin16::bytes : LW::parts + RECS * MAXSEG * 16u;
    static_assert(!LW::parts_alias || (RECS == 1 && LW::parts + MAXSEG * 16u <= LW::gh_base), "segment sums alias H^1..");
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
    const Record *__restrict__ recs = (const Record *)descs;
    const TlsRecord *__restrict__ trecs = (const TlsRecord *)descs;
    {
        const uint32_t grp = blockIdx.x;
        (void)grp;
        WIN_STAMP(0);
    }
    const uint32_t lane = threadIdx.x & 63u, slot = threadIdx.x / KW, j = lane % KW;
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u;
    const uint32_t rl = slot / MAXSEG, seg = slot % MAXSEG;
    const uint32_t ngroups = (nrecs + RECS - 1u) / RECS;
    auto join_mul = [&](uint32_t tab, u32x4 x) -> u32x4 {
        if constexpr (KW >= 8)
            return ghash_mul_coop<KW>(lds, tab, x, j);
        else
            return ghash_mul_join<JW>(lds, tab, x);
    };
    /* one record group's descriptor and segment walk */
    struct Group {
        Record rec;
        Walk sw;
        uint32_t r, ctype, plen, nseg, Tw, t0, n0, n1, n2;
        bool in_batch, valid, whole, active;
    };
    auto setup = [&](uint32_t grp) -> Group {
        Group g;
        g.r = grp * RECS + rl;
        g.in_batch = rl < RECS && g.r < nrecs;
        g.rec = Record{0, 0, 0, 0, 0, FRAME ? 5u : 0u};
        g.ctype = 0u;
        g.valid = g.in_batch;
        if (FRAME) {
            if (g.in_batch) {
                const TlsRecord t = trecs[g.r];
                g.rec.seq = t.seq;
                if (SEAL) {
                    g.rec.src = t.src;
                    g.rec.dst = t.dst + 5u;
                    g.rec.len = t.len;
                    g.ctype = t.type;
                    g.valid = t.len <= PTLS_MI355X_TLS_MAX_FRAGMENT; /* larger: not a TLS record, nothing written */
                } else {
                    g.rec.src = t.src + 5u;
                    g.rec.dst = t.dst;
                    g.rec.len = t.len >= 16u ? t.len - 16u : 0u;
                    g.valid = t.len >= 16u;
                }
            }
        } else if (g.in_batch) {
            g.rec = recs[g.r];
        }
        g.plen = FRAME && SEAL ? g.rec.len + 1u : g.rec.len;
        const uint32_t A = FRAME ? 1u : (g.rec.aadlen + 15u) / 16u;
        g.sw = window_segment(A, (g.plen + 15u) / 16u, seg, &g.nseg, (uint32_t)KW, (uint32_t)SEG);
        g.whole = g.nseg > MAXSEG; /* larger than a TLS record: its first slot walks it all */
        g.active = g.valid && (g.whole ? seg == 0u : seg < g.nseg);
        uint32_t Tw = g.active ? (g.whole ? make_walk(g.plen, g.rec.aadlen, (uint32_t)KW, walk_out16(dst + g.rec.dst)).T
                                          : g.sw.T)
                               : 0u;
        /* first step holding a real position (segments that are mostly front padding start late) */
        uint32_t tf = g.active && !g.whole && (int32_t)g.sw.pad > 0 ? (uint32_t)(int32_t)g.sw.pad / (uint32_t)KW
                                                                    : (g.active ? 0u : ~0u);
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            Tw = max(Tw, shfl_xor_u32(Tw, o));
            tf = min(tf, shfl_xor_u32(tf, o));
        }
        g.Tw = Tw;
        g.t0 = tf == ~0u ? 0u : tf & ~1u;
        g.n1 = iv1 ^ bswap32((uint32_t)(g.rec.seq >> 32));
        g.n2 = iv2 ^ bswap32((uint32_t)g.rec.seq);
        g.n0 = conn != nullptr && g.in_batch ? iv0 ^ bswap32(conn[g.r]) : iv0;
        return g;
    };
    /* latency kernels: the first group's descriptor is loaded before the LDS fill, its latency hidden under it (the
     * wide kernels, at the 128-VGPR cap, keep nothing live across the fill) */
    Group gr;
    if constexpr (LATENCY)
        gr = setup(blockIdx.x);
    if constexpr (LW::parts_alias) {
        /*
         * One pass: every thread loads its <= 18 vectors of the image (the AES rows, kept once per device in win_aes,
         * then the key image's tables from gh[0] on) before storing any, so the fill costs one memory latency.
         * (LDS DMA, global_load_lds_dwordx4, measured 2.3 us for the same image but left the walk 24 VGPRs short at
         * the 168-VGPR cap of 3 waves per SIMD, spilling inside the AES rounds.)
         */
        constexpr uint32_t NV = LayoutWin16::bytes / 16u, PER = (NV + THREADS - 1u) / THREADS;
        const u32x4 *gk = (const u32x4 *)&ki->gh[0][0][0][0];
        u32x4 v[PER];
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k) {
            const uint32_t i = threadIdx.x + k * THREADS;
            if (i < NV)
                v[k] = i < 0x1000u ? win_aes[i] : gk[i - 0x1000u];
        }
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k) {
            const uint32_t i = threadIdx.x + k * THREADS;
            if (i < NV)
                *(u32x4 *)(lds + 16u * i) = v[k];
        }
    } else {
        fill_lds_window(lds, c_tabs.t0, ki, threadIdx.x, blockDim.x, (uint32_t)KW, (uint32_t)SEG);
    }
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

    /* persistent: the workgroup fills its LDS once and takes record groups with a grid stride */
    for (uint32_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        if (!LATENCY || grp != blockIdx.x)
            gr = setup(grp);
        const uint32_t r = gr.r, ctype = gr.ctype, plen = gr.plen, nseg = gr.nseg;
        const bool in_batch = gr.in_batch, valid = gr.valid, whole = gr.whole, active = gr.active;
        const Record &rec = gr.rec;
        const Walk &sw = gr.sw;
        (void)ctype;
        u32x4 part = lane_walk_seg<NR, KW, SEAL, FRAME, LW, WIN_PF>(lds, lanesel, rk, j, rec, active, gr.Tw, gr.n0, gr.n1,
                                                                  gr.n2, src, dst, aad, (const uint8_t *)descs, gr.ctype,
                                                                  !whole, sw, gr.t0);
        if constexpr (KW >= 4) {
            part = dpp_xor_reduce4<KW>(part);
        } else {
#pragma unroll
            for (int o = 1; o < KW; o <<= 1)
                part ^= shfl_xor_u32x4(part, o);
        }
        WIN_STAMP(2);
        if constexpr (LW::parts_alias)
            __syncthreads(); /* every lane's scaling multiply is done: the sums may overwrite H^1.. */
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
                g = join_mul(LW::gh64, g) ^
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
                    *(u32x4 *)(lds + LW::parts + (rl * MAXSEG + seg) * 16u) = join_mul(LW::gh256, a) ^ b;
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
                        acc = join_mul(LW::ghpair, acc) ^
                              *(const u32x4 *)(lds + LW::parts + (rl * MAXSEG + window_group_start(g, ns)) * 16u);
                } else {
                    for (uint32_t k = window_group_end(0u, ns); k < ns; k += 4u)
                        acc = join_mul(LW::gh256, acc) ^
                              *(const u32x4 *)(lds + LW::parts + (rl * MAXSEG + k) * 16u);
                }
            }
            WIN_STAMP(4);
            window_finish<SEAL, FRAME>(acc, valid, rec, plen, r, j, (uint32_t)KW, dst, status, types);
        }
        __syncthreads(); /* the segment sums of this pass are consumed before the next pass writes them */
        WIN_STAMP(5);
    }
}

/*
 * Split window kernels (single-record latency): a record's 32-position segments (16 lanes each, one two-block trip) are
 * cut into runs of SPLIT_RUNSEG = 8 aligned to the record's end, and each run is walked by its own 128-thread
 * workgroup (one wave per SIMD) on its own CU: grid = records x SPLIT_MAXRUN, workgroup k of record r takes run k of R
 * (idle if k >= R).  A run joins its segment sums locally (groups of 4 with H^32, the two groups chained with H^128,
 * all with the slot's 16 lanes cooperating, ghash_mul_coop) and scales the result by H^(256 m) to the record's end
 * (m runs follow it).  The run then stores its partial, and the workgroup whose arrival ticket is the record's last XORs the R
 * partials -- E_K(J0) and, for open, the received tag are already folded into the last run's -- and finishes the
 * record (window_finish): tag and header, or verification, zeroing, status and padding strip.  The last arrival
 * resets the record's ticket, so the counters are zero between launches.  No workgroup waits for another.
 * A record of more than SPLIT_RUNSEG x SPLIT_MAXRUN segments (larger than a TLS record) is walked whole by run 0.
 */
template <int NR, bool SEAL, bool FRAME>
__device__ __forceinline__ void split_body(const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2,
                                           const void *__restrict__ descs, uint32_t nrecs, const uint8_t *src, uint8_t *dst,
                                           const uint8_t *__restrict__ aad, uint32_t *__restrict__ status,
                                           uint8_t *__restrict__ types, const uint32_t *__restrict__ conn,
                                           const u32x4 *__restrict__ win_aes, u32x4 *__restrict__ partials,
                                           uint32_t *__restrict__ tickets, uint8_t *lds, uint32_t r, uint32_t k)
{
    typedef LayoutSplit LW;
    constexpr int KW = 16;
    constexpr uint32_t SEG = 32, THREADS = SPLIT_THREADS;
    static_assert(THREADS / KW == SPLIT_RUNSEG, "one slot per segment of a run");
    /* after the walk: the 16 segment sums, then the arrival ticket, over the (dead) H^1 table */
    uint32_t *s_ticket = (uint32_t *)(lds + LW::parts + SPLIT_RUNSEG * 16u);
    uint32_t *s_hint = s_ticket + 1; /* the strip hint of open (two words) */
    if (r >= nrecs)
        return;
    /* the record (the same for every thread: scalar loads) */
    Record rec = {0, 0, 0, 0, 0, FRAME ? 5u : 0u};
    uint32_t ctype = 0u;
    bool valid = true;
    if (FRAME) {
        const TlsRecord t = ((const TlsRecord *)descs)[r];
        rec.seq = t.seq;
        if (SEAL) {
            rec.src = t.src;
            rec.dst = t.dst + 5u;
            rec.len = t.len;
            ctype = t.type;
            valid = t.len <= PTLS_MI355X_TLS_MAX_FRAGMENT;
        } else {
            rec.src = t.src + 5u;
            rec.dst = t.dst;
            rec.len = t.len >= 16u ? t.len - 16u : 0u;
            valid = t.len >= 16u;
        }
    } else {
        rec = ((const Record *)descs)[r];
    }
    const uint32_t plen = FRAME && SEAL ? rec.len + 1u : rec.len;
    const uint32_t A = FRAME ? 1u : (rec.aadlen + 15u) / 16u, C = (plen + 15u) / 16u;
    const uint32_t nseg = (A + C + 1u + SEG - 1u) / SEG;
    const bool whole = nseg > SPLIT_RUNSEG * SPLIT_MAXRUN;
    const uint32_t R = !valid || whole ? 1u : (nseg + SPLIT_RUNSEG - 1u) / SPLIT_RUNSEG;
    if (k >= R)
        return; /* uniform: the whole workgroup leaves before any barrier */
    SPLIT_STAMP(0);
    const uint32_t m = R - 1u - k; /* runs after this one */
    /* segment of slot 0 (negative: run 0's leading slots are empty), and the run's real segments */
    const int32_t first = (int32_t)nseg - (int32_t)(SPLIT_RUNSEG * (R - k));
    const uint32_t ns_run = whole ? 1u : (uint32_t)((int32_t)SPLIT_RUNSEG + min(first, 0));
    const uint32_t lane = threadIdx.x & 63u, slot = threadIdx.x / KW, j = lane % KW;
    const uint32_t lanesel = (lane & 31u) * 4u | 0x10000u;
    const int32_t segi = first + (int32_t)slot;
    const bool active = valid && (whole ? slot == 0u : segi >= 0 && segi < (int32_t)nseg);
    uint32_t nseg_chk;
    const Walk sw = window_segment(A, C, segi >= 0 ? (uint32_t)segi : 0u, &nseg_chk, (uint32_t)KW, SEG);
    uint32_t Tw = active ? (whole ? make_walk(plen, rec.aadlen, (uint32_t)KW, walk_out16(dst + rec.dst)).T : sw.T) : 0u;
    uint32_t tf = active && !whole && (int32_t)sw.pad > 0 ? (uint32_t)(int32_t)sw.pad / (uint32_t)KW : (active ? 0u : ~0u);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        Tw = max(Tw, shfl_xor_u32(Tw, o));
        tf = min(tf, shfl_xor_u32(tf, o));
    }
    const uint32_t t0 = tf == ~0u ? 0u : tf & ~1u;
    {
        /*
         * One pass: each thread loads its 40 vectors of the image before storing any.  (Loading the tables only the
         * scaling and the join read -- H^1..H^8, H^32, H^128, H^(256 m) -- by LDS DMA during the walk measured 2 us
         * SLOWER per window: profiles/r02l_split_ab.txt.)
         */
        constexpr uint32_t NV = LW::bytes / 16u, PER = NV / THREADS;
        static_assert(NV % THREADS == 0u, "whole passes");
        const u32x4 *gk = (const u32x4 *)&ki->gh[0][0][0][0];
        const u32x4 *gr = split_run_table(ki, m);
#if GCM_SPLIT_GLDS
        /*
         * LDS DMA (global_load_lds_dwordx4): a wave-instruction writes 64 x 16 B contiguously at a wave-uniform LDS
         * base, lane l's vector from its own global address, with no VGPR round trip and no ds_write transfer.  At one
         * wave per SIMD the walk has registers to spare, so nothing spills (unlike the 3-wave win16 layout).
         */
        const uint32_t wbase = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q) {
            const uint32_t i = threadIdx.x + q * THREADS;
            const u32x4 *g = i < 0x1000u ? win_aes + i : i < LW::gh_run / 16u ? gk + (i - 0x1000u) : gr + (i - LW::gh_run / 16u);
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1))) *)g,
                                             (void __attribute__((address_space(3))) *)(lds + 16u * (q * THREADS + wbase)),
                                             16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* this wave's DMA has landed; the barrier below covers the rest */
#else
        u32x4 v[PER];
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q) {
            const uint32_t i = threadIdx.x + q * THREADS;
            v[q] = i < 0x1000u ? win_aes[i] : i < LW::gh_run / 16u ? gk[i - 0x1000u] : gr[i - LW::gh_run / 16u];
        }
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q)
            *(u32x4 *)(lds + 16u * (threadIdx.x + q * THREADS)) = v[q];
#endif
    }
    uint32_t rk[4 * (NR + 1)];
#pragma unroll
    for (int i = 0; i < 4 * (NR + 1); ++i)
        rk[i] = ki->rk[i];
    __syncthreads();
    SPLIT_STAMP(1);

    const uint32_t n1 = iv1 ^ bswap32((uint32_t)(rec.seq >> 32)), n2 = iv2 ^ bswap32((uint32_t)rec.seq);
    const uint32_t n0 = conn != nullptr ? iv0 ^ bswap32(conn[r]) : iv0;
    u32x4 part = lane_walk_seg<NR, KW, SEAL, FRAME, LW, 1>(lds, lanesel, rk, j, rec, active, Tw, n0, n1, n2, src, dst, aad,
                                                          (const uint8_t *)descs, ctype, !whole, sw, t0);
    SPLIT_STAMP(2);
    part = dpp_xor_reduce4<KW>(part);
    /*
     * open: this run's plaintext reaches L2 before its arrival ticket, since the last run's window_finish reads it back
     * (padding strip) or zeroes it (failure).  seal: window_finish writes only the tag and the header, bytes no run
     * writes, so nothing orders this run's ciphertext (kernel completion does); the publishing lane's fence below
     * still orders its partial before its ticket.  Waiting for the stores here cost ~1.3 us per window.
     */
    if (R > 1u && !SEAL)
        __threadfence();
    __syncthreads(); /* every lane's scaling multiply is done: the sums may overwrite H^1.. */
    if (active && j == 0u)
        *(u32x4 *)(lds + LW::parts + slot * 16u) = part;
    __syncthreads();
    SPLIT_STAMP(3);
    /* the run's local join over its ns_run real segments; li = slot - off is the index among them */
    const uint32_t off = first < 0 ? (uint32_t)(-first) : 0u;
    const uint32_t li = slot - off;
    const bool real = valid && slot >= off && li < ns_run;
    if (real && window_group_leader(li, ns_run)) {
        u32x4 g = *(const u32x4 *)(lds + LW::parts + slot * 16u);
        for (uint32_t q = li + 1u; q < window_group_end(li, ns_run); ++q)
            g = ghash_mul_coop<KW>(lds, LW::gh_group, g, j) ^ *(const u32x4 *)(lds + LW::parts + (off + q) * 16u);
        *(u32x4 *)(lds + LW::parts + slot * 16u) = g;
    }
    __syncthreads();
    u32x4 acc = {0u, 0u, 0u, 0u};
    if (real && li == 0u) {
        acc = *(const u32x4 *)(lds + LW::parts + off * 16u);
        for (uint32_t q = window_group_end(0u, ns_run); q < ns_run; q += 4u)
            acc = ghash_mul_coop<KW>(lds, LW::gh_chain, acc, j) ^ *(const u32x4 *)(lds + LW::parts + (off + q) * 16u);
        if (m != 0u)
            acc = ghash_mul_coop<KW>(lds, LW::gh_run, acc, j);
        if (R > 1u && j == 0u) {
            /* publish the run's partial, then take an arrival ticket (release: the partial and this run's output) */
            partials[SPLIT_PSLOTS * r + k] = acc;
            __threadfence();
            *s_ticket = atomicAdd(&tickets[r], 1u);
        }
    }
    SPLIT_STAMP(4);
    if (R > 1u) {
        __syncthreads();
        SPLIT_STAMP(5);
        if (*s_ticket != R - 1u)
            return; /* not the last run of the record */
        SPLIT_STAMP_LAST(6);
        __threadfence(); /* acquire: every run's partial and output */
        if (real && li == 0u) {
            acc = u32x4{0u, 0u, 0u, 0u};
            for (uint32_t q = 0; q < R; ++q)
                acc ^= partials[SPLIT_PSLOTS * r + q];
            if (FRAME && !SEAL && j == 1u) {
                /*
                 * The padding strip's first 16 bytes, loaded beside the partials (one L2 round trip for both, instead of
                 * a second one in window_finish): almost every record's content type is in its last 16 bytes.  If they
                 * are all zero the finish scans the whole record (0xffffffff).
                 */
                uint32_t found, ty;
                strip_scan(dst + rec.dst, plen >= 16u ? plen - 16u : 0u, plen, found, ty);
                s_hint[0] = found == 0xfffffffeu && plen > 16u ? 0xffffffffu : found;
                s_hint[1] = ty;
            }
            if (j == 0u)
                tickets[r] = 0u; /* every run has arrived: zero for the next launch */
        }
    }
    /* the record's result to every thread (window_finish runs on all 256) */
    if (real && li == 0u && j == 0u)
        *(u32x4 *)(lds + LW::parts) = acc;
    __syncthreads();
    acc = *(const u32x4 *)(lds + LW::parts);
    const bool hinted = FRAME && !SEAL && R > 1u; /* s_hint written by the last-arrival block above */
    window_finish<SEAL, FRAME>(acc, valid, rec, plen, r, threadIdx.x, THREADS, dst, status, types,
                               hinted ? s_hint[0] : 0xffffffffu, hinted ? s_hint[1] : 0u);
    SPLIT_STAMP_LAST(7);
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

/* multi-key batches (K = 4, GH8): the records of many keys in one launch, `order` sorted by key (gcm_batch_body_mk) */
#define MI355X_GCM_KERNEL_MK(NAME, NR, SEAL, FRAME)                                                                    \
    extern "C" __global__ __launch_bounds__(WG_THREADS) void NAME(                                                     \
        const MkKey *__restrict__ keys, uint32_t nkeys, uint32_t *__restrict__ ctr, uint32_t *__restrict__ wg_key,     \
        const void *__restrict__ descs, const uint32_t *__restrict__ order, uint32_t nrecs, const uint8_t *src,        \
        uint8_t *dst, const uint8_t *__restrict__ aad, uint32_t *__restrict__ st, uint8_t *__restrict__ types,         \
        const uint32_t *__restrict__ conn)                                                                             \
    {                                                                                                                  \
        gcm_batch_body_mk<NR, 4, SEAL, FRAME>(descs, order, nrecs, src, dst, aad, st, types, conn,                    \
                                              MkLaunch{keys, nkeys, ctr, wg_key});                                     \
    }
MI355X_GCM_KERNEL_MK(mi355x_gcm_seal_aes128_k4_mk, 10, true, false)
MI355X_GCM_KERNEL_MK(mi355x_gcm_seal_aes256_k4_mk, 14, true, false)
MI355X_GCM_KERNEL_MK(mi355x_gcm_open_aes128_k4_mk, 10, false, false)
MI355X_GCM_KERNEL_MK(mi355x_gcm_open_aes256_k4_mk, 14, false, false)
MI355X_GCM_KERNEL_MK(mi355x_tls_seal_aes128_k4_mk, 10, true, true)
MI355X_GCM_KERNEL_MK(mi355x_tls_seal_aes256_k4_mk, 14, true, true)
MI355X_GCM_KERNEL_MK(mi355x_tls_open_aes128_k4_mk, 10, false, true)
MI355X_GCM_KERNEL_MK(mi355x_tls_open_aes256_k4_mk, 14, false, true)

/*
 * A multi-key record whose key index is out of range is not processed: seal writes nothing, open reports it as failing
 * (status 0xffffffff, type 0) with its output untouched -- never a record under another session's key.
 */
template <bool FRAME>
__device__ __forceinline__ void mk_reject(uint32_t r, uint32_t *__restrict__ st, uint8_t *__restrict__ types)
{
    if (st != nullptr) {
        st[r] = 0xffffffffu;
        if (FRAME && types != nullptr)
            types[r] = 0u;
    }
}

#define MI355X_WIN_KERNEL(NAME, NR, SEAL, FRAME, THREADS, KW)                                                              \
    extern "C" __global__ __launch_bounds__(THREADS) void NAME(                                                        \
        const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2, const void *__restrict__ descs,     \
        uint32_t nrecs, const uint8_t *src, uint8_t *dst, const uint8_t *__restrict__ aad, uint32_t *__restrict__ st,   \
        uint8_t *__restrict__ types, const uint32_t *__restrict__ conn, const u32x4 *__restrict__ win_aes)             \
    {                                                                                                                  \
        window_body<NR, SEAL, FRAME, THREADS, KW>(ki, iv0, iv1, iv2, descs, nrecs, src, dst, aad, st, types, conn,     \
                                                  win_aes);                                                            \
    }
/* single-record latency kernels: 32-position segments (4 steps of 8 lanes), one record per 512-thread group */
#ifndef MI355X_WIN32_THREADS
#define MI355X_WIN32_THREADS 512
#endif
#define MI355X_WIN32_KERNEL(NAME, NR, SEAL, FRAME)                                                                     \
    extern "C" __global__ __launch_bounds__(MI355X_WIN32_THREADS) void NAME(                                           \
        const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2, const void *__restrict__ descs,     \
        uint32_t nrecs, const uint8_t *src, uint8_t *dst, const uint8_t *__restrict__ aad, uint32_t *__restrict__ st,   \
        uint8_t *__restrict__ types, const uint32_t *__restrict__ conn, const u32x4 *__restrict__ win_aes)             \
    {                                                                                                                  \
        window_body<NR, SEAL, FRAME, MI355X_WIN32_THREADS, 8, 32>(ki, iv0, iv1, iv2, descs, nrecs, src, dst, aad, st,  \
                                                                  types, conn, win_aes);                             \
    }
MI355X_WIN32_KERNEL(mi355x_tls_win32_seal_aes128, 10, true, true)
MI355X_WIN32_KERNEL(mi355x_tls_win32_seal_aes256, 14, true, true)
MI355X_WIN32_KERNEL(mi355x_tls_win32_open_aes128, 10, false, true)
MI355X_WIN32_KERNEL(mi355x_tls_win32_open_aes256, 14, false, true)
MI355X_WIN32_KERNEL(mi355x_gcm_win32_seal_aes128, 10, true, false)
MI355X_WIN32_KERNEL(mi355x_gcm_win32_seal_aes256, 14, true, false)
MI355X_WIN32_KERNEL(mi355x_gcm_win32_open_aes128, 10, false, false)
MI355X_WIN32_KERNEL(mi355x_gcm_win32_open_aes256, 14, false, false)
/*
 * 16-lane single-record latency kernels: 32-position segments walked by 16 lanes in 2 steps (LayoutWin16), one
 * record (33 segments x 16 lanes = 528 lanes) per 576-thread group.
 */
#define MI355X_WIN16_KERNEL(NAME, NR, SEAL, FRAME)                                                                     \
    extern "C" __global__ __launch_bounds__(576) void NAME(                                                            \
        const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2, const void *__restrict__ descs,     \
        uint32_t nrecs, const uint8_t *src, uint8_t *dst, const uint8_t *__restrict__ aad, uint32_t *__restrict__ st,   \
        uint8_t *__restrict__ types, const uint32_t *__restrict__ conn, const u32x4 *__restrict__ win_aes)             \
    {                                                                                                                  \
        window_body<NR, SEAL, FRAME, 576, 16, 32, LayoutWin16>(ki, iv0, iv1, iv2, descs, nrecs, src, dst, aad, st,     \
                                                               types, conn, win_aes);                                \
    }
MI355X_WIN16_KERNEL(mi355x_tls_win16_seal_aes128, 10, true, true)
MI355X_WIN16_KERNEL(mi355x_tls_win16_seal_aes256, 14, true, true)
MI355X_WIN16_KERNEL(mi355x_tls_win16_open_aes128, 10, false, true)
MI355X_WIN16_KERNEL(mi355x_tls_win16_open_aes256, 14, false, true)
MI355X_WIN16_KERNEL(mi355x_gcm_win16_seal_aes128, 10, true, false)
MI355X_WIN16_KERNEL(mi355x_gcm_win16_seal_aes256, 14, true, false)
MI355X_WIN16_KERNEL(mi355x_gcm_win16_open_aes128, 10, false, false)
MI355X_WIN16_KERNEL(mi355x_gcm_win16_open_aes256, 14, false, false)

/* multi-key 16-lane kernels: one record per workgroup (grid = records), its key from its key index */
#define MI355X_WIN16_KERNEL_MK(NAME, NR, SEAL, FRAME)                                                                  \
    extern "C" __global__ __launch_bounds__(576) void NAME(                                                            \
        const MkKey *__restrict__ keys, uint32_t nkeys, const uint32_t *__restrict__ key_idx,                          \
        const void *__restrict__ descs, uint32_t nrecs, const uint8_t *src, uint8_t *dst,                              \
        const uint8_t *__restrict__ aad, uint32_t *__restrict__ st, uint8_t *__restrict__ types,                       \
        const uint32_t *__restrict__ conn, const u32x4 *__restrict__ win_aes)                                          \
    {                                                                                                                  \
        const uint32_t r = blockIdx.x, k = r < nrecs ? key_idx[r] : 0u;                                                \
        if (r >= nrecs)                                                                                                \
            return;                                                                                                    \
        if (k >= nkeys) {                                                                                              \
            if (!SEAL && threadIdx.x == 0u)                                                                            \
                mk_reject<FRAME>(r, st, types);                                                                        \
            return;                                                                                                    \
        }                                                                                                              \
        const MkKey key = keys[k];                                                                                     \
        window_body<NR, SEAL, FRAME, 576, 16, 32, LayoutWin16>(key.ki, key.iv0, key.iv1, key.iv2, descs, nrecs, src,   \
                                                               dst, aad, st, types, conn, win_aes);                    \
    }
MI355X_WIN16_KERNEL_MK(mi355x_tls_win16_seal_aes128_mk, 10, true, true)
MI355X_WIN16_KERNEL_MK(mi355x_tls_win16_seal_aes256_mk, 14, true, true)
MI355X_WIN16_KERNEL_MK(mi355x_tls_win16_open_aes128_mk, 10, false, true)
MI355X_WIN16_KERNEL_MK(mi355x_tls_win16_open_aes256_mk, 14, false, true)
MI355X_WIN16_KERNEL_MK(mi355x_gcm_win16_seal_aes128_mk, 10, true, false)
MI355X_WIN16_KERNEL_MK(mi355x_gcm_win16_seal_aes256_mk, 14, true, false)
MI355X_WIN16_KERNEL_MK(mi355x_gcm_win16_open_aes128_mk, 10, false, false)
MI355X_WIN16_KERNEL_MK(mi355x_gcm_win16_open_aes256_mk, 14, false, false)

/*
 * Split window kernels (split_body): SPLIT_MAXRUN 128-thread workgroups per record, each walking one run of 8
 * segments on its own CU; partials and arrival tickets in the context's split buffer.
 */
#define MI355X_SPLIT_KERNEL(NAME, NR, SEAL, FRAME)                                                                     \
    extern "C" __global__ __launch_bounds__(SPLIT_THREADS) void NAME(                                                  \
        const KeyImage *__restrict__ ki, uint32_t iv0, uint32_t iv1, uint32_t iv2, const void *__restrict__ descs,     \
        uint32_t nrecs, const uint8_t *src, uint8_t *dst, const uint8_t *__restrict__ aad, uint32_t *__restrict__ st,   \
        uint8_t *__restrict__ types, const uint32_t *__restrict__ conn, const u32x4 *__restrict__ win_aes,             \
        u32x4 *__restrict__ partials, uint32_t *__restrict__ tickets)                                                  \
    {                                                                                                                  \
        __shared__ __attribute__((aligned(16))) uint8_t lds[LayoutSplit::bytes];                                       \
        split_body<NR, SEAL, FRAME>(ki, iv0, iv1, iv2, descs, nrecs, src, dst, aad, st, types, conn, win_aes,           \
                                    partials, tickets, lds, blockIdx.x / SPLIT_MAXRUN, blockIdx.x % SPLIT_MAXRUN);     \
    }
MI355X_SPLIT_KERNEL(mi355x_tls_wins_seal_aes128, 10, true, true)
MI355X_SPLIT_KERNEL(mi355x_tls_wins_seal_aes256, 14, true, true)
MI355X_SPLIT_KERNEL(mi355x_tls_wins_open_aes128, 10, false, true)
MI355X_SPLIT_KERNEL(mi355x_tls_wins_open_aes256, 14, false, true)
MI355X_SPLIT_KERNEL(mi355x_gcm_wins_seal_aes128, 10, true, false)
MI355X_SPLIT_KERNEL(mi355x_gcm_wins_seal_aes256, 14, true, false)
MI355X_SPLIT_KERNEL(mi355x_gcm_wins_open_aes128, 10, false, false)
MI355X_SPLIT_KERNEL(mi355x_gcm_wins_open_aes256, 14, false, false)

/* multi-key split kernels: each record's key from its key index (a workgroup walks one run of one record) */
#define MI355X_SPLIT_KERNEL_MK(NAME, NR, SEAL, FRAME)                                                                  \
    extern "C" __global__ __launch_bounds__(SPLIT_THREADS) void NAME(                                                  \
        const MkKey *__restrict__ keys, uint32_t nkeys, const uint32_t *__restrict__ key_idx,                          \
        const void *__restrict__ descs, uint32_t nrecs, const uint8_t *src, uint8_t *dst,                              \
        const uint8_t *__restrict__ aad, uint32_t *__restrict__ st, uint8_t *__restrict__ types,                       \
        const uint32_t *__restrict__ conn, const u32x4 *__restrict__ win_aes, u32x4 *__restrict__ partials,             \
        uint32_t *__restrict__ tickets)                                                                                \
    {                                                                                                                  \
        __shared__ __attribute__((aligned(16))) uint8_t lds[LayoutSplit::bytes];                                       \
        const uint32_t r = blockIdx.x / SPLIT_MAXRUN, k = r < nrecs ? key_idx[r] : 0u;                                 \
        if (r >= nrecs)                                                                                                \
            return;                                                                                                    \
        if (k >= nkeys) {                                                                                              \
            if (!SEAL && blockIdx.x % SPLIT_MAXRUN == 0u && threadIdx.x == 0u)                                         \
                mk_reject<FRAME>(r, st, types);                                                                        \
            return;                                                                                                    \
        }                                                                                                              \
        const MkKey key = keys[k];                                                                                     \
        split_body<NR, SEAL, FRAME>(key.ki, key.iv0, key.iv1, key.iv2, descs, nrecs, src, dst, aad, st, types, conn,   \
                                    win_aes, partials, tickets, lds, r, blockIdx.x % SPLIT_MAXRUN);                    \
    }
MI355X_SPLIT_KERNEL_MK(mi355x_tls_wins_seal_aes128_mk, 10, true, true)
MI355X_SPLIT_KERNEL_MK(mi355x_tls_wins_seal_aes256_mk, 14, true, true)
MI355X_SPLIT_KERNEL_MK(mi355x_tls_wins_open_aes128_mk, 10, false, true)
MI355X_SPLIT_KERNEL_MK(mi355x_tls_wins_open_aes256_mk, 14, false, true)
MI355X_SPLIT_KERNEL_MK(mi355x_gcm_wins_seal_aes128_mk, 10, true, false)
MI355X_SPLIT_KERNEL_MK(mi355x_gcm_wins_seal_aes256_mk, 14, true, false)
MI355X_SPLIT_KERNEL_MK(mi355x_gcm_wins_open_aes128_mk, 10, false, false)
MI355X_SPLIT_KERNEL_MK(mi355x_gcm_wins_open_aes256_mk, 14, false, false)

/* the AES rows of the window image (window_image_vec, v < 4096), once per device: the 16-lane kernels copy them */
extern "C" __global__ void mi355x_win_aes_image(u32x4 *out)
{
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    if (v < 0x10000u / 16u)
        out[v] = window_image_vec(c_tabs.t0, nullptr, v, 8u, 32u);
}
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

/* ================================================================== cold kernels ========= */

/*
 * Key image setup (ptls_fusion_aesgcm_new, lib/fusion.c:775-795): one 1024-thread workgroup.
 *   1. thread 0: key expansion and H = E_K(0^128);
 *   2. wave 0: the 14 powers H^2..H^8, H^16, H^32, ..., H^1024 by wave-parallel multiplies
 *      (lane l forms Y x^l and Y x^(l+64), masks them by bits l, l+64 of X, the wave XOR-reduces);
 *   3. all threads: the 15 x 128 single-bit products P x^k (gf_mul_xpow), into LDS;
 *   4. all threads: the 15 x 32 x 16 nibble-table entries, each the XOR of <= 4 single-bit products.
 * Bit-identical to build_key_image (tests/test_kernel_model.py checks the same steps on the host).
 */
__device__ __forceinline__ Gf128 gf_wave_reduce(Gf128 v)
{
    uint32_t w[4] = {(uint32_t)(v.hi >> 32), (uint32_t)v.hi, (uint32_t)(v.lo >> 32), (uint32_t)v.lo};
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (int d = 0; d < 4; ++d)
            w[d] ^= shfl_xor_u32(w[d], o);
    return Gf128{((uint64_t)w[0] << 32) | w[1], ((uint64_t)w[2] << 32) | w[3]};
}

/* X * Y, every lane of the wave taking part (all lanes return the product) */
__device__ __forceinline__ Gf128 gf_mul_wave(Gf128 X, Gf128 Y, uint32_t lane) { return gf_wave_reduce(gf_mul_lane_share(X, Y, lane)); }

extern "C" __global__ __launch_bounds__(1024) void mi355x_gcm_setup(const uint8_t *key, uint32_t keylen, KeyImage *ki,
                                                                    int *rc)
{
    __shared__ Gf128 s_pow[KEY_IMAGE_TABLES];
    __shared__ Gf128 s_bit[KEY_IMAGE_TABLES][128];
    __shared__ uint32_t s_ok;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    if (tid == 0) {
        s_ok = 0u;
        if (keylen == 16u || keylen == 32u) {
            uint8_t k[32], h[16];
            for (uint32_t i = 0; i < keylen; ++i)
                k[i] = key[i];
            uint32_t rk[60];
            for (int i = 0; i < 60; ++i)
                rk[i] = 0u;
            const uint32_t nr = aes_expand_key(c_tabs.sbox, k, keylen, rk);
            const uint8_t zero[16] = {0};
            aes_encrypt_bytes(c_tabs.sbox, rk, nr, zero, h);
            for (int i = 0; i < 60; ++i)
                ki->rk[i] = rk[i];
            ki->rounds = nr;
            ki->key_size = keylen;
            ki->pad_[0] = ki->pad_[1] = 0u;
            for (int i = 0; i < 16; ++i)
                ki->H[i] = h[i];
            for (int i = 0; i < 32; ++i)
                k[i] = 0u;
            s_pow[0] = gf_from_bytes(h);
            s_ok = 1u;
        }
        *rc = s_ok ? 0 : -1;
    }
    __syncthreads();
    if (!s_ok)
        return;
    if (tid < 64u) {
        const Gf128 h = s_pow[0];
        Gf128 p = h;
        for (uint32_t e = 2; e <= (uint32_t)MAX_K; ++e) { /* H^2 .. H^8 */
            p = gf_mul_wave(p, h, lane);
            if (lane == 0)
                s_pow[e - 1] = p;
        }
        p = gf_mul_wave(p, p, lane); /* H^16 */
        if (lane == 0)
            s_pow[MAX_K + 4] = p;
        p = gf_mul_wave(p, p, lane); /* H^32 */
        if (lane == 0)
            s_pow[MAX_K + 2] = p;
        p = gf_mul_wave(p, p, lane); /* H^64 */
        if (lane == 0)
            s_pow[MAX_K] = p;
        p = gf_mul_wave(p, p, lane); /* H^128 */
        if (lane == 0)
            s_pow[MAX_K + 3] = p;
        p = gf_mul_wave(p, p, lane); /* H^256 */
        if (lane == 0)
            s_pow[MAX_K + 1] = p;
        const Gf128 p256 = p;
        p = gf_mul_wave(p, p, lane); /* H^512 */
        if (lane == 0)
            s_pow[MAX_K + 5] = p;
        const Gf128 p768 = gf_mul_wave(p, p256, lane); /* H^768 */
        if (lane == 0)
            s_pow[MAX_K + 7] = p768;
        p = gf_mul_wave(p, p, lane); /* H^1024 */
        if (lane == 0)
            s_pow[MAX_K + 6] = p;
    }
    __syncthreads();
    for (uint32_t i = tid; i < KEY_IMAGE_TABLES * 128u; i += blockDim.x)
        s_bit[i >> 7][i & 127u] = gf_mul_xpow(s_pow[i >> 7], i & 127u);
    __syncthreads();
    for (uint32_t i = tid; i < KEY_IMAGE_TABLES * 32u * 16u; i += blockDim.x)
        key_image_store_entry(ki, s_bit, i);
}

/* round keys of the ECB/CTR ciphers (one thread: a key schedule is 60 words) */
extern "C" __global__ void mi355x_aes_setup(const uint8_t *key, uint32_t keylen, AesKeys *out, int *rc)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        uint8_t k[32];
        for (uint32_t i = 0; i < keylen && i < 32u; ++i)
            k[i] = key[i];
        AesKeys ks;
        *rc = build_aes_keys(c_tabs.sbox, k, keylen, &ks);
        *out = ks;
        for (int i = 0; i < 32; ++i)
            k[i] = 0u;
    }
}

/*
 * AES-ECB over nblocks 16-byte blocks, grid-stride, one block per thread: encryption (FIPS-197 Cipher,
 * lib/fusion.c:187-197 aesecb_encrypt) or decryption (InvCipher, the equivalent inverse cipher of
 * FIPS-197 5.3.5).  The 1 KiB table and the (inverse) S-box sit in LDS.  Cold path: header protection
 * masks, the ECB/CTR cipher objects.
 */
template <bool DEC>
__device__ __forceinline__ void aes_ecb_body(const uint32_t *__restrict__ k, uint32_t nr, const uint8_t *in, uint8_t *out,
                                             uint32_t nblocks)
{
    __shared__ uint32_t s_t[256];
    __shared__ uint8_t s_s[256];
    for (uint32_t i = threadIdx.x; i < 256u; i += blockDim.x) {
        s_t[i] = DEC ? c_tabs.td0[i] : c_tabs.t0[i];
        s_s[i] = DEC ? c_tabs.inv_sbox[i] : c_tabs.sbox[i];
    }
    uint32_t rk[60];
    for (uint32_t i = 0; i < 4u * (nr + 1u); ++i)
        rk[i] = k[i];
    __syncthreads();
    for (uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < nblocks; b += (uint64_t)gridDim.x * blockDim.x) {
        const size_t off = (size_t)b * 16u; /* 64-bit: a batch may reach 2^32 - 1 blocks (64 GiB) */
        const u32x4 v = *(const u32x4_u *)(in + off);
        uint32_t w[4] = {v[0], v[1], v[2], v[3]};
        aes_ecb_block<DEC>(s_t, s_s, rk, nr, w);
        *(u32x4_u *)(out + off) = u32x4{w[0], w[1], w[2], w[3]};
    }
}

extern "C" __global__ __launch_bounds__(256) void mi355x_aes_ecb_enc(const uint32_t *k, uint32_t nr, const uint8_t *in,
                                                                     uint8_t *out, uint32_t nblocks)
{
    aes_ecb_body<false>(k, nr, in, out, nblocks);
}

extern "C" __global__ __launch_bounds__(256) void mi355x_aes_ecb_dec(const uint32_t *k, uint32_t nr, const uint8_t *in,
                                                                     uint8_t *out, uint32_t nblocks)
{
    aes_ecb_body<true>(k, nr, in, out, nblocks);
}

/*
 * Stop at the first failure (PTLS_MI355X_OPEN_STOP_AT_FAILURE): picotls stops reading at a record that
 * fails (aead_decrypt's SIZE_MAX -> PTLS_ALERT_BAD_RECORD_MAC, lib/picotls.c:650-652, or an all-zero
 * inner plaintext -> PTLS_ALERT_UNEXPECTED_MESSAGE, :4790) and never advances seq past it.  Record i is
 * "behind a failure" when a record j < i of the same connection (equal conn_ids over a contiguous run)
 * failed: fail_pos[i] = i for a failed record, else ~0; an inclusive min-scan by connection gives the
 * first failure at or before i; records strictly behind it are reset to NOT_PROCESSED and zeroed.
 */
extern "C" __global__ void mi355x_tls_fail_pos(const uint32_t *__restrict__ status, uint32_t n, uint32_t *fail_pos)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        fail_pos[i] = status[i] >= PTLS_MI355X_TLS_UNEXPECTED_MESSAGE ? i : 0xffffffffu;
}

extern "C" __global__ void mi355x_tls_truncate(const TlsRecord *__restrict__ recs, uint32_t n, const uint32_t *first_fail,
                                               uint8_t *dst, uint32_t *status, uint8_t *types)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || first_fail[i] >= i)
        return;
    status[i] = PTLS_MI355X_TLS_NOT_PROCESSED;
    types[i] = 0u;
    const TlsRecord t = recs[i];
    const uint32_t plen = t.len >= 16u ? t.len - 16u : 0u;
    uint8_t *p = dst + t.dst;
    for (uint32_t off = 0; off < plen; off += 16u) {
        if (plen - off >= 16u)
            *(u32x4_u *)(p + off) = u32x4{0u, 0u, 0u, 0u};
        else
            store_partial(p + off, plen - off, u32x4{0u, 0u, 0u, 0u});
    }
}

/*
 * Delivery of opened records (ptls_mi355x_tls_deliver_records): picotls' receive loop on the device.  Workgroup
 * (part, g) of a part's records [k0, k0 + n): thread 0 walks them in order as handle_input does -- stop at the first
 * failed record, at the first record of another inner content type (unless any_type: then one record of any type),
 * or at the first one that would overflow the capacity -- and the delivered records' plaintexts are copied back to
 * back into out, record i by the groups with i % gridDim.y == g.  The slots (plaintext, type, padding, as the open
 * kernels leave them) are read from `slots`; out is written once, at the compact offsets (no host memmove).  Parts
 * of more than DELIVER_MAX records are not handled here (the host falls back to its own loop).
 */
constexpr uint32_t DELIVER_MAX = PTLS_MI355X_DELIVER_MAX;

struct DeliverPart {
    const uint8_t *slots; /* record i's slot at slots + recs[i].dst */
    uint8_t *out;
    uint64_t capacity;
    uint32_t k0, n, any_type, pad_;
};
static_assert(sizeof(DeliverPart) == sizeof(ptls_mi355x_tls_deliver_t), "delivery layout");

/* dst[0, len) <- src[0, len) by one workgroup: 16-byte accesses when src and dst share their alignment mod 16 (slots
 * 16-aligned, plaintexts of whole 16-B blocks), else 4-byte stores from aligned source dwords (v_alignbyte) */
__device__ __forceinline__ void copy_bytes(uint8_t *dst, const uint8_t *src, uint32_t len, uint32_t tid, uint32_t nthr)
{
    const uint32_t a = (uint32_t)((uintptr_t)dst & 15u);
    if (a == (uint32_t)((uintptr_t)src & 15u)) {
        const uint32_t head = ((16u - a) & 15u) < len ? ((16u - a) & 15u) : len;
        if (tid < head)
            dst[tid] = src[tid];
        const uint32_t body = (len - head) / 16u, tail0 = head + 16u * body;
        const u32x4 *s4 = (const u32x4 *)(src + head);
        u32x4 *d4 = (u32x4 *)(dst + head);
        for (uint32_t w = tid; w < body; w += nthr)
            d4[w] = s4[w];
        if (tid < len - tail0)
            dst[tail0 + tid] = src[tail0 + tid];
        return;
    }
    const uint32_t head = ((4u - (a & 3u)) & 3u) < len ? ((4u - (a & 3u)) & 3u) : len;
    if (tid < head)
        dst[tid] = src[tid];
    const uint32_t body = (len - head) / 4u, tail0 = head + 4u * body;
    const uint8_t *s = src + head;
    const uint32_t sh = (uint32_t)((uintptr_t)s & 3u);
    const uint32_t *sa = (const uint32_t *)(s - sh);
    uint32_t *d = (uint32_t *)(dst + head);
    for (uint32_t w = tid; w < body; w += nthr) {
        const uint32_t lo = sa[w];
        const uint32_t hi = sh ? sa[w + 1] : 0u; /* (inside the slot: the type byte follows the plaintext) */
        d[w] = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
    }
    if (tid < len - tail0)
        dst[tail0 + tid] = src[tail0 + tid];
}

/* workgroup (part, g) of G: off[DELIVER_MAX + 1] and *ndone in LDS */
__device__ __forceinline__ void deliver_body(const TlsRecord *__restrict__ recs, const uint32_t *__restrict__ status,
                                             const uint8_t *__restrict__ types, const DeliverPart *__restrict__ parts,
                                             uint32_t part, uint32_t g, uint32_t G, uint32_t *off, uint32_t *ndone_)
{
    uint32_t &ndone = *ndone_;
    const DeliverPart p = parts[part];
    const uint32_t n = p.n < DELIVER_MAX ? p.n : DELIVER_MAX;
    /*
     * Every thread loads some records' status and type (in parallel: one dependent load per record in thread 0's loop
     * cost ~2 us each, 92 us for a 16-record window), leaving in off[i] the plaintext length, or ~0 where the receive
     * loop stops (a failure, or another content type); thread 0 then walks off[] in LDS.
     */
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
        const uint32_t st = status[p.k0 + i];
        const uint8_t ty = types[p.k0 + i];
        off[i] = st >= PTLS_MI355X_TLS_NOT_PROCESSED || (!p.any_type && ty != 23u) ? 0xffffffffu : st;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t o = 0u, i = 0u;
        for (; i < n; ++i) {
            const uint32_t st = off[i];
            if (st == 0xffffffffu || (uint64_t)o + st > p.capacity)
                break;
            off[i] = o;
            o += st;
            if (p.any_type) {
                ++i;
                break;
            }
        }
        off[i] = o;
        ndone = i;
    }
    __syncthreads();
    const uint32_t nd = ndone;
    for (uint32_t i = g; i < nd; i += G) {
        const uint64_t rdst = recs[p.k0 + i].dst;
        copy_bytes(p.out + off[i], p.slots + rdst, off[i + 1] - off[i], threadIdx.x, blockDim.x);
    }
}

extern "C" __global__ __launch_bounds__(256) void mi355x_tls_deliver(const TlsRecord *__restrict__ recs,
                                                                      const uint32_t *__restrict__ status,
                                                                      const uint8_t *__restrict__ types,
                                                                      const DeliverPart *__restrict__ parts)
{
    __shared__ uint32_t off[DELIVER_MAX + 1];
    __shared__ uint32_t ndone;
    deliver_body(recs, status, types, parts, blockIdx.x, blockIdx.y, gridDim.y, off, &ndone);
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

/* ---- multi-key prep (ptls_mi355x_*_multikey): records sorted by key, each key's range in the key table ---- */
/* sort input: the record's key index (out of range -> nkeys, sorted after every key) and its descriptor index */
extern "C" __global__ void mi355x_mk_keys(const uint32_t *__restrict__ key_idx, uint32_t n, uint32_t nkeys,
                                          uint32_t *__restrict__ keys, uint32_t *__restrict__ vals)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t k = key_idx[i];
        keys[i] = k < nkeys ? k : nkeys;
        vals[i] = i;
    }
}

/*
 * Grouping by key as a counting sort (nkeys + 1 buckets up to MK_LDS_BUCKETS, the last for out-of-range indices): each
 * workgroup counts its MK_PER_BLOCK records' keys in LDS and adds them to the global counts; an exclusive scan gives
 * each key's first position; each workgroup counts again, reserves its run of every key with one global atomic, and
 * places its records by LDS atomics.  Not stable (within a key the order is the atomics'), which a multi-key launch does
 * not need.  (hipcub's radix sort took ~82 us for 1 M keys of 7 bits: a block sort and ten merge passes.)
 */
constexpr uint32_t MK_LDS_BUCKETS = 8192, MK_PER_BLOCK = 4096;

/*
 * A wave's LDS counter adds.  Same-address LDS atomics of a wave serialise, so a wave whose lanes all carry one key (a
 * batch of one session, or a session's contiguous run) takes one atomic for the whole wave; any other wave one atomic
 * per lane, as before (measured: serving the lanes key by key with ballots costs more than the LDS's own serialisation
 * once a wave holds two or more keys, profiles/r06x_mk_prep.txt).  Returns the counter's value before the lane's unit
 * (its slot in the key's run).  Called by the whole wave (uniform trip counts).
 */
__device__ __forceinline__ uint32_t mk_lds_add(uint32_t *h, uint32_t k, bool valid)
{
    const uint64_t act = __ballot(valid);
    if (act == 0ull)
        return 0u;
    const int src = __builtin_ctzll(act);
    const uint32_t k0 = (uint32_t)__shfl((int)k, src, 64);
    if (__ballot(valid && k == k0) == act) { /* one key in the wave: one atomic */
        const uint32_t lane = __lane_id();
        uint32_t base = 0u;
        if (lane == (uint32_t)src)
            base = atomicAdd(&h[k0], (uint32_t)__popcll(act));
        base = (uint32_t)__shfl((int)base, src, 64);
        return base + (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
    }
    return valid ? atomicAdd(&h[k], 1u) : 0u;
}

extern "C" __global__ __launch_bounds__(1024) void mi355x_mk_count(const uint32_t *__restrict__ key_idx, uint32_t n,
                                                                   uint32_t nkeys, uint32_t *__restrict__ counts)
{
    __shared__ uint32_t h[MK_LDS_BUCKETS];
    const uint32_t nb = nkeys + 1u;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
        h[b] = 0u;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * MK_PER_BLOCK, i1 = min(n, i0 + MK_PER_BLOCK);
    for (uint32_t b0 = i0; b0 < i1; b0 += blockDim.x) { /* uniform over the block: every wave calls mk_lds_add */
        const uint32_t i = b0 + threadIdx.x;
        const bool valid = i < i1;
        const uint32_t k = valid ? key_idx[i] : 0u;
        (void)mk_lds_add(h, k < nkeys ? k : nkeys, valid);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
        if (h[b] != 0u)
            atomicAdd(counts + b, h[b]);
}

extern "C" __global__ __launch_bounds__(1024) void mi355x_mk_scatter(const uint32_t *__restrict__ key_idx, uint32_t n,
                                                                     uint32_t nkeys, uint32_t *__restrict__ cursor,
                                                                     uint32_t *__restrict__ order)
{
    __shared__ uint32_t h[MK_LDS_BUCKETS];
    const uint32_t nb = nkeys + 1u;
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
        h[b] = 0u;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * MK_PER_BLOCK, i1 = min(n, i0 + MK_PER_BLOCK);
    for (uint32_t b0 = i0; b0 < i1; b0 += blockDim.x) {
        const uint32_t i = b0 + threadIdx.x;
        const bool valid = i < i1;
        const uint32_t k = valid ? key_idx[i] : 0u;
        (void)mk_lds_add(h, k < nkeys ? k : nkeys, valid);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) /* this block's run of key b: one global atomic */
        if (h[b] != 0u)
            h[b] = atomicAdd(cursor + b, h[b]);
    __syncthreads();
    for (uint32_t b0 = i0; b0 < i1; b0 += blockDim.x) {
        const uint32_t i = b0 + threadIdx.x;
        const bool valid = i < i1;
        const uint32_t k = valid ? key_idx[i] : 0u;
        const uint32_t pos = mk_lds_add(h, k < nkeys ? k : nkeys, valid);
        if (valid)
            order[pos] = i;
    }
}

/* every key's range empty and its group counter zero (before mi355x_mk_bounds) */
extern "C" __global__ void mi355x_mk_reset(MkKey *__restrict__ keys, uint32_t nkeys, uint32_t *__restrict__ ctr)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nkeys) {
        keys[k].first = 0u;
        keys[k].end = 0u;
        ctr[k] = 0u;
    }
}

/* each key's range [first, end) in the sorted order; an out-of-range key's record fails an open (mk_reject) */
__device__ __forceinline__ uint32_t mk_sorted_key(const uint32_t *sorted, const uint32_t *key_idx, const uint32_t *order,
                                                  uint32_t i, uint32_t nkeys)
{
    if (sorted != nullptr)
        return sorted[i];
    const uint32_t k = key_idx[order[i]]; /* a caller's order (ptls_mi355x_order_by_key) */
    return k < nkeys ? k : nkeys;
}

extern "C" __global__ void mi355x_mk_bounds(const uint32_t *__restrict__ sorted, const uint32_t *__restrict__ key_idx,
                                            const uint32_t *__restrict__ order, uint32_t n, uint32_t nkeys,
                                            MkKey *__restrict__ keys, uint32_t *__restrict__ st,
                                            uint8_t *__restrict__ types, uint32_t frame)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t k = mk_sorted_key(sorted, key_idx, order, i, nkeys);
    if (k >= nkeys) {
        if (frame)
            mk_reject<true>(order[i], st, types);
        else
            mk_reject<false>(order[i], st, types);
        return;
    }
    if (i == 0u || mk_sorted_key(sorted, key_idx, order, i - 1u, nkeys) != k)
        keys[k].first = i;
    if (i + 1u == n || mk_sorted_key(sorted, key_idx, order, i + 1u, nkeys) != k)
        keys[k].end = i + 1u;
}

/*
 * mi355x_mk_reset + mi355x_mk_bounds in one pass (up to MK_LDS_BUCKETS - 1 keys, so a thread's run of empty keys is
 * short): in the sorted order, the record where a new key starts also writes the ranges of the keys skipped since the
 * previous record's key (empty: first = end = i), the last record those above its key (first = end = n), and threads
 * below nkeys zero the group counters.  One launch fewer per multi-key call.
 */
extern "C" __global__ void mi355x_mk_bounds_all(const uint32_t *__restrict__ key_idx, const uint32_t *__restrict__ order,
                                                uint32_t n, uint32_t nkeys, MkKey *__restrict__ keys,
                                                uint32_t *__restrict__ ctr, uint32_t *__restrict__ st,
                                                uint8_t *__restrict__ types, uint32_t frame)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, lane = __lane_id();
    if (i < nkeys)
        ctr[i] = 0u;
    /* each record's key gathered once (key_idx[order[i]]); its neighbours' from the adjacent lanes, a wave's two edge
     * lanes gathering their own (every lane takes part in the shuffles) */
    const uint32_t k = i < n ? mk_sorted_key(nullptr, key_idx, order, i, nkeys) : nkeys;
    uint32_t kp = (uint32_t)__shfl_up((int)k, 1, 64), kn = (uint32_t)__shfl_down((int)k, 1, 64);
    if (i >= n)
        return;
    if (lane == 0u && i != 0u)
        kp = mk_sorted_key(nullptr, key_idx, order, i - 1u, nkeys);
    if (lane == 63u && i + 1u < n)
        kn = mk_sorted_key(nullptr, key_idx, order, i + 1u, nkeys);
    if (i == 0u || k != kp) {
        for (uint32_t e = i == 0u ? 0u : kp + 1u; e < k && e < nkeys; ++e) { /* keys with no record */
            keys[e].first = i;
            keys[e].end = i;
        }
        if (k < nkeys)
            keys[k].first = i;
    }
    if (k >= nkeys) {
        if (frame)
            mk_reject<true>(order[i], st, types);
        else
            mk_reject<false>(order[i], st, types);
    } else if (i + 1u == n || kn != k) {
        keys[k].end = i + 1u;
    }
    if (i + 1u == n)
        for (uint32_t e = k + 1u; e < nkeys; ++e) { /* keys above the last record's */
            keys[e].first = n;
            keys[e].end = n;
        }
}

/* stop-at-failure segments of a multi-key open: a connection is (key, connection id) */
extern "C" __global__ void mi355x_mk_segkeys(const uint32_t *__restrict__ key_idx, const uint32_t *__restrict__ conn,
                                             uint32_t n, uint64_t *__restrict__ out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = (uint64_t)key_idx[i] << 32 | (conn != nullptr ? conn[i] : 0u);
}

/* ================================================================== host side ============ */

typedef void (*batch_kernel_t)(const KeyImage *, uint32_t, uint32_t, uint32_t, const void *, const uint32_t *, uint32_t,
                               const uint8_t *, uint8_t *, const uint8_t *, uint32_t *, uint8_t *, uint32_t *,
                               uint32_t, const uint32_t *);
typedef void (*win_kernel_t)(const KeyImage *, uint32_t, uint32_t, uint32_t, const void *, uint32_t, const uint8_t *,
                             uint8_t *, const uint8_t *, uint32_t *, uint8_t *, const uint32_t *, const u32x4 *);
typedef void (*split_kernel_t)(const KeyImage *, uint32_t, uint32_t, uint32_t, const void *, uint32_t, const uint8_t *,
                               uint8_t *, const uint8_t *, uint32_t *, uint8_t *, const uint32_t *, const u32x4 *, u32x4 *,
                               uint32_t *);

constexpr uint32_t WORK_SLOTS = 256; /* per-context ring of work counters: one per launch in flight */

/*
 * Per-device resources shared by every context on the device (created on first use, kept for the
 * process): the stream and the pinned, mapped staging buffer of the synchronous calls (slot calls, ECB
 * cipher, key setup).  The mutex serialises those calls per device; the buffer never holds key material
 * or records after a call returns.
 */
struct DeviceShared {
    std::mutex mu;
    hipStream_t stream = nullptr;
    uint8_t *d_stage = nullptr;     /* device staging (records above the zero-copy limit) */
    uint8_t *h_stage = nullptr;     /* pinned host staging (mapped, coherent) */
    uint8_t *h_stage_dev = nullptr; /* h_stage as the GPU addresses it */
    size_t cap = 0;
    u32x4 *d_win_aes = nullptr;     /* the 64 KiB AES image of the 16-lane window kernels (mi355x_win_aes_image) */
    bool copies_ready = false;      /* ptls_mi355x_prepare_copies done */
};

struct st_ptls_mi355x_aesgcm_context {
    int device;
    int num_cu;
    uint32_t key_size;
    KeyImage *d_ki;
    DeviceShared *shared;
    uint32_t *d_work;               /* WORK_SLOTS dynamic-scheduling ticket counters, set once at setup */
    uint32_t work_base[WORK_SLOTS]; /* each counter's value at the start of its next launch */
    uint32_t work_next;
    void *d_scratch;                /* order_by_length / stop-at-failure workspace */
    size_t scratch_cap;
    u32x4 *d_split;                 /* split window kernels: SPLIT_MAXRUN partials per record, then the tickets */
    size_t split_cap;               /* records the buffer holds */
    /*
     * Stream ordering of the shared resources (work slots, split tickets, scratch).  A context launches on the first
     * stream it is given ("home"); while every launch goes there, stream order alone keeps two launches from sharing a
     * resource at once.  The first launch on another stream synchronises the device once (everything queued before it
     * is done) and switches the context to multi-stream mode: from then on each use of a resource records that
     * resource's event on the stream of the use, right after the use, and the next use on any stream first waits on
     * it -- never an event recorded later on a stored stream handle, which may have been destroyed since.
     */
    hipStream_t home;
    bool home_set, multi;
    hipEvent_t work_ev[WORK_SLOTS]; /* multi-stream mode: the slot's last launch (created on first use) */
    bool work_ev_valid[WORK_SLOTS];
    hipEvent_t split_ev, scratch_ev;
    bool split_ev_valid, scratch_ev_valid;
    /* multi-key launches led by this context: the key table last uploaded (pinned host copy), where it went, and the
     * event after its upload (the host copy is rewritten only once that copy is done) */
    MkKey *mk_host;
    size_t mk_cap, mk_n;
    const void *mk_dev;
    hipEvent_t mk_ev;
    bool mk_ev_valid;
};

struct st_ptls_mi355x_aes_context {
    int device;
    int num_cu;
    uint32_t key_size, rounds;
    AesKeys *d_keys;
    DeviceShared *shared;
};

static thread_local char g_err[256];
/* the tuning knobs below are process-wide and may be set from any thread: atomics, each read once per decision */
static std::atomic<int> g_lanes{4};
/* framing batches of at most this many records go to the window kernels (ptls_mi355x_set_tls_window_records) */
static std::atomic<size_t> g_window_records{16384};
/* AEAD batches (section 3) of at most this many records go to the window kernels (ptls_mi355x_set_aead_window_records):
 * the single-record slot calls and small batches, where 4 lanes per record would leave the GPU idle */
static std::atomic<size_t> g_aead_window_records{2048}; /* break-even of 1400-B records (scripts/window_bench.py aead_batches) */
/* single-record slot calls staging at most this many bytes run zero-copy (ptls_mi355x_set_slot_zero_copy_bytes) */
static std::atomic<size_t> g_slot_zero_copy_bytes{1u << 20};
/* starting value of new contexts' work counters (ptls_mi355x_set_work_ticket_origin; tests the 2^32 wrap) */
static std::atomic<uint32_t> g_ticket_origin{0u};
/* window batches of at most this many records use 32-position segments (ptls_mi355x_set_seg32_records;
 * SIZE_MAX = the device's CU count) */
static std::atomic<size_t> g_seg32_records{SIZE_MAX};
/* window batches of at most this many records use the 16-lane single-record kernels (ptls_mi355x_set_win16_records;
 * SIZE_MAX = the device's CU count); they take precedence over the 32-position 8-lane ones */
static std::atomic<size_t> g_win16_records{SIZE_MAX};
/* window batches of at most this many records use the split kernels, SPLIT_MAXRUN workgroups per record
 * (ptls_mi355x_set_split_records; SIZE_MAX = CU count / SPLIT_MAXRUN); they take precedence over the others */
static std::atomic<size_t> g_split_records{SIZE_MAX};

static int fail(const char *what, hipError_t e)
{
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return -1;
}

/*
 * Errors met where the API returns nothing (the free paths: ptls_fusion_aesgcm_free is void, include/picotls/fusion.h:
 * 60).  A synchronisation there is where an asynchronous fault of earlier work surfaces; it is printed, kept for
 * ptls_mi355x_device_check, and never dropped, so the next unrelated call is not the one blamed for it.
 */
static std::mutex g_deferred_mu;
constexpr int MAX_DEVICES = 64;
static char g_deferred[MAX_DEVICES][256]; /* per device ordinal: the first error deferred on it since its last check */

extern "C" void ptls_mi355x_defer_error(const char *what, int err)
{
    if (err == (int)hipSuccess)
        return;
    const char *msg = hipGetErrorString((hipError_t)err);
    fprintf(stderr, "ptls_mi355x: %s: %s\n", what, msg);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAX_DEVICES)
        dev = 0; /* (the free paths run with the context's device current: DeviceGuard) */
    std::lock_guard<std::mutex> lk(g_deferred_mu);
    if (g_deferred[dev][0] == 0)
        snprintf(g_deferred[dev], sizeof(g_deferred[dev]), "%s: %s", what, msg);
}

static void defer(const char *what, hipError_t e) { ptls_mi355x_defer_error(what, (int)e); }

#define HIPCHK(call)                                                                                                   \
    do {                                                                                                               \
        hipError_t e_ = (call);                                                                                        \
        if (e_ != hipSuccess)                                                                                          \
            return fail(#call, e_);                                                                                    \
    } while (0)

/* runs `body` with the context's device current, restoring the caller's device; ok = false if it could not be made
 * current (an absent ordinal: the caller's device stays current, so the caller must check before doing work) */
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) {
            ok = false;
            prev = -1;
        } else if (prev != dev) {
            ok = hipSetDevice(dev) == hipSuccess;
            if (!ok) {
                (void)hipGetLastError();
                prev = -1;
            }
        } else {
            prev = -1;
        }
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

static std::mutex g_shared_mu;
static DeviceShared *g_shared[64];

/* the device's shared resources (the device must be current) */
static DeviceShared *device_shared(int dev)
{
    if (dev < 0 || dev >= 64) {
        snprintf(g_err, sizeof(g_err), "device ordinal %d out of range", dev);
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_shared_mu);
    if (g_shared[dev] == nullptr) {
        DeviceShared *d = new (std::nothrow) DeviceShared();
        if (d == nullptr)
            return nullptr;
        hipError_t e = hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            fail("hipStreamCreateWithFlags", e);
            delete d;
            return nullptr;
        }
        e = hipMalloc(&d->d_win_aes, 0x10000);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(mi355x_win_aes_image, dim3(16), dim3(256), 0, d->stream, d->d_win_aes);
            e = hipGetLastError();
        }
        if (e == hipSuccess)
            e = hipStreamSynchronize(d->stream);
        if (e != hipSuccess) {
            fail("window AES image", e);
            if (d->d_win_aes)
                (void)hipFree(d->d_win_aes);
            (void)hipStreamDestroy(d->stream);
            delete d;
            return nullptr;
        }
        g_shared[dev] = d;
    }
    return g_shared[dev];
}

/* a kernel between the copies of ptls_mi355x_prepare_copies (it only has to run) */
__global__ void mi355x_copy_warm(uint32_t *p) { p[threadIdx.x] = threadIdx.x; }

/*
 * The HIP runtime sets up parts of its copy machinery on first need, inside the hipMemcpyAsync call that needs it:
 * the first host <-> device copy of 64 KiB or more, the first time four streams each have a copy and a kernel in
 * flight, and again whenever more copies are in flight than ever before (8 per stream) -- each stalled that call
 * 8-30 ms (scripts/probe_h2d.c).  A record layer moving windows by DMA hit these mid-stream, at whatever window first
 * grew its groups or its copies in flight that far: a timed stream of 64 coalesced windows then ran at 1-2 GiB/s
 * instead of 21.  This pays them once per process and device, up front: [64 KiB H2D, kernel,
 * 64 KiB D2H] x depth on four streams at once, depth 1, 4, 16 and 64 (768 copies in flight at the last), synchronised
 * after each depth.
 */
int ptls_mi355x_prepare_copies(void)
{
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    DeviceShared *d = device_shared(dev);
    if (d == nullptr)
        return -1;
    std::lock_guard<std::mutex> lk(d->mu);
    if (d->copies_ready)
        return 0;
    const size_t n = 64u << 10;
    uint8_t *h = nullptr, *dv = nullptr;
    hipStream_t st[4] = {};
    hipError_t e = hipHostMalloc((void **)&h, 4 * n, hipHostMallocDefault);
    if (e == hipSuccess)
        e = hipMalloc((void **)&dv, 4 * n);
    for (int i = 0; i < 4 && e == hipSuccess; ++i)
        e = hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking);
    if (e == hipSuccess)
        memset(h, 0, 4 * n);
    for (int depth = 1; depth <= 64 && e == hipSuccess; depth *= 4) {
        for (int k = 0; k < depth && e == hipSuccess; ++k)
            for (int i = 0; i < 4 && e == hipSuccess; ++i) { /* (one stream's copies are ordered: one buffer each) */
                e = hipMemcpyAsync(dv + i * n, h + i * n, n, hipMemcpyHostToDevice, st[i]);
                if (e == hipSuccess) {
                    hipLaunchKernelGGL(mi355x_copy_warm, dim3(1), dim3(64), 0, st[i], (uint32_t *)(dv + i * n));
                    e = hipGetLastError();
                }
                if (e == hipSuccess)
                    e = hipMemcpyAsync(h + i * n, dv + i * n, n, hipMemcpyDeviceToHost, st[i]);
            }
        for (int i = 0; i < 4; ++i)
            if (st[i] != nullptr) {
                const hipError_t es = hipStreamSynchronize(st[i]);
                e = e == hipSuccess ? es : e;
            }
    }
    for (int i = 0; i < 4; ++i)
        if (st[i] != nullptr)
            (void)hipStreamDestroy(st[i]);
    if (dv != nullptr)
        defer("prepare copies: hipFree", hipFree(dv));
    if (h != nullptr)
        defer("prepare copies: hipHostFree", hipHostFree(h));
    if (e != hipSuccess)
        return fail("prepare copies", e);
    d->copies_ready = true;
    return 0;
}

/* grows the shared staging to `need` bytes (caller holds d->mu) */
static int ensure_stage(DeviceShared *d, size_t need)
{
    if (need <= d->cap)
        return 0;
    size_t cap = d->cap ? d->cap : 4096;
    while (cap < need)
        cap *= 2;
    const size_t cap_old = d->cap;
    d->cap = 0; /* (nothing is left half-freed for a later call if a free below fails) */
    if (d->d_stage) {
        /* the last copied call's clear of the staging may still be queued on the device stream: it ends first (an
         * explicit wait, not hipFree's implicit one) */
        HIPCHK(hipStreamSynchronize(d->stream));
        JNOTE("hipFree shared staging", d->d_stage, cap_old);
        HIPCHK(hipFree(d->d_stage));
    }
    d->d_stage = nullptr;
    if (d->h_stage) {
        JNOTE("hipHostFree shared staging", d->h_stage_dev, cap_old);
        HIPCHK(hipHostFree(d->h_stage));
    }
    d->h_stage = nullptr;
    d->h_stage_dev = nullptr;
    HIPCHK(hipMalloc(&d->d_stage, cap));
    /* coherent: the GPU's zero-copy reads never see stale cache lines of a previous call */
    HIPCHK(hipHostMalloc(&d->h_stage, cap, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void **)&d->h_stage_dev, d->h_stage, 0));
    JNOTE("hipMalloc shared staging", d->d_stage, cap);
    JNOTE("hipHostMalloc shared staging (device view)", d->h_stage_dev, cap);
    d->cap = cap;
    return 0;
}

/* ------------------------------------------------------------------ kernel selection ----- */

struct LaunchPlan {
    const char *name = "";
    batch_kernel_t batch = nullptr;
    win_kernel_t win = nullptr;
    split_kernel_t split = nullptr;
    uint32_t blocks = 0, threads = 0;
    uint32_t k = 0; /* batch kernels: lanes per record (the work-ticket count of the launch follows it) */
};

#define KN(f) {#f, f}
struct BatchEntry {
    const char *name;
    batch_kernel_t f;
};
struct WinEntry {
    const char *name;
    win_kernel_t f;
};
struct SplitEntry {
    const char *name;
    split_kernel_t f;
};

/*
 * The kernel a batch of n records runs on (launch_batch, ptls_mi355x_kernel_name):
 *  - framing (section 4) batches of at most g_window_records and AEAD batches of at most g_aead_window_records
 *    go to the window kernels: up to one record per CU the 32-position single-record kernels (win32), up to
 *    15 records per CU the 3-record latency groups (win), above that the persistent 15-record groups (winw);
 *  - larger batches go to the batch kernels (K lanes per record; framing always K = 4).
 */
static LaunchPlan plan_launch(bool seal, bool frame, uint32_t key_size, size_t n, int num_cu)
{
    LaunchPlan p;
    const int a256 = key_size == 32 ? 1 : 0, s = seal ? 1 : 0, f = frame ? 1 : 0;
    if (n <= (frame ? g_window_records.load() : g_aead_window_records.load())) {
        static const WinEntry table[2][2][2][2] = {
            /* [frame][wide][seal][aes256] */
            {{{KN(mi355x_gcm_win_open_aes128), KN(mi355x_gcm_win_open_aes256)},
              {KN(mi355x_gcm_win_seal_aes128), KN(mi355x_gcm_win_seal_aes256)}},
             {{KN(mi355x_gcm_winw_open_aes128), KN(mi355x_gcm_winw_open_aes256)},
              {KN(mi355x_gcm_winw_seal_aes128), KN(mi355x_gcm_winw_seal_aes256)}}},
            {{{KN(mi355x_tls_win_open_aes128), KN(mi355x_tls_win_open_aes256)},
              {KN(mi355x_tls_win_seal_aes128), KN(mi355x_tls_win_seal_aes256)}},
             {{KN(mi355x_tls_winw_open_aes128), KN(mi355x_tls_winw_open_aes256)},
              {KN(mi355x_tls_winw_seal_aes128), KN(mi355x_tls_winw_seal_aes256)}}}};
        static const WinEntry table32[2][2][2] = {
            /* [frame][seal][aes256]: 32-position segments, one record per group */
            {{KN(mi355x_gcm_win32_open_aes128), KN(mi355x_gcm_win32_open_aes256)},
             {KN(mi355x_gcm_win32_seal_aes128), KN(mi355x_gcm_win32_seal_aes256)}},
            {{KN(mi355x_tls_win32_open_aes128), KN(mi355x_tls_win32_open_aes256)},
             {KN(mi355x_tls_win32_seal_aes128), KN(mi355x_tls_win32_seal_aes256)}}};
        static const WinEntry table16[2][2][2] = {
            /* [frame][seal][aes256]: 32-position segments, 16 lanes each, one record per group */
            {{KN(mi355x_gcm_win16_open_aes128), KN(mi355x_gcm_win16_open_aes256)},
             {KN(mi355x_gcm_win16_seal_aes128), KN(mi355x_gcm_win16_seal_aes256)}},
            {{KN(mi355x_tls_win16_open_aes128), KN(mi355x_tls_win16_open_aes256)},
             {KN(mi355x_tls_win16_seal_aes128), KN(mi355x_tls_win16_seal_aes256)}}};
        static const SplitEntry table_split[2][2][2] = {
            /* [frame][seal][aes256]: runs of SPLIT_RUNSEG segments, SPLIT_MAXRUN workgroups per record */
            {{KN(mi355x_gcm_wins_open_aes128), KN(mi355x_gcm_wins_open_aes256)},
             {KN(mi355x_gcm_wins_seal_aes128), KN(mi355x_gcm_wins_seal_aes256)}},
            {{KN(mi355x_tls_wins_open_aes128), KN(mi355x_tls_wins_open_aes256)},
             {KN(mi355x_tls_wins_seal_aes128), KN(mi355x_tls_wins_seal_aes256)}}};
        const size_t split_max = g_split_records.load(), win16_max = g_win16_records.load(),
                     seg32_max = g_seg32_records.load();
        if (n <= (split_max == SIZE_MAX ? (size_t)num_cu / SPLIT_MAXRUN : split_max) &&
            n <= 0xffffffffu / SPLIT_MAXRUN) {
            const SplitEntry &e = table_split[f][s][a256];
            p.name = e.name;
            p.split = e.f;
            p.threads = SPLIT_THREADS;
            p.blocks = (uint32_t)(n * SPLIT_MAXRUN);
            return p;
        }
        const bool wide = n > 15u * (uint64_t)num_cu; /* the wide groups (15 records) fill every CU */
        constexpr uint32_t per32 = (MI355X_WIN32_THREADS / 8u) / WIN_SEG32_MAXSEG; /* records per 32-position group */
        const bool win16 = !wide && n <= (win16_max == SIZE_MAX ? (size_t)num_cu : win16_max);
        const bool seg32 = !win16 && !wide && n <= (seg32_max == SIZE_MAX ? (size_t)per32 * num_cu : seg32_max);
        const WinEntry &e = win16 ? table16[f][s][a256] : seg32 ? table32[f][s][a256] : table[f][wide][s][a256];
        p.name = e.name;
        p.win = e.f;
        p.threads = win16 ? 576u : seg32 ? (uint32_t)MI355X_WIN32_THREADS : wide ? 1024u : 512u;
        const uint32_t per = win16 ? 1u : seg32 ? per32 : (p.threads / (wide ? 4u : 8u)) / WIN_MAXSEG;
        uint64_t blocks = (n + per - 1) / per;
        if (wide && blocks > (uint64_t)num_cu)
            blocks = (uint64_t)num_cu;
        p.blocks = (uint32_t)blocks;
        return p;
    }
    static const BatchEntry gcm[2][2][4] = {
        /* [seal][aes256][log2 K] */
        {{KN(mi355x_gcm_open_aes128_k1), KN(mi355x_gcm_open_aes128_k2), KN(mi355x_gcm_open_aes128_k4),
          KN(mi355x_gcm_open_aes128_k8)},
         {KN(mi355x_gcm_open_aes256_k1), KN(mi355x_gcm_open_aes256_k2), KN(mi355x_gcm_open_aes256_k4),
          KN(mi355x_gcm_open_aes256_k8)}},
        {{KN(mi355x_gcm_seal_aes128_k1), KN(mi355x_gcm_seal_aes128_k2), KN(mi355x_gcm_seal_aes128_k4),
          KN(mi355x_gcm_seal_aes128_k8)},
         {KN(mi355x_gcm_seal_aes256_k1), KN(mi355x_gcm_seal_aes256_k2), KN(mi355x_gcm_seal_aes256_k4),
          KN(mi355x_gcm_seal_aes256_k8)}}};
    static const BatchEntry tls[2][2] = {/* [seal][aes256] */
                                         {KN(mi355x_tls_open_aes128_k4), KN(mi355x_tls_open_aes256_k4)},
                                         {KN(mi355x_tls_seal_aes128_k4), KN(mi355x_tls_seal_aes256_k4)}};
    const int k = frame ? 4 : g_lanes.load();
    const int lk = k == 1 ? 0 : k == 2 ? 1 : k == 4 ? 2 : 3;
    const BatchEntry &e = frame ? tls[s][a256] : gcm[s][a256][lk];
    p.name = e.name;
    p.batch = e.f;
    p.k = (uint32_t)k;
    p.threads = WG_THREADS;
    const uint64_t ngroups = (n + (64 / k) - 1) / (64 / k), waves = WG_THREADS / 64;
    uint64_t blocks = (ngroups + waves - 1) / waves;
    if (blocks > (uint64_t)num_cu)
        blocks = (uint64_t)num_cu;
    p.blocks = (uint32_t)blocks;
    return p;
}
#undef KN

static inline uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

/*
 * Records the split buffer (partials + tickets, 84 B a record) holds when it must hold n: at least 4096 (344 KiB), else
 * the next power of two.  Growing it frees the old buffer, which synchronises the whole device -- a coalescing record
 * layer whose groups grow mid-stream (1, 2, 4 ... windows a launch) stalled ~8 ms at every growth.
 */
static size_t split_cap_for(size_t n)
{
    size_t cap = 4096;
    while (cap < n)
        cap *= 2;
    return cap;
}

/* a launch of ctx on `stream` is about to use shared resources (see the context's stream-ordering note) */
static int ctx_stream(ptls_mi355x_aesgcm_context_t *ctx, hipStream_t stream)
{
    if (!ctx->home_set) {
        ctx->home = stream;
        ctx->home_set = true;
    } else if (!ctx->multi && stream != ctx->home) {
        HIPCHK(hipDeviceSynchronize()); /* once: every launch queued so far, on any stream, is done */
        ctx->multi = true;
    }
    return 0;
}

/* multi-stream mode: `stream` waits for the resource's last use (if one was recorded) */
static int res_wait(ptls_mi355x_aesgcm_context_t *ctx, hipEvent_t ev, bool valid, hipStream_t stream)
{
    if (ctx->multi && valid)
        HIPCHK(hipStreamWaitEvent(stream, ev, 0));
    return 0;
}

/* multi-stream mode: the use just queued on `stream` is the resource's last (its event recorded there, now) */
static int res_used(ptls_mi355x_aesgcm_context_t *ctx, hipEvent_t *ev, bool *valid, hipStream_t stream)
{
    if (!ctx->multi)
        return 0;
    if (*ev == nullptr)
        HIPCHK(hipEventCreateWithFlags(ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(*ev, stream));
    *valid = true;
    return 0;
}

/* the journal entry of a record launch (fault_journal.c): every pointer argument, with its extent where it is known */
static void journal_records_launch(const char *kernel, hipStream_t stream, uint32_t blocks, uint32_t threads, size_t n,
                                   const void *ki, const void *recs, bool frame, const uint32_t *order, const uint8_t *src,
                                   const uint8_t *dst, const uint8_t *aad, const uint32_t *status, const uint8_t *types,
                                   const uint32_t *conn, const void *extra, size_t extra_len)
{
    const ptls_mi355x_journal_arg_t a[8] = {
        {"keyimg", ki, sizeof(KeyImage)},
        {"descs", recs, (uint64_t)n * (frame ? sizeof(TlsRecord) : sizeof(Record))},
        {"src", src, 0},
        {"dst", dst, 0},
        {"aad", aad, 0},
        {"status", status, status ? (uint64_t)n * 4u : 0u},
        {order ? "order" : conn ? "conn" : "types", order ? (const void *)order : conn ? (const void *)conn : types,
         (uint64_t)n * (order || conn ? 4u : 1u)},
        {"work", extra, extra_len}};
    ptls_mi355x_journal_launch(kernel, stream, blocks, threads, n, a, 8);
}

/* the split kernels' partials and tickets for n records, for a launch on `stream` (ordered after the last split launch) */
static int ensure_split(ptls_mi355x_aesgcm_context_t *ctx, size_t n, hipStream_t stream, uint32_t **tickets)
{
    if (ctx_stream(ctx, stream) != 0)
        return -1;
    if (ctx->split_cap < n) {
        if (ctx->d_split) {
            /* split launches of this context may be on any stream: the device is idle before the buffer goes
             * (an explicit wait, not hipFree's implicit one) */
            HIPCHK(hipDeviceSynchronize());
            JNOTE("hipFree split buffer", ctx->d_split, ctx->split_cap * (SPLIT_PSLOTS * sizeof(u32x4) + sizeof(uint32_t)));
            HIPCHK(hipFree(ctx->d_split));
        }
        ctx->d_split = nullptr;
        ctx->split_cap = 0;
        ctx->split_ev_valid = false;
        const size_t cap = split_cap_for(n);
        HIPCHK(hipMalloc(&ctx->d_split, cap * (SPLIT_PSLOTS * sizeof(u32x4) + sizeof(uint32_t))));
        JNOTE("hipMalloc split buffer", ctx->d_split, cap * (SPLIT_PSLOTS * sizeof(u32x4) + sizeof(uint32_t)));
        HIPCHK(hipMemsetAsync((uint8_t *)ctx->d_split + cap * SPLIT_PSLOTS * sizeof(u32x4), 0, cap * sizeof(uint32_t),
                              stream));
        ctx->split_cap = cap;
    }
    /* the tickets are shared: order after the previous split launch */
    if (res_wait(ctx, ctx->split_ev, ctx->split_ev_valid, stream) != 0)
        return -1;
    *tickets = (uint32_t *)((uint8_t *)ctx->d_split + ctx->split_cap * SPLIT_PSLOTS * sizeof(u32x4));
    return 0;
}

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
    const LaunchPlan p = plan_launch(seal, frame, ctx->key_size, n, ctx->num_cu);
    const uint8_t *iv = (const uint8_t *)static_iv12;
    DeviceGuard guard(ctx->device);
    if (p.split != nullptr) {
        /* partials and tickets for n records (tickets are zero between launches: each record's last run resets its) */
        uint32_t *tickets = nullptr;
        if (ensure_split(ctx, n, stream, &tickets) != 0)
            return -1;
        journal_records_launch(p.name, stream, p.blocks, p.threads, n, ctx->d_ki, recs, frame, order, src, dst, aad, status,
                               types, conn, ctx->d_split, ctx->split_cap * (SPLIT_PSLOTS * sizeof(u32x4) + sizeof(uint32_t)));
        hipLaunchKernelGGL(p.split, dim3(p.blocks), dim3(p.threads), 0, stream, ctx->d_ki, le32(iv), le32(iv + 4),
                           le32(iv + 8), recs, (uint32_t)n, src, dst, aad, status, types, conn,
                           (const u32x4 *)ctx->shared->d_win_aes, ctx->d_split, tickets);
        HIPCHK(hipGetLastError());
        return res_used(ctx, &ctx->split_ev, &ctx->split_ev_valid, stream);
    }
    if (p.win != nullptr) {
        journal_records_launch(p.name, stream, p.blocks, p.threads, n, ctx->d_ki, recs, frame, order, src, dst, aad, status,
                               types, conn, ctx->shared->d_win_aes, 0x10000);
        hipLaunchKernelGGL(p.win, dim3(p.blocks), dim3(p.threads), 0, stream, ctx->d_ki, le32(iv), le32(iv + 4),
                           le32(iv + 8), recs, (uint32_t)n, src, dst, aad, status, types, conn,
                           (const u32x4 *)ctx->shared->d_win_aes);
        HIPCHK(hipGetLastError());
        return 0;
    }
    /*
     * Work counters are never reset: every wave takes tickets until one is out of range, so a launch consumes
     * exactly ngroups + (its waves) tickets, and the next launch on the slot starts there.  A slot is reused
     * every WORK_SLOTS launches; in multi-stream mode the new launch first waits on the slot's event, recorded
     * right after its previous launch, so two launches never share a counter at once.  The slot's base is
     * committed only once the launch has been accepted.
     */
    const uint32_t k = p.k; /* the plan's: a concurrent ptls_mi355x_set_lanes_per_record does not split the two */
    const uint32_t ngroups = (uint32_t)((n + (64 / k) - 1) / (64 / k));
    const uint32_t wslot = ctx->work_next % WORK_SLOTS;
    uint32_t *work = ctx->d_work + wslot;
    const uint32_t work_base = ctx->work_base[wslot];
    if (ctx_stream(ctx, stream) != 0 || res_wait(ctx, ctx->work_ev[wslot], ctx->work_ev_valid[wslot], stream) != 0)
        return -1;
    journal_records_launch(p.name, stream, p.blocks, p.threads, n, ctx->d_ki, recs, frame, order, src, dst, aad, status,
                           types, conn, work, 4);
    hipLaunchKernelGGL(p.batch, dim3(p.blocks), dim3(p.threads), 0, stream, ctx->d_ki, le32(iv), le32(iv + 4),
                       le32(iv + 8), recs, order, (uint32_t)n, src, dst, aad, status, types, work, work_base, conn);
    HIPCHK(hipGetLastError());
    ctx->work_base[wslot] = work_base + ngroups + p.blocks * (uint32_t)(WG_THREADS / 64);
    ++ctx->work_next;
    return res_used(ctx, &ctx->work_ev[wslot], &ctx->work_ev_valid[wslot], stream);
}

static inline size_t up16(size_t x) { return (x + 15) & ~(size_t)15; }

/*
 * The workspace of order_by_length and the stop-at-failure scan, for a use on `stream`.  Launches of one context may
 * go to any streams, and they share this buffer: in multi-stream mode a use first waits on the event recorded right
 * after the previous use (scratch_done), as the split tickets and the work slots do.  Growing it waits for the last
 * use before the old buffer is freed.
 */
static int ensure_scratch(ptls_mi355x_aesgcm_context_t *ctx, size_t need, hipStream_t stream)
{
    if (ctx_stream(ctx, stream) != 0 || res_wait(ctx, ctx->scratch_ev, ctx->scratch_ev_valid, stream) != 0)
        return -1;
    if (need <= ctx->scratch_cap)
        return 0;
    if (ctx->d_scratch) {
        HIPCHK(hipStreamSynchronize(stream)); /* the last use (ordered before this stream's queue above) is done */
        JNOTE("hipFree scratch", ctx->d_scratch, ctx->scratch_cap);
        HIPCHK(hipFree(ctx->d_scratch));
    }
    ctx->d_scratch = nullptr;
    need = need < 2 * ctx->scratch_cap ? 2 * ctx->scratch_cap : need; /* (doubling: few growths, each a sync) */
    ctx->scratch_cap = 0;
    HIPCHK(hipMalloc(&ctx->d_scratch, need));
    JNOTE("hipMalloc scratch", ctx->d_scratch, need);
    ctx->scratch_cap = need;
    return 0;
}

/* the scratch use just queued on `stream` (after ensure_scratch and its launches) */
static int scratch_done(ptls_mi355x_aesgcm_context_t *ctx, hipStream_t stream)
{
    return res_used(ctx, &ctx->scratch_ev, &ctx->scratch_ev_valid, stream);
}

extern "C" {

const char *ptls_mi355x_last_error(void) { return g_err; }

int ptls_mi355x_is_supported(void)
{
    int n = 0, dev = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || hipGetDevice(&dev) != hipSuccess)
        return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess)
        return 0;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

int ptls_mi355x_set_lanes_per_record(int k)
{
    if (k != 1 && k != 2 && k != 4 && k != 8)
        return -1;
    return g_lanes.exchange(k);
}

int ptls_mi355x_get_lanes_per_record(void) { return g_lanes; }

size_t ptls_mi355x_set_tls_window_records(size_t n)
{
    return g_window_records.exchange(n);
}

size_t ptls_mi355x_set_aead_window_records(size_t n)
{
    return g_aead_window_records.exchange(n);
}

size_t ptls_mi355x_set_split_records(size_t n)
{
    return g_split_records.exchange(n);
}

size_t ptls_mi355x_set_win16_records(size_t n)
{
    return g_win16_records.exchange(n);
}

size_t ptls_mi355x_set_seg32_records(size_t n)
{
    return g_seg32_records.exchange(n);
}

uint32_t ptls_mi355x_set_work_ticket_origin(uint32_t origin)
{
    return g_ticket_origin.exchange(origin);
}

size_t ptls_mi355x_set_slot_zero_copy_bytes(size_t n)
{
    return g_slot_zero_copy_bytes.exchange(n);
}

int ptls_mi355x_batch_ghash_reads(int k)
{
    switch (k) {
    case 1: return Layout<1>::gh8 ? 16 : 32;
    case 2: return Layout<2>::gh8 ? 16 : 32;
    case 4: return Layout<4>::gh8 ? 16 : 32;
    case 8: return Layout<8>::gh8 ? 16 : 32;
    default: return -1;
    }
}

const char *ptls_mi355x_kernel_name(int is_seal, size_t key_size, size_t n, int framing)
{
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        ncu = 256;
    return plan_launch(is_seal != 0, framing != 0, key_size == 32 ? 32u : 16u, n, ncu).name;
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
    int rc = -1;
    hipDeviceProp_t prop;
    DeviceShared *d = nullptr;
    g_err[0] = 0;
    if (hipGetDevice(&ctx->device) != hipSuccess || hipGetDeviceProperties(&prop, ctx->device) != hipSuccess ||
        (d = device_shared(ctx->device)) == nullptr)
        goto Fail;
    ctx->shared = d;
    ctx->num_cu = prop.multiProcessorCount;
    if (hipMalloc(&ctx->d_ki, sizeof(KeyImage)) != hipSuccess ||
        hipMalloc(&ctx->d_work, WORK_SLOTS * sizeof(uint32_t)) != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "context allocation: %s", hipGetErrorString(hipGetLastError()));
        goto Fail;
    }
    JNOTE("hipMalloc key image", ctx->d_ki, sizeof(KeyImage));
    JNOTE("hipMalloc work counters", ctx->d_work, WORK_SLOTS * sizeof(uint32_t));
    ctx->work_base[0] = g_ticket_origin; /* (read once: the counters below start where the bases say) */
    for (uint32_t i = 1; i < WORK_SLOTS; ++i)
        ctx->work_base[i] = ctx->work_base[0];
    {
        /* the key goes through the shared pinned staging (zero-copy read by the setup kernel), cleared after */
        std::lock_guard<std::mutex> lk(d->mu);
        if (ensure_stage(d, 64 + 16) != 0)
            goto Fail;
        memcpy(d->h_stage, key, key_size);
        *(volatile int *)(d->h_stage + 64) = -2;
        if (hipMemsetD32Async((hipDeviceptr_t)ctx->d_work, (int)ctx->work_base[0], WORK_SLOTS, d->stream) != hipSuccess) {
            snprintf(g_err, sizeof(g_err), "work counters: %s", hipGetErrorString(hipGetLastError()));
            goto Fail;
        }
        (void)hipGetLastError(); /* a stale error of an unrelated earlier call is not this launch's */
        hipLaunchKernelGGL(mi355x_gcm_setup, dim3(1), dim3(1024), 0, d->stream, d->h_stage_dev, (uint32_t)key_size,
                           ctx->d_ki, (int *)(d->h_stage_dev + 64));
        const hipError_t e1 = hipGetLastError(), e2 = hipStreamSynchronize(d->stream);
        memset(d->h_stage, 0, key_size);
        rc = *(volatile int *)(d->h_stage + 64);
        if (e1 != hipSuccess || e2 != hipSuccess || rc != 0) {
            snprintf(g_err, sizeof(g_err), "key setup kernel: launch %s, synchronize %s, status %d",
                     hipGetErrorString(e1), hipGetErrorString(e2), rc);
            goto Fail;
        }
    }
    return ctx;
Fail:
    if (g_err[0] == 0)
        snprintf(g_err, sizeof(g_err), "context setup failed: %s", hipGetErrorString(hipGetLastError()));
    ptls_mi355x_aesgcm_free(ctx);
    return nullptr;
}

/* release (the caller gets the first error) or free (nothing to return it to: every error deferred, see defer) */
static int context_release(ptls_mi355x_aesgcm_context_t *ctx, bool deferred)
{
    if (ctx == nullptr)
        return 0;
    DeviceGuard guard(ctx->device);
    int rc = 0;
    auto chk = [&](const char *what, hipError_t e) {
        if (e == hipSuccess)
            return;
        if (deferred)
            defer(what, e);
        else if (rc == 0)
            rc = fail(what, e);
        else /* a later error of the same release: printed (the first one is returned) */
            fprintf(stderr, "ptls_mi355x: %s: %s\n", what, hipGetErrorString(e));
    };
    /* launches on caller streams may still read the key image; a fault of any earlier work surfaces here */
    chk("context free: hipDeviceSynchronize", hipDeviceSynchronize());
    if (ctx->d_ki) {
        /* clear key material, as ptls_fusion_aesgcm_free does; ordered before the free on the null stream */
        chk("context free: clearing the key image", hipMemsetAsync(ctx->d_ki, 0, sizeof(KeyImage), nullptr));
        chk("context free: hipDeviceSynchronize", hipDeviceSynchronize());
        JNOTE("hipFree key image", ctx->d_ki, sizeof(KeyImage));
        chk("context free: hipFree(key image)", hipFree(ctx->d_ki));
    }
    if (ctx->d_work) {
        JNOTE("hipFree work counters", ctx->d_work, WORK_SLOTS * sizeof(uint32_t));
        chk("context free: hipFree(work counters)", hipFree(ctx->d_work));
    }
    if (ctx->d_scratch) {
        JNOTE("hipFree scratch", ctx->d_scratch, ctx->scratch_cap);
        chk("context free: hipFree(scratch)", hipFree(ctx->d_scratch));
    }
    if (ctx->d_split) {
        JNOTE("hipFree split buffer", ctx->d_split, ctx->split_cap * (SPLIT_PSLOTS * sizeof(u32x4) + sizeof(uint32_t)));
        chk("context free: hipFree(split buffer)", hipFree(ctx->d_split));
    }
    for (uint32_t i = 0; i < WORK_SLOTS; ++i)
        if (ctx->work_ev[i])
            chk("context free: hipEventDestroy", hipEventDestroy(ctx->work_ev[i]));
    if (ctx->split_ev)
        chk("context free: hipEventDestroy", hipEventDestroy(ctx->split_ev));
    if (ctx->scratch_ev)
        chk("context free: hipEventDestroy", hipEventDestroy(ctx->scratch_ev));
    if (ctx->mk_ev)
        chk("context free: hipEventDestroy", hipEventDestroy(ctx->mk_ev));
    if (ctx->mk_host)
        chk("context free: hipHostFree(key table)", hipHostFree(ctx->mk_host));
    free(ctx);
    return rc;
}

int ptls_mi355x_aesgcm_release(ptls_mi355x_aesgcm_context_t *ctx) { return context_release(ctx, false); }

void ptls_mi355x_aesgcm_free(ptls_mi355x_aesgcm_context_t *ctx) { (void)context_release(ctx, true); }

ptls_mi355x_aesgcm_context_t *ptls_mi355x_aesgcm_new_on(int device, const void *key, size_t key_size, size_t capacity)
{
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || device < 0 || device >= n) {
        if (e != hipSuccess)
            (void)hipGetLastError();
        snprintf(g_err, sizeof(g_err), "device ordinal %d is not present (%d HIP device%s%s%s)", device,
                 e == hipSuccess ? n : 0, (e == hipSuccess ? n : 0) == 1 ? "" : "s", e == hipSuccess ? "" : ": ",
                 e == hipSuccess ? "" : hipGetErrorString(e));
        return nullptr;
    }
    DeviceGuard guard(device);
    if (!guard.ok) {
        snprintf(g_err, sizeof(g_err), "device ordinal %d could not be made current", device);
        return nullptr;
    }
    return ptls_mi355x_aesgcm_new(key, key_size, capacity);
}

int ptls_mi355x_device_check(void)
{
    /*
     * The current device's deferred error comes first, read and cleared before any HIP call: a sticky fault makes
     * every call fail, and an error a free path met earlier must be reported by this check, not left queued for a
     * later one.  (A fault with no deferred error is then named by the first HIP call below.)
     */
    int dev = 0;
    const hipError_t g = hipGetDevice(&dev);
    if (g != hipSuccess || dev < 0 || dev >= MAX_DEVICES)
        dev = 0;
    char deferred[256];
    {
        std::lock_guard<std::mutex> lk(g_deferred_mu);
        snprintf(deferred, sizeof(deferred), "%s", g_deferred[dev]);
        g_deferred[dev][0] = 0;
    }
    if (g != hipSuccess) {
        JNOTE("device check: hipGetDevice failed", nullptr, 0);
        if (deferred[0] != 0)
            snprintf(g_err, sizeof(g_err), "%s (then hipGetDevice: %s)", deferred, hipGetErrorString(g));
        else
            fail("hipGetDevice(&dev)", g);
        return -1;
    }
    const hipError_t s = hipDeviceSynchronize();
    const hipError_t l = hipGetLastError();
    JNOTE(s == hipSuccess && l == hipSuccess && deferred[0] == 0 ? "device check: ok" : "device check: error", nullptr, 0);
    if (deferred[0] != 0) {
        snprintf(g_err, sizeof(g_err), "%s", deferred);
        return -1;
    }
    if (s != hipSuccess)
        return fail("hipDeviceSynchronize", s);
    if (l != hipSuccess)
        return fail("pending HIP error", l);
    return 0;
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
    return ptls_mi355x_tls_open_records_ex(ctx, static_iv12, recs, nullptr, n, src, dst, status, types, 0, stream);
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
    return ptls_mi355x_tls_open_records_ex(ctx, static_iv12, recs, conn_ids, n, src, dst, status, types, 0, stream);
}

int ptls_mi355x_tls_open_records_ex(ptls_mi355x_aesgcm_context_t *ctx, const void *static_iv12,
                                    const ptls_mi355x_tls_record_t *recs, const uint32_t *conn_ids, size_t n,
                                    const uint8_t *src, uint8_t *dst, uint32_t *status, uint8_t *types, int flags,
                                    void *stream_)
{
    if (n != 0 && (status == nullptr || types == nullptr)) {
        snprintf(g_err, sizeof(g_err), "tls_open_records needs status and types");
        return -1;
    }
    if ((flags & ~PTLS_MI355X_OPEN_STOP_AT_FAILURE) != 0) {
        snprintf(g_err, sizeof(g_err), "unknown flags %#x", flags);
        return -1;
    }
    hipStream_t stream = (hipStream_t)stream_;
    if (launch_batch(ctx, false, static_iv12, recs, nullptr, n, src, dst, nullptr, status, stream, true, types,
                     conn_ids) != 0)
        return -1;
    if (n == 0 || !(flags & PTLS_MI355X_OPEN_STOP_AT_FAILURE))
        return 0;
    DeviceGuard guard(ctx->device);
    size_t temp = 0;
    rocprim::constant_iterator<uint32_t> one_conn(0u);
    if (conn_ids != nullptr)
        HIPCHK(hipcub::DeviceScan::InclusiveScanByKey(nullptr, temp, conn_ids, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                      hipcub::Min(), (uint32_t)n, hipcub::Equality(), stream));
    else
        HIPCHK(hipcub::DeviceScan::InclusiveScanByKey(nullptr, temp, one_conn, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                                      hipcub::Min(), (uint32_t)n, hipcub::Equality(), stream));
    const size_t arr = ((n * sizeof(uint32_t)) + 255) & ~(size_t)255;
    if (ensure_scratch(ctx, 2 * arr + temp, stream) != 0)
        return -1;
    uint8_t *base = (uint8_t *)ctx->d_scratch;
    uint32_t *pos = (uint32_t *)base, *first = (uint32_t *)(base + arr);
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(mi355x_tls_fail_pos, dim3(g), dim3(256), 0, stream, status, (uint32_t)n, pos);
    HIPCHK(hipGetLastError());
    if (conn_ids != nullptr)
        HIPCHK(hipcub::DeviceScan::InclusiveScanByKey(base + 2 * arr, temp, conn_ids, pos, first, hipcub::Min(), (uint32_t)n,
                                                      hipcub::Equality(), stream));
    else
        HIPCHK(hipcub::DeviceScan::InclusiveScanByKey(base + 2 * arr, temp, one_conn, pos, first, hipcub::Min(), (uint32_t)n,
                                                      hipcub::Equality(), stream));
    hipLaunchKernelGGL(mi355x_tls_truncate, dim3(g), dim3(256), 0, stream, (const TlsRecord *)recs, (uint32_t)n, first,
                       dst, status, types);
    HIPCHK(hipGetLastError());
    return scratch_done(ctx, stream);
}

int ptls_mi355x_tls_deliver_records(ptls_mi355x_aesgcm_context_t *ctx, const ptls_mi355x_tls_record_t *recs,
                                    const uint32_t *status, const uint8_t *types, const ptls_mi355x_tls_deliver_t *parts,
                                    size_t nparts, size_t max_records, void *stream_)
{
    if (nparts == 0)
        return 0;
    if (max_records > DELIVER_MAX || nparts > 65535) {
        snprintf(g_err, sizeof(g_err), "deliver: more than %u records in a part, or too many parts", DELIVER_MAX);
        return -1;
    }
    DeviceGuard guard(ctx->device);
    unsigned groups = (unsigned)(max_records < 64 ? (max_records ? max_records : 1) : 64); /* a record per group */
    hipLaunchKernelGGL(mi355x_tls_deliver, dim3((unsigned)nparts, groups), dim3(256), 0, (hipStream_t)stream_,
                       (const TlsRecord *)recs, status, types, (const DeliverPart *)parts);
    HIPCHK(hipGetLastError());
    return 0;
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
    if (ensure_scratch(ctx, 3 * arr + temp, stream) != 0)
        return -1;
    uint8_t *base = (uint8_t *)ctx->d_scratch;
    uint32_t *keys_in = (uint32_t *)base, *keys_out = (uint32_t *)(base + arr), *vals_in = (uint32_t *)(base + 2 * arr);
    hipLaunchKernelGGL(mi355x_sort_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, (const Record *)recs,
                       (uint32_t)n, keys_in, vals_in);
    HIPCHK(hipGetLastError());
    HIPCHK(hipcub::DeviceRadixSort::SortPairsDescending(base + 3 * arr, temp, keys_in, keys_out, vals_in, order, (int)n, 0,
                                                        24, stream));
    return scratch_done(ctx, stream);
}

/* ------------------------------------------------------------------ multi-key batches ----- */

/*
 * The key table of a multi-key launch led by ctx, in its scratch at `dev`: uploaded from a pinned host copy only when
 * the keys, their IVs or the table's place changed (a caller that sends its sessions' batches again pays nothing).
 */
static int mk_upload(ptls_mi355x_aesgcm_context_t *ctx, ptls_mi355x_aesgcm_context_t *const *ctxs, const uint8_t *ivs,
                     size_t nkeys, void *dev, hipStream_t stream)
{
    bool same = ctx->mk_dev == dev && ctx->mk_n == nkeys && ctx->mk_host != nullptr;
    for (size_t k = 0; same && k < nkeys; ++k)
        same = ctx->mk_host[k].ki == ctxs[k]->d_ki && ctx->mk_host[k].iv0 == le32(ivs + 12 * k) &&
               ctx->mk_host[k].iv1 == le32(ivs + 12 * k + 4) && ctx->mk_host[k].iv2 == le32(ivs + 12 * k + 8);
    if (same)
        return 0;
    if (ctx->mk_ev_valid) /* the previous upload has read the pinned copy */
        HIPCHK(hipEventSynchronize(ctx->mk_ev));
    if (ctx->mk_cap < nkeys) {
        if (ctx->mk_host)
            HIPCHK(hipHostFree(ctx->mk_host));
        ctx->mk_host = nullptr;
        ctx->mk_cap = 0;
        HIPCHK(hipHostMalloc((void **)&ctx->mk_host, nkeys * sizeof(MkKey), hipHostMallocDefault));
        ctx->mk_cap = nkeys;
    }
    for (size_t k = 0; k < nkeys; ++k)
        ctx->mk_host[k] = MkKey{ctxs[k]->d_ki, le32(ivs + 12 * k), le32(ivs + 12 * k + 4), le32(ivs + 12 * k + 8), 0u, 0u, 0u};
    ctx->mk_n = 0;
    ctx->mk_dev = nullptr;
    HIPCHK(hipMemcpyAsync(dev, ctx->mk_host, nkeys * sizeof(MkKey), hipMemcpyHostToDevice, stream));
    if (ctx->mk_ev == nullptr)
        HIPCHK(hipEventCreateWithFlags(&ctx->mk_ev, hipEventDisableTiming));
    HIPCHK(hipEventRecord(ctx->mk_ev, stream));
    ctx->mk_ev_valid = true;
    ctx->mk_n = nkeys;
    ctx->mk_dev = dev;
    return 0;
}

/*
 * The records grouped by key into `order` on `stream` (mi355x_mk_count / _scatter; hipcub's radix sort above
 * MK_LDS_BUCKETS - 1 keys), in the scratch `work` of mk_group_bytes(n, nkeys) bytes.
 */
static size_t mk_group_bytes(size_t n, size_t nkeys)
{
    const size_t arr = (n * 4 + 255) & ~(size_t)255;
    if (nkeys + 1 <= MK_LDS_BUCKETS) { /* counts, cursors, the scan's workspace */
        size_t temp = 0;
        (void)hipcub::DeviceScan::ExclusiveSum(nullptr, temp, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)(nkeys + 1),
                                               (hipStream_t)0);
        return 2 * (((nkeys + 1) * 4 + 255) & ~(size_t)255) + temp;
    }
    uint32_t bits = 1;
    while (bits < 32 && (1ull << bits) <= nkeys)
        ++bits;
    size_t temp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                             (uint32_t *)nullptr, (int)n, 0, (int)bits, (hipStream_t)0);
    return 3 * arr + temp;
}

static int mk_group(const uint32_t *key_idx, size_t n, size_t nkeys, uint32_t *order, uint8_t *work, hipStream_t stream)
{
    if (nkeys + 1 <= MK_LDS_BUCKETS) {
        const size_t ab = ((nkeys + 1) * 4 + 255) & ~(size_t)255;
        uint32_t *counts = (uint32_t *)work, *cursor = (uint32_t *)(work + ab);
        size_t temp = 0; /* (the scan's workspace lives after the cursors: mk_group_bytes) */
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, temp, counts, cursor, (int)(nkeys + 1), stream));
        const unsigned blocks = (unsigned)((n + MK_PER_BLOCK - 1) / MK_PER_BLOCK);
        HIPCHK(hipMemsetAsync(counts, 0, (nkeys + 1) * 4, stream));
        hipLaunchKernelGGL(mi355x_mk_count, dim3(blocks), dim3(1024), 0, stream, key_idx, (uint32_t)n, (uint32_t)nkeys,
                           counts);
        HIPCHK(hipGetLastError());
        HIPCHK(hipcub::DeviceScan::ExclusiveSum(work + 2 * ab, temp, counts, cursor, (int)(nkeys + 1), stream));
        hipLaunchKernelGGL(mi355x_mk_scatter, dim3(blocks), dim3(1024), 0, stream, key_idx, (uint32_t)n, (uint32_t)nkeys,
                           cursor, order);
        HIPCHK(hipGetLastError());
        return 0;
    }
    const size_t arr = (n * 4 + 255) & ~(size_t)255;
    uint32_t bits = 1;
    while (bits < 32 && (1ull << bits) <= nkeys)
        ++bits;
    size_t temp = 0;
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                              (uint32_t *)nullptr, (int)n, 0, (int)bits, stream));
    uint32_t *keys_in = (uint32_t *)work, *keys_out = (uint32_t *)(work + arr), *vals_in = (uint32_t *)(work + 2 * arr);
    hipLaunchKernelGGL(mi355x_mk_keys, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, key_idx, (uint32_t)n,
                       (uint32_t)nkeys, keys_in, vals_in);
    HIPCHK(hipGetLastError());
    HIPCHK(hipcub::DeviceRadixSort::SortPairs(work + 3 * arr, temp, keys_in, keys_out, vals_in, order, (int)n, 0, (int)bits,
                                              stream));
    return 0;
}

/* bytes of a multi-key launch's scratch before its sort arrays: the key table, the group counters, the broadcast slots */
static size_t mk_prefix(size_t nkeys, int num_cu)
{
    return ((nkeys * sizeof(MkKey) + 255) & ~(size_t)255) + ((nkeys * 4 + 255) & ~(size_t)255) +
           (((size_t)num_cu * 4 + 255) & ~(size_t)255);
}

/* the kernel family of a multi-key batch of n records (the same selection setters as plan_launch) */
enum MkFamily { MK_SPLIT, MK_WIN16, MK_BATCH };
static MkFamily mk_family(bool frame, size_t n, int num_cu)
{
    if (n <= (frame ? g_window_records.load() : g_aead_window_records.load())) {
        const size_t split_max = g_split_records.load(), win16_max = g_win16_records.load();
        if (n <= (split_max == SIZE_MAX ? (size_t)num_cu / SPLIT_MAXRUN : split_max) && n <= 0xffffffffu / SPLIT_MAXRUN)
            return MK_SPLIT;
        if (n <= (win16_max == SIZE_MAX ? (size_t)num_cu : win16_max))
            return MK_WIN16;
    }
    return MK_BATCH;
}

static const char *mk_kernel_name(bool seal, bool frame, uint32_t key_size, size_t n, int num_cu)
{
    static const char *names[3][2][2][2] = {
        /* [family][frame][seal][aes256] */
        {{{"mi355x_gcm_wins_open_aes128_mk", "mi355x_gcm_wins_open_aes256_mk"},
          {"mi355x_gcm_wins_seal_aes128_mk", "mi355x_gcm_wins_seal_aes256_mk"}},
         {{"mi355x_tls_wins_open_aes128_mk", "mi355x_tls_wins_open_aes256_mk"},
          {"mi355x_tls_wins_seal_aes128_mk", "mi355x_tls_wins_seal_aes256_mk"}}},
        {{{"mi355x_gcm_win16_open_aes128_mk", "mi355x_gcm_win16_open_aes256_mk"},
          {"mi355x_gcm_win16_seal_aes128_mk", "mi355x_gcm_win16_seal_aes256_mk"}},
         {{"mi355x_tls_win16_open_aes128_mk", "mi355x_tls_win16_open_aes256_mk"},
          {"mi355x_tls_win16_seal_aes128_mk", "mi355x_tls_win16_seal_aes256_mk"}}},
        {{{"mi355x_gcm_open_aes128_k4_mk", "mi355x_gcm_open_aes256_k4_mk"},
          {"mi355x_gcm_seal_aes128_k4_mk", "mi355x_gcm_seal_aes256_k4_mk"}},
         {{"mi355x_tls_open_aes128_k4_mk", "mi355x_tls_open_aes256_k4_mk"},
          {"mi355x_tls_seal_aes128_k4_mk", "mi355x_tls_seal_aes256_k4_mk"}}}};
    return names[mk_family(frame, n, num_cu)][frame][seal][key_size == 32];
}

typedef void (*mk_batch_kernel_t)(const MkKey *, uint32_t, uint32_t *, uint32_t *, const void *, const uint32_t *, uint32_t,
                                  const uint8_t *, uint8_t *, const uint8_t *, uint32_t *, uint8_t *, const uint32_t *);
typedef void (*mk_split_kernel_t)(const MkKey *, uint32_t, const uint32_t *, const void *, uint32_t, const uint8_t *,
                                  uint8_t *, const uint8_t *, uint32_t *, uint8_t *, const uint32_t *, const u32x4 *, u32x4 *,
                                  uint32_t *);
typedef void (*mk_win16_kernel_t)(const MkKey *, uint32_t, const uint32_t *, const void *, uint32_t, const uint8_t *,
                                  uint8_t *, const uint8_t *, uint32_t *, uint8_t *, const uint32_t *, const u32x4 *);

/*
 * One launch over the records of nkeys keys (contexts ctxs[k], static IVs ivs[12 k ..]); record i uses key key_idx[i].
 * ctxs[0] leads: its scratch holds the key table, the counters and the sort, its split buffer the split kernels' state.
 *  - up to a fifth of the CUs' records: the split kernels, each workgroup on its record's key;
 *  - up to one record per CU: the 16-lane kernels, likewise;
 *  - above: the batch kernels' multi-key phases, over the records sorted by key (a stable device radix sort on the key
 *    index, then each key's range, both on `stream` before the launch).
 * Every key must be on ctxs[0]'s device with its key size.  A record whose key index is >= nkeys is not processed
 * (open: status 0xffffffff).
 */
static int launch_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys, bool seal,
                           bool frame, const void *recs, const uint32_t *key_idx, const uint32_t *conn, size_t n,
                           const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *status, uint8_t *types,
                           hipStream_t stream, const uint32_t *given_order = nullptr)
{
    if (n == 0)
        return 0;
    if (ctxs == nullptr || nkeys == 0 || nkeys > (1u << 24) || static_ivs == nullptr || key_idx == nullptr) {
        snprintf(g_err, sizeof(g_err), "multi-key batch: contexts, IVs and key indices are required (1..2^24 keys)");
        return -1;
    }
    if (n > 0xffffffffull) {
        snprintf(g_err, sizeof(g_err), "batch of %zu records exceeds 2^32-1", n);
        return -1;
    }
    ptls_mi355x_aesgcm_context_t *ctx = ctxs[0];
    for (size_t k = 0; k < nkeys; ++k)
        if (ctxs[k] == nullptr || ctxs[k]->device != ctx->device || ctxs[k]->key_size != ctx->key_size) {
            snprintf(g_err, sizeof(g_err), "multi-key batch: key %zu is %s", k,
                     ctxs[k] == nullptr ? "NULL" : "on another device or of another key size");
            return -1;
        }
    DeviceGuard guard(ctx->device);
    const bool a256 = ctx->key_size == 32;
    const MkFamily fam = mk_family(frame, n, ctx->num_cu);
    const uint32_t grid = (uint32_t)ctx->num_cu;
    /* scratch: key table | counters | broadcast slots (mk_prefix) | sort keys in, out | values in | order | sort temp */
    const size_t a_tab = (nkeys * sizeof(MkKey) + 255) & ~(size_t)255, a_ctr = (nkeys * 4 + 255) & ~(size_t)255,
                 a_wg = ((size_t)grid * 4 + 255) & ~(size_t)255,
                 arr = fam == MK_BATCH && given_order == nullptr ? (n * 4 + 255) & ~(size_t)255 : 0;
    const size_t gbytes = arr != 0 ? mk_group_bytes(n, nkeys) : 0;
    const size_t need = a_tab + a_ctr + a_wg + arr + gbytes;
    if (ensure_scratch(ctx, need, stream) != 0)
        return -1;
    uint8_t *base = (uint8_t *)ctx->d_scratch;
    MkKey *tab = (MkKey *)base;
    uint32_t *ctr = (uint32_t *)(base + a_tab), *wg = (uint32_t *)(base + a_tab + a_ctr);
    uint8_t *sb = base + a_tab + a_ctr + a_wg;
    uint32_t *order = (uint32_t *)sb; /* the records grouped by key, then the grouping's workspace */
    if (mk_upload(ctx, ctxs, (const uint8_t *)static_ivs, nkeys, tab, stream) != 0)
        return -1;
    const char *name = mk_kernel_name(seal, frame, ctx->key_size, n, ctx->num_cu);
    if (fam == MK_SPLIT) {
        static const mk_split_kernel_t ks[2][2][2] = {
            {{mi355x_gcm_wins_open_aes128_mk, mi355x_gcm_wins_open_aes256_mk},
             {mi355x_gcm_wins_seal_aes128_mk, mi355x_gcm_wins_seal_aes256_mk}},
            {{mi355x_tls_wins_open_aes128_mk, mi355x_tls_wins_open_aes256_mk},
             {mi355x_tls_wins_seal_aes128_mk, mi355x_tls_wins_seal_aes256_mk}}};
        uint32_t *tickets = nullptr;
        if (ensure_split(ctx, n, stream, &tickets) != 0)
            return -1;
        journal_records_launch(name, stream, (uint32_t)(n * SPLIT_MAXRUN), SPLIT_THREADS, n, tab, recs, frame, key_idx, src,
                               dst, aad, status, types, conn, ctx->d_split,
                               ctx->split_cap * (SPLIT_PSLOTS * sizeof(u32x4) + sizeof(uint32_t)));
        hipLaunchKernelGGL(ks[frame][seal][a256], dim3((uint32_t)(n * SPLIT_MAXRUN)), dim3(SPLIT_THREADS), 0, stream, tab,
                           (uint32_t)nkeys, key_idx, recs, (uint32_t)n, src, dst, aad, status, types, conn,
                           (const u32x4 *)ctx->shared->d_win_aes, ctx->d_split, tickets);
        HIPCHK(hipGetLastError());
        if (res_used(ctx, &ctx->split_ev, &ctx->split_ev_valid, stream) != 0)
            return -1;
        return scratch_done(ctx, stream);
    }
    if (fam == MK_WIN16) {
        static const mk_win16_kernel_t kw[2][2][2] = {
            {{mi355x_gcm_win16_open_aes128_mk, mi355x_gcm_win16_open_aes256_mk},
             {mi355x_gcm_win16_seal_aes128_mk, mi355x_gcm_win16_seal_aes256_mk}},
            {{mi355x_tls_win16_open_aes128_mk, mi355x_tls_win16_open_aes256_mk},
             {mi355x_tls_win16_seal_aes128_mk, mi355x_tls_win16_seal_aes256_mk}}};
        journal_records_launch(name, stream, (uint32_t)n, 576, n, tab, recs, frame, key_idx, src, dst, aad, status, types,
                               conn, ctx->shared->d_win_aes, 0x10000);
        hipLaunchKernelGGL(kw[frame][seal][a256], dim3((uint32_t)n), dim3(576), 0, stream, tab, (uint32_t)nkeys, key_idx,
                           recs, (uint32_t)n, src, dst, aad, status, types, conn, (const u32x4 *)ctx->shared->d_win_aes);
        HIPCHK(hipGetLastError());
        return scratch_done(ctx, stream);
    }
    static const mk_batch_kernel_t kb[2][2][2] = {
        {{mi355x_gcm_open_aes128_k4_mk, mi355x_gcm_open_aes256_k4_mk},
         {mi355x_gcm_seal_aes128_k4_mk, mi355x_gcm_seal_aes256_k4_mk}},
        {{mi355x_tls_open_aes128_k4_mk, mi355x_tls_open_aes256_k4_mk},
         {mi355x_tls_seal_aes128_k4_mk, mi355x_tls_seal_aes256_k4_mk}}};
    const unsigned g = (unsigned)((n + 255) / 256), gk = (unsigned)((nkeys + 255) / 256);
    if (given_order == nullptr) { /* the records grouped by key here */
        if (mk_group(key_idx, n, nkeys, order, sb + arr, stream) != 0)
            return -1;
    } else { /* the caller's order (ptls_mi355x_order_by_key), e.g. shared by a batch's seal and open */
        order = (uint32_t *)given_order;
    }
    if (nkeys + 1 <= MK_LDS_BUCKETS) { /* ranges and counters in one launch (mi355x_mk_bounds_all) */
        const size_t th = n > nkeys ? n : nkeys;
        hipLaunchKernelGGL(mi355x_mk_bounds_all, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, stream, key_idx, order,
                           (uint32_t)n, (uint32_t)nkeys, tab, ctr, seal ? nullptr : status, seal ? nullptr : types,
                           frame ? 1u : 0u);
        HIPCHK(hipGetLastError());
    } else {
        hipLaunchKernelGGL(mi355x_mk_reset, dim3(gk), dim3(256), 0, stream, tab, (uint32_t)nkeys, ctr);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(mi355x_mk_bounds, dim3(g), dim3(256), 0, stream, nullptr, key_idx, order, (uint32_t)n,
                           (uint32_t)nkeys, tab, seal ? nullptr : status, seal ? nullptr : types, frame ? 1u : 0u);
        HIPCHK(hipGetLastError());
    }
    /* groups: at most n / 16 + nkeys (each key's last group partial); a CU's worth of waves per workgroup */
    const uint64_t groups = n / 16 + nkeys, blocks = (groups + 15) / 16;
    const uint32_t nb = (uint32_t)(blocks < grid ? blocks : grid);
    journal_records_launch(name, stream, nb, WG_THREADS, n, tab, recs, frame, order, src, dst, aad, status, types, conn, ctr,
                           nkeys * 4);
    hipLaunchKernelGGL(kb[frame][seal][a256], dim3(nb), dim3(WG_THREADS), 0, stream, tab, (uint32_t)nkeys, ctr, wg, recs,
                       order, (uint32_t)n, src, dst, aad, status, types, conn);
    HIPCHK(hipGetLastError());
    return scratch_done(ctx, stream);
}

int ptls_mi355x_seal_batch_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys,
                                    const ptls_mi355x_record_t *recs, const uint32_t *key_idx, size_t n,
                                    const uint8_t *src, uint8_t *dst, const uint8_t *aad, void *stream)
{
    return launch_multikey(ctxs, static_ivs, nkeys, true, false, recs, key_idx, nullptr, n, src, dst, aad, nullptr, nullptr,
                           (hipStream_t)stream);
}

int ptls_mi355x_open_batch_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys,
                                    const ptls_mi355x_record_t *recs, const uint32_t *key_idx, size_t n,
                                    const uint8_t *src, uint8_t *dst, const uint8_t *aad, uint32_t *status, void *stream)
{
    if (n != 0 && status == nullptr) {
        snprintf(g_err, sizeof(g_err), "open_batch_multikey needs status");
        return -1;
    }
    return launch_multikey(ctxs, static_ivs, nkeys, false, false, recs, key_idx, nullptr, n, src, dst, aad, status, nullptr,
                           (hipStream_t)stream);
}

int ptls_mi355x_tls_seal_records_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys,
                                          const ptls_mi355x_tls_record_t *recs, const uint32_t *key_idx,
                                          const uint32_t *conn_ids, size_t n, const uint8_t *src, uint8_t *dst,
                                          void *stream)
{
    return launch_multikey(ctxs, static_ivs, nkeys, true, true, recs, key_idx, conn_ids, n, src, dst, nullptr, nullptr,
                           nullptr, (hipStream_t)stream);
}

int ptls_mi355x_tls_open_records_multikey(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs, size_t nkeys,
                                          const ptls_mi355x_tls_record_t *recs, const uint32_t *key_idx,
                                          const uint32_t *conn_ids, size_t n, const uint8_t *src, uint8_t *dst,
                                          uint32_t *status, uint8_t *types, int flags, void *stream_)
{
    if (n != 0 && (status == nullptr || types == nullptr)) {
        snprintf(g_err, sizeof(g_err), "tls_open_records_multikey needs status and types");
        return -1;
    }
    if ((flags & ~PTLS_MI355X_OPEN_STOP_AT_FAILURE) != 0) {
        snprintf(g_err, sizeof(g_err), "unknown flags %#x", flags);
        return -1;
    }
    hipStream_t stream = (hipStream_t)stream_;
    if (launch_multikey(ctxs, static_ivs, nkeys, false, true, recs, key_idx, conn_ids, n, src, dst, nullptr, status, types,
                        stream) != 0)
        return -1;
    if (n == 0 || !(flags & PTLS_MI355X_OPEN_STOP_AT_FAILURE))
        return 0;
    /* stop at each connection's first failure; a connection is (key, connection id): consecutive records of one */
    ptls_mi355x_aesgcm_context_t *ctx = ctxs[0];
    DeviceGuard guard(ctx->device);
    size_t temp = 0;
    HIPCHK(hipcub::DeviceScan::InclusiveScanByKey(nullptr, temp, (uint64_t *)nullptr, (uint32_t *)nullptr,
                                                  (uint32_t *)nullptr, hipcub::Min(), (uint32_t)n, hipcub::Equality(),
                                                  stream));
    const size_t arr = ((n * sizeof(uint32_t)) + 255) & ~(size_t)255, arr64 = ((n * sizeof(uint64_t)) + 255) & ~(size_t)255;
    if (ensure_scratch(ctx, 2 * arr + arr64 + temp, stream) != 0)
        return -1;
    uint8_t *base = (uint8_t *)ctx->d_scratch;
    uint32_t *pos = (uint32_t *)base, *first = (uint32_t *)(base + arr);
    uint64_t *seg = (uint64_t *)(base + 2 * arr);
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(mi355x_mk_segkeys, dim3(g), dim3(256), 0, stream, key_idx, conn_ids, (uint32_t)n, seg);
    HIPCHK(hipGetLastError());
    hipLaunchKernelGGL(mi355x_tls_fail_pos, dim3(g), dim3(256), 0, stream, status, (uint32_t)n, pos);
    HIPCHK(hipGetLastError());
    HIPCHK(hipcub::DeviceScan::InclusiveScanByKey(base + 2 * arr + arr64, temp, seg, pos, first, hipcub::Min(), (uint32_t)n,
                                                  hipcub::Equality(), stream));
    hipLaunchKernelGGL(mi355x_tls_truncate, dim3(g), dim3(256), 0, stream, (const TlsRecord *)recs, (uint32_t)n, first, dst,
                       status, types);
    HIPCHK(hipGetLastError());
    ctx->mk_dev = nullptr; /* the scan wrote over the key table's place: upload it again next time */
    return scratch_done(ctx, stream);
}

int ptls_mi355x_order_by_key(ptls_mi355x_aesgcm_context_t *ctx, const uint32_t *key_idx, size_t n, size_t nkeys,
                             uint32_t *order, void *stream_)
{
    if (n == 0)
        return 0;
    if (n > 0x7fffffffull || nkeys == 0 || nkeys > (1u << 24) || key_idx == nullptr || order == nullptr) {
        snprintf(g_err, sizeof(g_err), "order_by_key: key indices, an order array, 1..2^24 keys, under 2^31 records");
        return -1;
    }
    DeviceGuard guard(ctx->device);
    hipStream_t stream = (hipStream_t)stream_;
    /* behind the place a multi-key launch led by ctx keeps its key table, counters and slots: those survive the sort */
    const size_t pre = mk_prefix(nkeys, ctx->num_cu);
    if (ensure_scratch(ctx, pre + mk_group_bytes(n, nkeys), stream) != 0)
        return -1;
    if (mk_group(key_idx, n, nkeys, order, (uint8_t *)ctx->d_scratch + pre, stream) != 0)
        return -1;
    return scratch_done(ctx, stream);
}

int ptls_mi355x_seal_batch_multikey_ordered(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs,
                                            size_t nkeys, const ptls_mi355x_record_t *recs, const uint32_t *key_idx,
                                            const uint32_t *order, size_t n, const uint8_t *src, uint8_t *dst,
                                            const uint8_t *aad, void *stream)
{
    if (n != 0 && order == nullptr) {
        snprintf(g_err, sizeof(g_err), "seal_batch_multikey_ordered needs the order (ptls_mi355x_order_by_key)");
        return -1;
    }
    return launch_multikey(ctxs, static_ivs, nkeys, true, false, recs, key_idx, nullptr, n, src, dst, aad, nullptr, nullptr,
                           (hipStream_t)stream, order);
}

int ptls_mi355x_open_batch_multikey_ordered(ptls_mi355x_aesgcm_context_t *const *ctxs, const void *static_ivs,
                                            size_t nkeys, const ptls_mi355x_record_t *recs, const uint32_t *key_idx,
                                            const uint32_t *order, size_t n, const uint8_t *src, uint8_t *dst,
                                            const uint8_t *aad, uint32_t *status, void *stream)
{
    if (n != 0 && (order == nullptr || status == nullptr)) {
        snprintf(g_err, sizeof(g_err), "open_batch_multikey_ordered needs the order and status");
        return -1;
    }
    return launch_multikey(ctxs, static_ivs, nkeys, false, false, recs, key_idx, nullptr, n, src, dst, aad, status, nullptr,
                           (hipStream_t)stream, order);
}

const char *ptls_mi355x_kernel_name_multikey(int is_seal, size_t key_size, size_t n, int framing)
{
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        ncu = 256;
    return mk_kernel_name(is_seal != 0, framing != 0, key_size == 32 ? 32u : 16u, n, ncu);
}

/*
 * Single record in host memory (the slot calls), on the device's shared stream and staging.  Stage layout
 * (device and pinned host alike):
 *   [0, 64) descriptor | [64, 64 + A) aad | [D, D + inlen + 16) data (in place) | status
 */

/* the record's result out of the staging (which is then cleared): seal 0; open 1 verified, 0 not */
static int finish_single(DeviceShared *d, bool seal, void *output, size_t inlen, size_t off_data, size_t off_status,
                         size_t total)
{
    const size_t outlen = seal ? inlen + 16 : inlen;
    if (outlen)
        memcpy(output, d->h_stage + off_data, outlen);
    uint32_t st;
    memcpy(&st, d->h_stage + off_status, 4);
    memset(d->h_stage, 0, total);
    if (seal)
        return 0;
    return st == (uint32_t)inlen ? 1 : 0;
}

/* test hook (ptls_mi355x_test_inject_engine_errors): the next n single-record calls fail as a GPU error would */
static std::atomic<unsigned> g_inject_errors{0u};

static int single_record_staged(ptls_mi355x_aesgcm_context_t *ctx, DeviceShared *d, bool seal, void *output,
                                const void *input, size_t inlen, const void *nonce12, const void *aad, size_t aadlen,
                                const void *tag, size_t off_aad, size_t off_data, size_t off_status, size_t total);

static int single_record(ptls_mi355x_aesgcm_context_t *ctx, bool seal, void *output, const void *input, size_t inlen,
                         const void *nonce12, const void *aad, size_t aadlen, const void *tag)
{
    if (ctx == nullptr) {
        snprintf(g_err, sizeof(g_err), "no engine context");
        return -1;
    }
    if (inlen > 0xffffffffu || aadlen > 0xffffffffu) {
        snprintf(g_err, sizeof(g_err), "record too large");
        return -1;
    }
    for (unsigned n = g_inject_errors.load(); n != 0u;)
        if (g_inject_errors.compare_exchange_weak(n, n - 1u)) {
            snprintf(g_err, sizeof(g_err), "injected engine error (ptls_mi355x_test_inject_engine_errors)");
            return -1;
        }
    DeviceGuard guard(ctx->device);
    DeviceShared *d = ctx->shared;
    std::lock_guard<std::mutex> lk(d->mu);
    const size_t off_aad = 64, off_data = off_aad + up16(aadlen), off_status = off_data + up16(inlen + 16);
    const size_t total = off_status + 16;
    if (ensure_stage(d, total) != 0)
        return -1;
    const int rc = single_record_staged(ctx, d, seal, output, input, inlen, nonce12, aad, aadlen, tag, off_aad, off_data,
                                        off_status, total);
    if (rc < 0) /* a failed call leaves nothing of the record in the pinned staging */
        memset(d->h_stage, 0, total);
    return rc;
}

static int single_record_staged(ptls_mi355x_aesgcm_context_t *ctx, DeviceShared *d, bool seal, void *output,
                                const void *input, size_t inlen, const void *nonce12, const void *aad, size_t aadlen,
                                const void *tag, size_t off_aad, size_t off_data, size_t off_status, size_t total)
{
    Record rec = {off_data, off_data, off_aad, 0, (uint32_t)inlen, (uint32_t)aadlen};
    memcpy(d->h_stage, &rec, sizeof(rec));
    if (aadlen)
        memcpy(d->h_stage + off_aad, aad, aadlen);
    if (inlen)
        memcpy(d->h_stage + off_data, input, inlen);
    if (!seal)
        memcpy(d->h_stage + off_data + inlen, tag, 16);
    /*
     * Zero-copy up to g_slot_zero_copy_bytes staged bytes: the kernel reads the record from the pinned staging
     * buffer over PCIe and writes the result back into it, so a call is one launch and one synchronisation
     * instead of an H2D copy, the launch, a D2H copy and the synchronisation.  Larger records are copied.
     */
    const bool zc = total <= g_slot_zero_copy_bytes;
    uint8_t *base = zc ? d->h_stage_dev : d->d_stage;
    if (!zc)
        HIPCHK(hipMemcpyAsync(d->d_stage, d->h_stage, off_status, hipMemcpyHostToDevice, d->stream));
    /* one record: the window kernels (8-lane segments in parallel, leading pad steps skipped) are as fast as the
     * batch walk at 64 B and faster above it (scripts/slot_latency.py, profiles/r01f_slot_latency.txt) */
    if (launch_batch(ctx, seal, nonce12, (const Record *)base, nullptr, 1, base, base, base,
                     (uint32_t *)(base + off_status), d->stream, false, nullptr, nullptr) != 0)
        return -1;
    const size_t outlen = seal ? inlen + 16 : inlen;
    if (!zc) {
        HIPCHK(hipMemcpyAsync(d->h_stage + off_data, d->d_stage + off_data, outlen, hipMemcpyDeviceToHost, d->stream));
        if (!seal)
            HIPCHK(hipMemcpyAsync(d->h_stage + off_status, d->d_stage + off_status, 4, hipMemcpyDeviceToHost,
                                  d->stream));
    }
    HIPCHK(hipStreamSynchronize(d->stream));
    if (!zc)
        HIPCHK(hipMemsetAsync(d->d_stage, 0, total, d->stream)); /* nothing of the record stays on the device */
    return finish_single(d, seal, output, inlen, off_data, off_status, total);
}

unsigned ptls_mi355x_test_inject_engine_errors(unsigned n) { return g_inject_errors.exchange(n); }

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

/* nblocks of AES-ECB on host buffers through the shared staging: zero-copy up to the slot limit */
static int ecb_host(int device, int num_cu, DeviceShared *d, const uint32_t *d_keys, uint32_t nr, bool dec, void *output,
                    const void *input, size_t nblocks)
{
    if (nblocks == 0)
        return 0;
    if (nblocks > 0xffffffffu / 16) {
        snprintf(g_err, sizeof(g_err), "too many blocks");
        return -1;
    }
    DeviceGuard guard(device);
    std::lock_guard<std::mutex> lk(d->mu);
    const size_t bytes = 16 * nblocks;
    if (ensure_stage(d, bytes) != 0)
        return -1;
    memcpy(d->h_stage, input, bytes);
    const bool zc = bytes <= g_slot_zero_copy_bytes;
    uint8_t *base = zc ? d->h_stage_dev : d->d_stage;
    if (!zc)
        HIPCHK(hipMemcpyAsync(d->d_stage, d->h_stage, bytes, hipMemcpyHostToDevice, d->stream));
    uint64_t blocks = (nblocks + 255) / 256;
    if (blocks > 8ull * (uint64_t)num_cu)
        blocks = 8ull * (uint64_t)num_cu;
    hipLaunchKernelGGL(dec ? mi355x_aes_ecb_dec : mi355x_aes_ecb_enc, dim3((unsigned)blocks), dim3(256), 0, d->stream,
                       d_keys, nr, base, base, (uint32_t)nblocks);
    HIPCHK(hipGetLastError());
    if (!zc)
        HIPCHK(hipMemcpyAsync(d->h_stage, d->d_stage, bytes, hipMemcpyDeviceToHost, d->stream));
    HIPCHK(hipStreamSynchronize(d->stream));
    memcpy(output, d->h_stage, bytes);
    memset(d->h_stage, 0, bytes);
    if (!zc)
        HIPCHK(hipMemsetAsync(d->d_stage, 0, bytes, d->stream));
    return 0;
}

int ptls_mi355x_aesecb_encrypt(ptls_mi355x_aesgcm_context_t *ctx, void *output, const void *input, size_t nblocks)
{
    /* the key image starts with the FIPS-197 schedule (KeyImage::rk) */
    return ecb_host(ctx->device, ctx->num_cu, ctx->shared, ctx->d_ki->rk, ctx->key_size == 32 ? 14u : 10u, false, output,
                    input, nblocks);
}

ptls_mi355x_aes_context_t *ptls_mi355x_aes_new(const void *key, size_t key_size)
{
    if (key_size != 16 && key_size != 32) {
        snprintf(g_err, sizeof(g_err), "unsupported key size %zu", key_size);
        return nullptr;
    }
    ptls_mi355x_aes_context_t *ctx = (ptls_mi355x_aes_context_t *)calloc(1, sizeof(*ctx));
    if (ctx == nullptr)
        return nullptr;
    ctx->key_size = (uint32_t)key_size;
    ctx->rounds = key_size == 32 ? 14u : 10u;
    int rc = -1;
    DeviceShared *d = nullptr;
    if (hipGetDevice(&ctx->device) != hipSuccess ||
        hipDeviceGetAttribute(&ctx->num_cu, hipDeviceAttributeMultiprocessorCount, ctx->device) != hipSuccess ||
        (d = device_shared(ctx->device)) == nullptr || hipMalloc(&ctx->d_keys, sizeof(AesKeys)) != hipSuccess)
        goto Fail;
    ctx->shared = d;
    {
        std::lock_guard<std::mutex> lk(d->mu);
        if (ensure_stage(d, 64 + 16) != 0)
            goto Fail;
        memcpy(d->h_stage, key, key_size);
        *(volatile int *)(d->h_stage + 64) = -2;
        (void)hipGetLastError();
        hipLaunchKernelGGL(mi355x_aes_setup, dim3(1), dim3(64), 0, d->stream, d->h_stage_dev, (uint32_t)key_size,
                           ctx->d_keys, (int *)(d->h_stage_dev + 64));
        const hipError_t e1 = hipGetLastError(), e2 = hipStreamSynchronize(d->stream);
        memset(d->h_stage, 0, key_size);
        rc = *(volatile int *)(d->h_stage + 64);
        if (e1 != hipSuccess || e2 != hipSuccess || rc != 0)
            goto Fail;
    }
    return ctx;
Fail:
    if (g_err[0] == 0)
        snprintf(g_err, sizeof(g_err), "cipher setup failed: %s", hipGetErrorString(hipGetLastError()));
    ptls_mi355x_aes_free(ctx);
    return nullptr;
}

void ptls_mi355x_aes_free(ptls_mi355x_aes_context_t *ctx)
{
    if (ctx == nullptr)
        return;
    DeviceGuard guard(ctx->device);
    if (ctx->d_keys) {
        defer("cipher free: hipDeviceSynchronize", hipDeviceSynchronize());
        defer("cipher free: clearing the round keys", hipMemsetAsync(ctx->d_keys, 0, sizeof(AesKeys), nullptr));
        defer("cipher free: hipStreamSynchronize", hipStreamSynchronize(nullptr));
        defer("cipher free: hipFree", hipFree(ctx->d_keys));
    }
    free(ctx);
}

int ptls_mi355x_aes_ecb(ptls_mi355x_aes_context_t *ctx, int is_enc, void *output, const void *input, size_t nblocks)
{
    return ecb_host(ctx->device, ctx->num_cu, ctx->shared, is_enc ? ctx->d_keys->rk : ctx->d_keys->dk, ctx->rounds, !is_enc,
                    output, input, nblocks);
}

int ptls_mi355x_aes_ecb_batch(ptls_mi355x_aes_context_t *ctx, int is_enc, uint8_t *dst, const uint8_t *src, size_t nblocks,
                              void *stream)
{
    if (nblocks == 0)
        return 0;
    if (nblocks > 0xffffffffull) {
        snprintf(g_err, sizeof(g_err), "too many blocks");
        return -1;
    }
    DeviceGuard guard(ctx->device);
    uint64_t blocks = (nblocks + 255) / 256;
    if (blocks > 8ull * (uint64_t)ctx->num_cu)
        blocks = 8ull * (uint64_t)ctx->num_cu;
    hipLaunchKernelGGL(is_enc ? mi355x_aes_ecb_enc : mi355x_aes_ecb_dec, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, is_enc ? ctx->d_keys->rk : ctx->d_keys->dk, ctx->rounds, src, dst,
                       (uint32_t)nblocks);
    HIPCHK(hipGetLastError());
    return 0;
}

} /* extern "C" */

#if GCM_WIN_TIMING
/* measurement builds: the phase stamps of the last window launch (s_memrealtime ticks, 100 MHz) */
extern "C" int ptls_mi355x_debug_window_times(uint64_t *out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_win_times), sizeof(uint64_t) * 32) == hipSuccess ? 0 : -1;
}
#endif
