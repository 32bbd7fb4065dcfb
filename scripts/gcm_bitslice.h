/*
 * scripts/gcm_bitslice.h -- bitsliced AES-CTR in the quad layout (a MEASUREMENT engine: scripts/probe_bs.hip and
 * the host kernel model's test use it; the product does not).
 *
 * Why: the T-table AES of gcm_core.h is bound by the LDS array (ds_read_b32 serves 32 lanes per
 * clock; 133 reads per AES-128 block) while the VALU idles half the time.  Bitsliced AES needs no
 * table reads at all, so waves running it use the idle VALU beside waves running T-tables.
 *
 * Layout ("quad layout"): the 4 lanes of a quad (q = lane & 3) encrypt 8 blocks together.  Lane q
 * holds AES state ROW q of the 8 blocks in 8 bit-plane registers p[0..7]: p[i] holds bit i of
 * each state byte, byte c of the register is column c, bit b of that byte is block b.
 *   SubBytes    the Boyar-Peralta depth-16 circuit (34 AND + 94 XOR/XNOR, scripts/sbox_circuit.py
 *               checks it on all 256 inputs) on the 8 planes: 32 S-boxes per gate;
 *   ShiftRows   row q rotates its columns by q: one rotate of each plane by 8q bits;
 *   MixColumns  the 4 rows of a column sit in the quad's 4 lanes: DPP quad_perm brings rows q+1
 *               and q-1 (out_q = 2(a_q + a_q+1) + (a_q+1 + a_q+2) + a_q+3, xtime on planes);
 *   AddRoundKey XOR with the round key's planes for row q, read from LDS (2 ds_read_b128/round).
 * Counter blocks nonce || BE32(ctr0 + b), b = 0..7, enter as planes (an 8x8 bit transpose of the
 * counter bytes); the keystream leaves as whole blocks: an 8x8 bit transpose per byte column, a
 * 4x4 dword transpose across the quad (DPP), a 4x4 byte transpose (v_perm).  Lane t then holds
 * blocks t and t + 4 -- exactly the two positions of an 8-position step that lane j = t of the
 * K = 4 record walk hashes (stride-4 Horner chains).
 *
 * Everything is written once over a lane-value type: on the GPU a uint32_t per lane (QuadOpsDev,
 * cross-lane moves through DPP), on the host a Quad4 holding the four lanes in lockstep
 * (QuadOpsHost), so the CPU tests run the same code.
 */
#pragma once
#include "../rapido_amd/csrc/gcm_core.h"

namespace mi355x {
#include "gcm_sbox.h"

/* DPP quad_perm controls: lane q of the quad takes lane ((CTRL >> 2q) & 3) */
enum : int {
    QP_NEXT = 0x39,  /* q + 1 */
    QP_PREV = 0x93,  /* q - 1 */
    QP_SWAP1 = 0xB1, /* q ^ 1 */
    QP_SWAP2 = 0x4E, /* q ^ 2 */
};

/* LDS image of the round-key planes: round r, row q, plane i at r*128 + q*32 + 4i (1920 B for 15 rounds) */
enum : uint32_t { KEYPLANE_BYTES = 15u * 128u };

/*
 * Fills the key-plane image for rounds 0..nr: dword (r, q, i) has byte c = 0xff if bit i of round-key
 * byte (row q, column c) is set.  rk = LE dwords of the key schedule (rk[4r + c] = column c).
 */
GCM_HD void fill_keyplanes(uint8_t *dst, const uint32_t *rk, uint32_t nr, uint32_t tid, uint32_t nthr)
{
    for (uint32_t x = tid; x < 32u * (nr + 1u); x += nthr) {
        const uint32_t r = x >> 5, q = (x >> 3) & 3u, i = x & 7u;
        uint32_t v = 0;
        for (uint32_t c = 0; c < 4; ++c)
            v |= ((rk[4 * r + c] >> (8 * q + i)) & 1u) ? (0xffu << (8 * c)) : 0u;
        *(uint32_t *)(dst + 128u * r + 32u * q + 4u * i) = v;
    }
}

/* ------------------------------------------------------------------ lane-value operations ---- */

#if defined(__HIPCC__)
/* one lane of a wave: the value type is the lane's own uint32_t */
struct QuadOpsDev {
    typedef uint32_t V;
    uint32_t rowshift; /* 8 * q */
    uint32_t q;
    __device__ explicit QuadOpsDev(uint32_t lane) : rowshift(8u * (lane & 3u)), q(lane & 3u) {}
    template <int CTRL>
    __device__ __forceinline__ uint32_t qperm(uint32_t x) const
    {
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
    }
    /* ShiftRows for row q: rotate right by 8q bits (one v_alignbit_b32 with a per-lane shift) */
    __device__ __forceinline__ uint32_t rotr_row(uint32_t x) const { return __builtin_amdgcn_alignbit(x, x, rowshift); }
    /* lanes with (q & m) != 0 take a, the others b */
    __device__ __forceinline__ uint32_t sel(uint32_t a, uint32_t b, uint32_t m) const { return (q & m) ? a : b; }
    __device__ __forceinline__ uint32_t row() const { return q; }
};
#endif

#if !defined(__HIPCC__)
/* host model: the 4 lanes of a quad in lockstep */
struct Quad4 {
    uint32_t v[4];
};
static inline Quad4 q4(uint32_t c) { return Quad4{{c, c, c, c}}; }
#define MI355X_Q4_BINOP(OP)                                                                                            \
    static inline Quad4 operator OP(Quad4 a, Quad4 b)                                                                  \
    {                                                                                                                  \
        for (int k = 0; k < 4; ++k)                                                                                    \
            a.v[k] = a.v[k] OP b.v[k];                                                                                 \
        return a;                                                                                                      \
    }                                                                                                                  \
    static inline Quad4 operator OP(Quad4 a, uint32_t b)                                                               \
    {                                                                                                                  \
        for (int k = 0; k < 4; ++k)                                                                                    \
            a.v[k] = a.v[k] OP b;                                                                                      \
        return a;                                                                                                      \
    }
MI355X_Q4_BINOP(^)
MI355X_Q4_BINOP(&)
MI355X_Q4_BINOP(|)
MI355X_Q4_BINOP(+)
MI355X_Q4_BINOP(>>)
MI355X_Q4_BINOP(<<)
MI355X_Q4_BINOP(*)
#undef MI355X_Q4_BINOP
static inline Quad4 operator~(Quad4 a)
{
    for (int k = 0; k < 4; ++k)
        a.v[k] = ~a.v[k];
    return a;
}
static inline Quad4 &operator^=(Quad4 &a, Quad4 b) { return a = a ^ b; }
static inline Quad4 perm(Quad4 hi, Quad4 lo, uint32_t sel)
{
    for (int k = 0; k < 4; ++k)
        lo.v[k] = perm(hi.v[k], lo.v[k], sel);
    return lo;
}

struct QuadOpsHost {
    typedef Quad4 V;
    template <int CTRL>
    Quad4 qperm(Quad4 x) const
    {
        Quad4 r;
        for (int k = 0; k < 4; ++k)
            r.v[k] = x.v[(CTRL >> (2 * k)) & 3];
        return r;
    }
    Quad4 rotr_row(Quad4 x) const
    {
        for (int k = 1; k < 4; ++k)
            x.v[k] = (x.v[k] >> (8 * k)) | (x.v[k] << (32 - 8 * k));
        return x;
    }
    Quad4 sel(Quad4 a, Quad4 b, uint32_t m) const
    {
        for (int k = 0; k < 4; ++k)
            if (!(k & m))
                a.v[k] = b.v[k];
        return a;
    }
    Quad4 row() const { return Quad4{{0u, 1u, 2u, 3u}}; }
};

/* the 8 key planes of one round for each lane's row (addr per lane) */
static inline void load_keyplanes(const uint8_t *lds, Quad4 addr, Quad4 k[8])
{
    for (int l = 0; l < 4; ++l)
        for (int i = 0; i < 8; ++i)
            k[i].v[l] = lds_u32(lds, addr.v[l] + 4u * (uint32_t)i);
}
#endif

#if defined(__HIPCC__)
/* the 8 key planes of one round for the lane's row: two ds_read_b128 */
__device__ __forceinline__ void load_keyplanes(const uint8_t *lds, uint32_t addr, uint32_t k[8])
{
    const u32x4 a = lds_u32x4(lds, addr), b = lds_u32x4(lds, addr + 16u);
    k[0] = a[0], k[1] = a[1], k[2] = a[2], k[3] = a[3];
    k[4] = b[0], k[5] = b[1], k[6] = b[2], k[7] = b[3];
}
#endif

/* ------------------------------------------------------------------ the round function ------ */

/* the S-box circuit (sbox_bs), lut3 and the two-input gates on uint32_t lanes come from gcm_sbox.h; these are their host overloads for the quad model */
#if !defined(__HIPCC__)
template <uint32_t TT>
static inline Quad4 lut3(Quad4 a, Quad4 b, Quad4 c)
{
    for (int k = 0; k < 4; ++k)
        a.v[k] = lut3<TT>(a.v[k], b.v[k], c.v[k]);
    return a;
}
static inline Quad4 gx(Quad4 a, Quad4 b) { return a ^ b; }
static inline Quad4 ga(Quad4 a, Quad4 b) { return a & b; }
static inline Quad4 gxn(Quad4 a, Quad4 b) { return ~(a ^ b); }
#endif

/*
 * MixColumns across the quad: out_q = 2 a_q + 3 a_q+1 + a_q+2 + a_q+3 = xtime(t) + (colsum + a_q) with
 * t = a_q + a_q+1 and colsum = t + t_q+2 (the XOR of the whole column): two DPP ops per plane.
 */
template <class O, class V>
GCM_HD void mixcolumns_bs(const O &o, V p[8])
{
    V t[8], c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        t[i] = p[i] ^ o.template qperm<QP_NEXT>(p[i]);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        c[i] = gx(t[i] ^ o.template qperm<QP_SWAP2>(t[i]), p[i]); /* colsum + a_q = a_q+1 + a_q+2 + a_q+3 */
    /* xtime on planes: bit i <- bit i-1, bit 7 folds into bits 0, 1, 3, 4 (x^8 = x^4 + x^3 + x + 1) */
    p[0] = gx(t[7], c[0]);
    p[1] = gx(gx(t[0], t[7]), c[1]);
    p[2] = gx(t[1], c[2]);
    p[3] = gx(gx(t[2], t[7]), c[3]);
    p[4] = gx(gx(t[3], t[7]), c[4]);
    p[5] = gx(t[4], c[5]);
    p[6] = gx(t[5], c[6]);
    p[7] = gx(t[6], c[7]);
}

/*
 * AES-NR of the quad's 8 blocks in plane form (in place).  keyplanes(r, k) loads round r's 8 planes
 * for the lane's row.
 */
template <int NR, class O, class V, class KF>
GCM_HD void aes_bs(const O &o, V p[8], const KF &keyplanes)
{
    V k[8];
    keyplanes(0, k);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        p[i] = p[i] ^ k[i];
    /* rounds as a loop, not unrolled: one round's temporaries live at a time (VGPR budget) */
#pragma unroll 1
    for (int r = 1; r < NR; ++r) {
        sbox_bs(p);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            p[i] = o.rotr_row(p[i]);
        mixcolumns_bs(o, p);
        keyplanes(r, k);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            p[i] = p[i] ^ k[i];
    }
    sbox_bs(p);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        p[i] = o.rotr_row(p[i]);
    keyplanes(NR, k);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        p[i] = p[i] ^ k[i];
}

/* G independent plane sets through AES-NR at once (instruction-level parallelism for the VALU issue) */
template <int NR, int G, class O, class V, class KF>
GCM_HD void aes_bs_multi(const O &o, V (*p)[8], const KF &keyplanes)
{
    V k[8];
    keyplanes(0, k);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i)
            p[g][i] = p[g][i] ^ k[i];
#pragma unroll 1
    for (int r = 1; r < NR; ++r) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            sbox_bs(p[g]);
#pragma unroll
            for (int i = 0; i < 8; ++i)
                p[g][i] = o.rotr_row(p[g][i]);
            mixcolumns_bs(o, p[g]);
        }
        keyplanes(r, k);
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int i = 0; i < 8; ++i)
                p[g][i] = p[g][i] ^ k[i];
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
        sbox_bs(p[g]);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            p[g][i] = o.rotr_row(p[g][i]);
    }
    keyplanes(NR, k);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i)
            p[g][i] = p[g][i] ^ k[i];
}

/* ------------------------------------------------------------------ into and out of planes --- */

/* in place: the 8x8 bit matrix with row b in byte b of {lo (rows 0-3), hi (rows 4-7)} is transposed */
template <class V>
GCM_HD void transpose8x8(V &lo, V &hi)
{
    V t = ((lo >> 4u) ^ hi) & 0x0f0f0f0fu;
    hi = hi ^ t;
    lo = lo ^ (t << 4u);
    t = (lo ^ (lo >> 14u)) & 0x0000ccccu;
    lo = lo ^ t ^ (t << 14u);
    t = (hi ^ (hi >> 14u)) & 0x0000ccccu;
    hi = hi ^ t ^ (t << 14u);
    t = (lo ^ (lo >> 7u)) & 0x00aa00aau;
    lo = lo ^ t ^ (t << 7u);
    t = (hi ^ (hi >> 7u)) & 0x00aa00aau;
    hi = hi ^ t ^ (t << 7u);
}

/*
 * Planes of the 8 counter blocks nonce || BE32(ctr0 + b), b = 0..7, for the lane's row q
 * (n0..n2: the nonce as LE dwords).  Columns 0-2 of row q are nonce bytes 4c + q (same for all 8
 * blocks: a byte of 0x00 or 0xff per plane); column 3 is byte q of the big-endian counter.
 */
template <class O, class V>
GCM_HD void ctr_planes_bs(const O &o, V n0, V n1, V n2, V ctr0, V p[8])
{
    const V sh = o.row() << 3u;
    const V x = ((n0 >> sh) & 0xffu) | (((n1 >> sh) & 0xffu) << 8u) | (((n2 >> sh) & 0xffu) << 16u);
    const V csh = (o.row() ^ 3u) << 3u; /* byte q of BE32(v) is byte 3 - q of v */
    V lo = ((ctr0 >> csh) & 0xffu) | (((ctr0 + 1u) >> csh) & 0xffu) << 8u | (((ctr0 + 2u) >> csh) & 0xffu) << 16u |
           (((ctr0 + 3u) >> csh) & 0xffu) << 24u;
    V hi = (((ctr0 + 4u) >> csh) & 0xffu) | (((ctr0 + 5u) >> csh) & 0xffu) << 8u |
           (((ctr0 + 6u) >> csh) & 0xffu) << 16u | (((ctr0 + 7u) >> csh) & 0xffu) << 24u;
    transpose8x8(lo, hi); /* byte i of {lo, hi}: bit b = bit i of the counter byte of block b */
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const V z = i < 4 ? (lo >> (uint32_t)(8 * i)) : (hi >> (uint32_t)(8 * (i - 4)));
        p[i] = (((x >> (uint32_t)i) & 0x010101u) * 0xffu) | (z << 24u);
    }
}

/*
 * The 8 planes back to whole blocks: returns, in lane t, the keystream of blocks t (ks_a) and t + 4
 * (ks_b) of the quad, as LE dwords in memory order.
 */
template <class O, class V>
GCM_HD void planes_to_blocks_bs(const O &o, V p[8], V ks_a[4], V ks_b[4])
{
    /* 1: per byte column, the 8x8 (plane i, block b) bit matrix -> p[b] byte c = keystream byte 4c + q of block b */
#pragma unroll
    for (int j = 4; j >= 1; j >>= 1) {
        const uint32_t m = j == 4 ? 0x0f0f0f0fu : j == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k & j)
                continue;
            const V t = ((p[k] >> (uint32_t)j) ^ p[k + j]) & m;
            p[k + j] = p[k + j] ^ t;
            p[k] = p[k] ^ (t << (uint32_t)j);
        }
    }
    /* 2: 4x4 dword transpose across the quad, per half h: lane t receives p[4h + t] of lanes 0..3 */
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        V *a = p + 4 * h;
#pragma unroll
        for (int k = 0; k < 4; k += 2) {
            const V send = o.sel(a[k], a[k + 1], 1u);
            const V recv = o.template qperm<QP_SWAP1>(send);
            a[k + 1] = o.sel(a[k + 1], recv, 1u);
            a[k] = o.sel(recv, a[k], 1u);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const V send = o.sel(a[k], a[k + 2], 2u);
            const V recv = o.template qperm<QP_SWAP2>(send);
            a[k + 2] = o.sel(a[k + 2], recv, 2u);
            a[k] = o.sel(recv, a[k], 2u);
        }
    }
    /* 3: a[q] byte c = block byte 4c + q  ->  dword d = bytes 4d .. 4d + 3 */
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const V *a = p + 4 * h;
        V *ks = h ? ks_b : ks_a;
        const V lo01 = perm(a[1], a[0], 0x05010400u), hi01 = perm(a[1], a[0], 0x07030602u);
        const V lo23 = perm(a[3], a[2], 0x05010400u), hi23 = perm(a[3], a[2], 0x07030602u);
        ks[0] = perm(lo23, lo01, 0x05040100u);
        ks[1] = perm(lo23, lo01, 0x07060302u);
        ks[2] = perm(hi23, hi01, 0x05040100u);
        ks[3] = perm(hi23, hi01, 0x07060302u);
    }
}

/*
 * AES-NR-CTR keystream of blocks nonce || BE32(ctr0 + b), b = 0..7, by the quad: lane t receives
 * blocks t and t + 4.  Key planes at lds[kp_base ...] (fill_keyplanes).
 */
template <int NR, class O, class V>
GCM_HD void ctr_keystream_bs(const O &o, const uint8_t *lds, uint32_t kp_base, V n0, V n1, V n2, V ctr0, V ks_a[4],
                             V ks_b[4])
{
    V p[8];
    ctr_planes_bs(o, n0, n1, n2, ctr0, p);
    const V kaddr = (o.row() << 5u) + kp_base;
    auto keyplanes = [&](int r, V k[8]) { load_keyplanes(lds, kaddr + (uint32_t)(128 * r), k); };
    aes_bs<NR>(o, p, keyplanes);
    planes_to_blocks_bs(o, p, ks_a, ks_b);
}

/* two groups of 8 counter blocks (ctr0a.., ctr0b..) at once: lane t receives blocks t and t + 4 of each */
template <int NR, class O, class V>
GCM_HD void ctr_keystream_bs2(const O &o, const uint8_t *lds, uint32_t kp_base, V n0, V n1, V n2, V ctr0a, V ctr0b,
                              V ks[4][4])
{
    V p[2][8];
    ctr_planes_bs(o, n0, n1, n2, ctr0a, p[0]);
    ctr_planes_bs(o, n0, n1, n2, ctr0b, p[1]);
    const V kaddr = (o.row() << 5u) + kp_base;
    auto keyplanes = [&](int r, V k[8]) { load_keyplanes(lds, kaddr + (uint32_t)(128 * r), k); };
    aes_bs_multi<NR, 2>(o, p, keyplanes);
    planes_to_blocks_bs(o, p[0], ks[0], ks[1]);
    planes_to_blocks_bs(o, p[1], ks[2], ks[3]);
}

} // namespace mi355x
