/*
 * scripts/gcm_sbox.h -- the AES S-box as a bitsliced circuit on the VALU, and an in-lane bitsliced last AES round
 * for two blocks (a MEASUREMENT header: included by scripts/gcm_bitslice.h inside namespace mi355x, built into
 * the host kernel model of the CPU tests and into the r02 ablation variant; the product does not use it).
 *
 * The T-table AES of gcm_core.h reads 16 S-box bytes from the LDS in the last round of every block.
 * aes_last_round_bs2 computes that round for TWO blocks of a lane on the VALU instead: the 32 state bytes are
 * transposed into 8 bit planes of 32 bits (3 levels of swap-moves over the 8 state words), the Boyar-Peralta
 * S-box circuit runs on the planes (92 gates: 54 three-input LUTs, 38 two-input gates, scripts/sbox_lut3.py),
 * the planes are transposed back, and ShiftRows + the round key are byte permutes.  212 VALU ops per two blocks
 * replace 32 LDS reads and their 32 address perms.  Measured in the batch open walk (r02d ablation,
 * profiles/r02d_ablate_paired_bitsliced_last_round.txt): 9 % SLOWER -- the kernel is co-limited by VALU issue
 * and the LDS, so moving work from one to the other does not pay ("Negative results").
 */

/* any 3-input boolean function, bit-parallel: one v_bitop3_b32; table index = (a << 2) | (b << 1) | c */
template <uint32_t TT>
GCM_HD uint32_t lut3(uint32_t a, uint32_t b, uint32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
#else
    uint32_t r = 0;
    for (uint32_t idx = 0; idx < 8; ++idx)
        if ((TT >> idx) & 1u)
            r |= ((idx & 4u) ? a : ~a) & ((idx & 2u) ? b : ~b) & ((idx & 1u) ? c : ~c);
    return r;
#endif
}

/*
 * Two-input gates pinned to VOP2 encodings (v_xor/v_and/v_xnor_b32: 2 clk per wave64).  Measured issue costs
 * on gfx950 (scripts/isa_rates.hip, profiles/r02a_isa_rates.json, r02c_isa_rates2.json): v_bitop3_b32 also
 * issues in 2 clk when its three sources are three DIFFERENT VGPRs (or an inline constant), but in ~3.4 when a
 * source is an SGPR or the same VGPR twice; v_perm_b32, v_alignbit_b32, v_bfe/v_and_or/v_lshl_or and DPP ops
 * take ~3.4 whatever their operands, as does a VOP2 op with an SGPR source.  So a two-input gate is a VOP2 op,
 * never a v_bitop3_b32 with a repeated operand; the asm keeps the compiler from re-fusing it.
 */
#if defined(__HIP_DEVICE_COMPILE__)
GCM_HD uint32_t gx(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
GCM_HD uint32_t ga(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_and_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
GCM_HD uint32_t gxn(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_xnor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
#else
GCM_HD uint32_t gx(uint32_t a, uint32_t b) { return a ^ b; }
GCM_HD uint32_t ga(uint32_t a, uint32_t b) { return a & b; }
GCM_HD uint32_t gxn(uint32_t a, uint32_t b) { return ~(a ^ b); }
#endif

#ifndef GCM_SBOX_LUT3
#define GCM_SBOX_LUT3 1
#endif

/* SubBytes on 8 planes (in place): the Boyar-Peralta circuit; U0 / S0 is the most significant bit */
template <class V>
GCM_HD void sbox_bs(V p[8])
{
    const V U0 = p[7], U1 = p[6], U2 = p[5], U3 = p[4], U4 = p[3], U5 = p[2], U6 = p[1], U7 = p[0];
#if GCM_SBOX_LUT3
    /* the circuit mapped onto 92 three-input LUTs (scripts/sbox_lut3.py --emit) */
    const V T1 = gx(U0, U3);
    const V T2 = gx(U0, U5);
    const V T3 = gx(U0, U6);
    const V T4 = gx(U3, U5);
    const V T5 = gx(U4, U6);
    const V T6 = lut3<0x96>(U4, U6, T1);
    const V T7 = gx(U1, U2);
    const V T8 = gx(U7, T6);
    const V T10 = lut3<0x96>(U1, U2, T6);
    const V T11 = gx(U1, U5);
    const V T13 = lut3<0x96>(U3, U5, T3);
    const V T15 = lut3<0x96>(U1, U5, T5);
    const V T16 = lut3<0x96>(U2, U5, T5);
    const V T17 = lut3<0x96>(U7, T7, T16);
    const V T19 = lut3<0x96>(U3, U7, T7);
    const V T20 = lut3<0x96>(U0, U3, T19);
    const V T22 = lut3<0x96>(U6, U7, T7);
    const V T23 = lut3<0x96>(U0, U5, T22);
    const V T24 = lut3<0x96>(U0, U5, T10);
    const V T25 = gx(T17, T20);
    const V T27 = lut3<0x96>(U2, U5, T1);
    const V M1 = lut3<0x28>(T3, T4, T6);
    const V M2 = lut3<0x28>(U7, T6, T23);
    const V M3 = lut3<0x9c>(T6, T11, T13);
    const V M5 = lut3<0x6a>(U7, T19, M1);
    const V M6 = lut3<0x28>(U0, U6, T16);
    const V M7 = lut3<0x06>(U6, U7, T7);
    const V M8 = lut3<0xbe>(U0, U6, T16);
    const V M10 = lut3<0x6a>(T17, T20, M6);
    const V M11 = lut3<0x28>(U0, U3, T15);
    const V M13 = lut3<0x6a>(T4, T27, M11);
    const V M15 = lut3<0x6a>(T2, T10, M11);
    const V M20 = lut3<0x96>(M2, M3, M13);
    const V M21 = lut3<0x96>(T24, M5, M15);
    const V M22 = lut3<0x96>(M7, M8, M13);
    const V M23 = lut3<0x96>(T25, M10, M15);
    const V M24 = gx(M22, M23);
    const V M25 = ga(M20, M22);
    const V M27 = gx(M20, M21);
    const V M29 = lut3<0x28>(M23, M25, M27);
    const V M30 = lut3<0x48>(M21, M24, M25);
    const V M31 = ga(M20, M23);
    const V M34 = ga(M21, M22);
    const V M37 = gx(M21, M29);
    const V M38 = lut3<0xb4>(M25, M27, M31);
    const V M39 = gx(M23, M30);
    const V M40 = lut3<0x9c>(M24, M25, M34);
    const V M41 = gx(M38, M40);
    const V M42 = gx(M37, M39);
    const V M43 = gx(M37, M38);
    const V M44 = gx(M39, M40);
    const V M45 = gx(M41, M42);
    const V M46 = ga(T6, M44);
    const V M48 = ga(U7, M39);
    const V M50 = lut3<0x28>(U7, T7, M38);
    const V M51 = ga(T17, M37);
    const V M52 = ga(T15, M42);
    const V M53 = ga(T27, M45);
    const V M55 = lut3<0x28>(T3, T4, M44);
    const V M56 = lut3<0x28>(T2, T22, M40);
    const V M58 = lut3<0x28>(U0, U6, M43);
    const V M61 = lut3<0x28>(U0, U3, M42);
    const V M62 = lut3<0x28>(U3, U5, M45);
    const V M63 = lut3<0x28>(U0, U5, M41);
    const V L0 = gx(M61, M62);
    const V L1 = gx(M50, M56);
    const V L2 = gx(M46, M48);
    const V L3 = lut3<0x6a>(T8, M40, M55);
    const V L4 = lut3<0x6a>(T10, M41, M58);
    const V L5 = lut3<0x6a>(T16, M43, M61);
    const V L6 = gx(M62, L5);
    const V L7 = gx(M46, L3);
    const V L8 = lut3<0x6a>(T22, M38, M51);
    const V L9 = gx(M52, M53);
    const V L10 = gx(M53, L4);
    const V L11 = lut3<0x6a>(T20, M37, L2);
    const V L13 = gx(M50, L0);
    const V L17 = lut3<0x6a>(T19, M39, L1);
    const V L18 = gx(M58, L8);
    const V L22 = lut3<0x96>(M48, M51, L3);
    const V L24 = lut3<0x96>(M55, L1, L9);
    const V L26 = gx(L7, L9);
    const V L28 = lut3<0x96>(M52, M61, L11);
    const V L29 = gx(L11, L17);
    const V S0 = gx(L6, L24);
    const V S1 = lut3<0x69>(M56, L0, L26);
    const V S2 = lut3<0x69>(M63, L4, L28);
    const V S3 = lut3<0x96>(L1, L6, L7);
    const V S4 = lut3<0x96>(L0, L1, L22);
    const V S5 = lut3<0x96>(L6, L10, L29);
    const V S6 = lut3<0x69>(L8, L10, L13);
    const V S7 = lut3<0x69>(L2, L6, L18);
#else
    /* the 128 gates as VOP2 ops (2 clk each): cheaper than the 92-LUT cover (4 clk each) */
    const V T1 = gx(U0, U3); const V T2 = gx(U0, U5); const V T3 = gx(U0, U6); const V T4 = gx(U3, U5);
    const V T5 = gx(U4, U6); const V T6 = gx(T1, T5); const V T7 = gx(U1, U2); const V T8 = gx(U7, T6);
    const V T9 = gx(U7, T7); const V T10 = gx(T6, T7); const V T11 = gx(U1, U5); const V T12 = gx(U2, U5);
    const V T13 = gx(T3, T4); const V T14 = gx(T6, T11); const V T15 = gx(T5, T11); const V T16 = gx(T5, T12);
    const V T17 = gx(T9, T16); const V T18 = gx(U3, U7); const V T19 = gx(T7, T18); const V T20 = gx(T1, T19);
    const V T21 = gx(U6, U7); const V T22 = gx(T7, T21); const V T23 = gx(T2, T22); const V T24 = gx(T2, T10);
    const V T25 = gx(T20, T17); const V T26 = gx(T3, T16); const V T27 = gx(T1, T12); const V M1 = ga(T13, T6);
    const V M2 = ga(T23, T8); const V M3 = gx(T14, M1); const V M4 = ga(T19, U7); const V M5 = gx(M4, M1);
    const V M6 = ga(T3, T16); const V M7 = ga(T22, T9); const V M8 = gx(T26, M6); const V M9 = ga(T20, T17);
    const V M10 = gx(M9, M6); const V M11 = ga(T1, T15); const V M12 = ga(T4, T27); const V M13 = gx(M12, M11);
    const V M14 = ga(T2, T10); const V M15 = gx(M14, M11); const V M16 = gx(M3, M2); const V M17 = gx(M5, T24);
    const V M18 = gx(M8, M7); const V M19 = gx(M10, M15); const V M20 = gx(M16, M13); const V M21 = gx(M17, M15);
    const V M22 = gx(M18, M13); const V M23 = gx(M19, T25); const V M24 = gx(M22, M23); const V M25 = ga(M22, M20);
    const V M26 = gx(M21, M25); const V M27 = gx(M20, M21); const V M28 = gx(M23, M25); const V M29 = ga(M28, M27);
    const V M30 = ga(M26, M24); const V M31 = ga(M20, M23); const V M32 = ga(M27, M31); const V M33 = gx(M27, M25);
    const V M34 = ga(M21, M22); const V M35 = ga(M24, M34); const V M36 = gx(M24, M25); const V M37 = gx(M21, M29);
    const V M38 = gx(M32, M33); const V M39 = gx(M23, M30); const V M40 = gx(M35, M36); const V M41 = gx(M38, M40);
    const V M42 = gx(M37, M39); const V M43 = gx(M37, M38); const V M44 = gx(M39, M40); const V M45 = gx(M42, M41);
    const V M46 = ga(M44, T6); const V M47 = ga(M40, T8); const V M48 = ga(M39, U7); const V M49 = ga(M43, T16);
    const V M50 = ga(M38, T9); const V M51 = ga(M37, T17); const V M52 = ga(M42, T15); const V M53 = ga(M45, T27);
    const V M54 = ga(M41, T10); const V M55 = ga(M44, T13); const V M56 = ga(M40, T23); const V M57 = ga(M39, T19);
    const V M58 = ga(M43, T3); const V M59 = ga(M38, T22); const V M60 = ga(M37, T20); const V M61 = ga(M42, T1);
    const V M62 = ga(M45, T4); const V M63 = ga(M41, T2); const V L0 = gx(M61, M62); const V L1 = gx(M50, M56);
    const V L2 = gx(M46, M48); const V L3 = gx(M47, M55); const V L4 = gx(M54, M58); const V L5 = gx(M49, M61);
    const V L6 = gx(M62, L5); const V L7 = gx(M46, L3); const V L8 = gx(M51, M59); const V L9 = gx(M52, M53);
    const V L10 = gx(M53, L4); const V L11 = gx(M60, L2); const V L12 = gx(M48, M51); const V L13 = gx(M50, L0);
    const V L14 = gx(M52, M61); const V L15 = gx(M55, L1); const V L16 = gx(M56, L0); const V L17 = gx(M57, L1);
    const V L18 = gx(M58, L8); const V L19 = gx(M63, L4); const V L20 = gx(L0, L1); const V L21 = gx(L1, L7);
    const V L22 = gx(L3, L12); const V L23 = gx(L18, L2); const V L24 = gx(L15, L9); const V L25 = gx(L6, L10);
    const V L26 = gx(L7, L9); const V L27 = gx(L8, L10); const V L28 = gx(L11, L14); const V L29 = gx(L11, L17);
    const V S0 = gx(L6, L24); const V S1 = gxn(L16, L26); const V S2 = gxn(L19, L28); const V S3 = gx(L6, L21);
    const V S4 = gx(L20, L22); const V S5 = gx(L25, L29); const V S6 = gxn(L13, L27); const V S7 = gxn(L6, L23);
#endif
    p[7] = S0;
    p[6] = S1;
    p[5] = S2;
    p[4] = S3;
    p[3] = S4;
    p[2] = S5;
    p[1] = S6;
    p[0] = S7;
}

/* a constant held in a VGPR (v_bitop3_b32 with an SGPR source issues at ~3.4 clk instead of 2) */
GCM_HD uint32_t vconst(uint32_t c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(c));
#endif
    return c;
}

/* swap-move: exchanges the bits of a selected by (m << n) with the bits of b selected by m */
GCM_HD void swapmove(uint32_t &a, uint32_t &b, uint32_t m, uint32_t n)
{
    const uint32_t t = lut3<0x28>(a >> n, b, m); /* (a >> n ^ b) & m */
    b = gx(b, t);
    a = gx(a, t << n);
}

/*
 * 8 x 8 bit transpose in every byte lane of 8 words: bit i of byte q of w[r] <-> bit r of byte q of w[i]
 * (an involution).  After it, w[i] is the bit plane of bit i of the 32 bytes (byte q of word r at bit r of byte
 * q), the layout sbox_bs works on.  m4 / m2 / m1: 0x0f0f0f0f, 0x33333333, 0x55555555 in VGPRs.
 */
GCM_HD void transpose8_bytes(uint32_t w[8], uint32_t m4, uint32_t m2, uint32_t m1)
{
#pragma unroll
    for (int i = 0; i < 4; ++i)
        swapmove(w[i], w[i + 4], m4, 4);
#pragma unroll
    for (int i = 0; i < 8; i += 4) {
        swapmove(w[i], w[i + 2], m2, 2);
        swapmove(w[i + 1], w[i + 3], m2, 2);
    }
#pragma unroll
    for (int i = 0; i < 8; i += 2)
        swapmove(w[i], w[i + 1], m1, 1);
}

/*
 * The last AES round of two blocks: a[4], b[4] (LE column words after round NR-1) become the output of
 * SubBytes, ShiftRows and AddRoundKey with the round key k[0..3].  Bit-identical to the T-table last round.
 */
GCM_HD void aes_last_round_bs2(uint32_t a[4], uint32_t b[4], const uint32_t *k)
{
    const uint32_t m4 = vconst(0x0f0f0f0fu), m2 = vconst(0x33333333u), m1 = vconst(0x55555555u);
    uint32_t w[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    transpose8_bytes(w, m4, m2, m1);
    sbox_bs(w);
    transpose8_bytes(w, m4, m2, m1);
    /* ShiftRows: output column j takes row r from column j + r */
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        a[j] = xor3(perm(w[(j + 1) & 3], w[j], 0x0c0c0500u), perm(w[(j + 3) & 3], w[(j + 2) & 3], 0x07020c0cu), k[j]);
        b[j] = xor3(perm(w[4 + ((j + 1) & 3)], w[4 + j], 0x0c0c0500u),
                    perm(w[4 + ((j + 3) & 3)], w[4 + ((j + 2) & 3)], 0x07020c0cu), k[j]);
    }
}
