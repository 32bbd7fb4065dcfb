/*
 * scripts/isa_rates.hip -- issue-rate microbenchmark of the VALU forms an AES T-table round can be built
 * from (measurement only, never linked into the engine).  Every variant runs the same instruction
 * 8 x 64 times per loop trip over 8 independent register chains, 16 waves per CU on every CU; the time
 * per wave-instruction per SIMD is reported relative to v_xor_b32 (a VOP2 op: 2 clk per wave64 on a
 * SIMD-32).  Built and run standalone:
 *   hipcc --offload-arch=gfx950 -O3 scripts/isa_rates.hip -o scripts/_bin/isa_rates && scripts/_bin/isa_rates
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R8(X) X X X X X X X X
#define R64(X) R8(R8(X))

/* one step of all 8 chains: OP is an asm template over %0..%7 (chains), %8 (vgpr operand), %9 (sgpr) */
#define CHAIN8(OP)                                                                                                     \
    OP(0) OP(1) OP(2) OP(3) OP(4) OP(5) OP(6) OP(7)

#define STR_(x) #x
#define STR(x) STR_(x)

#define OP_XOR(c) "v_xor_b32 %" STR(c) ", %" STR(c) ", %8\n\t"
#define OP_ADD(c) "v_add_u32 %" STR(c) ", %" STR(c) ", %8\n\t"
#define OP_PERM_S(c) "v_perm_b32 %" STR(c) ", %" STR(c) ", %8, %9\n\t"
#define OP_PERM_V(c) "v_perm_b32 %" STR(c) ", %" STR(c) ", %8, %10\n\t"
#define OP_B3_S(c) "v_bitop3_b32 %" STR(c) ", %" STR(c) ", %8, %9 bitop3:0x96\n\t"
#define OP_B3_V(c) "v_bitop3_b32 %" STR(c) ", %" STR(c) ", %8, %10 bitop3:0x96\n\t"
#define OP_SDWA_MOV(c) "v_mov_b32_sdwa %" STR(c) ", %8 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2\n\t"
#define OP_SDWA_OR(c) "v_or_b32_sdwa %" STR(c) ", %" STR(c) ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2\n\t"
#define OP_SDWA_SHL(c) "v_lshlrev_b32_sdwa %" STR(c) ", 8, %" STR(c) " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2\n\t"
#define OP_ANDOR(c) "v_and_or_b32 %" STR(c) ", %" STR(c) ", %9, %8\n\t"
#define OP_LSHLOR(c) "v_lshl_or_b32 %" STR(c) ", %" STR(c) ", 8, %8\n\t"
#define OP_BFI(c) "v_bfi_b32 %" STR(c) ", %9, %" STR(c) ", %8\n\t"
#define OP_BFE(c) "v_bfe_u32 %" STR(c) ", %" STR(c) ", 8, 8\n\t"
#define OP_ALIGN(c) "v_alignbit_b32 %" STR(c) ", %" STR(c) ", %" STR(c) ", 16\n\t"
#define OP_DPP(c) "v_xor_b32_dpp %" STR(c) ", %" STR(c) ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define OP_CND(c) "v_cndmask_b32 %" STR(c) ", %" STR(c) ", %8, vcc\n\t"
#define OP_MAD24(c) "v_mad_u32_u24 %" STR(c) ", %" STR(c) ", %8, %10\n\t"
#define OP_LSHR(c) "v_lshrrev_b32 %" STR(c) ", 8, %" STR(c) "\n\t"
#define OP_XAD(c) "v_xad_u32 %" STR(c) ", %" STR(c) ", %8, %10\n\t"
#define OP_PK_MOV(c) "v_pk_mov_b32 v[%" STR(c) ":%" STR(c) "+1], v[%" STR(c) ":%" STR(c) "+1], v[%" STR(c) ":%" STR(c) "+1] op_sel:[0,1]\n\t"
#define OP_BITOP3_2(c) "v_bitop3_b32 %" STR(c) ", %" STR(c) ", %8, %8 bitop3:0x3c\n\t"
#define OP_OR3(c) "v_or3_b32 %" STR(c) ", %" STR(c) ", %8, %10\n\t"
#define OP_LSHLADD(c) "v_lshl_add_u32 %" STR(c) ", %" STR(c) ", 8, %8\n\t"

#define KERNEL(NAME, OP)                                                                                               \
    extern "C" __global__ __launch_bounds__(1024) void NAME(uint32_t iters, uint32_t *out, uint32_t sk)              \
    {                                                                                                                  \
        uint32_t x0 = threadIdx.x, x1 = x0 * 3u, x2 = x0 * 5u, x3 = x0 * 7u, x4 = x0 * 11u, x5 = x0 * 13u,          \
                 x6 = x0 * 17u, x7 = x0 * 19u;                                                                         \
        uint32_t y = threadIdx.x * 0x9e3779b9u, z = threadIdx.x ^ 0x0c020100u;                                       \
        for (uint32_t it = 0; it < iters; ++it) {                                                                      \
            asm volatile(R64(CHAIN8(OP))                                                                               \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)            \
                         : "v"(y), "s"(sk), "v"(z)                                                                     \
                         : "vcc");                                                                                     \
        }                                                                                                              \
        out[blockIdx.x * blockDim.x + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                            \
    }

KERNEL(k_xor, OP_XOR)
KERNEL(k_add, OP_ADD)
KERNEL(k_perm_s, OP_PERM_S)
KERNEL(k_perm_v, OP_PERM_V)
KERNEL(k_b3_s, OP_B3_S)
KERNEL(k_b3_v, OP_B3_V)
KERNEL(k_sdwa_mov, OP_SDWA_MOV)
KERNEL(k_sdwa_or, OP_SDWA_OR)
KERNEL(k_sdwa_shl, OP_SDWA_SHL)
KERNEL(k_andor, OP_ANDOR)
KERNEL(k_lshlor, OP_LSHLOR)
KERNEL(k_bfi, OP_BFI)
KERNEL(k_bfe, OP_BFE)
KERNEL(k_align, OP_ALIGN)
KERNEL(k_dpp, OP_DPP)
KERNEL(k_cnd, OP_CND)
KERNEL(k_mad24, OP_MAD24)
KERNEL(k_lshr, OP_LSHR)
KERNEL(k_xad, OP_XAD)
KERNEL(k_b3_2, OP_BITOP3_2)
KERNEL(k_or3, OP_OR3)
KERNEL(k_lshladd, OP_LSHLADD)


/* explicit registers (clobbered), 8 chains v40..v47 and sources v48.., to see VGPR-bank effects (bank = reg % 4) */
#define XR(NAME, BODY8)                                                                                                \
    extern "C" __global__ __launch_bounds__(1024) void NAME(uint32_t iters, uint32_t *out, uint32_t sk)              \
    {                                                                                                                  \
        uint32_t r = 0;                                                                                                \
        asm volatile("v_mov_b32 v40, %0\n v_mov_b32 v41, %0\n v_mov_b32 v42, %0\n v_mov_b32 v43, %0\n"                \
                     "v_mov_b32 v44, %0\n v_mov_b32 v45, %0\n v_mov_b32 v46, %0\n v_mov_b32 v47, %0\n"                \
                     "v_mov_b32 v48, %0\n v_mov_b32 v49, %0\n v_mov_b32 v50, %0\n v_mov_b32 v51, %0\n"                \
                     "v_mov_b32 v52, %0\n v_mov_b32 v53, %0\n v_mov_b32 v54, %0\n v_mov_b32 v55, %0\n"                \
                     :: "v"(threadIdx.x) : "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55"); \
        for (uint32_t it = 0; it < iters; ++it)                                                                        \
            asm volatile(R64(BODY8) ::: "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55"); \
        asm volatile("v_mov_b32 %0, v40" : "=v"(r));                                                                  \
        out[blockIdx.x * blockDim.x + threadIdx.x] = r;                                                                \
    }
/* chains v40..v47 (banks 0..3,0..3); sources chosen per variant */
#define B3_DISTINCT "v_bitop3_b32 v40, v40, v49, v50 bitop3:0x96\n v_bitop3_b32 v41, v41, v50, v51 bitop3:0x96\n" \
                    "v_bitop3_b32 v42, v42, v51, v48 bitop3:0x96\n v_bitop3_b32 v43, v43, v48, v49 bitop3:0x96\n" \
                    "v_bitop3_b32 v44, v44, v49, v50 bitop3:0x96\n v_bitop3_b32 v45, v45, v50, v51 bitop3:0x96\n" \
                    "v_bitop3_b32 v46, v46, v51, v48 bitop3:0x96\n v_bitop3_b32 v47, v47, v48, v49 bitop3:0x96\n"
#define B3_SAMEBANK "v_bitop3_b32 v40, v40, v48, v52 bitop3:0x96\n v_bitop3_b32 v41, v41, v49, v53 bitop3:0x96\n" \
                    "v_bitop3_b32 v42, v42, v50, v54 bitop3:0x96\n v_bitop3_b32 v43, v43, v51, v55 bitop3:0x96\n" \
                    "v_bitop3_b32 v44, v44, v48, v52 bitop3:0x96\n v_bitop3_b32 v45, v45, v49, v53 bitop3:0x96\n" \
                    "v_bitop3_b32 v46, v46, v50, v54 bitop3:0x96\n v_bitop3_b32 v47, v47, v51, v55 bitop3:0x96\n"
#define B3_CONST    "v_bitop3_b32 v40, v40, v49, s0 bitop3:0x96\n v_bitop3_b32 v41, v41, v50, s0 bitop3:0x96\n" \
                    "v_bitop3_b32 v42, v42, v51, s0 bitop3:0x96\n v_bitop3_b32 v43, v43, v48, s0 bitop3:0x96\n" \
                    "v_bitop3_b32 v44, v44, v49, s0 bitop3:0x96\n v_bitop3_b32 v45, v45, v50, s0 bitop3:0x96\n" \
                    "v_bitop3_b32 v46, v46, v51, s0 bitop3:0x96\n v_bitop3_b32 v47, v47, v48, s0 bitop3:0x96\n"
#define B3_INL      "v_bitop3_b32 v40, v40, v49, 7 bitop3:0x96\n v_bitop3_b32 v41, v41, v50, 7 bitop3:0x96\n" \
                    "v_bitop3_b32 v42, v42, v51, 7 bitop3:0x96\n v_bitop3_b32 v43, v43, v48, 7 bitop3:0x96\n" \
                    "v_bitop3_b32 v44, v44, v49, 7 bitop3:0x96\n v_bitop3_b32 v45, v45, v50, 7 bitop3:0x96\n" \
                    "v_bitop3_b32 v46, v46, v51, 7 bitop3:0x96\n v_bitop3_b32 v47, v47, v48, 7 bitop3:0x96\n"
#define PERM_DISTINCT "v_perm_b32 v40, v40, v49, v50\n v_perm_b32 v41, v41, v50, v51\n" \
                    "v_perm_b32 v42, v42, v51, v48\n v_perm_b32 v43, v43, v48, v49\n" \
                    "v_perm_b32 v44, v44, v49, v50\n v_perm_b32 v45, v45, v50, v51\n" \
                    "v_perm_b32 v46, v46, v51, v48\n v_perm_b32 v47, v47, v48, v49\n"
#define XOR_SAMEBANK "v_xor_b32 v40, v40, v48\n v_xor_b32 v41, v41, v49\n v_xor_b32 v42, v42, v50\n v_xor_b32 v43, v43, v51\n" \
                    "v_xor_b32 v44, v44, v48\n v_xor_b32 v45, v45, v49\n v_xor_b32 v46, v46, v50\n v_xor_b32 v47, v47, v51\n"
#define XOR_SGPR    "v_xor_b32 v40, s0, v40\n v_xor_b32 v41, s0, v41\n v_xor_b32 v42, s0, v42\n v_xor_b32 v43, s0, v43\n" \
                    "v_xor_b32 v44, s0, v44\n v_xor_b32 v45, s0, v45\n v_xor_b32 v46, s0, v46\n v_xor_b32 v47, s0, v47\n"
#define AND_OR_DISTINCT "v_and_or_b32 v40, v40, v49, v50\n v_and_or_b32 v41, v41, v50, v51\n" \
                    "v_and_or_b32 v42, v42, v51, v48\n v_and_or_b32 v43, v43, v48, v49\n" \
                    "v_and_or_b32 v44, v44, v49, v50\n v_and_or_b32 v45, v45, v50, v51\n" \
                    "v_and_or_b32 v46, v46, v51, v48\n v_and_or_b32 v47, v47, v48, v49\n"
#define LSHR_ONLY   "v_lshrrev_b32 v40, 8, v49\n v_lshrrev_b32 v41, 8, v50\n v_lshrrev_b32 v42, 8, v51\n v_lshrrev_b32 v43, 8, v48\n" \
                    "v_lshrrev_b32 v44, 8, v49\n v_lshrrev_b32 v45, 8, v50\n v_lshrrev_b32 v46, 8, v51\n v_lshrrev_b32 v47, 8, v48\n"
XR(x_b3_distinct, B3_DISTINCT)
XR(x_b3_samebank, B3_SAMEBANK)
XR(x_b3_const, B3_CONST)
XR(x_b3_inl, B3_INL)
XR(x_perm_distinct, PERM_DISTINCT)
XR(x_xor_samebank, XOR_SAMEBANK)
XR(x_xor_sgpr, XOR_SGPR)
XR(x_andor_distinct, AND_OR_DISTINCT)
XR(x_lshr, LSHR_ONLY)

typedef void (*kfn)(uint32_t, uint32_t *, uint32_t);
struct Var {
    const char *name;
    kfn k;
};

int main()
{
    const Var vars[] = {{"v_xor_b32 (VOP2)", k_xor},
                        {"v_add_u32 (VOP2)", k_add},
                        {"v_perm_b32 v,v,s", k_perm_s},
                        {"v_perm_b32 v,v,v", k_perm_v},
                        {"v_bitop3_b32 v,v,s", k_b3_s},
                        {"v_bitop3_b32 v,v,v", k_b3_v},
                        {"v_bitop3_b32 v,v,v(same)", k_b3_2},
                        {"v_mov_b32_sdwa preserve", k_sdwa_mov},
                        {"v_or_b32_sdwa byte", k_sdwa_or},
                        {"v_lshlrev_b32_sdwa byte", k_sdwa_shl},
                        {"v_and_or_b32 v,s,v", k_andor},
                        {"v_lshl_or_b32 v,8,v", k_lshlor},
                        {"v_lshl_add_u32 v,8,v", k_lshladd},
                        {"v_or3_b32 v,v,v", k_or3},
                        {"v_bfi_b32 s,v,v", k_bfi},
                        {"v_bfe_u32 v,8,8", k_bfe},
                        {"v_alignbit_b32 rot16", k_align},
                        {"v_xor_b32_dpp quad_perm", k_dpp},
                        {"v_cndmask_b32 vcc", k_cnd},
                        {"v_mad_u32_u24 v,v,v", k_mad24},
                        {"v_lshrrev_b32 (VOP2)", k_lshr},
                        {"v_xad_u32 v,v,v", k_xad},
                        {"x: v_bitop3 3 distinct VGPR banks", x_b3_distinct},
                        {"x: v_bitop3 3 VGPRs one bank", x_b3_samebank},
                        {"x: v_bitop3 v,v,s0", x_b3_const},
                        {"x: v_bitop3 v,v,inline const", x_b3_inl},
                        {"x: v_perm 3 distinct VGPR banks", x_perm_distinct},
                        {"x: v_xor_b32 2 VGPRs one bank", x_xor_samebank},
                        {"x: v_xor_b32 s,v (VOP2 SGPR)", x_xor_sgpr},
                        {"x: v_and_or_b32 3 distinct banks", x_andor_distinct},
                        {"x: v_lshrrev_b32 (no dependency)", x_lshr}};
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    uint32_t *out = nullptr;
    if (hipMalloc(&out, (size_t)ncu * 1024 * 4) != hipSuccess)
        return 1;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const uint32_t iters = 1024;
    double ref = 0;
    printf("{\"what\": \"scripts/isa_rates.hip: 8x64 instructions per trip over 8 chains, 16 waves/CU, %d CUs\", \"rows\": [\n", ncu);
    for (size_t v = 0; v < sizeof(vars) / sizeof(vars[0]); ++v) {
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(vars[v].k, dim3(ncu), dim3(1024), 0, 0, iters, out, 0x0c020100u);
            hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess)
                return 2;
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best)
                best = ms;
        }
        /* wave-instructions per SIMD: 4 waves per SIMD x iters x 512 */
        const double per_simd = 4.0 * iters * 512.0;
        const double ns = best * 1e6 / per_simd;
        if (v == 0)
            ref = ns;
        printf("  {\"op\": \"%s\", \"ms\": %.3f, \"ns_per_wave_instr_per_simd\": %.4f, \"clk_rel_vop2x2\": %.2f}%s\n",
               vars[v].name, best, ns, 2.0 * ns / ref, v + 1 < sizeof(vars) / sizeof(vars[0]) ? "," : "");
        fflush(stdout);
    }
    printf("]}\n");
    return 0;
}
