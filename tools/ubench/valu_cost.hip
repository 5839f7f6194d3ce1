// valu_cost.hip -- issue cost of single VALU opcodes on a saturated SIMD, in MFMA-calibrated
// cycles: one 256*W-thread block per CU (W waves per SIMD), every wave runs 16 independent
// chains of the opcode; the clock is calibrated by v_mfma_f32_32x32x16_f16 (32 cycles per
// instruction per SIMD at the dense f16 peak) and v_mfma_i32_32x32x32_i8 is reported beside it.
// Companion of mfma_split.hip (which shows MFMA and VALU cycles ADD on a SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 1024
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v2f __attribute__((ext_vector_type(2)));

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define OUTS16 "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]), \
               "+v"(f[8]), "+v"(f[9]), "+v"(f[10]), "+v"(f[11]), "+v"(f[12]), "+v"(f[13]), "+v"(f[14]), "+v"(f[15])
#define OUTS8P "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), "+v"(g[6]), "+v"(g[7])

#define I_FMA(i) "v_fma_f32 %" #i ", %" #i ", %16, %17\n\t"
#define I_FMAC(i) "v_fmac_f32 %" #i ", %16, %17\n\t"
#define I_ADD(i) "v_add_f32 %" #i ", %" #i ", %16\n\t"
#define I_MUL(i) "v_mul_f32 %" #i ", %" #i ", %16\n\t"
#define I_EXP(i) "v_exp_f32 %" #i ", %" #i "\n\t"
#define I_MAX(i) "v_max_f32 %" #i ", %" #i ", %16\n\t"
#define I_MAX3(i) "v_max3_f32 %" #i ", %" #i ", %16, %17\n\t"
#define I_MAXI(i) "v_max_i32 %" #i ", %" #i ", %16\n\t"
#define I_PERM(i) "v_perm_b32 %" #i ", %" #i ", %16, %17\n\t"
#define I_CVT(i) "v_cvt_f32_i32 %" #i ", %" #i "\n\t"
#define I_MOV(i) "v_mov_b32 %" #i ", %16\n\t"
#define I_FMAAK(i) "v_fmaak_f32 %" #i ", %" #i ", %16, 0x4b400000\n\t"
#define I_DPP(i) "v_max_i32_dpp %" #i ", %" #i ", %16 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
#define I_PL(i) "v_permlane32_swap_b32 %" #i ", %16\n\t"
#define I_SUB(i) "v_sub_f32 %" #i ", %" #i ", %16\n\t"
#define I_ADDU(i) "v_add_u32 %" #i ", %" #i ", %16\n\t"
#define I_FMAS(i) "v_fma_f32 %" #i ", %" #i ", %16, %18\n\t"
#define I_CVTPK(i) "v_cvt_pk_f16_f32 %" #i ", %" #i ", %16\n\t"
#define I_RCP(i) "v_rcp_f32 %" #i ", %" #i "\n\t"
#define I_MAX3I(i) "v_max3_i32 %" #i ", %" #i ", %16, %17\n\t"
#define I_MULS(i) "v_mul_f32 %" #i ", %18, %" #i "\n\t"
#define I_FMACS(i) "v_fmac_f32 %" #i ", %18, %16\n\t"
#define I_ADDS(i) "v_add_f32 %" #i ", %18, %" #i "\n\t"
#define I_CMPS(i) "v_cmp_lt_f32 vcc, %18, %" #i "\n\t"
#define I_CMPV(i) "v_cmp_lt_f32 vcc, %16, %" #i "\n\t"
#define I_FMA_MIX(i) "v_fma_mix_f32 %" #i ", %" #i ", %16, %17\n\t"
// r04: ways to pack the low 16 bits of two registers (the int8 kernel's f16-subnormal P operand pairs)
#define I_SDWA(i) "v_mov_b32_sdwa %" #i ", %16 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0\n\t"
#define I_PACKF16(i) "v_pack_b32_f16 %" #i ", %" #i ", %16\n\t"
#define I_LSHLOR(i) "v_lshl_or_b32 %" #i ", %16, 16, %" #i "\n\t"
#define I_BFI(i) "v_bfi_b32 %" #i ", %17, %" #i ", %16\n\t"
#define I_ADDSDWA(i) "v_add_f32_sdwa %" #i ", %" #i ", %16 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD\n\t"

#define P8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define I_PKFMA(i) "v_pk_fma_f32 %" #i ", %" #i ", %8, %9\n\t"
#define I_PKFMAB(i) "v_pk_fma_f32 %" #i ", %" #i ", %8, %9 op_sel_hi:[1,0,0]\n\t"
#define I_PKADD(i) "v_pk_add_f32 %" #i ", %" #i ", %8\n\t"
#define I_PKMUL(i) "v_pk_mul_f32 %" #i ", %" #i ", %8\n\t"
#define I_PKMOV(i) "v_pk_mov_b32 %" #i ", %8, %9 op_sel:[0,1]\n\t"

enum {
    OP_FMA, OP_FMAC, OP_ADD, OP_MUL, OP_EXP, OP_MAX, OP_MAX3, OP_MAXI, OP_PERM, OP_CVT, OP_MOV, OP_FMAAK, OP_DPP, OP_PL,
    OP_SUB, OP_ADDU, OP_FMAS, OP_CVTPK, OP_RCP, OP_MAX3I, OP_FMAMIX, OP_PKFMA, OP_PKFMAB, OP_PKADD, OP_PKMUL, OP_PKMOV,
    OP_MULS, OP_FMACS, OP_ADDS, OP_CMPS, OP_CMPV, OP_SDWA, OP_PACKF16, OP_LSHLOR, OP_BFI, OP_ADDSDWA, OP_MFMA16, OP_MFMA8,
    OP_N
};
static const char* kNames[OP_N] = {
    "v_fma_f32", "v_fmac_f32", "v_add_f32", "v_mul_f32", "v_exp_f32", "v_max_f32", "v_max3_f32", "v_max_i32",
    "v_perm_b32", "v_cvt_f32_i32", "v_mov_b32", "v_fmaak_f32", "v_max_i32_dpp", "v_permlane32_swap", "v_sub_f32",
    "v_add_u32", "v_fma_f32 (sgpr)", "v_cvt_pk_f16_f32", "v_rcp_f32", "v_max3_i32", "v_fma_mix_f32", "v_pk_fma_f32",
    "v_pk_fma_f32 bcast", "v_pk_add_f32", "v_pk_mul_f32", "v_pk_mov_b32", "v_mul_f32 (sgpr, vop2)",
    "v_fmac_f32 (sgpr, vop2)", "v_add_f32 (sgpr, vop2)", "v_cmp_lt_f32 (sgpr)", "v_cmp_lt_f32 (vgpr)",
    "v_mov_b32_sdwa WORD_1", "v_pack_b32_f16", "v_lshl_or_b32", "v_bfi_b32", "v_add_f32_sdwa",
    "mfma_f32_32x32x16_f16", "mfma_i32_32x32x32_i8"};

template <int OP>
__device__ float body(float seed, float sx) {
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = seed + j;
    v2f g[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = v2f{seed + j, seed - j};
    const float x = seed * 0.5f, y = seed * 0.25f;
    const v2f px = {x, y}, py = {y, x};
    v8h a = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
    v4i ai = {(int)seed, 1, 2, 3};
    v16f c0, c1;
    v16i ci0, ci1;
    for (int it = 0; it < ITERS; ++it) {
#define ASM16(I) asm volatile(R16(I) : OUTS16 : "v"(x), "v"(y), "s"(sx))
#define ASM8P(I) asm volatile(P8(I) : OUTS8P : "v"(px), "v"(py))
        if constexpr (OP == OP_FMA) ASM16(I_FMA);
        if constexpr (OP == OP_FMAC) ASM16(I_FMAC);
        if constexpr (OP == OP_ADD) ASM16(I_ADD);
        if constexpr (OP == OP_MUL) ASM16(I_MUL);
        if constexpr (OP == OP_EXP) ASM16(I_EXP);
        if constexpr (OP == OP_MAX) ASM16(I_MAX);
        if constexpr (OP == OP_MAX3) ASM16(I_MAX3);
        if constexpr (OP == OP_MAXI) ASM16(I_MAXI);
        if constexpr (OP == OP_PERM) ASM16(I_PERM);
        if constexpr (OP == OP_CVT) ASM16(I_CVT);
        if constexpr (OP == OP_MOV) ASM16(I_MOV);
        if constexpr (OP == OP_FMAAK) ASM16(I_FMAAK);
        if constexpr (OP == OP_DPP) ASM16(I_DPP);
        if constexpr (OP == OP_PL) ASM16(I_PL);
        if constexpr (OP == OP_SUB) ASM16(I_SUB);
        if constexpr (OP == OP_ADDU) ASM16(I_ADDU);
        if constexpr (OP == OP_FMAS) ASM16(I_FMAS);
        if constexpr (OP == OP_CVTPK) ASM16(I_CVTPK);
        if constexpr (OP == OP_RCP) ASM16(I_RCP);
        if constexpr (OP == OP_MAX3I) ASM16(I_MAX3I);
        if constexpr (OP == OP_FMAMIX) ASM16(I_FMA_MIX);
        if constexpr (OP == OP_MULS) ASM16(I_MULS);
        if constexpr (OP == OP_FMACS) ASM16(I_FMACS);
        if constexpr (OP == OP_ADDS) ASM16(I_ADDS);
        if constexpr (OP == OP_CMPS) asm volatile(R16(I_CMPS) : OUTS16 : "v"(x), "v"(y), "s"(sx) : "vcc");
        if constexpr (OP == OP_CMPV) asm volatile(R16(I_CMPV) : OUTS16 : "v"(x), "v"(y), "s"(sx) : "vcc");
        if constexpr (OP == OP_SDWA) ASM16(I_SDWA);
        if constexpr (OP == OP_PACKF16) ASM16(I_PACKF16);
        if constexpr (OP == OP_LSHLOR) ASM16(I_LSHLOR);
        if constexpr (OP == OP_BFI) ASM16(I_BFI);
        if constexpr (OP == OP_ADDSDWA) ASM16(I_ADDSDWA);
        if constexpr (OP == OP_PKFMA) { ASM8P(I_PKFMA); ASM8P(I_PKFMA); }
        if constexpr (OP == OP_PKFMAB) { ASM8P(I_PKFMAB); ASM8P(I_PKFMAB); }
        if constexpr (OP == OP_PKADD) { ASM8P(I_PKADD); ASM8P(I_PKADD); }
        if constexpr (OP == OP_PKMUL) { ASM8P(I_PKMUL); ASM8P(I_PKMUL); }
        if constexpr (OP == OP_PKMOV) { ASM8P(I_PKMOV); ASM8P(I_PKMOV); }
        if constexpr (OP == OP_MFMA16)
#pragma unroll
            for (int u = 0; u < 8; ++u)
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %2, 0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %2, 0"
                             : "=a"(c0), "=a"(c1) : "v"(a));
        if constexpr (OP == OP_MFMA8)
#pragma unroll
            for (int u = 0; u < 8; ++u)
                asm volatile("v_mfma_i32_32x32x32_i8 %0, %2, %2, 0\n\tv_mfma_i32_32x32x32_i8 %1, %2, %2, 0"
                             : "=a"(ci0), "=a"(ci1) : "v"(ai));
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    float s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += f[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += g[j].x + g[j].y;
    if constexpr (OP == OP_MFMA16) {
        float r;
        asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(c0[0]));
        s += r;
    }
    if constexpr (OP == OP_MFMA8) {
        int r;
        asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(ci0[0]));
        s += r;
    }
    return s;
}

template <int OP>
__global__ __launch_bounds__(1024) void k(float* out, float seed, float sx) {
    out[blockIdx.x * blockDim.x + threadIdx.x] = body<OP>(seed, sx);
}

template <int OP>
float run(int W) {  // ns per instruction per SIMD
    const int blocks = 256, threads = 256 * W;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    hipLaunchKernelGGL((k<OP>), dim3(blocks), dim3(threads), 0, 0, out, 1.0f, 0.5f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<OP>), dim3(blocks), dim3(threads), 0, 0, out, 1.0f, 0.5f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5 * 1e6f / (ITERS * 16.0f * W);
}

template <int OP>
void row(float ns_per_cycle) {
    const float t2 = run<OP>(2), t4 = run<OP>(4);
    std::printf("%-24s  W2 %6.2f cyc   W4 %6.2f cyc   (%.3f / %.3f ns)\n", kNames[OP], t2 / ns_per_cycle,
                t4 / ns_per_cycle, t2, t4);
}

template <int... OPS>
void rows(float c, std::integer_sequence<int, OPS...>) {
    (row<OPS>(c), ...);
}

int main() {
    const float mf = run<OP_MFMA16>(4);
    const float c = mf / 32.0f;  // ns per cycle: the f16 32x32x16 MFMA issues every 32 cycles
    std::printf("calibration: mfma_f32_32x32x16_f16 %.3f ns per instruction per SIMD = 32 cycles -> %.3f GHz\n", mf,
                1.0f / c);
    rows(c, std::make_integer_sequence<int, OP_N>{});
    return 0;
}
