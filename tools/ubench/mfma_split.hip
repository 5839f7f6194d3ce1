// mfma_split.hip -- can the matrix core and the VALU of one SIMD execute at the same time?
// One block per CU of 256*(M+V) threads: waves 0..4M-1 (M per SIMD) issue only independent
// MFMAs (AGPR or VGPR destination, C = 0), the other 4V waves (V per SIMD) issue only v_fma_f32
// (16 independent chains, so a wave is never latency-bound).  Each MFMA wave issues ITERS*4
// MFMAs, each VALU wave ITERS*4*NV/V fmas, so the totals per SIMD are fixed as V varies.
// Serialised execution:  t(both) = t(mfma alone) + t(valu alone);  overlapped: the max.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define F16C "v_fma_f32 %0, %0, %16, %17\n\tv_fma_f32 %1, %1, %16, %17\n\tv_fma_f32 %2, %2, %16, %17\n\tv_fma_f32 %3, %3, %16, %17\n\t" \
             "v_fma_f32 %4, %4, %16, %17\n\tv_fma_f32 %5, %5, %16, %17\n\tv_fma_f32 %6, %6, %16, %17\n\tv_fma_f32 %7, %7, %16, %17\n\t" \
             "v_fma_f32 %8, %8, %16, %17\n\tv_fma_f32 %9, %9, %16, %17\n\tv_fma_f32 %10, %10, %16, %17\n\tv_fma_f32 %11, %11, %16, %17\n\t" \
             "v_fma_f32 %12, %12, %16, %17\n\tv_fma_f32 %13, %13, %16, %17\n\tv_fma_f32 %14, %14, %16, %17\n\tv_fma_f32 %15, %15, %16, %17"

// FORM 0: MFMA D in AGPRs, 1: D in arch VGPRs, 2: D and the A/B operands all in AGPRs
// (no arch-VGPR port touched by the MFMA wave at all)
template <int FORM>
__device__ float mfma_wave(float seed) {
    v8h a = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
    v16f c0, c1;
    if constexpr (FORM == 2) asm volatile("" : "+a"(a));
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (FORM == 2)
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %2, 0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %2, 0\n\t"
                         "v_mfma_f32_32x32x16_f16 %0, %2, %2, 0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %2, 0"
                         : "=a"(c0), "=a"(c1) : "a"(a));
        else if constexpr (FORM == 0)
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %2, 0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %2, 0\n\t"
                         "v_mfma_f32_32x32x16_f16 %0, %2, %2, 0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %2, 0"
                         : "=a"(c0), "=a"(c1) : "v"(a));
        else
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %2, %2, 0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %2, 0\n\t"
                         "v_mfma_f32_32x32x16_f16 %0, %2, %2, 0\n\tv_mfma_f32_32x32x16_f16 %1, %2, %2, 0"
                         : "=v"(c0), "=v"(c1) : "v"(a));
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    float r0, r1;
    if constexpr (FORM != 1) {
        asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r0) : "a"(c0[0]));
        asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r1) : "a"(c1[0]));
    } else {
        r0 = c0[0];
        r1 = c1[0];
    }
    return r0 + r1;
}

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define I_EXP(i) "v_exp_f32 %" #i ", %" #i "\n\t"
#define I_ADD(i) "v_add_f32 %" #i ", %" #i ", %16\n\t"
#define I_MAX3(i) "v_max3_i32 %" #i ", %" #i ", %16, %17\n\t"
#define I_PERM(i) "v_perm_b32 %" #i ", %" #i ", %16, %17\n\t"
#define I_DPP(i) "v_max_i32_dpp %" #i ", %" #i ", %16 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
#define OUTS16 "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]), \
               "+v"(f[8]), "+v"(f[9]), "+v"(f[10]), "+v"(f[11]), "+v"(f[12]), "+v"(f[13]), "+v"(f[14]), "+v"(f[15])
// VOP: 0 v_fma_f32, 1 v_exp_f32, 2 v_add_f32, 3 v_max3_i32, 4 v_perm_b32, 5 v_max_i32_dpp
template <int VOP>
__device__ float valu_wave(float seed, int groups) {
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = seed + j;
    const float x = seed * 0.5f, y = seed * 0.25f;
    for (int i = 0; i < groups; ++i) {
        if constexpr (VOP == 0) asm volatile(F16C : OUTS16 : "v"(x), "v"(y));
        if constexpr (VOP == 1) asm volatile(R16(I_EXP) : OUTS16 : "v"(x), "v"(y));
        if constexpr (VOP == 2) asm volatile(R16(I_ADD) : OUTS16 : "v"(x), "v"(y));
        if constexpr (VOP == 3) asm volatile(R16(I_MAX3) : OUTS16 : "v"(x), "v"(y));
        if constexpr (VOP == 4) asm volatile(R16(I_PERM) : OUTS16 : "v"(x), "v"(y));
        if constexpr (VOP == 5) asm volatile(R16(I_DPP) : OUTS16 : "v"(x), "v"(y));
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += f[j];
    return s;
}

template <int FORM, int VOP = 0>
__global__ __launch_bounds__(1024) void k(float* out, float seed, int m_waves, int valu_groups) {
    const int wave = threadIdx.x >> 6;
    float r;
    if (wave < 4 * m_waves)
        r = mfma_wave<FORM>(seed);
    else
        r = valu_wave<VOP>(seed, valu_groups);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int FORM, int VOP = 0>
float run(int M, int V, int NV) {
    const int blocks = 256;
    const int threads = 256 * (M + V);
    if (threads == 0) return 0.0f;
    // total fmas per SIMD = ITERS * 4 * NV, split over V waves, in groups of 16
    const int groups = V ? ITERS * 4 * NV / (16 * V) : 0;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    hipLaunchKernelGGL((k<FORM, VOP>), dim3(blocks), dim3(threads), 0, 0, out, 1.0f, M, groups);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<FORM, VOP>), dim3(blocks), dim3(threads), 0, 0, out, 1.0f, M, groups);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5 * 1e6f / (ITERS * 4.0f);  // ns per MFMA-slot per SIMD
}

int main() {
    std::printf("ns per slot per SIMD (slot = 1 MFMA 32x32x16 f16 on the MFMA wave + NV v_fma_f32 spread over V VALU waves)\n");
    auto R = [](int form, int M, int V, int NV) {
        return form == 0 ? run<0>(M, V, NV) : form == 1 ? run<1>(M, V, NV) : run<2>(M, V, NV);
    };
    const char* fname[3] = {"agpr", "vgpr", "all-agpr"};
    for (int form = 0; form < 3; ++form)
        for (int NV : {8, 16, 32}) {
            for (int V : {1, 2, 3}) {
                const float tm = R(form, 1, 0, NV), tv = R(form, 0, V, NV), tb = R(form, 1, V, NV);
                std::printf("%s NV%-2d V%d  mfma %.2f  valu %.2f  both %.2f   (sum %.2f, max %.2f)\n",
                            fname[form], NV, V, tm, tv, tb, tm + tv, tm > tv ? tm : tv);
            }
        }
    // other VALU opcodes beside AGPR-form MFMAs (3 VALU waves per SIMD, 16 opcodes per MFMA)
    const char* vname[6] = {"v_fma_f32", "v_exp_f32", "v_add_f32", "v_max3_i32", "v_perm_b32", "v_max_i32_dpp"};
    auto RV = [](int vop, int M, int V, int NV) {
        switch (vop) {
            case 1: return run<0, 1>(M, V, NV);
            case 2: return run<0, 2>(M, V, NV);
            case 3: return run<0, 3>(M, V, NV);
            case 4: return run<0, 4>(M, V, NV);
            case 5: return run<0, 5>(M, V, NV);
            default: return run<0, 0>(M, V, NV);
        }
    };
    for (int vop = 0; vop < 6; ++vop) {
        const float tm = RV(vop, 1, 0, 16), tv = RV(vop, 0, 3, 16), tb = RV(vop, 1, 3, 16);
        std::printf("agpr + %-14s NV16 V3  mfma %.2f  valu %.2f  both %.2f   (sum %.2f, max %.2f)\n", vname[vop], tm, tv,
                    tb, tm + tv, tm > tv ? tm : tv);
    }
    return 0;
}
