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

__device__ float valu_wave(float seed, int groups) {
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = seed + j;
    const float x = seed * 0.5f, y = seed * 0.25f;
    for (int i = 0; i < groups; ++i)
        asm volatile(F16C : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]),
                     "+v"(f[8]), "+v"(f[9]), "+v"(f[10]), "+v"(f[11]), "+v"(f[12]), "+v"(f[13]), "+v"(f[14]), "+v"(f[15])
                     : "v"(x), "v"(y));
    float s = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) s += f[j];
    return s;
}

template <int FORM>
__global__ __launch_bounds__(1024) void k(float* out, float seed, int m_waves, int valu_groups) {
    const int wave = threadIdx.x >> 6;
    float r;
    if (wave < 4 * m_waves)
        r = mfma_wave<FORM>(seed);
    else
        r = valu_wave(seed, valu_groups);
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <int FORM>
float run(int M, int V, int NV) {
    const int blocks = 256;
    const int threads = 256 * (M + V);
    if (threads == 0) return 0.0f;
    // total fmas per SIMD = ITERS * 4 * NV, split over V waves, in groups of 16
    const int groups = V ? ITERS * 4 * NV / (16 * V) : 0;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    hipLaunchKernelGGL((k<FORM>), dim3(blocks), dim3(threads), 0, 0, out, 1.0f, M, groups);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<FORM>), dim3(blocks), dim3(threads), 0, 0, out, 1.0f, M, groups);
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
    return 0;
}
