// mfma_own.hip -- does a wave's OWN independent VALU overlap its MFMAs, per accumulator form?
// Each wave loops { MFMA 32x32x16 f16 ; NV independent v_fma_f32 (8 chains) } with W waves per
// SIMD (block = 256*W threads, one block per CU).  Forms:
//   0 VGPR C/D accumulate in place     1 AGPR C/D accumulate in place
//   2 VGPR D, C = 0 (no accumulate)    3 AGPR D, C = 0
//   4 AGPR accumulate + 8 v_accvgpr_read of a DIFFERENT (finished) AGPR block per MFMA
// Prints ns per MFMA per SIMD (wall); 32 cycles at the clock is the MFMA floor.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define F8 "v_fma_f32 %0, %0, %8, %9\n\tv_fma_f32 %1, %1, %8, %9\n\tv_fma_f32 %2, %2, %8, %9\n\tv_fma_f32 %3, %3, %8, %9\n\t" \
           "v_fma_f32 %4, %4, %8, %9\n\tv_fma_f32 %5, %5, %8, %9\n\tv_fma_f32 %6, %6, %8, %9\n\tv_fma_f32 %7, %7, %8, %9\n\t"

template <int FORM, int NV>
__device__ float body(float seed) {
    v8h a = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
    v16f c = {}, c2 = {};
    float f0 = seed, f1 = seed + 1, f2 = seed + 2, f3 = seed + 3, f4 = seed + 4, f5 = seed + 5, f6 = seed + 6,
          f7 = seed + 7, x = seed * 0.5f, y = seed * 0.25f;
    if constexpr (FORM == 4) asm volatile("" : "+a"(c2));
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (FORM == 0)
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, %0" : "+v"(c) : "v"(a));
            else if constexpr (FORM == 1 || FORM == 4)
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, %0" : "+a"(c) : "v"(a));
            else if constexpr (FORM == 2)
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, 0" : "=v"(c) : "v"(a));
            else
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, 0" : "=a"(c) : "v"(a));
            if constexpr (FORM == 4) {
                float r0, r1, r2, r3, r4, r5, r6, r7;
                asm volatile("v_accvgpr_read_b32 %0, %8\n\tv_accvgpr_read_b32 %1, %9\n\tv_accvgpr_read_b32 %2, %10\n\t"
                             "v_accvgpr_read_b32 %3, %11\n\tv_accvgpr_read_b32 %4, %12\n\tv_accvgpr_read_b32 %5, %13\n\t"
                             "v_accvgpr_read_b32 %6, %14\n\tv_accvgpr_read_b32 %7, %15"
                             : "=v"(r0), "=v"(r1), "=v"(r2), "=v"(r3), "=v"(r4), "=v"(r5), "=v"(r6), "=v"(r7)
                             : "a"(c2[0]), "a"(c2[1]), "a"(c2[2]), "a"(c2[3]), "a"(c2[4]), "a"(c2[5]), "a"(c2[6]),
                               "a"(c2[7]));
                f0 += r0; f1 += r1; f2 += r2; f3 += r3; f4 += r4; f5 += r5; f6 += r6; f7 += r7;
            }
#pragma unroll
            for (int v = 0; v < NV / 8; ++v)
                asm volatile(F8 : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
                             : "v"(x), "v"(y));
        }
    }
    return c[0] + c[15] + f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
}

template <int FORM, int NV, int W>
__global__ __launch_bounds__(256 * W) void k(float* out, float seed) {
    out[blockIdx.x * 256 * W + threadIdx.x] = body<FORM, NV>(seed);
}

template <int FORM, int NV, int W>
float run() {
    const int blocks = 256;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * W * 4);
    hipLaunchKernelGGL((k<FORM, NV, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<FORM, NV, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5 * 1e6f / (ITERS * 4.0f * W);  // ns per MFMA per SIMD
}

template <int FORM, int W>
void row() {
    std::printf("form %d W %d  NV0 %.2f  NV8 %.2f  NV16 %.2f  NV24 %.2f  NV32 %.2f  NV48 %.2f ns/MFMA\n", FORM, W,
                run<FORM, 0, W>(), run<FORM, 8, W>(), run<FORM, 16, W>(), run<FORM, 24, W>(), run<FORM, 32, W>(),
                run<FORM, 48, W>());
}

int main() {
    row<0, 1>(); row<1, 1>(); row<2, 1>(); row<3, 1>(); row<4, 1>();
    row<0, 2>(); row<1, 2>(); row<2, 2>(); row<3, 2>(); row<4, 2>();
    row<0, 3>(); row<1, 3>(); row<2, 3>(); row<3, 3>();
    return 0;
}
