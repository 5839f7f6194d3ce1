// mfma_dtype.hip -- does a wave's own independent VALU hide behind its MFMAs, per MFMA opcode?
// Each wave loops { MFMA ; NV independent v_fma_f32 (8 chains) } with W waves per SIMD (block =
// 256*W threads, one block per CU), 4 independent accumulators rotated so consecutive MFMAs do
// not depend on each other.  Prints ns per MFMA per SIMD.  If the MFMA blocked the SIMD's VALU
// for its whole duration, NV fmas add ~NV*2 cycles; if only its issue slot, they are free
// until NV*4 (one wave) exceeds the MFMA's cycles.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 1024
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef __bf16 v8b __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

#define F8 "v_fma_f32 %0, %0, %8, %9\n\tv_fma_f32 %1, %1, %8, %9\n\tv_fma_f32 %2, %2, %8, %9\n\tv_fma_f32 %3, %3, %8, %9\n\t" \
           "v_fma_f32 %4, %4, %8, %9\n\tv_fma_f32 %5, %5, %8, %9\n\tv_fma_f32 %6, %6, %8, %9\n\tv_fma_f32 %7, %7, %8, %9\n\t"
#define F4 "v_fma_f32 %0, %0, %8, %9\n\tv_fma_f32 %1, %1, %8, %9\n\tv_fma_f32 %2, %2, %8, %9\n\tv_fma_f32 %3, %3, %8, %9\n\t"

// OP 0: 32x32x16 f16   1: 32x32x16 bf16   2: 32x32x32 i8   3: 16x16x32 f16
template <int OP, int NV>
__device__ float body(float seed) {
    v8h a = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
    v8b ab;
    for (int i = 0; i < 8; ++i) ab[i] = (__bf16)(seed + i);
    v4i ai = {(int)seed, 1, 2, 3};
    v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
    v16i i0 = {}, i1 = {}, i2 = {}, i3 = {};
    v4f s0 = {}, s1 = {}, s2 = {}, s3 = {};
    float f0 = seed, f1 = seed + 1, f2 = seed + 2, f3 = seed + 3, f4 = seed + 4, f5 = seed + 5, f6 = seed + 6,
          f7 = seed + 7, x = seed * 0.5f, y = seed * 0.25f;
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (OP == 0) {
                v16f& c = u == 0 ? c0 : u == 1 ? c1 : u == 2 ? c2 : c3;
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, %0" : "+v"(c) : "v"(a));
            } else if constexpr (OP == 1) {
                v16f& c = u == 0 ? c0 : u == 1 ? c1 : u == 2 ? c2 : c3;
                asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %1, %0" : "+v"(c) : "v"(ab));
            } else if constexpr (OP == 2) {
                v16i& c = u == 0 ? i0 : u == 1 ? i1 : u == 2 ? i2 : i3;
                asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %1, %0" : "+v"(c) : "v"(ai));
            } else {
                v4f& c = u == 0 ? s0 : u == 1 ? s1 : u == 2 ? s2 : s3;
                asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %1, %0" : "+v"(c) : "v"(a));
            }
            if constexpr (NV == 4)
                asm volatile(F4 : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
                             : "v"(x), "v"(y));
#pragma unroll
            for (int v = 0; v < NV / 8; ++v)
                asm volatile(F8 : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
                             : "v"(x), "v"(y));
        }
    }
    float r = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
    r += c0[0] + c1[1] + c2[2] + c3[3] + (float)(i0[0] + i1[1] + i2[2] + i3[3]) + s0[0] + s1[1] + s2[2] + s3[3];
    return r;
}

template <int OP, int NV, int W>
__global__ __launch_bounds__(256 * W) void k(float* out, float seed) {
    out[blockIdx.x * 256 * W + threadIdx.x] = body<OP, NV>(seed);
}

template <int OP, int NV, int W>
float run() {
    const int blocks = 256;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * W * 4);
    hipLaunchKernelGGL((k<OP, NV, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<OP, NV, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5 * 1e6f / (ITERS * 4.0f * W);  // ns per MFMA per SIMD
}

template <int OP, int W>
void row(const char* name) {
    std::printf("%-22s W %d  NV0 %6.2f  NV4 %6.2f  NV8 %6.2f  NV16 %6.2f  NV32 %6.2f ns/MFMA\n", name, W,
                run<OP, 0, W>(), run<OP, 4, W>(), run<OP, 8, W>(), run<OP, 16, W>(), run<OP, 32, W>());
}

int main() {
    row<0, 1>("32x32x16 f16");
    row<1, 1>("32x32x16 bf16");
    row<2, 1>("32x32x32 i8");
    row<3, 1>("16x16x32 f16");
    row<0, 2>("32x32x16 f16");
    row<1, 2>("32x32x16 bf16");
    row<2, 2>("32x32x32 i8");
    row<3, 2>("16x16x32 f16");
    return 0;
}
