// mfma_fill.hip -- which VALU hides behind a wave's own MFMA, by instruction class and order?
// Each wave loops { MFMA ; filler block F } (4 independent accumulators rotated), W waves per SIMD;
// the filler instructions rotate over 16 independent register chains (throughput-, not latency-bound)
// (block = 256*W threads, one block per CU).  Filler blocks (8 independent register chains):
//   fmaN    N v_fma_f32            expN    N v_exp_f32          permN  N v_perm_b32
//   eNfM    N v_exp_f32 then M v_fma_f32      fMeN   M v_fma_f32 then N v_exp_f32
// For each (W, F) prints ns per MFMA per SIMD with the MFMA, the same loop without the MFMA
// (filler alone) and the MFMA alone; hidden = alone(F) + alone(MFMA) - both, in cycles at the
// MFMA-calibrated clock (MFMA alone = 32 cycles).  MFMA: v_mfma_i32_32x32x32_i8 (the int8
// kernel's Q@K^T) or v_mfma_f32_32x32x16_f16 (its P@V and the fp16 kernel), argument 1.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#define ITERS 1024
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define R8 "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3), "+v"(f4), "+v"(f5), "+v"(f6), "+v"(f7)
#define R8B "+v"(g0), "+v"(g1), "+v"(g2), "+v"(g3), "+v"(g4), "+v"(g5), "+v"(g6), "+v"(g7)
#define FMA(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n\t"
#define EXP(i) "v_exp_f32 %" #i ", %" #i "\n\t"
#define PERM(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n\t"

// one instruction of class C on chain j (j < 8)
template <int C>
__device__ __forceinline__ void one8(int j, float& f0, float& f1, float& f2, float& f3, float& f4, float& f5, float& f6,
                                     float& f7, float x, float y) {
#define CASE(J)                                                                        \
    case J:                                                                            \
        if constexpr (C == 0) asm volatile(FMA(J) : R8 : "v"(x), "v"(y));              \
        else if constexpr (C == 1) asm volatile(EXP(J) : R8 : "v"(x), "v"(y));         \
        else asm volatile(PERM(J) : R8 : "v"(x), "v"(y));                              \
        break;
    switch (j) { CASE(0) CASE(1) CASE(2) CASE(3) CASE(4) CASE(5) CASE(6) CASE(7) }
#undef CASE
}
#define F16ARGS float &f0, float &f1, float &f2, float &f3, float &f4, float &f5, float &f6, float &f7, \
                float &g0, float &g1, float &g2, float &g3, float &g4, float &g5, float &g6, float &g7
template <int C>
__device__ __forceinline__ void one(int j, F16ARGS, float x, float y) {
    if (j < 8) one8<C>(j, f0, f1, f2, f3, f4, f5, f6, f7, x, y);
    else one8<C>(j - 8, g0, g1, g2, g3, g4, g5, g6, g7, x, y);
}

// filler: NA instructions of class CA, then NB of class CB (chains rotate over 8 registers)
template <int CA, int NA, int CB, int NB, bool MF, int OP>
__device__ float body(float seed) {
    v8h a = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
    v4i ai = {(int)seed, 1, 2, 3};
    v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
    v16i i0 = {}, i1 = {}, i2 = {}, i3 = {};
    float f0 = seed, f1 = seed + 1, f2 = seed + 2, f3 = seed + 3, f4 = seed + 4, f5 = seed + 5, f6 = seed + 6,
          f7 = seed + 7, x = seed * 0.5f, y = seed * 0.25f;
    float g0 = seed + 8, g1 = seed + 9, g2 = seed + 10, g3 = seed + 11, g4 = seed + 12, g5 = seed + 13, g6 = seed + 14,
          g7 = seed + 15;
    int cnt = 0;  // chains rotate over 16 registers across the whole loop (each chain's next op >= 16 ops later)
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (MF) {
                if constexpr (OP == 0) {
                    v16i& c = u == 0 ? i0 : u == 1 ? i1 : u == 2 ? i2 : i3;
                    asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %1, %0" : "+v"(c) : "v"(ai));
                } else {
                    v16f& c = u == 0 ? c0 : u == 1 ? c1 : u == 2 ? c2 : c3;
                    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, %0" : "+v"(c) : "v"(a));
                }
            }
#pragma unroll
            for (int n = 0; n < NA; ++n) one<CA>((u * (NA + NB) + n) & 15, f0, f1, f2, f3, f4, f5, f6, f7, g0, g1, g2, g3, g4, g5, g6, g7, x, y);
#pragma unroll
            for (int n = 0; n < NB; ++n) one<CB>((u * (NA + NB) + NA + n) & 15, f0, f1, f2, f3, f4, f5, f6, f7, g0, g1, g2, g3, g4, g5, g6, g7, x, y);
        }
    }
    float r = f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7 + g0 + g1 + g2 + g3 + g4 + g5 + g6 + g7 + cnt;
    r += c0[0] + c1[1] + c2[2] + c3[3] + (float)(i0[0] + i1[1] + i2[2] + i3[3]);
    return r;
}

template <int CA, int NA, int CB, int NB, bool MF, int OP, int W>
__global__ __launch_bounds__(256 * W) void k(float* out, float seed) {
    out[blockIdx.x * 256 * W + threadIdx.x] = body<CA, NA, CB, NB, MF, OP>(seed);
}

template <int CA, int NA, int CB, int NB, bool MF, int OP, int W>
float run() {
    const int blocks = 256;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * W * 4);
    hipLaunchKernelGGL((k<CA, NA, CB, NB, MF, OP, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((k<CA, NA, CB, NB, MF, OP, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 10 * 1e6f / (ITERS * 4.0f * W);  // ns per MFMA slot per SIMD
}

template <int OP, int W>
float mfma_alone() { return run<0, 0, 0, 0, true, OP, W>(); }

template <int CA, int NA, int CB, int NB, int OP, int W>
void row(const char* name, float m) {
    const float both = run<CA, NA, CB, NB, true, OP, W>(), alone = run<CA, NA, CB, NB, false, OP, W>();
    const float cyc = 32.0f / m;  // cycles per ns at the MFMA-calibrated clock
    std::printf("%s W%d %-8s both %6.2f  filler %6.2f  mfma %6.2f ns | filler %5.1f cyc, hidden %5.1f cyc\n",
                OP == 0 ? "i8 " : "f16", W, name, both, alone, m, alone * cyc, (alone + m - both) * cyc);
}

template <int OP, int W>
void table() {
    const float m = mfma_alone<OP, W>();
    row<0, 4, 0, 0, OP, W>("fma4", m);
    row<0, 8, 0, 0, OP, W>("fma8", m);
    row<0, 16, 0, 0, OP, W>("fma16", m);
    row<1, 2, 0, 0, OP, W>("exp2", m);
    row<1, 4, 0, 0, OP, W>("exp4", m);
    row<1, 8, 0, 0, OP, W>("exp8", m);
    row<2, 4, 0, 0, OP, W>("perm4", m);
    row<2, 8, 0, 0, OP, W>("perm8", m);
    row<1, 4, 0, 8, OP, W>("e4f8", m);
    row<0, 8, 1, 4, OP, W>("f8e4", m);
    row<1, 2, 0, 12, OP, W>("e2f12", m);
    row<0, 12, 1, 2, OP, W>("f12e2", m);
}

int main(int argc, char** argv) {
    const bool f16 = argc > 1 && !std::strcmp(argv[1], "f16");
    if (f16) {
        table<1, 1>(); table<1, 2>(); table<1, 3>(); table<1, 4>();
    } else {
        table<0, 1>(); table<0, 2>(); table<0, 3>(); table<0, 4>();
    }
    return 0;
}
