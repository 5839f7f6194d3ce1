// valu_mix.hip -- do two different VALU opcodes from two waves on one SIMD share issue
// (time = sum of the two streams) or co-issue (time = max)?  Block = 512 threads = 8 waves =
// 2 per SIMD; waves 0-3 run opcode X, waves 4-7 opcode Y (8 independent chains each).
// Also: both opcodes interleaved inside ONE wave's stream (2 waves per SIMD running it).
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096
#define B8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define O_FMA(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n\t"
#define O_ADD(i) "v_add_f32 %" #i ", %" #i ", %8\n\t"
#define O_EXP(i) "v_exp_f32 %" #i ", %" #i "\n\t"
#define O_CVT(i) "v_cvt_f32_i32 %" #i ", %" #i "\n\t"
#define O_MAX(i) "v_max_f32 %" #i ", %" #i ", %8\n\t"
#define O_CPK(i) "v_cvt_pk_f16_f32 %" #i ", %" #i ", %8\n\t"
#define O_PERM(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n\t"
#define O_MAX3(i) "v_max3_i32 %" #i ", %" #i ", %8, %9\n\t"

template <int OP>
__device__ __forceinline__ void op8(float& a0, float& a1, float& a2, float& a3, float& a4, float& a5, float& a6,
                                    float& a7, float x, float y) {
#define ASM8(S) asm volatile(B8(S) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y))
    if constexpr (OP == 0) ASM8(O_FMA);
    if constexpr (OP == 1) ASM8(O_ADD);
    if constexpr (OP == 2) ASM8(O_EXP);
    if constexpr (OP == 3) ASM8(O_CVT);
    if constexpr (OP == 4) ASM8(O_MAX);
    if constexpr (OP == 5) ASM8(O_CPK);
    if constexpr (OP == 6) ASM8(O_PERM);
    if constexpr (OP == 7) ASM8(O_MAX3);
#undef ASM8
}

// MODE 0: this wave runs X only; MODE 1: X and Y interleaved (8 X then 8 Y per step)
template <int X, int Y, int MODE>
__device__ float stream(float seed) {
    float a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
          a7 = seed + 7, x = seed * 0.5f, y = seed * 0.25f;
    float b0 = a0, b1 = a1, b2 = a2, b3 = a3, b4 = a4, b5 = a5, b6 = a6, b7 = a7;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            op8<X>(a0, a1, a2, a3, a4, a5, a6, a7, x, y);
            if constexpr (MODE == 1) op8<Y>(b0, b1, b2, b3, b4, b5, b6, b7, x, y);
        }
    }
    return a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7;
}

// CFG 0: waves 0-3 X, 4-7 Y (two streams, one per wave);  CFG 1: all 8 waves X+Y interleaved
template <int X, int Y, int CFG>
__global__ __launch_bounds__(512) void k(float* out, float seed) {
    const int wave = threadIdx.x >> 6;
    float r;
    if constexpr (CFG == 0)
        r = wave < 4 ? stream<X, X, 0>(seed) : stream<Y, Y, 0>(seed);
    else
        r = stream<X, Y, 1>(seed);
    out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <int X, int Y, int CFG>
float run() {
    const int blocks = 256;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * 512 * 4);
    hipLaunchKernelGGL((k<X, Y, CFG>), dim3(blocks), dim3(512), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<X, Y, CFG>), dim3(blocks), dim3(512), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5;
}

static const char* NAMES[] = {"fma", "add", "exp", "cvt_f32_i32", "max_f32", "cvt_pk_f16", "perm", "max3_i32"};

template <int X, int Y>
void row() {
    const float xx = run<X, X, 0>(), yy = run<Y, Y, 0>(), xy = run<X, Y, 0>(), il = run<X, Y, 1>();
    // per SIMD: 2 waves x 131072 instructions of the stream; cycles at 2.1 GHz per instruction
    std::printf("%-12s %-12s  X|X %.4f  Y|Y %.4f  X|Y %.4f  (X+Y)|(X+Y) %.4f ms\n", NAMES[X], NAMES[Y], xx, yy, xy, il);
}

int main() {
    std::printf("two waves per SIMD; X|Y = one wave of X beside one wave of Y; (X+Y) = both interleaved in each wave\n");
    row<0, 0>();
    row<3, 3>();
    row<3, 0>();
    row<3, 1>();
    row<2, 0>();
    row<2, 3>();
    row<4, 0>();
    row<5, 0>();
    row<6, 0>();
    row<7, 0>();
    row<5, 3>();
    row<2, 2>();
    return 0;
}
