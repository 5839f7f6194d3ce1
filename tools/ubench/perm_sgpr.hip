// perm_sgpr.hip -- issue cost of v_perm_b32 (the P pack) with its byte selector in an SGPR (as the
// compiler emits it) or a VGPR, and of v_fma_f32 with a VGPR vs an SGPR multiplier, at W waves/SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096
template <int C>
__device__ __forceinline__ void op(float& f, float x, unsigned sv, unsigned vv, float sx) {
    if constexpr (C == 0) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(f) : "v"(x), "s"(sv));
    else if constexpr (C == 1) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(f) : "v"(x), "v"(vv));
    else if constexpr (C == 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f) : "v"(x), "v"(x));
    else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f) : "s"(sx), "v"(x));
}
template <int C, int W>
__global__ __launch_bounds__(256 * W) void kern(float* out, unsigned sel, float seed) {
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = seed + j;
    const float x = seed * 0.5f;
    const unsigned vv = sel + (threadIdx.x >> 12);  // a VGPR copy of the selector
    for (int it = 0; it < ITERS; ++it)
#pragma unroll
        for (int j = 0; j < 16; ++j) op<C>(f[j], x, sel, vv, seed);
    float r = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) r += f[j];
    out[blockIdx.x * 256 * W + threadIdx.x] = r;
}
template <int C, int W>
void row(const char* name) {
    float* out;
    (void)hipMalloc(&out, (size_t)256 * 256 * W * 4);
    hipLaunchKernelGGL((kern<C, W>), dim3(256), dim3(256 * W), 0, 0, out, 0x05040100u, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((kern<C, W>), dim3(256), dim3(256 * W), 0, 0, out, 0x05040100u, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::printf("W%d %-16s %.3f ns per instruction per SIMD\n", W, name, ms / 5 * 1e6 / (ITERS * 16.0 * W));
    (void)hipFree(out);
}
template <int W>
void table() {
    row<0, W>("perm sel=SGPR");
    row<1, W>("perm sel=VGPR");
    row<2, W>("fma all-VGPR");
    row<3, W>("fma SGPR src");
}
int main() {
    table<2>();
    table<3>();
    table<4>();
    return 0;
}
