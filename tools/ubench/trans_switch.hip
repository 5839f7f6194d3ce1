// trans_switch.hip -- does interleaving transcendental (v_exp_f32) and full-rate (v_fma_f32) VALU work
// cost more than issuing each class in one run?  Every variant issues the same 16 v_exp_f32 and 32
// v_fma_f32 per loop iteration (16 independent register chains, each chain's next use >= 16 ops away),
// grouped as K runs of {16/K exps, 32/K fmas}: K = 1 (one switch pair per iteration) .. 16.  Also a
// "perm" row: 8 v_perm_b32 (the P pack) in K runs with 32 fmas.  W waves per SIMD (block = 256*W threads,
// one block per CU).  Prints cycles per iteration per SIMD at the clock from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 2048

template <int C>
__device__ __forceinline__ void op(float& f, float x, float y) {
    if constexpr (C == 0) asm volatile("v_exp_f32 %0, %0" : "+v"(f));
    else if constexpr (C == 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f) : "v"(x), "v"(y));
    else asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(f) : "v"(x), "v"(y));
}

// NT trans-class (CT) ops and NF fmas per iteration, in K runs; chains rotate over 16 registers
template <int CT, int NT, int NF, int K>
__device__ float body(float seed, long long* cyc) {
    float f[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) f[j] = seed + 0.001f * j;
    const float x = 0.999f, y = 1e-4f;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
        int c = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int n = 0; n < NT / K; ++n) op<CT>(f[(c++) & 15], x, y);
#pragma unroll
            for (int n = 0; n < NF / K; ++n) op<1>(f[(c++) & 15], x, y);
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
    float r = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) r += f[j];
    return r;
}

template <int CT, int NT, int NF, int K, int W>
__global__ __launch_bounds__(256 * W) void kern(float* out, long long* cyc, float seed) {
    out[blockIdx.x * 256 * W + threadIdx.x] = body<CT, NT, NF, K>(seed, cyc);
}

template <int CT, int NT, int NF, int K, int W>
void row(const char* name) {
    const int blocks = 256;
    float* out;
    long long* cyc;
    (void)hipMalloc(&out, (size_t)blocks * 256 * W * 4);
    (void)hipMalloc(&cyc, 8);
    hipLaunchKernelGGL((kern<CT, NT, NF, K, W>), dim3(blocks), dim3(256 * W), 0, 0, out, cyc, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    const int reps = 5;
    for (int i = 0; i < reps; ++i)
        hipLaunchKernelGGL((kern<CT, NT, NF, K, W>), dim3(blocks), dim3(256 * W), 0, 0, out, cyc, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long c = 0;
    (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    // s_memtime counts the shader clock: cycles per iteration per SIMD = (cycles / ITERS) / W
    std::printf("W%d %-10s K=%2d  %7.1f cycles/iter/SIMD  (%.1f ns/iter/SIMD)\n", W, name, K, (double)c / ITERS / W,
                ms / reps * 1e6 / ITERS / W);
    (void)hipFree(out);
    (void)hipFree(cyc);
}

template <int W>
void table() {
    row<0, 16, 0, 1, W>("exp16");
    row<1, 0, 32, 1, W>("fma32");
    row<0, 16, 32, 1, W>("e16f32");
    row<0, 16, 32, 2, W>("e16f32");
    row<0, 16, 32, 4, W>("e16f32");
    row<0, 16, 32, 8, W>("e16f32");
    row<0, 16, 32, 16, W>("e16f32");
    row<2, 8, 0, 1, W>("perm8");
    row<2, 8, 32, 1, W>("p8f32");
    row<2, 8, 32, 4, W>("p8f32");
    row<2, 8, 32, 8, W>("p8f32");
}

int main() {
    table<1>();
    table<2>();
    table<3>();
    table<4>();
    return 0;
}
