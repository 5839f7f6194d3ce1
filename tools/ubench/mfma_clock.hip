// mfma_clock.hip -- which MFMA shape holds the higher clock under the fp16 kernel's load?
// Each "unit" is 32 matrix-core cycles: one 32x32 MFMA or two 16x16 MFMAs of the same dtype
// (same FLOPs), followed by NV independent v_fma_f32 on data that changes every unit.  Three
// waves per SIMD (768-thread blocks, one per CU at a time), operands random per lane and rotated
// over four register sets so the multiplier inputs toggle every MFMA, as in a real kernel.
// After ~1 s of back-to-back launches it times 40 launches (hipEvents) and reads the in-kernel
// clock from s_memtime / s_memrealtime stamps of wave 0 of every block (written to a buffer of
// their own by an ordinary vector store).  Prints ns per unit per SIMD, the clock, and cycles
// per unit (= ns x GHz): equal cycles at a higher clock is the DVFS lever of
// MI355X_MICROARCH.md 'DVFS give-back' item 7 / cdna_hip_programming.md rule 28.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define ITERS 2048
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

#define F6 "v_fma_f32 %0, %0, %6, %7\n\tv_fma_f32 %1, %1, %6, %7\n\tv_fma_f32 %2, %2, %6, %7\n\t" \
           "v_fma_f32 %3, %3, %6, %7\n\tv_fma_f32 %4, %4, %6, %7\n\tv_fma_f32 %5, %5, %6, %7\n\t"

// OP 0: 32x32x16 f16   1: 2 x 16x16x32 f16   2: 32x32x32 i8   3: 2 x 16x16x64 i8
template <int OP, int NV>
__global__ __launch_bounds__(768) void k(float* out, uint64_t* stamps, uint32_t seed) {
    const uint32_t tid = blockIdx.x * 768 + threadIdx.x;
    v8h a[4];
    v4i ai[4];
    for (int s = 0; s < 4; ++s)
        for (int i = 0; i < 8; ++i) {
            const uint32_t h = hash(seed ^ (tid * 64 + s * 8 + i));
            a[s][i] = (_Float16)((float)(h & 0xffff) * (2.0f / 65536.0f) - 1.0f);
            if (i < 4) ai[s][i] = (int)hash(h);
        }
    v16f c0 = {}, c1 = {};
    v4f d0 = {}, d1 = {}, d2 = {}, d3 = {};
    v16i i0 = {}, i1 = {};
    v4i j0 = {}, j1 = {}, j2 = {}, j3 = {};
    float f[6];
    for (int i = 0; i < 6; ++i) f[i] = (float)(hash(tid + 77 * i) & 0xffff) * (1.0f / 65536.0f);
    float x = 0.75f + (float)(hash(tid) & 0xff) * (1.0f / 4096.0f), y = (float)(hash(tid + 9) & 0xff) * (1.0f / 512.0f);
    uint64_t t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const v8h& p = a[u];
            const v8h& q = a[(u + 1) & 3];
            if constexpr (OP == 0) {
                v16f& c = (u & 1) ? c1 : c0;
                c = __builtin_amdgcn_mfma_f32_32x32x16_f16(p, q, c, 0, 0, 0);
            } else if constexpr (OP == 1) {
                v4f& e = (u & 1) ? d1 : d0;
                v4f& g = (u & 1) ? d3 : d2;
                e = __builtin_amdgcn_mfma_f32_16x16x32_f16(p, q, e, 0, 0, 0);
                g = __builtin_amdgcn_mfma_f32_16x16x32_f16(q, p, g, 0, 0, 0);
            } else if constexpr (OP == 2) {
                v16i& c = (u & 1) ? i1 : i0;
                c = __builtin_amdgcn_mfma_i32_32x32x32_i8(ai[u], ai[(u + 1) & 3], c, 0, 0, 0);
            } else {
                v4i& e = (u & 1) ? j1 : j0;
                v4i& g = (u & 1) ? j3 : j2;
                e = __builtin_amdgcn_mfma_i32_16x16x64_i8(ai[u], ai[(u + 1) & 3], e, 0, 0, 0);
                g = __builtin_amdgcn_mfma_i32_16x16x64_i8(ai[(u + 1) & 3], ai[u], g, 0, 0, 0);
            }
#pragma unroll
            for (int v = 0; v < NV / 6; ++v)
                asm volatile(F6 : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]) : "v"(x), "v"(y));
        }
    }
    if (threadIdx.x == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    float r = f[0] + f[1] + f[2] + f[3] + f[4] + f[5];
    r += c0[0] + c1[1] + d0[0] + d1[1] + d2[2] + d3[3] + (float)(i0[0] + i1[1] + j0[0] + j1[1] + j2[2] + j3[3]);
    out[tid] = r;
}

template <int OP, int NV>
void run(const char* name) {
    const int blocks = 256 * 4;
    float* out;
    uint64_t* st;
    (void)hipMalloc(&out, (size_t)blocks * 768 * 4);
    (void)hipMalloc(&st, (size_t)blocks * 16);
    auto launch = [&](uint32_t s) { hipLaunchKernelGGL((k<OP, NV>), dim3(blocks), dim3(768), 0, 0, out, st, s); };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    // warm: ~1 s of back-to-back launches so the clock settles
    (void)hipEventRecord(e0);
    launch(1);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms1;
    (void)hipEventElapsedTime(&ms1, e0, e1);
    const int warm = (int)(1000.0f / (ms1 > 0.01f ? ms1 : 0.01f)) + 1;
    for (int i = 0; i < warm; ++i) launch(2 + i);
    const int reps = 40;
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) launch(1000 + i);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    uint64_t* h = new uint64_t[2 * blocks];
    (void)hipMemcpy(h, st, (size_t)blocks * 16, hipMemcpyDeviceToHost);
    double cyc = 0, real = 0;
    for (int b = 0; b < blocks; ++b) {
        cyc += (double)h[2 * b];
        real += (double)h[2 * b + 1];
    }
    const double ghz = cyc / real * 0.1;  // s_memrealtime ticks at 100 MHz
    // units per SIMD per launch: blocks/256 rounds x 3 waves x ITERS x 4
    const double units = (double)blocks / 256 * 3 * ITERS * 4;
    const double ns = ms / reps * 1e6 / units;
    std::printf("%-22s NV %2d  %7.3f ns/unit/SIMD  clock %5.3f GHz  %6.1f cycles/unit\n", name, NV, ns, ghz, ns * ghz);
    delete[] h;
    (void)hipFree(out);
    (void)hipFree(st);
}

int main(int argc, char** argv) {
    if (argc > 1) {  // r06: the fp16 tile's density after the lazy base (~9 VALU per MFMA)
        run<0, 6>("32x32x16 f16");
        run<1, 6>("2x 16x16x32 f16");
        run<0, 12>("32x32x16 f16");
        run<1, 12>("2x 16x16x32 f16");
        run<0, 6>("32x32x16 f16");
        run<1, 6>("2x 16x16x32 f16");
        return 0;
    }
    run<0, 0>("32x32x16 f16");
    run<1, 0>("2x 16x16x32 f16");
    run<0, 12>("32x32x16 f16");
    run<1, 12>("2x 16x16x32 f16");
    run<0, 18>("32x32x16 f16");
    run<1, 18>("2x 16x16x32 f16");
    run<2, 0>("32x32x32 i8");
    run<3, 0>("2x 16x16x64 i8");
    run<2, 18>("32x32x32 i8");
    run<3, 18>("2x 16x16x64 i8");
    return 0;
}
