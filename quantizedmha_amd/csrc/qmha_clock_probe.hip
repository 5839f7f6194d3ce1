// qmha_clock_probe.hip -- the shader clock the chip holds under an attention-like MFMA + VALU mix, measured
// in-kernel (libqmha_probe.so, loaded by bench.py after the headline; not part of libqmha.so).
//
// Why: the main kernels are VALU-issue bound, so their time is cycles / clock, and MI355X boxes of this pool
// hold different clocks under the same code (power cap, DVFS: profiles/r05/box_spread/).  bench.py reports
// the clock beside the time so that two bench lines compare in cycles per tile, not only in ms.
//
// Each wave loops over "units" of one v_mfma_i32_32x32x32_i8 (operands that change every unit, so the
// multipliers toggle) followed by 3 v_exp_f32 and 21 v_fma_f32 on independent registers -- the int8 d = 64
// main kernel's mix per MFMA (6 MFMAs, ~19 transcendental and ~120 other VALU per tile).
// Three waves per SIMD (768-thread workgroups, four rounds of one workgroup per CU).  Wave 0 of every
// workgroup reads s_memtime (shader clock cycles) and s_memrealtime (100 MHz) before and after its loop and
// writes both differences with an ordinary vector store; clock = cycles / ticks * 100 MHz.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

#define QMHA_PROBE_F7                                                                                          \
    "v_fma_f32 %0, %0, %7, %8\n\tv_fma_f32 %1, %1, %7, %8\n\tv_fma_f32 %2, %2, %7, %8\n\tv_fma_f32 %3, %3, %7, %8\n\t" \
    "v_fma_f32 %4, %4, %7, %8\n\tv_fma_f32 %5, %5, %7, %8\n\tv_fma_f32 %6, %6, %7, %8\n\t"

__global__ __launch_bounds__(768) void qmha_clock_probe_kernel(int iters, float* __restrict__ sink,
                                                               unsigned long long* __restrict__ stamps) {
    const uint32_t tid = blockIdx.x * 768 + threadIdx.x;
    v4i a[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) a[s][i] = (int)mix32(tid * 16 + s * 4 + i);
    v16i c0 = {}, c1 = {};
    float f[7], e[3];
#pragma unroll
    for (int i = 0; i < 7; ++i) f[i] = (float)(mix32(tid + 77 * i) & 0xffff) * (1.0f / 65536.0f);
    const float x = 0.75f + (float)(mix32(tid) & 0xff) * (1.0f / 4096.0f);
    const float y = (float)(mix32(tid + 9) & 0xff) * (1.0f / 512.0f);
    const float z = -(float)(mix32(tid + 5) & 0xff) * (1.0f / 64.0f);  // exp2 arguments in (-4, 0]
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            v16i& c = (u & 1) ? c1 : c0;
            c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[u], a[(u + 1) & 3], c, 0, 0, 0);
            asm volatile("v_exp_f32 %0, %3\n\tv_exp_f32 %1, %3\n\tv_exp_f32 %2, %3" : "=v"(e[0]), "=v"(e[1]), "=v"(e[2]) : "v"(z));
#pragma unroll
            for (int v = 0; v < 3; ++v)
                asm volatile(QMHA_PROBE_F7 : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6])
                             : "v"(x), "v"(y));
        }
    }
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    float r = e[0] + e[1] + e[2];
#pragma unroll
    for (int i = 0; i < 7; ++i) r += f[i];
    sink[tid] = r + (float)(c0[0] + c1[5]);
}

}  // namespace

// out[0] shader clock in GHz (s_memtime cycles / s_memrealtime ticks), out[1] ns per unit per SIMD (hipEvents
// over the timed launches), out[2] cycles per unit (= out[1] * out[0]), out[3] timed milliseconds.
// warm: untimed launches first; launches: timed ones.  0 on success, else the HIP error code.
extern "C" int qmha_clock_probe(int warm, int launches, double* out) {
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return (int)e;
    const int blocks = 4 * cus, iters = 1024;
    float* sink = nullptr;
    unsigned long long* st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    unsigned long long* h = new unsigned long long[2 * blocks];
    float ms = 0.0f;
    if ((e = hipMalloc(&sink, (size_t)blocks * 768 * sizeof(float))) != hipSuccess) goto done;
    if ((e = hipMalloc(&st, (size_t)blocks * 2 * sizeof(unsigned long long))) != hipSuccess) goto done;
    if ((e = hipEventCreate(&e0)) != hipSuccess || (e = hipEventCreate(&e1)) != hipSuccess) goto done;
    for (int i = 0; i < warm; ++i) hipLaunchKernelGGL(qmha_clock_probe_kernel, dim3(blocks), dim3(768), 0, 0, iters, sink, st);
    if ((e = hipEventRecord(e0, 0)) != hipSuccess) goto done;
    for (int i = 0; i < launches; ++i) hipLaunchKernelGGL(qmha_clock_probe_kernel, dim3(blocks), dim3(768), 0, 0, iters, sink, st);
    if ((e = hipGetLastError()) != hipSuccess) goto done;
    if ((e = hipEventRecord(e1, 0)) != hipSuccess || (e = hipEventSynchronize(e1)) != hipSuccess) goto done;
    if ((e = hipEventElapsedTime(&ms, e0, e1)) != hipSuccess) goto done;
    if ((e = hipMemcpy(h, st, (size_t)blocks * 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost)) != hipSuccess) goto done;
    {
        double cyc = 0.0, ticks = 0.0;
        for (int b = 0; b < blocks; ++b) {
            cyc += (double)h[2 * b];
            ticks += (double)h[2 * b + 1];
        }
        const double ghz = ticks > 0.0 ? cyc / ticks * 0.1 : 0.0;
        const double units = (double)blocks * 3.0 / cus * iters * 4.0;  // per SIMD per launch (12 waves per block)
        const double ns = launches > 0 ? (double)ms / launches * 1e6 / units : 0.0;
        out[0] = ghz;
        out[1] = ns;
        out[2] = ns * ghz;
        out[3] = ms;
    }
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipFree(st);
    if (sink) (void)hipFree(sink);
    delete[] h;
    return (int)e;
}
