// mfma_fill2.hip -- r06: which VALU instruction classes hide behind MFMAs, for the classes the attention
// kernels issue (round-5 VERDICT items 3 and 4: price each VALU instruction of the int8 per-tensor and the fp16
// tiles against the class it falls in).  Extends mfma_fill.hip (r03: fma / exp / perm) to:
//   fma  v_fma_f32      fmac v_fmac_f32    add  v_add_f32     mul   v_mul_f32      exp  v_exp_f32
//   perm v_perm_b32     cu8  v_cvt_pk_u8_f32                  cf16  v_cvt_pk_f16_f32
//   max3 v_max3_f32     pfma v_pk_fma_f32  pmul v_pk_mul_f32  padd  v_pk_add_f32   rcp  v_rcp_f32
// Each wave loops { MFMA ; 8 filler instructions } over 16 independent registers (throughput-bound; exp, rcp and
// cvt read loop-invariant inputs, so no chain reaches inf / NaN),
// W waves per SIMD (one 256*W-thread block per CU).  Printed per (MFMA, W, class): ns per slot per SIMD with
// the MFMA ("both"), without it ("filler"), the MFMA alone, the filler's cycles and the cycles of it that hid
// (alone(F) + alone(MFMA) - both) at the MFMA-calibrated clock (one 32x32 MFMA = 32 cycles).
// Also checks v_cvt_pk_u8_f32's rounding on chosen values (the per-tensor P quantisation).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define ITERS 1024
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v2f __attribute__((ext_vector_type(2)));

enum { FMA, FMAC, ADD, MUL, EXP, PERM, CU8, CF16, MAX3, PFMA, PMUL, PADD, RCP, NCLS };
static const char* kName[NCLS] = {"fma", "fmac", "add", "mul", "exp", "perm", "cu8", "cf16", "max3", "pfma", "pmul", "padd", "rcp"};

// one instruction of class C on chain register r (x, y: loop-invariant operands)
template <int C>
__device__ __forceinline__ void op(float& r, v2f& q, float x, float y, v2f xx) {
    if constexpr (C == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
    else if constexpr (C == FMAC) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
    else if constexpr (C == ADD) asm volatile("v_add_f32 %0, %0, %1" : "+v"(r) : "v"(x));
    else if constexpr (C == MUL) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(r) : "v"(x));
    else if constexpr (C == EXP) asm volatile("v_exp_f32 %0, %1" : "+v"(r) : "v"(y));
    else if constexpr (C == PERM) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
    else if constexpr (C == CU8) asm volatile("v_cvt_pk_u8_f32 %0, %1, 1, %0" : "+v"(r) : "v"(x));
    else if constexpr (C == CF16) asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
    else if constexpr (C == MAX3) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(r) : "v"(x), "v"(y));
    else if constexpr (C == PFMA) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(q) : "v"(xx));
    else if constexpr (C == PMUL) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(q) : "v"(xx));
    else if constexpr (C == PADD) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(q) : "v"(xx));
    else asm volatile("v_rcp_f32 %0, %1" : "+v"(r) : "v"(x));
}

template <int C, bool MF, int OP>
__device__ float body(float seed) {
    v8h a = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
    v4i ai = {(int)seed, 1, 2, 3};
    v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
    v16i i0 = {}, i1 = {}, i2 = {}, i3 = {};
    float f[16];
    v2f q[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        f[j] = 0.5f + seed * 0.001f * j;
        q[j] = v2f{f[j], f[j] + 1.0f};
    }
    const float x = 0.999f + seed * 1e-6f, y = 1e-3f * seed;
    const v2f xx = {x, x};
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
            for (int n = 0; n < 8; ++n) op<C>(f[(u * 8 + n) & 15], q[(u * 8 + n) & 15], x, y, xx);
        }
    }
    float r = 0.0f;
#pragma unroll
    for (int j = 0; j < 16; ++j) r += f[j] + q[j][0] + q[j][1];
    r += c0[0] + c1[1] + c2[2] + c3[3] + (float)(i0[0] + i1[1] + i2[2] + i3[3]);
    return r;
}

template <int C, bool MF, int OP, int W>
__global__ __launch_bounds__(256 * W) void k(float* out, float seed) {
    out[blockIdx.x * 256 * W + threadIdx.x] = body<C, MF, OP>(seed);
}

template <int C, bool MF, int OP, int W>
float run() {
    const int blocks = 256;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * W * 4);
    hipLaunchKernelGGL((k<C, MF, OP, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((k<C, MF, OP, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(out);
    return ms / 10 * 1e6f / (ITERS * 4.0f * W);  // ns per MFMA slot per SIMD
}

template <int C, int OP, int W>
void row(float m) {
    const float both = run<C, true, OP, W>(), alone = run<C, false, OP, W>();
    const float cyc = 32.0f / m;
    std::printf("%s W%d %-5s both %6.2f  filler %6.2f  mfma %6.2f ns | filler %5.1f cyc (%4.2f per op), hidden %5.1f cyc\n",
                OP == 0 ? "i8 " : "f16", W, kName[C], both, alone, m, alone * cyc, alone * cyc / 8, (alone + m - both) * cyc);
}

template <int OP, int W, int C = 0>
void table(float m) {
    if constexpr (C < NCLS) {
        row<C, OP, W>(m);
        table<OP, W, C + 1>(m);
    }
}

// the MFMA alone: the same loop with no filler
template <int OP>
__device__ float mfma_body(float seed) {
    v8h a = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
    v4i ai = {(int)seed, 1, 2, 3};
    v16f c0 = {}, c1 = {}, c2 = {}, c3 = {};
    v16i i0 = {}, i1 = {}, i2 = {}, i3 = {};
    for (int it = 0; it < ITERS; ++it) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if constexpr (OP == 0) {
                v16i& c = u == 0 ? i0 : u == 1 ? i1 : u == 2 ? i2 : i3;
                asm volatile("v_mfma_i32_32x32x32_i8 %0, %1, %1, %0" : "+v"(c) : "v"(ai));
            } else {
                v16f& c = u == 0 ? c0 : u == 1 ? c1 : u == 2 ? c2 : c3;
                asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, %0" : "+v"(c) : "v"(a));
            }
        }
    }
    return c0[0] + c1[1] + c2[2] + c3[3] + (float)(i0[0] + i1[1] + i2[2] + i3[3]);
}
template <int OP, int W>
__global__ __launch_bounds__(256 * W) void km(float* out, float seed) {
    out[blockIdx.x * 256 * W + threadIdx.x] = mfma_body<OP>(seed);
}
template <int OP, int W>
float mfma_only() {
    const int blocks = 256;
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * W * 4);
    hipLaunchKernelGGL((km<OP, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL((km<OP, W>), dim3(blocks), dim3(256 * W), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 10 * 1e6f / (ITERS * 4.0f * W);
}
template <int OP, int W>
void config() { table<OP, W>(mfma_only<OP, W>()); }

// ---- v_cvt_pk_u8_f32 rounding
__global__ void cvt_u8(const float* in, unsigned* out, int n) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i < n) {
        unsigned r;
        asm volatile("v_cvt_pk_u8_f32 %0, %1, 0, 0" : "=v"(r) : "v"(in[i]));
        out[i] = r;
    }
}

int main(int argc, char** argv) {
    (void)argc;
    (void)argv;
    // rounding of v_cvt_pk_u8_f32 (byte 0 of dword 0)
    const float vals[] = {0.0f, 0.25f, 0.5f, 0.75f, 1.0f, 1.5f, 2.5f, 3.5f, 0.49999997f, 0.50000006f, 126.5f, 127.4f,
                          127.5f, 254.5f, 255.4f, 255.5f, 256.0f, 300.0f, -0.4f, -1.0f, 1e-30f, __builtin_nanf("")};
    const int n = sizeof(vals) / sizeof(vals[0]);
    float* din;
    unsigned* dout;
    (void)hipMalloc(&din, n * 4);
    (void)hipMalloc(&dout, n * 4);
    (void)hipMemcpy(din, vals, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(cvt_u8, dim3(1), dim3(64), 0, 0, din, dout, n);
    unsigned h[64];
    (void)hipMemcpy(h, dout, n * 4, hipMemcpyDeviceToHost);
    std::printf("# v_cvt_pk_u8_f32 x -> byte (rintf(x) for comparison)\n");
    for (int i = 0; i < n; ++i) std::printf("cvt_pk_u8 %-12.9g -> %3u   rintf %g\n", vals[i], h[i] & 0xff, __builtin_rintf(vals[i]));
    std::printf("# filler classes: ns per MFMA slot per SIMD, 8 filler instructions per MFMA\n");
    config<0, 3>();  // the int8 kernels: i8 MFMA, 3 waves per SIMD
    config<1, 3>();  // their f16 P@V MFMA
    config<1, 4>();  // the fp16 kernel: 4 waves per SIMD
    config<0, 2>();
    return 0;
}
