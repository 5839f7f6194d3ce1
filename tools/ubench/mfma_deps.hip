// mfma_deps.hip -- why do the int8 kernel's MFMAs not hide behind its VALU the way an isolated
// MFMA + {exp, fma} mix does (tools/ubench/mfma_fill.hip)?  One "tile" per loop iteration with the
// kernel's proportions: 6 MFMAs (2 x v_mfma_i32_32x32x32_i8, 4 x v_mfma_f32_32x32x16_f16), and per
// MFMA 3 v_exp_f32 + 21 v_fma_f32 on independent register chains, each MFMA in its own sched_barrier
// region with its VALU.  Variants add one feature of the real kernel at a time:
//   LDS  : every MFMA's A operand is read from LDS (ds_read_b128) in the region before it
//   USE  : the P@V results are consumed by VALU (16 fmas folding each f16 accumulator into O)
//          one region after the MFMA that produced them, the Q@K^T result by the next iteration
//   CHAIN: the fillers form the softmax's dependent chain (fma -> exp -> fma) instead of
//          independent chains
//   LDSFAR: (with LDS) the six operands of iteration i+1 are read during iteration i (>= 3 regions
//          ahead) instead of one region ahead
//   USEFAR: (with USE) the P@V results are folded one iteration later (>= 6 regions after the MFMA)
// For each variant: ns per tile per SIMD with the MFMAs, and with every MFMA replaced by nothing
// (same VALU / LDS stream); the difference is what the 6 MFMAs cost (192 cycles if nothing hides).
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 512
#define FENCE() __builtin_amdgcn_sched_barrier(0)
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef int v16i __attribute__((ext_vector_type(16)));

enum { LDS = 1, USE = 2, CHAIN = 4, NOMFMA = 8, LDSFAR = 16, USEFAR = 32 };

template <int N>
__device__ __forceinline__ void pin(float (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

template <int F, int W>
__global__ __launch_bounds__(256 * W) void kern(float* out, float seed) {
    __shared__ __attribute__((aligned(16))) int lds[W * 4 * 64 * 4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < W * 4 * 64 * 4; i += blockDim.x) lds[i] = i;
    __syncthreads();
    int* mylds = lds + wave * 64 * 4;
    float f[24];
#pragma unroll
    for (int j = 0; j < 24; ++j) f[j] = seed + 0.01f * j;
    float o[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) o[j] = 0.0f;
    const float sc = seed * 1e-3f;
    v8h a16 = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
    v4i a8 = {(int)seed, 1, 2, 3};
    v16i s0 = {}, s1 = {};
    v16f p0 = {}, p1 = {};
    auto opnd = [&](int k) {  // an MFMA operand: from LDS (LDS) or the register copy
        if constexpr (F & LDS) {
            int off = 4 * lane + 0 * k;
            asm volatile("" : "+v"(off));  // a fresh read every time (no CSE across the loop)
            v4i x = *reinterpret_cast<const v4i*>(mylds + off);
            return x;
        } else {
            v4i x = a8 + v4i{k, 0, 0, 0};  // distinct operands: no CSE of identical MFMAs
            asm volatile("" : "+v"(x));
            return x;
        }
    };
    auto fill = [&]() {  // 3 exps + 21 fmas
        if constexpr (F & CHAIN) {
            // softmax-like: x = fma(s, c, -k); p = exp(x); q = fma(p, inv, magic), chains of 3
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                f[j] = __builtin_amdgcn_exp2f(fmaf(f[j + 3], sc, -0.5f));
                f[j + 6] = fmaf(f[j], 127.0f, 12582912.0f);
            }
#pragma unroll
            for (int j = 9; j < 24; ++j) f[j] = fmaf(f[j], 0.999f, sc);
        } else {
#pragma unroll
            for (int j = 0; j < 3; ++j) f[j] = __builtin_amdgcn_exp2f(f[j]);
#pragma unroll
            for (int j = 3; j < 24; ++j) f[j] = fmaf(f[j], 0.999f, sc);
        }
        pin(f);
    };
    auto fold = [&](const v16f& p, int base) {  // O += p * s (the per-tile fold)
        if constexpr (F & USE) {
#pragma unroll
            for (int j = 0; j < 16; ++j) o[base + j] = fmaf(p[j], sc, o[base + j]);
            pin(o);
        }
    };
    v4i nx[6];
    v16f q0 = {}, q1 = {};  // USEFAR: the previous iteration's P@V results
    if constexpr ((F & LDSFAR) != 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) nx[k] = opnd(k);
    }
    for (int it = 0; it < ITERS; ++it) {
        v4i op[6];
        if constexpr ((F & LDSFAR) != 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) op[k] = nx[k];
        } else {
            op[0] = opnd(0);
            op[1] = opnd(1);
        }
        auto late = [&](int k) {
            if constexpr (!(F & LDSFAR)) op[k] = opnd(k);
        };
        auto foldp = [&](const v16f& p, const v16f& q, int base) {
            if constexpr ((F & USEFAR) != 0) fold(q, base); else fold(p, base);
        };
        FENCE();
        if constexpr (!(F & NOMFMA)) s0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(op[0], a8, s0, 0, 0, 0);
        fill();
        if constexpr ((F & USEFAR) != 0) fold(q1, 16);
        FENCE();
        late(2);
        if constexpr (!(F & NOMFMA)) s1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(op[1], a8, s1, 0, 0, 0);
        fill();
        if constexpr ((F & USEFAR) != 0) fold(q0, 0);
        FENCE();
        late(3);
        if constexpr (!(F & NOMFMA)) p0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, op[2]), a16, v16f{}, 0, 0, 0);
        fill();
        if constexpr ((F & LDSFAR) != 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) nx[k] = opnd(k);
        }
        FENCE();
        late(4);
        if constexpr (!(F & NOMFMA)) p1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, op[3]), a16, v16f{}, 0, 0, 0);
        fill();
        FENCE();
        late(5);
        if constexpr (!(F & NOMFMA)) p0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, op[4]), a16, p0, 0, 0, 0);
        fill();
        if constexpr (!(F & USEFAR)) fold(p1, 16);  // p1 (first k-step) one region ago
        FENCE();
        if constexpr (!(F & NOMFMA)) p1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(v8h, op[5]), a16, p1, 0, 0, 0);
        fill();
        if constexpr (!(F & USEFAR)) fold(p0, 0);
        FENCE();
        (void)foldp;
        if constexpr (F & USE) {  // the next tile's scores feed the next iteration's exps
            f[3] += (float)s0[0] * 1e-9f;
            f[4] += (float)s1[1] * 1e-9f;
        }
        if constexpr ((F & USEFAR) != 0) {
            q0 = p0;
            q1 = p1;
        }
        if constexpr (!(F & NOMFMA)) {
            asm volatile("" : "+v"(s0), "+v"(s1), "+v"(p0), "+v"(p1));
        }
    }
    float r = 0;
#pragma unroll
    for (int j = 0; j < 24; ++j) r += f[j];
#pragma unroll
    for (int j = 0; j < 32; ++j) r += o[j];
    r += p0[0] + p1[1] + (float)(s0[2] + s1[3]);
    for (int k = 0; k < 6; ++k) r += (float)nx[k][0] * 0.0f;
    out[blockIdx.x * 256 * W + threadIdx.x] = r;
}

template <int F, int W>
float run() {
    float* out;
    (void)hipMalloc(&out, (size_t)256 * 256 * W * 4);
    hipLaunchKernelGGL((kern<F, W>), dim3(256), dim3(256 * W), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((kern<F, W>), dim3(256), dim3(256 * W), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5 * 1e6f / (ITERS * W);  // ns per tile per SIMD
}

template <int F, int W>
void row(const char* name) {
    const float with = run<F, W>(), without = run<F | NOMFMA, W>();
    std::printf("W%d %-16s with MFMA %7.2f ns/tile/SIMD  without %7.2f  -> the 6 MFMAs cost %6.2f ns\n", W, name, with,
                without, with - without);
}

template <int W>
void table() {
    row<0, W>("base");
    row<LDS, W>("lds");
    row<USE, W>("use");
    row<CHAIN, W>("chain");
    row<LDS | USE, W>("lds+use");
    row<LDS | USE | CHAIN, W>("lds+use+chain");
    row<LDS | LDSFAR | USE | CHAIN, W>("ldsfar+use+chain");
    row<LDS | USE | USEFAR | CHAIN, W>("lds+usefar+chain");
    row<LDS | LDSFAR | USE | USEFAR | CHAIN, W>("far+far+chain");
}

int main() {
    table<2>();
    table<3>();
    return 0;
}
