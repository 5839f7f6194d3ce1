// mfma_coexec.hip -- does a VALU stream on one wave overlap an MFMA stream on another wave of
// the same SIMD?  Block = 512 threads = 8 waves = 2 per SIMD; waves 0-3 run an MFMA chain
// (accumulator in arch VGPRs = hipcc's -amdgpu-mfma-vgpr-form, or in AGPRs) or idle, waves 4-7
// run a stream of one VALU opcode (8 independent chains).  Wall time per configuration.
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096

typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v2f __attribute__((ext_vector_type(2)));

#define B8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)
#define OPS3(i) "v_fma_f32 %" #i ", %" #i ", %8, %9\n\t"
#define OPS2(i) "v_add_f32 %" #i ", %" #i ", %8\n\t"
#define OPSM(i) "v_mul_f32 %" #i ", %" #i ", %8\n\t"
#define OPSE(i) "v_exp_f32 %" #i ", %" #i "\n\t"
#define OPSC(i) "v_cvt_f32_i32 %" #i ", %" #i "\n\t"
#define OPSX(i) "v_max_f32 %" #i ", %" #i ", %8\n\t"
#define OPSP(i) "v_perm_b32 %" #i ", %" #i ", %8, %9\n\t"
#define OPSH(i) "v_cvt_pk_f16_f32 %" #i ", %" #i ", %8\n\t"
#define OPSF(i) "v_fmac_f32 %" #i ", %8, %9\n\t"
#define OPSS(i) "v_sub_f32 %" #i ", %" #i ", %8\n\t"
#define OPSV(i) "v_mov_b32 %" #i ", %8\n\t"
#define OPS3I(i) "v_max3_i32 %" #i ", %" #i ", %8, %9\n\t"
#define OPSD(i) "v_max_i32_dpp %" #i ", %" #i ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
#define OPSMX(i) "v_fma_mixlo_f16 %" #i ", %" #i ", %8, %9\n\t"
#define OPSI(i) "v_max_i32 %" #i ", %" #i ", %8\n\t"

template <int OP>
__device__ float valu(float seed) {
    float a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
          a7 = seed + 7, x = seed * 0.5f, y = seed * 0.25f;
    v2f b0 = {seed, 1}, b1 = {2, seed}, b2 = {3, 4}, b3 = {seed, seed}, px = {x, y};
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#define ASM8(S) asm volatile(B8(S) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y))
            if constexpr (OP == 0) ASM8(OPS3);
            if constexpr (OP == 1) ASM8(OPS2);
            if constexpr (OP == 2) ASM8(OPSM);
            if constexpr (OP == 3) ASM8(OPSE);
            if constexpr (OP == 4) ASM8(OPSC);
            if constexpr (OP == 5) ASM8(OPSX);
            if constexpr (OP == 6) ASM8(OPSP);
            if constexpr (OP == 7) ASM8(OPSH);
            if constexpr (OP == 8) ASM8(OPSF);
            if constexpr (OP == 11) ASM8(OPSS);
            if constexpr (OP == 12) ASM8(OPSV);
            if constexpr (OP == 13) ASM8(OPS3I);
            if constexpr (OP == 14) ASM8(OPSD);
            if constexpr (OP == 15) ASM8(OPSMX);
            if constexpr (OP == 16) ASM8(OPSI);
            if constexpr (OP == 17)
                asm volatile("v_permlane32_swap_b32 %0, %1\n\tv_permlane32_swap_b32 %2, %3\n\tv_permlane32_swap_b32 %4, %5\n\t"
                             "v_permlane32_swap_b32 %6, %7\n\tv_permlane32_swap_b32 %1, %2\n\tv_permlane32_swap_b32 %3, %4\n\t"
                             "v_permlane32_swap_b32 %5, %6\n\tv_permlane32_swap_b32 %7, %0"
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            if constexpr (OP == 18) {  // AGPR -> VGPR reads (8 per group, from a resident AGPR block)
                asm volatile("v_accvgpr_read_b32 %0, a0\n\tv_accvgpr_read_b32 %1, a1\n\tv_accvgpr_read_b32 %2, a2\n\t"
                             "v_accvgpr_read_b32 %3, a3\n\tv_accvgpr_read_b32 %4, a4\n\tv_accvgpr_read_b32 %5, a5\n\t"
                             "v_accvgpr_read_b32 %6, a6\n\tv_accvgpr_read_b32 %7, a7"
                             : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3), "=v"(a4), "=v"(a5), "=v"(a6), "=v"(a7)::"a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7");
            }
            if constexpr (OP == 9)
                asm volatile("v_pk_fma_f32 %0, %0, %4, %4\n\tv_pk_fma_f32 %1, %1, %4, %4\n\tv_pk_fma_f32 %2, %2, %4, %4\n\t"
                             "v_pk_fma_f32 %3, %3, %4, %4\n\tv_pk_fma_f32 %0, %0, %4, %4\n\tv_pk_fma_f32 %1, %1, %4, %4\n\t"
                             "v_pk_fma_f32 %2, %2, %4, %4\n\tv_pk_fma_f32 %3, %3, %4, %4"
                             : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "v"(px));
            if constexpr (OP == 10)
                asm volatile("v_pk_add_f32 %0, %0, %4\n\tv_pk_add_f32 %1, %1, %4\n\tv_pk_add_f32 %2, %2, %4\n\t"
                             "v_pk_add_f32 %3, %3, %4\n\tv_pk_add_f32 %0, %0, %4\n\tv_pk_add_f32 %1, %1, %4\n\t"
                             "v_pk_add_f32 %2, %2, %4\n\tv_pk_add_f32 %3, %3, %4"
                             : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "v"(px));
        }
    }
    return a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0.x + b1.y + b2.x + b3.y;
}

// MA: 0 idle, 1 MFMA acc in VGPRs, 2 MFMA acc in AGPRs, 3 same VALU stream as the B waves
template <int MA, int OP>
__global__ __launch_bounds__(512) void k(float* out, float seed) {
    const int wave = threadIdx.x >> 6;
    float r = 0.0f;
    if (wave < 4) {
        if constexpr (MA == 1 || MA == 2) {
            v8h a = {(_Float16)seed, 1, 2, 3, 4, 5, 6, 7};
            v16f c = {};
            for (int i = 0; i < ITERS; ++i) {
                if constexpr (MA == 1)
                    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, %0\n\tv_mfma_f32_32x32x16_f16 %0, %1, %1, %0\n\t"
                                 "v_mfma_f32_32x32x16_f16 %0, %1, %1, %0\n\tv_mfma_f32_32x32x16_f16 %0, %1, %1, %0"
                                 : "+v"(c) : "v"(a));
                else
                    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %1, %0\n\tv_mfma_f32_32x32x16_f16 %0, %1, %1, %0\n\t"
                                 "v_mfma_f32_32x32x16_f16 %0, %1, %1, %0\n\tv_mfma_f32_32x32x16_f16 %0, %1, %1, %0"
                                 : "+a"(c) : "v"(a));
            }
            r = c[0] + c[15];
        } else if constexpr (MA == 3) {
            r = valu<OP>(seed);
        }
    } else {
        r = valu<OP>(seed);
    }
    out[blockIdx.x * 512 + threadIdx.x] = r;
}

template <int MA, int OP>
float run() {
    const int blocks = 256;  // one 8-wave block per CU: 2 waves per SIMD
    float* out;
    (void)hipMalloc(&out, (size_t)blocks * 512 * 4);
    hipLaunchKernelGGL((k<MA, OP>), dim3(blocks), dim3(512), 0, 0, out, 1.0f);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((k<MA, OP>), dim3(blocks), dim3(512), 0, 0, out, 1.0f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipFree(out);
    return ms / 5;
}

template <int OP>
void row(const char* name) {
    std::printf("%-18s alone %.4f  x2 %.4f  +mfma(vgpr) %.4f  +mfma(agpr) %.4f ms\n", name, run<0, OP>(), run<3, OP>(),
                run<1, OP>(), run<2, OP>());
}

int main() {
    std::printf("mfma(vgpr) alone %.4f ms, mfma(agpr) alone %.4f ms (16384 x 32x32x16 per SIMD)\n", run<1, 99>(), run<2, 99>());
    row<0>("v_fma_f32");
    row<1>("v_add_f32");
    row<1>("v_add_f32");
    row<2>("v_mul_f32");
    row<3>("v_exp_f32");
    row<4>("v_cvt_f32_i32");
    row<5>("v_max_f32");
    row<6>("v_perm_b32");
    row<7>("v_cvt_pk_f16_f32");
    row<8>("v_fmac_f32");
    row<9>("v_pk_fma_f32");
    row<10>("v_pk_add_f32");
    row<11>("v_sub_f32");
    row<12>("v_mov_b32");
    row<13>("v_max3_i32");
    row<14>("v_max_i32_dpp");
    row<15>("v_fma_mixlo_f16");
    row<16>("v_max_i32");
    row<17>("permlane32_swap");
    row<18>("v_accvgpr_read");
    return 0;
}
