// valu_rate.hip -- gfx950 VALU issue-rate microbenchmark (cycles per wave64 instruction per
// SIMD) for the instructions that dominate the attention softmax.  Each wave runs ITERS x 8
// independent instructions of one kind between two s_memtime stamps; with W waves per SIMD
// resident the SIMD's cost per instruction = cycles / (W * instructions per wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define ITERS 2048

#define BODY8(INS)                                                                      \
    asm volatile(INS " %0, %8\n\t" INS " %1, %8\n\t" INS " %2, %8\n\t" INS " %3, %8\n\t"     \
                 INS " %4, %8\n\t" INS " %5, %8\n\t" INS " %6, %8\n\t" INS " %7, %8"           \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x))
#define BODY8_2(INS)                                                                        \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" \
                 INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"     \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x))
#define BODY8_PK(INS)                                                                       \
    asm volatile(INS " %0, %0, %8, %8\n\t" INS " %1, %1, %8, %8\n\t" INS " %2, %2, %8, %8\n\t" \
                 INS " %3, %3, %8, %8"                                                            \
                 : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "v"(y))
#define BODY8_PK2(INS)                                                                      \
    asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8" \
                 : "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3) : "v"(y))
#define BODY8_3(INS)                                                                        \
    asm volatile(INS " %0, %0, %8, %8\n\t" INS " %1, %1, %8, %8\n\t" INS " %2, %2, %8, %8\n\t" \
                 INS " %3, %3, %8, %8\n\t" INS " %4, %4, %8, %8\n\t" INS " %5, %5, %8, %8\n\t" \
                 INS " %6, %6, %8, %8\n\t" INS " %7, %7, %8, %8"                                \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x))

template <int OP>
__global__ __launch_bounds__(256) void k(float* out, unsigned long long* cyc, float seed) {
    float a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
          a7 = seed + 7, x = seed * 0.5f;
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 b0 = {seed, seed}, b1 = {seed, 1}, b2 = {2, seed}, b3 = {3, 3}, y = {x, x};
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int i = 0; i < ITERS; ++i) {
        if constexpr (OP == 0) BODY8("v_cvt_f32_i32");
        if constexpr (OP == 1) BODY8_3("v_fma_f32");
        if constexpr (OP == 2) BODY8("v_exp_f32");
        if constexpr (OP == 3) BODY8_3("v_perm_b32");
        if constexpr (OP == 4) BODY8_3("v_max3_i32");
        if constexpr (OP == 5) BODY8_2("v_add_f32");
        if constexpr (OP == 6) BODY8_2("v_mul_f32");
        if constexpr (OP == 7) BODY8("v_rcp_f32");
        if constexpr (OP == 8) BODY8("v_mov_b32");
        if constexpr (OP == 9) { BODY8_PK("v_pk_fma_f32"); BODY8_PK("v_pk_fma_f32"); }
        if constexpr (OP == 10) { BODY8_PK2("v_pk_mul_f32"); BODY8_PK2("v_pk_mul_f32"); }
        if constexpr (OP == 11) BODY8_2("v_fmac_f32");
        if constexpr (OP == 12) BODY8_2("v_cvt_pk_f16_f32");
        if constexpr (OP == 13) BODY8_2("v_sub_f32");
        if constexpr (OP == 14) BODY8_2("v_max_f32");
        if constexpr (OP == 15) BODY8_2("v_max_i32");
        if constexpr (OP == 16) BODY8_3("v_fma_mixlo_f16");
#define PLBODY(INS)                                                                                  \
    asm volatile(INS " %0, %1\n\t" INS " %2, %3\n\t" INS " %4, %5\n\t" INS " %6, %7\n\t" INS " %1, %2\n\t" \
                 INS " %3, %4\n\t" INS " %5, %6\n\t" INS " %7, %0"                                             \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7))
        if constexpr (OP == 17) PLBODY("v_permlane32_swap_b32");
        if constexpr (OP == 18) PLBODY("v_permlane16_swap_b32");
        if constexpr (OP == 19) {
#define DPP(i) "v_max_i32_dpp %" #i ", %" #i ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
            asm volatile(DPP(0) DPP(1) DPP(2) DPP(3) DPP(4) DPP(5) DPP(6) DPP(7)
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
        }
        if constexpr (OP == 20) {  // dependent chain: every fma reads the previous result
            asm volatile("v_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\t"
                         "v_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1"
                         : "+v"(a0) : "v"(x));
        }
        if constexpr (OP == 21) {  // dependent chain of exp
            asm volatile("v_exp_f32 %0, %0\n\tv_exp_f32 %0, %0\n\tv_exp_f32 %0, %0\n\tv_exp_f32 %0, %0\n\t"
                         "v_exp_f32 %0, %0\n\tv_exp_f32 %0, %0\n\tv_exp_f32 %0, %0\n\tv_exp_f32 %0, %0"
                         : "+v"(a0));
        }
        if constexpr (OP == 22) {  // cvt -> fma -> exp dependent triples, 8 per iteration (as the tile code)
            asm volatile("v_cvt_f32_i32 %0, %0\n\tv_fma_f32 %0, %0, %8, %8\n\tv_exp_f32 %0, %0\n\t"
                         "v_cvt_f32_i32 %1, %1\n\tv_fma_f32 %1, %1, %8, %8\n\tv_exp_f32 %1, %1\n\t"
                         "v_cvt_f32_i32 %2, %2\n\tv_fma_f32 %2, %2, %8, %8\n\tv_exp_f32 %2, %2\n\t"
                         "v_cvt_f32_i32 %3, %3\n\tv_fma_f32 %3, %3, %8, %8\n\tv_exp_f32 %3, %3\n\t"
                         "v_cvt_f32_i32 %4, %4\n\tv_fma_f32 %4, %4, %8, %8\n\tv_exp_f32 %4, %4\n\t"
                         "v_cvt_f32_i32 %5, %5\n\tv_fma_f32 %5, %5, %8, %8\n\tv_exp_f32 %5, %5\n\t"
                         "v_cvt_f32_i32 %6, %6\n\tv_fma_f32 %6, %6, %8, %8\n\tv_exp_f32 %6, %6\n\t"
                         "v_cvt_f32_i32 %7, %7\n\tv_fma_f32 %7, %7, %8, %8\n\tv_exp_f32 %7, %7"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
        }
        if constexpr (OP == 23) {  // same 24 instructions, phase-separated (independent neighbours)
            asm volatile("v_cvt_f32_i32 %0, %0\n\tv_cvt_f32_i32 %1, %1\n\tv_cvt_f32_i32 %2, %2\n\tv_cvt_f32_i32 %3, %3\n\t"
                         "v_cvt_f32_i32 %4, %4\n\tv_cvt_f32_i32 %5, %5\n\tv_cvt_f32_i32 %6, %6\n\tv_cvt_f32_i32 %7, %7\n\t"
                         "v_fma_f32 %0, %0, %8, %8\n\tv_fma_f32 %1, %1, %8, %8\n\tv_fma_f32 %2, %2, %8, %8\n\tv_fma_f32 %3, %3, %8, %8\n\t"
                         "v_fma_f32 %4, %4, %8, %8\n\tv_fma_f32 %5, %5, %8, %8\n\tv_fma_f32 %6, %6, %8, %8\n\tv_fma_f32 %7, %7, %8, %8\n\t"
                         "v_exp_f32 %0, %0\n\tv_exp_f32 %1, %1\n\tv_exp_f32 %2, %2\n\tv_exp_f32 %3, %3\n\t"
                         "v_exp_f32 %4, %4\n\tv_exp_f32 %5, %5\n\tv_exp_f32 %6, %6\n\tv_exp_f32 %7, %7"
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x));
        }
    }
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0.x + b1.y + b2.x + b3.y;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char* name, int blocks_per_cu) {
    const int nb = 256 * blocks_per_cu;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, nb * 256 * 4);
    hipMalloc(&cyc, nb * 4 * 8);
    hipLaunchKernelGGL(k<OP>, dim3(nb), dim3(256), 0, 0, out, cyc, 1.0f);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(nb), dim3(256), 0, 0, out, cyc, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(nb * 4);
    hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (auto v : c) avg += v;
    avg /= c.size();
    const double waves_per_simd = blocks_per_cu;  // 4 waves per block, one per SIMD
    const double instr = (OP == 22 || OP == 23 ? 24.0 : 8.0) * ITERS;
    std::printf("%-16s waves/SIMD=%d  cycles/instr/SIMD=%.2f  (wall %.3f ms, wave cycles %.0f)\n", name, blocks_per_cu,
                avg / (instr * waves_per_simd), ms, avg);
    hipFree(out);
    hipFree(cyc);
}

int main(int argc, char** argv) {
    if (argc > 1) {  // extended set only
        for (int w : {1, 2, 4}) {
            run<17>("permlane32_swap", w);
            run<18>("permlane16_swap", w);
            run<19>("v_max_i32_dpp", w);
            run<20>("fma dep chain", w);
            run<21>("exp dep chain", w);
            run<22>("cvt-fma-exp chains", w);
            run<23>("cvt|fma|exp phased", w);
            run<1>("v_fma_f32", w);
            run<2>("v_exp_f32", w);
            run<9>("v_pk_fma_f32", w);
            run<12>("v_cvt_pk_f16_f32", w);
        }
        return 0;
    }
    for (int w : {4, 8}) {
        run<0>("v_cvt_f32_i32", w);
        run<1>("v_fma_f32", w);
        run<2>("v_exp_f32", w);
        run<3>("v_perm_b32", w);
        run<4>("v_max3_i32", w);
        run<5>("v_add_f32", w);
        run<6>("v_mul_f32", w);
        run<7>("v_rcp_f32", w);
        run<8>("v_mov_b32", w);
        run<9>("v_pk_fma_f32", w);
        run<10>("v_pk_mul_f32", w);
        run<11>("v_fmac_f32", w);
        run<12>("v_cvt_pk_f16_f32", w);
        run<13>("v_sub_f32", w);
        run<14>("v_max_f32", w);
        run<15>("v_max_i32", w);
    }
    return 0;
}
