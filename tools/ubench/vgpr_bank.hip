// vgpr_bank.hip -- does the VGPR bank of an operand change a VALU instruction's issue cost on
// gfx950?  Each wave runs ITERS x 16 independent instructions (16 destinations, reuse distance
// 16) with hand-picked register numbers; bank = register number mod 4.  Reports cycles per
// wave64 instruction per SIMD with W waves per SIMD (s_memtime around the loop).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>
#include <vector>

#define ITERS 1024

// 16 instructions: dst v[20+i]; the form picks the sources per i
#define R(n) "v" #n
template <int FORM>
__device__ __forceinline__ void body() {
#define I16(F)                                                                                           \
    F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(8) F(9) F(10) F(11) F(12) F(13) F(14) F(15)
    // dst bank i, a bank i+1, b bank i+2 (all distinct); "same" forms put a in the dst bank
#define FMA_DIST(i) "v_fma_f32 v[20+" #i "], v[41+" #i "], v[64+((" #i "+2)&3)], v[20+" #i "]\n\t"
#define FMA_SAME(i) "v_fma_f32 v[20+" #i "], v[40+" #i "], v[64+((" #i "+2)&3)], v[20+" #i "]\n\t"
#define FMA_ALL(i) "v_fma_f32 v[20+" #i "], v[40+" #i "], v[64+(" #i "&3)], v[20+" #i "]\n\t"
#define FMAC_DIST(i) "v_fmac_f32 v[20+" #i "], v[41+" #i "], v[64+((" #i "+2)&3)]\n\t"
#define FMAC_SAME(i) "v_fmac_f32 v[20+" #i "], v[40+" #i "], v[64+((" #i "+2)&3)]\n\t"
#define FMA_SGPR(i) "v_fma_f32 v[20+" #i "], v[41+" #i "], s8, v[20+" #i "]\n\t"
#define FMAAK_DIST(i) "v_fmaak_f32 v[20+" #i "], v[41+" #i "], v[64+((" #i "+2)&3)], 0x4b400000\n\t"
#define FMAAK_SAME(i) "v_fmaak_f32 v[20+" #i "], v[40+" #i "], v[64+(" #i "&3)], 0x4b400000\n\t"
#define FMAAK_SGPR(i) "v_fma_f32 v[20+" #i "], v[41+" #i "], s8, v[64+((" #i "+2)&3)]\n\t"
#define ADD_DIST(i) "v_add_f32 v[20+" #i "], v[41+" #i "], v[64+((" #i "+2)&3)]\n\t"
#define ADD_SAME(i) "v_add_f32 v[20+" #i "], v[40+" #i "], v[64+(" #i "&3)]\n\t"
#define FMA3_NEW(i) "v_fma_f32 v[20+" #i "], v[41+" #i "], v[64+((" #i "+2)&3)], v[67-((" #i ")&3)]\n\t"
#define CLOB                                                                                              \
    "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", \
        "v35", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52",    \
        "v53", "v54", "v55", "v56", "v64", "v65", "v66", "v67", "s8"
    if constexpr (FORM == 0) asm volatile(I16(FMA_DIST) ::: CLOB);
    if constexpr (FORM == 1) asm volatile(I16(FMA_SAME) ::: CLOB);
    if constexpr (FORM == 2) asm volatile(I16(FMA_ALL) ::: CLOB);
    if constexpr (FORM == 3) asm volatile(I16(FMAC_DIST) ::: CLOB);
    if constexpr (FORM == 4) asm volatile(I16(FMAC_SAME) ::: CLOB);
    if constexpr (FORM == 5) asm volatile(I16(FMA_SGPR) ::: CLOB);
    if constexpr (FORM == 6) asm volatile(I16(FMAAK_DIST) ::: CLOB);
    if constexpr (FORM == 7) asm volatile(I16(FMAAK_SAME) ::: CLOB);
    if constexpr (FORM == 8) asm volatile(I16(FMAAK_SGPR) ::: CLOB);
    if constexpr (FORM == 9) asm volatile(I16(ADD_DIST) ::: CLOB);
    if constexpr (FORM == 10) asm volatile(I16(ADD_SAME) ::: CLOB);
    if constexpr (FORM == 11) asm volatile(I16(FMA3_NEW) ::: CLOB);
}

static const char* kNames[] = {"fma a,b,d banks distinct", "fma a==d bank", "fma a,b,d one bank",
                               "fmac distinct",            "fmac a==d bank", "fma a, sgpr, d",
                               "fmaak distinct",           "fmaak a,b same", "fma a, sgpr, b(no d)",
                               "add distinct",             "add same bank",  "fma a,b,c -> new d"};

template <int FORM>
__global__ __launch_bounds__(256) void k(float* out, unsigned long long* cyc) {
    asm volatile(
        "v_mov_b32 v20, 1.0\n\tv_mov_b32 v21, 1.0\n\tv_mov_b32 v22, 1.0\n\tv_mov_b32 v23, 1.0\n\t"
        "v_mov_b32 v24, 1.0\n\tv_mov_b32 v25, 1.0\n\tv_mov_b32 v26, 1.0\n\tv_mov_b32 v27, 1.0\n\t"
        "v_mov_b32 v28, 1.0\n\tv_mov_b32 v29, 1.0\n\tv_mov_b32 v30, 1.0\n\tv_mov_b32 v31, 1.0\n\t"
        "v_mov_b32 v32, 1.0\n\tv_mov_b32 v33, 1.0\n\tv_mov_b32 v34, 1.0\n\tv_mov_b32 v35, 1.0\n\t"
        "v_mov_b32 v40, 0.5\n\tv_mov_b32 v41, 0.5\n\tv_mov_b32 v42, 0.5\n\tv_mov_b32 v43, 0.5\n\t"
        "v_mov_b32 v44, 0.5\n\tv_mov_b32 v45, 0.5\n\tv_mov_b32 v46, 0.5\n\tv_mov_b32 v47, 0.5\n\t"
        "v_mov_b32 v48, 0.5\n\tv_mov_b32 v49, 0.5\n\tv_mov_b32 v50, 0.5\n\tv_mov_b32 v51, 0.5\n\t"
        "v_mov_b32 v52, 0.5\n\tv_mov_b32 v53, 0.5\n\tv_mov_b32 v54, 0.5\n\tv_mov_b32 v55, 0.5\n\t"
        "v_mov_b32 v56, 0.5\n\tv_mov_b32 v64, 0.5\n\tv_mov_b32 v65, 0.5\n\tv_mov_b32 v66, 0.5\n\t"
        "v_mov_b32 v67, 0.5\n\ts_mov_b32 s8, 0.5" ::: CLOB);
    unsigned long long t0, t1;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    for (int i = 0; i < ITERS; ++i) body<FORM>();
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    float r;
    asm volatile("v_add_f32 %0, v20, v35" : "=v"(r)::CLOB);
    out[blockIdx.x * 256 + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int FORM>
void run(int w) {
    const int nb = 256 * w;
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, nb * 256 * 4);
    hipMalloc(&cyc, nb * 4 * 8);
    hipLaunchKernelGGL(k<FORM>, dim3(nb), dim3(256), 0, 0, out, cyc);
    hipLaunchKernelGGL(k<FORM>, dim3(nb), dim3(256), 0, 0, out, cyc);
    hipDeviceSynchronize();
    std::vector<unsigned long long> c(nb * 4);
    hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
    double avg = 0;
    for (auto v : c) avg += v;
    avg /= c.size();
    std::printf("%-26s waves/SIMD=%d  cycles/instr/SIMD=%.2f\n", kNames[FORM], w, avg / (16.0 * ITERS * w));
    hipFree(out);
    hipFree(cyc);
}

template <int F>
void all(int w) {
    run<F>(w);
    if constexpr (F + 1 < 12) all<F + 1>(w);
}

int main() {
    for (int w : {1, 2, 3, 4}) all<0>(w);
    return 0;
}
