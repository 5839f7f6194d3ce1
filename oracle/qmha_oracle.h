/*
 * qmha_oracle.h -- CPU restatement of the reference's attention algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in quantizedmha_amd/ (the product) may
 * include, link or call this code; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker.
 *
 * Every function restates one reference routine (MattJBorowski1991/QuantizedMHA,
 * snapshot mounted at /root/reference) and cites the file:line it follows.
 * All tensors are fp32 row-major [B][N][d_model] (batch outermost); head k owns
 * columns [k*d, (k+1)*d) with d = d_model / h (include/launchers.h:42,50-52).
 *
 * Pinning (see DESIGN.md "Oracle"):
 *  - oracle_cpu_reference_rope is checked bit-for-bit against the reference's own
 *    utils/verify.cu compiled from /root/reference into oracle/_ref/.
 *  - oracle_cpu_attention is checked against tests/generate_golden.cpp's cpu_mha
 *    golden vectors (tests/golden/*), produced by the reference generator itself.
 *  - oracle_fa_fp32 / oracle_fa_fp16 / oracle_fa_int8 restate the kernels'
 *    per-block algorithms (the reference kernels are CUDA and cannot run here);
 *    they are pinned by the reference's all-ones KAT (drivers/main.cu:73-101), by
 *    convergence to cpu_mha goldens, and -- for int8 -- by exact integer checks.
 *    Beyond that the int8 restatement is "parity unpinned" (SURVEY.md 8c).
 */
#ifndef QMHA_ORACLE_H
#define QMHA_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* utils/verify.cu:25-104 -- MHA with RoPE applied to q_i and k_j, single thread,
 * one batch element.  Bit-exact with the reference build (same libm, no FMA). */
void oracle_cpu_reference_rope(const float *Q, const float *K, const float *V, float *out,
                               int N, int d_model, int h);

/* utils/verify.cu:153-172 -- returns index of first mismatch, or -1 if all match
 * (non-finite values count as mismatch). */
long oracle_verify_results(const float *got, const float *ref, size_t n, float eps, float rel);

/* tests/generate_golden.cpp:53-92 (cpu_mha) -- plain softmax(QK^T/sqrt(d))V, no RoPE. */
void oracle_cpu_attention(const float *Q, const float *K, const float *V, float *out,
                          int B, int N, int d_model, int h, int nthreads);

/* mha_kernels/fa_tc_int8_b.cu:33-152 (fp32_to_int8sram) -- symmetric absmax
 * quantisation of one rows x cols block (leading dimension ld).  Writes dst
 * row-major with leading dimension ldd and returns the scale. */
float oracle_quantize_block(const float *src, int rows, int cols, int ld, int8_t *dst, int ldd);

/* Quantise every 32-row group of every head: Xi[B][h][N][d] int8, scales[B][h][N/32]. */
void oracle_quantize_heads(const float *X, int B, int N, int d_model, int h,
                           int8_t *Xi, float *scales);

/* Integer Q_int8 @ K_int8^T for one head: S[N][N] int32 (exact). */
void oracle_qk_int32(const int8_t *Qi, const int8_t *Ki, int N, int d, int32_t *S);

/* mha_kernels/fa_tc_int8_b.cu:247-579, intended semantics:
 * per-32-row-group int8 Q/K/V, per 32x32 tile int8 P, int32 products, fp32
 * online softmax with m0 = 0. */
void oracle_fa_int8(const float *Q, const float *K, const float *V, float *out,
                    int B, int N, int d_model, int h, int nthreads);

/* Per-tensor int8 mode (fa_tc_int8_pt, not a reference kernel; see qmha_oracle.c): each
 * head's [N, d] slice quantised with one scale (the fp32_to_int8sram arithmetic over the
 * whole slice); scales[B][h]. */
void oracle_quantize_heads_pt(const float *X, int B, int N, int d_model, int h,
                              int8_t *Xi, float *scales);
/* fa_tc_int8_pt: per-head-slice int8 Q/K/V, static P scale 1/127, int32 products, fp32
 * online softmax with m0 = 0, O = alpha*O + (Pi.Vi), out = O*(sV/127)/l. */
void oracle_fa_int8_pt(const float *Q, const float *K, const float *V, float *out,
                       int B, int N, int d_model, int h, int nthreads);

/* mha_kernels/fa_tc_v1a.cu:101-413 -- fp16 (RNE) operands, fp32 accumulation,
 * P stored as half(p), m0 = 0, epilogue guard 1e-10. */
void oracle_fa_fp16(const float *Q, const float *K, const float *V, float *out,
                    int B, int N, int d_model, int h, int nthreads);
/* The fp16 GPU kernel's contract (r06): the above in base 2 with a lazy softmax base (moves only when a
 * row's tile max passes it by > 8 log2 units); differs from oracle_fa_fp16 in the rounding of half(p). */
void oracle_fa_fp16_lazy(const float *Q, const float *K, const float *V, float *out,
                         int B, int N, int d_model, int h, int nthreads);

/* mha_kernels/fa.cu:24-400 -- fp32 scalar FlashAttention, fmaf dot products
 * (nvcc contracts acc += a*b), m0 = 0, Bc = 32, epilogue guard 1e-10. */
void oracle_fa_fp32(const float *Q, const float *K, const float *V, float *out,
                    int B, int N, int d_model, int h, int nthreads);

/* __float2half (round to nearest even) and back. */
uint16_t oracle_f32_to_f16(float x);
float oracle_f16_to_f32(uint16_t hbits);

/* inputs/data.cu:9-30 is mt19937-based; restated by tests via numpy.  This helper
 * fills an all-ones input (the driver's correctness-check data, data.cu:24-28). */
void oracle_fill_ones(float *x, size_t n);

#ifdef __cplusplus
}
#endif
#endif
