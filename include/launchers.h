/*
 * launchers.h -- C-ABI of the MI355X-native quantized multi-head attention library.
 *
 * Drop-in for the reference's include/launchers.h (MattJBorowski1991/QuantizedMHA).
 * Plain C types only: device pointers, sizes and an opaque stream handle (hipStream_t
 * passed as void*), so cgo/ctypes/JNI/N-API bindings need no HIP or torch headers.
 *
 * Libraries (built by tools/build.py):
 *   libqmha.so                 every entry point below; `solve` bound to fa_tc_int8_b
 *   libqmha_fa_tc_int8_b.so    `solve` bound to the INT8 path      (make KERNEL=fa_tc_int8_b)
 *   libqmha_fa_tc_v1a.so       `solve` bound to the FP16 MFMA path (make KERNEL=fa_tc_v1a)
 *   libqmha_fa.so              `solve` bound to the scalar path    (make KERNEL=fa)
 *   libqmha_fa_mfma.so         `solve` bound to fa's contract on the fp32 matrix cores
 *   libqmha_unfused.so         `solve` bound to the 3-kernel path  (make KERNEL=unfused)
 *   libqmha_fa_tc_int8_pt.so   `solve` bound to the per-tensor int8 mode (no reference kernel)
 * mirroring the reference's one-kernel-per-binary build (Makefile:39-53,
 * extensions/torch/setup.py:21-43).
 */
#ifndef QMHA_LAUNCHERS_H
#define QMHA_LAUNCHERS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Kernel variants (names as in the reference's mha_kernels/ and setup.py:114-124). */
typedef enum {
    QMHA_FA = 0,           /* mha_kernels/fa.cu         : fp32 scalar, no matrix cores   */
    QMHA_FA_TC_V1A = 1,    /* mha_kernels/fa_tc_v1a.cu  : fp16 MFMA, fp32 accumulation   */
    QMHA_FA_TC_INT8_B = 2, /* mha_kernels/fa_tc_int8_b.cu: int8 MFMA, per-32-row scales  */
    QMHA_UNFUSED = 3,      /* mha_kernels/unfused.cu    : QK^T, softmax, PV (3 kernels)   */
    QMHA_FA_MFMA = 4,      /* fa.cu's fp32 contract on v_mfma_f32_32x32x2_f32 (no reference
                              counterpart: the matrix-core sibling of the scalar `fa`)    */
    QMHA_FA_TC_INT8_PT = 5 /* per-tensor int8 mode (no reference counterpart: BASELINE.json's
                              "per-tensor Q/K/V quant", SURVEY 0.2's optional flag): one scale
                              per head slice of Q/K/V, static P scale 1/127, O accumulated on
                              the matrix core                                              */
} qmha_variant_t;

/* Status codes of the extended entry points. */
enum {
    QMHA_OK = 0,
    QMHA_ERR_INVALID = 1, /* shape/argument precondition failed (checked before launch) */
    QMHA_ERR_HIP = 2,     /* a HIP runtime call or kernel launch failed                  */
    QMHA_ERR_NOMEM = 3,   /* workspace allocation failed                                 */
    QMHA_ERR_NOSYS = 4    /* variant / head size not built into this library             */
};

/*
 * solve -- replaces the reference's `extern "C" void solve(...)` declared at
 * include/launchers.h:9-10 and defined per kernel (e.g. mha_kernels/fa_tc_int8_b.cu:600-609).
 *
 * Q, K, V, output: DEVICE pointers, fp32, contiguous [N, d_model] row-major; head k owns
 * columns [k*d, (k+1)*d), d = d_model / h.  output is fully overwritten.
 * Blocking: the result is complete on return (reference launchers.h:64).  Scratch is
 * owned by the library.  Preconditions (the reference asserts N % 32 on the device,
 * fa_tc_int8_b.cu:422-423): N % 32 == 0, d_model == h*d, d % 32 == 0 (config.h:32) and d <= 256
 * (fa_tc_int8_pt, the per-tensor mode with no reference counterpart: d in {32, 64, 128}).  The
 * reference's d is a compile-time constant (config.h:28); here it is a runtime value.
 * On a violated precondition or HIP error `solve` prints one line to stderr and returns
 * (the reference returns void and ignores errors).
 */
void solve(const float *Q, const float *K, const float *V, float *output, int N, int d_model, int h);

/*
 * qmha_solve_ex -- batched, asynchronous, status-returning form of `solve`.
 * Q/K/V/O are [B, N, d_model] fp32 device tensors (batch outermost; B calls of the
 * reference `solve`).  Work is enqueued on `stream` (hipStream_t, NULL = default stream)
 * and the call returns without synchronising.  A library-owned workspace is cached per
 * (device, stream); see qmha_solve_ws for caller-owned scratch (graph capture).
 */
int qmha_solve_ex(const float *Q, const float *K, const float *V, float *O, int B, int N, int d_model, int h,
                  int variant, void *stream);

/* Bytes of scratch qmha_solve_ws needs for this problem (0 for variants without). */
size_t qmha_workspace_size(int B, int N, int d_model, int h, int variant);

/* As qmha_solve_ex with caller-owned device scratch of >= qmha_workspace_size bytes
 * (256-byte aligned).  Makes no allocation and no synchronisation: capturable in a hipGraph. */
int qmha_solve_ws(const float *Q, const float *K, const float *V, float *O, int B, int N, int d_model, int h,
                  int variant, void *workspace, size_t workspace_bytes, void *stream);

/* Blocking convenience used by the per-variant `solve` shims and the JAX raw-pointer
 * binding (extensions/jax/jax_ext.cpp:12-28): batch 1, synchronises the device stream. */
int qmha_solve_variant(const float *Q, const float *K, const float *V, float *O, int N, int d_model, int h,
                       int variant);

/*
 * qmha_quantize_int8 -- the INT8 path's pre-pass as a standalone op:
 * per 32-row group of every head, scale = max(absmax/127, 1e-8) and
 * x_i8 = clamp(rint(x / scale), -128, 127) (fa_tc_int8_b.cu:33-152, fp32_to_int8sram).
 * X: [B, N, d_model] fp32 device.  Xi: [B][h][N][d] int8 device.  scales: [B][h][N/32].
 * layout 0 = row-major rows (Q, K operand); layout 1 = V^T MFMA operand order
 * ([B][h][N/32][d][32], kv slots permuted as documented in DESIGN.md); layout 2 = row-major rows
 * with ONE scale per head slice (the fa_tc_int8_pt per-tensor mode; scales: [B][h]).
 */
int qmha_quantize_int8(const float *X, int B, int N, int d_model, int h, int8_t *Xi, float *scales, int layout,
                       void *stream);

/*
 * qmha_debug_qk_int32 -- test hook for the bit-exact KAT: quantises Q and K exactly as the
 * INT8 path does and writes S = Q_i8 K_i8^T (int32) of head `head` (batch 0) computed by
 * the same v_mfma_i32_32x32x32_i8 operand path into S[N][N] (device).  Blocking.
 */
int qmha_debug_qk_int32(const float *Q, const float *K, int N, int d_model, int h, int head, int32_t *S);

/*
 * Test hook (the bit-exact int32 Q@K^T check, reference fa_tc_int8_b.cu:484,496,514):
 * runs the PRODUCTION int8 schedule (same kernel template and flags as qmha_solve_ex, plus the
 * FL_DUMP stores) and writes what that kernel itself computed: O as qmha_solve_ex would, the
 * int32 S = Qi Ki^T of every (sequence, head) as its MFMAs produced it (accumulator bias
 * removed) into S[B*h][N][N], its in-register int8 Q operand into Qi[B*h][N][d] and the Q
 * group scales into sQ[B*h][N/32].  N >= 64.  Device pointers; blocking.
 */
int qmha_debug_fa_int8_dump(const float *Q, const float *K, const float *V, float *O, int B, int N, int d_model,
                            int h, int32_t *S, int8_t *Qi, float *sQ);

/* As qmha_debug_fa_int8_dump for the per-tensor mode (QMHA_FA_TC_INT8_PT): its production schedule
 * plus the stores; Qi is quantised with the head slice's scale, and sQ[B*h][N/32] holds that one
 * scale in every group's entry.  N >= 32.  Device pointers; blocking. */
int qmha_debug_fa_int8_pt_dump(const float *Q, const float *K, const float *V, float *O, int B, int N, int d_model,
                               int h, int32_t *S, int8_t *Qi, float *sQ);

/* Test hook: bound, in ticks of the 100 MHz real-time clock, of the per-tensor pre-pass's wait for the
 * other parts of a head slice (default 200000 = 2 ms; 0 makes every part take its fallback, reducing
 * the whole slice itself; negative makes every call take the two-pass form that slices of more parts
 * than one XCD holds at once always take -- the same scales, bit-identical output).  Returns the
 * previous bound. */
int64_t qmha_debug_set_pt_wait(int64_t ticks);

/* Variant name ("fa", "fa_tc_v1a", "fa_tc_int8_b", "unfused", "fa_mfma", "fa_tc_int8_pt") -> id, or -1. */
int qmha_variant_from_name(const char *name);
const char *qmha_variant_name(int variant);
const char *qmha_status_string(int status);
const char *qmha_version(void);
/* Last HIP error string recorded by a failing call on this thread ("" if none). */
const char *qmha_last_error(void);

/*
 * Kernel timing for roofline reporting (bench.py): when enabled, qmha_solve_* record a
 * hipEvent pair around every launch of the dominant ("main") kernel and of the pre-pass.
 * The int8 and fp16 paths split a call into batch chunks whose pre-pass runs on a library
 * stream, overlapped with the previous chunk's main kernel (qmha_set_overlap_chunks, default 1 = off).
 * qmha_profile_collect synchronises those events and returns the summed main-kernel and
 * pre-pass milliseconds and the number of calls since the last collect, then clears the record.
 */
void qmha_profile_enable(int on);
/* Number of batch chunks for the pre-pass / main-kernel overlap (1..16, 1 = off); returns the
 * previous value.  Results are bit-identical for every setting. */
int qmha_set_overlap_chunks(int n);
int qmha_profile_collect(double *main_ms, long long *launches, double *prepass_ms);

/* Release all library-owned workspaces (optional; also released at process exit). */
void qmha_release_workspaces(void);

#ifdef __cplusplus
}
#endif
#endif /* QMHA_LAUNCHERS_H */
