// qmha_kernels.hpp -- internal (non-ABI) launcher declarations shared by the kernel
// translation units and the C-ABI layer (qmha_api.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace qmha {

inline constexpr size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Tuning knob for benchmarking kernel geometries: env var "<waves>x<stages>" (e.g. "8x2")
// read once per variable; returns waves*10+stages, or 0 (= built-in default).
int tune_config(const char* env_name);

// ---- INT8 (fa_tc_int8_b) ---------------------------------------------------------------
struct Int8Workspace {
    int8_t* Qi;  // [B*H][N][D]  (test hook only: nullptr in the production carve)
    int8_t* Ki;  // [B*H][N][D]
    _Float16* Vh;  // [B*H][N/32][D][32]  quantised V as f16 integers (f16 operand slot order)
    float* sQ;   // [B*H][N/32]  (per-tensor mode: [B*H], one scale per head slice)
    float* sK;
    float* sV;
    uint32_t* slice_sync;  // per-tensor mode only: [2][3][B*H] slice absmax bits and part arrivals (qmha_pt_quant_kernel)
};
size_t int8_workspace_bytes(int B, int N, int H, int D, bool with_q = false);
Int8Workspace int8_carve(void* ws, int B, int N, int H, int D, bool with_q = false);
// v_mode 0: V to `vout` as int8 in the i8 operand order; 1: as f16 integers (main path)
// first_tensor = 1 skips Q (the main kernels quantise Q themselves); 0 quantises Q, K, V;
// num_tensors (default: all from first_tensor on) limits the roles launched (the standalone op)
hipError_t launch_quant_int8(const float* Q, const float* K, const float* V, const Int8Workspace& w, void* vout,
                             int v_mode, int B, int N, int H, int D, int d_model, hipStream_t stream,
                             int first_tensor = 0, int num_tensors = -1);
// ---- INT8 per-tensor mode (fa_tc_int8_pt) ----------------------------------------------
// layout: Ki, Vh as fa_tc_int8_b, then slice_sync [2][3][B*H] uint32, then sQ, sK, sV [B*H] each
size_t int8_pt_workspace_bytes(int B, int N, int H, int D);
Int8Workspace int8_pt_carve(void* ws, int B, int N, int H, int D);
// one pass: K / V quantised with their head-slice scales from registers, sQ (qmha_pt_quant_kernel)
// the per-tensor pre-pass's bounded wait in 100 MHz ticks (default 200000 = 2 ms; 0 forces the
// fallback); returns the previous value
long long set_pt_wait_ticks(long long ticks);
hipError_t launch_quant_int8_pt(const float* Q, const float* K, const float* V, const Int8Workspace& w, int B, int N,
                                int H, int D, int d_model, hipStream_t stream);
// the standalone op's per-tensor layout: X in the K role only (int8 rows, one scale per head slice)
hipError_t launch_quant_int8_pt_rows(const float* X, const Int8Workspace& w, int B, int N, int H, int D, int d_model,
                                     hipStream_t stream);
hipError_t launch_fa_int8_pt_main(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int D,
                                  int d_model, hipStream_t stream);
// Qf: the caller's fp32 Q (the main kernel quantises each Q group into its MFMA operand)
hipError_t launch_fa_int8_main(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int D,
                               int d_model, hipStream_t stream);
hipError_t launch_debug_qk_int32(const Int8Workspace& w, int N, int D, int bh, int32_t* S, hipStream_t stream);
// what the production int8 kernel computed (FL_DUMP instance): S [B*H][N][N] int32 (bias
// removed), Qi [B*H][N][D] (its in-register Q operand), sQ [B*H][N/32]
struct QkDump {
    int32_t* S;
    int8_t* Qi;
    float* sQ;
};
hipError_t launch_fa_int8_dump(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int D,
                               int d_model, QkDump dbg, hipStream_t stream);
hipError_t launch_fa_int8_pt_dump(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int D,
                                  int d_model, QkDump dbg, hipStream_t stream);

// ---- FP16 (fa_tc_v1a) ------------------------------------------------------------------
struct F16Workspace {
    _Float16* Qh;  // unused (nullptr): the main kernel converts Q in registers
    _Float16* Kh;  // [B*H][N][D]
    _Float16* Vt;  // [B*H][N/32][D][32]  (f16 operand slot order)
};
size_t f16_workspace_bytes(int B, int N, int H, int D);
F16Workspace f16_carve(void* ws, int B, int N, int H, int D);
hipError_t launch_convert_f16(const float* Q, const float* K, const float* V, const F16Workspace& w, int B, int N,
                              int H, int D, int d_model, hipStream_t stream);
hipError_t launch_fa_f16_main(const F16Workspace& w, const float* Qf, float* O, int B, int N, int H, int D, int d_model,
                              hipStream_t stream);

// ---- FP32 (fa: scalar VALU kernel; fa_mfma: the same contract on v_mfma_f32_32x32x2_f32) -----
hipError_t launch_fa_f32(const float* Q, const float* K, const float* V, float* O, int B, int N, int H, int D,
                         int d_model, bool mfma, hipStream_t stream);

// ---- unfused 3-kernel baseline (unfused.cu) --------------------------------------------
size_t unfused_workspace_bytes(int B, int N, int H, int D);
hipError_t launch_unfused(const float* Q, const float* K, const float* V, float* O, void* ws, int B, int N, int H,
                          int D, int d_model, hipStream_t stream);

}  // namespace qmha
