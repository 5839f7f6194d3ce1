// qmha_prepass.hip -- the K/V pre-passes of the int8 and fp16 paths (and the standalone
// qmha_quantize_int8 op), in a translation unit of their own: they read the caller's Q/K/V, so they
// keep IEEE NaN semantics (the main-kernel sources are built with -fno-honor-nans, round-2 ADVICE).
//   qmha_quant_int8_kernel  fa_tc_int8_b.cu:33-152 (fp32_to_int8sram): per 32-row group of every
//                           head, sc = max(absmax/127, 1e-8), x_i8 = clamp(rint(x * (1/sc))) --
//                           K as int8 rows, V as f16-valued integers in the MFMA V^T operand order
//   qmha_convert_f16_kernel fa_tc_v1a.cu:300-330: K as f16 rows, V in the f16 V^T operand order (RNE)
#include "qmha_common.hpp"
#include "qmha_kernels.hpp"

namespace qmha {

#ifndef QMHA_PRE_NT
#define QMHA_PRE_NT 1
#endif
#if QMHA_PRE_NT
#define QMHA_PRE_LOAD(p) __builtin_nontemporal_load(p)
#else
#define QMHA_PRE_LOAD(p) (*(p))
#endif
// ---------------------------------------------------------------------------------------
// Pre-pass: quantise Q, K, V (fa_tc_int8_b.cu:33-152, fp32_to_int8sram).
// One wave per (tensor, bh, group); blockIdx.y = tensor (0 Q, 1 K, 2 V).
// v_mode 0: V as int8 in the i8 V^T operand order (qmha_quantize_int8 layout 1)
// v_mode 1: V as f16-valued integers in the f16 V^T operand order (main kernel input)
// ---------------------------------------------------------------------------------------
// One wave quantises one 32-row group of V (b, k, g) into the V^T operand order through its
// LDS tile `vtr` (D * QMHA_VT_PITCH bytes): coalesced 16-byte loads (instruction i covers rows
// i, NI+i, ...: 256-byte row segments), so lane (rq, c4) holds NI CONSECUTIVE rows of columns
// 4 c4..4 c4+3.  In the slot order consecutive kv rows 4a..4a+3 are 4 consecutive slots
// (kv_of_slot_f16), so each column of the lane is 8-byte ds_write_b64 pieces; the [d][32] tile
// is read back in 8-byte pieces and stored as 16-byte lines.  Loads are non-temporal: fp32
// K/V are read exactly once per call.
// v_mode 0: V as int8 in the i8 V^T operand order (qmha_quantize_int8 layout 1)
// v_mode 1: V as f16-valued integers in the f16 V^T operand order (main kernel input)
// slice_sc > 0: per-tensor mode, quantise with that scale (no per-group scale stored)
template <int D, int VMODE>
__device__ __forceinline__ void quant_v_group(const float* __restrict__ V, void* __restrict__ Vout,
                                              float* __restrict__ sV, char* vtr, int lane, int b, int k, int g,
                                              int bh, int N, int G, int d_model, float slice_sc = 0.0f) {
    constexpr int C4 = D / 4, NI = 32 / (64 / C4);
    const int rq = lane / C4, c4 = lane % C4;  // rows NI*rq .. NI*rq+NI-1, columns 4 c4 .. +3
    v4f x[NI];
    float amax = 0.0f;
    const float* base = V + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D + 4 * c4;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        x[i] = QMHA_PRE_LOAD(reinterpret_cast<const v4f*>(base + (size_t)(NI * rq + i) * d_model));
#pragma unroll
        for (int c = 0; c < 4; ++c) amax = fmaxf(amax, fabsf(x[i][c]));
    }
    const float sc = slice_sc > 0.0f ? slice_sc : qmha_scale_from_absmax(wave_max64(amax));
    const float inv = 1.0f / sc;
    if constexpr (VMODE == 1)
        vt_group_store<D, true>(vtr, x, inv, lane, static_cast<char*>(Vout) + ((size_t)bh * G + g) * (size_t)(64 * D));
    else
        vt8_group_store<D>(vtr, x, inv, lane, static_cast<char*>(Vout) + ((size_t)bh * G + g) * (size_t)(32 * D));
    if (lane == 0 && slice_sc == 0.0f) sV[(size_t)bh * G + g] = sc;
}

// Per-tensor mode (fa_tc_int8_pt): the scale of a head's whole [N, d] slice from the absmax of
// its G 32-row groups (qmha_group_absmax_kernel): max is exact in any order, so this equals the
// fp32_to_int8sram arithmetic over the whole slice (fa_tc_int8_b.cu:56-106).  One wave per
// (tensor, bh) slice reads its G group maxima once and writes the slice scale to s{Q,K,V}[bh]
// (round-3 ADVICE: every quantising wave used to re-reduce all G maxima of its slice, G^2 reads
// per slice -- 16 MB per slice and tensor at N = 65536).
__global__ __launch_bounds__(256) void qmha_slice_scale_kernel(const float* __restrict__ gmax, float* __restrict__ sQ,
                                                               float* __restrict__ sK, float* __restrict__ sV, int BH,
                                                               int G, int first_tensor) {
    const int tensor = blockIdx.y + first_tensor;
    const int lane = threadIdx.x & 63;
    const int bh = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (bh >= BH) return;  // wave-uniform
    const float* gm = gmax + ((size_t)tensor * BH + bh) * G;
    float m = 0.0f;
    for (int i = lane; i < G; i += 64) m = fmaxf(m, gm[i]);
    const float sc = qmha_scale_from_absmax(wave_max64(m));
    float* s_out = tensor == 0 ? sQ : (tensor == 1 ? sK : sV);
    if (lane == 0 && s_out) s_out[bh] = sc;
}

// One wave quantises one 32-row group of Q or K (b, k, g) into int8 rows [bh][N][D].
template <int D>
__device__ __forceinline__ void quant_row_group(const float* __restrict__ X, int8_t* __restrict__ Xi,
                                                float* __restrict__ sX, int lane, int b, int k, int g, int bh, int N,
                                                int G, int d_model, float slice_sc = 0.0f) {
    constexpr int C4 = D / 4, RPI = 64 / C4, NI = 32 / RPI;
    const int ri = lane / C4, ci = lane % C4;
    v4f v[NI];
    float amax = 0.0f;
    const float* base = X + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D + 4 * ci;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        v[i] = QMHA_PRE_LOAD(reinterpret_cast<const v4f*>(base + (size_t)(i * RPI + ri) * d_model));
#pragma unroll
        for (int c = 0; c < 4; ++c) amax = fmaxf(amax, fabsf(v[i][c]));
    }
    const float sc = slice_sc > 0.0f ? slice_sc : qmha_scale_from_absmax(wave_max64(amax));  // :104
    const float inv = 1.0f / sc;                                                            // :106 (correctly rounded)
    int8_t* dst = Xi + ((size_t)bh * N + (size_t)g * QMHA_GROUP) * D + 4 * ci;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) w |= ((uint32_t)(uint8_t)qmha_quant_i8(v[i][c], inv)) << (8 * c);
        *reinterpret_cast<uint32_t*>(dst + (size_t)(i * RPI + ri) * D) = w;
    }
    if (lane == 0 && slice_sc == 0.0f) sX[(size_t)bh * G + g] = sc;
}

// ---------------------------------------------------------------------------------------
// Pre-pass: quantise Q, K, V (fa_tc_int8_b.cu:33-152, fp32_to_int8sram).
// One wave per (tensor, bh, group); blockIdx.y = tensor (0 Q, 1 K, 2 V).
// ---------------------------------------------------------------------------------------
// PT (per-tensor mode): every group of a head slice is quantised with the slice's scale, read from
// s{K,V}[bh] (qmha_slice_scale_kernel)
template <int D, int VMODE, bool PT = false>
__global__ __launch_bounds__(256) void qmha_quant_int8_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
    int8_t* __restrict__ Qi, int8_t* __restrict__ Ki, void* __restrict__ Vout,
    float* __restrict__ sQ, float* __restrict__ sK, float* __restrict__ sV,
    int N, int H, int d_model, int total_groups, int first_tensor) {
    __shared__ __attribute__((aligned(16))) char vtr[4][D * QMHA_VT_PITCH];
    const int tensor = blockIdx.y + first_tensor;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int item = blockIdx.x * 4 + wave;  // (bh, g)
    if (item >= total_groups) return;        // wave-uniform
    const int G = N / QMHA_GROUP;
    const int bh = item / G, g = item % G;
    const int b = bh / H, k = bh % H;
    float slice_sc = 0.0f;
    if constexpr (PT) slice_sc = (tensor == 0 ? sQ : (tensor == 1 ? sK : sV))[bh];
    if (tensor == 2)
        quant_v_group<D, VMODE>(V, Vout, sV, vtr[wave], lane, b, k, g, bh, N, G, d_model, slice_sc);
    else
        quant_row_group<D>(tensor == 0 ? Q : K, tensor == 0 ? Qi : Ki, tensor == 0 ? sQ : sK, lane, b, k, g, bh, N, G,
                           d_model, slice_sc);
}

// Per-tensor mode, first pass: the absmax of every 32-row group of every head of Q, K and V
// (blockIdx.y = tensor), one wave per group, gmax = [3][B*H][G].  Reads the three fp32 tensors once.
template <int D>
__global__ __launch_bounds__(256) void qmha_group_absmax_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                                const float* __restrict__ V, float* __restrict__ gmax,
                                                                int N, int H, int d_model, int total_groups,
                                                                int first_tensor = 0) {
    constexpr int C4 = D / 4, RPI = 64 / C4, NI = 32 / RPI;
    const int tensor = blockIdx.y + first_tensor;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int item = blockIdx.x * 4 + wave;
    if (item >= total_groups) return;  // wave-uniform
    const int G = N / QMHA_GROUP;
    const int bh = item / G, g = item % G;
    const int b = bh / H, k = bh % H;
    const int ri = lane / C4, ci = lane % C4;
    const float* X = tensor == 0 ? Q : (tensor == 1 ? K : V);
    const float* base = X + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D + 4 * ci;
    float amax = 0.0f;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        const v4f v = QMHA_PRE_LOAD(reinterpret_cast<const v4f*>(base + (size_t)(i * RPI + ri) * d_model));
#pragma unroll
        for (int c = 0; c < 4; ++c) amax = fmaxf(amax, fabsf(v[c]));
    }
    amax = wave_max64(amax);
    if (lane == 0) gmax[(size_t)tensor * total_groups + item] = amax;
}


template <int D>
__global__ __launch_bounds__(256) void qmha_convert_f16_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
    _Float16* __restrict__ Qh, _Float16* __restrict__ Kh, _Float16* __restrict__ Vt,
    int N, int H, int d_model, int total_groups, int first_tensor) {
    constexpr int C4 = D / 4, RPI = 64 / C4, NI = 32 / RPI;
    const int tensor = blockIdx.y + first_tensor;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int item = blockIdx.x * 4 + wave;
    const bool active = item < total_groups;
    const int G = N / QMHA_GROUP;
    const int bh = active ? item / G : 0, g = active ? item % G : 0;
    const int b = bh / H, k = bh % H;
    const float* X = tensor == 0 ? Q : (tensor == 1 ? K : V);
    if (tensor == 2) {
        // V^T operand order through a per-wave LDS transpose (vt_group_store, shared with the
        // int8 pre-pass): coalesced 16-byte non-temporal loads of NI consecutive rows per lane
        __shared__ __attribute__((aligned(16))) char vtr[4][D * QMHA_VT_PITCH];
        if (active) {
            const int rq = lane / C4, c4 = lane % C4;
            const float* base = V + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D + 4 * c4;
            v4f x[NI];
#pragma unroll
            for (int i = 0; i < NI; ++i)
                x[i] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(base + (size_t)(NI * rq + i) * d_model));
            vt_group_store<D, false>(vtr[wave], x, 1.0f, lane,
                                     reinterpret_cast<char*>(Vt + ((size_t)bh * G + g) * (size_t)(32 * D)));
        }
        return;
    }
    const int ri = lane / C4, ci = lane % C4;
    v4f v[NI];
    if (active) {
        const float* base = X + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D + 4 * ci;
#pragma unroll
        for (int i = 0; i < NI; ++i)
            v[i] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(base + (size_t)(i * RPI + ri) * d_model));
    }
    if (active) {  // Q, K: f16 rows
        _Float16* dst = (tensor == 0 ? Qh : Kh) + ((size_t)bh * N + (size_t)g * QMHA_GROUP) * D + 4 * ci;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            v4h hv;
#pragma unroll
            for (int c = 0; c < 4; ++c) hv[c] = (_Float16)v[i][c];  // RNE (= __float2half)
            *reinterpret_cast<v4h*>(dst + (size_t)(i * RPI + ri) * D) = hv;
        }
    }
}


// ---------------------------------------------------------------------------------------
// Every other head size the reference accepts (d % 32 == 0, include/config.h:32; d = 96, 160, 192,
// 224, 256): one wave per (tensor, bh, 32-row group) as above, with a lane map that works for any
// d -- lane l holds the 16-byte quads l, l + 64, ... of the group's 32 x d block (row = q / (d/4)),
// coalesced along each row -- and the V^T operand written through the wave's LDS tile element by
// element (2-byte / 1-byte scattered writes; these head sizes are not the tuned path).
// QUANT: the int8 quantiser (fa_tc_int8_b.cu:33-152) -- rows as int8, V as f16-valued integers
// (VMODE 1) or int8 (VMODE 0); otherwise the fp16 conversion (fa_tc_v1a.cu:300-330) -- rows and V
// as f16 (RNE).
// ---------------------------------------------------------------------------------------
template <int D, int VMODE, bool QUANT>
__global__ __launch_bounds__(256) void qmha_prepass_any_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, void* __restrict__ Qo,
    void* __restrict__ Ko, void* __restrict__ Vout, float* __restrict__ sQ, float* __restrict__ sK,
    float* __restrict__ sV, int N, int H, int d_model, int total_groups, int first_tensor) {
    constexpr int C4 = D / 4, NQ = D / 8;                 // quads per row, quads per lane
    constexpr int VB = (VMODE == 1 || !QUANT) ? 64 : 32;  // V^T operand bytes per d-row (32 slots)
    __shared__ __attribute__((aligned(16))) char vtr[4][D * 64];
    const int tensor = blockIdx.y + first_tensor;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int item = blockIdx.x * 4 + wave;
    if (item >= total_groups) return;  // wave-uniform
    const int G = N / QMHA_GROUP;
    const int bh = item / G, g = item % G;
    const int b = bh / H, k = bh % H;
    const float* X = tensor == 0 ? Q : (tensor == 1 ? K : V);
    const float* base = X + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D;
    v4f x[NQ];
    float amax = 0.0f;
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const int q = i * 64 + lane, row = q / C4, c4 = q % C4;
        x[i] = QMHA_PRE_LOAD(reinterpret_cast<const v4f*>(base + (size_t)row * d_model + 4 * c4));
#pragma unroll
        for (int c = 0; c < 4; ++c) amax = fmaxf(amax, fabsf(x[i][c]));
    }
    float sc = 1.0f, inv = 1.0f;
    if constexpr (QUANT) {
        sc = qmha_scale_from_absmax(wave_max64(amax));  // fa_tc_int8_b.cu:104
        inv = 1.0f / sc;                                // :106
        float* s_out = tensor == 0 ? sQ : (tensor == 1 ? sK : sV);
        if (lane == 0 && s_out) s_out[(size_t)bh * G + g] = sc;
    }
    if (tensor < 2) {  // rows [bh][N][D]
        char* dst = static_cast<char*>(tensor == 0 ? Qo : Ko);
        if (!dst) return;
#pragma unroll
        for (int i = 0; i < NQ; ++i) {
            const int q = i * 64 + lane, row = q / C4, c4 = q % C4;
            const size_t e0 = ((size_t)bh * N + (size_t)g * QMHA_GROUP + row) * D + 4 * c4;
            if constexpr (QUANT) {
                uint32_t w = 0;
#pragma unroll
                for (int c = 0; c < 4; ++c) w |= ((uint32_t)(uint8_t)qmha_quant_i8(x[i][c], inv)) << (8 * c);
                *reinterpret_cast<uint32_t*>(dst + e0) = w;
            } else {
                v4h hv;
#pragma unroll
                for (int c = 0; c < 4; ++c) hv[c] = (_Float16)x[i][c];  // RNE (= __float2half)
                *reinterpret_cast<v4h*>(dst + 2 * e0) = hv;
            }
        }
        return;
    }
    // V: the [D][32 slots] V^T operand block of this group through the wave's LDS tile
    char* T = vtr[wave];
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const int q = i * 64 + lane, row = q / C4, c4 = q % C4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int d = 4 * c4 + c;
            if constexpr (!QUANT)
                *reinterpret_cast<_Float16*>(T + d * 64 + 2 * slot_of_kv_f16(row)) = (_Float16)x[i][c];
            else if constexpr (VMODE == 1)
                *reinterpret_cast<_Float16*>(T + d * 64 + 2 * slot_of_kv_f16(row)) = (_Float16)qmha_quant_i8(x[i][c], inv);
            else
                *reinterpret_cast<int8_t*>(T + d * 32 + slot_of_kv_i8(row)) = (int8_t)qmha_quant_i8(x[i][c], inv);
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    char* dst = static_cast<char*>(Vout) + ((size_t)bh * G + g) * (size_t)(VB * D);
    constexpr int LINES = D * VB / 16;
#pragma unroll
    for (int u = lane; u < LINES; u += 64) *reinterpret_cast<v4i*>(dst + 16 * u) = *reinterpret_cast<const v4i*>(T + 16 * u);
}

template <int D, int VMODE, bool QUANT>
static hipError_t prepass_any_d(const float* Q, const float* K, const float* V, void* Qo, void* Ko, void* Vout, float* sQ,
                                float* sK, float* sV, int B, int N, int H, int d_model, int first_tensor, int num_tensors,
                                hipStream_t stream) {
    const int total = B * H * (N / QMHA_GROUP);
    dim3 grid((total + 3) / 4, num_tensors > 0 ? num_tensors : 3 - first_tensor);
    hipLaunchKernelGGL((qmha_prepass_any_kernel<D, VMODE, QUANT>), grid, dim3(256), 0, stream, Q, K, V, Qo, Ko, Vout, sQ, sK,
                       sV, N, H, d_model, total, first_tensor);
    return hipGetLastError();
}

template <int D>
static hipError_t quant_int8_d(const float* Q, const float* K, const float* V, const Int8Workspace& w, void* vout,
                               int v_mode, int B, int N, int H, int d_model, int first_tensor, int num_tensors,
                               hipStream_t stream) {
    const int total = B * H * (N / QMHA_GROUP);
    dim3 grid((total + 3) / 4, num_tensors > 0 ? num_tensors : 3 - first_tensor);
    if (v_mode == 0)
        hipLaunchKernelGGL((qmha_quant_int8_kernel<D, 0>), grid, dim3(256), 0, stream, Q, K, V, w.Qi, w.Ki, vout, w.sQ,
                           w.sK, w.sV, N, H, d_model, total, first_tensor);
    else
        hipLaunchKernelGGL((qmha_quant_int8_kernel<D, 1>), grid, dim3(256), 0, stream, Q, K, V, w.Qi, w.Ki, vout, w.sQ,
                           w.sK, w.sV, N, H, d_model, total, first_tensor);
    return hipGetLastError();
}

// Two launches over the whole batch: the group absmax of Q, K, V, then K / V quantised with their
// slice scales.  (r03: batch chunks of ~96 MiB of K + V, each absmax pass followed at once by its
// quantisation so the re-read of K / V could come from the Infinity Cache, measured 0.260 against
// 0.230 ms at C4, profiles/r03/pt/ab_chunk/)
// Three launches over the whole batch: the group absmax of Q, K, V (reads the fp32 tensors once),
// the slice scales, then K / V quantised with them (reads K / V again: 1.54 GB per call at C4, at
// the HBM roofline).  r03: batch chunks of ~96 MiB of K + V, each absmax pass followed at once by
// its quantisation so the re-read could come from the Infinity Cache, measured 0.260 against 0.230
// ms (profiles/r03/pt/ab_chunk/); r04: one workgroup per head slice doing both passes back to back
// (re-read from the cache) measured 0.270 ms: one workgroup per 1 MiB slice is latency-bound
// (3.7 TB/s on its 1.0 GB of HBM traffic; profiles/r04/ab_pt_prepass/)
template <int D>
static hipError_t quant_int8_pt_d(const float* Q, const float* K, const float* V, const Int8Workspace& w, int B, int N,
                                  int H, int d_model, hipStream_t stream) {
    const int G = N / QMHA_GROUP, BH = B * H;
    const int total = BH * G;
    hipLaunchKernelGGL((qmha_group_absmax_kernel<D>), dim3((total + 3) / 4, 3), dim3(256), 0, stream, Q, K, V, w.gmax, N,
                       H, d_model, total);
    hipLaunchKernelGGL(qmha_slice_scale_kernel, dim3((BH + 3) / 4, 3), dim3(256), 0, stream, (const float*)w.gmax, w.sQ,
                       w.sK, w.sV, BH, G, 0);
    // K and V quantised with their slice scales (blockIdx.y = tensor - 1); Q by the main kernel
    hipLaunchKernelGGL((qmha_quant_int8_kernel<D, 1, true>), dim3((total + 3) / 4, 2), dim3(256), 0, stream, Q, K, V,
                       nullptr, w.Ki, (void*)w.Vh, w.sQ, w.sK, w.sV, N, H, d_model, total, 1);
    return hipGetLastError();
}

template <int D>
static hipError_t quant_int8_pt_rows_d(const float* X, const Int8Workspace& w, int B, int N, int H, int d_model,
                                       hipStream_t stream) {
    const int G = N / QMHA_GROUP, BH = B * H;
    const int total = BH * G;
    // X in the K role (tensor 1) of a [3][B*H][G] gmax table: absmax, slice scales, then int8 rows
    hipLaunchKernelGGL((qmha_group_absmax_kernel<D>), dim3((total + 3) / 4, 1), dim3(256), 0, stream, X, X, X, w.gmax, N,
                       H, d_model, total, 1);
    hipLaunchKernelGGL(qmha_slice_scale_kernel, dim3((BH + 3) / 4, 1), dim3(256), 0, stream, (const float*)w.gmax, nullptr,
                       w.sK, nullptr, BH, G, 1);
    hipLaunchKernelGGL((qmha_quant_int8_kernel<D, 1, true>), dim3((total + 3) / 4, 1), dim3(256), 0, stream, X, X, X,
                       nullptr, w.Ki, nullptr, nullptr, w.sK, nullptr, N, H, d_model, total, 1);
    return hipGetLastError();
}

hipError_t launch_quant_int8_pt_rows(const float* X, const Int8Workspace& w, int B, int N, int H, int D, int d_model,
                                     hipStream_t stream) {
    switch (D) {
        case 32: return quant_int8_pt_rows_d<32>(X, w, B, N, H, d_model, stream);
        case 64: return quant_int8_pt_rows_d<64>(X, w, B, N, H, d_model, stream);
        case 128: return quant_int8_pt_rows_d<128>(X, w, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_quant_int8_pt(const float* Q, const float* K, const float* V, const Int8Workspace& w, int B, int N,
                                int H, int D, int d_model, hipStream_t stream) {
    switch (D) {
        case 32: return quant_int8_pt_d<32>(Q, K, V, w, B, N, H, d_model, stream);
        case 64: return quant_int8_pt_d<64>(Q, K, V, w, B, N, H, d_model, stream);
        case 128: return quant_int8_pt_d<128>(Q, K, V, w, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_quant_int8(const float* Q, const float* K, const float* V, const Int8Workspace& w, void* vout,
                             int v_mode, int B, int N, int H, int D, int d_model, hipStream_t stream, int first_tensor,
                             int num_tensors) {
    if (first_tensor < 0 || first_tensor > 2 || (num_tensors > 0 && first_tensor + num_tensors > 3))
        return hipErrorInvalidValue;
    switch (D) {
        case 32: return quant_int8_d<32>(Q, K, V, w, vout, v_mode, B, N, H, d_model, first_tensor, num_tensors, stream);
        case 64: return quant_int8_d<64>(Q, K, V, w, vout, v_mode, B, N, H, d_model, first_tensor, num_tensors, stream);
        case 128: return quant_int8_d<128>(Q, K, V, w, vout, v_mode, B, N, H, d_model, first_tensor, num_tensors, stream);
#define QMHA_CASE(d)                                                                                                      \
    case d:                                                                                                               \
        return v_mode == 0 ? prepass_any_d<d, 0, true>(Q, K, V, w.Qi, w.Ki, vout, w.sQ, w.sK, w.sV, B, N, H, d_model,     \
                                                       first_tensor, num_tensors, stream)                                \
                           : prepass_any_d<d, 1, true>(Q, K, V, w.Qi, w.Ki, vout, w.sQ, w.sK, w.sV, B, N, H, d_model,     \
                                                       first_tensor, num_tensors, stream);
        QMHA_CASE(96) QMHA_CASE(160) QMHA_CASE(192) QMHA_CASE(224) QMHA_CASE(256)
#undef QMHA_CASE
        default: return hipErrorInvalidValue;
    }
}


template <int D>
static hipError_t convert_f16_d(const float* Q, const float* K, const float* V, const F16Workspace& w, int B, int N,
                                int H, int d_model, hipStream_t stream) {
    const int total = B * H * (N / QMHA_GROUP);
    // K and V only: the main kernel converts Q itself (blockIdx.y = tensor - 1)
    hipLaunchKernelGGL((qmha_convert_f16_kernel<D>), dim3((total + 3) / 4, 2), dim3(256), 0, stream, Q, K, V, w.Qh,
                       w.Kh, w.Vt, N, H, d_model, total, 1);
    return hipGetLastError();
}

hipError_t launch_convert_f16(const float* Q, const float* K, const float* V, const F16Workspace& w, int B, int N,
                              int H, int D, int d_model, hipStream_t stream) {
    switch (D) {
        case 32: return convert_f16_d<32>(Q, K, V, w, B, N, H, d_model, stream);
        case 64: return convert_f16_d<64>(Q, K, V, w, B, N, H, d_model, stream);
        case 128: return convert_f16_d<128>(Q, K, V, w, B, N, H, d_model, stream);
#define QMHA_CASE(d) \
    case d: return prepass_any_d<d, 1, false>(Q, K, V, w.Qh, w.Kh, w.Vt, nullptr, nullptr, nullptr, B, N, H, d_model, 1, -1, stream);
        QMHA_CASE(96) QMHA_CASE(160) QMHA_CASE(192) QMHA_CASE(224) QMHA_CASE(256)
#undef QMHA_CASE
        default: return hipErrorInvalidValue;
    }
}

}  // namespace qmha
