// qmha_prepass.hip -- the K/V pre-passes of the int8 and fp16 paths (and the standalone
// qmha_quantize_int8 op), in a translation unit of their own: they read the caller's Q/K/V, so they
// keep IEEE NaN semantics (the main-kernel sources are built with -fno-honor-nans, round-2 ADVICE).
//   qmha_quant_int8_kernel  fa_tc_int8_b.cu:33-152 (fp32_to_int8sram): per 32-row group of every
//                           head, sc = max(absmax/127, 1e-8), x_i8 = clamp(rint(x * (1/sc))) --
//                           K as int8 rows, V as f16-valued integers in the MFMA V^T operand order
//   qmha_convert_f16_kernel fa_tc_v1a.cu:300-330: K as f16 rows, V in the f16 V^T operand order (RNE)
#include <atomic>

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
template <int D, int VMODE>
__device__ __forceinline__ void quant_v_group(const float* __restrict__ V, void* __restrict__ Vout,
                                              float* __restrict__ sV, char* vtr, int lane, int b, int k, int g,
                                              int bh, int N, int G, int d_model) {
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
    const float sc = qmha_scale_from_absmax(wave_max64(amax));
    const float inv = 1.0f / sc;
    if constexpr (VMODE == 1)
        vt_group_store<D, true>(vtr, x, inv, lane, static_cast<char*>(Vout) + ((size_t)bh * G + g) * (size_t)(64 * D));
    else
        vt8_group_store<D>(vtr, x, inv, lane, static_cast<char*>(Vout) + ((size_t)bh * G + g) * (size_t)(32 * D));
    if (lane == 0) sV[(size_t)bh * G + g] = sc;
}

// One wave quantises one 32-row group of Q or K (b, k, g) into int8 rows [bh][N][D].
template <int D>
__device__ __forceinline__ void quant_row_group(const float* __restrict__ X, int8_t* __restrict__ Xi,
                                                float* __restrict__ sX, int lane, int b, int k, int g, int bh, int N,
                                                int G, int d_model) {
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
    const float sc = qmha_scale_from_absmax(wave_max64(amax));  // :104
    const float inv = 1.0f / sc;                                                            // :106 (correctly rounded)
    int8_t* dst = Xi + ((size_t)bh * N + (size_t)g * QMHA_GROUP) * D + 4 * ci;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
        uint32_t w = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) w |= ((uint32_t)(uint8_t)qmha_quant_i8(v[i][c], inv)) << (8 * c);
        *reinterpret_cast<uint32_t*>(dst + (size_t)(i * RPI + ri) * D) = w;
    }
    if (lane == 0) sX[(size_t)bh * G + g] = sc;
}

// ---------------------------------------------------------------------------------------
// Pre-pass: quantise Q, K, V (fa_tc_int8_b.cu:33-152, fp32_to_int8sram).
// One wave per (tensor, bh, group); blockIdx.y = tensor (0 Q, 1 K, 2 V).
// ---------------------------------------------------------------------------------------
template <int D, int VMODE>
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
    if (tensor == 2)
        quant_v_group<D, VMODE>(V, Vout, sV, vtr[wave], lane, b, k, g, bh, N, G, d_model);
    else
        quant_row_group<D>(tensor == 0 ? Q : K, tensor == 0 ? Qi : Ki, tensor == 0 ? sQ : sK, lane, b, k, g, bh, N, G,
                           d_model);
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

// ---------------------------------------------------------------------------------------
// Per-tensor mode, single read (r04): the slice scale needs the absmax of a whole [N, d] head slice
// before any of its values are quantised.  A slice of K or V is split over `gkv` workgroups; each
// loads its part (12 waves x PW 32-row groups, 32 KiB per wave) into REGISTERS, reduces it, and
// publishes the part's absmax to the slice with one agent-scope atomicMax (non-negative float bits
// order as unsigned ints; max is exact in any order) followed by an atomicAdd on the slice's arrival
// counter (both returning, so the max is performed before the arrival is).  Lane 0 then polls the
// counter (agent-scope loads, s_sleep) until all gkv parts have arrived, reads the slice maximum, and
// the workgroup quantises the data it still holds -- K and V are read from HBM once, not twice.
// Q needs only its slice scale (the main kernel quantises Q): its parts reduce and publish, and the
// last part to arrive writes sQ.  The parts of a slice are consecutive items of one XCD's block
// sequence (below), so they are normally resident together.  The wait is bounded: past the bound the
// workgroup reduces the whole slice itself (the same maximum), so no dispatch order can deadlock it.
// sync = [2][3][B*H] uint32 (max bits, arrivals), zeroed by qmha_zero_u32_kernel in the same call.
// ---------------------------------------------------------------------------------------
// (zeroed by a kernel, not hipMemsetAsync: under graph capture a memset node did not re-zero on replays,
// DESIGN.md 5.2b)
__global__ __launch_bounds__(256) void qmha_zero_u32_kernel(uint32_t* __restrict__ p, int n) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = 0u;
}

// The part's absmax into the slice maximum, PERFORMED before the caller's arrival increment: a
// returning atomic and a wait on it (a non-returning global_atomic_umax may still be in flight when
// the following atomicAdd lands, and a reader that sees all arrivals would then read a maximum short
// of this part's -- observed as a rare wrong slice scale before this wait was added)
__device__ __forceinline__ void publish_max(uint32_t* mx, float m) {
    const uint32_t old = __hip_atomic_fetch_max(mx, __float_as_uint(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(old) : "memory");
}

// 12-wave workgroups (three waves per SIMD, one workgroup per CU): r04 A/Bs at C4 (profiles/r04/ab_pt_single_read/)
// 0.198 ms against 0.206 ms for 4-wave workgroups with the same 32 KiB per wave, 0.204 ms for 48 KiB per
// wave; 8-wave workgroups 0.198, 6-wave 0.210 against 0.200 ms on another box
constexpr int kPtWaves = 12;
__device__ __forceinline__ float wg_max(const float (&pm)[kPtWaves]) {
    float m = pm[0];
#pragma unroll
    for (int i = 1; i < kPtWaves; ++i) m = fmaxf(m, pm[i]);
    return m;
}
// 32-row groups a wave holds in registers: 32 KiB per wave (128 VGPRs of data), 16 KiB at d = 128
// (its 2-group form spills under the 12-wave register budget)
template <int D>
constexpr int pt_groups_per_wave() { return D == 128 ? 1 : 256 / D; }

template <int D>
__global__ __launch_bounds__(64 * kPtWaves) void qmha_pt_quant_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, int8_t* __restrict__ Ki,
    _Float16* __restrict__ Vh, float* __restrict__ sQ, float* __restrict__ sK, float* __restrict__ sV,
    uint32_t* __restrict__ sync, int N, int H, int d_model, int BH, int gkv, int gq, int kv_first, int kv_tensors,
    int with_q, unsigned long long wait_ticks, int phase) {
    constexpr int C4 = D / 4, NI = D / 8, RPI = 64 / C4;
    constexpr int PW = pt_groups_per_wave<D>();
    constexpr int NW = kPtWaves;
    constexpr int GPB = NW * PW;  // groups per workgroup
    __shared__ __attribute__((aligned(16))) char vtr[kPtWaves][D * QMHA_VT_PITCH];
    __shared__ float part_max[kPtWaves];
    __shared__ float slice_max;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int G = N / QMHA_GROUP;
    uint32_t* smax = sync;
    uint32_t* scnt = sync + 3 * BH;
    // logical item order: per head slice bh its K parts, V parts, Q parts; each XCD takes a contiguous
    // range of items (xcd_remap), so the parts of a slice are dispatched together by ONE XCD's
    // dispatcher (consecutive blocks otherwise land on eight different XCDs, which dispatch them
    // at unrelated times) and every XCD gets the same mix of K / V / Q work
    const int per_bh = kv_tensors * gkv + (with_q ? gq : 0);
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = item / per_bh, r = item % per_bh;
    if (phase == 2 && r >= kv_tensors * gkv) return;  // Q's scale was written by phase 1
    if (phase == 1 || r >= kv_tensors * gkv) {
        // ---- slice absmax only (workgroup-uniform branch): Q in every phase; phase 1 (the two-pass form,
        // for slices of more parts than an XCD holds at once) K and V too, without waiting
        const bool isq = r >= kv_tensors * gkv;
        const int tt = isq ? 0 : kv_first + r / gkv;
        const int part = isq ? r - kv_tensors * gkv : r % gkv;
        const int np = isq ? gq : gkv;
        const float* X = tt == 0 ? Q : (tt == 1 ? K : V);
        const int b = bh / H, k = bh % H;
        const int ri = lane / C4, ci = lane % C4;
        const int per = (G + np - 1) / np;
        float amax = 0.0f;
        for (int g = part * per + wave; g < min(G, (part + 1) * per); g += NW) {
            const float* base = X + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D + 4 * ci;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(base + (size_t)(i * RPI + ri) * d_model));
#pragma unroll
                for (int c = 0; c < 4; ++c) amax = fmaxf(amax, fabsf(v[c]));  // IEEE: a NaN is dropped
            }
        }
        amax = wave_max64(amax);
        if (lane == 0) part_max[wave] = amax;
        __syncthreads();
        if (threadIdx.x == 0) {
            const float m = wg_max(part_max);
            publish_max(&smax[(size_t)tt * BH + bh], m);
            if (isq) {
                const uint32_t old = atomicAdd(&scnt[bh], 1u);
                if (old + 1 == (uint32_t)gq)  // the last part: every max is in
                    sQ[bh] = qmha_scale_from_absmax(__uint_as_float(__hip_atomic_load(&smax[bh], __ATOMIC_RELAXED,
                                                                                       __HIP_MEMORY_SCOPE_AGENT)));
            }
        }
        return;
    }
    // ---- K / V: part `part` of slice bh of tensor t, held in registers across the wait
    const int t = kv_first + r / gkv, part = r % gkv;
    const int b = bh / H, k = bh % H;
    const bool isv = t == 2;
    const float* X = isv ? V : K;
    // K rows: lane (ri, ci) holds rows i * RPI + ri, columns 4 ci..; V: lane (rq, c4) holds NI
    // consecutive rows of columns 4 c4.. (the vt_group_store map)
    const int r0 = isv ? (lane / C4) * NI : lane / C4, rs = isv ? 1 : RPI, cc = lane % C4;
    v4f x[PW][NI];
    float amax = 0.0f;
#pragma unroll
    for (int j = 0; j < PW; ++j) {
        const int g = part * GPB + wave * PW + j;
        if (g < G) {
            const float* base = X + ((size_t)b * N + (size_t)g * QMHA_GROUP + r0) * d_model + (size_t)k * D + 4 * cc;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                x[j][i] = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(base + (size_t)(i * rs) * d_model));
#pragma unroll
                for (int c = 0; c < 4; ++c) amax = fmaxf(amax, fabsf(x[j][i][c]));
            }
        }
    }
    amax = wave_max64(amax);
    if (lane == 0) part_max[wave] = amax;
    __syncthreads();
    if (threadIdx.x == 0 && phase == 2) {  // the two-pass form: phase 1 (a previous launch) left the maximum
        slice_max = __uint_as_float(__hip_atomic_load(&smax[(size_t)t * BH + bh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    } else if (threadIdx.x == 0) {
        const float m = wg_max(part_max);
        uint32_t* mx = &smax[(size_t)t * BH + bh];
        uint32_t* cn = &scnt[(size_t)t * BH + bh];
        publish_max(mx, m);
        uint32_t c = atomicAdd(cn, 1u) + 1;
        // the other parts of this slice are consecutive workgroups dispatched around this one:
        // normally a few microseconds; bounded at wait_ticks of the 100 MHz real-time clock (2 ms), then
        // the fallback (0 forces it: qmha_debug_set_pt_wait, the test of that path)
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (c < (uint32_t)gkv && __builtin_amdgcn_s_memrealtime() - t0 < wait_ticks) {
            __builtin_amdgcn_s_sleep(2);
            c = __hip_atomic_load(cn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        slice_max = c >= (uint32_t)gkv ? __uint_as_float(__hip_atomic_load(mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                                       : -1.0f;
    }
    __syncthreads();
    float sm = slice_max;
    if (sm < 0.0f) {  // fallback (never taken when the slice's parts are co-resident): reduce the slice here
        const int ri = lane / C4, ci = lane % C4;
        float a2 = 0.0f;
        for (int g = wave; g < G; g += NW) {
            const float* base = X + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D + 4 * ci;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const v4f v = *reinterpret_cast<const v4f*>(base + (size_t)(i * RPI + ri) * d_model);
#pragma unroll
                for (int c = 0; c < 4; ++c) a2 = fmaxf(a2, fabsf(v[c]));
            }
        }
        a2 = wave_max64(a2);
        __syncthreads();
        if (lane == 0) part_max[wave] = a2;
        __syncthreads();
        sm = wg_max(part_max);
    }
    const float sc = qmha_scale_from_absmax(sm);  // fa_tc_int8_b.cu:104, over the whole slice
    const float inv = 1.0f / sc;                  // :106 (correctly rounded)
    if (part == 0 && threadIdx.x == 0) (isv ? sV : sK)[bh] = sc;
#pragma unroll
    for (int j = 0; j < PW; ++j) {
        const int g = part * GPB + wave * PW + j;
        if (g >= G) continue;  // wave-uniform
        if (isv) {
            if (Vh)
                vt_group_store<D, true>(vtr[wave], x[j], inv, lane,
                                        reinterpret_cast<char*>(Vh) + ((size_t)bh * G + g) * (size_t)(64 * D));
        } else {
            int8_t* dst = Ki + ((size_t)bh * N + (size_t)g * QMHA_GROUP) * D + 4 * cc;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                uint32_t w = 0;
#pragma unroll
                for (int c = 0; c < 4; ++c) w |= ((uint32_t)(uint8_t)qmha_quant_i8(x[j][i][c], inv)) << (8 * c);
                *reinterpret_cast<uint32_t*>(dst + (size_t)(i * RPI + r0) * D) = w;
            }
        }
    }
}

// Per-tensor pre-pass history: r03 ran three launches (group absmax of Q, K, V; slice
// scales; K / V quantised with them -- reading K / V twice, 1.54 GB per call at C4: 0.230 ms); batch
// chunks meant to re-read from the Infinity Cache measured 0.260 ms, one workgroup per slice 0.270 ms.
// r04 ships the single-read kernel above: 1.0 GB per call, 0.198 ms.
// bounded wait of the parts of a slice, in ticks of the 100 MHz real-time clock (qmha_debug_set_pt_wait)
// (negative: every call takes the two-pass form, the test of that path)
static std::atomic<long long> g_pt_wait_ticks{200000};
long long set_pt_wait_ticks(long long ticks) { return g_pt_wait_ticks.exchange(ticks); }

// workgroups of qmha_pt_quant_kernel<D> one XCD holds at once (HIP's occupancy answer x CUs / 8 XCDs,
// cached per device); 0 if unknown
template <int D>
static int pt_resident_per_xcd() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    int r = cache[dev].load(std::memory_order_relaxed);
    if (r <= 0) {
        int n = 0, c = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, qmha_pt_quant_kernel<D>, 64 * kPtWaves, 0) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0 || c <= 0)
            return 0;
        r = n * c / 8;
        cache[dev].store(r, std::memory_order_relaxed);
    }
    return r;
}

// single-read launch (qmha_pt_quant_kernel): per head slice its K parts, V parts, Q parts (12 waves x
// pt_groups_per_wave<D>() groups each); the slice counters / maxima zeroed by a kernel of this call
template <int D>
static hipError_t quant_int8_pt1_d(const float* Q, const float* K, const float* V, const Int8Workspace& w, int B, int N,
                                   int H, int d_model, bool rows_only, hipStream_t stream) {
    const int G = N / QMHA_GROUP, BH = B * H;
    constexpr int GPB = kPtWaves * pt_groups_per_wave<D>();
    const int gkv = (G + GPB - 1) / GPB;
    uint32_t* sync = w.slice_sync;  // [2][3][BH]
    // zeroed by a kernel of this call (a kernel node under graph capture; caller scratch is arbitrary)
    hipLaunchKernelGGL(qmha_zero_u32_kernel, dim3((6 * BH + 255) / 256), dim3(256), 0, stream, sync, 6 * BH);
    const int kv_tensors = rows_only ? 1 : 2, with_q = rows_only ? 0 : 1;
    const int grid = kv_tensors * BH * gkv + (with_q ? BH * gkv : 0);
    // the single read needs every part of a slice resident at once; a slice of more parts than one XCD
    // holds (d = 128 beyond N = 12288, d = 64 beyond 49152, d = 32 beyond 98304 at one workgroup per CU)
    // would leave each part waiting out the bound -- those run the two-pass form instead: phase 1 publishes
    // every part's absmax, phase 2 re-reads K / V and quantises them with the slice maxima (round-4 ADVICE)
    const int resident = pt_resident_per_xcd<D>();
    const long long wait_ticks = g_pt_wait_ticks.load();
    if (resident <= 0 || gkv > resident || wait_ticks < 0) {
        for (int phase = 1; phase <= 2; ++phase)
            hipLaunchKernelGGL((qmha_pt_quant_kernel<D>), dim3(grid), dim3(64 * kPtWaves), 0, stream, Q, K, V, w.Ki,
                               rows_only ? nullptr : w.Vh, w.sQ, w.sK, w.sV, sync, N, H, d_model, BH, gkv, gkv, 1,
                               kv_tensors, with_q, 0ull, phase);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((qmha_pt_quant_kernel<D>), dim3(grid), dim3(64 * kPtWaves), 0, stream, Q, K, V, w.Ki,
                       rows_only ? nullptr : w.Vh, w.sQ, w.sK, w.sV, sync, N, H, d_model, BH, gkv, gkv, 1, kv_tensors,
                       with_q, (unsigned long long)wait_ticks, 0);
    return hipGetLastError();
}

template <int D>
static hipError_t quant_int8_pt_d(const float* Q, const float* K, const float* V, const Int8Workspace& w, int B, int N,
                                  int H, int d_model, hipStream_t stream) {
    return quant_int8_pt1_d<D>(Q, K, V, w, B, N, H, d_model, false, stream);
}

// the standalone op's per-tensor layout: X in the K role only (int8 rows, sK = the slice scales)
template <int D>
static hipError_t quant_int8_pt_rows_d(const float* X, const Int8Workspace& w, int B, int N, int H, int d_model,
                                       hipStream_t stream) {
    return quant_int8_pt1_d<D>(X, X, X, w, B, N, H, d_model, true, stream);
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
