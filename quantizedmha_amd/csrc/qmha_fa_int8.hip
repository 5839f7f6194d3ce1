// qmha_fa_int8.hip -- fused INT8 FlashAttention-2 forward for gfx950 (MI355X).
//
// Drop-in for the reference's fa_tc_int8_b (mha_kernels/fa_tc_int8_b.cu:408-609) with its
// *intended* numerics:
//   per 32-row group of Q, K, V:  s = max(absmax/127, 1e-8), x_i8 = clamp(rint(x * (1/s)))
//   S = Qi Ki^T (int32, exact)        -> scores = S * sQ * sK / sqrt(d)
//   online softmax, m0 = 0            -> p = exp(scores - m), l = alpha*l + sum(p)
//   per 32x32 tile P: sP from max p   -> Pi = rint(p / sP)
//   O = alpha*O + (Pi Vi)[int32] * sP * sV,   out = O / l  (0 if l <= 1e-20)
//
// Two launches per call:
//   1. qmha_quant_int8_kernel: reads fp32 Q/K/V once, writes int8 Q/K (row-major per head)
//      and V in the permuted V^T operand layout, plus one fp32 scale per 32-row group.
//      Bit-identical to the reference quantiser (same fp32 ops, RNE rounding).
//   2. qmha_fa_int8_kernel: one workgroup = WAVES waves = WAVES*32 query rows of one head;
//      each wave owns exactly one 32-row Q group (= one Q quantisation group).  K/V int8
//      tiles stream HBM -> registers -> LDS (double buffered, XOR-swizzled for
//      conflict-free ds_read_b128).  Both products run on v_mfma_i32_32x32x32_i8 with
//      swapped operands (S^T = K Q^T, O^T = V^T P^T) so that every query's statistics are
//      lane-local and P^T feeds the second MFMA straight from registers.
#include "qmha_common.hpp"
#include "qmha_kernels.hpp"

namespace qmha {

// log2(e): the softmax runs in base 2 (v_exp_f32), scores pre-multiplied by log2(e).
static constexpr float kLog2e = 1.4426950408889634f;

// ---------------------------------------------------------------------------------------
// Pre-pass: quantise Q, K, V (fa_tc_int8_b.cu:33-152, fp32_to_int8sram).
// One wave per (tensor, bh, group); blockIdx.y = tensor (0 Q, 1 K, 2 V).
// ---------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void qmha_quant_int8_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
    int8_t* __restrict__ Qi, int8_t* __restrict__ Ki, int8_t* __restrict__ Vt,
    float* __restrict__ sQ, float* __restrict__ sK, float* __restrict__ sV,
    int N, int H, int d_model, int total_groups) {
    constexpr int C4 = D / 4;        // float4 per row
    constexpr int RPI = 64 / C4;     // rows per load instruction
    constexpr int NI = 32 / RPI;     // load instructions per lane
    __shared__ __attribute__((aligned(16))) int8_t vtile[4][32 * D];

    const int tensor = blockIdx.y;
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int item = blockIdx.x * 4 + wave;  // (bh, g)
    const bool active = item < total_groups;
    const int G = N / QMHA_GROUP;
    const int bh = active ? item / G : 0, g = active ? item % G : 0;
    const int b = bh / H, k = bh % H;
    const float* X = tensor == 0 ? Q : (tensor == 1 ? K : V);

    const int ri = lane / C4, ci = lane % C4;
    v4f v[NI];
    float amax = 0.0f;
    if (active) {
        const float* base = X + ((size_t)b * N + (size_t)g * QMHA_GROUP) * d_model + (size_t)k * D + 4 * ci;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            v[i] = *reinterpret_cast<const v4f*>(base + (size_t)(i * RPI + ri) * d_model);
#pragma unroll
            for (int c = 0; c < 4; ++c) amax = fmaxf(amax, fabsf(v[i][c]));
        }
    }
    amax = wave_max64(amax);
    const float sc = qmha_scale_from_absmax(amax);  // :104
    const float inv = 1.0f / sc;                     // :106 (correctly rounded division)

    if (tensor < 2) {
        if (active) {
            int8_t* dst = (tensor == 0 ? Qi : Ki) + ((size_t)bh * N + (size_t)g * QMHA_GROUP) * D + 4 * ci;
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                uint32_t w = 0;
#pragma unroll
                for (int c = 0; c < 4; ++c) w |= ((uint32_t)(uint8_t)qmha_quant_i8(v[i][c], inv)) << (8 * c);
                *reinterpret_cast<uint32_t*>(dst + (size_t)(i * RPI + ri) * D) = w;
            }
            if (lane == 0) (tensor == 0 ? sQ : sK)[item] = sc;
        }
    } else {
        // V: transpose through LDS into [D][32] with the i8 operand slot permutation.
        int8_t* tile = vtile[wave];
        if (active) {
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int row = i * RPI + ri;  // kv within group
                const int slot = slot_of_kv_i8(row);
#pragma unroll
                for (int c = 0; c < 4; ++c) tile[(4 * ci + c) * 32 + slot] = (int8_t)qmha_quant_i8(v[i][c], inv);
            }
        }
        __syncthreads();
        if (active) {
            int8_t* dst = Vt + ((size_t)bh * G + g) * (size_t)(32 * D);
            constexpr int CH = 32 * D / 16;
#pragma unroll
            for (int c = lane; c < CH; c += 64)
                reinterpret_cast<v4i*>(dst)[c] = reinterpret_cast<const v4i*>(tile)[c];
            if (lane == 0) sV[item] = sc;
        }
    }
}

// LDS XOR swizzle for a row of RB bytes read as 16-byte chunks by ds_read_b128 with one
// row per lane (rows 0..31 of a 32x32 operand): conflict-free per 16-lane group.
template <int RB>
__device__ __forceinline__ int chunk_swz(int row) {
    constexpr int rows_per_bankrow = 256 / RB >= 1 ? 256 / RB : 1;
    constexpr int cpr = RB / 16;
    return (row / rows_per_bankrow) & (cpr - 1);
}

// ---------------------------------------------------------------------------------------
// Main kernel.
// ---------------------------------------------------------------------------------------
template <int D, int WAVES, int SG>
__global__ __launch_bounds__(WAVES * 64) void qmha_fa_int8_kernel(
    const int8_t* __restrict__ Qi, const int8_t* __restrict__ Ki, const int8_t* __restrict__ Vt,
    const float* __restrict__ sQ, const float* __restrict__ sK, const float* __restrict__ sV,
    float* __restrict__ O, int N, int H, int d_model, int nqb, float c_log2) {
    constexpr int KS = D / 32;               // MFMA k-steps (QK) and d-blocks (PV)
    constexpr int STAGE_BYTES = SG * 32 * D;  // per tensor per stage
    constexpr int NT = WAVES * 64;
    constexpr int CH = STAGE_BYTES / 16;      // 16-byte chunks per tensor per stage
    constexpr int CPT = (CH + NT - 1) / NT;
    __shared__ __attribute__((aligned(16))) int8_t lds[2][2 * STAGE_BYTES];

    const int G = N / QMHA_GROUP;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = wg / nqb, qb = wg % nqb;
    const int b = bh / H, k = bh % H;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int qg = qb * WAVES + wave;
    const bool active = qg < G;  // wave-uniform
    const int half = lane >> 5, col = lane & 31;

    v4i qop[KS];
    float cq = 0.0f;
    if (active) {
        const int8_t* qp = Qi + ((size_t)bh * N + (size_t)qg * QMHA_GROUP + col) * D + 16 * half;
#pragma unroll
        for (int s = 0; s < KS; ++s) qop[s] = *reinterpret_cast<const v4i*>(qp + 32 * s);
        cq = sQ[(size_t)bh * G + qg] * c_log2;
    } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) qop[s] = v4i{0, 0, 0, 0};
    }

    v16f o[KS];
#pragma unroll
    for (int m = 0; m < KS; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[m][r] = 0.0f;
    float m_run = 0.0f;  // m0 = 0 (fa_tc_int8_b.cu:402), log2 units
    float l_run = 0.0f;

    const int8_t* kbase = Ki + (size_t)bh * N * D;
    const int8_t* vbase = Vt + (size_t)bh * N * D;
    const float* skb = sK + (size_t)bh * G;
    const float* svb = sV + (size_t)bh * G;
    const int nst = (G + SG - 1) / SG;

    v4i kst[CPT], vst[CPT];
    auto gload = [&](int st) {
        const int g0 = st * SG;
        const int nch = min(SG, G - g0) * 32 * D / 16;
        const v4i* ks = reinterpret_cast<const v4i*>(kbase + (size_t)g0 * 32 * D);
        const v4i* vs = reinterpret_cast<const v4i*>(vbase + (size_t)g0 * 32 * D);
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            const int idx = tid + c * NT;
            if (idx < nch) {
                kst[c] = ks[idx];
                vst[c] = vs[idx];
            }
        }
    };
    auto lstore = [&](int buf, int st) {
        const int g0 = st * SG;
        const int nch = min(SG, G - g0) * 32 * D / 16;
        int8_t* L = lds[buf];
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
            const int idx = tid + c * NT;
            if (idx < nch) {
                const int row = idx / (D / 16), cc = idx % (D / 16);
                *reinterpret_cast<v4i*>(L + row * D + 16 * (cc ^ chunk_swz<D>(row))) = kst[c];
                const int grp = idx / (2 * D), w = idx % (2 * D);
                const int d = w >> 1, hh = w & 1;
                *reinterpret_cast<v4i*>(L + STAGE_BYTES + grp * 32 * D + d * 32 + 16 * (hh ^ chunk_swz<32>(d))) = vst[c];
            }
        }
    };

    gload(0);
    lstore(0, 0);
    __syncthreads();

    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) gload(st + 1);
        if (active) {
            const int g0 = st * SG;
            const int ngr = min(SG, G - g0);
            const int8_t* L = lds[buf];
#pragma unroll
            for (int gi = 0; gi < SG; ++gi) {
                if (gi < ngr) {
                    const int t = g0 + gi;
                    // ---- S^T = K Q^T (int32) --------------------------------------------
                    v16i s = {};
                    const int krow = gi * 32 + col;
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks) {
                        const v4i kop = *reinterpret_cast<const v4i*>(L + krow * D + 16 * ((2 * ks + half) ^ chunk_swz<D>(krow)));
                        s = __builtin_amdgcn_mfma_i32_32x32x32_i8(kop, qop[ks], s, 0, 0, 0);
                    }
                    // ---- online softmax (fa_tc_int8_b.cu:281-346) ----------------------
                    int mx = s[0];
#pragma unroll
                    for (int r = 1; r < 16; ++r) mx = max(mx, (int)s[r]);
                    mx = half_swap_max_i(mx);
                    const float c = cq * skb[t];  // sQ*sK*log2(e)/sqrt(d) > 0
                    const float m_new = fmaxf(m_run, (float)mx * c);
                    const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
                    // ---- P tile scale (fa_tc_int8_b.cu:359): max p = exp(rowmax - m) ----
                    const float pmax = half_max32(__builtin_amdgcn_exp2f(fmaf((float)mx, c, -m_new)));
                    const float sp = fmaxf(pmax / 127.0f, 1e-8f);
                    const float invp = 1.0f / sp;
                    float rs = 0.0f;
                    float y[16];
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const float p = __builtin_amdgcn_exp2f(fmaf((float)s[r], c, -m_new));
                        rs += p;
                        y[r] = fmaf(p, invp, QMHA_MAGIC_RNE);  // rint(p/sP) in the low byte
                    }
                    v4i pop;
#pragma unroll
                    for (int i = 0; i < 4; ++i) pop[i] = (int)pack4_lowbytes(y[4 * i], y[4 * i + 1], y[4 * i + 2], y[4 * i + 3]);
                    rs = half_swap_add(rs);
                    l_run = fmaf(alpha, l_run, rs);  // :336
                    m_run = m_new;
                    if (__builtin_amdgcn_ballot_w64(alpha != 1.0f)) {  // :344, exact skip when alpha == 1
#pragma unroll
                        for (int m = 0; m < KS; ++m)
#pragma unroll
                            for (int r = 0; r < 16; ++r) o[m][r] *= alpha;
                    }
                    // ---- O^T += (V^T P^T)[int32] * sP * sV (:366-371) -------------------
                    const float scale = sp * svb[t];
#pragma unroll
                    for (int m = 0; m < KS; ++m) {
                        const int d = 32 * m + col;
                        const v4i vop = *reinterpret_cast<const v4i*>(L + STAGE_BYTES + gi * 32 * D + d * 32 + 16 * (half ^ chunk_swz<32>(d)));
                        v16i pv = {};
                        pv = __builtin_amdgcn_mfma_i32_32x32x32_i8(vop, pop, pv, 0, 0, 0);
#pragma unroll
                        for (int r = 0; r < 16; ++r) o[m][r] = fmaf((float)pv[r], scale, o[m][r]);
                    }
                }
            }
        }
        if (st + 1 < nst) lstore(buf ^ 1, st + 1);
        __syncthreads();
    }

    // ---- epilogue (fa_tc_int8_b.cu:540-578): out = O / l, 0 if l <= 1e-20 -----------------
    if (active) {
        const bool ok = l_run > 1e-20f;
        float* orow = O + ((size_t)b * N + (size_t)qg * QMHA_GROUP + col) * d_model + (size_t)k * D + 4 * half;
#pragma unroll
        for (int m = 0; m < KS; ++m)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                v4f w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = ok ? o[m][4 * g4 + j] / l_run : 0.0f;
                *reinterpret_cast<v4f*>(orow + 32 * m + 8 * g4) = w;
            }
    }
}

// ---------------------------------------------------------------------------------------
// Debug: the int32 S = Qi Ki^T tiles of one head through the same MFMA operand path
// (for the bit-exact KAT in tests/).  One wave per 32x32 tile.
// ---------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(64) void qmha_debug_qk_int32_kernel(const int8_t* __restrict__ Qi, const int8_t* __restrict__ Ki,
                                                                int N, int bh, int32_t* __restrict__ S) {
    constexpr int KS = D / 32;
    const int qg = blockIdx.x, kg = blockIdx.y;
    const int lane = threadIdx.x, half = lane >> 5, col = lane & 31;
    const int8_t* qp = Qi + ((size_t)bh * N + (size_t)qg * 32 + col) * D + 16 * half;
    const int8_t* kp = Ki + ((size_t)bh * N + (size_t)kg * 32 + col) * D + 16 * half;
    v16i s = {};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
        s = __builtin_amdgcn_mfma_i32_32x32x32_i8(*reinterpret_cast<const v4i*>(kp + 32 * ks),
                                                  *reinterpret_cast<const v4i*>(qp + 32 * ks), s, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 16; ++r) S[((size_t)qg * 32 + col) * N + (size_t)kg * 32 + acc_row(r, half)] = s[r];
}

// ---------------------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------------------
size_t int8_workspace_bytes(int B, int N, int H, int D) {
    const size_t e = (size_t)B * H * N * D;
    const size_t s = (size_t)B * H * (N / QMHA_GROUP) * sizeof(float);
    return 3 * align_up(e, 256) + 3 * align_up(s, 256);
}

Int8Workspace int8_carve(void* ws, int B, int N, int H, int D) {
    Int8Workspace w;
    const size_t e = align_up((size_t)B * H * N * D, 256);
    const size_t s = align_up((size_t)B * H * (N / QMHA_GROUP) * sizeof(float), 256);
    char* p = static_cast<char*>(ws);
    w.Qi = reinterpret_cast<int8_t*>(p);
    w.Ki = reinterpret_cast<int8_t*>(p + e);
    w.Vt = reinterpret_cast<int8_t*>(p + 2 * e);
    w.sQ = reinterpret_cast<float*>(p + 3 * e);
    w.sK = reinterpret_cast<float*>(p + 3 * e + s);
    w.sV = reinterpret_cast<float*>(p + 3 * e + 2 * s);
    return w;
}

template <int D>
static hipError_t quant_int8_d(const float* Q, const float* K, const float* V, const Int8Workspace& w,
                               int B, int N, int H, int d_model, hipStream_t stream) {
    const int total = B * H * (N / QMHA_GROUP);
    dim3 grid((total + 3) / 4, 3);
    hipLaunchKernelGGL((qmha_quant_int8_kernel<D>), grid, dim3(256), 0, stream, Q, K, V, w.Qi, w.Ki, w.Vt, w.sQ, w.sK,
                       w.sV, N, H, d_model, total);
    return hipGetLastError();
}

hipError_t launch_quant_int8(const float* Q, const float* K, const float* V, const Int8Workspace& w, int B, int N,
                             int H, int D, int d_model, hipStream_t stream) {
    switch (D) {
        case 32: return quant_int8_d<32>(Q, K, V, w, B, N, H, d_model, stream);
        case 64: return quant_int8_d<64>(Q, K, V, w, B, N, H, d_model, stream);
        case 128: return quant_int8_d<128>(Q, K, V, w, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

template <int D>
static hipError_t fa_int8_d(const Int8Workspace& w, float* O, int B, int N, int H, int d_model, hipStream_t stream) {
    constexpr int WAVES = 4, SG = 2;
    const int G = N / QMHA_GROUP;
    const int nqb = (G + WAVES - 1) / WAVES;
    const int nwg = B * H * nqb;
    const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2e;  // inv_sqrt_d: fa_tc_int8_b.cu:587
    hipLaunchKernelGGL((qmha_fa_int8_kernel<D, WAVES, SG>), dim3(nwg), dim3(WAVES * 64), 0, stream, w.Qi, w.Ki, w.Vt,
                       w.sQ, w.sK, w.sV, O, N, H, d_model, nqb, c_log2);
    return hipGetLastError();
}

hipError_t launch_fa_int8_main(const Int8Workspace& w, float* O, int B, int N, int H, int D, int d_model,
                               hipStream_t stream) {
    switch (D) {
        case 32: return fa_int8_d<32>(w, O, B, N, H, d_model, stream);
        case 64: return fa_int8_d<64>(w, O, B, N, H, d_model, stream);
        case 128: return fa_int8_d<128>(w, O, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_debug_qk_int32(const Int8Workspace& w, int N, int D, int bh, int32_t* S, hipStream_t stream) {
    const int G = N / QMHA_GROUP;
    switch (D) {
        case 32: hipLaunchKernelGGL((qmha_debug_qk_int32_kernel<32>), dim3(G, G), dim3(64), 0, stream, w.Qi, w.Ki, N, bh, S); break;
        case 64: hipLaunchKernelGGL((qmha_debug_qk_int32_kernel<64>), dim3(G, G), dim3(64), 0, stream, w.Qi, w.Ki, N, bh, S); break;
        case 128: hipLaunchKernelGGL((qmha_debug_qk_int32_kernel<128>), dim3(G, G), dim3(64), 0, stream, w.Qi, w.Ki, N, bh, S); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace qmha
