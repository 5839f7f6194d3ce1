// qmha_fa_f32.hip -- fp32 FlashAttention forward for gfx950: the reference's `fa`
// (mha_kernels/fa.cu:211-425) as a scalar kernel (variant fa: fp32 operands, VALU fmaf, LDS
// tiling only -- BASELINE config 2 "no tensor cores") and the same contract on the fp32 matrix
// cores (variant fa_mfma).  Both: Bc = 32 online softmax with m0 = 0 (:279), epilogue guard
// 1e-10 (:371).  The scalar kernel follows fa.cu's summation order exactly:
//   S[r][j]  = fmaf chain over k = 0..d-1 from 0 (matmul_warp_tiled, :63-86 under nvcc's
//              default FMA contraction), then * (1/sqrt(d))          -> bit-identical S
//   O[r][:] *= alpha;  O[r][c] += (fmaf chain over the tile's 32 kv of P*V)  (:93-94)
// exp is exp2(x * log2 e) on v_exp_f32 (2 VALU ops; OCML's expf is ~13 per element with its
// range checks, and its SGPR constants run at the slow issue rate): p differs from the
// reference's expf by ~1e-6 relative, so O agrees with the oracle to ~1e-6, not bitwise.
#include "qmha_common.hpp"
#include "qmha_kernels.hpp"

namespace qmha {

// e^x as 2^(x log2 e): the rounding of x log2 e costs |x| * 2^-24 relative (< 2e-6 for the
// |x| < 30 a softmax sees before p underflows), v_exp_f32 itself ~1 ulp
__device__ __forceinline__ float exp_e(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

// ---------------------------------------------------------------------------------------
// `fa`: the scalar kernel (VALU fmaf only, LDS tiling, no matrix cores -- BASELINE config 2 as
// written, the reference's no-tensor-core comparison point, README.md:12).  One workgroup = NT
// threads = NT/8 * RPT query rows of one (batch, head); thread (rp = tid / 8, c = tid % 8) owns
// rows rp + (NT/8) i (i < RPT).  S phase: columns 4c..4c+3 of the 32-key tile, K kept
// transposed in LDS so the four keys come in one ds_read_b128, Q read four k at a time; P@V
// phase: output columns 32h + 4c .. +3.  Every K / V / P vector read from LDS feeds RPT rows
// (RPT = 4: ~0.1 b128 reads per FMA).  Every S and P@V sum keeps the reference's sequential
// fmaf order (fa.cu:63-86 under nvcc's default contraction; :93-94): S is bit-identical to the
// oracle's, O differs only through exp.  K/V of tile t+1 are prefetched into registers while
// tile t computes (fa.cu stages them through shared memory the same way, :300-330).
template <int D, int RPT, int NT>
__global__ __launch_bounds__(NT) void qmha_fa_f32_v3_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                             const float* __restrict__ V, float* __restrict__ O, int N,
                                                             int H, int d_model, float inv_sqrt_d) {
    constexpr int QS = D + 4;   // q row stride (floats): b128 row reads hit distinct banks
    constexpr int KTS = 36;     // transposed K: [D][32 keys + 4]
    constexpr int VS = D + 4;   // V rows
    constexpr int PS = 36;      // P rows [R][32 + 4]
    constexpr int CH = D / 32;  // 4-column output chunks per thread
    constexpr int RS = NT / 8;            // row groups = row stride between a thread's rows
    constexpr int R = RS * RPT;           // query rows per workgroup
    constexpr int LD = 32 * D / 4 / NT;   // float4 of K (and of V) per thread per tile
    static_assert(LD >= 1, "d >= 32");
    __shared__ __attribute__((aligned(16))) float qs[R * QS];
    __shared__ __attribute__((aligned(16))) float kt[D * KTS];
    __shared__ __attribute__((aligned(16))) float vs[32 * VS];
    __shared__ __attribute__((aligned(16))) float ps[R * PS];

    const int G = N / QMHA_GROUP;
    const int nqb = (N + R - 1) / R;  // R-row query blocks
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = wg / nqb, qb = wg % nqb;
    const int b = bh / H, k = bh % H;
    const int tid = threadIdx.x, rp = tid >> 3, c = tid & 7;
    const size_t head_off = (size_t)b * N * d_model + (size_t)k * D;
    const int row0 = qb * R;

    for (int i = tid; i < R * D / 4; i += NT) {
        const int row = i / (D / 4), c4 = i % (D / 4);
        v4f x = {0.0f, 0.0f, 0.0f, 0.0f};
        if (row0 + row < N) x = *reinterpret_cast<const v4f*>(Q + head_off + (size_t)(row0 + row) * d_model + 4 * c4);
        *reinterpret_cast<v4f*>(&qs[row * QS + 4 * c4]) = x;
    }
    float o[RPT][CH][4];
#pragma unroll
    for (int i = 0; i < RPT; ++i)
#pragma unroll
        for (int h = 0; h < CH; ++h)
#pragma unroll
            for (int e = 0; e < 4; ++e) o[i][h][e] = 0.0f;
    float m_prev[RPT], l[RPT];  // m0 = 0 (fa.cu:279)
#pragma unroll
    for (int i = 0; i < RPT; ++i) m_prev[i] = l[i] = 0.0f;

    v4f kreg[LD], vreg[LD];
    auto gload = [&](int t) {
#pragma unroll
        for (int j = 0; j < LD; ++j) {
            const int i = tid + NT * j, row = i / (D / 4), c4 = i % (D / 4);
            const size_t g = head_off + (size_t)(t * 32 + row) * d_model + 4 * c4;
            kreg[j] = *reinterpret_cast<const v4f*>(K + g);
            vreg[j] = *reinterpret_cast<const v4f*>(V + g);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int j = 0; j < LD; ++j) {
            const int i = tid + NT * j, row = i / (D / 4), c4 = i % (D / 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) kt[(4 * c4 + e) * KTS + row] = kreg[j][e];
            *reinterpret_cast<v4f*>(&vs[row * VS + 4 * c4]) = vreg[j];
        }
    };

    gload(0);
    for (int t = 0; t < G; ++t) {
        __syncthreads();  // the previous tile's kt/vs/ps reads are done
        lstore();
        __syncthreads();
        if (t + 1 < G) gload(t + 1);  // in flight during this tile's compute
        // ---- S = Q K^T (fa.cu:24-102): sequential fmaf chain over k from 0, then * 1/sqrt(d)
        float sacc[RPT][4] = {};
#pragma unroll 4
        for (int kk = 0; kk < D; kk += 4) {
            v4f qv[RPT];
#pragma unroll
            for (int i = 0; i < RPT; ++i) qv[i] = *reinterpret_cast<const v4f*>(&qs[(rp + RS * i) * QS + kk]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const v4f kv = *reinterpret_cast<const v4f*>(&kt[(kk + e) * KTS + 4 * c]);
#pragma unroll
                for (int i = 0; i < RPT; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) sacc[i][j] = fmaf(qv[i][e], kv[j], sacc[i][j]);
            }
        }
        // ---- online softmax per row (fa.cu:106-209); the row's 32 scores live on 8 lanes
        float alpha[RPT];
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            float mx = m_prev[i];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                sacc[i][j] *= inv_sqrt_d;  // fa.cu:141
                mx = fmaxf(mx, sacc[i][j]);
            }
            mx = fmaxf(mx, __shfl_xor(mx, 1));
            mx = fmaxf(mx, __shfl_xor(mx, 2));
            mx = fmaxf(mx, __shfl_xor(mx, 4));
            v4f pv;
            float rs = 0.0f;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pv[j] = exp_e(sacc[i][j] - mx);  // fa.cu:167
                rs += pv[j];
            }
            *reinterpret_cast<v4f*>(&ps[(rp + RS * i) * PS + 4 * c]) = pv;
            rs += __shfl_xor(rs, 1);
            rs += __shfl_xor(rs, 2);
            rs += __shfl_xor(rs, 4);
            alpha[i] = exp_e(m_prev[i] - mx);  // fa.cu:187
            l[i] = fmaf(alpha[i], l[i], rs);  // fa.cu:190
            m_prev[i] = mx;
        }
        __syncthreads();
        // ---- O = alpha*O + P V (fa.cu:93-94,199): sequential fmaf chain over the tile's keys
        float acc[RPT][CH][4] = {};
#pragma unroll 2
        for (int kv = 0; kv < 32; kv += 4) {
            v4f pr[RPT];
#pragma unroll
            for (int i = 0; i < RPT; ++i) pr[i] = *reinterpret_cast<const v4f*>(&ps[(rp + RS * i) * PS + kv]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
#pragma unroll
                for (int h = 0; h < CH; ++h) {
                    const v4f vv = *reinterpret_cast<const v4f*>(&vs[(kv + e) * VS + 32 * h + 4 * c]);
#pragma unroll
                    for (int i = 0; i < RPT; ++i)
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[i][h][j] = fmaf(pr[i][e], vv[j], acc[i][h][j]);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < RPT; ++i)
#pragma unroll
            for (int h = 0; h < CH; ++h)
#pragma unroll
                for (int j = 0; j < 4; ++j) o[i][h][j] = __fadd_rn(__fmul_rn(o[i][h][j], alpha[i]), acc[i][h][j]);
    }
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        const int row = row0 + rp + RS * i;
        if (row >= N) continue;
        const bool ok = l[i] > 1e-10f;  // fa.cu:371
        float* orow = O + head_off + (size_t)row * d_model;
#pragma unroll
        for (int h = 0; h < CH; ++h) {
            v4f w;
#pragma unroll
            for (int j = 0; j < 4; ++j) w[j] = ok ? o[i][h][j] / l[i] : 0.0f;
            *reinterpret_cast<v4f*>(orow + 32 * h + 4 * c) = w;
        }
    }
}

// ---------------------------------------------------------------------------------------
// v4: the same contract on the fp32 matrix cores.  v_mfma_f32_32x32x2_f32 (exact fp32
// products, fp32 accumulation; 64 FLOP/clk/SIMD, the fp32 vector rate) for both products, so
// the FMAs leave the VALU and the LDS operand traffic per FLOP drops 32x.  One workgroup = 4
// waves = 128 query rows of one head, one 32-row group per wave; swapped products as in the
// int8/fp16 kernels: S^T = K Q^T (lane (q, h) holds 16 keys of query q), O^T = V^T P^T with P^T
// straight from the S^T accumulator (step r of P@V takes accumulator register r; its two keys
// 8(r/4) + 4h + r%4 select the V^T operand).  The d order of the Q.K dot is d = s + h D/2 (lane
// half h supplies the second k-entry of each 32x32x2 step), the key order of P.V is the
// accumulator's: both differ from fa.cu's sequential fmaf chains only by fp32 rounding order.
// Softmax arithmetic as v3 (scores * 1/sqrt(d), m0 = 0, alpha, l = fma(alpha, l, rowsum),
// O = O*alpha + PV, guard 1e-10).
// ---------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256, D <= 64 ? 3 : (D <= 128 ? 2 : 1)) void qmha_fa_f32_mfma_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, float* __restrict__ O,
    int N, int H, int d_model, float inv_sqrt_d) {
    constexpr int HD = D / 2, MB = D / 32;
    constexpr int KST = D + 4;  // K rows (floats): b128 reads of 32 rows spread over the banks
    constexpr int VST = 36;     // V^T rows [D][32 keys + 4]
    constexpr int LD = 32 * D / 4 / 256;  // float4 of K (and of V) per thread per tile
    static_assert(LD >= 1, "d >= 32");
    __shared__ __attribute__((aligned(16))) float kl[32 * KST];
    __shared__ __attribute__((aligned(16))) float vt[D * VST];

    const int G = N / QMHA_GROUP;
    const int nqb = (G + 3) / 4;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = wg / nqb, qb = wg % nqb;
    const int b = bh / H, k = bh % H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int half = lane >> 5, col = lane & 31;
    const int qg = qb * 4 + wave;
    const bool active = qg < G;  // wave-uniform; an inactive wave still stages and syncs
    const size_t head_off = (size_t)b * N * d_model + (size_t)k * D;

    float qop[HD];  // Q[q][h D/2 + s], s < D/2: the B operand of Q.K step s
    {
        const float* qrow = Q + head_off + (size_t)(qg * QMHA_GROUP + col) * d_model + half * HD;
#pragma unroll
        for (int j = 0; j < HD / 4; ++j) {
            v4f x = {0.0f, 0.0f, 0.0f, 0.0f};
            if (active) x = *reinterpret_cast<const v4f*>(qrow + 4 * j);
#pragma unroll
            for (int e = 0; e < 4; ++e) qop[4 * j + e] = x[e];
        }
    }
    v16f o[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) o[m] = v16f{};
    float m_prev = 0.0f, l = 0.0f;  // m0 = 0 (fa.cu:279)

    v4f kreg[LD], vreg[LD];
    auto gload = [&](int t) {
#pragma unroll
        for (int j = 0; j < LD; ++j) {
            const int i = tid + 256 * j, row = i / (D / 4), c4 = i % (D / 4);
            const size_t g = head_off + (size_t)(t * 32 + row) * d_model + 4 * c4;
            kreg[j] = *reinterpret_cast<const v4f*>(K + g);
            vreg[j] = *reinterpret_cast<const v4f*>(V + g);
        }
    };
    auto lstore = [&]() {
#pragma unroll
        for (int j = 0; j < LD; ++j) {
            const int i = tid + 256 * j, row = i / (D / 4), c4 = i % (D / 4);
            *reinterpret_cast<v4f*>(&kl[row * KST + 4 * c4]) = kreg[j];
#pragma unroll
            for (int e = 0; e < 4; ++e) vt[(4 * c4 + e) * VST + row] = vreg[j][e];
        }
    };

    gload(0);
    for (int t = 0; t < G; ++t) {
        __syncthreads();  // the previous tile's kl / vt reads are done
        lstore();
        __syncthreads();
        if (t + 1 < G) gload(t + 1);  // in flight during this tile's MFMAs
        // ---- S^T = K Q^T (fa.cu:24-102), then * 1/sqrt(d) (:141)
        v16f s = v16f{};
#pragma unroll
        for (int j = 0; j < HD / 4; ++j) {
            const v4f kv = *reinterpret_cast<const v4f*>(&kl[col * KST + half * HD + 4 * j]);
#pragma unroll
            for (int e = 0; e < 4; ++e) s = __builtin_amdgcn_mfma_f32_32x32x2f32(kv[e], qop[4 * j + e], s, 0, 0, 0);
        }
        // ---- online softmax (fa.cu:106-209): 16 keys per lane, the two lane halves joined
        float mx = m_prev;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            s[r] *= inv_sqrt_d;
            mx = fmaxf(mx, s[r]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        float p[16], rs = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            p[r] = exp_e(s[r] - mx);  // fa.cu:167
            rs += p[r];
        }
        rs += __shfl_xor(rs, 32);
        const float alpha = exp_e(m_prev - mx);  // fa.cu:187
        l = fmaf(alpha, l, rs);                   // fa.cu:190
        m_prev = mx;
        // ---- O = alpha*O + P V (fa.cu:93-94,199)
#pragma unroll
        for (int m = 0; m < MB; ++m) {
            v16f a = v16f{};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const v4f vv = *reinterpret_cast<const v4f*>(&vt[(32 * m + col) * VST + 8 * j + 4 * half]);
#pragma unroll
                for (int e = 0; e < 4; ++e) a = __builtin_amdgcn_mfma_f32_32x32x2f32(vv[e], p[4 * j + e], a, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) o[m][r] = __fadd_rn(__fmul_rn(o[m][r], alpha), a[r]);
        }
    }
    if (!active) return;
    // lane (q, h) holds O^T rows d = 32 m + 8 g + 4 h + e (e < 4) of query q
    const bool ok = l > 1e-10f;  // fa.cu:371
    float* orow = O + head_off + (size_t)(qg * QMHA_GROUP + col) * d_model + 4 * half;
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            v4f w;
#pragma unroll
            for (int e = 0; e < 4; ++e) w[e] = ok ? o[m][4 * g4 + e] / l : 0.0f;
            *reinterpret_cast<v4f*>(orow + 32 * m + 8 * g4) = w;
        }
}

template <int D>
static hipError_t fa_f32_mfma(const float* Q, const float* K, const float* V, float* O, int B, int N, int H,
                              int d_model, hipStream_t stream) {
    const int G = N / QMHA_GROUP;
    const float inv_sqrt_d = 1.0f / sqrtf((float)D);  // fa.cu:410
    hipLaunchKernelGGL((qmha_fa_f32_mfma_kernel<D>), dim3(B * H * ((G + 3) / 4)), dim3(256), 0, stream, Q, K, V, O, N,
                       H, d_model, inv_sqrt_d);
    return hipGetLastError();
}

template <int D, int RPT, int NT>
static hipError_t fa_f32_v3(const float* Q, const float* K, const float* V, float* O, int B, int N, int H, int d_model,
                            hipStream_t stream) {
    constexpr int R = NT / 8 * RPT;
    const float inv_sqrt_d = 1.0f / sqrtf((float)D);  // fa.cu:410
    hipLaunchKernelGGL((qmha_fa_f32_v3_kernel<D, RPT, NT>), dim3(B * H * ((N + R - 1) / R)), dim3(NT), 0, stream, Q, K,
                       V, O, N, H, d_model, inv_sqrt_d);
    return hipGetLastError();
}

hipError_t launch_fa_f32(const float* Q, const float* K, const float* V, float* O, int B, int N, int H, int D,
                         int d_model, bool mfma, hipStream_t stream) {
    if (mfma) {  // fa_mfma: v4 on the fp32 matrix cores (128 query rows per workgroup)
        switch (D) {
            case 32: return fa_f32_mfma<32>(Q, K, V, O, B, N, H, d_model, stream);
            case 64: return fa_f32_mfma<64>(Q, K, V, O, B, N, H, d_model, stream);
            case 128: return fa_f32_mfma<128>(Q, K, V, O, B, N, H, d_model, stream);
            case 96: return fa_f32_mfma<96>(Q, K, V, O, B, N, H, d_model, stream);
            case 160: return fa_f32_mfma<160>(Q, K, V, O, B, N, H, d_model, stream);
            case 192: return fa_f32_mfma<192>(Q, K, V, O, B, N, H, d_model, stream);
            case 224: return fa_f32_mfma<224>(Q, K, V, O, B, N, H, d_model, stream);
            case 256: return fa_f32_mfma<256>(Q, K, V, O, B, N, H, d_model, stream);
            default: return hipErrorInvalidValue;
        }
    }
#ifdef QMHA_ABLATION  // scalar-kernel geometry alternatives at d = 64: profiling builds only
    if (D == 64) {
        switch (tune_config("QMHA_F32_CFG")) {
            case 34: return fa_f32_v3<64, 4, 128>(Q, K, V, O, B, N, H, d_model, stream);
            case 36: return fa_f32_v3<64, 2, 256>(Q, K, V, O, B, N, H, d_model, stream);
            case 37: return fa_f32_v3<64, 2, 128>(Q, K, V, O, B, N, H, d_model, stream);
            default: break;
        }
    }
#endif
    // fa: the scalar kernel, 4 rows per thread (128 rows per workgroup; 64 above d = 64, whose
    // Q / K / V / P tiles would otherwise take up to 280 KiB of LDS: 146 KiB at d = 256)
    switch (D) {
        case 32: return fa_f32_v3<32, 4, 256>(Q, K, V, O, B, N, H, d_model, stream);
        case 64: return fa_f32_v3<64, 4, 256>(Q, K, V, O, B, N, H, d_model, stream);
        case 128: return fa_f32_v3<128, 2, 256>(Q, K, V, O, B, N, H, d_model, stream);
        case 96: return fa_f32_v3<96, 2, 256>(Q, K, V, O, B, N, H, d_model, stream);
        case 160: return fa_f32_v3<160, 2, 256>(Q, K, V, O, B, N, H, d_model, stream);
        case 192: return fa_f32_v3<192, 2, 256>(Q, K, V, O, B, N, H, d_model, stream);
        case 224: return fa_f32_v3<224, 2, 256>(Q, K, V, O, B, N, H, d_model, stream);
        case 256: return fa_f32_v3<256, 2, 256>(Q, K, V, O, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace qmha
