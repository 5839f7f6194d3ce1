// qmha_fa_f32.hip -- scalar fp32 FlashAttention forward (no matrix cores), gfx950.
//
// Drop-in for the reference's fa (mha_kernels/fa.cu:211-425): fp32 operands, LDS tiling
// only, Bc = 32 online softmax with m0 = 0 (:279), epilogue guard 1e-10 (:371).
// Numerics follow fa.cu exactly where the order is defined by the reference:
//   S[r][j]  = fmaf chain over k = 0..d-1 from 0 (matmul_warp_tiled, :63-86 under nvcc's
//              default FMA contraction), then * (1/sqrt(d))          -> bit-identical S
//   O[r][:] *= alpha;  O[r][c] += (fmaf chain over the tile's 32 kv of P*V)  (:93-94)
// exp/sum use the GPU's expf, so O agrees with the oracle to ~1e-6, not bitwise.
//
// One workgroup = 32 query rows of one (batch, head), 256 threads = 4 wave64; thread
// (r = tid/8, c = tid%8) owns S[r][c + 8j] (j < 4) and O[r][c + 8j] (j < D/8).
#include "qmha_common.hpp"
#include "qmha_kernels.hpp"

namespace qmha {

template <int D>
__global__ __launch_bounds__(256) void qmha_fa_f32_kernel(const float* __restrict__ Q, const float* __restrict__ K,
                                                          const float* __restrict__ V, float* __restrict__ O, int N,
                                                          int H, int d_model, float inv_sqrt_d) {
    constexpr int DP = D + 1;  // padded row: column reads of K are conflict-free
    constexpr int OPT = D / 8;
    __shared__ float qs[32 * D];
    __shared__ float ks[32 * DP];
    __shared__ float vs[32 * D];
    __shared__ float ps[32 * 33];

    const int G = N / QMHA_GROUP;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = wg / G, qg = wg % G;
    const int b = bh / H, k = bh % H;
    const int tid = threadIdx.x, r = tid >> 3, c = tid & 7;
    const size_t head_off = (size_t)b * N * d_model + (size_t)k * D;

    for (int i = tid; i < 32 * D / 4; i += 256) {
        const int row = i / (D / 4), c4 = i % (D / 4);
        *reinterpret_cast<v4f*>(&qs[row * D + 4 * c4]) =
            *reinterpret_cast<const v4f*>(Q + head_off + (size_t)(qg * 32 + row) * d_model + 4 * c4);
    }
    float o[OPT];
#pragma unroll
    for (int j = 0; j < OPT; ++j) o[j] = 0.0f;
    float m_prev = 0.0f, l = 0.0f;

    for (int t = 0; t < G; ++t) {
        __syncthreads();  // previous tile's ks/vs/ps reads are done
        for (int i = tid; i < 32 * D / 4; i += 256) {
            const int row = i / (D / 4), c4 = i % (D / 4);
            const size_t g = head_off + (size_t)(t * 32 + row) * d_model + 4 * c4;
            const v4f kv = *reinterpret_cast<const v4f*>(K + g);
            const v4f vv = *reinterpret_cast<const v4f*>(V + g);
#pragma unroll
            for (int e = 0; e < 4; ++e) ks[row * DP + 4 * c4 + e] = kv[e];
            *reinterpret_cast<v4f*>(&vs[row * D + 4 * c4]) = vv;
        }
        __syncthreads();
        float s[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int kk = 0; kk < D; ++kk) {
            const float qv = qs[r * D + kk];
#pragma unroll
            for (int j = 0; j < 4; ++j) s[j] = fmaf(qv, ks[(c + 8 * j) * DP + kk], s[j]);
        }
        float mx = m_prev;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            s[j] *= inv_sqrt_d;  // fa.cu:141
            mx = fmaxf(mx, s[j]);
        }
        mx = fmaxf(mx, __shfl_xor(mx, 1));
        mx = fmaxf(mx, __shfl_xor(mx, 2));
        mx = fmaxf(mx, __shfl_xor(mx, 4));
        float rs = 0.0f;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float p = expf(s[j] - mx);  // fa.cu:167
            ps[r * 33 + c + 8 * j] = p;
            rs += p;
        }
        rs += __shfl_xor(rs, 1);
        rs += __shfl_xor(rs, 2);
        rs += __shfl_xor(rs, 4);
        const float alpha = expf(m_prev - mx);  // fa.cu:187
        l = fmaf(alpha, l, rs);                 // fa.cu:190
        m_prev = mx;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < OPT; ++j) {
            const int d = c + 8 * j;
            float acc = 0.0f;
#pragma unroll 8
            for (int kv = 0; kv < 32; ++kv) acc = fmaf(ps[r * 33 + kv], vs[kv * D + d], acc);
            o[j] = __fadd_rn(__fmul_rn(o[j], alpha), acc);  // fa.cu:199 then :94 (C += acc), no contraction
        }
    }
    float* orow = O + head_off + (size_t)(qg * 32 + r) * d_model;
    const bool ok = l > 1e-10f;
#pragma unroll
    for (int j = 0; j < OPT; ++j) orow[c + 8 * j] = ok ? o[j] / l : 0.0f;
}

template <int D>
static hipError_t fa_f32_d(const float* Q, const float* K, const float* V, float* O, int B, int N, int H, int d_model,
                           hipStream_t stream) {
    const int G = N / QMHA_GROUP;
    const float inv_sqrt_d = 1.0f / sqrtf((float)D);  // fa.cu:410
    hipLaunchKernelGGL((qmha_fa_f32_kernel<D>), dim3(B * H * G), dim3(256), 0, stream, Q, K, V, O, N, H, d_model,
                       inv_sqrt_d);
    return hipGetLastError();
}

hipError_t launch_fa_f32(const float* Q, const float* K, const float* V, float* O, int B, int N, int H, int D,
                         int d_model, hipStream_t stream) {
    switch (D) {
        case 32: return fa_f32_d<32>(Q, K, V, O, B, N, H, d_model, stream);
        case 64: return fa_f32_d<64>(Q, K, V, O, B, N, H, d_model, stream);
        case 128: return fa_f32_d<128>(Q, K, V, O, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace qmha
