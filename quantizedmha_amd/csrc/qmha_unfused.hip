// qmha_unfused.hip -- the reference's unfused 3-kernel baseline (mha_kernels/unfused.cu:7-185)
// for gfx950: S = alpha * Q K^T into an N x N fp32 scratch, row softmax, O = P V.
// Numerics follow unfused.cu: fp32 dot products (on the fp32 matrix cores: exact products,
// fp32 accumulation in the MFMA's order instead of the reference's ascending fmaf chain,
// :40,:74), S = alpha * sum (:80), softmax = exp(x - max) / sum (:130-166) with the row held
// in registers (one read and one write of S).  Scratch is bounded by processing heads in chunks (the reference keeps
// one N x N pair per stream, launchers.h:35-39).
#include "qmha_common.hpp"
#include "qmha_kernels.hpp"

namespace qmha {

static constexpr size_t kUnfusedScratchCap = (size_t)1 << 31;  // bytes of S per chunk

// C[bh][i][j] (ldc) = alpha * sum_k A[i][k] * B(k, j); B(k, j) = Bm[j][k] if BT else Bm[k][j].
// 64x64 output tile per workgroup, 256 threads x (4 x 4) outputs, 16-deep k slabs.
template <bool BT>
__global__ __launch_bounds__(256) void qmha_gemm_f32_kernel(const float* __restrict__ A, long long a_bh, int lda,
                                                            const float* __restrict__ Bm, long long b_bh, int ldb,
                                                            float* __restrict__ C, long long c_bh, int ldc, int M,
                                                            int Ncols, int Kd, float alpha, int H, int bh0,
                                                            long long a_b, long long b_b, long long c_b) {
    __shared__ float as[16][64 + 4];
    __shared__ float bs[16][64 + 4];
    const int bh = bh0 + blockIdx.z;
    const int b = bh / H, k = bh % H;
    const float* Ab = A + (long long)b * a_b + (long long)k * a_bh;
    const float* Bb = Bm + (long long)b * b_b + (long long)k * b_bh;
    float* Cb = C + (long long)b * c_b + (long long)k * c_bh;
    const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
    const int tid = threadIdx.x, ty = tid / 16, tx = tid % 16;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < Kd; k0 += 16) {
        for (int e = tid; e < 16 * 64; e += 256) {
            const int r = e / 16, kk = e % 16;  // A tile: 64 rows x 16 k
            const int gi = i0 + r, gk = k0 + kk;
            as[kk][r] = (gi < M && gk < Kd) ? Ab[(long long)gi * lda + gk] : 0.0f;
            if (BT) {
                const int gj = j0 + r;
                bs[kk][r] = (gj < Ncols && gk < Kd) ? Bb[(long long)gj * ldb + gk] : 0.0f;
            }
        }
        if (!BT) {
            for (int e = tid; e < 16 * 64; e += 256) {
                const int kk = e / 64, c = e % 64;
                const int gk = k0 + kk, gj = j0 + c;
                bs[kk][c] = (gj < Ncols && gk < Kd) ? Bb[(long long)gk * ldb + gj] : 0.0f;
            }
        }
        __syncthreads();
        const int kmax = min(16, Kd - k0);
        for (int kk = 0; kk < kmax; ++kk) {
            float a[4], bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = as[kk][ty + 16 * u];
#pragma unroll
            for (int v = 0; v < 4; ++v) bv[v] = bs[kk][tx + 16 * v];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int v = 0; v < 4; ++v) acc[u][v] = fmaf(a[u], bv[v], acc[u][v]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
            const int gi = i0 + ty + 16 * u, gj = j0 + tx + 16 * v;
            if (gi < M && gj < Ncols) Cb[(long long)gi * ldc + gj] = alpha == 1.0f ? acc[u][v] : alpha * acc[u][v];
        }
}

// The same GEMM on the fp32 matrix cores: 64x64 output tile per workgroup, 4 waves of 32x32,
// v_mfma_f32_32x32x2_f32 over 16-deep k slabs staged in LDS exactly as above (exact fp32
// products and fp32 accumulation; the summation order is the MFMA's, not an ascending fmaf chain).
template <bool BT>
__global__ __launch_bounds__(256) void qmha_gemm_f32_mfma_kernel(const float* __restrict__ A, long long a_bh, int lda,
                                                                 const float* __restrict__ Bm, long long b_bh, int ldb,
                                                                 float* __restrict__ C, long long c_bh, int ldc, int M,
                                                                 int Ncols, int Kd, float alpha, int H, int bh0,
                                                                 long long a_b, long long b_b, long long c_b) {
    __shared__ float as[16][64 + 4];
    __shared__ float bs[16][64 + 4];
    const int bh = bh0 + blockIdx.z;
    const int b = bh / H, k = bh % H;
    const float* Ab = A + (long long)b * a_b + (long long)k * a_bh;
    const float* Bb = Bm + (long long)b * b_b + (long long)k * b_bh;
    float* Cb = C + (long long)b * c_b + (long long)k * c_bh;
    const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1, half = lane >> 5, col = lane & 31;
    v16f acc = v16f{};
    for (int k0 = 0; k0 < Kd; k0 += 16) {
        for (int e = tid; e < 16 * 64; e += 256) {
            const int r = e / 16, kk = e % 16;  // A tile: 64 rows x 16 k
            const int gi = i0 + r, gk = k0 + kk;
            as[kk][r] = (gi < M && gk < Kd) ? Ab[(long long)gi * lda + gk] : 0.0f;
            if (BT) {
                const int gj = j0 + r;
                bs[kk][r] = (gj < Ncols && gk < Kd) ? Bb[(long long)gj * ldb + gk] : 0.0f;
            }
        }
        if (!BT) {
            for (int e = tid; e < 16 * 64; e += 256) {
                const int kk = e / 64, c = e % 64;
                const int gk = k0 + kk, gj = j0 + c;
                bs[kk][c] = (gj < Ncols && gk < Kd) ? Bb[(long long)gk * ldb + gj] : 0.0f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k2 = 0; k2 < 8; ++k2)  // zero-filled past Kd, so whole slabs are safe
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(as[2 * k2 + half][32 * wr + col], bs[2 * k2 + half][32 * wc + col],
                                                        acc, 0, 0, 0);
        __syncthreads();
    }
    // lane (col, half) holds rows 8 (r/4) + 4 half + r%4 of column col of the wave's 32x32 block
    const int gj = j0 + 32 * wc + col;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int gi = i0 + 32 * wr + 8 * (r >> 2) + 4 * half + (r & 3);
        if (gi < M && gj < Ncols) Cb[(long long)gi * ldc + gj] = alpha == 1.0f ? acc[r] : alpha * acc[r];
    }
}

// In-place row softmax over rows of length N (unfused.cu:105-166), one workgroup per row.
__global__ __launch_bounds__(256) void qmha_softmax_rows_kernel(float* __restrict__ S, int N) {
    __shared__ float red[256];
    float* row = S + (long long)blockIdx.x * N;
    const int tid = threadIdx.x;
    float mx = -INFINITY;
    for (int i = tid; i < N; i += 256) mx = fmaxf(mx, row[i]);
    red[tid] = mx;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) red[tid] = fmaxf(red[tid], red[tid + s]);
        __syncthreads();
    }
    mx = red[0];
    __syncthreads();
    float sum = 0.0f;
    for (int i = tid; i < N; i += 256) {
        const float e = expf(row[i] - mx);
        row[i] = e;
        sum += e;
    }
    red[tid] = sum;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (tid < s) red[tid] = red[tid] + red[tid + s];
        __syncthreads();
    }
    sum = red[0];
    for (int i = tid; i < N; i += 256) row[i] = row[i] / sum;
}

// The same row softmax with the row held in registers: one read and one write of S instead of
// three reads and two writes (the pass is HBM-bound).  NV4 float4 per thread, N = 1024 * NV4.
__device__ __forceinline__ float block_reduce256(float v, float* red, bool is_max) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float w = __shfl_xor(v, o);
        v = is_max ? fmaxf(v, w) : v + w;
    }
    const int tid = threadIdx.x;
    __syncthreads();  // red[] of a previous reduction has been read
    if ((tid & 63) == 0) red[tid >> 6] = v;
    __syncthreads();
    return is_max ? fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])) : (red[0] + red[1]) + (red[2] + red[3]);
}

template <int NV4>
__global__ __launch_bounds__(256) void qmha_softmax_rows_reg_kernel(float* __restrict__ S, int N) {
    __shared__ float red[4];
    float* row = S + (long long)blockIdx.x * N;
    const int tid = threadIdx.x;
    v4f x[NV4];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
        x[i] = *reinterpret_cast<const v4f*>(row + 4 * (i * 256 + tid));
#pragma unroll
        for (int e = 0; e < 4; ++e) mx = fmaxf(mx, x[i][e]);
    }
    mx = block_reduce256(mx, red, true);
    float sum = 0.0f;
#pragma unroll
    for (int i = 0; i < NV4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            x[i][e] = expf(x[i][e] - mx);  // unfused.cu:145
            sum += x[i][e];
        }
    sum = block_reduce256(sum, red, false);
#pragma unroll
    for (int i = 0; i < NV4; ++i) {
        v4f w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = x[i][e] / sum;  // unfused.cu:160
        *reinterpret_cast<v4f*>(row + 4 * (i * 256 + tid)) = w;
    }
}

static hipError_t launch_softmax_rows(float* S, int rows, int N, hipStream_t stream) {
    switch (N) {  // register-resident rows for the common sizes, the three-pass kernel otherwise
        case 1024: hipLaunchKernelGGL((qmha_softmax_rows_reg_kernel<1>), dim3(rows), dim3(256), 0, stream, S, N); break;
        case 2048: hipLaunchKernelGGL((qmha_softmax_rows_reg_kernel<2>), dim3(rows), dim3(256), 0, stream, S, N); break;
        case 4096: hipLaunchKernelGGL((qmha_softmax_rows_reg_kernel<4>), dim3(rows), dim3(256), 0, stream, S, N); break;
        case 8192: hipLaunchKernelGGL((qmha_softmax_rows_reg_kernel<8>), dim3(rows), dim3(256), 0, stream, S, N); break;
        default: hipLaunchKernelGGL(qmha_softmax_rows_kernel, dim3(rows), dim3(256), 0, stream, S, N); break;
    }
    return hipGetLastError();
}

static int unfused_chunk(int BH, int N) {
    const size_t per = (size_t)N * N * sizeof(float);
    size_t c = kUnfusedScratchCap / per;
    if (c < 1) c = 1;
    if (c > (size_t)BH) c = BH;
    return (int)c;
}

size_t unfused_workspace_bytes(int B, int N, int H, int D) {
    (void)D;
    return align_up((size_t)unfused_chunk(B * H, N) * N * N * sizeof(float), 256);
}

hipError_t launch_unfused(const float* Q, const float* K, const float* V, float* O, void* ws, int B, int N, int H,
                          int D, int d_model, hipStream_t stream) {
    const int BH = B * H;
    const int chunk = unfused_chunk(BH, N);
    float* S = static_cast<float*>(ws);
    const float alpha = 1.0f / sqrtf((float)D);  // launchers.h:20
    const long long nd = (long long)N * d_model, nn = (long long)N * N;
    for (int bh0 = 0; bh0 < BH; bh0 += chunk) {
        const int cnt = min(chunk, BH - bh0);
        // S[c] = alpha * Q_bh K_bh^T ; S is indexed by (bh - bh0): use b = 0, k = bh - bh0 strides
        dim3 g1((N + 63) / 64, (N + 63) / 64, cnt);
        hipLaunchKernelGGL((qmha_gemm_f32_mfma_kernel<true>), g1, dim3(256), 0, stream, Q, (long long)D, d_model, K,
                           (long long)D, d_model, S - (long long)bh0 * nn, nn, N, N, N, D, alpha, H, bh0, nd, nd,
                           (long long)H * nn);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        e = launch_softmax_rows(S, cnt * N, N, stream);
        if (e != hipSuccess) return e;
        dim3 g3((D + 63) / 64, (N + 63) / 64, cnt);
        hipLaunchKernelGGL((qmha_gemm_f32_mfma_kernel<false>), g3, dim3(256), 0, stream, (const float*)(S - (long long)bh0 * nn),
                           nn, N, V, (long long)D, d_model, O, (long long)D, d_model, N, D, N, 1.0f, H, bh0,
                           (long long)H * nn, nd, nd);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace qmha
