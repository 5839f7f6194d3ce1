// qmha_fa_int8.hip -- fused INT8 FlashAttention-2 forward for gfx950 (MI355X).
//
// Drop-in for the reference's fa_tc_int8_b (mha_kernels/fa_tc_int8_b.cu:408-609) with its
// *intended* numerics:
//   per 32-row group of Q, K, V:  s = max(absmax/127, 1e-8), x_i8 = clamp(rint(x * (1/s)))
//   S = Qi Ki^T (int32, exact)        -> scores = S * sQ * sK / sqrt(d)
//   online softmax per 32-key tile, m0 = 0 -> p = exp(scores - m), l = alpha*l + sum(p)
//   per 32x32 tile P: sP = max(max p / 127, 1e-8), Pi = rint(p / sP)
//   O = alpha*O + (Pi Vi) * sP * sV,   out = O / l  (0 if l <= 1e-20)
//
// Two launches per call:
//   1. qmha_quant_int8_kernel (qmha_prepass.hip): reads fp32 K/V once; writes int8 K rows per head and the
//      quantised V integers in the MFMA V^T operand order, one fp32 scale per group.
//      Bit-identical to the reference quantiser (same fp32 ops, RNE rounding).  (With Q too
//      for qmha_quantize_int8 and the int32 Q@K^T test hook.)
//   2. the main kernel: one workgroup = 4 waves = 128 query rows of one head; each wave owns one
//      32-row Q group, quantises it in registers (the same arithmetic) and sweeps all KV groups.
//      K/V tiles stream L2 -> LDS by LDS-DMA (swizzled image, conflict-free ds_read_b128).
//      Both products use swapped operands (S^T = K Q^T, O^T = V^T P^T) so every query's
//      statistics are lane-local and P^T feeds the second MFMA from registers.
//        Q@K^T: v_mfma_i32_32x32x32_i8, exact int32 scores.
//        P@V  : the int8-valued operands Pi in [0,127], Vi in [-128,127] run on
//               v_mfma_f32_32x32x16_f16.  Both are exact in f16, every product and every
//               partial sum (|sum| <= 32*127*128 < 2^24) is exact in the fp32 accumulator,
//               so the result equals the reference's int32 (Pi Vi) bit for bit -- but it
//               arrives as fp32, saving the 32 int->float conversions per lane per tile.
//      d = 32 / 64 / 128: the software-pipelined qmha_fa_int8_pipe_kernel (P@V of tile t-1 and
//      Q@K^T of tile t+1 issued between the softmax chunks of tile t).  Every other head size the
//      reference accepts (d % 32 == 0, include/config.h:32; here up to 256): the one-tile-at-a-time
//      qmha_fa_int8_kernel (also N = 32, where there is nothing to pipeline).
//
// This is the production source: only the schedules the library ships.  The r01-r03 experiment
// branches (ablation perturbations, ring / DMA-split / TSHADOW / ACC1 schedules, the per-workgroup
// timeline) were kept in tools/ablation/qmha_fa_int8_ablation.hip until round 5 (git history, up to
// commit 6d5deec); DESIGN.md cites their measurements.
#include "qmha_common.hpp"
#include "qmha_kernels.hpp"

#include <atomic>
#include <type_traits>

namespace qmha {

// log2(e): the softmax runs in base 2 (v_exp_f32), scores pre-multiplied by log2(e).
static constexpr float kLog2e = 1.4426950408889634f;
// The per-tensor mode's lazy softmax base: a row's base moves only when the p of one of its
// key halves sum above 2047/127 on a tile, so every p <= 2047/127 and Pi = rint(127 p) <= 2047 stays below
// 2048, where the magic-number Pi bits are still the f16 encoding of Pi * 2^-24.
static constexpr float kPtSumCap = 2047.0f / 127.0f;

// A NaN in the caller's Q becomes 0 before the quantiser sees it, explicitly (integer test on the
// bits): the reference's fmaxf drops a NaN from the group absmax and __float2int_rn maps it to 0
// (the oracle's fp32_to_int8sram restatement).  This translation unit is built with
// -fno-honor-nans, so a float self-compare would be folded away (round-3 ADVICE).
__device__ __forceinline__ float nan_to_zero(float x) {
    return (__float_as_uint(x) & 0x7fffffffu) > 0x7f800000u ? 0.0f : x;
}

// In-kernel Q quantisation (fa_tc_int8_b.cu:33-152, the pre-pass arithmetic) straight into
// the Q^T MFMA operand: lane (col, half) loads the D/2 values of query row `col` it feeds to
// the i8 MFMA (bytes [32 s + 16 half, +16) of every k-step s), the wave reduces the group's
// absmax.  Returns the group scale sQ.  Saves the pre-pass a third of its HBM traffic.
// slice_sc > 0: the per-tensor mode's head-slice scale (no group absmax)
template <int D>
__device__ __forceinline__ float quant_q_operand(const float* __restrict__ row, int half, v4i (&qop)[D / 32],
                                                 float slice_sc = 0.0f) {
    constexpr int KS = D / 32;
    v4f x[KS][4];
    float amax = 0.0f;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
            x[s][c4] = *reinterpret_cast<const v4f*>(row + 32 * s + 16 * half + 4 * c4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                x[s][c4][e] = nan_to_zero(x[s][c4][e]);
                amax = fmaxf(amax, fabsf(x[s][c4][e]));
            }
        }
    const float sc = slice_sc > 0.0f ? slice_sc : qmha_scale_from_absmax(wave_max64(amax));
    const float inv = 1.0f / sc;
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
            uint32_t w = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) w |= ((uint32_t)(uint8_t)qmha_quant_i8(x[s][c4][e], inv)) << (8 * e);
            qop[s][c4] = (int)w;
        }
    return sc;
}

// Build-time flags of the main kernels:
//   FL_MAGIC  the Q@K^T chain starts from the bits of 1.5*2^23, so every int32 accumulator lane
//             reads as the float 1.5*2^23 + S (exact: |S| <= 127^2 d < 2^22 for d <= 256); float(S)
//             is one subtract (replaces a v_cvt_f32_i32)
//   FL_LB2 / FL_LB4  register budget of 2 waves per SIMD (256 VGPRs) / 4 (128); default 3 (pipe)
//   FL_LB1    (one-tile kernel, d > 128) one wave per SIMD: VGPRs + AGPRs (O alone is d/2 per lane)
//   FL_JIT    (pipe kernel) operands read right before their MFMA (fewer live VGPRs, d = 128)
//   FL_KFOLD  (pipe kernel, with FL_MAGIC) the exponent read straight off the biased
//             accumulator: the bias folded into the shift (see the kernel)
//   FL_DUMP   also store what the kernel itself computed: the int32 S^T of every tile (bias
//             removed), its in-register Q operand and sQ (qmha_debug_fa_int8_dump: the bit-exact
//             check of the production Q@K^T path; never the production launch)
//   FL_PT     (pipe kernel) the per-tensor mode fa_tc_int8_pt
// Measured and not shipped (the sources are in git history up to commit df5dced):
// the K/V pre-pass inside the sweep (FL_FUSED), P@V on the i8 matrix core per block (FL_I8PV) and per
// tensor (FL_PT | FL_I8PV), the fold as packed fmas (QMHA_FOLD_PK), 12-wave workgroups (QMHA_INT8_W64).
enum { FL_MAGIC = 1, FL_LB1 = 2, FL_LB2 = 4, FL_JIT = 8, FL_LB4 = 16, FL_KFOLD = 64, FL_DUMP = 256, FL_PT = 1048576 };

// ---------------------------------------------------------------------------------------
// One-tile-at-a-time main kernel (every head size; N = 32).
//
// One workgroup = 4 waves; each wave owns one 32-row Q group (= Q quantisation group) of one
// head and sweeps all KV groups of that head.  Per 32-key tile:
//   S^T = K Q^T            v_mfma_i32_32x32x32_i8 (int32, exact), D/32 k-steps
//   online softmax         lane-local per query (swapped product), m0 = 0
//   P tile scale sP        max over the 32x32 tile (DPP + permlane16)
//   Pi = rint(p / sP)      magic-number RNE, packed to f16
//   O^T += V^T P^T         v_mfma_f32_32x32x16_f16 on exact f16 integers (= the int32 product),
//                          D/32 d-blocks, folded into the anchored O with the tile's scale
// K/V stages of 2 groups double-buffered in LDS by LDS-DMA.
// ---------------------------------------------------------------------------------------
template <int D, int FL>
__global__ __launch_bounds__(256, (FL & FL_LB1) ? 1 : ((FL & FL_LB2) ? 2 : 4)) void qmha_fa_int8_kernel(
    const float* __restrict__ Qf, const int8_t* __restrict__ Ki, const _Float16* __restrict__ Vh,
    const float* __restrict__ sK, const float* __restrict__ sV,
    float* __restrict__ O, int N, int H, int d_model, int nqb, float c_log2, QkDump dbg) {
    constexpr int WAVES = 4, SG = 2;
    constexpr int KS = D / 32;                    // i8 MFMA k-steps (QK) and d-blocks (PV)
    constexpr int KBYTES = SG * 32 * D;           // K int8 per stage
    constexpr int VBYTES = SG * 32 * D * 2;       // V f16 per stage
    constexpr int KCH = KBYTES / 16, VCH = VBYTES / 16;
    constexpr bool MAGIC = FL & FL_MAGIC;
    constexpr bool DUMP = FL & FL_DUMP;
    static_assert(D % 32 == 0 && D <= 256, "d % 32 == 0 (include/config.h:32), d <= 256 (MAGIC range)");
    static_assert(KCH % 64 == 0 && VCH % 64 == 0, "a stage is whole KiB LDS-DMA pieces");
    static_assert((KCH / SG) % 64 == 0, "a KV group is whole KiB pieces (D >= 32)");
    __shared__ __attribute__((aligned(16))) int8_t lds[2][KBYTES + VBYTES];

    const int G = N / QMHA_GROUP;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = wg / nqb, qb = wg % nqb;
    const int b = bh / H, k = bh % H;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, col = lane & 31;
    const int qg = qb * WAVES + wave;
    const bool active = qg < G;  // wave-uniform; an inactive wave still stages and syncs

    v4i qop[KS];
    float cq = 0.0f;
    if (active) {
        const float* qrow = Qf + ((size_t)b * N + (size_t)qg * QMHA_GROUP + col) * d_model + (size_t)k * D;
        const float sq = quant_q_operand<D>(qrow, half, qop);
        cq = sq * c_log2;
        if constexpr (DUMP) {  // the Q operand as held in registers: lane (col, half), k-step s
            int8_t* qd = dbg.Qi + ((size_t)bh * N + (size_t)qg * QMHA_GROUP + col) * D + 16 * half;
#pragma unroll
            for (int s = 0; s < KS; ++s) *reinterpret_cast<v4i*>(qd + 32 * s) = qop[s];
            if (lane == 0) dbg.sQ[(size_t)bh * G + qg] = sq;
        }
    } else {  // padding group: computes on a zero Q, never stored
#pragma unroll
        for (int s = 0; s < KS; ++s) qop[s] = v4i{0, 0, 0, 0};
    }
    v16f o[KS];
#pragma unroll
    for (int m = 0; m < KS; ++m) o[m] = v16f{};
    float m_run = 0.0f;   // m0 = 0 (fa_tc_int8_b.cu:402), log2 units
    float l_run = 0.0f;   // anchored: l * 2^(anchor - m)
    float anchor = 0.0f;  // o = O * 2^(m - anchor), anchor <= m

    const int8_t* kbase = Ki + (size_t)bh * N * D;
    const char* vbase = reinterpret_cast<const char*>(Vh + (size_t)bh * N * D);
    const float* skb = sK + (size_t)bh * G;
    const float* svb = sV + (size_t)bh * G;
    const int nst = (G + SG - 1) / SG;

    // K/V stage staging by LDS-DMA (global_load_lds_dwordx4): each wave-instruction writes one
    // contiguous KiB of LDS; the swizzle of the LDS image is applied to the per-lane SOURCE
    // address instead (linear destination + swizzled source + swizzled read).
    auto issue = [&](int buf, int st) {
        const int ngr = min(SG, G - st * SG);
        const int8_t* ksrc = kbase + (size_t)st * KBYTES;
        const char* vsrc = vbase + (size_t)st * VBYTES;
        int8_t* L = lds[buf];
#pragma unroll
        for (int jj = 0; jj < (KCH / 64 + WAVES - 1) / WAVES; ++jj) {
            const int inst = wave + jj * WAVES;  // KiB piece of the K stage
            if (inst < KCH / 64 && inst * 64 < ngr * (KCH / SG)) {
                const int idx = inst * 64 + lane;  // LDS chunk this lane fills
                const int row = idx / (D / 16), cc = swz_src<D>(row, idx % (D / 16));
                __builtin_amdgcn_global_load_lds((gptr_t)(ksrc + row * D + 16 * cc), (lptr_t)(L + inst * 1024), 16, 0, 0);
            }
        }
#pragma unroll
        for (int jj = 0; jj < (VCH / 64 + WAVES - 1) / WAVES; ++jj) {
            const int inst = wave + jj * WAVES;
            if (inst < VCH / 64 && inst * 64 < ngr * (VCH / SG)) {
                const int idx = inst * 64 + lane;
                const int grp = idx / (4 * D), w = idx % (4 * D);
                const int d = w >> 2, cv = swz_src<64>(d, w & 3);
                __builtin_amdgcn_global_load_lds((gptr_t)(vsrc + grp * 64 * D + d * 64 + 16 * cv),
                                                 (lptr_t)(L + KBYTES + inst * 1024), 16, 0, 0);
            }
        }
    };

    v16i magic_blk;
#pragma unroll
    for (int r = 0; r < 16; ++r) magic_blk[r] = MAGIC ? 0x4B400000 : 0;
    if constexpr (MAGIC) asm volatile("" : "+v"(magic_blk));  // resident, not rematerialised per tile

    // S^T = K Q^T of tile gi of the stage in LDS
    auto qk = [&](const int8_t* L, int gi) {
        const int krow = gi * 32 + col;
        v16i s = magic_blk;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const v4i kop = *reinterpret_cast<const v4i*>(L + krow * D + 16 * swz_pos<D>(krow, 2 * ks + half));
            s = __builtin_amdgcn_mfma_i32_32x32x32_i8(kop, qop[ks], s, 0, 0, 0);
        }
        return s;
    };

    // one tile: online softmax (fa_tc_int8_b.cu:281-346), P quantisation (:359), P@V (:366-371)
    auto tile = [&](const int8_t* L, int gi, int t, const v16i& s) {
        if constexpr (DUMP) {  // S^T of tile t as the softmax below reads it (32x32 accumulator map)
            if (active) {
                int32_t* sd = dbg.S + ((size_t)bh * N + (size_t)qg * QMHA_GROUP + col) * N + (size_t)t * QMHA_GROUP;
#pragma unroll
                for (int r = 0; r < 16; ++r) sd[acc_row(r, half)] = MAGIC ? s[r] - 0x4B400000 : s[r];
            }
        }
        const float skt = skb[t], svt = svb[t];
        float p[16];
        v8h pop[2];
        const float c = cq * skt;  // sQ*sK*log2(e)/sqrt(d) >= 0
        const int mxi = half_swap_max_i(tree_max16_i(s));
        const float mx = MAGIC ? __int_as_float(mxi) - QMHA_MAGIC_RNE : (float)mxi;
        const float m_new = fmaxf(m_run, mx * c);
        // tile max of p = exp(row max - m), then the max over the 32 query rows (:359)
        const float pmax = half_max32_nonneg(__builtin_amdgcn_exp2f(fmaf(mx, c, -m_new)));
        const float sp = fmaxf(div127_fast(pmax), 1e-8f);  // sP = max(absmax/127, 1e-8)
        const float invp = rcp_fast(sp);                   // 1/sP
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float sv = MAGIC ? __int_as_float(s[r]) - QMHA_MAGIC_RNE : (float)s[r];
            p[r] = __builtin_amdgcn_exp2f(fmaf(sv, c, -m_new));
        }
        // Pi = rint(p/sP) as exact f16 integers (0..127)
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const float q0 = fmaf(p[r], invp, QMHA_MAGIC_RNE) - QMHA_MAGIC_RNE;
            const float q1 = fmaf(p[r + 1], invp, QMHA_MAGIC_RNE) - QMHA_MAGIC_RNE;
            const v2h h2 = __builtin_convertvector((v2f{q0, q1}), v2h);
            pop[r >> 3][r & 7] = h2[0];
            pop[r >> 3][(r & 7) + 1] = h2[1];
        }
        // row sum of the unquantised p (:336) + the other lane half
        const float rs = half_swap_add(tree_sum16(p));
        // Anchored running state: o = O * 2^(m - anchor), l_run = l * 2^(m - anchor).  The
        // reference's O = alpha*O + T*sP*sV and l = alpha*l + rowsum (:336,:344,:369-371)
        // become o += T*sP*sV*2^(m_t - anchor) and l_run += rowsum*2^(m_t - anchor):
        // mathematically identical, no per-tile pass over O and no alpha.
        // re-anchor before the shift is formed, so 2^(m_new - anchor) <= 2^48 whatever the jump
        // of the running max (a first tile ~100 log2 units above m0 = 0 would overflow it)
        if (__builtin_amdgcn_ballot_w64(m_new - anchor > 48.0f)) {
            const float f = __builtin_amdgcn_exp2f(anchor - m_new);
#pragma unroll
            for (int m = 0; m < KS; ++m) o[m] *= f;
            l_run *= f;
            anchor = m_new;
        }
        const float e = __builtin_amdgcn_exp2f(m_new - anchor);
        l_run = fmaf(rs, e, l_run);
        m_run = m_new;
        const float scale = sp * svt * e;
#pragma unroll
        for (int m = 0; m < KS; ++m) {
            const int d = 32 * m + col;
            const int8_t* vr = L + KBYTES + gi * 64 * D + d * 64;
            v16f acc = v16f{};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const v8h vop = *reinterpret_cast<const v8h*>(vr + 16 * swz_pos<64>(d, 2 * ks + half));
                acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(vop, pop[ks], acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) o[m][r] = fmaf(acc[r], scale, o[m][r]);
        }
    };

    issue(0, 0);
    qmha_dma_barrier();  // waits vmcnt(0): stage 0 has landed

    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) issue(buf ^ 1, st + 1);  // buf^1 was released by the previous barrier
        if (active) {
            const int g0 = st * SG;
            const int ngr = min(SG, G - g0);  // wave-uniform
            const int8_t* L = lds[buf];
            if (ngr == SG) {
#pragma unroll
                for (int gi = 0; gi < SG; ++gi) tile(L, gi, g0 + gi, qk(L, gi));
            } else {
                for (int gi = 0; gi < ngr; ++gi) tile(L, gi, g0 + gi, qk(L, gi));
            }
        }
        qmha_dma_barrier();  // vmcnt(0) + barrier: stage st+1 landed, stage st released
    }

    // ---- epilogue (fa_tc_int8_b.cu:540-578): out = O / l, 0 if l <= 1e-20 -----------------
    if (active) {
        const float unanchor = __builtin_amdgcn_exp2f(anchor - m_run);  // 2^(anchor - m)
        const float l = l_run * unanchor;
        const bool ok = l > 1e-20f;
        float* orow = O + ((size_t)b * N + (size_t)qg * QMHA_GROUP + col) * d_model + (size_t)k * D + 4 * half;
#pragma unroll
        for (int m = 0; m < KS; ++m)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                v4f w;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) w[jj] = ok ? (o[m][4 * g4 + jj] * unanchor) / l : 0.0f;
                *reinterpret_cast<v4f*>(orow + 32 * m + 8 * g4) = w;
            }
    }
}

// ---------------------------------------------------------------------------------------
// Software-pipelined main kernel (d = 32 / 64 / 128; one Q group per wave).
//
// Iteration t runs the softmax of tile t on the VALU while the matrix core executes
// P@V of tile t-1 and Q@K^T of tile t+1 -- all three independent -- so each wave covers its
// own MFMA time with its own VALU work instead of relying on co-resident waves.  The order
// inside an iteration is pinned with sched_barrier fences (chunks of softmax VALU between
// single MFMAs); every chained MFMA pair is split by VALU work.
// K/V: stages of 2 KV groups, a 3-deep LDS ring filled by LDS-DMA two tiles ahead; one
// barrier per stage, before its odd tile (the DMA of stage s+2 is issued right after it).
// ---------------------------------------------------------------------------------------
// fa_tc_int8_pt's MFMA placement: the j-th (j < 2) MFMA issued after VALU region s (s < 6) of an
// iteration, -1 for none; op 2m + ks = P@V of d-block m, k-step ks (tile t-1), op 8 + ks = Q@K^T
// k-step ks (tile t+1).  P@V(m, 1) trails P@V(m, 0) by >= 2 slots; Q@K^T sits mid-iteration so
// the next tile's scores land before its head.
__host__ __device__ constexpr int pt_slot_op(int D, int s, int j) {
    constexpr int d32[6][2] = {{0, -1}, {-1, -1}, {1, -1}, {8, -1}, {-1, -1}, {-1, -1}};
    constexpr int d64[6][2] = {{0, -1}, {2, -1}, {1, -1}, {8, -1}, {9, -1}, {3, -1}};
    constexpr int d128[6][2] = {{0, 2}, {4, 6}, {1, 3}, {8, 9}, {10, 11}, {5, 7}};
    return D == 32 ? d32[s][j] : D == 64 ? d64[s][j] : d128[s][j];
}

template <int N>
__device__ __forceinline__ void pin_regs(float (&v)[N], int lo, int hi) {
#pragma unroll
    for (int i = 0; i < N; ++i)
        if (i >= lo && i < hi) asm volatile("" : "+v"(v[i]));
}

template <int D, int WAVES, int FL>
__global__ __launch_bounds__(WAVES * 64, (FL & FL_LB2) ? 2 : ((FL & FL_LB4) ? 4 : 3)) void qmha_fa_int8_pipe_kernel(
    const float* __restrict__ Qf, const int8_t* __restrict__ Ki, const _Float16* __restrict__ Vh,
    const float* __restrict__ sK, const float* __restrict__ sV,
    float* __restrict__ O, int N, int H, int d_model, int nqb, float c_log2, QkDump dbg,
    const float* __restrict__ sQt = nullptr, int fair = 0) {
    constexpr int SG = 2, RING = 3, PF = RING - 1;  // PF: stages in flight ahead
    constexpr int KBYTES = SG * 32 * D;      // K int8 per stage
    constexpr int VBYTES = SG * 32 * D * 2;  // V f16 per stage
    constexpr int SBYTES = KBYTES + VBYTES;
    constexpr int KCH = KBYTES / 16, VCH = VBYTES / 16;
    constexpr bool MAGIC = FL & FL_MAGIC;
    __shared__ __attribute__((aligned(16))) int8_t lds[RING][SBYTES];

    const int G = N / QMHA_GROUP;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = wg / nqb, qb = wg % nqb;
    const int b = bh / H, k = bh % H;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int half = lane >> 5, col = lane & 31;
    const int qg = qb * WAVES + wave;
    const bool active = qg < G;  // wave-uniform; an inactive wave still stages and syncs

    v4i qop[D / 32];
    float cq = 0.0f;
    constexpr bool DUMP = FL & FL_DUMP;
    // FL_PT (fa_tc_int8_pt, per-tensor mode): sQt / sK / sV hold one scale per head slice, P is
    // quantised with the static scale 1/127, so every tile's P@V is in the same unit and
    // accumulates straight into O (the MFMA C operand); O is rescaled by alpha when a row's
    // running max moves (ballot-skipped otherwise) -- no P-tile max, no per-tile O fold
    constexpr bool PT = FL & FL_PT;
    if (active) {
        const float* qrow = Qf + ((size_t)b * N + (size_t)qg * QMHA_GROUP + col) * d_model + (size_t)k * D;
        const float sq = quant_q_operand<D>(qrow, half, qop, PT ? sQt[bh] : 0.0f);
        cq = sq * c_log2;
        if constexpr (DUMP) {  // the Q operand as held in registers: lane (col, half), k-step s
            int8_t* qd = dbg.Qi + ((size_t)bh * N + (size_t)qg * QMHA_GROUP + col) * D + 16 * half;
#pragma unroll
            for (int s = 0; s < D / 32; ++s) *reinterpret_cast<v4i*>(qd + 32 * s) = qop[s];
            if (lane == 0) dbg.sQ[(size_t)bh * G + qg] = sq;
        }
    } else {
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) qop[ks] = v4i{0, 0, 0, 0};
    }
    const int8_t* kbase = Ki + (size_t)bh * N * D;
    const char* vbase = reinterpret_cast<const char*>(Vh) + (size_t)bh * N * D * 2;
    const int sstride = PT ? 1 : G;  // PT: one scale per head slice
    const float* skb = sK + (size_t)bh * sstride;
    const float* svb = sV + (size_t)bh * sstride;
    const int nst = (G + SG - 1) / SG;

    // K / V stages arrive by buffer_load ... lds: the per-lane source offsets are fixed, the
    // stage offset rides in soffset, so a stage costs no address arithmetic on the VALU
    constexpr int KJ = (KCH / 64 + WAVES - 1) / WAVES, VJ = (VCH / 64 + WAVES - 1) / WAVES;
    // with at least one wave per piece of a stage, the V pieces go to the waves after the K pieces' (wave vw)
    constexpr bool SPREAD = WAVES >= KCH / 64 + VCH / 64;
    const int vw = SPREAD ? (wave + WAVES - KCH / 64) % WAVES : wave;
    int koff[KJ], voff[VJ];
#pragma unroll
    for (int jj = 0; jj < KJ; ++jj) {
        const int idx = (wave + jj * WAVES) * 64 + lane;
        const int row = idx / (D / 16), cc = swz_src<D>(row, idx % (D / 16));
        koff[jj] = row * D + 16 * cc;
    }
#pragma unroll
    for (int jj = 0; jj < VJ; ++jj) {
        const int idx = (vw + jj * WAVES) * 64 + lane;
        const int grp = idx / (4 * D), w = idx % (4 * D);
        const int d = w >> 2, cv = swz_src<64>(d, w & 3);
        voff[jj] = grp * 64 * D + d * 64 + 16 * cv;
    }
    // stage st into ring slot `slot` (= st % RING; a compile-time constant in the unrolled loop)
    auto issue_at = [&](int st, int slot) {
        const int ngr = min(SG, G - st * SG);
        int8_t* L = lds[slot];
#pragma unroll
        for (int jj = 0; jj < KJ; ++jj) {
            const int inst = wave + jj * WAVES;
            if (inst < KCH / 64 && inst * 64 < ngr * (KCH / SG))
                buffer_load_lds16(kbase, N * D, (lptr_t)(L + inst * 1024), koff[jj], st * KBYTES);
        }
#pragma unroll
        for (int jj = 0; jj < VJ; ++jj) {
            const int inst = vw + jj * WAVES;
            if (inst < VCH / 64 && inst * 64 < ngr * (VCH / SG))
                buffer_load_lds16(vbase, N * D * 2, (lptr_t)(L + KBYTES + inst * 1024), voff[jj], st * VBYTES);
        }
    };
    auto issue = [&](int st) { issue_at(st, st % RING); };
    // operand reads of the tile in ring slot `slot`, position `par` (0/1) of its stage
    auto kop_at = [&](int slot, int par, int ks) {
        const int8_t* L = lds[slot];
        const int krow = par * 32 + col;
        return *reinterpret_cast<const v4i*>(L + krow * D + 16 * swz_pos<D>(krow, 2 * ks + half));
    };
    auto vop_at = [&](int slot, int par, int m, int ks) {
        const int8_t* L = lds[slot];
        const int d = 32 * m + col;
        return *reinterpret_cast<const v8h*>(L + KBYTES + par * 64 * D + d * 64 + 16 * swz_pos<64>(d, 2 * ks + half));
    };
    auto kop_of = [&](int t, int ks) { return kop_at((t >> 1) % RING, t & 1, ks); };
    auto vop_of = [&](int t, int m, int ks) { return vop_at((t >> 1) % RING, t & 1, m, ks); };

    v16i magic_blk;
#pragma unroll
    for (int r = 0; r < 16; ++r) magic_blk[r] = MAGIC ? 0x4B400000 : 0;
    if constexpr (MAGIC) asm volatile("" : "+v"(magic_blk));

    // ---- MFMA schedule of one iteration, per head size.  An iteration issues the P@V MFMAs of
    // tile t-1 (PV(m, ks): d-block m < MB, 16-key half ks) and the Q@K^T chain of tile t+1
    // (QK(ks), ks < KS) between the six VALU chunks A..F of tile t's softmax; kSlot[c] MFMAs
    // follow chunk c, in kOps order.  Every chained pair (same accumulator) is split by VALU.
    constexpr int MB = D / 32;  // 32-wide d-blocks of O^T (PV accumulators)
    constexpr int KS = D / 32;  // 32-deep k-steps of the i8 Q@K^T
    constexpr int NOPS = 2 * MB + KS;
    constexpr int kSlot64[6] = {1, 1, 1, 1, 1, 1};
    constexpr int kOps64[6] = {0, 2, 1, 1000, 3, 1001};  // PV00 PV10 PV01 QK0 PV11 QK1
    constexpr int kSlot32[6] = {1, 0, 1, 1, 0, 0};
    constexpr int kOps32[3] = {0, 1, 1000};  // PV00 PV01 QK0
    constexpr int kSlot128[6] = {2, 2, 2, 2, 2, 2};
    // d = 128: A PV00 PV10 | B PV20 QK0 | C PV30 PV01 | D QK1 PV11 | E PV21 QK2 | F PV31 QK3 -- every
    // chained pair (PV(m,0) -> PV(m,1), QK(k) -> QK(k+1)) is separated by a VALU chunk and another MFMA
    constexpr int kOps128[12] = {0, 2, 4, 1000, 6, 1, 1001, 3, 5, 1002, 7, 1003};
    auto slot_n = [&](int c) { return D == 32 ? kSlot32[c] : (D == 64 ? kSlot64[c] : kSlot128[c]); };
    auto op_at = [&](int i) { return D == 32 ? kOps32[i] : (D == 64 ? kOps64[i] : kOps128[i]); };
    static_assert(D == 32 || D == 64 || D == 128, "pipelined kernel: d in {32, 64, 128}");
    static_assert(NOPS == (D == 32 ? 3 : (D == 64 ? 6 : 12)), "MFMA schedule table");

    v16f o[MB];                  // O^T, d-block m (anchored)
#pragma unroll
    for (int m = 0; m < MB; ++m) o[m] = v16f{};
    float m_run = 0.0f;          // m0 = 0 (fa_tc_int8_b.cu:402), log2 units
    float l_run = 0.0f;          // l * 2^(anchor - m) over this lane's half of the keys
    float anchor = 0.0f;
    v16i s_cur, s_nxt;           // S^T of tiles t and t+1
    auto qk = [&](const v4i& kk, int ks) {
        s_nxt = __builtin_amdgcn_mfma_i32_32x32x32_i8(kk, qop[ks], ks == 0 ? magic_blk : s_nxt, 0, 0, 0);
    };
    v8h pc[2], pp[2];            // P^T operand halves (16 keys each) of tiles t (current) and t-1 (pending)
    float scale_prev = 0.0f;
    v16f a[MB];                  // P@V accumulators of the pending tile
    constexpr bool JIT = FL & FL_JIT;  // operands read right before their MFMA (fewer live VGPRs)
    // FL_KFOLD (with FL_MAGIC): the exponent of key j is fma(A_j, c', -Kn) straight from the
    // biased accumulator A_j = 1.5*2^23 + S_j (as a float), with Kn = 1.5*2^23*c' + m.  c' is the
    // score scale rounded to 22 significant bits, so 1.5*2^23*c' is exact and the shift the
    // exponents actually get, m_eff = Kn - 1.5*2^23*c', is exact too (Sterbenz: |m| < 2^20 c').
    // So p'_j = 2^(s_j - m_eff) = p_j * 2^(m_eff - m) with |m_eff - m| <= ulp(Kn)/2 (~1e-4): the
    // per-row factor f = 2^(m_eff - m) (= 1 + (m_eff - m) ln 2 to < 1 ulp) is folded into the
    // row's 1/sP and its row-sum scale, because the P tile's one scale sP is shared by rows with
    // different f.  Saves the 16 bias subtractions per tile for 4 per-row operations.
    constexpr bool KFOLD = MAGIC && (FL & FL_KFOLD);
    static_assert(KFOLD, "the pipelined kernel ships with FL_MAGIC | FL_KFOLD");
    // per-tile head results: score scale c', running max m, Kn, row factor f, sP (with the 2^24 of
    // the f16-subnormal P entries), 1/sP (with f); PT: 127 f and the sum cap / f (carried across tiles)
    float h_c = 0.0f, h_m = 0.0f, h_k = 0.0f, h_f = 1.0f, h_sp = 0.0f, h_invp = 0.0f, h_cap = 0.0f;
    // PT: the score scale sQ * sK * log2(e) / sqrt(d) is one constant per head (KFOLD-rounded once)
    const float c_pt = PT ? __int_as_float((__float_as_int(cq * skb[0]) + 2) & ~3) : 0.0f;
    auto head = [&](const v16i& s, int t) {
        float c = PT ? c_pt : cq * skb[t];
        const int mxi = half_swap_max_i(tree_max16_i(s));
        if constexpr (!PT) c = __int_as_float((__float_as_int(c) + 2) & ~3);
        const float sfmax = __int_as_float(mxi) - QMHA_MAGIC_RNE;  // exact float(S_max)
        const float xm = sfmax * c;
        h_m = fmaxf(m_run, xm);
        h_k = fmaf(c, QMHA_MAGIC_RNE, h_m);
        const float delta = fmaf(c, -QMHA_MAGIC_RNE, h_k) - h_m;  // m_eff - m, exact
        h_f = fmaf(delta, 0.69314718055994531f, 1.0f);
        const float xmax = fmaf(sfmax, c, -h_m);
        h_c = c;
        const float pmax = half_max32_nonneg(__builtin_amdgcn_exp2f(xmax));
        // sP = max(pmax / 127, 1e-8) as pm / 127 with pm = max(pmax, 127e-8), and 1/sP by one
        // v_rcp: within ~2 ulp of the reference's rounded 1/sP, which moves a Pi only when p/sP
        // lies that close to a .5 boundary (the same class as exp2 vs expf).  h_sp carries the
        // 2^24 of the f16-subnormal P entries (Pi * 2^-24)
        const float sp = fmaxf(pmax, 1.27e-6f) * (1.0f / 127.0f);
        h_invp = __builtin_amdgcn_rcpf(sp);
        h_invp *= h_f;
        h_sp = sp * 16777216.0f;
    };

    // PT lazy base (r06): the base's constants -- Kn, the KFOLD row factor f, 127 f
    // (Pi = rint(p' 127 f), static P scale) -- change only when the base does, so they are carried across
    // tiles; the row max is computed on tile 0 (base = max(m0 = 0, row max), the exact rule) and on the
    // tiles whose key halves sum above kPtSumCap only
    auto pt_base = [&](float mb) {
        h_m = mb;
        h_k = fmaf(c_pt, QMHA_MAGIC_RNE, mb);
        const float delta = fmaf(c_pt, -QMHA_MAGIC_RNE, h_k) - mb;  // m_eff - m, exact
        h_f = fmaf(delta, 0.69314718055994531f, 1.0f);
        h_invp = 127.0f * h_f;
        h_cap = kPtSumCap / h_f;  // the cap on sum(p') = sum(p) / f
    };
    auto pt_rowmax = [&](const v16i& s) {  // RN(S_max * c), log2 units
        return (__int_as_float(half_swap_max_i(tree_max16_i(s))) - QMHA_MAGIC_RNE) * c_pt;
    };
    if constexpr (PT) pt_base(0.0f);
    issue(0);
    if (nst > 1) issue(1);
    qmha_dma_barrier();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qk(kop_of(0, ks), ks);
    s_cur = s_nxt;

#define QMHA_FENCE() __builtin_amdgcn_sched_barrier(0)
    // one pipeline iteration; HP / HN (compile time): a tile t-1 to finish / a tile t+1 to start.
    // PH (compile time): -1, or u with t = 6j + 1 + u, which fixes every ring slot and stage
    // position this iteration touches (the ring has 3 slots of 2 tiles: period 6), so operand
    // reads are LDS immediates and the per-tile slot arithmetic disappears
    auto iter = [&](int t, auto HP, auto HN, auto PH) {
        constexpr bool has_prev = decltype(HP)::value, has_next = decltype(HN)::value;
        constexpr int ph = decltype(PH)::value;
        const int odd = ph >= 0 ? ((1 + ph) & 1) : (t & 1);
        const int slot_p = ph >= 0 ? ((ph >> 1) % RING) : (((t - 1) >> 1) % RING);
        const int par_p = ph >= 0 ? (ph & 1) : ((t - 1) & 1);
        const int slot_nx = ph >= 0 ? (((2 + ph) >> 1) % RING) : (((t + 1) >> 1) % RING);
        const int par_n = ph >= 0 ? (ph & 1) : ((t + 1) & 1);
        auto vop = [&](int m, int ks) { return vop_at(slot_p, par_p, m, ks); };  // tile t-1
        auto kop = [&](int ks) { return kop_at(slot_nx, par_n, ks); };           // tile t+1
        const int dma_st = (t >> 1) + PF;
        const int dma_slot = ph >= 0 ? ((((1 + ph) >> 1) + PF) % RING) : (((t >> 1) + PF) % RING);
        if (odd) {  // uniform
            qmha_dma_barrier();  // stage (t+1)/2 landed; the stage (t-3)/2 slot is free
            if (dma_st < nst) issue_at(dma_st, dma_slot);
        }
        if constexpr (DUMP) {  // S^T of tile t as the softmax below reads it (32x32 accumulator map)
            if (active) {
                int32_t* sd = dbg.S + ((size_t)bh * N + (size_t)qg * QMHA_GROUP + col) * N + (size_t)t * QMHA_GROUP;
#pragma unroll
                for (int r = 0; r < 16; ++r) sd[acc_row(r, half)] = s_cur[r] - 0x4B400000;
            }
        }
        // operand reads for this iteration's MFMAs (JIT: right before each MFMA instead)
        v8h vv[MB][2];
        v4i kk[KS];
        if constexpr (has_prev && !JIT) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int m = 0; m < MB; ++m) vv[m][ks] = vop(m, ks);
        }
        if constexpr (has_next && !JIT) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) kk[ks] = kop(ks);
        }
        QMHA_FENCE();
        // the MFMAs that follow VALU chunk c (compile-time after unrolling)
        int op_i = 0;
        auto mfmas = [&](int c) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (j < slot_n(c)) {
                    const int op = op_at(op_i++);
                    if (op >= 1000) {
                        const int ks = op - 1000;
                        if (has_next) qk(JIT ? kop(ks) : kk[ks], ks);
                    } else {
                        const int m = op >> 1, ks = op & 1;
                        if (has_prev)
                            a[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(JIT ? vop(m, ks) : vv[m][ks], pp[ks],
                                                                          ks == 0 ? v16f{} : a[m], 0, 0, 0);
                    }
                }
            }
        };
        // ---- A: row max, running max, P-tile max (fa_tc_int8_b.cu:286-303, :359)
        head(s_cur, t);
        QMHA_FENCE();
        const float c = h_c, m_new = h_m, kn = h_k;
        // re-anchor (rare) before this tile's shift 2^(m_new - anchor) is formed, so it stays <= 2^48
        // however far the running max jumps (a first tile ~100 log2 units above m0 = 0 would
        // overflow it); the pending tile t-1 carries its factor in scale_prev
        if (__builtin_amdgcn_ballot_w64(m_new - anchor > 48.0f)) {
            const float f = __builtin_amdgcn_exp2f(anchor - m_new);
#pragma unroll
            for (int m = 0; m < MB; ++m) o[m] *= f;
            l_run *= f;
            scale_prev *= f;
            anchor = m_new;
        }
        mfmas(0);
        QMHA_FENCE();
        // ---- B: P scale, scores of rows 0..7
        const float sp = h_sp, invp = h_invp;
        const float e = __builtin_amdgcn_exp2f(m_new - anchor);
        float x[16];
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = fmaf(__int_as_float(s_cur[r]), c, -kn);
        QMHA_FENCE();
        mfmas(1);
        QMHA_FENCE();
        // ---- C: scores of rows 8..15
#pragma unroll
        for (int r = 8; r < 16; ++r) x[r] = fmaf(__int_as_float(s_cur[r]), c, -kn);
        QMHA_FENCE();
        mfmas(2);
        QMHA_FENCE();
        // ---- D: p = exp2, rows 0..7
        float p[16];
#pragma unroll
        for (int r = 0; r < 8; ++r) p[r] = __builtin_amdgcn_exp2f(x[r]);
        QMHA_FENCE();
        mfmas(3);
        QMHA_FENCE();
        // ---- E: p = exp2, rows 8..15
#pragma unroll
        for (int r = 8; r < 16; ++r) p[r] = __builtin_amdgcn_exp2f(x[r]);
        QMHA_FENCE();
        mfmas(4);
        QMHA_FENCE();
        // ---- F: Pi = rint(p/sP) (:317-321), carried as the f16 subnormal Pi * 2^-24:
        // fma(p, 1/sP, 1.5 * 2^23) rounds half-even to an integer whose float bits end in Pi,
        // and those low 16 bits are exactly the f16 encoding of Pi * 2^-24; one byte permute
        // packs two entries.  P@V then yields T * 2^-24 exactly (T < 2^20); the O scale
        // carries the 2^24 back.
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float t0 = fmaf(p[2 * r], invp, QMHA_MAGIC_RNE), t1 = fmaf(p[2 * r + 1], invp, QMHA_MAGIC_RNE);
            const v2h h2 = __builtin_bit_cast(v2h, __builtin_amdgcn_perm(__float_as_uint(t1), __float_as_uint(t0), 0x05040100u));
            pc[r >> 2][2 * (r & 3)] = h2[0];
            pc[r >> 2][2 * (r & 3) + 1] = h2[1];
        }
        QMHA_FENCE();
        mfmas(5);
        QMHA_FENCE();
        // ---- G: row sum (unquantised p, :336), anchored l, this tile's O scale
        // this lane's 16 keys only: the two halves of l are joined once, in the epilogue
        const float rs = tree_sum16(p);
        l_run = fmaf(rs, e * h_f, l_run);
        m_run = m_new;
        // sp carries 2^24 (P entries are Pi * 2^-24)
        const float scale_t = sp * svb[t] * e;
        // ---- H: fold the pending tile's P@V into O (o += T * sP * sV * 2^(m - anchor))
        if constexpr (has_prev) {
#pragma unroll
            for (int m = 0; m < MB; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r) o[m][r] = fmaf(a[m][r], scale_prev, o[m][r]);
        }
        QMHA_FENCE();
        // rotate the pipeline
        pp[0] = pc[0];
        pp[1] = pc[1];
        scale_prev = scale_t;
        if constexpr (has_next) s_cur = s_nxt;
    };
    // ---- FL_PT: the per-tensor iteration as explicit sched_barrier regions (the generic body above
    // keeps its live ranges for the per-block fold and spills in this mode).  Six regions R0..R5 of
    // VALU work; after region s the MFMAs of pt_slot_op(D, s, .) issue (transcendental /
    // quarter-rate work first in each region, full-rate work after it); operands are read from LDS
    // in the region before their slot's predecessor (two slots ahead).  P@V accumulates straight
    // into O; O takes tile t-1's alpha at the start of iteration t (before P@V of t-1 lands, after
    // P@V of t-2 has), so no MFMA result is waited on.
    float alpha_prev = 1.0f;  // the alpha of the tile whose P@V this iteration adds
    bool rescale_prev = false;  // wave-uniform: that tile rebased some row (alpha_prev != 1 somewhere)
    auto iter_pt = [&](int t, auto HP, auto HN, auto PH) {
        constexpr bool has_prev = decltype(HP)::value, has_next = decltype(HN)::value;
        constexpr int ph = decltype(PH)::value;
        const int odd = ph >= 0 ? ((1 + ph) & 1) : (t & 1);
        const int slot_p = ph >= 0 ? ((ph >> 1) % RING) : (((t - 1) >> 1) % RING);
        const int par_p = ph >= 0 ? (ph & 1) : ((t - 1) & 1);
        const int slot_nx = ph >= 0 ? (((2 + ph) >> 1) % RING) : (((t + 1) >> 1) % RING);
        const int par_n = ph >= 0 ? (ph & 1) : ((t + 1) & 1);
        const int dma_st = (t >> 1) + PF;
        const int dma_slot = ph >= 0 ? ((((1 + ph) >> 1) + PF) % RING) : (((t >> 1) + PF) % RING);
        if (odd) {  // uniform
            qmha_dma_barrier();  // stage (t+1)/2 landed; the stage (t-3)/2 slot is free
            if (dma_st < nst) issue_at(dma_st, dma_slot);
        }
        if constexpr (DUMP) {  // S^T of tile t as the softmax below reads it (32x32 accumulator map)
            if (active) {
                int32_t* sd = dbg.S + ((size_t)bh * N + (size_t)qg * QMHA_GROUP + col) * N + (size_t)t * QMHA_GROUP;
#pragma unroll
                for (int r = 0; r < 16; ++r) sd[acc_row(r, half)] = s_cur[r] - 0x4B400000;
            }
        }
        v8h vv[MB][2];
        v4i kk[KS];
        auto rd_slot = [&](int s) {  // operands of slot s's MFMAs
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int op = pt_slot_op(D, s, j);
                if (op >= 0 && op < 8) {
                    if constexpr (has_prev)
                        if ((op >> 1) < MB) vv[(op >> 1) % MB][op & 1] = vop_at(slot_p, par_p, op >> 1, op & 1);
                } else if (op >= 8) {
                    if constexpr (has_next)
                        if (op - 8 < KS) kk[(op - 8) % KS] = kop_at(slot_nx, par_n, op - 8);
                }
            }
        };
        auto mf_slot = [&](int s) {  // slot s's MFMAs
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int op = pt_slot_op(D, s, j);
                if (op >= 0 && op < 8) {
                    if constexpr (has_prev) {
                        const int m = (op >> 1) % MB;
                        if ((op >> 1) < MB) o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vv[m][op & 1], pp[op & 1], o[m], 0, 0, 0);
                    }
                } else if (op >= 8) {
                    if constexpr (has_next)
                        if (op - 8 < KS) qk(kk[(op - 8) % KS], op - 8);
                }
            }
        };
        float x[16], p[16], q[16];
        auto exps = [&](int r0, int r1) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (r >= r0 && r < r1) p[r] = __builtin_amdgcn_exp2f(x[r]);
        };
        auto quant = [&](int r0, int r1) {
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if (r >= r0 && r < r1) q[r] = fmaf(p[r], h_invp, QMHA_MAGIC_RNE);
        };
        auto perms = [&](int j0, int j1) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j >= j0 && j < j1) {
                    const v2h h2 = __builtin_bit_cast(v2h, __builtin_amdgcn_perm(__float_as_uint(q[2 * j + 1]),
                                                                               __float_as_uint(q[2 * j]), 0x05040100u));
                    pc[j >> 2][2 * (j & 3)] = h2[0];
                    pc[j >> 2][2 * (j & 3) + 1] = h2[1];
                }
            asm volatile("" : "+v"(pc[0]), "+v"(pc[1]));  // no IR-level sinking past this region
        };
        rd_slot(0);
        rd_slot(1);
        QMHA_FENCE();
        // ---- R0: tile 0 sets the base (max(m0, row max)); then O *= alpha of tile t-1
        if constexpr (!has_prev) {
            pt_base(fmaxf(m_run, pt_rowmax(s_cur)));
            m_run = h_m;
        }
        const float c = c_pt, kn = h_k;
        QMHA_FENCE();
        if constexpr (has_prev) {
            if (rescale_prev) {
#pragma unroll
                for (int m = 0; m < MB; ++m) o[m] *= alpha_prev;
            }
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = fmaf(__int_as_float(s_cur[r]), c, -kn);
        pin_regs(x, 0, 8);
        QMHA_FENCE();
        mf_slot(0);
        QMHA_FENCE();
        // ---- R1
        exps(0, 4);
        QMHA_FENCE();
        rd_slot(2);
#pragma unroll
        for (int r = 8; r < 16; ++r) x[r] = fmaf(__int_as_float(s_cur[r]), c, -kn);
        pin_regs(x, 8, 16);
        quant(0, 4);
        float rs0 = (p[0] + p[1]) + (p[2] + p[3]);
        asm volatile("" : "+v"(rs0));
        QMHA_FENCE();
        mf_slot(1);
        QMHA_FENCE();
        // ---- R2
        exps(4, 8);
        perms(0, 2);
        QMHA_FENCE();
        rd_slot(3);
        quant(4, 8);
        float rs1 = (p[4] + p[5]) + (p[6] + p[7]);
        asm volatile("" : "+v"(rs1));
        QMHA_FENCE();
        mf_slot(2);
        QMHA_FENCE();
        // ---- R3
        exps(8, 12);
        perms(2, 4);
        QMHA_FENCE();
        rd_slot(4);
        quant(8, 12);
        float rs2 = (p[8] + p[9]) + (p[10] + p[11]);
        asm volatile("" : "+v"(rs2));
        QMHA_FENCE();
        mf_slot(3);
        QMHA_FENCE();
        // ---- R4
        exps(12, 16);
        perms(4, 6);
        QMHA_FENCE();
        rd_slot(5);
        quant(12, 16);
        float rs3 = (p[12] + p[13]) + (p[14] + p[15]);
        asm volatile("" : "+v"(rs3));
        QMHA_FENCE();
        mf_slot(4);
        QMHA_FENCE();
        // ---- R5
        perms(6, 8);
        QMHA_FENCE();
        float ts = (rs0 + rs1) + (rs2 + rs3);  // this lane's key half: sum(p') (sum(p) = sum(p') f)
        float alpha_t = 1.0f;
        bool rescale_t = false;
        if constexpr (has_prev) {  // (tile 0 set its base to the row max: p <= 1)
            const uint64_t over = __builtin_amdgcn_ballot_w64(ts > h_cap);
            if (over) {  // rare (wave-uniform): rebase the rows with a half above the cap, redo the tile's P
                rescale_t = true;
                const float xm = pt_rowmax(s_cur);
                const uint32_t rows = (uint32_t)over | (uint32_t)(over >> 32);
                const float mb = ((rows >> col) & 1u) ? xm : m_run;
                alpha_t = __builtin_amdgcn_exp2f(m_run - mb);
                l_run *= alpha_t;
                pt_base(mb);
                m_run = mb;
#pragma unroll
                for (int r = 0; r < 16; ++r) x[r] = fmaf(__int_as_float(s_cur[r]), c_pt, -h_k);
                exps(0, 16);
                quant(0, 16);
                perms(0, 8);
                ts = tree_sum16(p);
            }
        }
        l_run = fmaf(ts, h_f, l_run);  // l = alpha l + sum(p)
        QMHA_FENCE();
        mf_slot(5);
        QMHA_FENCE();
        pp[0] = pc[0];
        pp[1] = pc[1];
        alpha_prev = alpha_t;
        rescale_prev = rescale_t;
        if constexpr (has_next) s_cur = s_nxt;
    };
    auto run_iter = [&](int t, auto HP, auto HN, auto PH) {
        if constexpr (PT)
            iter_pt(t, HP, HN, PH);
        else
            iter(t, HP, HN, PH);
    };
    using T1 = std::integral_constant<bool, true>;
    using F0 = std::integral_constant<bool, false>;
    // G >= 2 (the per-block launcher routes N < 64 elsewhere): first, interior, last tile; G == 1
    // (the per-tensor mode at N = 32): one tile, its P@V in the drain
    using DYN = std::integral_constant<int, -1>;
    if (PT && G == 1) {
        if constexpr (PT) run_iter(0, F0{}, F0{}, DYN{});
    } else {
        // fair != 0 (grids of at most 8 rounds of workgroups, the launcher's choice): a workgroup's
        // waves lower their issue priority quarter by quarter of their sweep (3 .. 0), so the
        // workgroups sharing a SIMD -- which the age-ordered arbiter otherwise finishes one after the
        // other, the last ones running alone at a fraction of the SIMD's throughput -- advance together
        // (one C4 sequence per call -3.3 %, the reference's shape -3.7 %)
        auto set_prio = [&](int tt) {
            const int q = (4 * tt) / G;  // wave-uniform
            if (q <= 0)
                __builtin_amdgcn_s_setprio(3);
            else if (q == 1)
                __builtin_amdgcn_s_setprio(2);
            else if (q == 2)
                __builtin_amdgcn_s_setprio(1);
            else
                __builtin_amdgcn_s_setprio(0);
        };
        if (fair) set_prio(0);
        run_iter(0, F0{}, T1{}, DYN{});
        int t = 1;
        constexpr int PER = 2 * RING;  // ring period in tiles
        for (; t + PER <= G - 1; t += PER) {
            if (fair) set_prio(t);
            run_iter(t, T1{}, T1{}, std::integral_constant<int, 0>{});
            run_iter(t + 1, T1{}, T1{}, std::integral_constant<int, 1>{});
            run_iter(t + 2, T1{}, T1{}, std::integral_constant<int, 2>{});
            run_iter(t + 3, T1{}, T1{}, std::integral_constant<int, 3>{});
            run_iter(t + 4, T1{}, T1{}, std::integral_constant<int, 4>{});
            run_iter(t + 5, T1{}, T1{}, std::integral_constant<int, 5>{});
        }
        for (; t < G - 1; ++t) run_iter(t, T1{}, T1{}, DYN{});
        run_iter(G - 1, T1{}, F0{}, DYN{});
    }
#undef QMHA_FENCE
    // drain: P@V of the last tile
    {
        const int t = G - 1;
        if constexpr (PT) {
            if (rescale_prev) {  // O still owes the last tile's alpha
#pragma unroll
                for (int m = 0; m < MB; ++m) o[m] *= alpha_prev;
            }
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int m = 0; m < MB; ++m)
                    o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vop_of(t, m, ks), pp[ks], o[m], 0, 0, 0);
        } else {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int m = 0; m < MB; ++m)
                    a[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vop_of(t, m, ks), pp[ks], ks == 0 ? v16f{} : a[m], 0, 0, 0);
#pragma unroll
            for (int m = 0; m < MB; ++m) o[m] += a[m] * scale_prev;
        }
    }
    // ---- epilogue (fa_tc_int8_b.cu:540-578): out = O / l, 0 if l <= 1e-20
    // lane (col, half) holds O^T rows d = 32 m + 8 g4 + 4 half + jj of query col
    if (active) {
        // PT: O is in units of 2^-24 (the f16-subnormal P entries) times sV / 127: 2^24 * sV / 127
        // rescales it exactly to the oracle's O * (sV / 127)
        const float unanchor = PT ? 16777216.0f * (svb[0] / 127.0f) : __builtin_amdgcn_exp2f(anchor - m_run);
        const float l = PT ? half_swap_add(l_run) : half_swap_add(l_run) * unanchor;
        const bool ok = l > 1e-20f;
        float* orow = O + ((size_t)b * N + (size_t)qg * QMHA_GROUP + col) * d_model + (size_t)k * D + 4 * half;
#pragma unroll
        for (int m = 0; m < MB; ++m)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
                v4f w;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) w[jj] = ok ? (o[m][4 * g4 + jj] * unanchor) / l : 0.0f;
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
// Production layout: Ki [B*H][N][D], Vh (f16 V^T operand blocks, 2 bytes per element), sK, sV
// [B*H][N/32] (the main kernel quantises Q in registers).  with_q adds Qi and sQ at the end for the
// int32 Q@K^T test hook, whose pre-pass quantises Q too.
size_t int8_workspace_bytes(int B, int N, int H, int D, bool with_q) {
    const size_t e = align_up((size_t)B * H * N * D, 256);
    const size_t s = align_up((size_t)B * H * (N / QMHA_GROUP) * sizeof(float), 256);
    return e + 2 * e + 2 * s + (with_q ? e + s : 0);
}

Int8Workspace int8_carve(void* ws, int B, int N, int H, int D, bool with_q) {
    Int8Workspace w{};
    const size_t e = align_up((size_t)B * H * N * D, 256);
    const size_t s = align_up((size_t)B * H * (N / QMHA_GROUP) * sizeof(float), 256);
    char* p = static_cast<char*>(ws);
    w.Ki = reinterpret_cast<int8_t*>(p);
    w.Vh = reinterpret_cast<_Float16*>(p + e);
    w.sK = reinterpret_cast<float*>(p + 3 * e);
    w.sV = reinterpret_cast<float*>(p + 3 * e + s);
    w.Qi = with_q ? reinterpret_cast<int8_t*>(p + 3 * e + 2 * s) : nullptr;
    w.sQ = with_q ? reinterpret_cast<float*>(p + 4 * e + 2 * s) : nullptr;
    return w;
}

template <int D, int FL>
static hipError_t fa_int8_launch(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int d_model,
                                 hipStream_t stream, QkDump dbg = QkDump{}) {
    const int G = N / QMHA_GROUP;
    const int nqb = (G + 3) / 4;
    const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2e;  // inv_sqrt_d: fa_tc_int8_b.cu:587
    hipLaunchKernelGGL((qmha_fa_int8_kernel<D, FL>), dim3(B * H * nqb), dim3(256), 0, stream, Qf, w.Ki, w.Vh, w.sK, w.sV,
                       O, N, H, d_model, nqb, c_log2, dbg);
    return hipGetLastError();
}

// Rounds of workgroups a grid of `nwg` takes on this device at the kernel's occupancy (HIP's own
// occupancy answer, cached per kernel instance and device); 0 if unknown.
template <int D, int WAVES, int FL>
static long long pipe_slots() {
    static std::atomic<long long> slots_of[64];  // resident workgroups per device (one word: no torn pair)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    long long slots = slots_of[dev].load(std::memory_order_relaxed);
    if (slots <= 0) {
        int n = 0, c = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, qmha_fa_int8_pipe_kernel<D, WAVES, FL>, WAVES * 64, 0) != hipSuccess ||
            hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0 || c <= 0)
            return 0;
        slots = (long long)n * c;
        slots_of[dev].store(slots, std::memory_order_relaxed);
    }
    return slots;
}
template <int D, int WAVES, int FL>
static int pipe_rounds(long long nwg) {
    const long long slots = pipe_slots<D, WAVES, FL>();
    return slots > 0 ? (int)((nwg + slots - 1) / slots) : 0;
}
// issue-priority fairness (the kernel's `fair`) for grids of at most this many rounds: measured
// -3.3 % (one round), -3.7 % (two), -2.4 % (eight, d = 32), and not adopted at C4's 10.7 rounds
// (profiles/r04/ab_fair/)
constexpr int kFairMaxRounds = 8;

template <int D, int WAVES, int FL>
static hipError_t fa_int8_pipe_launch(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H,
                                      int d_model, hipStream_t stream, QkDump dbg = QkDump{}) {
    const int G = N / QMHA_GROUP;
    if (G < 2) return fa_int8_launch<D, 0>(w, Qf, O, B, N, H, d_model, stream);  // no pipeline to fill
    const int nqb = (G + WAVES - 1) / WAVES;
    const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2e;
    const int rounds = pipe_rounds<D, WAVES, FL>((long long)B * H * nqb);
    const int fair = rounds > 0 && rounds <= kFairMaxRounds;
    hipLaunchKernelGGL((qmha_fa_int8_pipe_kernel<D, WAVES, FL>), dim3(B * H * nqb), dim3(WAVES * 64), 0, stream, Qf,
                       w.Ki, w.Vh, w.sK, w.sV, O, N, H, d_model, nqb, c_log2, dbg, (const float*)nullptr, fair);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Per-tensor mode on 16x16 MFMAs (shipped at d = 64): the fp16 v3 kernel's tile
// (qmha_fa_f16.hip) with the per-tensor contract of the pipe kernel's iter_pt: Q@K^T on
// v_mfma_i32_16x16x64_i8 from the magic-biased accumulator (KFOLD exponent), P quantised with the static
// scale into f16-subnormal pairs, P@V on v_mfma_f32_16x16x32_f16 straight into O, the lazy base per query
// triggered by a lane's key quarter.  Same K rows in the kap16 key order as the fp16 v3 kernel, the V^T
// slot order unchanged.  No software pipeline: four waves per SIMD interleave instead.
// ---------------------------------------------------------------------------------------
__host__ __device__ constexpr int kap16_i8(int kb, int m) { return 16 * (m >> 3) + 4 * ((m >> 2) & 1) + (m & 3) + 8 * kb; }

template <int D, int WAVES, int SG, bool DUMP>
__global__ __launch_bounds__(WAVES * 64, D > 64 ? 2 : 4) void qmha_fa_int8_pt_v3_kernel(
    const float* __restrict__ Qf, const int8_t* __restrict__ Ki, const _Float16* __restrict__ Vh,
    const float* __restrict__ sQt, const float* __restrict__ sK, const float* __restrict__ sV, float* __restrict__ O,
    int N, int H, int d_model, int nqb, float c_log2, QkDump dbg) {
    constexpr int KS = D / 64;            // QK k-steps (K = 64)
    constexpr int DB = D / 16;            // PV d-blocks of 16 rows
    constexpr int RB = D;                 // K row bytes (int8)
    constexpr int KBYTES = SG * 32 * RB;  // K per stage
    constexpr int VBYTES = SG * 32 * D * 2;
    constexpr int KCH = KBYTES / 16, VCH = VBYTES / 16;
    static_assert(KCH % 64 == 0 && VCH % 64 == 0 && (KCH / SG) % 64 == 0, "whole KiB LDS-DMA pieces");
    __shared__ __attribute__((aligned(16))) char lds[2][KBYTES + VBYTES];

    const int G = N / QMHA_GROUP;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = wg / nqb, qb0 = wg % nqb;
    const int b = bh / H, k = bh % H;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int qg = qb0 * WAVES + wave;
    const bool active = qg < G;
    const int grp = lane >> 4, r16 = lane & 15;

    // Q quantised with the slice scale into the QK B operand: query 16 qb + r16, d = 64 ks + 16 grp .. +15
    const float sq = sQt[bh];
    const float inv_q = 1.0f / sq;
    v4i qop[2][KS];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (active) {
                const float* qp = Qf + ((size_t)b * N + (size_t)qg * QMHA_GROUP + 16 * qb + r16) * d_model + (size_t)k * D +
                                  64 * ks + 16 * grp;
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4) {
                    const v4f x = *reinterpret_cast<const v4f*>(qp + 4 * c4);
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) w |= ((uint32_t)(uint8_t)qmha_quant_i8(nan_to_zero(x[e]), inv_q)) << (8 * e);
                    qop[qb][ks][c4] = (int)w;
                }
            } else {
                qop[qb][ks] = v4i{0, 0, 0, 0};
            }
        }
    if constexpr (DUMP) {  // the Q operand as held in registers (FL_DUMP twin: qmha_debug_fa_int8_pt_dump)
        if (active) {
#pragma unroll
            for (int qb = 0; qb < 2; ++qb)
#pragma unroll
                for (int ks = 0; ks < KS; ++ks)
                    *reinterpret_cast<v4i*>(dbg.Qi + ((size_t)bh * N + (size_t)qg * QMHA_GROUP + 16 * qb + r16) * D + 64 * ks +
                                            16 * grp) = qop[qb][ks];
            if (lane == 0) dbg.sQ[(size_t)bh * G + qg] = sq;
        }
    }
    // the score constant sQ * sK * log2(e) / sqrt(d), KFOLD-rounded to 22 bits (as the pipe kernel)
    const float c_pt = __int_as_float((__float_as_int((sq * c_log2) * sK[bh]) + 2) & ~3);
    const v4i magic4 = {0x4B400000, 0x4B400000, 0x4B400000, 0x4B400000};
    v4f o[DB][2];
#pragma unroll
    for (int m = 0; m < DB; ++m) o[m][0] = o[m][1] = v4f{};
    // per query (qb): base m, Kn, the KFOLD row factor f, 127 f, cap / f; l over this lane's keys
    float m_run[2] = {0.0f, 0.0f}, l_run[2] = {0.0f, 0.0f};
    float h_k[2], h_f[2], h_invp[2], h_cap[2];
    auto pt_base = [&](int qb, float mb) {
        m_run[qb] = mb;
        h_k[qb] = fmaf(c_pt, QMHA_MAGIC_RNE, mb);
        const float delta = fmaf(c_pt, -QMHA_MAGIC_RNE, h_k[qb]) - mb;  // m_eff - m, exact
        h_f[qb] = fmaf(delta, 0.69314718055994531f, 1.0f);
        h_invp[qb] = 127.0f * h_f[qb];
        h_cap[qb] = kPtSumCap / h_f[qb];
    };
    pt_base(0, 0.0f);
    pt_base(1, 0.0f);

    const char* kbase = reinterpret_cast<const char*>(Ki + (size_t)bh * N * D);
    const char* vbase = reinterpret_cast<const char*>(Vh + (size_t)bh * N * D);
    const int nst = (G + SG - 1) / SG;
    constexpr int KJ = (KCH / 64 + WAVES - 1) / WAVES, VJ = (VCH / 64 + WAVES - 1) / WAVES;
    int koff[KJ], voff[VJ];
#pragma unroll
    for (int jj = 0; jj < KJ; ++jj) {
        const int idx = (wave + jj * WAVES) * 64 + lane;
        const int row = idx / (RB / 16), cc = (idx % (RB / 16)) ^ kswz16<RB>(row);
        koff[jj] = row * RB + 16 * cc;
    }
#pragma unroll
    for (int jj = 0; jj < VJ; ++jj) {
        const int idx = (wave + jj * WAVES) * 64 + lane;
        const int gq = idx / (4 * D), w = idx % (4 * D);
        const int d = w >> 2, cv = (w & 3) ^ vswz16(d);
        voff[jj] = gq * 64 * D + d * 64 + 16 * cv;
    }
    auto issue = [&](int buf, int st) {
        const int ngr = min(SG, G - st * SG);
        char* L = lds[buf];
#pragma unroll
        for (int jj = 0; jj < KJ; ++jj) {
            const int inst = wave + jj * WAVES;
            if (inst < KCH / 64 && inst * 64 < ngr * (KCH / SG))
                buffer_load_lds16(kbase, N * RB, (lptr_t)(L + inst * 1024), koff[jj], st * KBYTES);
        }
#pragma unroll
        for (int jj = 0; jj < VJ; ++jj) {
            const int inst = wave + jj * WAVES;
            if (inst < VCH / 64 && inst * 64 < ngr * (VCH / SG))
                buffer_load_lds16(vbase, N * D * 2, (lptr_t)(L + KBYTES + inst * 1024), voff[jj], st * VBYTES);
        }
    };
    struct S4 {
        v4i v[2][2];  // [kb][qb]: magic-biased int32 S^T, rows kap16_i8(kb, 4 grp + i), query 16 qb + r16
    };
    auto qk = [&](const char* L, int gi) {
        S4 s;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const int krow = gi * 32 + kap16_i8(kb, r16);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const v4i kop = *reinterpret_cast<const v4i*>(L + krow * RB + 16 * ((4 * ks + grp) ^ kswz16<RB>(krow)));
#pragma unroll
                for (int qb = 0; qb < 2; ++qb)
                    s.v[kb][qb] = __builtin_amdgcn_mfma_i32_16x16x64_i8(kop, qop[qb][ks], ks == 0 ? magic4 : s.v[kb][qb], 0, 0, 0);
            }
        }
        return s;
    };
    auto rowmax_xm = [&](const S4& s, int qb) {  // RN(S_max * c) of the query's 32 keys (4 lanes x 8)
        int mx = max(max(max(s.v[0][qb][0], s.v[0][qb][1]), max(s.v[0][qb][2], s.v[0][qb][3])),
                     max(max(s.v[1][qb][0], s.v[1][qb][1]), max(s.v[1][qb][2], s.v[1][qb][3])));
        mx = max(mx, __shfl_xor(mx, 16));
        mx = max(mx, __shfl_xor(mx, 32));
        return (__int_as_float(mx) - QMHA_MAGIC_RNE) * c_pt;
    };
    auto tile = [&](const char* L, int gi, const S4& s, bool first, int t) {
        if constexpr (DUMP) {  // S^T of tile t as the softmax below reads it (bias removed)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                int32_t* sd = dbg.S + ((size_t)bh * N + (size_t)qg * QMHA_GROUP + 16 * qb + r16) * N + (size_t)t * QMHA_GROUP;
#pragma unroll
                for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                    for (int i = 0; i < 4; ++i) sd[kap16_i8(kb, 4 * grp + i)] = s.v[kb][qb][i] - 0x4B400000;
            }
        }
        v8h vop[DB];  // V^T rows 16 m + r16, slots 8 grp .. +7
#pragma unroll
        for (int m = 0; m < DB; ++m) {
            const int d = 16 * m + r16;
            vop[m] = *reinterpret_cast<const v8h*>(L + KBYTES + gi * 64 * D + d * 64 + 16 * (grp ^ vswz16(d)));
        }
        if (first) {  // tile 0 sets the base: max(m0 = 0, row max), the exact rule
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) pt_base(qb, fmaxf(m_run[qb], rowmax_xm(s, qb)));
        }
        float p[2][8], q[2][8], ts[2];
        auto softmax_p = [&](int qb) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                p[qb][j] = __builtin_amdgcn_exp2f(fmaf(__int_as_float(s.v[j >> 2][qb][j & 3]), c_pt, -h_k[qb]));
                q[qb][j] = fmaf(p[qb][j], h_invp[qb], QMHA_MAGIC_RNE);  // Pi = rint(127 p) in the low bits
            }
            const float a0 = p[qb][0] + p[qb][1], a1 = p[qb][2] + p[qb][3], a2 = p[qb][4] + p[qb][5], a3 = p[qb][6] + p[qb][7];
            ts[qb] = (a0 + a1) + (a2 + a3);
        };
        softmax_p(0);
        softmax_p(1);
        if (!first) {
            const uint64_t over0 = __builtin_amdgcn_ballot_w64(ts[0] > h_cap[0]);
            const uint64_t over1 = __builtin_amdgcn_ballot_w64(ts[1] > h_cap[1]);
            if (over0 | over1) {  // rare (wave-uniform): rebase the queries with a key quarter above the cap
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) {
                    const uint64_t over = qb ? over1 : over0;
                    const float xm = rowmax_xm(s, qb);
                    const uint32_t q16 = (uint32_t)(over | (over >> 32));
                    const uint32_t rows = (q16 | (q16 >> 16)) & 0xffffu;
                    const float mb = ((rows >> r16) & 1u) ? xm : m_run[qb];
                    const float alpha = __builtin_amdgcn_exp2f(m_run[qb] - mb);
                    l_run[qb] *= alpha;
#pragma unroll
                    for (int m = 0; m < DB; ++m) o[m][qb] *= alpha;
                    pt_base(qb, mb);
                    softmax_p(qb);
                }
            }
        }
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            l_run[qb] = fmaf(ts[qb], h_f[qb], l_run[qb]);  // l = alpha l + sum(p)
            v4i pw;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                pw[i] = (int)__builtin_amdgcn_perm(__float_as_uint(q[qb][2 * i + 1]), __float_as_uint(q[qb][2 * i]), 0x05040100u);
            const v8h pop = __builtin_bit_cast(v8h, pw);
#pragma unroll
            for (int m = 0; m < DB; ++m) o[m][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vop[m], pop, o[m][qb], 0, 0, 0);
        }
    };

    issue(0, 0);
    qmha_dma_barrier();
    int t = 0;
    auto stage = [&](auto BUF, int st) {
        constexpr int buf = decltype(BUF)::value;
        if (st + 1 < nst) issue(buf ^ 1, st + 1);
        if (active) {
            const char* L = lds[buf];
            const int ngr = G - st * SG;  // < SG only in a partial last stage (uniform)
#pragma unroll
            for (int gi = 0; gi < SG; ++gi) {
                if (gi == 0 || gi < ngr) tile(L, gi, qk(L, gi), t == 0, st * SG + gi);
                ++t;
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        qmha_dma_barrier();
    };
    int st = 0;
    for (; st + 2 <= nst; st += 2) {
        stage(std::integral_constant<int, 0>{}, st);
        stage(std::integral_constant<int, 1>{}, st + 1);
    }
    if (st < nst) stage(std::integral_constant<int, 0>{}, st);
    if (active) {
        // O is in units of 2^-24 (the f16-subnormal P entries) times sV / 127
        const float unanchor = 16777216.0f * (sV[bh] / 127.0f);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            float l = l_run[qb];
            l += __shfl_xor(l, 16);
            l += __shfl_xor(l, 32);
            const bool ok = l > 1e-20f;
            float* orow = O + ((size_t)b * N + (size_t)qg * QMHA_GROUP + 16 * qb + r16) * d_model + (size_t)k * D + 4 * grp;
#pragma unroll
            for (int m = 0; m < DB; ++m) {
                v4f w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = ok ? (o[m][qb][j] * unanchor) / l : 0.0f;
                *reinterpret_cast<v4f*>(orow + 16 * m) = w;
            }
        }
    }
}

// ---- per-tensor mode (fa_tc_int8_pt) -----------------------------------------------------
size_t int8_pt_workspace_bytes(int B, int N, int H, int D) {
    const size_t e = align_up((size_t)B * H * N * D, 256);
    const size_t g = align_up((size_t)6 * B * H * sizeof(uint32_t), 256);  // slice_sync [2][3][B*H]
    const size_t s = align_up((size_t)B * H * sizeof(float), 256);
    return e + 2 * e + g + 3 * s;
}

Int8Workspace int8_pt_carve(void* ws, int B, int N, int H, int D) {
    const size_t e = align_up((size_t)B * H * N * D, 256);
    const size_t g = align_up((size_t)6 * B * H * sizeof(uint32_t), 256);  // slice_sync [2][3][B*H]
    const size_t s = align_up((size_t)B * H * sizeof(float), 256);
    char* p = static_cast<char*>(ws);
    Int8Workspace w{};
    w.Ki = reinterpret_cast<int8_t*>(p);
    w.Vh = reinterpret_cast<_Float16*>(p + e);
    w.slice_sync = reinterpret_cast<uint32_t*>(p + 3 * e);
    w.sQ = reinterpret_cast<float*>(p + 3 * e + g);
    w.sK = reinterpret_cast<float*>(p + 3 * e + g + s);
    w.sV = reinterpret_cast<float*>(p + 3 * e + g + 2 * s);
    return w;
}

template <int D, int FL, int WAVES = 4>
static hipError_t fa_int8_pt_launch(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int d_model,
                                    hipStream_t stream, QkDump dbg = QkDump{}) {
    const int G = N / QMHA_GROUP;
    const int nqb = (G + WAVES - 1) / WAVES;
    const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2e;
    const int rounds = pipe_rounds<D, WAVES, FL | FL_PT>((long long)B * H * nqb);
    const int fair = rounds > 0 && rounds <= kFairMaxRounds;
    hipLaunchKernelGGL((qmha_fa_int8_pipe_kernel<D, WAVES, FL | FL_PT>), dim3(B * H * nqb), dim3(WAVES * 64), 0, stream,
                       Qf, w.Ki, w.Vh, w.sK, w.sV, O, N, H, d_model, nqb, c_log2, dbg, (const float*)w.sQ, fair);
    return hipGetLastError();
}

// Pipelined-kernel flags per head size.  d = 128: 4 d-blocks of O and of P@V accumulators -> 2
// waves per SIMD, operands read at their MFMA.  Per-tensor mode at d = 32: a 4-wave register
// budget (128 VGPRs; 131 otherwise, i.e. 3 waves/SIMD).  Other head sizes: the one-tile kernel
// with the magic-biased accumulator at a 2-wave budget, 1 wave above d = 128 (O alone is d/2 VGPRs
// per lane; at 2 waves d = 160 / 192 spill 176 / 372 bytes per lane to scratch).
constexpr int kD64Flags = FL_MAGIC | FL_KFOLD, kD32Flags = FL_MAGIC | FL_KFOLD;
constexpr int kD128Flags = FL_MAGIC | FL_KFOLD | FL_JIT | FL_LB2, kPtD32Extra = FL_LB4;
template <int D>
constexpr int kAnyFlags = FL_MAGIC | (D > 128 ? FL_LB1 : FL_LB2);

template <int D, int XFL = 0>
static hipError_t fa_int8_d(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int d_model,
                            hipStream_t stream, QkDump dbg = QkDump{}) {
    if constexpr (D == 32) return fa_int8_pipe_launch<D, 4, kD32Flags | XFL>(w, Qf, O, B, N, H, d_model, stream, dbg);
    else if constexpr (D == 64) return fa_int8_pipe_launch<D, 4, kD64Flags | XFL>(w, Qf, O, B, N, H, d_model, stream, dbg);
    else if constexpr (D == 128) return fa_int8_pipe_launch<D, 4, kD128Flags | XFL>(w, Qf, O, B, N, H, d_model, stream, dbg);
    else return fa_int8_launch<D, kAnyFlags<D> | XFL>(w, Qf, O, B, N, H, d_model, stream, dbg);
}

// compute units of the current device (cached per device); 0 if unknown
static long long device_cus() {
    static std::atomic<int> cus_of[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
    int c = cus_of[dev].load(std::memory_order_relaxed);
    if (c <= 0) {
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) return 0;
        cus_of[dev].store(c, std::memory_order_relaxed);
    }
    return c;
}

template <int D, int WAVES, bool DUMP = false>
static hipError_t fa_int8_pt_v3_launch(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int d_model,
                                       hipStream_t stream, QkDump dbg = QkDump{}) {
    const int G = N / QMHA_GROUP;
    const int nqb = (G + WAVES - 1) / WAVES;
    const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2e;
    hipLaunchKernelGGL((qmha_fa_int8_pt_v3_kernel<D, WAVES, 2, DUMP>), dim3(B * H * nqb), dim3(WAVES * 64), 0, stream, Qf,
                       w.Ki, w.Vh, w.sQ, w.sK, w.sV, O, N, H, d_model, nqb, c_log2, dbg);
    return hipGetLastError();
}

hipError_t launch_fa_int8_pt_main(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int D,
                                  int d_model, hipStream_t stream) {
    switch (D) {
        case 32: return fa_int8_pt_launch<32, kD32Flags | kPtD32Extra>(w, Qf, O, B, N, H, d_model, stream);
        // d = 64: the 16x16 kernel (v3), same box, alternating: C4 -4.4 %, B = 2 -6.7 %, but B = 1 +7.2 %
        // (256 workgroups = 2 waves per SIMD, which the unpipelined tile cannot hide latency with).  At
        // d = 128 it measured +1.6 % (193 VGPRs, 2 waves per SIMD), so the scheduled pipe kernel keeps
        // d = 32 / 128 (profiles/r06/ab_pt_mma16/)
        case 64: {
            // 8-wave workgroups; grids of at most one such workgroup per CU (2 waves per SIMD, e.g. one
            // sequence of H16 N4096) run 4-wave ones instead, whose two workgroups per CU do not share a
            // barrier phase: same box, alternating, B1 N4096 H16 -2.0 %, B1 N8192 H8 -2.6 %, but B2 +6 %
            // and C4 +2.6 % (profiles/r06/ab_pt_mma16/w4/).  WAVES changes no value: bit-identical.
            const long long wgs8 = (long long)B * H * ((N / QMHA_GROUP + 7) / 8), cus = device_cus();
            if (cus > 0 && wgs8 <= cus) return fa_int8_pt_v3_launch<64, 4>(w, Qf, O, B, N, H, d_model, stream);
            return fa_int8_pt_v3_launch<64, 8>(w, Qf, O, B, N, H, d_model, stream);
        }
        case 128: return fa_int8_pt_launch<128, kD128Flags>(w, Qf, O, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

#define QMHA_INT8_D_CASES(X) X(32) X(64) X(96) X(128) X(160) X(192) X(224) X(256)

hipError_t launch_fa_int8_main(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int D,
                               int d_model, hipStream_t stream) {
    switch (D) {
#define QMHA_CASE(d) \
    case d: return fa_int8_d<d>(w, Qf, O, B, N, H, d_model, stream);
        QMHA_INT8_D_CASES(QMHA_CASE)
#undef QMHA_CASE
        default: return hipErrorInvalidValue;
    }
}

// The production int8 schedule with FL_DUMP: same kernel template, same flags plus the stores
// of what it computed (S^T per tile, Q operand, sQ), at every head size.
hipError_t launch_fa_int8_dump(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int D,
                               int d_model, QkDump dbg, hipStream_t stream) {
    if ((D == 32 || D == 64 || D == 128) && N / QMHA_GROUP < 2) return hipErrorInvalidValue;  // pipelined: N >= 64
    switch (D) {
#define QMHA_CASE(d) \
    case d: return fa_int8_d<d, FL_DUMP>(w, Qf, O, B, N, H, d_model, stream, dbg);
        QMHA_INT8_D_CASES(QMHA_CASE)
#undef QMHA_CASE
        default: return hipErrorInvalidValue;
    }
}

// The per-tensor mode's production schedule with FL_DUMP (same flags and workgroup size as
// launch_fa_int8_pt_main, plus the stores)
hipError_t launch_fa_int8_pt_dump(const Int8Workspace& w, const float* Qf, float* O, int B, int N, int H, int D,
                                  int d_model, QkDump dbg, hipStream_t stream) {
    switch (D) {
        case 32: return fa_int8_pt_launch<32, kD32Flags | kPtD32Extra | FL_DUMP>(w, Qf, O, B, N, H, d_model, stream, dbg);
        case 64: return fa_int8_pt_v3_launch<64, 8, true>(w, Qf, O, B, N, H, d_model, stream, dbg);
        case 128: return fa_int8_pt_launch<128, kD128Flags | FL_DUMP>(w, Qf, O, B, N, H, d_model, stream, dbg);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_debug_qk_int32(const Int8Workspace& w, int N, int D, int bh, int32_t* S, hipStream_t stream) {
    const int G = N / QMHA_GROUP;
    switch (D) {
#define QMHA_CASE(d)                                                                                                    \
    case d:                                                                                                             \
        hipLaunchKernelGGL((qmha_debug_qk_int32_kernel<d>), dim3(G, G), dim3(64), 0, stream, w.Qi, w.Ki, N, bh, S); \
        break;
        QMHA_INT8_D_CASES(QMHA_CASE)
#undef QMHA_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace qmha
