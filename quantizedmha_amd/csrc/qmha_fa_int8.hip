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
//   1. qmha_quant_int8_kernel: reads fp32 Q/K/V once; writes int8 Q and K rows per head and
//      the quantised V integers in the MFMA V^T operand order, one fp32 scale per group.
//      Bit-identical to the reference quantiser (same fp32 ops, RNE rounding).
//   2. qmha_fa_int8_kernel: one workgroup = WAVES waves = WAVES*32 query rows of one head;
//      each wave owns exactly one 32-row Q group (= one Q quantisation group).  K/V tiles
//      stream HBM -> registers -> LDS (double buffered, XOR-swizzled, conflict-free
//      ds_read_b128).  Both products use swapped operands (S^T = K Q^T, O^T = V^T P^T) so
//      every query's statistics are lane-local and P^T feeds the second MFMA from registers.
//        Q@K^T: v_mfma_i32_32x32x32_i8, exact int32 scores.
//        P@V  : the int8-valued operands Pi in [0,127], Vi in [-128,127] run on
//               v_mfma_f32_32x32x16_f16.  Both are exact in f16, every product and every
//               partial sum (|sum| <= 32*127*128 < 2^24) is exact in the fp32 accumulator,
//               so the result equals the reference's int32 (Pi Vi) bit for bit -- but it
//               arrives as fp32, saving the 32 int->float conversions per lane per tile
//               that dominate an int32 epilogue (VALU is this kernel's bound).
//      Software pipelining: the Q@K^T MFMAs of tile t+1 are issued before the softmax of
//      tile t, so the matrix pipe runs under the VALU work of the same wave.
#include "qmha_common.hpp"
#include "qmha_kernels.hpp"

#include <cstdlib>

namespace qmha {

// log2(e): the softmax runs in base 2 (v_exp_f32), scores pre-multiplied by log2(e).
static constexpr float kLog2e = 1.4426950408889634f;

// ---------------------------------------------------------------------------------------
// Pre-pass: quantise Q, K, V (fa_tc_int8_b.cu:33-152, fp32_to_int8sram).
// One wave per (tensor, bh, group); blockIdx.y = tensor (0 Q, 1 K, 2 V).
// v_mode 0: V as int8 in the i8 V^T operand order (qmha_quantize_int8 layout 1)
// v_mode 1: V as f16-valued integers in the f16 V^T operand order (main kernel input)
// ---------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256) void qmha_quant_int8_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
    int8_t* __restrict__ Qi, int8_t* __restrict__ Ki, void* __restrict__ Vout,
    float* __restrict__ sQ, float* __restrict__ sK, float* __restrict__ sV,
    int N, int H, int d_model, int total_groups, int v_mode) {
    constexpr int C4 = D / 4;        // float4 per row
    constexpr int RPI = 64 / C4;     // rows per load instruction
    constexpr int NI = 32 / RPI;     // load instructions per lane
    __shared__ __attribute__((aligned(16))) _Float16 vtile[4][32 * D];

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
    } else if (v_mode == 0) {
        // int8 [D][32] with the i8 operand slot permutation, transposed through LDS
        int8_t* tile = reinterpret_cast<int8_t*>(vtile[wave]);
        if (active) {
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int slot = slot_of_kv_i8(i * RPI + ri);
#pragma unroll
                for (int c = 0; c < 4; ++c) tile[(4 * ci + c) * 32 + slot] = (int8_t)qmha_quant_i8(v[i][c], inv);
            }
        }
        __syncthreads();
        if (active) {
            int8_t* dst = static_cast<int8_t*>(Vout) + ((size_t)bh * G + g) * (size_t)(32 * D);
            constexpr int CH = 32 * D / 16;
#pragma unroll
            for (int c = lane; c < CH; c += 64)
                reinterpret_cast<v4i*>(dst)[c] = reinterpret_cast<const v4i*>(tile)[c];
            if (lane == 0) sV[item] = sc;
        }
    } else {
        // f16-valued integers [D][32] with the f16 operand slot permutation
        _Float16* tile = vtile[wave];
        if (active) {
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int slot = slot_of_kv_f16(i * RPI + ri);
#pragma unroll
                for (int c = 0; c < 4; ++c) tile[(4 * ci + c) * 32 + slot] = (_Float16)qmha_quant_i8(v[i][c], inv);
            }
        }
        __syncthreads();
        if (active) {
            _Float16* dst = static_cast<_Float16*>(Vout) + ((size_t)bh * G + g) * (size_t)(32 * D);
            constexpr int CH = 32 * D * 2 / 16;
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
// ABL: ablation bitmask for profiling builds only (0 in production; results are wrong
// otherwise): 1 = no exp2 on P, 2 = no P@V MFMA, 4 = no Q@K^T MFMA, 8 = no P-tile max
// reduction, 16 = no compute at all (K/V staging and barriers only), 64 = no K/V staging and
// no barriers (every stage recomputes on LDS buffer 0), 32 = phase-separated softmax,
// 128 = magic-offset Q@K^T accumulator + packed score/sum arithmetic + anchored l,
// 256 = no Q@K^T prefetch across tiles, 512 = 2 waves/SIMD register budget.
template <int D, int WAVES, int SG, int ABL = 0>
// 2nd launch bound = minimum waves per SIMD: 4 caps the allocation at 128 VGPRs, so four
// waves share each SIMD (the VALU-bound softmax needs them to fill the issue slots).
__global__ __launch_bounds__(WAVES * 64, (ABL & 512) ? 2 : 4) void qmha_fa_int8_kernel(
    const int8_t* __restrict__ Qi, const int8_t* __restrict__ Ki, const _Float16* __restrict__ Vh,
    const float* __restrict__ sQ, const float* __restrict__ sK, const float* __restrict__ sV,
    float* __restrict__ O, int N, int H, int d_model, int nqb, float c_log2) {
    constexpr int KS = D / 32;                    // i8 MFMA k-steps (QK) and d-blocks (PV)
    constexpr int KBYTES = SG * 32 * D;           // K int8 per stage
    constexpr int VBYTES = SG * 32 * D * 2;       // V f16 per stage
    constexpr int NT = WAVES * 64;
    constexpr int KCH = KBYTES / 16, VCH = VBYTES / 16;
    static_assert(KCH % 64 == 0 && VCH % 64 == 0, "a stage is whole KiB LDS-DMA pieces");
    static_assert((KCH / SG) % 64 == 0, "a KV group is whole KiB pieces (D >= 32)");
    __shared__ __attribute__((aligned(16))) int8_t lds[2][KBYTES + VBYTES];

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
    float anchor = 0.0f;  // o = O * 2^(m_run - anchor), anchor <= m_run

    const int8_t* kbase = Ki + (size_t)bh * N * D;
    const char* vbase = reinterpret_cast<const char*>(Vh + (size_t)bh * N * D);
    const float* skb = sK + (size_t)bh * G;
    const float* svb = sV + (size_t)bh * G;
    const int nst = (G + SG - 1) / SG;

    // K/V stage staging by LDS-DMA (global_load_lds_dwordx4): each wave-instruction writes one
    // contiguous KiB of LDS; the XOR swizzle of the LDS image is applied to the per-lane
    // SOURCE address instead (linear destination + swizzled source + swizzled read).
    auto issue = [&](int buf, int st) {
        const int ngr = min(SG, G - st * SG);
        const int8_t* ksrc = kbase + (size_t)st * KBYTES;
        const char* vsrc = vbase + (size_t)st * VBYTES;
        int8_t* L = lds[buf];
#pragma unroll
        for (int j = 0; j < (KCH / 64 + WAVES - 1) / WAVES; ++j) {
            const int inst = wave + j * WAVES;  // KiB piece of the K stage
            if (inst < KCH / 64 && inst * 64 < ngr * (KCH / SG)) {
                const int idx = inst * 64 + lane;              // LDS chunk this lane fills
                const int row = idx / (D / 16), cc = (idx % (D / 16)) ^ chunk_swz<D>(row);
                __builtin_amdgcn_global_load_lds((gptr_t)(ksrc + row * D + 16 * cc), (lptr_t)(L + inst * 1024), 16, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < (VCH / 64 + WAVES - 1) / WAVES; ++j) {
            const int inst = wave + j * WAVES;
            if (inst < VCH / 64 && inst * 64 < ngr * (VCH / SG)) {
                const int idx = inst * 64 + lane;
                const int grp = idx / (4 * D), w = idx % (4 * D);
                const int d = w >> 2, cv = (w & 3) ^ chunk_swz<64>(d);
                __builtin_amdgcn_global_load_lds((gptr_t)(vsrc + grp * 64 * D + d * 64 + 16 * cv),
                                                 (lptr_t)(L + KBYTES + inst * 1024), 16, 0, 0);
            }
        }
    };
    // S^T = K Q^T (int32) of tile gi of the stage in LDS
    // ABL&128: the Q@K^T chain starts from the bit pattern of 1.5*2^23, so each int32 lane of
    // the result reads as the float 1.5*2^23 + S (exact: |S| <= 2^21) -- one packed subtract
    // then yields float(S) for two scores, replacing two v_cvt_f32_i32.
    v16i magic_blk;
#pragma unroll
    for (int r = 0; r < 16; ++r) magic_blk[r] = 0x4B400000;
    asm volatile("" : "+v"(magic_blk));  // keep it resident, not rematerialised per tile
    auto qk = [&](const int8_t* L, int gi) {
        v16i s = (ABL & 128) ? magic_blk : v16i{};
        const int krow = gi * 32 + col;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const v4i kop = *reinterpret_cast<const v4i*>(L + krow * D + 16 * ((2 * ks + half) ^ chunk_swz<D>(krow)));
            if constexpr (ABL & 4) {
                asm volatile("" : "+v"(s) : "v"(kop), "v"(qop[ks]));
            } else {
                s = __builtin_amdgcn_mfma_i32_32x32x32_i8(kop, qop[ks], s, 0, 0, 0);
            }
        }
        return s;
    };
    // one tile: online softmax (fa_tc_int8_b.cu:281-346), P quantisation (:359), P@V (:366-371)
    auto tile = [&](const int8_t* L, int gi, int t, const v16i& s) {
        const float c = cq * skb[t];  // sQ*sK*log2(e)/sqrt(d) > 0
        const float mx = (ABL & 128) ? __int_as_float(half_swap_max_i(tree_max16_i(s))) - QMHA_MAGIC_RNE
                                     : (float)half_swap_max_i(tree_max16_i(s));
        const float m_new = fmaxf(m_run, mx * c);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        float p[16];
        v8h pop[2];
        float sp, invp;
        // tile max of p = exp(tile row max - m), then the max over the 32 query rows
        auto pscale = [&]() {
            const float pmax = (ABL & 8) ? fmaf(mx, c, -m_new) : half_max32_nonneg(__builtin_amdgcn_exp2f(fmaf(mx, c, -m_new)));
            sp = fmaxf(div127_fast(pmax), 1e-8f);  // sP = max(absmax/127, 1e-8)
            invp = rcp_fast(sp);                   // 1/sP
        };
        if constexpr (ABL & 128) {
            pscale();
            const v2f mg = {QMHA_MAGIC_RNE, QMHA_MAGIC_RNE}, cc = {c, c}, nm = {-m_new, -m_new};
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
                v2f x = v2f{__int_as_float(s[r]), __int_as_float(s[r + 1])} - mg;  // float(S), exact
                x = __builtin_elementwise_fma(x, cc, nm);
                p[r] = __builtin_amdgcn_exp2f(x[0]);
                p[r + 1] = __builtin_amdgcn_exp2f(x[1]);
            }
        } else if constexpr (ABL & 32) {
            // phase-separated: every phase is 16 independent instructions
#pragma unroll
            for (int r = 0; r < 16; ++r) p[r] = (float)s[r];
            __builtin_amdgcn_sched_barrier(0);
            pscale();
#pragma unroll
            for (int r = 0; r < 16; ++r) p[r] = fmaf(p[r], c, -m_new);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if constexpr (!(ABL & 1)) p[r] = __builtin_amdgcn_exp2f(p[r]);
            __builtin_amdgcn_sched_barrier(0);
        } else {
            pscale();
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                p[r] = fmaf((float)s[r], c, -m_new);
                if constexpr (!(ABL & 1)) p[r] = __builtin_amdgcn_exp2f(p[r]);
            }
        }
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            // Pi = rint(p/sP) as an exact f16 integer (0..127)
            const float q0 = fmaf(p[r], invp, QMHA_MAGIC_RNE) - QMHA_MAGIC_RNE;
            const float q1 = fmaf(p[r + 1], invp, QMHA_MAGIC_RNE) - QMHA_MAGIC_RNE;
            const v2h h2 = __builtin_convertvector((v2f{q0, q1}), v2h);
            pop[r >> 3][r & 7] = h2[0];
            pop[r >> 3][(r & 7) + 1] = h2[1];
        }
        float rs;
        if constexpr (ABL & 128) {
            // pairwise tree in packed form (p[r], p[r+1] are adjacent registers)
            v2f t0 = v2f{p[0], p[1]} + v2f{p[2], p[3]}, t1 = v2f{p[4], p[5]} + v2f{p[6], p[7]};
            v2f t2 = v2f{p[8], p[9]} + v2f{p[10], p[11]}, t3 = v2f{p[12], p[13]} + v2f{p[14], p[15]};
            const v2f u = (t0 + t1) + (t2 + t3);
            rs = half_swap_add(u[0] + u[1]);
        } else {
            rs = half_swap_add(tree_sum16(p));
        }
        const float e_anchor = __builtin_amdgcn_exp2f(m_new - anchor);
        if constexpr (ABL & 128) {
            l_run = fmaf(rs, e_anchor, l_run);  // anchored l: l_run holds l * 2^(anchor - m)
        } else {
            l_run = fmaf(alpha, l_run, rs);  // :336
        }
        m_run = m_new;
        // Anchored accumulator: o holds O * 2^(m - anchor), so the reference's per-tile
        // rescale O *= alpha (:344) is folded into this tile's O scale factor
        //   O_t = alpha_t O_{t-1} + sP sV T_t   <=>   o_t = o_{t-1} + sP sV 2^(m_t - anchor) T_t
        // (mathematically identical; no per-tile pass over O and no branch in the hot loop).
        const float scale = sp * svb[t] * e_anchor;
#pragma unroll
        for (int m = 0; m < KS; ++m) {
            const int d = 32 * m + col;
            const int8_t* vr = L + KBYTES + gi * 64 * D + d * 64;
            v16f acc = {};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const v8h vop = *reinterpret_cast<const v8h*>(vr + 16 * ((2 * ks + half) ^ chunk_swz<64>(d)));
                if constexpr (ABL & 2) {
                    asm volatile("" : "+v"(acc) : "v"(vop), "v"(pop[ks]));
                } else {
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(vop, pop[ks], acc, 0, 0, 0);
                }
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) o[m][r] = fmaf(acc[r], scale, o[m][r]);
        }
    };

    issue(0, 0);
    __syncthreads();  // waits vmcnt(0): stage 0 has landed

    for (int st = 0; st < nst; ++st) {
        const int buf = (ABL & 64) ? 0 : (st & 1);
        if (!(ABL & 64) && st + 1 < nst) issue(buf ^ 1, st + 1);  // buf^1 was released by the previous barrier
        if (active && !(ABL & 16)) {
            const int g0 = st * SG;
            const int ngr = min(SG, G - g0);  // wave-uniform
            const int8_t* L = lds[buf];
            if ((ABL & 256) && ngr == SG) {
#pragma unroll
                for (int gi = 0; gi < SG; ++gi) {
                    const v16i sc = qk(L, gi);
                    tile(L, gi, g0 + gi, sc);
                }
            } else if (ngr == SG) {
                // straight-line stage: Q@K^T of tile gi+1 is issued before tile gi's softmax
                v16i s_cur = qk(L, 0);
#pragma unroll
                for (int gi = 0; gi < SG; ++gi) {
                    v16i s_nxt = {};
                    if (gi + 1 < SG) s_nxt = qk(L, gi + 1);
                    // pin the pipeline depth to one tile: without this fence the scheduler
                    // hoists every Q@K^T of the stage and the live S tiles cost occupancy
                    __builtin_amdgcn_sched_barrier(0);
                    QMHA_ISA_MARK();
                    tile(L, gi, g0 + gi, s_cur);
                    QMHA_ISA_MARK();
                    __builtin_amdgcn_sched_barrier(0);
                    s_cur = s_nxt;
                }
            } else {
                for (int gi = 0; gi < ngr; ++gi) tile(L, gi, g0 + gi, qk(L, gi));
            }
            // re-anchor (rare, once per stage): keep 2^(m - anchor) far from fp32 overflow
            if (__builtin_amdgcn_ballot_w64(m_run - anchor > 48.0f)) {
                const float f = __builtin_amdgcn_exp2f(anchor - m_run);
#pragma unroll
                for (int m = 0; m < KS; ++m)
#pragma unroll
                    for (int r = 0; r < 16; ++r) o[m][r] *= f;
                if constexpr (ABL & 128) l_run *= f;
                anchor = m_run;
            }
        }
        if constexpr (!(ABL & 64)) __syncthreads();  // vmcnt(0) + barrier: stage st+1 landed, stage st released
    }

    // ---- epilogue (fa_tc_int8_b.cu:540-578): out = O / l, 0 if l <= 1e-20 -----------------
    if (active) {
        const float unanchor = __builtin_amdgcn_exp2f(anchor - m_run);  // o * 2^(anchor - m) = O
        if constexpr (ABL & 128) l_run *= unanchor;
        const bool ok = l_run > 1e-20f;
#pragma unroll
        for (int m = 0; m < KS; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) o[m][r] *= unanchor;
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
    return 2 * align_up(e, 256) + align_up(2 * e, 256) + 3 * align_up(s, 256);
}

Int8Workspace int8_carve(void* ws, int B, int N, int H, int D) {
    Int8Workspace w;
    const size_t e = align_up((size_t)B * H * N * D, 256);
    const size_t e2 = align_up((size_t)B * H * N * D * 2, 256);
    const size_t s = align_up((size_t)B * H * (N / QMHA_GROUP) * sizeof(float), 256);
    char* p = static_cast<char*>(ws);
    w.Qi = reinterpret_cast<int8_t*>(p);
    w.Ki = reinterpret_cast<int8_t*>(p + e);
    w.Vh = reinterpret_cast<_Float16*>(p + 2 * e);
    w.sQ = reinterpret_cast<float*>(p + 2 * e + e2);
    w.sK = reinterpret_cast<float*>(p + 2 * e + e2 + s);
    w.sV = reinterpret_cast<float*>(p + 2 * e + e2 + 2 * s);
    return w;
}

template <int D>
static hipError_t quant_int8_d(const float* Q, const float* K, const float* V, const Int8Workspace& w, void* vout,
                               int v_mode, int B, int N, int H, int d_model, hipStream_t stream) {
    const int total = B * H * (N / QMHA_GROUP);
    dim3 grid((total + 3) / 4, 3);
    hipLaunchKernelGGL((qmha_quant_int8_kernel<D>), grid, dim3(256), 0, stream, Q, K, V, w.Qi, w.Ki, vout, w.sQ, w.sK,
                       w.sV, N, H, d_model, total, v_mode);
    return hipGetLastError();
}

hipError_t launch_quant_int8(const float* Q, const float* K, const float* V, const Int8Workspace& w, void* vout,
                             int v_mode, int B, int N, int H, int D, int d_model, hipStream_t stream) {
    switch (D) {
        case 32: return quant_int8_d<32>(Q, K, V, w, vout, v_mode, B, N, H, d_model, stream);
        case 64: return quant_int8_d<64>(Q, K, V, w, vout, v_mode, B, N, H, d_model, stream);
        case 128: return quant_int8_d<128>(Q, K, V, w, vout, v_mode, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

template <int D, int WAVES, int SG, int ABL = 0>
static hipError_t fa_int8_launch(const Int8Workspace& w, float* O, int B, int N, int H, int d_model,
                                 hipStream_t stream) {
    const int G = N / QMHA_GROUP;
    const int nqb = (G + WAVES - 1) / WAVES;
    const int nwg = B * H * nqb;
    const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2e;  // inv_sqrt_d: fa_tc_int8_b.cu:587
    hipLaunchKernelGGL((qmha_fa_int8_kernel<D, WAVES, SG, ABL>), dim3(nwg), dim3(WAVES * 64), 0, stream, w.Qi, w.Ki, w.Vh,
                       w.sQ, w.sK, w.sV, O, N, H, d_model, nqb, c_log2);
    return hipGetLastError();
}

template <int D>
static hipError_t fa_int8_d(const Int8Workspace& w, float* O, int B, int N, int H, int d_model, hipStream_t stream) {
    if constexpr (D == 64) {
        switch (tune_config("QMHA_INT8_CFG")) {
            case 44: return fa_int8_launch<D, 4, 4>(w, O, B, N, H, d_model, stream);
            case 82: return fa_int8_launch<D, 8, 2>(w, O, B, N, H, d_model, stream);
            default: break;
        }
#ifdef QMHA_ABLATION
        static const int abl = std::getenv("QMHA_INT8_ABL") ? std::atoi(std::getenv("QMHA_INT8_ABL")) : 0;
        switch (abl) {
            case 1: return fa_int8_launch<D, 4, 2, 1>(w, O, B, N, H, d_model, stream);
            case 2: return fa_int8_launch<D, 4, 2, 2>(w, O, B, N, H, d_model, stream);
            case 4: return fa_int8_launch<D, 4, 2, 4>(w, O, B, N, H, d_model, stream);
            case 6: return fa_int8_launch<D, 4, 2, 6>(w, O, B, N, H, d_model, stream);
            case 8: return fa_int8_launch<D, 4, 2, 8>(w, O, B, N, H, d_model, stream);
            case 9: return fa_int8_launch<D, 4, 2, 9>(w, O, B, N, H, d_model, stream);
            case 15: return fa_int8_launch<D, 4, 2, 15>(w, O, B, N, H, d_model, stream);
            case 16: return fa_int8_launch<D, 4, 2, 16>(w, O, B, N, H, d_model, stream);
            case 32: return fa_int8_launch<D, 4, 2, 32>(w, O, B, N, H, d_model, stream);
            case 64: return fa_int8_launch<D, 4, 2, 64>(w, O, B, N, H, d_model, stream);
            case 128: return fa_int8_launch<D, 4, 2, 128>(w, O, B, N, H, d_model, stream);
            case 384: return fa_int8_launch<D, 4, 2, 384>(w, O, B, N, H, d_model, stream);
            case 256: return fa_int8_launch<D, 4, 2, 256>(w, O, B, N, H, d_model, stream);
            case 512: return fa_int8_launch<D, 4, 2, 512>(w, O, B, N, H, d_model, stream);
            case 640: return fa_int8_launch<D, 4, 2, 640>(w, O, B, N, H, d_model, stream);
            case 896: return fa_int8_launch<D, 4, 2, 896>(w, O, B, N, H, d_model, stream);
            case 65: return fa_int8_launch<D, 4, 2, 65>(w, O, B, N, H, d_model, stream);
            case 70: return fa_int8_launch<D, 4, 2, 70>(w, O, B, N, H, d_model, stream);
            case 79: return fa_int8_launch<D, 4, 2, 79>(w, O, B, N, H, d_model, stream);
            default: break;
        }
#endif
    }
    return fa_int8_launch<D, 4, 2>(w, O, B, N, H, d_model, stream);
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
