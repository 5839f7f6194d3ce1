// qmha_fa_f16.hip -- fused FP16-MFMA FlashAttention-2 forward for gfx950 (MI355X).
//
// Drop-in for the reference's fa_tc_v1a (mha_kernels/fa_tc_v1a.cu:222-439):
//   Q, K, V -> __float2half (RNE);  S = Qh Kh^T with fp32 accumulation;  s = S / sqrt(d)
//   online softmax with m0 = 0 (:290): p = exp(s - m), l = alpha*l + sum(p) (fp32 p)
//   P stored as half(p) (:174);  O = alpha*O + Ph Vh (fp32 accumulate, :218)
//   out = O / l, 0 if l <= 1e-10 (:384-388)
//
// Same skeleton as the INT8 kernel: a conversion pre-pass (qmha_prepass.hip) writes K as f16 rows and V in the
// f16 V^T operand order; the main kernel converts its Q group into registers, streams K/V
// tiles through LDS-DMA-filled swizzled LDS and runs both products on
// v_mfma_f32_32x32x16_f16 with swapped operands.  The O accumulator is the MFMA C operand,
// so the P@V accumulation costs no VALU; alpha == 1 rescales are skipped exactly.
#include "qmha_common.hpp"
#include "qmha_kernels.hpp"

#include <type_traits>

namespace qmha {

static constexpr float kLog2eH = 1.4426950408889634f;
// the lazy base's cap: a row's base moves only when the p of one of its key halves sum above 2^12 on a
// tile, so every p stays <= 4096, far from the f16 maximum (65504)
static constexpr float kLazySumCap = 4096.0f;


// ---------------------------------------------------------------------------------------
// Main kernel: K/V staged by LDS-DMA (global_load_lds, swizzled source / linear LDS image),
// one 32-key tile at a time, Q@K^T of the next tile issued before the current softmax
// (FL_PREFETCH).  One wave = one 32-row Q group.
// ---------------------------------------------------------------------------------------
// F16_VPRE: the tile's V^T operands are read from LDS before its softmax, so the P@V MFMAs do
// not wait on their LDS reads
// F16_UNROLL: two stages per loop trip, so each stage's LDS buffer is a compile-time constant and
// every operand read is a base register plus an immediate (no per-tile address arithmetic)
// F16_LB1: a one-wave-per-SIMD register budget (VGPRs + AGPRs) for d > 128, whose O alone is d/2 VGPRs
// (Measured and not shipped, in git history up to commit df5dced: the K / V conversion inside the sweep,
// F16_FUSED; the per-phase s_memtime stamps, F16_STAMP.)
enum { F16_PREFETCH = 1, F16_LB4 = 4, F16_VPRE = 8, F16_UNROLL = 16, F16_LB1 = 32 };

template <int D, int WAVES, int SG, int FL>
__global__ __launch_bounds__(WAVES * 64, (FL & F16_LB4) ? 4 : ((FL & F16_LB1) ? 1 : 2)) void qmha_fa_f16_v2_kernel(
    const float* __restrict__ Qf, const _Float16* __restrict__ Kh, const _Float16* __restrict__ Vt,
    float* __restrict__ O, int N, int H, int d_model, int nqb, float c_log2) {
    QMHA_ENABLE_AGPR_MFMA();
    // the score scale lives in a VGPR: a VOP3 fma reading an SGPR issues at the slow rate
    // (~4.3 instead of ~2.5 cycles per wave64 on gfx950, profiles/r02/ubench_valu_cost.txt)
    asm volatile("" : "+v"(c_log2));
    constexpr int KS = D / 16;           // QK k-steps (K = 16)
    constexpr int MB = D / 32;           // PV d-blocks
    constexpr int RB = 2 * D;            // K row bytes
    constexpr int KBYTES = SG * 32 * RB; // K per stage
    constexpr int VBYTES = SG * 32 * D * 2;
    constexpr int KCH = KBYTES / 16, VCH = VBYTES / 16;
    static_assert(KCH % 64 == 0 && VCH % 64 == 0 && (KCH / SG) % 64 == 0, "whole KiB LDS-DMA pieces");
    __shared__ __attribute__((aligned(16))) char lds[2][KBYTES + VBYTES];

    const int G = N / QMHA_GROUP;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int bh = wg / nqb, qb = wg % nqb;
    const int b = bh / H, k = bh % H;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int qg = qb * WAVES + wave;
    const bool active = qg < G;
    const int half = lane >> 5, col = lane & 31;

    v8h qop[KS];
    if (active) {
        // Q converted in-kernel (RNE, __float2half) straight into the operand: elements
        // [16 s + 8 half, +8) of query row col (saves the pre-pass its Q traffic)
        const float* qp = Qf + ((size_t)b * N + (size_t)qg * QMHA_GROUP + col) * d_model + (size_t)k * D + 8 * half;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const v4f a = *reinterpret_cast<const v4f*>(qp + 16 * s), c = *reinterpret_cast<const v4f*>(qp + 16 * s + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                qop[s][e] = (_Float16)a[e];
                qop[s][4 + e] = (_Float16)c[e];
            }
        }
    } else {
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int e = 0; e < 8; ++e) qop[s][e] = (_Float16)0.0f;
    }
    v16f o[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) o[m] = v16f{};
    float m_run = 0.0f, l_run = 0.0f;  // m0 = 0 (fa_tc_v1a.cu:290); l_run per lane half

    const char* kbase = reinterpret_cast<const char*>(Kh + (size_t)bh * N * D);
    const char* vbase = reinterpret_cast<const char*>(Vt + (size_t)bh * N * D);
    const int nst = (G + SG - 1) / SG;

    // stages arrive by buffer_load ... lds: fixed per-lane source offsets, the stage offset in soffset
    constexpr int KJ = (KCH / 64 + WAVES - 1) / WAVES, VJ = (VCH / 64 + WAVES - 1) / WAVES;
    int koff[KJ], voff[VJ];
#pragma unroll
    for (int jj = 0; jj < KJ; ++jj) {
        const int idx = (wave + jj * WAVES) * 64 + lane;
        const int row = idx / (RB / 16), cc = swz_src<RB>(row, idx % (RB / 16));
        koff[jj] = row * RB + 16 * cc;
    }
#pragma unroll
    for (int jj = 0; jj < VJ; ++jj) {
        const int idx = (wave + jj * WAVES) * 64 + lane;
        const int grp = idx / (4 * D), w = idx % (4 * D);
        const int d = w >> 2, cv = swz_src<64>(d, w & 3);
        voff[jj] = grp * 64 * D + d * 64 + 16 * cv;
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
    // S^T = K Q^T (fp32 accumulate) of tile gi of the stage in LDS
    auto qk = [&](const char* L, int gi) {
        v16f s = {};
        const int krow = gi * 32 + col;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const v8h kop = *reinterpret_cast<const v8h*>(L + krow * RB + 16 * swz_pos<RB>(krow, 2 * ks + half));
            s = __builtin_amdgcn_mfma_f32_32x32x16_f16(kop, qop[ks], s, 0, 0, 0);
        }
        return s;
    };
    // online softmax of one tile (fa_tc_v1a.cu:101-220) and O = alpha*O + P V (:207,:218)
    auto tile = [&](const char* L, int gi, const v16f& s) {
        v8h vpre[MB][2];
        if constexpr (FL & F16_VPRE) {
#pragma unroll
            for (int m = 0; m < MB; ++m)
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    const int d = 32 * m + col;
                    vpre[m][ks] = *reinterpret_cast<const v8h*>(L + KBYTES + gi * 64 * D + d * 64 +
                                                                16 * swz_pos<64>(d, 2 * ks + half));
                }
        }
        // Lazy base (r06): p = exp2(x - m_run) against a per-row base m_run (m0 = 0 as the
        // reference, :290) that moves to the tile's row max only when the tile's p of one of the row's two
        // key halves (this lane's 16, its partner lane's 16) sum above kLazySumCap -- so every p <= 2^12 and
        // the O / l rescale of the reference's every-tile alpha (:187-199) happens only then.  The row max is
        // computed on those tiles only; the sum is the row sum l needs anyway.  The result differs from the
        // reference's only in the rounding of half(p) (p scaled by 2^delta, not a power of two).
        float p[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) p[r] = __builtin_amdgcn_exp2f(fmaf(s[r], c_log2, -m_run));
        float ts = tree_sum16(p);  // this lane's half of the keys; the halves are joined once, in the epilogue
        const uint64_t over = __builtin_amdgcn_ballot_w64(ts > kLazySumCap);
        if (over) {  // rare (wave-uniform): rebase the rows with a half above the cap, recompute the tile
            float mx = fmaxf(fmaxf(s[0], s[1]), s[2]);  // max3 chain
#pragma unroll
            for (int r = 3; r < 15; r += 2) mx = fmaxf(fmaxf(mx, s[r]), s[r + 1]);
            mx = half_swap_max(fmaxf(mx, s[15]));
            const uint32_t rows = (uint32_t)over | (uint32_t)(over >> 32);
            const float m_b = ((rows >> col) & 1u) ? mx * c_log2 : m_run;  // per row; alpha 1 for the others
            const float alpha = __builtin_amdgcn_exp2f(m_run - m_b);
            l_run *= alpha;
#pragma unroll
            for (int m = 0; m < MB; ++m) o[m] *= alpha;
            m_run = m_b;
#pragma unroll
            for (int r = 0; r < 16; ++r) p[r] = __builtin_amdgcn_exp2f(fmaf(s[r], c_log2, -m_run));
            ts = tree_sum16(p);
        }
        v8h pop[2];
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
            const v2h h2 = __builtin_convertvector((v2f{p[r], p[r + 1]}), v2h);  // __float2half (RNE), :174
            pop[r >> 3][r & 7] = h2[0];
            pop[r >> 3][(r & 7) + 1] = h2[1];
        }
        l_run += ts;  // :198 (alpha folded into the rebase above)
#pragma unroll
        for (int m = 0; m < MB; ++m) {
            const int d = 32 * m + col;
            const char* vr = L + KBYTES + gi * 64 * D + d * 64;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const v8h vop = (FL & F16_VPRE) ? vpre[m][ks]
                                                : *reinterpret_cast<const v8h*>(vr + 16 * swz_pos<64>(d, 2 * ks + half));
                o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vop, pop[ks], o[m], 0, 0, 0);
            }
        }
    };

    issue(0, 0);
    qmha_dma_barrier();
    if constexpr (FL & F16_UNROLL) {
        auto stage = [&](auto BUF, int st) {
            constexpr int buf = decltype(BUF)::value;
            if (st + 1 < nst) issue(buf ^ 1, st + 1);
            if (active) {
                const char* L = lds[buf];
                const int ngr = G - st * SG;  // < SG only in a partial last stage (uniform)
#pragma unroll
                for (int gi = 0; gi < SG; ++gi) {
                    if (gi == 0 || gi < ngr) tile(L, gi, qk(L, gi));
                    __builtin_amdgcn_sched_barrier(0);  // one tile's registers at a time
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
    } else
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        if (st + 1 < nst) issue(buf ^ 1, st + 1);
        if (active) {
            const int ngr = min(SG, G - st * SG);
            const char* L = lds[buf];
            if ((FL & F16_PREFETCH) && ngr == SG) {
                v16f s_cur = qk(L, 0);
#pragma unroll
                for (int gi = 0; gi < SG; ++gi) {
                    v16f s_nxt = {};
                    if (gi + 1 < SG) s_nxt = qk(L, gi + 1);
                    __builtin_amdgcn_sched_barrier(0);
                    tile(L, gi, s_cur);
                    __builtin_amdgcn_sched_barrier(0);
                    s_cur = s_nxt;
                }
            } else {
                for (int gi = 0; gi < ngr; ++gi) tile(L, gi, qk(L, gi));
            }
        }
        qmha_dma_barrier();
    }
    if (active) {
        l_run = half_swap_add(l_run);
        const bool ok = l_run > 1e-10f;  // fa_tc_v1a.cu:384-388
        float* orow = O + ((size_t)b * N + (size_t)qg * QMHA_GROUP + col) * d_model + (size_t)k * D + 4 * half;
#pragma unroll
        for (int m = 0; m < MB; ++m)
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
// v3 (shipped at d = 64 / 128): the same tile and contract on v_mfma_f32_16x16x32_f16.  At the
// fp16 tile's VALU density after the lazy base (~9 VALU per 32 matrix-core cycles) the 16x16 shape holds
// a higher clock than 32x32x16 (tools/ubench/mfma_clock nv6: -6 % per unit at 6 fmas, -4 % at 12).
// Same staging as v2 (K rows, V^T slots in kv_of_slot_f16 order); the K rows are read in the key order
// kap(kb, m) that leaves each lane group's eight keys per query exactly where the PV B operand wants
// them: lane l = 16 g + r holds, per query block qb, S^T[kap(kb, 4 g + i)][16 qb + r] (kb = 0, 1,
// i = 0..3), and B operand element j of the P@V MFMA is V^T slot 8 g + j, i.e. kv_of_slot_f16(8 g + j)
// = kap(j >> 2, 4 g + (j & 3)).  Per lane: two queries (r, 16 + r) with eight keys each per tile.
// ---------------------------------------------------------------------------------------
__host__ __device__ constexpr int kap16(int kb, int m) { return 16 * (m >> 3) + 4 * ((m >> 2) & 1) + (m & 3) + 8 * kb; }
static_assert(kap16(0, 0) == kv_of_slot_f16(0) && kap16(1, 3) == kv_of_slot_f16(7) && kap16(0, 4) == kv_of_slot_f16(8) &&
                  kap16(1, 7) == kv_of_slot_f16(15) && kap16(0, 8) == kv_of_slot_f16(16) && kap16(1, 15) == kv_of_slot_f16(31),
              "lane group g's PV slots 8 g + j hold keys kap16(j >> 2, 4 g + (j & 3))");

template <int D, int WAVES, int SG>
__global__ __launch_bounds__(WAVES * 64, D > 64 ? 2 : 4) void qmha_fa_f16_v3_kernel(
    const float* __restrict__ Qf, const _Float16* __restrict__ Kh, const _Float16* __restrict__ Vt,
    float* __restrict__ O, int N, int H, int d_model, int nqb, float c_log2) {
    QMHA_ENABLE_AGPR_MFMA();
    asm volatile("" : "+v"(c_log2));
    constexpr int KS = D / 32;            // QK k-steps (K = 32)
    constexpr int DB = D / 16;            // PV d-blocks of 16 rows
    constexpr int RB = 2 * D;             // K row bytes
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

    // Q converted in-kernel (RNE) into the QK B operand: query 16 qb + r16, d = 32 ks + 8 grp .. +7
    v8h qop[2][KS];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if (active) {
                const float* qp = Qf + ((size_t)b * N + (size_t)qg * QMHA_GROUP + 16 * qb + r16) * d_model + (size_t)k * D +
                                  32 * ks + 8 * grp;
                const v4f a = *reinterpret_cast<const v4f*>(qp), c = *reinterpret_cast<const v4f*>(qp + 4);
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    qop[qb][ks][e] = (_Float16)a[e];
                    qop[qb][ks][4 + e] = (_Float16)c[e];
                }
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) qop[qb][ks][e] = (_Float16)0.0f;
            }
        }
    v4f o[DB][2];
#pragma unroll
    for (int m = 0; m < DB; ++m) o[m][0] = o[m][1] = v4f{};
    float m_run[2] = {0.0f, 0.0f}, l_run[2] = {0.0f, 0.0f};  // m0 = 0 (fa_tc_v1a.cu:290); l over this lane's keys

    const char* kbase = reinterpret_cast<const char*>(Kh + (size_t)bh * N * D);
    const char* vbase = reinterpret_cast<const char*>(Vt + (size_t)bh * N * D);
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
    // S^T blocks [kb][qb] of tile gi: rows kap16(kb, .) of the K tile against query block qb
    struct S4 {
        v4f v[2][2];
    };
    auto qk = [&](const char* L, int gi) {
        S4 s;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            const int krow = gi * 32 + kap16(kb, r16);
            s.v[kb][0] = s.v[kb][1] = v4f{};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const v8h kop = *reinterpret_cast<const v8h*>(L + krow * RB + 16 * ((4 * ks + grp) ^ kswz16<RB>(krow)));
#pragma unroll
                for (int qb = 0; qb < 2; ++qb) s.v[kb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kop, qop[qb][ks], s.v[kb][qb], 0, 0, 0);
            }
        }
        return s;
    };
    // online softmax of one tile (fa_tc_v1a.cu:101-220) and O += P V; the lazy base as v2, triggered by a
    // lane's eight keys of a query (a key quarter: lane groups g = 0..3) summing above kLazySumCap
    auto tile = [&](const char* L, int gi, const S4& s) {
        v8h vop[DB];  // V^T rows 16 m + r16, slots 8 grp .. +7 (read before the softmax, as v2's F16_VPRE)
#pragma unroll
        for (int m = 0; m < DB; ++m) {
            const int d = 16 * m + r16;
            vop[m] = *reinterpret_cast<const v8h*>(L + KBYTES + gi * 64 * D + d * 64 + 16 * (grp ^ vswz16(d)));
        }
        float p[2][8];
        float ts[2];
        auto softmax_p = [&]() {
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    p[qb][j] = __builtin_amdgcn_exp2f(fmaf(s.v[j >> 2][qb][j & 3], c_log2, -m_run[qb]));
                float q0 = p[qb][0] + p[qb][1], q1 = p[qb][2] + p[qb][3], q2 = p[qb][4] + p[qb][5], q3 = p[qb][6] + p[qb][7];
                ts[qb] = (q0 + q1) + (q2 + q3);
            }
        };
        softmax_p();
        const uint64_t over0 = __builtin_amdgcn_ballot_w64(ts[0] > kLazySumCap);
        const uint64_t over1 = __builtin_amdgcn_ballot_w64(ts[1] > kLazySumCap);
        if (over0 | over1) {  // rare (wave-uniform): rebase the queries with a key quarter above the cap
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) {
                const uint64_t over = qb ? over1 : over0;
                float mx = fmaxf(fmaxf(s.v[0][qb][0], s.v[0][qb][1]), fmaxf(s.v[0][qb][2], s.v[0][qb][3]));
                mx = fmaxf(mx, fmaxf(fmaxf(s.v[1][qb][0], s.v[1][qb][1]), fmaxf(s.v[1][qb][2], s.v[1][qb][3])));
                mx = fmaxf(mx, __shfl_xor(mx, 16));  // the query's four lane groups
                mx = fmaxf(mx, __shfl_xor(mx, 32));
                const uint32_t q16 = (uint32_t)(over | (over >> 32));
                const uint32_t rows = (q16 | (q16 >> 16)) & 0xffffu;
                const float m_b = ((rows >> r16) & 1u) ? mx * c_log2 : m_run[qb];
                const float alpha = __builtin_amdgcn_exp2f(m_run[qb] - m_b);
                l_run[qb] *= alpha;
#pragma unroll
                for (int m = 0; m < DB; ++m) o[m][qb] *= alpha;
                m_run[qb] = m_b;
            }
            softmax_p();
        }
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            l_run[qb] += ts[qb];  // :198 (alpha folded into the rebase above)
            v8h pop;
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const v2h h2 = __builtin_convertvector((v2f{p[qb][j], p[qb][j + 1]}), v2h);  // __float2half (RNE), :174
                pop[j] = h2[0];
                pop[j + 1] = h2[1];
            }
#pragma unroll
            for (int m = 0; m < DB; ++m) o[m][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(vop[m], pop, o[m][qb], 0, 0, 0);
        }
    };

    issue(0, 0);
    qmha_dma_barrier();
    auto stage = [&](auto BUF, int st) {
        constexpr int buf = decltype(BUF)::value;
        if (st + 1 < nst) issue(buf ^ 1, st + 1);
        if (active) {
            const char* L = lds[buf];
            const int ngr = G - st * SG;  // < SG only in a partial last stage (uniform)
#pragma unroll
            for (int gi = 0; gi < SG; ++gi) {
                if (gi == 0 || gi < ngr) tile(L, gi, qk(L, gi));
                __builtin_amdgcn_sched_barrier(0);  // one tile's registers at a time
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
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
            float l = l_run[qb];
            l += __shfl_xor(l, 16);
            l += __shfl_xor(l, 32);
            const bool ok = l > 1e-10f;  // fa_tc_v1a.cu:384-388
            float* orow = O + ((size_t)b * N + (size_t)qg * QMHA_GROUP + 16 * qb + r16) * d_model + (size_t)k * D + 4 * grp;
#pragma unroll
            for (int m = 0; m < DB; ++m) {
                v4f w;
#pragma unroll
                for (int j = 0; j < 4; ++j) w[j] = ok ? o[m][qb][j] / l : 0.0f;
                *reinterpret_cast<v4f*>(orow + 16 * m) = w;
            }
        }
    }
}

// Kh, Vt (Q is converted in the main kernel)
size_t f16_workspace_bytes(int B, int N, int H, int D) { return 2 * align_up((size_t)B * H * N * D * 2, 256); }

F16Workspace f16_carve(void* ws, int B, int N, int H, int D) {
    const size_t e = align_up((size_t)B * H * N * D * 2, 256);
    char* p = static_cast<char*>(ws);
    F16Workspace w;
    w.Qh = nullptr;
    w.Kh = reinterpret_cast<_Float16*>(p);
    w.Vt = reinterpret_cast<_Float16*>(p + e);
    return w;
}

template <int D, int WAVES, int SG, int FL>
static hipError_t fa_f16_v2_launch(const F16Workspace& w, const float* Qf, float* O, int B, int N, int H, int d_model,
                                   hipStream_t stream) {
    const int G = N / QMHA_GROUP;
    const int nqb = (G + WAVES - 1) / WAVES;
    const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2eH;
    hipLaunchKernelGGL((qmha_fa_f16_v2_kernel<D, WAVES, SG, FL>), dim3(B * H * nqb), dim3(WAVES * 64), 0, stream, Qf,
                       w.Kh, w.Vt, O, N, H, d_model, nqb, c_log2);
    return hipGetLastError();
}

#ifndef QMHA_F16_WAVES
#define QMHA_F16_WAVES 8  // A/B builds: -DQMHA_F16_WAVES=4
#endif
#ifndef QMHA_F16_FL
#define QMHA_F16_FL (F16_LB4 | F16_VPRE | F16_UNROLL)  // V operands before the softmax: -1.7 % (profiles/r02/ab/f16_vpre)
#endif
template <int D>
static hipError_t fa_f16_d(const F16Workspace& w, const float* Qf, float* O, int B, int N, int H, int d_model,
                           hipStream_t stream) {
#ifdef QMHA_ABLATION  // tuning alternatives: profiling builds only
    if constexpr (D == 64) {
        switch (tune_config("QMHA_F16_CFG")) {
            case 420: return fa_f16_v2_launch<D, 4, 2, 0>(w, Qf, O, B, N, H, d_model, stream);
            case 421: return fa_f16_v2_launch<D, 4, 2, F16_PREFETCH>(w, Qf, O, B, N, H, d_model, stream);
            case 440: return fa_f16_v2_launch<D, 4, 4, 0>(w, Qf, O, B, N, H, d_model, stream);
            case 441: return fa_f16_v2_launch<D, 4, 4, F16_PREFETCH>(w, Qf, O, B, N, H, d_model, stream);
            case 424: return fa_f16_v2_launch<D, 4, 2, F16_LB4>(w, Qf, O, B, N, H, d_model, stream);
            case 425: return fa_f16_v2_launch<D, 4, 2, F16_LB4 | F16_PREFETCH>(w, Qf, O, B, N, H, d_model, stream);
            case 427: return fa_f16_v2_launch<D, 4, 2, F16_LB4 | F16_VPRE | F16_PREFETCH>(w, Qf, O, B, N, H, d_model, stream);
            case 447: return fa_f16_v2_launch<D, 4, 4, F16_LB4 | F16_VPRE>(w, Qf, O, B, N, H, d_model, stream);
            case 448: return fa_f16_v2_launch<D, 4, 4, F16_LB4 | F16_VPRE | F16_PREFETCH>(w, Qf, O, B, N, H, d_model, stream);
            case 429: return fa_f16_v2_launch<D, 4, 2, F16_VPRE>(w, Qf, O, B, N, H, d_model, stream);
            // workgroup size at the default flags (113 VGPRs: 4 waves/SIMD either way): each LDS-DMA
            // stage shared by 8 / 16 waves (1 / 0.5 pieces per wave and tile instead of 2)
            case 480: return fa_f16_v2_launch<D, 8, 2, QMHA_F16_FL>(w, Qf, O, B, N, H, d_model, stream);
            case 4160: return fa_f16_v2_launch<D, 16, 2, QMHA_F16_FL>(w, Qf, O, B, N, H, d_model, stream);
            case 484: return fa_f16_v2_launch<D, 8, 4, QMHA_F16_FL>(w, Qf, O, B, N, H, d_model, stream);
            default: break;
        }
    }
#endif
    // default: v2 (LDS-DMA staging, per-tile softmax), 4 waves/SIMD budget (r01 A/B: 1.54 ms vs
    // 1.71 ms for the interleaved-pair kernel at B16 H16 N4096 d64), 8-wave workgroups: each LDS-DMA
    // stage is shared by 8 waves (one 1-KiB piece per wave and tile instead of two) at the same
    // occupancy (r03m: main -2.1 % against 4-wave workgroups, 16 waves +0 %, profiles/r03/ab/f16_wg).
    // d = 128 keeps 4-wave workgroups: its 199 VGPRs do not fit the 8-wave register budget (111 spills).
    // Other head sizes (d % 32 == 0, include/config.h:32): 4-wave workgroups, the V operands read at
    // their MFMA, a 2-wave budget at d = 96 and 1 wave above d = 128
    // d = 64 / 128: the 16x16x32 kernel (v3), same box, alternating: C3 -2.5 %, d = 128 -1.9 %; at d = 32 it
    // measured +2.8 % (93 VGPRs, 5 waves per SIMD against v2's 6; at a 6-wave budget, spilling 11 registers,
    // +2.9 % / +9 %), so v2 keeps d = 32 (profiles/r06/ab_f16_mma16/)
    if constexpr (D == 64 || D == 128) {
        constexpr int W = D <= 64 ? QMHA_F16_WAVES : 4;
        const int G = N / QMHA_GROUP, nqb = (G + W - 1) / W;
        const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2eH;
        hipLaunchKernelGGL((qmha_fa_f16_v3_kernel<D, W, 2>), dim3(B * H * nqb), dim3(W * 64), 0, stream, Qf, w.Kh, w.Vt, O,
                           N, H, d_model, nqb, c_log2);
        return hipGetLastError();
    }
    if constexpr (D == 32 || D == 64 || D == 128)
        return fa_f16_v2_launch<D, (D <= 64 ? QMHA_F16_WAVES : 4), 2, QMHA_F16_FL>(w, Qf, O, B, N, H, d_model, stream);
    else
        return fa_f16_v2_launch<D, 4, 2, F16_UNROLL | (D > 128 ? F16_LB1 : 0)>(w, Qf, O, B, N, H, d_model, stream);
}

hipError_t launch_fa_f16_main(const F16Workspace& w, const float* Qf, float* O, int B, int N, int H, int D, int d_model,
                              hipStream_t stream) {
    switch (D) {
        case 32: return fa_f16_d<32>(w, Qf, O, B, N, H, d_model, stream);
        case 64: return fa_f16_d<64>(w, Qf, O, B, N, H, d_model, stream);
        case 128: return fa_f16_d<128>(w, Qf, O, B, N, H, d_model, stream);
        case 96: return fa_f16_d<96>(w, Qf, O, B, N, H, d_model, stream);
        case 160: return fa_f16_d<160>(w, Qf, O, B, N, H, d_model, stream);
        case 192: return fa_f16_d<192>(w, Qf, O, B, N, H, d_model, stream);
        case 224: return fa_f16_d<224>(w, Qf, O, B, N, H, d_model, stream);
        case 256: return fa_f16_d<256>(w, Qf, O, B, N, H, d_model, stream);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace qmha
