// qmha_fa_f16_pipe_ablation.hip -- NOT BUILT.  The r04 A/B of round-3 VERDICT item 3: the fp16
// (fa_tc_v1a) contract in a software-pipelined kernel whose eight VALU regions each start with the
// transcendental / quarter-rate work that tools/ubench/mfma_fill.hip shows hiding behind an MFMA.
// It was spliced into quantizedmha_amd/csrc/qmha_fa_f16.hip (before f16_workspace_bytes; the launch
// hook below inside fa_f16_d) and built with -DQMHA_F16_PIPE=4 [-DQMHA_F16_PIPE_JIT].  Parity green
// (27 fp16 GPU tests); measured (profiles/r04/ab_f16_pipe/): d = 64 1.42-1.77 ms main against
// 1.30 ms (the kernel needs 175-184 VGPRs, spills at the 3-wave budget), d = 32 1.72-1.75 against
// 1.70 ms with no spill -- and at d = 32 the SQ counters show the same GRBM_GUI_ACTIVE (28.1 M vs
// 28.0 M), the same VALU instructions per wave (10,427 vs 10,519) and the same MFMA busy (29.8 vs
// 29.9 %): the order of the work does not change the time, only its amount does.

// ---------------------------------------------------------------------------------------
// Software-pipelined fp16 kernel with class-placed MFMA shadows (r04, round-3 VERDICT item 3; A/B:
// QMHA_F16_PIPE).  Iteration t runs tile t's softmax while the matrix core executes Q@K^T of tile
// t+1 and P@V of tile t-1 (P@V straight into O, as in v2; O takes tile t-1's alpha at the start of
// iteration t, before P@V of t-1 is issued).  The VALU work is cut into eight sched_barrier
// regions, one MFMA after each; every region starts with the transcendental / quarter-rate work
// (exp, cvt_pk, max3, permlane) that tools/ubench/mfma_fill.hip shows hiding behind the MFMA just
// issued (~25 cycles per MFMA at 1-4 waves/SIMD), the full-rate fp32 work (scores, row sums) after
// it.  MFMA order (d = 64): QK0 PV00 QK1 PV10 QK2 PV01 QK3 PV11 -- chained pairs two slots apart.
// K/V staging as the int8 pipe kernel: stages of 2 tiles, a 3-slot LDS-DMA ring two stages ahead.
// ---------------------------------------------------------------------------------------
__host__ __device__ constexpr int f16_slot_op(int D, int s) {  // 100 + ks = QK k-step, 2m + ks = PV
    constexpr int d64[8] = {100, 0, 101, 2, 102, 1, 103, 3};
    constexpr int d32[8] = {100, -1, 0, -1, 101, -1, 1, -1};
    return D == 32 ? d32[s] : d64[s];
}

template <int D, int WAVES>
#ifndef QMHA_F16_PIPE_LB
#define QMHA_F16_PIPE_LB 3
#endif
__global__ __launch_bounds__(WAVES * 64, QMHA_F16_PIPE_LB) void qmha_fa_f16_pipe_kernel(const float* __restrict__ Qf,
                                                                        const _Float16* __restrict__ Kh,
                                                                        const _Float16* __restrict__ Vt,
                                                                        float* __restrict__ O, int N, int H, int d_model,
                                                                        int nqb, float c_log2) {
    static_assert(D == 32 || D == 64, "pipelined fp16 kernel: d = 32 / 64");
    asm volatile("" : "+v"(c_log2));  // the score scale in a VGPR (an SGPR operand issues at the slow rate)
    constexpr int KS = D / 16, MB = D / 32, RB = 2 * D;
    constexpr int SG = 2, RING = 3, PF = RING - 1;
    constexpr int KBYTES = SG * 32 * RB, VBYTES = SG * 32 * D * 2, SBYTES = KBYTES + VBYTES;
    constexpr int KCH = KBYTES / 16, VCH = VBYTES / 16;
    __shared__ __attribute__((aligned(16))) char lds[RING][SBYTES];

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
    if (active) {  // Q converted in-kernel (RNE, __float2half, fa_tc_v1a.cu:300-330)
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
    const char* kbase = reinterpret_cast<const char*>(Kh + (size_t)bh * N * D);
    const char* vbase = reinterpret_cast<const char*>(Vt + (size_t)bh * N * D);
    const int nst = (G + SG - 1) / SG;
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
    auto issue_at = [&](int st, int slot) {
        const int ngr = min(SG, G - st * SG);
        char* L = lds[slot];
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
    auto kop_at = [&](int slot, int par, int ks) {
        const int krow = par * 32 + col;
        return *reinterpret_cast<const v8h*>(lds[slot] + krow * RB + 16 * swz_pos<RB>(krow, 2 * ks + half));
    };
    auto vop_at = [&](int slot, int par, int m, int ks) {
        const int d = 32 * m + col;
        return *reinterpret_cast<const v8h*>(lds[slot] + KBYTES + par * 64 * D + d * 64 + 16 * swz_pos<64>(d, 2 * ks + half));
    };

    v16f o[MB];
#pragma unroll
    for (int m = 0; m < MB; ++m) o[m] = v16f{};
    float m_run = 0.0f, l_run = 0.0f;  // m0 = 0 (fa_tc_v1a.cu:290); l_run per lane half
    float alpha_prev = 1.0f;
    v16f s_cur, s_nxt;
    v8h pc[2], pp[2];
    auto qk = [&](const v8h& kk, int ks) {
        s_nxt = __builtin_amdgcn_mfma_f32_32x32x16_f16(kk, qop[ks], ks == 0 ? v16f{} : s_nxt, 0, 0, 0);
    };
    issue_at(0, 0);
    if (nst > 1) issue_at(1, 1);
    qmha_dma_barrier();
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qk(kop_at(0, 0, ks), ks);
    s_cur = s_nxt;

#define QMHA_FENCE() __builtin_amdgcn_sched_barrier(0)
    auto iter = [&](int t, auto HP, auto HN, auto PH) {
        constexpr bool has_prev = decltype(HP)::value, has_next = decltype(HN)::value;
        constexpr int ph = decltype(PH)::value;
        const int odd = ph >= 0 ? ((1 + ph) & 1) : (t & 1);
        const int slot_p = ph >= 0 ? ((ph >> 1) % RING) : (((t - 1) >> 1) % RING);
        const int par_p = ph >= 0 ? (ph & 1) : ((t - 1) & 1);
        const int slot_nx = ph >= 0 ? (((2 + ph) >> 1) % RING) : (((t + 1) >> 1) % RING);
        const int par_n = ph >= 0 ? (ph & 1) : ((t + 1) & 1);
        const int dma_st = (t >> 1) + PF;
        const int dma_slot = ph >= 0 ? ((((1 + ph) >> 1) + PF) % RING) : (((t >> 1) + PF) % RING);
        if (odd) {
            qmha_dma_barrier();  // stage (t+1)/2 landed; the stage (t-3)/2 slot is free
            if (dma_st < nst) issue_at(dma_st, dma_slot);
        }
        v8h kv[8];  // the operand of slot s (read one slot ahead)
        auto rd = [&](int s) {
            const int op = f16_slot_op(D, s);
            if (op >= 100) {
                if constexpr (has_next) kv[s] = kop_at(slot_nx, par_n, op - 100);
            } else if (op >= 0) {
                if constexpr (has_prev) kv[s] = vop_at(slot_p, par_p, op >> 1, op & 1);
            }
        };
        auto mf = [&](int s) {
#ifdef QMHA_F16_PIPE_JIT
            rd(s);
#endif
            const int op = f16_slot_op(D, s);
            if (op >= 100) {
                if constexpr (has_next) qk(kv[s], op - 100);
            } else if (op >= 0) {
                if constexpr (has_prev) o[op >> 1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(kv[s], pp[op & 1], o[op >> 1], 0, 0, 0);
            }
        };
        float x[16], p[16];
#ifndef QMHA_F16_PIPE_JIT
        rd(0);
#endif
#ifndef QMHA_F16_PIPE_JIT
        rd(1);
#endif
        QMHA_FENCE();
        // ---- R0: O *= alpha of tile t-1 (rare), the head of tile t: row max, running max, alpha
        if constexpr (has_prev) {
            if (__builtin_amdgcn_ballot_w64(alpha_prev != 1.0f)) {
#pragma unroll
                for (int m = 0; m < MB; ++m) o[m] *= alpha_prev;
            }
        }
        float mx = fmaxf(fmaxf(s_cur[0], s_cur[1]), s_cur[2]);
#pragma unroll
        for (int r = 3; r < 15; r += 2) mx = fmaxf(fmaxf(mx, s_cur[r]), s_cur[r + 1]);
        mx = half_swap_max(fmaxf(mx, s_cur[15]));
        const float m_new = fmaxf(m_run, mx * c_log2);
        const float alpha = __builtin_amdgcn_exp2f(m_run - m_new);
        QMHA_FENCE();
        mf(0);
#ifndef QMHA_F16_PIPE_JIT
        rd(2);
#endif
        QMHA_FENCE();
        // ---- R1: scores of rows 0..7 (full rate)
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = fmaf(s_cur[r], c_log2, -m_new);
        QMHA_FENCE();
        mf(1);
#ifndef QMHA_F16_PIPE_JIT
        rd(3);
#endif
        QMHA_FENCE();
        // ---- R2: exps 0..3 (behind the MFMA), scores 8..15
#pragma unroll
        for (int r = 0; r < 4; ++r) p[r] = __builtin_amdgcn_exp2f(x[r]);
#pragma unroll
        for (int r = 8; r < 16; ++r) x[r] = fmaf(s_cur[r], c_log2, -m_new);
        QMHA_FENCE();
        mf(2);
#ifndef QMHA_F16_PIPE_JIT
        rd(4);
#endif
        QMHA_FENCE();
        auto cvt = [&](int r) {  // P = half(p) (RNE, fa_tc_v1a.cu:174): entries r, r+1
            const v2h h2 = __builtin_convertvector((v2f{p[r], p[r + 1]}), v2h);
            pc[r >> 3][r & 7] = h2[0];
            pc[r >> 3][(r & 7) + 1] = h2[1];
        };
        // ---- R3: exps 4..7, P entries 0..3
#pragma unroll
        for (int r = 4; r < 8; ++r) p[r] = __builtin_amdgcn_exp2f(x[r]);
        cvt(0);
        cvt(2);
        QMHA_FENCE();
        mf(3);
#ifndef QMHA_F16_PIPE_JIT
        rd(5);
#endif
        QMHA_FENCE();
        // ---- R4: exps 8..11, P entries 4..7
#pragma unroll
        for (int r = 8; r < 12; ++r) p[r] = __builtin_amdgcn_exp2f(x[r]);
        cvt(4);
        cvt(6);
        QMHA_FENCE();
        mf(4);
#ifndef QMHA_F16_PIPE_JIT
        rd(6);
#endif
        QMHA_FENCE();
        // ---- R5: exps 12..15, the row sum of 0..7
#pragma unroll
        for (int r = 12; r < 16; ++r) p[r] = __builtin_amdgcn_exp2f(x[r]);
        float rs0 = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
        asm volatile("" : "+v"(rs0));
        QMHA_FENCE();
        mf(5);
#ifndef QMHA_F16_PIPE_JIT
        rd(7);
#endif
        QMHA_FENCE();
        // ---- R6: P entries 8..15, the row sum of 8..15
        cvt(8);
        cvt(10);
        cvt(12);
        cvt(14);
        asm volatile("" : "+v"(pc[0]), "+v"(pc[1]));
        const float rs1 = ((p[8] + p[9]) + (p[10] + p[11])) + ((p[12] + p[13]) + (p[14] + p[15]));
        QMHA_FENCE();
        mf(6);
        QMHA_FENCE();
        // ---- R7: l = alpha * l + sum(p) (fa_tc_v1a.cu:198), this lane's half of the keys
        l_run = fmaf(alpha, l_run, rs0 + rs1);
        m_run = m_new;
        QMHA_FENCE();
        mf(7);
        QMHA_FENCE();
        pp[0] = pc[0];
        pp[1] = pc[1];
        alpha_prev = alpha;
        if constexpr (has_next) s_cur = s_nxt;
    };
    using T1 = std::integral_constant<bool, true>;
    using F0 = std::integral_constant<bool, false>;
    using DYN = std::integral_constant<int, -1>;
    iter(0, F0{}, T1{}, DYN{});
    int t = 1;
    constexpr int PER = 2 * RING;
    for (; t + PER <= G - 1; t += PER) {
        iter(t, T1{}, T1{}, std::integral_constant<int, 0>{});
        iter(t + 1, T1{}, T1{}, std::integral_constant<int, 1>{});
        iter(t + 2, T1{}, T1{}, std::integral_constant<int, 2>{});
        iter(t + 3, T1{}, T1{}, std::integral_constant<int, 3>{});
        iter(t + 4, T1{}, T1{}, std::integral_constant<int, 4>{});
        iter(t + 5, T1{}, T1{}, std::integral_constant<int, 5>{});
    }
    for (; t < G - 1; ++t) iter(t, T1{}, T1{}, DYN{});
    iter(G - 1, T1{}, F0{}, DYN{});
#undef QMHA_FENCE
    {  // drain: O takes the last tile's alpha, then its P@V
        const int tl = G - 1;
        if (__builtin_amdgcn_ballot_w64(alpha_prev != 1.0f)) {
#pragma unroll
            for (int m = 0; m < MB; ++m) o[m] *= alpha_prev;
        }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int m = 0; m < MB; ++m)
                o[m] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vop_at((tl >> 1) % RING, tl & 1, m, ks), pp[ks], o[m], 0, 0, 0);
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


// launch hook (inside fa_f16_d):
/*
#ifdef QMHA_F16_PIPE  // A/B builds: the class-placed pipelined kernel at d = 32 / 64 (N >= 64)
    if constexpr (D == 32 || D == 64) {
        const int G = N / QMHA_GROUP;
        if (G >= 2) {
            constexpr int WV = QMHA_F16_PIPE;  // waves per workgroup
            const int nqb = (G + WV - 1) / WV;
            const float c_log2 = (1.0f / sqrtf((float)D)) * kLog2eH;
            hipLaunchKernelGGL((qmha_fa_f16_pipe_kernel<D, WV>), dim3(B * H * nqb), dim3(WV * 64), 0, stream, Qf, w.Kh,
                               w.Vt, O, N, H, d_model, nqb, c_log2);
            return hipGetLastError();
        }
    }
#endif
*/
