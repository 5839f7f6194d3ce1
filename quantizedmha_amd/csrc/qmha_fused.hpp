// qmha_fused.hpp -- the K / V pre-pass done by a sweep kernel's own workgroups: one
// launch per call instead of two, the pre-pass's HBM traffic running under the VALU-bound sweep.  Shared
// by the per-block int8 kernel (FL_FUSED: K / V quantised, fa_tc_int8_b.cu:33-152) and the fp16 kernel
// (F16_FUSED: K / V converted to f16, fa_tc_v1a.cu:300-330); the caller supplies the per-group producer.
//
// Work split.  Workgroup v's "own" groups are the KV groups with the indices of its Q groups (q-block qb:
// groups WAVES qb .. WAVES qb + WAVES - 1 of head v / nqb, one per wave).  The dispatcher deals
// workgroups to the 8 XCDs round-robin and xcd_remap gives each XCD a contiguous range [c0, c1) of
// logical ids, dispatched in order; R workgroups of a range are resident at once.
//   * the first R of a range (the first round) produce their own groups, plus the groups of the range's
//     first head that belong to the previous range (q-blocks before c0);
//   * workgroup v produces the own groups of v + R (same range): a round ahead of their consumers.
// Every workgroup then waits until all G groups of its head are flagged.  A group is always produced by a
// workgroup dispatched no later than its consumers, so the wait cannot deadlock under in-order dispatch
// (heads longer than a round, nqb > R, are routed to the two launches by the host); it is bounded anyway
// (wait_ticks, s_memrealtime): past the bound a wave produces the missing groups itself (bit-identical
// bytes, so duplicate producers are harmless).  tests/test_fused_schedule.py restates the split on the CPU.
// Coherence.  Producers write with agent-coherent (sc1) stores, wait for them (vmcnt(0)), then set the
// flag; consumers poll the flags with agent-coherent loads.  A consumer's caches hold no line of a group
// before that group is flagged: the kernel starts with invalidated caches, a group's K / V blocks are
// whole lines, and anything smaller (the int8 scales) is padded to whole lines per head and read only
// after the whole head is flagged.  tests/test_gpu_zfused.py runs every fused call on scratch that holds
// a poison pattern or another input's bytes, so a stale read cannot pass unseen.
#pragma once
#include "qmha_common.hpp"

namespace qmha {

struct FusedCtl {
    uint32_t* ready;       // [B*H][G]: 1 once group g's operands are written (zeroed by the call)
    int R;                 // resident workgroups per XCD (the launcher's occupancy answer)
    int mode;              // 0 production; 1 test: every group produced by a workgroup of another XCD
    long long wait_ticks;  // bound of the wait, 100 MHz ticks
    int ablate;            // measurements only (results wrong): bit 0 no wait for the head's groups; bit 2 no
                           // production at all (the sweep on whatever the scratch holds); bits 1, 3: the
                           // producer's (qmha_fa_int8.hip produce_kv_group)
};

// xcd_remap's logical range [lo, hi) of XCD x for a grid of nwg workgroups
__device__ __forceinline__ void xcd_range(int nwg, int x, int& lo, int& hi) {
    const int q8 = nwg / 8, r8 = nwg % 8;
    lo = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
    hi = lo + (x < r8 ? q8 + 1 : q8);
}

// Publish group g of head slice bh: every store of it has completed (the producer's sc1 stores), then the flag
__device__ __forceinline__ void fused_flag(const FusedCtl& f, int bh, int g, int G, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(f.ready + (size_t)bh * G + g, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wait until all G groups of head bh are flagged; past the bound, wave `wave` of WAVES produces the missing
// groups g with g % WAVES == wave itself (every wave of the workgroup does its share).  produce(bh, g)
// writes and flags one group.
template <int WAVES, class Produce>
__device__ __forceinline__ void fused_wait_head(const FusedCtl& f, int bh, int G, int wave, int lane, Produce&& produce) {
    const uint32_t* rd = f.ready + (size_t)bh * G;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    bool self = false;
    for (;;) {
        bool all = true;
        for (int g0 = 0; g0 < G; g0 += 64) {
            const int g = g0 + lane;
            const uint32_t v = g < G ? __hip_atomic_load(rd + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1u;
            uint64_t miss = __builtin_amdgcn_ballot_w64(v != 1u);
            if (miss) {
                all = false;
                if (self)
                    for (; miss; miss &= miss - 1) {
                        const int gg = g0 + __builtin_ctzll(miss);
                        if (gg % WAVES == wave) produce(bh, gg);
                    }
            }
        }
        if (all) break;
        if (!self && __builtin_amdgcn_s_memrealtime() - t0 > f.wait_ticks)
            self = true;
        else
            __builtin_amdgcn_s_sleep(2);
    }
    asm volatile("" ::: "memory");
}

// This workgroup's share of the production (see the header), then the wait for its own head; ends with a
// workgroup barrier (the producers' LDS tiles may alias the sweep's LDS ring).  wg = the logical id
// (xcd_remap of blockIdx.x), bh = its head slice.
template <int WAVES, class Produce>
__device__ __forceinline__ void fused_produce_and_wait(const FusedCtl& f, int wg, int bh, int nqb, int G, int wave,
                                                       int lane, Produce&& produce) {
    const int nwg = gridDim.x;
    int c0, c1;
    xcd_range(nwg, blockIdx.x % 8, c0, c1);
    const int pos = wg - c0;
    // the production list: n_own (its own groups, or the test rule's), n_orph (the range's first head's
    // q-blocks that lie in the previous range), then the groups of workgroup v_ahead -- before the wait
    // for its own head if a consumer of them may already be waiting
    int n_own = 0, n_orph = 0, n_pre = 0, n_total = 0, v_own = wg, v_ahead = 0, orph0 = 0, Rp = 1;
    if (f.mode == 0) {
        const int R = f.R, j0 = c0 % nqb;
        Rp = min(R, c1 - c0);
        orph0 = c0 - j0 + pos;  // workgroup ids c0 - j0 + pos + m * Rp < c0
        v_ahead = wg + R;
        const bool first = pos < R, ahead = v_ahead < c1;
        // early: a consumer of those groups is already dispatched (the first round of the range, or this
        // workgroup's own head when a head is longer than a round)
        const bool early = ahead && (v_ahead / nqb) * nqb <= (first ? c0 + Rp - 1 : wg);
        n_own = first ? 1 : 0;
        n_orph = first && pos < j0 ? (j0 - 1 - pos) / Rp + 1 : 0;
        n_pre = n_own + n_orph + (early ? 1 : 0);
        n_total = n_pre + (ahead && !early ? 1 : 0);
    } else {  // test: workgroup pos of range x produces the own groups of workgroup pos of range x - 1
        int p0, p1;
        xcd_range(nwg, (blockIdx.x + 7) % 8, p0, p1);
        v_own = p0 + pos;
        n_own = n_pre = n_total = v_own < p1 ? 1 : 0;
    }
    if (f.ablate & 4) n_pre = n_total = 0;
    for (int it = 0;; ++it) {  // wave-uniform; one inlined copy of the producer
        if (it == n_pre && !(f.ablate & 5)) fused_wait_head<WAVES>(f, bh, G, wave, lane, produce);
        if (it >= n_total) break;
        const int v = it < n_own ? v_own : (it < n_own + n_orph ? orph0 + (it - n_own) * Rp : v_ahead);
        const int g = (v % nqb) * WAVES + wave;
        if (g < G) produce(v / nqb, g);
    }
    __syncthreads();
}

}  // namespace qmha
