// qmha_common.hpp -- shared device/host helpers for the MI355X (gfx950) attention path.
//
// Layout vocabulary used throughout (DESIGN.md "Data layout in HBM"):
//   X      : caller fp32 tensor [B][N][d_model], head k owns columns [k*D, (k+1)*D)
//            (reference include/launchers.h:42,50-52).
//   group  : 32 consecutive sequence rows of one head -- the reference's Br = Bc = 32
//            quantisation block (include/config.h:10-11, fa_tc_int8_b.cu:484,496,518).
//   bh     : flattened (batch, head) index, b*H + k.
//   Xi     : int8 [bh][N][D] row-major (Q, K after the pre-pass).
//   Vt     : V as the MFMA "V^T" operand: per group a [D][32] block whose 32 kv slots are
//            permuted so that byte 16*h + e of row d holds kv = (e&3) + 8*(e>>2) + 4*h,
//            i.e. exactly the kv order in which a 32x32 MFMA accumulator hands P^T to a
//            lane (see kv_of_slot_i8 below).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define QMHA_GROUP 32

// MFMA accumulators in AGPRs (A/B builds only).  r01 read tools/ubench/mfma_coexec.hip as "a VALU
// stream overlaps another wave's MFMAs only with AGPR accumulators"; r02's mfma_split.hip shows
// MFMA and VALU issue cycles ADD on a SIMD in every form once the VALU side is saturated
// (profiles/r02/ubench_mfma_split*.txt), so production builds keep -amdgpu-mfma-vgpr-form.  The
// compiler selects the AGPR form only for functions that may use AGPRs, which this empty
// clobber declares; the build drops -amdgpu-mfma-vgpr-form when QMHA_MFMA_AGPR is set.
#ifdef QMHA_MFMA_AGPR
#define QMHA_ENABLE_AGPR_MFMA() asm volatile("" ::: "a0")
#else
#define QMHA_ENABLE_AGPR_MFMA() ((void)0)
#endif

// ISA inspection builds (-DQMHA_ISA_MARKS): an s_nop 15 fence around a code region so
// tools/isa.py can cut it out of the disassembly.  Empty in every real build.
#ifdef QMHA_ISA_MARKS
#define QMHA_ISA_MARK() asm volatile("s_nop 15" ::: "memory")
#else
#define QMHA_ISA_MARK() ((void)0)
#endif

// address-space pointer types for __builtin_amdgcn_global_load_lds (LDS-DMA)
typedef __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;
// buffer resource word 3 on gfx9-family parts (raw buffer, 32-bit data format)
#define QMHA_BUF_DWORD3 0x00020000

// 16 bytes per lane from base + voff + soff (bytes; nrec = bytes addressable from base) into
// LDS at dst (wave-uniform) + 16 * lane: buffer_load_dwordx4 ... lds.  Uniform base / nrec
// keep the resource in SGPRs; reads past nrec return zeros.
__device__ __forceinline__ void buffer_load_lds16(const void* base, int nrec, lptr_t dst, int voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, nrec, QMHA_BUF_DWORD3),
                                             dst, 16, voff, soff, 0, 0);
}

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef _Float16 v8h __attribute__((ext_vector_type(8)));
typedef _Float16 v2h __attribute__((ext_vector_type(2)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef _Float16 v4h __attribute__((ext_vector_type(4)));
typedef int v2i __attribute__((ext_vector_type(2)));

// --------------------------------------------------------------------------
// MFMA accumulator maps (gfx950, every 32x32 shape):
//   lane l, register r  ->  column = l & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5)
// With the "swapped" products used by every kernel here (S^T = K Q^T and O^T = V^T P^T)
// the column is the query row, so all per-query statistics are lane-local.
// --------------------------------------------------------------------------
__host__ __device__ constexpr int acc_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// int8 32x32x32: operand element e (0..15) of lane half h pairs with accumulator row
// acc_row(e, h) of the S^T tile, so the V^T operand slot 16*h + e must hold that kv.
__host__ __device__ constexpr int kv_of_slot_i8(int slot) { return acc_row(slot & 15, slot >> 4); }
__host__ __device__ constexpr int slot_of_kv_i8(int kv) { return 16 * ((kv >> 2) & 1) + 4 * (kv >> 3) + (kv & 3); }

// f16 32x32x16: k-step s (0,1) takes accumulator registers 8s..8s+7; element e of lane
// half h pairs with acc_row(8s + e, h) = 16s + 4h + (e & 3) + 8 * (e >> 2).
__host__ __device__ constexpr int kv_of_slot_f16(int slot) {
    return 16 * (slot >> 4) + 4 * ((slot >> 3) & 1) + (slot & 3) + 8 * ((slot >> 2) & 1);
}
__host__ __device__ constexpr int slot_of_kv_f16(int kv) {
    return 16 * (kv >> 4) + 8 * ((kv >> 2) & 1) + (kv & 3) + 4 * ((kv >> 3) & 1);
}

// LDS layout of a row of RB bytes read as 16-byte chunks by ds_read_b128 with one row per lane
// (rows 0..31 of a 32 x RB operand).  swz_pos<RB>(row, c) = the LDS chunk slot holding source
// chunk c of `row`; swz_src<RB>(row, j) = the source chunk stored in slot j.  Power-of-two chunk
// counts (d = 32 / 64 / 128 / 256): an XOR swizzle, conflict-free per 16-lane group (an
// involution, so both directions are the same).  Other counts (d = 96 / 160 / 192 / 224): a
// rotation by the row's bank-row index (a bijection for any count).
template <int RB>
__device__ __forceinline__ int swz_rot(int row) {
    constexpr int rows_per_bankrow = 256 / RB >= 1 ? 256 / RB : 1;
    constexpr int cpr = RB / 16;
    if constexpr ((cpr & (cpr - 1)) == 0) return (row / rows_per_bankrow) & (cpr - 1);
    else return (row / rows_per_bankrow) % cpr;
}
template <int RB>
__device__ __forceinline__ int swz_pos(int row, int c) {
    constexpr int cpr = RB / 16;
    if constexpr ((cpr & (cpr - 1)) == 0) return c ^ swz_rot<RB>(row);
    else return (c + swz_rot<RB>(row)) % cpr;
}
template <int RB>
__device__ __forceinline__ int swz_src(int row, int j) {
    constexpr int cpr = RB / 16;
    if constexpr ((cpr & (cpr - 1)) == 0) return j ^ swz_rot<RB>(row);
    else return (j + cpr - swz_rot<RB>(row)) % cpr;
}

// LDS chunk swizzles of the 16x16-MFMA kernels (qmha_fa_f16.hip v3, qmha_fa_int8.hip pt v3): slot =
// chunk ^ swz(row).  A ds_read_b128 lane group (16 lanes: one 256-byte bank row) reads, in the kap16 key
// order, K rows {0-3, 20-23} at chunk c and {4-7, 16-19} at chunk c ^ 1 (+8 kb), and V^T rows (d)
// r16 = {0-3, 12-15} at chunk g and {4-11} at chunk g ^ 1.  swz_rot's (row / rows-per-bank-row) puts two
// of those four row quads on the same slots (2-way: SQ_LDS_BANK_CONFLICT was half of all LDS cycles);
// these XOR masks give every lane of a group its own 16-byte slot (checked exhaustively in
// tests/test_abi.py::test_lds_swizzle16_conflict_free).
template <int RB>
__host__ __device__ constexpr int kswz16(int row) {
    static_assert(RB == 64 || RB == 128 || RB == 256, "64 / 128 / 256-byte K rows");
    if constexpr (RB == 64) return 2 * ((row >> 4) & 1);
    else if constexpr (RB == 128) return ((row >> 1) & 1) ^ (2 * ((row >> 2) & 1)) ^ (4 * ((row >> 4) & 1));
    else return (row & 1) ^ (2 * ((row >> 1) & 1)) ^ (4 * ((row >> 2) & 1)) ^ (8 * ((row >> 4) & 1));
}
// V^T operand rows: 64 bytes (32 keys of f16) per d row
__host__ __device__ constexpr int vswz16(int d) { return (2 * ((d >> 2) & 1)) ^ (3 * ((d >> 3) & 1)); }

// --------------------------------------------------------------------------
// cross-lane helpers (wave64)
// --------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}

// Combine the two 32-lane halves (lanes l and l^32 hold the same query row).
__device__ __forceinline__ float half_swap_max(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(x), __float_as_int(x), false, false);
    return fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}
__device__ __forceinline__ float half_swap_add(float x) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_int(x), __float_as_int(x), false, false);
    return __int_as_float(r[0]) + __int_as_float(r[1]);
}
__device__ __forceinline__ int half_swap_max_i(int x) {
    auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return max((int)r[0], (int)r[1]);
}

// Max over the 32 lanes of each half (result in every lane of that half).
__device__ __forceinline__ float half_max32(float x) {
    x = fmaxf(x, dpp_mov<0xB1>(x));   // quad_perm(1,0,3,2)
    x = fmaxf(x, dpp_mov<0x4E>(x));   // quad_perm(2,3,0,1)
    x = fmaxf(x, dpp_mov<0x141>(x));  // row_half_mirror
    x = fmaxf(x, dpp_mov<0x140>(x));  // row_mirror
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_int(x), __float_as_int(x), false, false);
    return fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}

// Max over the 32 lanes of each half for NON-NEGATIVE floats, on the bit patterns (integer
// max orders non-negative IEEE floats; avoids the NaN-canonicalising v_max_f32 pairs).
template <int CTRL>
__device__ __forceinline__ int dpp_mov_i(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ float half_max32_nonneg(float xf) {
    int x = __float_as_int(xf);
    x = max(x, dpp_mov_i<0xB1>(x));
    x = max(x, dpp_mov_i<0x4E>(x));
    x = max(x, dpp_mov_i<0x141>(x));
    x = max(x, dpp_mov_i<0x140>(x));
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return __int_as_float(max((int)r[0], (int)r[1]));
}

// Max over all 64 lanes.
__device__ __forceinline__ float wave_max64(float x) { return half_swap_max(half_max32(x)); }

// --------------------------------------------------------------------------
// The reference quantiser (fa_tc_int8_b.cu:104-106,136-140), elementwise part.
// --------------------------------------------------------------------------
__device__ __forceinline__ float qmha_scale_from_absmax(float absmax) {
    return fmaxf(absmax / 127.0f, 1e-8f);
}
__device__ __forceinline__ int qmha_quant_i8(float v, float inv) {
    int q = __float2int_rn(v * inv);
    return q < -128 ? -128 : (q > 127 ? 127 : q);
}

// x / 127 and 1 / x with two fma corrections (Markstein): the correctly rounded quotient
// except in rare double-rounding cases, in 3 VALU ops instead of the ~10-op IEEE sequence.
// Valid for normal, finite x (the P-tile maxima and scales they are used on).
__device__ __forceinline__ float div127_fast(float x) {
    const float r = 1.0f / 127.0f;
    const float q = x * r;
    return fmaf(fmaf(-q, 127.0f, x), r, q);
}
__device__ __forceinline__ float rcp_fast(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    return fmaf(fmaf(-x, r, 1.0f), r, r);
}

// Balanced-tree reductions of 16 register values (independent chains for ILP).
// 16 values in 8 v_max3 / v_max (5 + 2 + 1)
__device__ __forceinline__ int tree_max16_i(const v16i& s) {
    int a = max(max(s[0], s[1]), s[2]), b = max(max(s[3], s[4]), s[5]);
    int c = max(max(s[6], s[7]), s[8]), d = max(max(s[9], s[10]), s[11]);
    int e = max(max(s[12], s[13]), s[14]);
    return max(max(max(a, b), c), max(max(d, e), (int)s[15]));
}
__device__ __forceinline__ float tree_sum16(const float* p) {
    float a = (p[0] + p[1]) + (p[2] + p[3]), b = (p[4] + p[5]) + (p[6] + p[7]);
    float c = (p[8] + p[9]) + (p[10] + p[11]), d = (p[12] + p[13]) + (p[14] + p[15]);
    return (a + b) + (c + d);
}

// Round-half-even of a non-negative x < 2^22 into the low mantissa bits:
// fma(p, inv, 1.5 * 2^23) is exactly rint(p*inv) + 1.5*2^23.
#define QMHA_MAGIC_RNE 12582912.0f

__device__ __forceinline__ uint32_t pack4_lowbytes(float a, float b, float c, float d) {
    uint32_t t01 = __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x0c0c0400u);
    uint32_t t23 = __builtin_amdgcn_perm(__float_as_uint(d), __float_as_uint(c), 0x0c0c0400u);
    return __builtin_amdgcn_perm(t23, t01, 0x05040100u);
}

// Workgroup barrier after LDS-DMA (global_load_lds): every wave first drains its own DMA
// (vmcnt(0)) so that after the barrier all waves see the whole stage in LDS.  __syncthreads()
// alone is not enough: the compiler may drop the vmcnt wait before s_barrier when no LDS read
// of the issuing wave depends on it (observed in the pipelined int8 kernel -> a cross-wave race).
__device__ __forceinline__ void qmha_dma_barrier() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// XCD-aware remap of a linear workgroup id: the dispatcher deals ids round-robin over the
// 8 XCDs, so give each XCD a contiguous range of work items (consecutive q-blocks of the
// same head share K/V in that XCD's L2).  Bijective for any nwg (cdna guide T1).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    const int q = nwg / 8, r = nwg % 8;
    const int xcd = orig % 8, slot = orig / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + slot;
}

// --------------------------------------------------------------------------
// Pre-pass writer of one 32-row group of V as the f16 V^T MFMA operand ([D][32 slots] f16, kv
// slots in kv_of_slot_f16 order), shared by the int8 (QUANT: the quantised integers) and the
// fp16 (RNE f16 values) pre-passes.  Lane (rq, c4) = (lane / (D/4), lane % (D/4)) holds the
// D/8 CONSECUTIVE rows rq*D/8 .. of columns 4 c4 .. 4 c4 + 3 (x[i] = row rq*D/8 + i), loaded
// as coalesced 16-byte pieces.  Consecutive kv rows 4a..4a+3 are 4 consecutive slots, so each
// column goes to this wave's LDS tile T (D rows of PITCH bytes) as 8-byte pieces; the tile is
// read back in 8-byte pieces and stored to dst as whole 16-byte lines.
// --------------------------------------------------------------------------
// The 8-byte chunks of LDS row d are XOR-swizzled by (d >> 4) & 7: the 16 lanes of a ds_write_b64
// lane group write 16 rows d = 4 c4 + c (stride 4 rows = 72 dwords = bank +8), which without the
// swizzle hit only 4 bank pairs (4-way conflict; r02 PMC: SQ_LDS_BANK_CONFLICT 4.19 M of 6.29 M
// LDS-active cycles in the int8 pre-pass); with it the writes are conflict-free for d = 32/64/128
// (tools/lds_banks.py models both sides; the 8-byte read-back stays at its 2-way floor).
constexpr int QMHA_VT_PITCH = 64 + 8;  // bytes per d-row of the LDS tile (8-byte pad)
__device__ __forceinline__ int vt_chunk_swz(int d) { return (d >> 4) & 7; }
// The two halves of vt_group_store: vt_tile_write puts hf(a, c) -- this lane's four f16 values of column
// 4 c4 + c, kv rows NI rq + 4a .. +3 (one 8-byte chunk) -- into the wave's LDS tile; vt_tile_store reads the
// tile back as 16-byte lines and stores them to dst (a caller may rewrite the tile in between).
template <int D, class HF>
__device__ __forceinline__ void vt_tile_write(char* T, int lane, HF&& hf) {
    constexpr int C4 = D / 4, NI = D / 8;
    const int rq = lane / C4, c4 = lane % C4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int d = 4 * c4 + c;
#pragma unroll
        for (int a = 0; a < NI / 4; ++a) {  // kv rows NI rq + 4a .. +3 -> 4 consecutive slots (one 8-byte chunk)
            const int chunk = slot_of_kv_f16(NI * rq + 4 * a) >> 2;
            *reinterpret_cast<v4h*>(T + d * QMHA_VT_PITCH + 8 * (chunk ^ vt_chunk_swz(d))) = hf(a, c);
        }
    }
}
template <int D>
__device__ __forceinline__ void vt_tile_store(const char* T, int lane, char* dst) {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    constexpr int LINES = D * 64 / 16;  // 16-byte output lines of the group
#pragma unroll
    for (int u = lane; u < LINES; u += 64) {
        const int d = u >> 2, q = u & 3;
        const v2i lo = *reinterpret_cast<const v2i*>(T + d * QMHA_VT_PITCH + 8 * ((2 * q) ^ vt_chunk_swz(d)));
        const v2i hi = *reinterpret_cast<const v2i*>(T + d * QMHA_VT_PITCH + 8 * ((2 * q + 1) ^ vt_chunk_swz(d)));
        *reinterpret_cast<v4i*>(dst + 16 * u) = v4i{lo[0], lo[1], hi[0], hi[1]};
    }
}
template <int D, bool QUANT>
__device__ __forceinline__ void vt_group_store(char* T, const v4f (&x)[D / 8], float inv, int lane, char* dst) {
    vt_tile_write<D>(T, lane, [&](int a, int c) {
        v4h h;
#pragma unroll
        for (int e = 0; e < 4; ++e) h[e] = QUANT ? (_Float16)qmha_quant_i8(x[4 * a + e][c], inv) : (_Float16)x[4 * a + e][c];
        return h;
    });
    vt_tile_store<D>(T, lane, dst);
}

// The same for the int8 V^T operand ([D][32 slots] bytes, kv_of_slot_i8 order; the standalone
// qmha_quantize_int8 layout 1): four consecutive kv rows are four consecutive slots, so a lane
// packs its 4-row runs of one column into one dword (ds_write_b32 instead of byte stores).
constexpr int QMHA_VT8_PITCH = 32 + 4;  // bytes per d-row of the int8 LDS tile
template <int D>
__device__ __forceinline__ void vt8_group_store(char* T, const v4f (&x)[D / 8], float inv, int lane, char* dst) {
    constexpr int C4 = D / 4, NI = D / 8;
    const int rq = lane / C4, c4 = lane % C4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int d = 4 * c4 + c;
#pragma unroll
        for (int a = 0; a < NI / 4; ++a) {  // kv rows NI rq + 4a .. +3 -> 4 consecutive slots
            uint32_t w = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) w |= ((uint32_t)(uint8_t)qmha_quant_i8(x[4 * a + e][c], inv)) << (8 * e);
            *reinterpret_cast<uint32_t*>(T + d * QMHA_VT8_PITCH + slot_of_kv_i8(NI * rq + 4 * a)) = w;
        }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    constexpr int LINES = D * 32 / 16;  // 16-byte output lines of the group
#pragma unroll
    for (int u = lane; u < LINES; u += 64) {
        const int d = u >> 1, q = u & 1;
        const uint32_t* r = reinterpret_cast<const uint32_t*>(T + d * QMHA_VT8_PITCH + 16 * q);
        *reinterpret_cast<v4i*>(dst + 16 * u) = v4i{(int)r[0], (int)r[1], (int)r[2], (int)r[3]};
    }
}
