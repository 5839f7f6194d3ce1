// qmha_api.cpp -- the C-ABI (include/launchers.h): argument checks, workspace ownership,
// variant dispatch, profiling hooks.  Replaces the reference's launch<KernelFn> per-head
// slicer (include/launchers.h:16-72): no per-call cudaMalloc/cudaFree, no extract/concat
// copies (kernels read and write the strided [N, d_model] head slices directly), all B*H
// heads in one grid, and errors are reported instead of ignored.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/launchers.h"
#include "qmha_kernels.hpp"

#define QMHA_VERSION_STRING "qmha-mi355x 0.1.0 (gfx950)"

namespace {

thread_local std::string g_last_error;

int hip_fail(hipError_t e, const char* what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return QMHA_ERR_HIP;
}

#define QMHA_HIP_TRY(expr, what)                 \
    do {                                         \
        hipError_t _e = (expr);                  \
        if (_e != hipSuccess) return hip_fail(_e, what); \
    } while (0)

int check_shape(const void* Q, const void* K, const void* V, const void* O, int B, int N, int d_model, int h,
                int variant, int* D_out) {
    if (!Q || !K || !V || !O) {
        g_last_error = "null tensor pointer";
        return QMHA_ERR_INVALID;
    }
    if (B < 1 || N < 1 || d_model < 1 || h < 1) {
        g_last_error = "B, N, d_model and h must be positive";
        return QMHA_ERR_INVALID;
    }
    if (d_model % h != 0) {  // config.h:27
        g_last_error = "d_model must be divisible by h";
        return QMHA_ERR_INVALID;
    }
    if (N % 32 != 0) {  // fa_tc_int8_b.cu:422-423 (N % Br), Br = Bc = 32
        g_last_error = "N must be a multiple of 32";
        return QMHA_ERR_INVALID;
    }
    const int D = d_model / h;
    if (variant < QMHA_FA || variant > QMHA_FA_TC_INT8_PT) {
        g_last_error = "unknown variant";
        return QMHA_ERR_INVALID;
    }
    if (D % 32 != 0) {  // config.h:32: static_assert(d % 32 == 0)
        g_last_error = "head size d = d_model/h must be a multiple of 32";
        return QMHA_ERR_INVALID;
    }
    if (D > 256) {  // the reference has no upper bound; here the int8 magic-biased accumulator's range
        g_last_error = "head size d = d_model/h above 256 is not built";
        return QMHA_ERR_NOSYS;
    }
    if (variant == QMHA_FA_TC_INT8_PT && D != 32 && D != 64 && D != 128) {  // no reference counterpart
        g_last_error = "fa_tc_int8_pt is built for d = 32, 64, 128 only";
        return QMHA_ERR_NOSYS;
    }
    if ((size_t)B * N * d_model > (size_t)INT32_MAX * 4) {
        g_last_error = "tensor too large";
        return QMHA_ERR_INVALID;
    }
    *D_out = D;
    return QMHA_OK;
}

// ---- profiling --------------------------------------------------------------------------
// Per call: event pairs around every pre-pass launch (on the pre-pass stream) and every main
// launch (on the caller's stream); qmha_profile_collect sums them per call.
struct ProfRec {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pre, main;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRec> g_prof_recs;
std::vector<hipEvent_t> g_event_pool;

hipEvent_t take_event() {
    if (!g_event_pool.empty()) {
        hipEvent_t e = g_event_pool.back();
        g_event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// ---- pre-pass / main-kernel overlap (int8 and fp16 paths) ------------------------------
// The HBM-bound pre-pass (quantise / convert) of batch chunk c+1 runs on a library-owned
// second stream while the compute-bound main kernel of chunk c runs on the caller's stream.
// Chunks are disjoint slices of the same workspace arrays, so only "pre(c) before main(c)"
// and "previous call done before pre(0)" need ordering.  QMHA_OVERLAP_CHUNKS (default 1 =
// off: measured slower at C4, the co-running pre-pass slows the main kernel more than it hides,
// profiles/r01/overlap_sweep.txt) sets the number of chunks.
struct SideStream {
    hipStream_t s = nullptr;
    hipEvent_t start = nullptr;
    std::vector<hipEvent_t> ready;
};
std::mutex g_side_mu;
std::map<std::tuple<int, void*, std::thread::id>, SideStream> g_side;  // keyed like the workspace slots

std::atomic<int> g_overlap_chunks{-1};  // -1: not yet read from QMHA_OVERLAP_CHUNKS

int overlap_chunks(int B) {
    int c = g_overlap_chunks.load();
    if (c < 0) {
#ifdef QMHA_ABLATION  // profiling builds: QMHA_OVERLAP_CHUNKS sets the default (production: the API only)
        const char* e = std::getenv("QMHA_OVERLAP_CHUNKS");
        c = e ? std::atoi(e) : 1;
#else
        c = 1;
#endif
        c = c < 1 ? 1 : (c > 16 ? 16 : c);
        g_overlap_chunks.store(c);
    }
    return c > B ? B : c;
}

int get_side(hipStream_t stream, int nchunks, SideStream** out) {
    int dev = 0;
    QMHA_HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    std::lock_guard<std::mutex> lk(g_side_mu);
    SideStream& ss = g_side[{dev, (void*)stream, stream == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id()}];
    if (!ss.s) {
        QMHA_HIP_TRY(hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking), "hipStreamCreate");
        QMHA_HIP_TRY(hipEventCreateWithFlags(&ss.start, hipEventDisableTiming), "hipEventCreate");
    }
    while ((int)ss.ready.size() < nchunks) {
        hipEvent_t e = nullptr;
        QMHA_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        ss.ready.push_back(e);
    }
    *out = &ss;
    return QMHA_OK;
}

// ---- library-owned workspaces, one per (device, stream) --------------------------------
// Threading contract: any number of host threads may call every entry point at once.
// The reference gets that from per-call cudaMalloc'd scratch and private streams (include/launchers.h:
// 27-33, freed at :64-71); here the scratch is cached, so a call LEASES its (device, stream) slot: the
// slot's mutex is held from the moment the buffer is handed out until the call's last kernel that uses
// it has been enqueued.  Calls on one stream therefore enqueue one whole call after another (pre-pass and
// main kernel of a call are never separated by another call's pre-pass), and the stream runs them in that
// order.  Calls on different streams use different slots.  hipStreamPerThread names a different stream
// in every thread, so its slot key carries the thread id.  A slot that must grow never frees the buffer
// other enqueued work may still read: the old buffer is retired behind an event recorded on the slot's
// stream and freed once that event has completed (checked at the slot's next lease, or at release).
struct WsKey {
    int dev;
    void* stream;
    std::thread::id tid;  // hipStreamPerThread only
    bool operator<(const WsKey& o) const {
        if (dev != o.dev) return dev < o.dev;
        if (stream != o.stream) return stream < o.stream;
        return tid < o.tid;
    }
};
struct WsSlot {
    std::mutex lease;  // held across a call's enqueue
    void* ptr = nullptr;
    size_t bytes = 0;
    std::vector<std::pair<void*, hipEvent_t>> retired;  // grown-out buffers, freed once their event completed
};
std::mutex g_ws_mu;  // guards the map only (slots are never erased while the library is in use)
std::map<WsKey, std::unique_ptr<WsSlot>> g_ws;

// free the retired buffers whose last reader has completed (all when `wait`); caller holds the lease
void reap_retired(WsSlot& s, bool wait) {
    auto it = s.retired.begin();
    while (it != s.retired.end()) {
        if (wait) (void)hipEventSynchronize(it->second);
        else if (hipEventQuery(it->second) != hipSuccess) {
            ++it;
            continue;
        }
        (void)hipEventDestroy(it->second);
        (void)hipFree(it->first);
        it = s.retired.erase(it);
    }
}

// A held workspace: the buffer stays this call's until the lease is destroyed (after the last enqueue).
struct WsLease {
    std::unique_lock<std::mutex> lk;
    void* ptr = nullptr;
};

int lease_workspace(size_t need, hipStream_t stream, WsLease* out) {
    out->ptr = nullptr;
    int dev = 0;
    QMHA_HIP_TRY(hipGetDevice(&dev), "hipGetDevice");
    WsSlot* slot;
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        const WsKey key{dev, (void*)stream, stream == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id()};
        std::unique_ptr<WsSlot>& sp = g_ws[key];
        if (!sp) sp.reset(new WsSlot);
        slot = sp.get();
    }
    out->lk = std::unique_lock<std::mutex>(slot->lease);
    WsSlot& s = *slot;
    if (!s.retired.empty()) reap_retired(s, false);
    if (need == 0) return QMHA_OK;
    if (s.bytes < need) {
        if (s.ptr) {
            // work already enqueued on this stream may still read the old buffer: retire it behind an event
            hipEvent_t ev = nullptr;
            QMHA_HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
            const hipError_t e = hipEventRecord(ev, stream);
            if (e != hipSuccess) {
                (void)hipEventDestroy(ev);
                return hip_fail(e, "hipEventRecord");
            }
            s.retired.emplace_back(s.ptr, ev);
            s.ptr = nullptr;
            s.bytes = 0;
        }
        const size_t alloc = qmha::align_up(need + need / 8, 1 << 20);
        if (hipMalloc(&s.ptr, alloc) != hipSuccess) {
            s.ptr = nullptr;
            g_last_error = "hipMalloc of workspace failed";
            return QMHA_ERR_NOMEM;
        }
        s.bytes = alloc;
    }
    out->ptr = s.ptr;
    return QMHA_OK;
}

size_t workspace_bytes(int B, int N, int H, int D, int variant) {
    switch (variant) {
        case QMHA_FA_TC_INT8_B: return qmha::int8_workspace_bytes(B, N, H, D);
        case QMHA_FA_TC_INT8_PT: return qmha::int8_pt_workspace_bytes(B, N, H, D);
        case QMHA_FA_TC_V1A: return qmha::f16_workspace_bytes(B, N, H, D);
        case QMHA_UNFUSED: return qmha::unfused_workspace_bytes(B, N, H, D);
        default: return 0;
    }
}

qmha::Int8Workspace int8_slice(const qmha::Int8Workspace& w, size_t b0, int N, int H, int D) {
    const size_t e = b0 * H * N * D, g = b0 * H * (N / 32);  // 32-row quantisation groups
    return qmha::Int8Workspace{nullptr, w.Ki + e, w.Vh + e, nullptr, w.sK + g, w.sV + g};
}
qmha::F16Workspace f16_slice(const qmha::F16Workspace& w, size_t b0, int N, int H, int D) {
    const size_t e = b0 * H * N * D;
    return qmha::F16Workspace{nullptr, w.Kh + e, w.Vt + e};
}

int run(const float* Q, const float* K, const float* V, float* O, int B, int N, int d_model, int h, int variant,
        void* ws, size_t ws_bytes, hipStream_t stream) {
    const int D = d_model / h;
    const size_t need = workspace_bytes(B, N, h, D, variant);
    if (ws_bytes < need) {
        g_last_error = "workspace too small";
        return QMHA_ERR_INVALID;
    }
    bool prof;
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        prof = g_prof_on;
    }
    ProfRec rec;
    auto mark = [&](std::vector<std::pair<hipEvent_t, hipEvent_t>>& v, hipStream_t s, bool begin) -> int {
        if (!prof) return QMHA_OK;
        hipEvent_t e;
        {
            std::lock_guard<std::mutex> lk(g_prof_mu);
            e = take_event();
        }
        if (!e) {
            g_last_error = "hipEventCreate failed";
            return QMHA_ERR_HIP;
        }
        if (begin) v.push_back({e, nullptr});
        else v.back().second = e;
        QMHA_HIP_TRY(hipEventRecord(e, s), "hipEventRecord");
        return QMHA_OK;
    };
#define QMHA_MARK(vec, s, begin)                       \
    do {                                               \
        int _st = mark(vec, s, begin);                 \
        if (_st != QMHA_OK) return _st;                \
    } while (0)

    if (variant == QMHA_FA_TC_INT8_B || variant == QMHA_FA_TC_V1A) {
        const size_t slab = (size_t)N * d_model;  // floats per sequence
        const int nc = overlap_chunks(B);
        SideStream* side = nullptr;
        if (nc > 1) {
            int st = get_side(stream, nc, &side);
            if (st != QMHA_OK) return st;
            QMHA_HIP_TRY(hipEventRecord(side->start, stream), "hipEventRecord");
            QMHA_HIP_TRY(hipStreamWaitEvent(side->s, side->start, 0), "hipStreamWaitEvent");
        }
        const hipStream_t pre_s = nc > 1 ? side->s : stream;
        const qmha::Int8Workspace w8 = variant == QMHA_FA_TC_INT8_B ? qmha::int8_carve(ws, B, N, h, D) : qmha::Int8Workspace{};
        const qmha::F16Workspace w16 = variant == QMHA_FA_TC_V1A ? qmha::f16_carve(ws, B, N, h, D) : qmha::F16Workspace{};
        // every pre-pass is enqueued first (the side stream runs ahead), then the main kernels
        for (int c = 0; c < nc; ++c) {
            const int b0 = (int)((long long)B * c / nc), b1 = (int)((long long)B * (c + 1) / nc), nb = b1 - b0;
            QMHA_MARK(rec.pre, pre_s, true);
            if (variant == QMHA_FA_TC_INT8_B) {
                const qmha::Int8Workspace w = int8_slice(w8, b0, N, h, D);
                QMHA_HIP_TRY(qmha::launch_quant_int8(Q + b0 * slab, K + b0 * slab, V + b0 * slab, w, w.Vh, /*v_mode=*/1, nb, N, h, D,
                                                     d_model, pre_s, /*first_tensor=*/1), "quant_int8 launch");
            } else {
                QMHA_HIP_TRY(qmha::launch_convert_f16(Q + b0 * slab, K + b0 * slab, V + b0 * slab, f16_slice(w16, b0, N, h, D),
                                                      nb, N, h, D, d_model, pre_s), "convert_f16 launch");
            }
            QMHA_MARK(rec.pre, pre_s, false);
            if (nc > 1) QMHA_HIP_TRY(hipEventRecord(side->ready[c], pre_s), "hipEventRecord");
        }
        for (int c = 0; c < nc; ++c) {
            const int b0 = (int)((long long)B * c / nc), b1 = (int)((long long)B * (c + 1) / nc), nb = b1 - b0;
            if (nc > 1) QMHA_HIP_TRY(hipStreamWaitEvent(stream, side->ready[c], 0), "hipStreamWaitEvent");
            QMHA_MARK(rec.main, stream, true);
            if (variant == QMHA_FA_TC_INT8_B) {
                QMHA_HIP_TRY(qmha::launch_fa_int8_main(int8_slice(w8, b0, N, h, D), Q + b0 * slab, O + b0 * slab, nb, N, h, D,
                                                       d_model, stream), "fa_int8 launch");
            } else {
                QMHA_HIP_TRY(qmha::launch_fa_f16_main(f16_slice(w16, b0, N, h, D), Q + b0 * slab, O + b0 * slab, nb, N, h, D,
                                                      d_model, stream), "fa_f16 launch");
            }
            QMHA_MARK(rec.main, stream, false);
        }
    } else if (variant == QMHA_FA_TC_INT8_PT) {
        // per-tensor mode: group absmax of Q, K, V + K/V quantisation with the head-slice scales
        // (two pre-pass launches), then the main kernel (Q quantised in registers)
        const qmha::Int8Workspace w = qmha::int8_pt_carve(ws, B, N, h, D);
        QMHA_MARK(rec.pre, stream, true);
        QMHA_HIP_TRY(qmha::launch_quant_int8_pt(Q, K, V, w, B, N, h, D, d_model, stream), "quant_int8_pt launch");
        QMHA_MARK(rec.pre, stream, false);
        QMHA_MARK(rec.main, stream, true);
        QMHA_HIP_TRY(qmha::launch_fa_int8_pt_main(w, Q, O, B, N, h, D, d_model, stream), "fa_int8_pt launch");
        QMHA_MARK(rec.main, stream, false);
    } else if (variant == QMHA_FA || variant == QMHA_FA_MFMA) {
        QMHA_MARK(rec.main, stream, true);
        QMHA_HIP_TRY(qmha::launch_fa_f32(Q, K, V, O, B, N, h, D, d_model, variant == QMHA_FA_MFMA, stream),
                     "fa_f32 launch");
        QMHA_MARK(rec.main, stream, false);
    } else if (variant == QMHA_UNFUSED) {
        QMHA_MARK(rec.main, stream, true);
        QMHA_HIP_TRY(qmha::launch_unfused(Q, K, V, O, ws, B, N, h, D, d_model, stream), "unfused launch");
        QMHA_MARK(rec.main, stream, false);
    } else {
        g_last_error = "unknown variant";
        return QMHA_ERR_INVALID;
    }
#undef QMHA_MARK
    if (prof) {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        g_prof_recs.push_back(std::move(rec));
    }
    return QMHA_OK;
}

}  // namespace

int qmha::tune_config(const char* env_name) {
    static std::mutex mu;
    static std::map<std::string, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(env_name);
    if (it != cache.end()) return it->second;
    int v = 0;
    if (const char* e = std::getenv(env_name)) {
        int w = 0, sg = 0;
        if (std::sscanf(e, "%dx%d", &w, &sg) == 2 && w > 0 && w < 10 && sg > 0 && sg < 10) {
            v = w * 10 + sg;  // "WAVESxSG"
        } else if (std::sscanf(e, "%d", &w) == 1 && w > 0) {
            v = w;  // a kernel-specific numeric geometry code
        }
    }
    cache[env_name] = v;
    return v;
}

extern "C" {

int qmha_solve_ws(const float* Q, const float* K, const float* V, float* O, int B, int N, int d_model, int h,
                  int variant, void* workspace, size_t workspace_bytes_, void* stream) {
    int D = 0;
    int st = check_shape(Q, K, V, O, B, N, d_model, h, variant, &D);
    if (st != QMHA_OK) return st;
    return run(Q, K, V, O, B, N, d_model, h, variant, workspace, workspace_bytes_, (hipStream_t)stream);
}

int qmha_solve_ex(const float* Q, const float* K, const float* V, float* O, int B, int N, int d_model, int h,
                  int variant, void* stream) {
    int D = 0;
    int st = check_shape(Q, K, V, O, B, N, d_model, h, variant, &D);
    if (st != QMHA_OK) return st;
    const size_t need = workspace_bytes(B, N, h, D, variant);
    WsLease ws;  // held until every kernel of this call is enqueued
    st = lease_workspace(need, (hipStream_t)stream, &ws);
    if (st != QMHA_OK) return st;
    return run(Q, K, V, O, B, N, d_model, h, variant, ws.ptr, need, (hipStream_t)stream);
}

size_t qmha_workspace_size(int B, int N, int d_model, int h, int variant) {
    if (B < 1 || N < 1 || h < 1 || d_model % h) return 0;
    return workspace_bytes(B, N, h, d_model / h, variant);
}

int qmha_solve_variant(const float* Q, const float* K, const float* V, float* O, int N, int d_model, int h,
                       int variant) {
    // blocking like the reference (launchers.h:64): hipStreamSynchronize.  r04 A/B: polling
    // hipStreamQuery was slower (profiles/r04/ab_sync/summary.txt); r05's spin on a stream-ordered host
    // flag saved ~1 us per call (profiles/r05/ab_solve_sync/) but pinned a host word per thread and a CPU
    // core per waiting thread, so r06 returned to the runtime's synchronisation (round-5 ADVICE)
    int st = qmha_solve_ex(Q, K, V, O, 1, N, d_model, h, variant, nullptr);
    if (st != QMHA_OK) return st;
    QMHA_HIP_TRY(hipStreamSynchronize(nullptr), "solve: hipStreamSynchronize");
    return QMHA_OK;
}

int qmha_quantize_int8(const float* X, int B, int N, int d_model, int h, int8_t* Xi, float* scales, int layout,
                       void* stream) {
    int D = 0;
    int st = check_shape(X, X, X, Xi, B, N, d_model, h, QMHA_FA_TC_INT8_B, &D);
    if (st != QMHA_OK) return st;
    if (!scales || layout < 0 || layout > 2) {
        g_last_error = "bad scales pointer or layout";
        return QMHA_ERR_INVALID;
    }
    if (layout == 2 && D != 32 && D != 64 && D != 128) {  // the per-tensor mode's quantiser
        g_last_error = "layout 2 (per-tensor scales) is built for d = 32, 64, 128 only";
        return QMHA_ERR_NOSYS;
    }
    if (layout == 2) {  // per-tensor (head-slice) scales: the single-read pass (slice counters in a workspace)
        const size_t need = qmha::align_up((size_t)6 * B * h * sizeof(uint32_t), 256);
        WsLease ws;  // held until the pass is enqueued
        st = lease_workspace(need, (hipStream_t)stream, &ws);
        if (st != QMHA_OK) return st;
        qmha::Int8Workspace w{};
        w.Ki = Xi;  // the K role: int8 rows
        w.sK = scales;
        w.slice_sync = static_cast<uint32_t*>(ws.ptr);
        QMHA_HIP_TRY(qmha::launch_quant_int8_pt_rows(X, w, B, N, h, D, d_model, (hipStream_t)stream), "quant_int8_pt launch");
        return QMHA_OK;
    }
    // The pre-pass kernel with X in one role only: the Q role (row layout) or the V role (the
    // V^T operand order); nothing else is written, no workspace is needed.
    qmha::Int8Workspace w{};
    void* vout = nullptr;
    int v_mode = 1, role = 0;
    if (layout == 0) {
        w.Qi = Xi;
        w.sQ = scales;
    } else {
        vout = Xi;
        v_mode = 0;
        w.sV = scales;
        role = 2;
    }
    QMHA_HIP_TRY(qmha::launch_quant_int8(X, X, X, w, vout, v_mode, B, N, h, D, d_model, (hipStream_t)stream, role, 1),
                 "quant_int8 launch");
    return QMHA_OK;
}

int qmha_debug_qk_int32(const float* Q, const float* K, int N, int d_model, int h, int head, int32_t* S) {
    int D = 0;
    int st = check_shape(Q, K, Q, S, 1, N, d_model, h, QMHA_FA_TC_INT8_B, &D);
    if (st != QMHA_OK) return st;
    if (head < 0 || head >= h) {
        g_last_error = "head out of range";
        return QMHA_ERR_INVALID;
    }
    const size_t need = qmha::int8_workspace_bytes(1, N, h, D, /*with_q=*/true);
    WsLease lease;
    st = lease_workspace(need, nullptr, &lease);
    if (st != QMHA_OK) return st;
    void* ws = lease.ptr;
    qmha::Int8Workspace w = qmha::int8_carve(ws, 1, N, h, D, /*with_q=*/true);
    QMHA_HIP_TRY(qmha::launch_quant_int8(Q, K, Q, w, w.Vh, 1, 1, N, h, D, d_model, nullptr), "quant_int8 launch");
    QMHA_HIP_TRY(qmha::launch_debug_qk_int32(w, N, D, head, S, nullptr), "debug_qk launch");
    lease.lk.unlock();
    QMHA_HIP_TRY(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
    return QMHA_OK;
}

int qmha_debug_fa_int8_dump(const float* Q, const float* K, const float* V, float* O, int B, int N, int d_model,
                            int h, int32_t* S, int8_t* Qi, float* sQ) {
    int D = 0;
    int st = check_shape(Q, K, V, O, B, N, d_model, h, QMHA_FA_TC_INT8_B, &D);
    if (st != QMHA_OK) return st;
    if (!S || !Qi || !sQ || ((D == 32 || D == 64 || D == 128) && N < 64)) {
        g_last_error = "debug dump: needs S/Qi/sQ buffers and, at d = 32 / 64 / 128, N >= 64 (the pipelined kernel)";
        return QMHA_ERR_INVALID;
    }
    const size_t need = qmha::int8_workspace_bytes(B, N, h, D);
    WsLease lease;
    st = lease_workspace(need, nullptr, &lease);
    if (st != QMHA_OK) return st;
    void* ws = lease.ptr;
    const qmha::Int8Workspace w = qmha::int8_carve(ws, B, N, h, D);
    QMHA_HIP_TRY(qmha::launch_quant_int8(Q, K, V, w, w.Vh, /*v_mode=*/1, B, N, h, D, d_model, nullptr, /*first_tensor=*/1),
                 "quant_int8 launch");
    QMHA_HIP_TRY(qmha::launch_fa_int8_dump(w, Q, O, B, N, h, D, d_model, qmha::QkDump{S, Qi, sQ}, nullptr),
                 "fa_int8 dump launch");
    lease.lk.unlock();
    QMHA_HIP_TRY(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
    return QMHA_OK;
}

int qmha_debug_fa_int8_pt_dump(const float* Q, const float* K, const float* V, float* O, int B, int N, int d_model,
                               int h, int32_t* S, int8_t* Qi, float* sQ) {
    int D = 0;
    int st = check_shape(Q, K, V, O, B, N, d_model, h, QMHA_FA_TC_INT8_PT, &D);
    if (st != QMHA_OK) return st;
    if (!S || !Qi || !sQ) {
        g_last_error = "debug dump: needs S/Qi/sQ buffers";
        return QMHA_ERR_INVALID;
    }
    const size_t need = qmha::int8_pt_workspace_bytes(B, N, h, D);
    WsLease lease;
    st = lease_workspace(need, nullptr, &lease);
    if (st != QMHA_OK) return st;
    void* ws = lease.ptr;
    const qmha::Int8Workspace w = qmha::int8_pt_carve(ws, B, N, h, D);
    QMHA_HIP_TRY(qmha::launch_quant_int8_pt(Q, K, V, w, B, N, h, D, d_model, nullptr), "quant_int8_pt launch");
    QMHA_HIP_TRY(qmha::launch_fa_int8_pt_dump(w, Q, O, B, N, h, D, d_model, qmha::QkDump{S, Qi, sQ}, nullptr),
                 "fa_int8_pt dump launch");
    lease.lk.unlock();
    QMHA_HIP_TRY(hipStreamSynchronize(nullptr), "hipStreamSynchronize");
    return QMHA_OK;
}

int qmha_variant_from_name(const char* name) {
    if (!name) return -1;
    if (!std::strcmp(name, "fa")) return QMHA_FA;
    if (!std::strcmp(name, "fa_tc_v1a")) return QMHA_FA_TC_V1A;
    if (!std::strcmp(name, "fa_tc_int8_b")) return QMHA_FA_TC_INT8_B;
    if (!std::strcmp(name, "unfused")) return QMHA_UNFUSED;
    if (!std::strcmp(name, "fa_mfma")) return QMHA_FA_MFMA;
    if (!std::strcmp(name, "fa_tc_int8_pt")) return QMHA_FA_TC_INT8_PT;
    return -1;
}

const char* qmha_variant_name(int v) {
    switch (v) {
        case QMHA_FA: return "fa";
        case QMHA_FA_TC_V1A: return "fa_tc_v1a";
        case QMHA_FA_TC_INT8_B: return "fa_tc_int8_b";
        case QMHA_UNFUSED: return "unfused";
        case QMHA_FA_MFMA: return "fa_mfma";
        case QMHA_FA_TC_INT8_PT: return "fa_tc_int8_pt";
        default: return "unknown";
    }
}

const char* qmha_status_string(int s) {
    switch (s) {
        case QMHA_OK: return "ok";
        case QMHA_ERR_INVALID: return "invalid argument";
        case QMHA_ERR_HIP: return "HIP error";
        case QMHA_ERR_NOMEM: return "out of device memory";
        case QMHA_ERR_NOSYS: return "not supported";
        default: return "unknown status";
    }
}

const char* qmha_version(void) { return QMHA_VERSION_STRING; }

const char* qmha_last_error(void) { return g_last_error.c_str(); }

int64_t qmha_debug_set_pt_wait(int64_t ticks) { return qmha::set_pt_wait_ticks(ticks); }

int qmha_set_overlap_chunks(int n) {
    const int prev = overlap_chunks(1 << 30);
    g_overlap_chunks.store(n < 1 ? 1 : (n > 16 ? 16 : n));
    return prev;
}

void qmha_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof_on = on != 0;
}

int qmha_profile_collect(double* main_ms, long long* launches, double* prepass_ms) {
    std::vector<ProfRec> recs;
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        recs.swap(g_prof_recs);
    }
    double tm = 0.0, tp = 0.0;
    for (auto& r : recs) {
        for (auto* v : {&r.main, &r.pre}) {
            for (auto& pr : *v) {
                QMHA_HIP_TRY(hipEventSynchronize(pr.second), "hipEventSynchronize");
                float a = 0.0f;
                QMHA_HIP_TRY(hipEventElapsedTime(&a, pr.first, pr.second), "hipEventElapsedTime");
                (v == &r.main ? tm : tp) += a;
            }
        }
    }
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        for (auto& r : recs)
            for (auto* v : {&r.main, &r.pre})
                for (auto& pr : *v) {
                    g_event_pool.push_back(pr.first);
                    g_event_pool.push_back(pr.second);
                }
    }
    if (main_ms) *main_ms = tm;
    if (prepass_ms) *prepass_ms = tp;
    if (launches) *launches = (long long)recs.size();
    return QMHA_OK;
}

void qmha_release_workspaces(void) {
    {
        std::lock_guard<std::mutex> lk(g_side_mu);
        for (auto& kv : g_side) {
            (void)hipStreamSynchronize(kv.second.s);
            for (hipEvent_t e : kv.second.ready) (void)hipEventDestroy(e);
            (void)hipEventDestroy(kv.second.start);
            (void)hipStreamDestroy(kv.second.s);
        }
        g_side.clear();
    }
    // each slot under its lease: a call still enqueueing on it finishes first; the buffers are freed
    // after the device has drained (work on any stream may still read them)
    std::lock_guard<std::mutex> lk(g_ws_mu);
    for (auto& kv : g_ws) {
        WsSlot& s = *kv.second;
        std::lock_guard<std::mutex> lease(s.lease);
        (void)hipDeviceSynchronize();
        reap_retired(s, true);
        if (s.ptr) (void)hipFree(s.ptr);
        s.ptr = nullptr;
        s.bytes = 0;
    }
}

#ifndef QMHA_NO_DEFAULT_SOLVE
// libqmha.so's `solve` = the north-star drop-in target, fa_tc_int8_b.
void solve(const float* Q, const float* K, const float* V, float* output, int N, int d_model, int h) {
    int st = qmha_solve_variant(Q, K, V, output, N, d_model, h, QMHA_FA_TC_INT8_B);
    if (st != QMHA_OK) std::fprintf(stderr, "qmha solve(fa_tc_int8_b): %s: %s\n", qmha_status_string(st), qmha_last_error());
}
#endif

}  // extern "C"
