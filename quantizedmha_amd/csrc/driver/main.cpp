// main.cpp -- HIP C++ host driver / profiling harness (reference drivers/main.cu:38-157).
//
// Same flow and flags as the reference: an all-ones correctness check against the cached
// CPU reference (RoPE, utils/verify.cu), then warmup + timed runs on cached mt19937(42)
// U[0,1) inputs.  Differences, all additive: the kernel is chosen at run time (--kernel
// is honoured instead of ignored), the problem size is a run-time argument instead of
// config.h, runs are timed with hipEvents (the reference relied on an external profiler),
// --check-random compares random-data output with plain CPU attention, and --json prints
// one summary line.  The kernels are reached only through the C-ABI (include/launchers.h).
#include <hip/hip_runtime.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/launchers.h"
#include "data.h"
#include "verify.h"

using namespace qmha_driver;

#define DRV_CHECK(call)                                                                             \
    do {                                                                                            \
        hipError_t _e = (call);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            std::fprintf(stderr, "HIP Error at: %s:%d: %s\n", __FILE__, __LINE__, hipGetErrorString(_e)); \
            return 1;                                                                               \
        }                                                                                           \
    } while (0)

static bool ensure_dir(const std::string& dir) {
    struct stat st = {};
    if (stat(dir.c_str(), &st) == 0 && S_ISDIR(st.st_mode)) return true;
    return mkdir(dir.c_str(), 0755) == 0;
}

static void usage(const char* argv0) {
    std::printf(
        "Usage: %s [--kernel=KERNEL] [--warmup=N] [--runs=M] [--check=0|1] [--no-check] [--random]\n"
        "          [--B=1] [--N=8192] [--d_model=1024] [--h=32] [--check-random] [--threads=T]\n"
        "          [--cache-dir=.cache] [--json]\n"
        "  KERNEL options: fa, fa_tc_v1a, fa_tc_int8_b, unfused, fa_mfma, fa_tc_int8_pt\n",
        argv0);
}

static bool take(const char* arg, const char* key, const char** val) {
    const size_t n = std::strlen(key);
    if (std::strncmp(arg, key, n) == 0) {
        *val = arg + n;
        return true;
    }
    return false;
}

static int run_solve(const DeviceTensors& d, int B, int N, int d_model, int h, int variant, hipStream_t s) {
    int st = qmha_solve_ex(d.Q, d.K, d.V, d.O, B, N, d_model, h, variant, s);
    if (st != QMHA_OK) {
        std::fprintf(stderr, "qmha_solve_ex: %s: %s\n", qmha_status_string(st), qmha_last_error());
        return 1;
    }
    return 0;
}

int main(int argc, char** argv) {
    // reference defaults: config.h:22-24 (N=8192, d_model=1024, h=32), main.cu:39-43
    std::string kernel = "fa_tc_int8_b";
    int warmup = 2, runs = 3, B = 1, N = 8192, d_model = 1024, h = 32;
    bool use_random = false, run_check = true, check_random = false, json = false;
    int threads = (int)std::max(1u, std::thread::hardware_concurrency());
    std::string cache_dir = ".cache";
    for (int i = 1; i < argc; ++i) {
        const char* v = nullptr;
        if (take(argv[i], "--kernel=", &v)) kernel = v;
        else if (!std::strcmp(argv[i], "-k") && i + 1 < argc) kernel = argv[++i];
        else if (take(argv[i], "--warmup=", &v)) warmup = std::atoi(v);
        else if (take(argv[i], "--runs=", &v)) runs = std::atoi(v);
        else if (take(argv[i], "--check=", &v)) run_check = std::atoi(v) != 0;
        else if (!std::strcmp(argv[i], "--no-check")) run_check = false;
        else if (!std::strcmp(argv[i], "--check")) run_check = true;
        else if (!std::strcmp(argv[i], "--random")) use_random = true;
        else if (!std::strcmp(argv[i], "--check-random")) check_random = true;
        else if (!std::strcmp(argv[i], "--json")) json = true;
        else if (take(argv[i], "--B=", &v)) B = std::atoi(v);
        else if (take(argv[i], "--N=", &v)) N = std::atoi(v);
        else if (take(argv[i], "--d_model=", &v)) d_model = std::atoi(v);
        else if (take(argv[i], "--h=", &v)) h = std::atoi(v);
        else if (take(argv[i], "--threads=", &v)) threads = std::max(1, std::atoi(v));
        else if (take(argv[i], "--cache-dir=", &v)) cache_dir = v;
        else if (!std::strcmp(argv[i], "--help")) {
            usage(argv[0]);
            return 0;
        } else {
            std::fprintf(stderr, "unknown argument: %s\n", argv[i]);
            usage(argv[0]);
            return 2;
        }
    }
    const int variant = qmha_variant_from_name(kernel.c_str());
    if (variant < 0) {
        std::fprintf(stderr, "unknown kernel '%s'\n", kernel.c_str());
        return 2;
    }
    hipDeviceProp_t prop{};
    DRV_CHECK(hipGetDeviceProperties(&prop, 0));
    std::printf("Device: %s (%s), %d CUs | kernel=%s B=%d N=%d d_model=%d h=%d\n", prop.name, prop.gcnArchName,
                prop.multiProcessorCount, kernel.c_str(), B, N, d_model, h);
    hipStream_t stream;
    DRV_CHECK(hipStreamCreate(&stream));

    std::vector<float> hQ, hK, hV, hO;
    DeviceTensors d;
    const char* check_status = "skipped";
    if (run_check) {
        std::printf("Initializing host data (constant values for correctness check)...\n");
        initialize_host_data(hQ, hK, hV, N, d_model, false);
        allocate_and_copy_to_device(hQ, hK, hV, 1, d);
        std::printf("Running correctness check \n");
        if (run_solve(d, 1, N, d_model, h, variant, stream)) return 1;
        DRV_CHECK(hipStreamSynchronize(stream));
        hO.resize(hQ.size());
        DRV_CHECK(hipMemcpy(hO.data(), d.O, hO.size() * sizeof(float), hipMemcpyDeviceToHost));
        std::vector<float> ref;
        ensure_dir(cache_dir);
        char name[512];
        std::snprintf(name, sizeof(name), "%s/ref_N%d_d%d.bin", cache_dir.c_str(), N, d_model);  // main.cu:15-19
        if (!load_reference(ref, name, N, d_model)) {
            std::printf("Computing CPU reference (multi-head attention with RoPE, %d threads)...\n", threads);
            cpu_reference(hQ, hK, hV, ref, N, d_model, h, threads);
            save_reference(ref, name, N, d_model);
        }
        if (!verify_results(hO, ref, 1e-3f, 1e-3f)) {  // main.cu:96
            std::fprintf(stderr, "Correctness check FAILED. Aborting.\n");
            cleanup_device_data(d);
            return 1;
        }
        std::printf("Correctness check PASSED.\n");
        check_status = "passed";
        cleanup_device_data(d);
    } else {
        std::printf("Skipping correctness check and CPU reference load/compute (--no-check / --check=0).\n");
    }

    ensure_dir(cache_dir);
    char input_cache[512];
    std::snprintf(input_cache, sizeof(input_cache), "%s/input_random_N%d_d%d.bin", cache_dir.c_str(), N, d_model);
    if (!load_inputs(hQ, hK, hV, input_cache, N, d_model)) {
        std::printf("Generating random input data for profiling...\n");
        initialize_host_data(hQ, hK, hV, N, d_model, true);
        save_inputs(hQ, hK, hV, input_cache, N, d_model);
    }
    if (use_random) {
        std::printf("Regenerating random input data (--random flag)...\n");
        initialize_host_data(hQ, hK, hV, N, d_model, true);
    }
    allocate_and_copy_to_device(hQ, hK, hV, B, d);

    std::printf("Running %d warmup iterations...\n", warmup);
    for (int i = 0; i < warmup; ++i) {
        if (run_solve(d, B, N, d_model, h, variant, stream)) return 1;
        DRV_CHECK(hipStreamSynchronize(stream));
    }
    std::printf("Running %d profiling iterations...\n", runs);
    hipEvent_t e0, e1;
    DRV_CHECK(hipEventCreate(&e0));
    DRV_CHECK(hipEventCreate(&e1));
    std::vector<float> ms;
    for (int r = 0; r < runs; ++r) {
        DRV_CHECK(hipEventRecord(e0, stream));
        if (run_solve(d, B, N, d_model, h, variant, stream)) return 1;
        DRV_CHECK(hipEventRecord(e1, stream));
        DRV_CHECK(hipEventSynchronize(e1));
        float t = 0.0f;
        DRV_CHECK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t);
    }
    double max_err = -1.0;
    const char* rand_status = "skipped";
    if (check_random) {
        hO.resize(hQ.size());
        DRV_CHECK(hipMemcpy(hO.data(), d.O, hO.size() * sizeof(float), hipMemcpyDeviceToHost));
        std::vector<float> ref;
        std::printf("Computing CPU attention (no RoPE, %d threads) for the random-data check...\n", threads);
        cpu_attention(hQ, hK, hV, ref, N, d_model, h, threads);
        // tolerances: fp32 1e-5, fp16 1e-3 (verify.cu default), int8 5e-3 (quantisation error)
        const bool int8 = variant == QMHA_FA_TC_INT8_B || variant == QMHA_FA_TC_INT8_PT;
        const float tol = int8 ? 5e-3f : (variant == QMHA_FA_TC_V1A ? 1e-3f : 1e-5f);
        const bool ok = verify_results(hO, ref, tol, tol, &max_err);
        rand_status = ok ? "passed" : "failed";
        std::printf("Random-data check %s (max abs err %.3g, tol %.1g).\n", rand_status, max_err, tol);
    }
    std::vector<float> sorted = ms;
    std::sort(sorted.begin(), sorted.end());
    const double med = sorted.empty() ? 0.0 : sorted[sorted.size() / 2];
    const double mn = sorted.empty() ? 0.0 : sorted.front();
    const double flops = 4.0 * B * (double)h * N * (double)N * (d_model / h);
    std::printf("Profiling complete: median %.4f ms, min %.4f ms, %.2f TFLOPS (4*B*H*N^2*d)\n", med, mn,
                med > 0 ? flops / (med * 1e-3) / 1e12 : 0.0);
    if (json)
        std::printf(
            "{\"kernel\": \"%s\", \"B\": %d, \"N\": %d, \"d_model\": %d, \"h\": %d, \"runs\": %d, \"ms_median\": %.6f, "
            "\"ms_min\": %.6f, \"tflops\": %.4f, \"check\": \"%s\", \"check_random\": \"%s\", \"max_abs_err\": %.4g}\n",
            kernel.c_str(), B, N, d_model, h, runs, med, mn, med > 0 ? flops / (med * 1e-3) / 1e12 : 0.0,
            check_status, rand_status, max_err);
    cleanup_device_data(d);
    DRV_CHECK(hipStreamDestroy(stream));
    return std::strcmp(rand_status, "failed") == 0 ? 1 : 0;
}
