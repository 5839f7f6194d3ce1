// verify.cpp -- HIP C++ host reimplementation of the reference's utils/verify.cu.
#pragma clang fp contract(off)
#include "verify.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <fstream>
#include <thread>

namespace qmha_driver {
namespace {

// verify.cu:9-23
inline void rope_inplace(float* row, int pos, int d) {
    const float base = 10000.0f;
    for (int k = 0; k < d / 2; ++k) {
        const float theta = std::pow(base, -static_cast<float>(2 * k) / d);
        const float angle = pos * theta;
        const float s = std::sin(angle), c = std::cos(angle);
        const float x = row[k], y = row[k + d / 2];
        row[k] = x * c - y * s;
        row[k + d / 2] = x * s + y * c;
    }
}

template <typename Fn>
void parallel_rows(int total, int threads, Fn fn) {
    threads = std::max(1, std::min(threads, total));
    if (threads == 1) {
        fn(0, total);
        return;
    }
    std::vector<std::thread> pool;
    const int per = (total + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const int lo = t * per, hi = std::min(total, lo + per);
        if (lo < hi) pool.emplace_back(fn, lo, hi);
    }
    for (auto& th : pool) th.join();
}

// One output row of one head; rope selects verify.cu (true) or plain attention (false).
void attention_row(const float* Q, const float* K, const float* V, float* out, int N, int d_model, int dh, int col,
                   int i, bool rope, std::vector<float>& scratch) {
    const float alpha = 1.0f / std::sqrt((float)dh);
    scratch.resize((size_t)N + 3 * dh);
    float* scores = scratch.data();
    float* q = scores + N;
    float* k = q + dh;
    float* acc = k + dh;
    for (int kk = 0; kk < dh; ++kk) q[kk] = Q[(size_t)i * d_model + col + kk];
    if (rope) rope_inplace(q, i, dh);
    float mx = -INFINITY;
    for (int j = 0; j < N; ++j) {
        for (int kk = 0; kk < dh; ++kk) k[kk] = K[(size_t)j * d_model + col + kk];
        if (rope) rope_inplace(k, j, dh);
        float s = 0.0f;
        for (int kk = 0; kk < dh; ++kk) s += q[kk] * k[kk];
        s *= alpha;
        scores[j] = s;
        if (s > mx) mx = s;
    }
    float sum = 0.0f;
    for (int j = 0; j < N; ++j) {
        const float e = std::exp(scores[j] - mx);
        scores[j] = e;
        sum += e;
    }
    for (int j = 0; j < N; ++j) scores[j] /= sum;
    for (int kk = 0; kk < dh; ++kk) acc[kk] = 0.0f;
    for (int j = 0; j < N; ++j) {
        const float w = scores[j];
        for (int kk = 0; kk < dh; ++kk) acc[kk] += w * V[(size_t)j * d_model + col + kk];
    }
    for (int kk = 0; kk < dh; ++kk) out[(size_t)i * d_model + col + kk] = acc[kk];
}

void run_all(const std::vector<float>& Q, const std::vector<float>& K, const std::vector<float>& V,
             std::vector<float>& out, int N, int d_model, int h, int threads, bool rope) {
    out.assign((size_t)N * d_model, 0.0f);
    const int dh = d_model / h;
    parallel_rows(N * h, threads, [&](int lo, int hi) {
        std::vector<float> scratch;
        for (int w = lo; w < hi; ++w)
            attention_row(Q.data(), K.data(), V.data(), out.data(), N, d_model, dh, (w / N) * dh, w % N, rope,
                          scratch);
    });
}

}  // namespace

void cpu_reference(const std::vector<float>& Q, const std::vector<float>& K, const std::vector<float>& V,
                   std::vector<float>& out, int N, int d_model, int h, int threads) {
    run_all(Q, K, V, out, N, d_model, h, threads, true);
}

void cpu_attention(const std::vector<float>& Q, const std::vector<float>& K, const std::vector<float>& V,
                   std::vector<float>& out, int N, int d_model, int h, int threads) {
    run_all(Q, K, V, out, N, d_model, h, threads, false);
}

bool verify_results(const std::vector<float>& got, const std::vector<float>& ref, float eps, float rel,
                    double* max_abs_err) {
    if (got.size() != ref.size()) {
        std::fprintf(stderr, " Size mismatch: %zu vs %zu\n", got.size(), ref.size());
        return false;
    }
    double worst = 0.0;
    bool ok = true;
    for (size_t i = 0; i < got.size(); ++i) {
        const float a = got[i], b = ref[i];
        if (!std::isfinite(a) || !std::isfinite(b)) {
            if (ok) std::fprintf(stderr, "Non-finite value at index %zu\n", i);
            ok = false;
            if (!max_abs_err) return false;
            continue;
        }
        worst = std::max(worst, (double)std::fabs(a - b));
        const float tol = std::max(eps, rel * std::fabs(b));
        if (std::fabs(a - b) > tol) {
            if (ok) std::fprintf(stderr, "Mismatch at index: %zu: got=%g ref=%g tol=%g\n", i, a, b, tol);
            ok = false;
            if (!max_abs_err) return false;
        }
    }
    if (max_abs_err) *max_abs_err = worst;
    return ok;
}

bool save_reference(const std::vector<float>& data, const std::string& path, int N, int d_model) {
    std::ofstream f(path, std::ios::binary);
    if (!f) {
        std::fprintf(stderr, "Failed to open %s for writing\n", path.c_str());
        return false;
    }
    f.write(reinterpret_cast<const char*>(&N), sizeof(int));
    f.write(reinterpret_cast<const char*>(&d_model), sizeof(int));
    f.write(reinterpret_cast<const char*>(data.data()), data.size() * sizeof(float));
    std::printf("Saved reference output to %s\n", path.c_str());
    return (bool)f;
}

bool load_reference(std::vector<float>& data, const std::string& path, int N, int d_model) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    int sN = 0, sd = 0;
    f.read(reinterpret_cast<char*>(&sN), sizeof(int));
    f.read(reinterpret_cast<char*>(&sd), sizeof(int));
    if (sN != N || sd != d_model) {
        std::fprintf(stderr, "Reference cache mismatch: expected N=%d d_model=%d but got N=%d d_model=%d\n", N,
                     d_model, sN, sd);
        return false;
    }
    data.assign((size_t)N * d_model, 0.0f);
    f.read(reinterpret_cast<char*>(data.data()), data.size() * sizeof(float));
    if (!f) return false;
    std::printf("Loaded reference output from %s\n", path.c_str());
    return true;
}

}  // namespace qmha_driver
