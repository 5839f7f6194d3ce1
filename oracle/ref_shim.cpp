// ref_shim.cpp -- C entry points around the REFERENCE's own utils/verify.cu,
// which is compiled unmodified from /root/reference by oracle/Makefile into
// oracle/_ref/libref_verify.so.  TEST INFRASTRUCTURE ONLY: used by tests/ to pin
// the oracle restatement and by bench.py's cpu_baseline leg ("kind": "reference").
#include <cstring>
#include <vector>

#include "verify.h"  // /root/reference/utils/verify.h (via -I)

extern "C" void ref_cpu_reference(const float *Q, const float *K, const float *V, float *out,
                                  int N, int d_model, int h) {
    const size_t n = (size_t)N * d_model;
    std::vector<float> q(Q, Q + n), k(K, K + n), v(V, V + n), o;
    cpu_reference(q, k, v, o, N, d_model, h);
    std::memcpy(out, o.data(), n * sizeof(float));
}

extern "C" int ref_verify_results(const float *got, const float *ref, size_t n, float eps, float rel) {
    std::vector<float> a(got, got + n), b(ref, ref + n);
    return verify_results(a, b, eps, rel) ? 1 : 0;
}

extern "C" int ref_save_reference(const float *data, size_t n, const char *filename, int N, int d_model) {
    std::vector<float> a(data, data + n);
    return save_reference(a, filename, N, d_model) ? 1 : 0;
}

extern "C" int ref_load_reference(float *data, size_t n, const char *filename, int N, int d_model) {
    std::vector<float> a;
    if (!load_reference(a, filename, N, d_model)) return 0;
    if (a.size() != n) return 0;
    std::memcpy(data, a.data(), n * sizeof(float));
    return 1;
}
