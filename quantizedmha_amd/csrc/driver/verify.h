// verify.h -- the host verify path (reference utils/verify.h, utils/verify.cu), HIP C++.
#pragma once
#include <string>
#include <vector>

namespace qmha_driver {

// utils/verify.cu:25-104: MHA with RoPE on q_i and k_j (the reference's check target).
// Same fp32 arithmetic as the reference (no contraction); rows are distributed over
// `threads` host threads, which does not change any result.
void cpu_reference(const std::vector<float>& Q, const std::vector<float>& K, const std::vector<float>& V,
                   std::vector<float>& out, int N, int d_model, int h, int threads = 1);

// Plain softmax(QK^T/sqrt(d))V (no RoPE) -- what the GPU kernels compute; used by
// --check-random (the reference has no random-data check: drivers/main.cu:109-127).
void cpu_attention(const std::vector<float>& Q, const std::vector<float>& K, const std::vector<float>& V,
                   std::vector<float>& out, int N, int d_model, int h, int threads = 1);

// utils/verify.cu:153-172: first failure printed, false on any mismatch / non-finite.
bool verify_results(const std::vector<float>& got, const std::vector<float>& ref, float eps = 1e-3f,
                    float rel = 1e-3f, double* max_abs_err = nullptr);

// utils/verify.cu:106-151: int N, int d_model, then N*d_model floats.
bool save_reference(const std::vector<float>& data, const std::string& path, int N, int d_model);
bool load_reference(std::vector<float>& data, const std::string& path, int N, int d_model);

}  // namespace qmha_driver
