// data.h -- host input generation and input cache (reference inputs/data.h, inputs/data.cu).
#pragma once
#include <string>
#include <vector>

namespace qmha_driver {

// inputs/data.cu:9-30: all-ones (correctness check) or std::mt19937(seed) U[0,1) drawn
// interleaved Q,K,V per element.  seed 42 is the reference's.
void initialize_host_data(std::vector<float>& Q, std::vector<float>& K, std::vector<float>& V, int N, int d_model,
                          bool use_random, unsigned seed = 42);

// Input cache, reference format (data.cu:54-108): int N, int d_model, Q, K, V (fp32).
bool save_inputs(const std::vector<float>& Q, const std::vector<float>& K, const std::vector<float>& V,
                 const std::string& path, int N, int d_model);
bool load_inputs(std::vector<float>& Q, std::vector<float>& K, std::vector<float>& V, const std::string& path, int N,
                 int d_model);

// Device buffers (data.cu:32-52).  Each tensor is [B][N][d_model]; the host data holds
// one batch element and is replicated B times.
struct DeviceTensors {
    float *Q = nullptr, *K = nullptr, *V = nullptr, *O = nullptr;
    size_t elems = 0;
};
void allocate_and_copy_to_device(const std::vector<float>& Q, const std::vector<float>& K,
                                 const std::vector<float>& V, int B, DeviceTensors& d);
void cleanup_device_data(DeviceTensors& d);

}  // namespace qmha_driver
