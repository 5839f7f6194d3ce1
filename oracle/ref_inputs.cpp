// ref_inputs.cpp -- restates inputs/data.cu:9-30 (initialize_host_data) and the
// input-cache format of inputs/data.cu:54-108 (save_inputs).  data.cu itself
// needs cuda_runtime.h, so its 20-line generator is restated here; built with
// g++ so std::mt19937 + std::uniform_real_distribution<float> produce the same
// libstdc++ sequence as the reference's host build.  TEST INFRASTRUCTURE ONLY.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s N d_model out.bin [ones]\n", argv[0]);
        return 2;
    }
    int N = std::atoi(argv[1]), d_model = std::atoi(argv[2]);
    bool ones = argc > 4;
    size_t total = (size_t)N * d_model;
    std::vector<float> Q(total), K(total), V(total);
    if (!ones) {
        std::mt19937 gen(42);
        std::uniform_real_distribution<float> dis(0.0f, 1.0f);
        for (size_t i = 0; i < total; ++i) {  // interleaved Q,K,V per index (data.cu:16-22)
            Q[i] = dis(gen);
            K[i] = dis(gen);
            V[i] = dis(gen);
        }
    } else {
        for (size_t i = 0; i < total; ++i) Q[i] = K[i] = V[i] = 1.0f;
    }
    FILE *f = std::fopen(argv[3], "wb");
    if (!f) return 1;
    std::fwrite(&N, sizeof(int), 1, f);
    std::fwrite(&d_model, sizeof(int), 1, f);
    std::fwrite(Q.data(), sizeof(float), total, f);
    std::fwrite(K.data(), sizeof(float), total, f);
    std::fwrite(V.data(), sizeof(float), total, f);
    std::fclose(f);
    return 0;
}
