// Compiled PyTorch extension `torch_ext` -- the drop-in for the reference's pybind module
// (extensions/torch/torch_ext.cpp:11-58, built per kernel by extensions/torch/setup.py:21-43).
// Same module name, function name, argument names/defaults and TORCH_CHECK messages, so
// `import torch_ext; torch_ext.flash_solve(Q, K, V, d_model, num_heads)` works unchanged.
// It is a thin shim over the C-ABI in libqmha.so (include/launchers.h): no kernel code here.
//
// Differences from the reference, all additive (same as quantizedmha_amd/torch_ext.py):
//   * `kernel` really selects the variant (the reference warns and runs its build-time kernel;
//     an unknown name still warns and routes to fa_tc_int8_b, torch_ext.cpp:32-34);
//   * a 3-D [B, N, d_model] input is B sequences in one launch;
//   * the work is enqueued on PyTorch's current HIP stream (ordered with the caller's other
//     ops) instead of private streams plus a blocking device synchronisation;
//   * a rejected shape raises (TORCH_CHECK on the C-ABI status) instead of a device assert.
#include <torch/extension.h>
// ROCm PyTorch reports HIP devices as device type "cuda": the guard / current-stream
// accessors for such tensors are the "MasqueradingAsCUDA" ones
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <string>

#include "launchers.h"

using torch::Tensor;

static Tensor flash_solve(const Tensor& Q, const Tensor& K, const Tensor& V, int64_t d_model, int64_t num_heads,
                          const std::string& kernel = "fa_tc_int8_b") {
    TORCH_CHECK(Q.is_cuda() && K.is_cuda() && V.is_cuda(), "Inputs must be CUDA tensors");
    TORCH_CHECK(Q.dtype() == torch::kFloat32, "Q must be float32");
    TORCH_CHECK(K.dtype() == torch::kFloat32, "K must be float32");
    TORCH_CHECK(V.dtype() == torch::kFloat32, "V must be float32");
    auto Qc = Q.contiguous();
    auto Kc = K.contiguous();
    auto Vc = V.contiguous();
    const int64_t q_elems = Qc.numel();
    TORCH_CHECK(d_model > 0 && q_elems % d_model == 0, "Q.numel() must be divisible by d_model");
    TORCH_CHECK(Kc.sizes() == Qc.sizes() && Vc.sizes() == Qc.sizes(), "Q, K and V must have the same shape");
    // [B, N, d_model] is B sequences; any other layout is one sequence of numel / d_model rows,
    // as in the reference (torch_ext.cpp:23-25), e.g. [N, h, d]
    const bool batched = Qc.dim() == 3 && Qc.size(2) == d_model;
    const int64_t B = batched ? Qc.size(0) : 1;
    const int64_t N = batched ? Qc.size(1) : q_elems / d_model;
    int variant = qmha_variant_from_name(kernel.c_str());
    if (variant < 0) {
        TORCH_WARN("Kernel selection supports fa, fa_tc_v1a, fa_tc_int8_b, unfused, fa_mfma, fa_tc_int8_pt; '", kernel,
                   "' routing to default 'fa_tc_int8_b'");
        variant = QMHA_FA_TC_INT8_B;
    }
    auto out = torch::empty_like(Qc);
    const c10::hip::HIPGuardMasqueradingAsCUDA guard(Qc.device());
    const hipStream_t stream = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(Qc.device().index()).stream();
    const int st = qmha_solve_ex(Qc.data_ptr<float>(), Kc.data_ptr<float>(), Vc.data_ptr<float>(),
                                 out.data_ptr<float>(), static_cast<int>(B), static_cast<int>(N),
                                 static_cast<int>(d_model), static_cast<int>(num_heads), variant, stream);
    TORCH_CHECK(st == QMHA_OK, "flash_solve(", kernel, "): ", qmha_status_string(st), ": ", qmha_last_error());
    return out;
}

PYBIND11_MODULE(torch_ext, m) {
    m.def("flash_solve", &flash_solve,
          "FlashAttention solve (HIP, MI355X)\n\n"
          "Args:\n"
          "  Q: Query tensor [N, d_model] (or [B, N, d_model])\n"
          "  K: Key tensor [N, d_model]\n"
          "  V: Value tensor [N, d_model]\n"
          "  d_model: Model dimension\n"
          "  num_heads: Number of attention heads\n"
          "  kernel: Kernel variant (default: 'fa_tc_int8_b')",
          pybind11::arg("Q"), pybind11::arg("K"), pybind11::arg("V"), pybind11::arg("d_model"),
          pybind11::arg("num_heads"), pybind11::arg("kernel") = "fa_tc_int8_b");
}
