// Python binding of the bench-only GEMM lab (scripts/lab/gemm_lab.hip), built
// into scripts/lab/_gemm_lab.so by `python -m epfl_megatron_amd.build --lab`
// and loaded by scripts/gemm_lab.py only: ablation builds stay out of the
// product extension (epfl_megatron_amd/_C.so).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <hip/hip_runtime.h>

namespace ema {
void gemm_lab(const void* a, const void* b, void* c, int64_t M, int64_t N, int64_t K, int variant,
              hipStream_t s);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("gemm_lab", [](const at::Tensor& a, const at::Tensor& b, at::Tensor c, int64_t variant) {
    TORCH_CHECK(a.is_cuda() && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16 &&
                    c.scalar_type() == at::kBFloat16 && a.is_contiguous() && b.is_contiguous() &&
                    c.is_contiguous() && a.size(1) == b.size(1) && c.size(0) == a.size(0) &&
                    c.size(1) == b.size(0) && a.size(1) % 64 == 0 && a.size(1) >= 128 &&
                    b.size(0) % 8 == 0,
                "gemm_lab: contiguous bf16 [M,K] x [N,K] -> [M,N], K % 64 == 0, K >= 128");
    TORCH_CHECK(a.size(0) * a.size(1) * 2 < (int64_t(1) << 31) && b.size(0) * b.size(1) * 2 < (int64_t(1) << 31),
                "gemm_lab: operands must be < 2 GiB (32-bit buffer offsets)");
    ema::gemm_lab(a.data_ptr(), b.data_ptr(), c.data_ptr(), a.size(0), b.size(0), a.size(1),
                  (int)variant, c10::hip::getCurrentHIPStream().stream());
  });
}
