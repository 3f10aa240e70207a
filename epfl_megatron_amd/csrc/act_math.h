// Scalar activation math shared by the elementwise kernels (activations.hip)
// and the GEMM epilogues (gemm_nt.hip): GLU gates act(x) / act'(x) in fp32.
#pragma once
#include <hip/hip_runtime.h>

namespace ema {

constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

template <int KIND>
__device__ __forceinline__ float act(float x) {
  if constexpr (KIND == 0) return x * sigmoidf_(x);                     // swiglu
  else if constexpr (KIND == 1) return 0.5f * x * (1.f + erff(x * kInvSqrt2));  // geglu
  else if constexpr (KIND == 2) return x > 0.f ? x : 0.f;               // reglu
  else return x;                                                        // liglu
}
template <int KIND>
__device__ __forceinline__ float dact(float x) {
  if constexpr (KIND == 0) {
    const float sg = sigmoidf_(x);
    return sg * (1.f + x * (1.f - sg));
  } else if constexpr (KIND == 1) {
    return 0.5f * (1.f + erff(x * kInvSqrt2)) + x * kInvSqrt2Pi * __expf(-0.5f * x * x);
  } else if constexpr (KIND == 2) {
    return x > 0.f ? 1.f : 0.f;
  } else {
    return 1.f;
  }
}

}  // namespace ema
