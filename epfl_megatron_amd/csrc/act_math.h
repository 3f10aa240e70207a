// Scalar activation math shared by the elementwise kernels (activations.hip)
// and the GEMM epilogues (gemm_nt.hip): GLU gates act(x) / act'(x) in fp32.
#pragma once
#include <hip/hip_runtime.h>

namespace ema {

constexpr float kInvSqrt2 = 0.70710678118654752f;
constexpr float kInvSqrt2Pi = 0.39894228040143268f;

// sigmoid(x) = 1 / (1 + 2^(-x log2 e)) on the hardware v_exp_f32 / v_rcp_f32
// (~1 ulp each): 4 VALU ops instead of the ~14 of an IEEE-exact division
// (hipcc's default fp32 divide is the div_scale / div_fmas / div_fixup
// sequence).  The results are rounded to bf16 / fp16, far coarser than the
// approximation.  In the GEMM epilogues these ops are the whole cost of the
// fused activation: one wave per SIMD issues each VALU op in 4 cycles.
// x -> -inf: 2^(+inf) = inf, rcp(inf) = 0; x -> +inf: rcp(1) = 1.
__device__ __forceinline__ float sigmoidf_(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}

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

// act(x) and act'(x) together, sharing one sigmoid (SwiGLU: act = x s,
// act' = s (1 + x (1 - s)) = s + act (1 - s)).
template <int KIND>
__device__ __forceinline__ void act_dact(float x, float& a, float& d) {
  if constexpr (KIND == 0) {
    const float sg = sigmoidf_(x);
    a = x * sg;
    d = __builtin_fmaf(a, 1.f - sg, sg);
  } else {
    a = act<KIND>(x);
    d = dact<KIND>(x);
  }
}

}  // namespace ema
