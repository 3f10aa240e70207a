// GLU family (SwiGLU / GeGLU / ReGLU / LiGLU) and GeLU (bias + tanh approx,
// exact erf) forward/backward for gfx950.
//
// GLU layout (reference megatron/model/glu_activations.py:18-21): the fc1
// output row [2F] splits into x1 = [0, F) ("up", w3) and x2 = [F, 2F) (gate,
// w1); y = x1 * act(x2).  Memory bound: one thread = one 16-byte vector of
// each operand, fp32 math, a single rounding per output.
#include "common.h"
#include "kernels.h"
#include "act_math.h"

namespace ema {
namespace {

template <typename T, int KIND>
__global__ __launch_bounds__(256) void glu_fwd_k(const T* __restrict__ x, T* __restrict__ y,
                                                 int64_t rows, int F) {
  constexpr int N = V16<T>::N;
  const int nv = F / N;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * nv) return;
  const int64_t r = t / nv;
  const int c = (int)(t % nv) * N;
  const T* xr = x + r * (2 * (int64_t)F);
  const V16<T> a = ld16(xr + c);
  const V16<T> g = ld16(xr + F + c);
  V16<T> o;
#pragma unroll
  for (int e = 0; e < N; ++e) o.v[e] = from_f<T>(to_f(a.v[e]) * act<KIND>(to_f(g.v[e])));
  st16(y + r * F + c, o);
}

template <typename T, int KIND>
__global__ __launch_bounds__(256) void glu_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                 T* __restrict__ dx, int64_t rows, int F) {
  constexpr int N = V16<T>::N;
  const int nv = F / N;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * nv) return;
  const int64_t r = t / nv;
  const int c = (int)(t % nv) * N;
  const T* xr = x + r * (2 * (int64_t)F);
  const V16<T> a = ld16(xr + c);
  const V16<T> g = ld16(xr + F + c);
  const V16<T> d = ld16(dy + r * F + c);
  V16<T> da, dg;
#pragma unroll
  for (int e = 0; e < N; ++e) {
    const float gv = to_f(g.v[e]), dv = to_f(d.v[e]);
    float av, dd;
    act_dact<KIND>(gv, av, dd);
    da.v[e] = from_f<T>(dv * av);
    dg.v[e] = from_f<T>(dv * to_f(a.v[e]) * dd);
  }
  T* dr = dx + r * (2 * (int64_t)F);
  st16(dr + c, da);
  st16(dr + F + c, dg);
}

__device__ __forceinline__ float gelu_tanh(float z) {
  return z * 0.5f * (1.f + tanhf(0.79788456f * z * (1.f + 0.044715f * z * z)));
}
__device__ __forceinline__ float dgelu_tanh(float z) {
  const float t = tanhf(0.79788456f * z * (1.f + 0.044715f * z * z));
  return 0.5f * z * ((1.f - t * t) * (0.79788456f + 0.1070322243f * z * z)) + 0.5f * (1.f + t);
}
__device__ __forceinline__ float gelu_erf(float z) { return 0.5f * z * (1.f + erff(z * kInvSqrt2)); }
__device__ __forceinline__ float dgelu_erf(float z) {
  return 0.5f * (1.f + erff(z * kInvSqrt2)) + z * kInvSqrt2Pi * __expf(-0.5f * z * z);
}

template <typename T, bool TANH>
__global__ __launch_bounds__(256) void gelu_fwd_k(const T* __restrict__ x, const T* __restrict__ bias,
                                                  T* __restrict__ y, int64_t rows, int F) {
  constexpr int N = V16<T>::N;
  const int nv = F / N;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * nv) return;
  const int64_t r = t / nv;
  const int c = (int)(t % nv) * N;
  const V16<T> a = ld16(x + r * F + c);
  V16<T> bv;
  if (bias) bv = ld16(bias + c);
  V16<T> o;
#pragma unroll
  for (int e = 0; e < N; ++e) {
    float z = to_f(a.v[e]);
    if (bias) z += to_f(bv.v[e]);
    o.v[e] = from_f<T>(TANH ? gelu_tanh(z) : gelu_erf(z));
  }
  st16(y + r * F + c, o);
}

template <typename T, bool TANH>
__global__ __launch_bounds__(256) void gelu_bwd_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                  const T* __restrict__ bias, T* __restrict__ dx,
                                                  int64_t rows, int F) {
  constexpr int N = V16<T>::N;
  const int nv = F / N;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * nv) return;
  const int64_t r = t / nv;
  const int c = (int)(t % nv) * N;
  const V16<T> a = ld16(x + r * F + c);
  const V16<T> d = ld16(dy + r * F + c);
  V16<T> bv;
  if (bias) bv = ld16(bias + c);
  V16<T> o;
#pragma unroll
  for (int e = 0; e < N; ++e) {
    float z = to_f(a.v[e]);
    if (bias) z += to_f(bv.v[e]);
    o.v[e] = from_f<T>(to_f(d.v[e]) * (TANH ? dgelu_tanh(z) : dgelu_erf(z)));
  }
  st16(dx + r * F + c, o);
}

#define EMA_GLU_KIND(kind, ...)                               \
  switch (kind) {                                             \
    case 0: { constexpr int K = 0; __VA_ARGS__; break; }      \
    case 1: { constexpr int K = 1; __VA_ARGS__; break; }      \
    case 2: { constexpr int K = 2; __VA_ARGS__; break; }      \
    default: { constexpr int K = 3; __VA_ARGS__; break; }     \
  }

template <typename T>
int64_t nblocks(int64_t rows, int F) {
  return (rows * (F / V16<T>::N) + 255) / 256;
}

}  // namespace

void glu_fwd(const void* x, void* y, int64_t rows, int F, int kind, int dt, hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, EMA_GLU_KIND(kind, hipLaunchKernelGGL((glu_fwd_k<T, K>),
      dim3(nblocks<T>(rows, F)), dim3(256), 0, s, (const T*)x, (T*)y, rows, F)));
}

void glu_bwd(const void* dy, const void* x, void* dx, int64_t rows, int F, int kind, int dt,
             hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, EMA_GLU_KIND(kind, hipLaunchKernelGGL((glu_bwd_k<T, K>),
      dim3(nblocks<T>(rows, F)), dim3(256), 0, s, (const T*)dy, (const T*)x, (T*)dx, rows, F)));
}

void gelu_fwd(const void* x, const void* bias, void* y, int64_t rows, int F, int approx, int dt,
              hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, {
    if (approx == 0)
      hipLaunchKernelGGL((gelu_fwd_k<T, true>), dim3(nblocks<T>(rows, F)), dim3(256), 0, s,
                         (const T*)x, (const T*)bias, (T*)y, rows, F);
    else
      hipLaunchKernelGGL((gelu_fwd_k<T, false>), dim3(nblocks<T>(rows, F)), dim3(256), 0, s,
                         (const T*)x, (const T*)bias, (T*)y, rows, F);
  });
}

void gelu_bwd(const void* dy, const void* x, const void* bias, void* dx, int64_t rows, int F,
              int approx, int dt, hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, {
    if (approx == 0)
      hipLaunchKernelGGL((gelu_bwd_k<T, true>), dim3(nblocks<T>(rows, F)), dim3(256), 0, s,
                         (const T*)dy, (const T*)x, (const T*)bias, (T*)dx, rows, F);
    else
      hipLaunchKernelGGL((gelu_bwd_k<T, false>), dim3(nblocks<T>(rows, F)), dim3(256), 0, s,
                         (const T*)dy, (const T*)x, (const T*)bias, (T*)dx, rows, F);
  });
}

}  // namespace ema
