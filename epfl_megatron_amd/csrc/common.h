// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64: lane = threadIdx.x & 63, reductions span 64 lanes;
//   * element types are __bf16 / _Float16 / float; math is fp32 in registers;
//     float -> bf16 uses the native v_cvt_pk_bf16_f32 (RNE, NaN-preserving);
//   * global traffic is 16 bytes per lane (8 x bf16, 4 x fp32) wherever the
//     layout allows (CDNA guide, Guideline 13);
//   * every launcher takes the caller's hipStream_t (PyTorch's current stream)
//     and performs no host synchronisation, so it is hipGraph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace ema {

typedef __bf16 bf16;
typedef _Float16 fp16;

template <typename T>
__device__ __forceinline__ float to_f(T x) { return (float)x; }
template <typename T>
__device__ __forceinline__ T from_f(float x) { return (T)x; }

// 16-byte vector of T.
template <typename T>
struct alignas(16) V16 {
  static constexpr int N = 16 / sizeof(T);
  T v[N];
};

template <typename T>
__device__ __forceinline__ V16<T> ld16(const T* p) {
  return *reinterpret_cast<const V16<T>*>(p);
}
template <typename T>
__device__ __forceinline__ void st16(T* p, const V16<T>& v) {
  *reinterpret_cast<V16<T>*>(p) = v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide reductions through LDS (blockDim.x multiple of 64, <= 1024).
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = (lane < nw) ? red[lane] : 0.f;
  return wave_sum(r);
}
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = (lane < nw) ? red[lane] : -INFINITY;
  return wave_max(r);
}

// XCD-aware block-id remap (MI355X: 8 XCDs, blocks dealt round-robin): gives
// each XCD a contiguous range of logical tiles so neighbours share its L2.
// Bijective for any grid size (CDNA guide §5 "XCD swizzle must be bijective").
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

}  // namespace ema

#define EMA_DISPATCH_FLOAT(dt, T, ...)                              \
  switch (dt) {                                                     \
    case ema::DT_F32: { typedef float T; __VA_ARGS__; break; }      \
    case ema::DT_F16: { typedef ema::fp16 T; __VA_ARGS__; break; }  \
    case ema::DT_BF16: { typedef ema::bf16 T; __VA_ARGS__; break; } \
  }
