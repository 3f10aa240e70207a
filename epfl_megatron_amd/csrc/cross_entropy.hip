// Vocab-parallel cross entropy for gfx950 (reference
// megatron/core/tensor_parallel/cross_entropy.py), reading bf16/fp16/fp32
// logits [rows, V] directly (fp32 math in registers; no fp32 logits copy).
//
// TP == 1: ONE pass per row with an online (max, sum-exp) pair per lane,
//          merged across the workgroup; loss = lse - z[target], lse saved.
// TP  > 1: row max -> (RCCL MAX) -> sum-exp + local target logit -> (RCCL SUM).
// Backward: dz = (exp(z - lse) - onehot) * dloss, written in the logits dtype.
// One 256-thread workgroup per row, 16-byte loads.
#include "common.h"
#include "kernels.h"

namespace ema {
namespace {

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <typename T>
__device__ __forceinline__ void row_online(const T* __restrict__ z, int V, float& m, float& s) {
  constexpr int N = V16<T>::N;
  m = -INFINITY;
  s = 0.f;
  for (int c = threadIdx.x * N; c < V; c += blockDim.x * N) {
    const V16<T> v = ld16(z + c);
    float lm = -INFINITY;
#pragma unroll
    for (int e = 0; e < N; ++e) lm = fmaxf(lm, to_f(v.v[e]));
    float ls = 0.f;
#pragma unroll
    for (int e = 0; e < N; ++e) ls += __expf(to_f(v.v[e]) - lm);
    online_merge(m, s, lm, ls);
  }
}

__device__ __forceinline__ void block_online_reduce(float& m, float& s) {
  __shared__ float sm[16], ss[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
  }
  if (lane == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  m = -INFINITY;
  s = 0.f;
  for (int i = 0; i < nw; ++i) online_merge(m, s, sm[i], ss[i]);
}

template <typename T>
__global__ __launch_bounds__(256) void ce_fused_k(const T* __restrict__ logits,
                                                  const int64_t* __restrict__ target,
                                                  float* __restrict__ loss, float* __restrict__ lse,
                                                  int V) {
  const int64_t row = blockIdx.x;
  const T* z = logits + row * V;
  float m, s;
  row_online(z, V, m, s);
  block_online_reduce(m, s);
  if (threadIdx.x == 0) {
    const float l = logf(s) + m;
    const int64_t t = target[row];
    const float zt = (t >= 0 && t < V) ? to_f(z[t]) : 0.f;
    lse[row] = l;
    loss[row] = l - zt;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_max_k(const T* __restrict__ logits, float* __restrict__ rmax,
                                                int V) {
  constexpr int N = V16<T>::N;
  __shared__ float red[16];
  const T* z = logits + (int64_t)blockIdx.x * V;
  float m = -INFINITY;
  for (int c = threadIdx.x * N; c < V; c += blockDim.x * N) {
    const V16<T> v = ld16(z + c);
#pragma unroll
    for (int e = 0; e < N; ++e) m = fmaxf(m, to_f(v.v[e]));
  }
  m = block_max(m, red);
  if (threadIdx.x == 0) rmax[blockIdx.x] = m;
}

template <typename T>
__global__ __launch_bounds__(256) void ce_sumexp_k(const T* __restrict__ logits,
                                                   const int64_t* __restrict__ target,
                                                   const float* __restrict__ rmax,
                                                   float* __restrict__ sumexp,
                                                   float* __restrict__ tlogit, int V, int64_t vstart) {
  constexpr int N = V16<T>::N;
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const T* z = logits + row * V;
  const float m = rmax[row];
  float s = 0.f;
  for (int c = threadIdx.x * N; c < V; c += blockDim.x * N) {
    const V16<T> v = ld16(z + c);
#pragma unroll
    for (int e = 0; e < N; ++e) s += __expf(to_f(v.v[e]) - m);
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    sumexp[row] = s;
    const int64_t t = target[row] - vstart;
    tlogit[row] = (t >= 0 && t < V) ? to_f(z[t]) : 0.f;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_k(const T* __restrict__ logits,
                                                const int64_t* __restrict__ target,
                                                const float* __restrict__ lse,
                                                const float* __restrict__ dloss,
                                                T* __restrict__ dz, int V, int64_t vstart) {
  constexpr int N = V16<T>::N;
  const int64_t row = blockIdx.x;
  const T* z = logits + row * V;
  T* o = dz + row * V;
  const float l = lse[row], g = dloss[row];
  const int64_t t = target[row] - vstart;
  for (int c = threadIdx.x * N; c < V; c += blockDim.x * N) {
    const V16<T> v = ld16(z + c);
    V16<T> r;
#pragma unroll
    for (int e = 0; e < N; ++e) {
      float p = __expf(to_f(v.v[e]) - l);
      if (c + e == t) p -= 1.f;
      r.v[e] = from_f<T>(p * g);
    }
    st16(o + c, r);
  }
}

}  // namespace

void ce_fwd_fused(const void* logits, const int64_t* target, float* loss, float* lse,
                  int64_t rows, int V, int dt, hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((ce_fused_k<T>), dim3(rows), dim3(256), 0, s,
                                               (const T*)logits, target, loss, lse, V));
}

void ce_row_max(const void* logits, float* rmax, int64_t rows, int V, int dt, hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((ce_max_k<T>), dim3(rows), dim3(256), 0, s,
                                               (const T*)logits, rmax, V));
}

void ce_sumexp_target(const void* logits, const int64_t* target, const float* rmax,
                      float* sumexp, float* tlogit, int64_t rows, int V, int64_t vstart, int dt,
                      hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((ce_sumexp_k<T>), dim3(rows), dim3(256), 0, s,
                                               (const T*)logits, target, rmax, sumexp, tlogit, V,
                                               vstart));
}

void ce_bwd(const void* logits, const int64_t* target, const float* lse, const float* dloss,
            void* dlogits, int64_t rows, int V, int64_t vstart, int dt, hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((ce_bwd_k<T>), dim3(rows), dim3(256), 0, s,
                                               (const T*)logits, target, lse, dloss, (T*)dlogits,
                                               V, vstart));
}

}  // namespace ema
