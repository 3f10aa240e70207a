// Fused scale -> mask -> softmax (non-flash attention path; reference kernels
// N1-N5).  One 256-thread workgroup per score row; the row stays in registers
// (EPT = elements per thread, templated), fp32 math, sk <= 8192.
//   mode 0: no mask;  mode 1: causal (col > row + (sk - sq) masked, written as 0);
//   mode 2: explicit mask [b, 1, sq, sk] (true = masked -> -10000 like the
//           reference; a fully masked row produces zeros).
#include "common.h"
#include "kernels.h"

namespace ema {
namespace {

template <typename T, int EPT>
__global__ __launch_bounds__(256) void softmax_fwd_k(const T* __restrict__ x,
                                                     const uint8_t* __restrict__ mask,
                                                     T* __restrict__ y, int64_t NP, int SQ, int SK,
                                                     float scale, int mode) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const int q = (int)(row % SQ);
  const int64_t b = row / (NP * SQ);
  const T* xr = x + row * SK;
  const uint8_t* mr = (mode == 2) ? mask + (b * SQ + q) * (int64_t)SK : nullptr;
  const int limit = (mode == 1) ? q + 1 : SK;  // causal: square scores (sq == sk)
  float v[EPT];
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int c = threadIdx.x + i * 256;
    float val = -INFINITY;
    if (c < SK) {
      if (c < limit) {
        val = to_f(xr[c]) * scale;
        if (mr && mr[c]) val = -10000.f;
      }
    }
    v[i] = val;
    m = fmaxf(m, val);
  }
  m = block_max(m, red);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const float e = (v[i] == -INFINITY) ? 0.f : __expf(v[i] - m);
    v[i] = e;
    s += e;
  }
  s = block_sum(s, red);
  const bool all_masked = (mode == 2) && (m == -10000.f);
  const float inv = all_masked ? 0.f : 1.f / s;
  T* yr = y + row * SK;
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < SK) yr[c] = from_f<T>(v[i] * inv);
  }
}

template <typename T, int EPT>
__global__ __launch_bounds__(256) void softmax_bwd_k(const T* __restrict__ dy, const T* __restrict__ y,
                                                     T* __restrict__ dx, int SK, float scale) {
  __shared__ float red[16];
  const int64_t row = blockIdx.x;
  const T* dr = dy + row * SK;
  const T* yr = y + row * SK;
  float yv[EPT], dv[EPT];
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int c = threadIdx.x + i * 256;
    yv[i] = c < SK ? to_f(yr[c]) : 0.f;
    dv[i] = c < SK ? to_f(dr[c]) : 0.f;
    dot += yv[i] * dv[i];
  }
  dot = block_sum(dot, red);
  T* xr = dx + row * SK;
#pragma unroll
  for (int i = 0; i < EPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < SK) xr[c] = from_f<T>(scale * yv[i] * (dv[i] - dot));
  }
}

#define EMA_EPT_SWITCH(sk, ...)                                   \
  {                                                               \
    const int ept_ = (sk + 255) / 256;                            \
    if (ept_ <= 1) { constexpr int E = 1; __VA_ARGS__; }          \
    else if (ept_ <= 2) { constexpr int E = 2; __VA_ARGS__; }     \
    else if (ept_ <= 4) { constexpr int E = 4; __VA_ARGS__; }     \
    else if (ept_ <= 8) { constexpr int E = 8; __VA_ARGS__; }     \
    else if (ept_ <= 16) { constexpr int E = 16; __VA_ARGS__; }   \
    else { constexpr int E = 32; __VA_ARGS__; }                   \
  }

}  // namespace

void softmax_fwd(const void* x, const uint8_t* mask, void* y, int64_t B, int64_t NP, int SQ,
                 int SK, float scale, int mode, int dt, hipStream_t s) {
  const int64_t rows = B * NP * SQ;
  EMA_DISPATCH_FLOAT(dt, T, EMA_EPT_SWITCH(SK, hipLaunchKernelGGL((softmax_fwd_k<T, E>),
      dim3(rows), dim3(256), 0, s, (const T*)x, mask, (T*)y, NP, SQ, SK, scale, mode)));
}

void softmax_bwd(const void* dy, const void* y, void* dx, int64_t rows, int SK, float scale,
                 int dt, hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, EMA_EPT_SWITCH(SK, hipLaunchKernelGGL((softmax_bwd_k<T, E>),
      dim3(rows), dim3(256), 0, s, (const T*)dy, (const T*)y, (T*)dx, SK, scale)));
}

}  // namespace ema
