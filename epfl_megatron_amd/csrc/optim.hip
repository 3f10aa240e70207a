// Flat-buffer optimizer kernels for gfx950.
//
// The whole model's fp32 state lives in flat buffers; a static chunk table
// (int64 [n, 4] = master_off, buf_off, length, meta; meta = group | norm<<8)
// maps 64K-element chunks to workgroups.  All offsets are multiples of 64
// elements, so every lane moves 16 bytes per access.
//
//   chunked_sumsq: per-chunk sum of squares of the gradient (chunks with the
//                  norm flag), then a fixed-order second pass -> deterministic.
//   flat_adam:     AdamW (apex FusedAdam math, bias correction) fused with the
//                  grad scaling (clip coef / loss scale) and the write-back of
//                  the bf16/fp16 model parameters: one streaming pass over
//                  grad, master, m, v (30 bytes moved per parameter).
#include "common.h"
#include "kernels.h"

namespace ema {
namespace {

__global__ __launch_bounds__(256) void sumsq_chunks_k(const float* __restrict__ g,
                                                      const int64_t* __restrict__ table,
                                                      float* __restrict__ partial) {
  __shared__ float red[16];
  const int64_t* row = table + 4 * (int64_t)blockIdx.x;
  const int64_t off = row[1], n = row[2], meta = row[3];
  float s = 0.f;
  if (meta >> 8) {
    const float* p = g + off;
    const int64_t n4 = n / 4;
    for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) {
      const float4 v = reinterpret_cast<const float4*>(p)[i];
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) s += p[i] * p[i];
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(1024) void sum_partials_k(const float* __restrict__ partial, int n,
                                                       float* __restrict__ out) {
  __shared__ float red[16];
  // Kahan-free but fixed-order: thread t sums t, t+1024, ... then tree reduce.
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += partial[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s;
}

template <typename TO>
__device__ __forceinline__ void store4(TO* p, float a, float b, float c, float d) {
  if constexpr (sizeof(TO) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
  } else {
    struct alignas(8) P4 { TO v[4]; } o;
    o.v[0] = from_f<TO>(a); o.v[1] = from_f<TO>(b); o.v[2] = from_f<TO>(c); o.v[3] = from_f<TO>(d);
    *reinterpret_cast<P4*>(p) = o;
  }
}

struct AdamScal {
  float gs, bc1, bc2;
};

__device__ __forceinline__ float adam_elem(float& p, float g, float& m, float& v, float lr,
                                           float wd, const AdamArgs& a, const AdamScal& c) {
  g *= c.gs;
  if (!a.adam_w_mode) g += wd * p;
  m = a.beta1 * m + (1.f - a.beta1) * g;
  v = a.beta2 * v + (1.f - a.beta2) * g * g;
  const float denom = sqrtf(v / c.bc2) + a.eps;
  float upd = (m / c.bc1) / denom;
  if (a.adam_w_mode) upd += wd * p;
  p -= lr * upd;
  return p;
}

template <typename TO, bool WRITE>
__global__ __launch_bounds__(256) void adam_k(float* __restrict__ master, TO* __restrict__ model,
                                              const float* __restrict__ grad,
                                              float* __restrict__ m, float* __restrict__ v,
                                              const int64_t* __restrict__ table, AdamArgs a) {
  AdamScal c{a.grad_scale, a.bc1, a.bc2};
  if (a.dev_state != nullptr) {
    if (a.dev_state[1] != 0.f) return;  // non-finite grad norm: skip the step
    const float step = a.dev_state[2];
    c.gs = a.dev_state[0];
    c.bc1 = 1.f - powf(a.beta1, step);
    c.bc2 = 1.f - powf(a.beta2, step);
  }
  const int64_t* row = table + 4 * (int64_t)blockIdx.x;
  const int64_t mo = row[0], bo = row[1], n = row[2];
  const int grp = (int)(row[3] & 0xFF);
  const float lr = a.lr[grp], wd = a.wd[grp];
  float* P = master + mo;
  float* M = m + mo;
  float* Vv = v + mo;
  const float* G = grad + bo;
  const int64_t n4 = n / 4;
  for (int64_t i = threadIdx.x; i < n4; i += blockDim.x) {
    float4 p = reinterpret_cast<float4*>(P)[i];
    const float4 g = reinterpret_cast<const float4*>(G)[i];
    float4 mm = reinterpret_cast<float4*>(M)[i];
    float4 vv = reinterpret_cast<float4*>(Vv)[i];
    adam_elem(p.x, g.x, mm.x, vv.x, lr, wd, a, c);
    adam_elem(p.y, g.y, mm.y, vv.y, lr, wd, a, c);
    adam_elem(p.z, g.z, mm.z, vv.z, lr, wd, a, c);
    adam_elem(p.w, g.w, mm.w, vv.w, lr, wd, a, c);
    reinterpret_cast<float4*>(P)[i] = p;
    reinterpret_cast<float4*>(M)[i] = mm;
    reinterpret_cast<float4*>(Vv)[i] = vv;
    if (WRITE) store4<TO>(model + bo + 4 * i, p.x, p.y, p.z, p.w);
  }
  for (int64_t i = n4 * 4 + threadIdx.x; i < n; i += blockDim.x) {
    float p = P[i], mm = M[i], vv = Vv[i];
    adam_elem(p, G[i], mm, vv, lr, wd, a, c);
    P[i] = p;
    M[i] = mm;
    Vv[i] = vv;
    if (WRITE) model[bo + i] = from_f<TO>(p);
  }
}

__global__ void opt_prep_k(const float* __restrict__ norm_sq, const float* __restrict__ inv_scale,
                           float clip, float* __restrict__ st) {
  if (threadIdx.x != 0) return;
  const float raw = norm_sq[0];
  const bool bad = !isfinite(raw);
  const float inv = inv_scale != nullptr ? inv_scale[0] : 1.f;
  const float gn = sqrtf(raw) * inv;
  float coef = 1.f;
  if (clip > 0.f) {
    const float cc = clip / (gn + 1.0e-6f);
    if (cc < 1.f) coef = cc;
  }
  st[0] = bad ? 0.f : coef * inv;
  st[1] = bad ? 1.f : 0.f;
  st[2] = st[2] + (bad ? 0.f : 1.f);
  st[3] = bad ? __builtin_nanf("") : gn;
}

}  // namespace

void opt_prep(const float* norm_sq, const float* inv_scale, float clip, float* st, hipStream_t s) {
  hipLaunchKernelGGL(opt_prep_k, dim3(1), dim3(64), 0, s, norm_sq, inv_scale, clip, st);
}

void chunked_sumsq(const float* grad, const int64_t* table, int n_chunks, float* partial,
                   float* out, hipStream_t s) {
  hipLaunchKernelGGL(sumsq_chunks_k, dim3(n_chunks), dim3(256), 0, s, grad, table, partial);
  hipLaunchKernelGGL(sum_partials_k, dim3(1), dim3(1024), 0, s, partial, n_chunks, out);
}

void flat_adam(float* master, void* model_out, int model_dt, const float* grad, float* m,
               float* v, const int64_t* table, int n_chunks, const AdamArgs& a, hipStream_t s) {
  if (model_out == nullptr) {
    hipLaunchKernelGGL((adam_k<float, false>), dim3(n_chunks), dim3(256), 0, s, master,
                       (float*)nullptr, grad, m, v, table, a);
    return;
  }
  EMA_DISPATCH_FLOAT(model_dt, TO, hipLaunchKernelGGL((adam_k<TO, true>), dim3(n_chunks),
                                                      dim3(256), 0, s, master, (TO*)model_out,
                                                      grad, m, v, table, a));
}

}  // namespace ema
