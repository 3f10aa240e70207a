// Fused residual + dropout(x [+ x2] [+ bias]) for gfx950 — the reference's
// bias_dropout_add (megatron/model/transformer.py:538-578, TorchScript-fused
// there) and, with the second addend, the Falcon parallel block's
// residual + attn + mlp in one pass.
//
// Dropout bits come from counter-based Philox-4x32-10 keyed by the torch CUDA
// generator's (seed, offset) — the caller advances the generator's offset by
// the counters used, so the stream is deterministic per seed, advances like
// any other dropout and, inside the tensor-parallel RNG tracker's fork, differs
// per TP rank exactly as the reference's dropout does.  The backward
// REGENERATES the mask from the same (seed, offset): no mask tensor is stored.
//
// Memory bound: one thread = 8 elements (one 16-byte bf16 vector per operand),
// two Philox blocks per thread (4 uniforms each), fp32 math, one rounding.
#include "common.h"
#include "kernels.h"

namespace ema {
namespace {

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(uint64_t ctr, uint64_t offset, uint64_t seed) {
  uint32_t c0 = (uint32_t)ctr, c1 = (uint32_t)(ctr >> 32);
  uint32_t c2 = (uint32_t)offset, c3 = (uint32_t)(offset >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {  // Philox-4x32 round (Salmon et al., SC'11)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n1 = (uint32_t)p1;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    const uint32_t n3 = (uint32_t)p0;
    c0 = n0;
    c1 = n1;
    c2 = n2;
    c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

// keep element e (0..7) of the thread's vector: 8 uniforms from 2 Philox blocks
__device__ __forceinline__ void keep_mask(uint64_t vec_idx, uint64_t offset, uint64_t seed,
                                          uint32_t thresh, bool keep[8]) {
  const U4 a = philox(2 * vec_idx, offset, seed);
  const U4 b = philox(2 * vec_idx + 1, offset, seed);
  keep[0] = a.x >= thresh; keep[1] = a.y >= thresh; keep[2] = a.z >= thresh; keep[3] = a.w >= thresh;
  keep[4] = b.x >= thresh; keep[5] = b.y >= thresh; keep[6] = b.z >= thresh; keep[7] = b.w >= thresh;
}

template <typename T>
struct V8 {
  T v[8];
};

template <typename T>
__global__ __launch_bounds__(256) void bda_fwd_k(const T* __restrict__ x, const T* __restrict__ x2,
                                                 const T* __restrict__ bias,
                                                 const T* __restrict__ res, T* __restrict__ out,
                                                 int64_t nvec, int hvec, uint32_t thresh,
                                                 float scale, uint64_t seed, uint64_t offset) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const V8<T> xv = reinterpret_cast<const V8<T>*>(x)[i];
  const V8<T> rv = reinterpret_cast<const V8<T>*>(res)[i];
  V8<T> x2v, bv;
  if (x2) x2v = reinterpret_cast<const V8<T>*>(x2)[i];
  if (bias) bv = reinterpret_cast<const V8<T>*>(bias)[i % hvec];
  bool keep[8];
  if (thresh) keep_mask((uint64_t)i, offset, seed, thresh, keep);
  V8<T> o;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float a = to_f(xv.v[e]);
    if (x2) a += to_f(x2v.v[e]);
    if (bias) a += to_f(bv.v[e]);
    if (thresh) a = keep[e] ? a * scale : 0.f;
    o.v[e] = from_f<T>(to_f(rv.v[e]) + a);
  }
  reinterpret_cast<V8<T>*>(out)[i] = o;
}

template <typename T>
__global__ __launch_bounds__(256) void bda_bwd_k(const T* __restrict__ dout, T* __restrict__ dx,
                                                 int64_t nvec, uint32_t thresh, float scale,
                                                 uint64_t seed, uint64_t offset) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nvec) return;
  const V8<T> g = reinterpret_cast<const V8<T>*>(dout)[i];
  bool keep[8];
  keep_mask((uint64_t)i, offset, seed, thresh, keep);
  V8<T> o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o.v[e] = from_f<T>(keep[e] ? to_f(g.v[e]) * scale : 0.f);
  reinterpret_cast<V8<T>*>(dx)[i] = o;
}

}  // namespace

void bias_dropout_add_fwd(const void* x, const void* x2, const void* bias, const void* res,
                          void* out, int64_t n, int64_t h, float p, uint64_t seed, uint64_t offset,
                          int dt, hipStream_t s) {
  const int64_t nvec = n / 8;
  const uint32_t thresh = p > 0.f ? (uint32_t)fminf(p * 4294967296.f, 4294967295.f) : 0u;
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const dim3 grid((unsigned)((nvec + 255) / 256));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(bda_fwd_k<bf16>, grid, dim3(256), 0, s, (const bf16*)x, (const bf16*)x2,
                       (const bf16*)bias, (const bf16*)res, (bf16*)out, nvec, (int)(h / 8), thresh,
                       scale, seed, offset);
  else if (dt == DT_F16)
    hipLaunchKernelGGL(bda_fwd_k<fp16>, grid, dim3(256), 0, s, (const fp16*)x, (const fp16*)x2,
                       (const fp16*)bias, (const fp16*)res, (fp16*)out, nvec, (int)(h / 8), thresh,
                       scale, seed, offset);
}

void bias_dropout_add_bwd(const void* dout, void* dx, int64_t n, float p, uint64_t seed,
                          uint64_t offset, int dt, hipStream_t s) {
  const int64_t nvec = n / 8;
  const uint32_t thresh = (uint32_t)fminf(p * 4294967296.f, 4294967295.f);
  const float scale = 1.f / (1.f - p);
  const dim3 grid((unsigned)((nvec + 255) / 256));
  if (dt == DT_BF16)
    hipLaunchKernelGGL(bda_bwd_k<bf16>, grid, dim3(256), 0, s, (const bf16*)dout, (bf16*)dx, nvec,
                       thresh, scale, seed, offset);
  else if (dt == DT_F16)
    hipLaunchKernelGGL(bda_bwd_k<fp16>, grid, dim3(256), 0, s, (const fp16*)dout, (fp16*)dx, nvec,
                       thresh, scale, seed, offset);
}

}  // namespace ema
