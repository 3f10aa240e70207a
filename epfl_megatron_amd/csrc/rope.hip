// In-place rotary embedding on the fused GQA QKV tensor [s, b, ng, r+2, hd].
//
// Meta-Llama convention: pairs (x[2i], x[2i+1]) rotate by angle pos * theta_i,
// computed in fp32 from a device-resident cos/sin table [max_pos, hd/2]
// (reference megatron/model/positional_embeddings.py:24-51).  The r query
// heads and the single key head of every group are rotated; v is untouched.
// Each thread handles 8 consecutive elements (one 16-byte bf16 vector =
// 4 pairs); `inverse` applies R^T.  `k_only` rotates just the key head of
// every group: the training path rotates Q inside the FlashAttention forward
// and un-rotates dQ/dK in the FlashAttention backward epilogues, so only K
// needs this pass there.
#include "common.h"
#include "kernels.h"

namespace ema {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void rope_k(T* __restrict__ qkv, const float* __restrict__ cosT,
                                              const float* __restrict__ sinT,
                                              const int64_t* __restrict__ pos, int64_t pos_sb,
                                              int S, int B, int G, int R, int HD, int64_t ss,
                                              int64_t sb, int64_t sg, int64_t sh, int offset,
                                              int inverse, int k_only, int64_t total) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int nv = HD / 8;                 // 8-element vectors per head
  const int d8 = (int)(t % nv);
  int64_t rest = t / nv;
  const int nh = k_only ? 1 : R + 1;
  const int h = (k_only ? R : 0) + (int)(rest % nh);  // 0..R-1 query heads, R = key head
  rest /= nh;
  const int g = (int)(rest % G);
  rest /= G;
  const int b = (int)(rest % B);
  const int s = (int)(rest / B);
  const int64_t p = pos ? pos[(int64_t)b * pos_sb + s] : (int64_t)(s + offset);
  T* ptr = qkv + (int64_t)s * ss + (int64_t)b * sb + (int64_t)g * sg + (int64_t)h * sh + d8 * 8;
  const float* cr = cosT + p * (HD / 2) + d8 * 4;
  const float* sr = sinT + p * (HD / 2) + d8 * 4;
  const float4 c = *reinterpret_cast<const float4*>(cr);
  float4 sn = *reinterpret_cast<const float4*>(sr);
  if (inverse) {
    sn.x = -sn.x; sn.y = -sn.y; sn.z = -sn.z; sn.w = -sn.w;
  }
  const float cc[4] = {c.x, c.y, c.z, c.w};
  const float ssn[4] = {sn.x, sn.y, sn.z, sn.w};
  if constexpr (sizeof(T) == 2) {
    V16<T> v = ld16(ptr);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x0 = to_f(v.v[2 * i]), x1 = to_f(v.v[2 * i + 1]);
      v.v[2 * i] = from_f<T>(x0 * cc[i] - x1 * ssn[i]);
      v.v[2 * i + 1] = from_f<T>(x0 * ssn[i] + x1 * cc[i]);
    }
    st16(ptr, v);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x0 = to_f(ptr[2 * i]), x1 = to_f(ptr[2 * i + 1]);
      ptr[2 * i] = from_f<T>(x0 * cc[i] - x1 * ssn[i]);
      ptr[2 * i + 1] = from_f<T>(x0 * ssn[i] + x1 * cc[i]);
    }
  }
}

}  // namespace

void rope_qkv_inplace(void* qkv, const float* cos, const float* sin, const int64_t* pos,
                      int64_t pos_stride_b, int S, int B, int G, int R, int HD, int64_t ss,
                      int64_t sb, int64_t sg, int64_t sh, int offset, int inverse, int k_only,
                      int dt, hipStream_t s) {
  const int64_t total = (int64_t)S * B * G * (k_only ? 1 : R + 1) * (HD / 8);
  if (total == 0) return;
  const int64_t blocks = (total + 255) / 256;
  EMA_DISPATCH_FLOAT(dt, T, hipLaunchKernelGGL((rope_k<T>), dim3(blocks), dim3(256), 0, s,
                                               (T*)qkv, cos, sin, pos, pos_stride_b, S, B, G, R,
                                               HD, ss, sb, sg, sh, offset, inverse, k_only, total));
}

}  // namespace ema
