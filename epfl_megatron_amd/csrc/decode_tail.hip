// Tail of one graphed greedy decode step (inference/hip_graph.py,
// GraphedGreedyDecoder), in ONE launch: per sequence the argmax over the
// vocabulary (first maximum, as torch.argmax), the next-token and history
// writes and the position increment; the last workgroup to finish advances
// the step index, the KV-cache slot and the valid-key count.  The eager form
// was seven launches (argmax, index_copy, copy, four adds: ~45 us per token at
// batch 1 with their graph seams, profiles/r4v_decode_b1_kernels.txt).
//
// Reference: megatron/text_generation/generation.py:179-264 samples on the
// host-driven loop (greedy = argmax of the last position's logits).
#include "common.h"
#include "kernels.h"

namespace ema {
namespace {

template <typename T>
struct Vec16;  // 16 bytes of T
template <>
struct Vec16<bf16> { typedef __attribute__((ext_vector_type(8))) unsigned short t; static constexpr int n = 8; };
template <>
struct Vec16<fp16> { typedef __attribute__((ext_vector_type(8))) unsigned short t; static constexpr int n = 8; };
template <>
struct Vec16<float> { typedef __attribute__((ext_vector_type(4))) float t; static constexpr int n = 4; };

template <typename T>
__device__ __forceinline__ float elem(const typename Vec16<T>::t& v, int e) {
  if constexpr (__is_same(T, float)) return v[e];
  else return (float)__builtin_bit_cast(T, (unsigned short)v[e]);
}

// (value, index) order of torch.argmax: larger value, then smaller index
__device__ __forceinline__ void take(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi)) {
    bv = v;
    bi = i;
  }
}

template <typename T>
__global__ __launch_bounds__(1024) void greedy_tail_k(const T* __restrict__ logits, int64_t ld, int V,
                                                     int64_t* tokens, int64_t* history,
                                                     int64_t hist_ld, int64_t* step_idx,
                                                     int64_t* pos, int64_t* slot, int* kv_len,
                                                     unsigned* counter) {
  typedef typename Vec16<T>::t vec;
  constexpr int NV = Vec16<T>::n;
  const int row = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const T* lr = logits + (int64_t)row * ld;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  // 16-B loads, 8 in flight per thread per round over 1024 threads (one
  // round covers a 32k fp32 vocabulary: the row is latency-, not
  // bandwidth-bound; ld and the row base are 16-B aligned: checked by the
  // host); the < NV tail element-wise
  constexpr int NT = 1024, UR = 8;
  const int nvec = V / NV;
  for (int v0 = tid; v0 < nvec; v0 += UR * NT) {
    vec x[UR];
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const int vi = v0 + u * NT;
      x[u] = vi < nvec ? reinterpret_cast<const vec*>(lr)[vi] : vec{};
    }
#pragma unroll
    for (int u = 0; u < UR; ++u) {
      const int vi = v0 + u * NT;
      if (vi < nvec) {
#pragma unroll
        for (int e = 0; e < NV; ++e) take(bv, bi, elem<T>(x[u], e), vi * NV + e);
      }
    }
  }
  for (int i = nvec * NV + tid; i < V; i += NT) take(bv, bi, (float)lr[i], i);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    take(bv, bi, ov, oi);
  }
  __shared__ float sv[NT / 64];
  __shared__ int si[NT / 64];
  if (lane == 0) {
    sv[wave] = bv;
    si[wave] = bi;
  }
  __syncthreads();
  if (tid != 0) return;
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) take(bv, bi, sv[w], si[w]);
  const int64_t s = *step_idx;
  tokens[row] = bi;
  history[(int64_t)row * hist_ld + s] = bi;
  pos[row] += 1;
  // every workgroup has read the step index (its history store used it)
  // before it arrives; the last one advances the shared counters and re-arms
  const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (prev == gridDim.x - 1) {
    *step_idx = s + 1;
    *slot += 1;
    *kv_len += 1;
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

void greedy_tail(const void* logits, int64_t ld, int V, int b, int dt, int64_t* tokens,
                 int64_t* history, int64_t hist_ld, int64_t* step_idx, int64_t* pos, int64_t* slot,
                 int* kv_len, unsigned* counter, hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, {
    hipLaunchKernelGGL((greedy_tail_k<T>), dim3((unsigned)b), dim3(1024), 0, s, (const T*)logits, ld,
                       V, tokens, history, hist_ld, step_idx, pos, slot, kv_len, counter);
  });
}

}  // namespace ema
