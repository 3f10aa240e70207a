// Single-token decode attention for gfx950 (KV-cached generation, sq == 1).
//
// The training FlashAttention kernel is the wrong shape for decode: one query
// row per (batch, head) leaves a 256-row workgroup idle, GQA heads re-read
// their group's K/V, and a whole (batch, head) walks its cache serially on
// one CU.  Decode is a memory-bound stream of the K/V cache, so this kernel
// splits the KEYS instead ("flash-decoding"):
//
//   pass 1 (grid = key chunks x KV groups x head slices x batch): a 256-thread
//     workgroup takes 256 keys of one KV group and up to RH query heads of
//     that group (GQA heads share every K/V byte they read):
//       * scores: lane = key, its K row (hd x 16 bit) against the RH query
//         vectors held in LDS (fp32, broadcast reads);
//       * chunk softmax statistics per head (max, sum of exp2) through wave
//         shuffles and a 4-wave LDS step; p stored to LDS;
//       * P.V: lane = head-dim pair, V rows read coalesced (one 256-B row per
//         wave instruction at hd 128), the 4 waves' partial sums added in LDS;
//       -> unnormalised partial O and (max, sum) per (chunk, head) in fp32.
//   pass 2 (one thread per output element group): rescale-and-sum the chunk
//     partials in chunk order (deterministic) and write O.
//
// With a device-side key count (DecodeParams::kv_len) the launch is
// independent of the step, so the whole decode step can be captured once in
// a hipGraph and replayed (inference/hip_graph.py).
//
// Used when it beats the FlashAttention forward on one query row (ops/attention.py
// flash_attn_func): GQA/MQA (r >= 2: each K/V byte is read once, not r times)
// and small grids (nq * b < 256); MHA with a full grid stays on FlashAttention
// (profiles/r2c_decode_bench.txt).  LDS-staging the K chunk (coalesced loads)
// was tried and lost: 82 KiB of LDS leaves one workgroup per CU.
//
// Reference: megatron/text_generation/forward_step.py drives the per-token
// forward; the reference decodes through the training attention path.
#include <type_traits>

#include "common.h"
#include "fa_common.h"
#include "kernels.h"

namespace ema {
namespace {

constexpr int DCH = 256;  // keys per chunk (= threads per workgroup)
// RH: query heads per workgroup = min(8, heads per KV group) rounded up to a
// power of two (MHA: 1, so no lane computes scores for absent heads)

template <typename T, int HD, int RH>
__global__ __launch_bounds__(256) void decode_partial_k(const DecodeParams p) {
  constexpr int HP = HD / 64;  // head-dim elements per lane in P.V (1 or 2)
  typedef typename fa::MT<T>::x8 x8;
  // HP consecutive 16-bit values of one V row (one dword at hd 128)
  typedef typename std::conditional<HP == 2, uint32_t, uint16_t>::type vpair;
  __shared__ float qs[RH][HD];
  __shared__ float ps[RH][DCH];
  __shared__ float red[4][RH];
  __shared__ float pacc[4][RH][HD];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = blockIdx.x;
  const int r = p.nq / p.nkv, nhs = (r + RH - 1) / RH;
  const int g = blockIdx.y / nhs, hs = blockIdx.y % nhs, b = blockIdx.z;
  const int h0 = hs * RH, nh = min(RH, r - h0);  // heads g*r + h0 .. + nh - 1
  const int k0 = chunk * DCH;
  const int sk = p.kv_len ? min(*p.kv_len, p.sk) : p.sk;
  const int nk = min(DCH, sk - k0);
  const float sl2 = p.scale * 1.4426950408889634f;
  const int nsplit = gridDim.x;
  if (nk <= 0) {  // chunk past the cached length (hipGraph decode): empty partial
    for (int i = tid; i < nh * HD; i += 256) {
      const int head = g * r + h0 + i / HD;
      p.ws_o[(((int64_t)b * p.nq + head) * nsplit + chunk) * HD + i % HD] = 0.f;
    }
    if (tid < nh) {
      const int64_t idx = ((int64_t)b * p.nq + g * r + h0 + tid) * nsplit + chunk;
      p.ws_ml[2 * idx] = -INFINITY;
      p.ws_ml[2 * idx + 1] = 0.f;
    }
    return;
  }

  // Every global load of the chunk is issued before anything waits: this
  // lane's K row (scores, lane = key), the V rows of this wave's keys (P.V,
  // lane = head-dim pair; rows past the length clamp to a valid one; all 64
  // for MHA) and the query vectors.  The earlier form waited out a load round trip
  // for Q, one for K and eight for V (8 rows in flight per lane), which made
  // this ~14 us kernel the largest non-GEMM cost of a decode step
  // (profiles/r3n_decode_b1_kernels.txt).
  const int key = k0 + (tid < nk ? tid : nk - 1);
  const T* krow = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)key * p.k_ss + (int64_t)g * p.k_sg;
  // (4-8 heads per workgroup: K is read inside the score loop, where the
  // scheduler does not hoist every query read beside 16 live K fragments)
  constexpr int KR = RH <= 2 ? HD / 8 : 1;
  x8 kv[KR];
  if constexpr (RH <= 2) {
#pragma unroll
    for (int c = 0; c < HD / 8; ++c) kv[c] = fa::ld8(krow + 8 * c);
  }
  // V rows in flight per lane: all 64 for 1-2 heads per workgroup; with 4-8
  // heads (GQA / MQA slices) the score / P.V registers leave room for 8
  constexpr int VU = RH <= 2 ? 64 : 8;
  vpair vv[VU];
  const T* vbase = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg + HP * lane;
  auto load_v = [&](int u0) {
#pragma unroll
    for (int u = 0; u < VU; ++u) {
      const int kc = min(k0 + wave * 64 + u0 + u, k0 + nk - 1);
      vv[u] = *reinterpret_cast<const vpair*>(vbase + (int64_t)kc * p.v_ss);
    }
  };
  load_v(0);
  // query vectors of this slice -> LDS (fp32)
  for (int i = tid; i < RH * HD; i += 256) {
    const int j = i / HD, d = i % HD;
    float v = 0.f;
    if (j < nh) {
      const int hh = h0 + j;
      const T* q = (const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg + (int64_t)hh * p.q_sh;
      v = (float)q[d];
    }
    qs[j][d] = v;
  }
  __syncthreads();

  // scores: lane = key
  float s[RH];
#pragma unroll
  for (int j = 0; j < RH; ++j) s[j] = 0.f;
  if (RH <= 2 || tid < nk) {  // (the branch also bounds hipcc's hoisting of the query reads)
#pragma unroll
    for (int c = 0; c < HD / 8; ++c) {
      x8 kc8;
      if constexpr (RH <= 2) kc8 = kv[c];
      else kc8 = fa::ld8(krow + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float kf = (float)kc8[e];
#pragma unroll
        for (int j = 0; j < RH; ++j) s[j] = __builtin_fmaf(kf, qs[j][8 * c + e], s[j]);
      }
    }
  }
  // chunk max per head
#pragma unroll
  for (int j = 0; j < RH; ++j) {
    s[j] = tid < nk ? s[j] * sl2 : -INFINITY;
    float m = s[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) red[wave][j] = m;
  }
  __syncthreads();
  float mx[RH];
#pragma unroll
  for (int j = 0; j < RH; ++j) mx[j] = fmaxf(fmaxf(red[0][j], red[1][j]), fmaxf(red[2][j], red[3][j]));
  __syncthreads();  // red is reused for the sums
#pragma unroll
  for (int j = 0; j < RH; ++j) {
    const float pj = tid < nk ? __builtin_amdgcn_exp2f(s[j] - mx[j]) : 0.f;
    ps[j][tid] = pj;
    float l = pj;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
    if (lane == 0) red[wave][j] = l;
  }
  __syncthreads();

  // P.V: wave w takes keys w*64 .. w*64+63 of the chunk (p = 0 past the length)
  float acc[RH][HP];
#pragma unroll
  for (int j = 0; j < RH; ++j)
#pragma unroll
    for (int e = 0; e < HP; ++e) acc[j][e] = 0.f;
#pragma unroll 1
  for (int u0 = 0; u0 < 64; u0 += VU) {
    if (u0 > 0) load_v(u0);
#pragma unroll
    for (int u = 0; u < VU; ++u) {
      const int kc = wave * 64 + u0 + u;
#pragma unroll
      for (int j = 0; j < RH; ++j) {
        const float pj = ps[j][kc];
#pragma unroll
        for (int e = 0; e < HP; ++e) {
          const uint16_t bits = (uint16_t)(vv[u] >> (16 * e));
          acc[j][e] = __builtin_fmaf(pj, (float)__builtin_bit_cast(T, bits), acc[j][e]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RH; ++j)
#pragma unroll
    for (int e = 0; e < HP; ++e) pacc[wave][j][HP * lane + e] = acc[j][e];
  __syncthreads();

  if (nsplit == 1) {  // one chunk holds every key: normalise and write O here (no combine pass)
    for (int i = tid; i < nh * HD; i += 256) {
      const int j = i / HD, d = i % HD;
      const int head = g * r + h0 + j;
      const float l = red[0][j] + red[1][j] + red[2][j] + red[3][j];
      const float o = pacc[0][j][d] + pacc[1][j][d] + pacc[2][j][d] + pacc[3][j][d];
      ((T*)p.o)[(int64_t)b * p.o_sb + (int64_t)head * p.o_sh + d] = (T)(l > 0.f ? o / l : 0.f);
    }
    return;
  }
  // partial outputs: [b][nq][split][HD] plus (max, sum) per (b, head, split)
  for (int i = tid; i < nh * HD; i += 256) {
    const int j = i / HD, d = i % HD;
    const int head = g * r + h0 + j;
    const float o = pacc[0][j][d] + pacc[1][j][d] + pacc[2][j][d] + pacc[3][j][d];
    p.ws_o[(((int64_t)b * p.nq + head) * nsplit + chunk) * HD + d] = o;
  }
  if (tid < nh) {
    const int head = g * r + h0 + tid;
    const int64_t idx = ((int64_t)b * p.nq + head) * nsplit + chunk;
    p.ws_ml[2 * idx] = mx[tid];
    p.ws_ml[2 * idx + 1] = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
  }
}

// O[b, head, :] = sum_s o_s 2^(m_s - M) / sum_s l_s 2^(m_s - M); 4 elements per thread
template <typename T, int HD>
__global__ __launch_bounds__(256) void decode_combine_k(const DecodeParams p, int nsplit) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)p.b * p.nq * (HD / 4);
  if (t >= total) return;
  const int d4 = (int)(t % (HD / 4));
  const int64_t bh = t / (HD / 4);
  const int head = (int)(bh % p.nq), b = (int)(bh / p.nq);
  const float* ml = p.ws_ml + 2 * bh * nsplit;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ml[2 * s]);
  float L = 0.f, o[4] = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < nsplit; ++s) {
    const float w = ml[2 * s] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(ml[2 * s] - M);
    L += ml[2 * s + 1] * w;
    const float* os = p.ws_o + (bh * nsplit + s) * HD + 4 * d4;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = __builtin_fmaf(os[e], w, o[e]);
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  T* out = (T*)p.o + (int64_t)b * p.o_sb + (int64_t)head * p.o_sh + 4 * d4;
  typename fa::MT<T>::x4 w4;
#pragma unroll
  for (int e = 0; e < 4; ++e) w4[e] = (T)(o[e] * inv);
  *reinterpret_cast<typename fa::MT<T>::x4*>(out) = w4;
}

template <typename T, int HD, int RH>
void launch_partial(const DecodeParams& p, int nsplit, hipStream_t s) {
  const int r = p.nq / p.nkv, nhs = (r + RH - 1) / RH;
  hipLaunchKernelGGL((decode_partial_k<T, HD, RH>), dim3(nsplit, p.nkv * nhs, p.b), dim3(256), 0, s, p);
}

template <typename T, int HD>
void launch(const DecodeParams& p, hipStream_t s) {
  const int r = p.nq / p.nkv;
  const int nsplit = flash_decode_splits(p.sk);
  if (r >= 8) launch_partial<T, HD, 8>(p, nsplit, s);
  else if (r >= 4) launch_partial<T, HD, 4>(p, nsplit, s);
  else if (r >= 2) launch_partial<T, HD, 2>(p, nsplit, s);
  else launch_partial<T, HD, 1>(p, nsplit, s);
  if (nsplit == 1) return;  // the partial kernel wrote O
  const int64_t total = (int64_t)p.b * p.nq * (HD / 4);
  hipLaunchKernelGGL((decode_combine_k<T, HD>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     s, p, nsplit);
}

}  // namespace

int flash_decode_splits(int sk) { return (sk + DCH - 1) / DCH; }

void flash_decode(const DecodeParams& p, int dt, hipStream_t s) {
  if (dt == DT_BF16) {
    if (p.hd == 128) launch<bf16, 128>(p, s);
    else launch<bf16, 64>(p, s);
  } else {
    if (p.hd == 128) launch<fp16, 128>(p, s);
    else launch<fp16, 64>(p, s);
  }
}

}  // namespace ema
