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
  if (nk <= 0) {  // chunk past the cached length (hipGraph decode): empty partial
    const int nsplit = gridDim.x;
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
  const int key = k0 + tid;
  float s[RH];
#pragma unroll
  for (int j = 0; j < RH; ++j) s[j] = 0.f;
  if (tid < nk) {
    const T* krow = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)key * p.k_ss + (int64_t)g * p.k_sg;
#pragma unroll
    for (int c = 0; c < HD / 8; ++c) {
      const typename fa::MT<T>::x8 kv = fa::ld8(krow + 8 * c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float kf = (float)kv[e];
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

  // P.V: wave w takes keys w*64 .. w*64+63 of the chunk, lane = head-dim pair
  float acc[RH][HP];
#pragma unroll
  for (int j = 0; j < RH; ++j)
#pragma unroll
    for (int e = 0; e < HP; ++e) acc[j][e] = 0.f;
  const T* vbase = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg + HP * lane;
  const int kend = min(64, nk - wave * 64);
  constexpr int U = 8;  // rows in flight per lane
  for (int kk0 = 0; kk0 < kend; kk0 += U) {
    float vf[U][HP];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kc = wave * 64 + min(kk0 + u, kend - 1);
      const T* vr = vbase + (int64_t)(k0 + kc) * p.v_ss;
#pragma unroll
      for (int e = 0; e < HP; ++e) vf[u][e] = (float)vr[e];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (kk0 + u < kend) {
        const int kc = wave * 64 + kk0 + u;
#pragma unroll
        for (int j = 0; j < RH; ++j) {
          const float pj = ps[j][kc];
#pragma unroll
          for (int e = 0; e < HP; ++e) acc[j][e] = __builtin_fmaf(pj, vf[u][e], acc[j][e]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < RH; ++j)
#pragma unroll
    for (int e = 0; e < HP; ++e) pacc[wave][j][HP * lane + e] = acc[j][e];
  __syncthreads();

  // partial outputs: [b][nq][split][HD] plus (max, sum) per (b, head, split)
  const int nsplit = gridDim.x;
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
