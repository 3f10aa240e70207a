// Single-token decode attention for gfx950 (KV-cached generation, sq == 1).
//
// The training FlashAttention kernel is the wrong shape for decode: one query
// row per (batch, head) leaves a 256-row workgroup idle, GQA heads re-read
// their group's K/V, and a whole (batch, head) walks its cache serially on
// one CU.  Decode is a memory-bound stream of the K/V cache, so this kernel
// splits the KEYS instead ("flash-decoding"):
//
//   pass 1 (grid = key chunks x KV groups x head slices x batch): a 256-thread
//     workgroup takes a chunk of keys of one KV group and up to RH query heads
//     of that group (GQA heads share every K/V byte they read):
//       * scores: K rows read coalesced (hd / 8 lanes per key row, 8 dims
//         each, against the same 8 dims of the RH query vectors in registers),
//         reduced over a row's lanes and gathered so that lane = key;
//       * chunk softmax statistics per head (max, sum of exp2) through wave
//         shuffles and a 4-wave LDS step; p stored to LDS;
//       * P.V: lane = head-dim pair, V rows read coalesced (one 256-B row per
//         wave instruction at hd 128), the 4 waves' partial sums added in LDS;
//       -> unnormalised partial O and (max, sum) per (chunk, head) in fp32.
//   combine: the last workgroup of a (batch, head slice) to finish (an
//     arrival counter, re-armed by that workgroup) rescales and sums the chunk
//     partials in chunk order (deterministic) and writes O: no second launch.
//   The chunk is 4 x KPW keys with KPW = 64 / 16 / 8 keys per wave, the
//   largest whose grid still covers the chip (batch-1 MHA at a few hundred
//   cached keys runs 8 keys per wave on 256 workgroups instead of 32).
//
// With a device-side key count (DecodeParams::kv_len) the launch is
// independent of the step, so the whole decode step can be captured once in
// a hipGraph and replayed (inference/hip_graph.py).
//
// Used when it beats the FlashAttention forward on one query row (ops/attention.py
// flash_attn_func): GQA/MQA (r >= 2: each K/V byte is read once, not r times)
// and small grids (nq * b < 256); MHA with a full grid stays on FlashAttention
// (profiles/r2c_decode_bench.txt).
//
// Reference: megatron/text_generation/forward_step.py drives the per-token
// forward; the reference decodes through the training attention path.
#include <type_traits>

#include "common.h"
#include "fa_common.h"
#include "kernels.h"

namespace ema {
namespace {

// RH: query heads per workgroup = min(8, heads per KV group) rounded up to a
// power of two (MHA: 1, so no lane computes scores for absent heads).
// KPW: keys per wave (chunk = 4 KPW keys per workgroup), picked per launch
// so that the grid covers the chip (decode_chunk).

template <typename T, int HD, int RH, int KPW>
__global__ __launch_bounds__(256) void decode_attn_k(const DecodeParams p) {
  constexpr int DCH = 4 * KPW;
  constexpr int HP = HD / 64;  // head-dim elements per lane in P.V (1 or 2)
  typedef typename fa::MT<T>::x8 x8;
  // HP consecutive 16-bit values of one V row (one dword at hd 128)
  typedef typename std::conditional<HP == 2, uint32_t, uint16_t>::type vpair;
  __shared__ float ps[RH][DCH];
  __shared__ float red[4][RH];
  __shared__ float pacc[4][RH][HD];
  __shared__ float qs[RH >= 4 ? RH : 1][HD];  // fp32 query vectors (lane = key scoring)
  __shared__ int last_sh;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = blockIdx.x;
  const int r = p.nq / p.nkv, nhs = (r + RH - 1) / RH;
  const int g = blockIdx.y / nhs, hs = blockIdx.y % nhs, b = blockIdx.z;
  const int h0 = hs * RH, nh = min(RH, r - h0);  // heads g*r + h0 .. + nh - 1
  const int k0 = chunk * DCH;
  const int sk = p.kv_len ? min(*p.kv_len, p.sk) : p.sk;
  const int nk = min(DCH, sk - k0);  // <= 0: chunk past the cached length (graph decode)
  const float sl2 = p.scale * 1.4426950408889634f;
  const int nsplit = gridDim.x;

  float mx[RH];
  if (nk > 0) {
    // Every global load of the chunk is issued before anything waits: the K
    // rows of this wave's KPW keys, their V rows (P.V: lane = head-dim pair;
    // rows past the length clamp to a valid one) and the query slices.  K is
    // read coalesced: one wave-instruction = KPI whole key rows, LPK = HD / 8
    // lanes per row holding 8 dims each.
    // (LK: 4-8 query heads per workgroup score lane = key against the query
    // vectors in LDS, reading the K row inside the score loop: the coalesced
    // form's 8 register-resident query slices and butterflies cost 2.5x there,
    // profiles/r4r_kpw.txt)
    constexpr bool LK = RH >= 4;
    constexpr int LPK = HD / 8, KPI = 64 / LPK, NI = LK ? 1 : KPW / KPI;
    static_assert(LK || (NI >= 1 && NI <= LPK), "keys per wave vs key rows per instruction");
    const int kl = lane / LPK, dc = LK ? 0 : 8 * (lane % LPK);
    const T* kbase = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg + dc;
    x8 kv[NI];
    if constexpr (!LK) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int kk = min(wave * KPW + i * KPI + kl, nk - 1);
        kv[i] = fa::ld8(kbase + (int64_t)(k0 + kk) * p.k_ss);
      }
    }
    // V rows in flight per lane: the whole wave's keys for 1-2 heads per
    // workgroup; with 4-8 heads the score / P.V registers leave room for 8
    constexpr int VU = (RH <= 2 || KPW <= 8) ? KPW : 8;
    vpair vv[VU];
    const T* vbase = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg + HP * lane;
    auto load_v = [&](int u0) {
#pragma unroll
      for (int u = 0; u < VU; ++u) {
        const int kc = min(k0 + wave * KPW + u0 + u, k0 + nk - 1);
        vv[u] = *reinterpret_cast<const vpair*>(vbase + (int64_t)kc * p.v_ss);
      }
    };
    load_v(0);
    x8 qv[LK ? 1 : RH];  // this lane's 8-dim slice of each query head (absent heads: zero)
    if constexpr (!LK) {
#pragma unroll
      for (int j = 0; j < RH; ++j) {
        const int hh = h0 + (j < nh ? j : 0);
        qv[j] = fa::ld8((const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg +
                        (int64_t)hh * p.q_sh + dc);
        if (j >= nh) qv[j] = x8{};
      }
    } else {
      for (int i = tid; i < RH * HD; i += 256) {
        const int j = i / HD, d = i % HD;
        qs[j][d] = j < nh ? (float)((const T*)p.q)[(int64_t)b * p.q_sb + (int64_t)g * p.q_sg +
                                                  (int64_t)(h0 + j) * p.q_sh + d] : 0.f;
      }
      __syncthreads();
    }

    // scores: one partial dot product per K instruction over the lane's 8
    // dims, summed over the LPK lanes of a key row by a transposing butterfly
    // (each stage halves the values a lane carries while NI > 1, then plain
    // xor steps) that leaves instruction m = (lane % LPK) / (LPK / NI) in the
    // lane; one gather hands lane L < KPW the score of the wave's key L
    float s[RH];
    if constexpr (LK) {
      const T* krow = kbase + (int64_t)(k0 + min(wave * KPW + lane, nk - 1)) * p.k_ss;
#pragma unroll
      for (int j = 0; j < RH; ++j) s[j] = 0.f;
      // (the branch and the 4-chunk rolled loop keep hipcc from hoisting all
      // RH x HD query reads ahead of the FMAs, which spills)
      if (lane < KPW && wave * KPW + lane < nk) {
#pragma unroll 1
        for (int c0 = 0; c0 < HD / 8; c0 += 4) {
          x8 kc8[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) kc8[c] = fa::ld8(krow + 8 * (c0 + c));
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float kf = (float)kc8[c][e];
#pragma unroll
              for (int j = 0; j < RH; ++j) s[j] = __builtin_fmaf(kf, qs[j][8 * (c0 + c) + e], s[j]);
            }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < (LK ? 0 : RH); ++j) {
      float v[NI];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        float d = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) d = __builtin_fmaf((float)kv[i][e], (float)qv[j][e], d);
        v[i] = d;
      }
#pragma unroll
      for (int st = 0; (LPK >> (st + 1)) >= 1; ++st) {
        const int o = LPK >> (st + 1), n = NI >> st;
        if (n > 1) {
          const bool hi = (lane & o) != 0;
#pragma unroll
          for (int m = 0; m < n / 2; ++m) {
            const float keep = hi ? v[m + n / 2] : v[m];
            const float send = hi ? v[m] : v[m + n / 2];
            v[m] = keep + __shfl_xor(send, o, 64);
          }
        } else {
          v[0] += __shfl_xor(v[0], o, 64);
        }
      }
      s[j] = __shfl(v[0], (lane % KPI) * LPK + (lane / KPI) * (LPK / NI), 64);
    }
    const int key = wave * KPW + lane;  // this lane's key within the chunk
    const bool kon = lane < KPW && key < nk;
    // chunk max per head
#pragma unroll
    for (int j = 0; j < RH; ++j) {
      s[j] = kon ? s[j] * sl2 : -INFINITY;
      float m = s[j];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      if (lane == 0) red[wave][j] = m;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < RH; ++j) mx[j] = fmaxf(fmaxf(red[0][j], red[1][j]), fmaxf(red[2][j], red[3][j]));
    __syncthreads();  // red is reused for the sums
#pragma unroll
    for (int j = 0; j < RH; ++j) {
      const float pj = kon ? __builtin_amdgcn_exp2f(s[j] - mx[j]) : 0.f;
      if (lane < KPW) ps[j][key] = pj;
      float l = pj;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o, 64);
      if (lane == 0) red[wave][j] = l;
    }
    __syncthreads();

    // P.V: wave w takes its keys w KPW .. w KPW + KPW - 1 (p = 0 past the length)
    float acc[RH][HP];
#pragma unroll
    for (int j = 0; j < RH; ++j)
#pragma unroll
      for (int e = 0; e < HP; ++e) acc[j][e] = 0.f;
#pragma unroll 1
    for (int u0 = 0; u0 < KPW; u0 += VU) {
      if (u0 > 0) load_v(u0);
#pragma unroll
      for (int u = 0; u < VU; ++u) {
        const int kc = wave * KPW + u0 + u;
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

    if (nsplit == 1) {  // one chunk holds every key: normalise and write O here
      for (int i = tid; i < nh * HD; i += 256) {
        const int j = i / HD, d = i % HD;
        const int head = g * r + h0 + j;
        const float l = red[0][j] + red[1][j] + red[2][j] + red[3][j];
        const float o = pacc[0][j][d] + pacc[1][j][d] + pacc[2][j][d] + pacc[3][j][d];
        ((T*)p.o)[(int64_t)b * p.o_sb + (int64_t)head * p.o_sh + d] = (T)(l > 0.f ? o / l : 0.f);
      }
      return;
    }
  }

  // chunk partials [b][nq][split][HD] and (max, sum) per (b, head, split);
  // chunks past the length leave an empty partial
  // The partials go out as write-through (agent-scope) stores, so they need no
  // release fence: drained (vmcnt 0) before the arrival is counted, and the
  // last workgroup of this (batch, head slice) to arrive acquires them (one
  // agent-scope acquire, then plain loads) and combines them: no second launch,
  // correct wherever the chunks ran (cdna_hip_programming.md, in-launch
  // split-K reduction).
  auto put = [](float* a, float v) { __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  for (int i = tid; i < nh * HD; i += 256) {
    const int j = i / HD, d = i % HD;
    const int head = g * r + h0 + j;
    const float o = nk > 0 ? pacc[0][j][d] + pacc[1][j][d] + pacc[2][j][d] + pacc[3][j][d] : 0.f;
    put(p.ws_o + (((int64_t)b * p.nq + head) * nsplit + chunk) * HD + d, o);
  }
  if (tid < nh) {
    const int head = g * r + h0 + tid;
    const int64_t idx = ((int64_t)b * p.nq + head) * nsplit + chunk;
    put(p.ws_ml + 2 * idx, nk > 0 ? mx[tid] : -INFINITY);
    put(p.ws_ml + 2 * idx + 1, nk > 0 ? red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid] : 0.f);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    unsigned* cnt = p.counters + (int64_t)b * gridDim.y + blockIdx.y;
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == (unsigned)nsplit - 1u;
    if (last) {
      // re-arm for the next launch (same stream: it starts after this one ends)
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    last_sh = last;
  }
  __syncthreads();
  if (!last_sh) return;
  // O = sum_s o_s 2^(m_s - M) / sum_s l_s 2^(m_s - M), splits in order
  // (deterministic); loads in batches of 8 independent splits
  for (int i = tid; i < nh * HD; i += 256) {
    const int j = i / HD, d = i % HD;
    const int head = g * r + h0 + j;
    const int64_t bh = (int64_t)b * p.nq + head;
    const float2* ml = reinterpret_cast<const float2*>(p.ws_ml) + bh * nsplit;
    const float* os = p.ws_o + bh * nsplit * HD + d;
    float M = -INFINITY;
    for (int s0 = 0; s0 < nsplit; s0 += 8) {
      float2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ml[min(s0 + u, nsplit - 1)];
#pragma unroll
      for (int u = 0; u < 8; ++u) M = fmaxf(M, v[u].x);
    }
    float L = 0.f, o = 0.f;
    for (int s0 = 0; s0 < nsplit; s0 += 8) {
      float2 v[8];
      float ov[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int sp = min(s0 + u, nsplit - 1);
        v[u] = ml[sp];
        ov[u] = os[(int64_t)sp * HD];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float w = (s0 + u >= nsplit || v[u].x == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(v[u].x - M);
        L = __builtin_fmaf(v[u].y, w, L);
        o = __builtin_fmaf(ov[u], w, o);
      }
    }
    ((T*)p.o)[(int64_t)b * p.o_sb + (int64_t)head * p.o_sh + d] = (T)(L > 0.f ? o / L : 0.f);
  }
}

// keys per wave (1-2 heads per workgroup): 64 when that grid covers the 256
// CUs, else 16 when its grid covers half of them, else 8
// (batch-1 MHA at 256 cached keys: 32 heads x 1 chunk of 256 left 224 CUs
// idle and each busy CU pulling 128 KiB; 16 keys per wave -> 128 workgroups)
int decode_kpw_auto(int b, int sk, int nq, int nkv) {
  const int r = nq / nkv, rh = r >= 8 ? 8 : r >= 4 ? 4 : r >= 2 ? 2 : 1;
  // 4-8 heads per workgroup score lane = key: fewer keys per wave idle lanes
  // (b = 1 GQA at 3000 keys: 29 us at 64, 53 at 16; profiles/r4s_kpw.txt)
  if (rh >= 4) return 64;
  const int64_t base = (int64_t)b * nkv * ((r + rh - 1) / rh);
  auto grid = [&](int kpw) { return base * ((sk + 4 * kpw - 1) / (4 * kpw)); };
  if (grid(64) >= 256) return 64;
  return grid(16) >= 128 ? 16 : 8;  // b = 1 MHA, 256 keys: 16 -> 7.0 us, 8 -> 7.4 (r4t_kpw)
}

template <typename T, int HD, int RH>
void launch_rh(const DecodeParams& p, int kpw, hipStream_t s) {
  const int r = p.nq / p.nkv, nhs = (r + RH - 1) / RH;
  const int nsplit = (p.sk + 4 * kpw - 1) / (4 * kpw);
  const dim3 grid(nsplit, p.nkv * nhs, p.b);
  if (kpw == 64) hipLaunchKernelGGL((decode_attn_k<T, HD, RH, 64>), grid, dim3(256), 0, s, p);
  else if (kpw == 16) hipLaunchKernelGGL((decode_attn_k<T, HD, RH, 16>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((decode_attn_k<T, HD, RH, 8>), grid, dim3(256), 0, s, p);
}

template <typename T, int HD>
void launch(const DecodeParams& p, hipStream_t s) {
  const int r = p.nq / p.nkv;
  const int kpw = p.kpw;
  if (r >= 8) launch_rh<T, HD, 8>(p, kpw, s);
  else if (r >= 4) launch_rh<T, HD, 4>(p, kpw, s);
  else if (r >= 2) launch_rh<T, HD, 2>(p, kpw, s);
  else launch_rh<T, HD, 1>(p, kpw, s);
}

}  // namespace

int flash_decode_kpw(int b, int sk, int nq, int nkv) { return decode_kpw_auto(b, sk, nq, nkv); }
int flash_decode_splits(int sk, int kpw) { return (sk + 4 * kpw - 1) / (4 * kpw); }
int flash_decode_counters(int b, int nq, int nkv) {
  const int r = nq / nkv, rh = r >= 8 ? 8 : r >= 4 ? 4 : r >= 2 ? 2 : 1;
  return b * nkv * ((r + rh - 1) / rh);
}

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
