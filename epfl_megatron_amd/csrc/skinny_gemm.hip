// Weight-streaming GEMM for decode-sized batches on gfx950, with the decode
// step's elementwise work fused into its prologue / epilogue:
//
//     Y[M, N] = f(norm(X)[M, K] · W[N, K]^T)        M <= 16, bf16/fp16, fp32 accumulate
//
// A token-by-token decode step multiplies a handful of rows by every weight
// of the model: the time is the weight stream from HBM.  hipBLASLt's skinny
// tiles reach ~3.2-3.9 TB/s on the Llama-2-7B projections
// (profiles/r2c_serve_decode_b8_kernel_stats.csv); here every CU streams with
// many loads in flight:
//   * workgroup = 8 waves (4 when K % 256 != 0) = 16 output features (rows of
//     W); wave w reduces the K slice [w K/8, (w+1) K/8) with v_mfma_f32_16x16x32 (A = 16 W rows x
//     32 k, B = the <= 16 X rows x 32 k; unused B columns are zero), 8 k-steps
//     of W loads issued ahead of their MFMAs;
//   * the per-wave partial 16 x 16 tiles are added through LDS and wave 0 writes
//     the M x 16 block of Y (fixed order: deterministic).
// Grid = N / 16 workgroups (256 .. 2000 on the 7B shapes).
//
// Fusions (one launch instead of a norm / rope / cache-write / GLU / residual
// kernel each; the numerics follow the unfused kernels' roundings):
//   * NORM: RMSNorm of X in the prologue.  Each wave sums the squares of the X
//     slice it streams anyway, the 8 partials meet in LDS, and every B operand
//     is formed as T(T(x * rstd) * g) — the rounding of rmsnorm_fwd_k.
//   * EPI_RES: Y = T(T(acc) + R), the residual add of the block.
//   * EPI_GLU: the 16 W rows are 8 "up" rows f0.. and the 8 matching "gate"
//     rows F + f0..; Y[m, f] = T(x1 * act(x2)) over the rounded pair (the
//     glu_fwd_k numerics); grid = F / 8.
//   * EPI_QKV: the fused GQA projection [ng, r+2, hd]: q and k heads get the
//     Meta-convention rotary embedding at the token's absolute position
//     (pairs 2i, 2i+1: inside one lane's 4 features), q goes to Y [M, nq*hd],
//     k and v straight into the KV cache slot (device-resident slot index, so
//     the step is graph-capturable).
// Shapes: M <= 16, N % 16 == 0, K % 128 == 0 (checked by the host).
#include <cstdlib>

#include "act_math.h"
#include "common.h"
#include "fa_common.h"
#include "kernels.h"

namespace ema {
namespace {

typedef __attribute__((ext_vector_type(4))) float f4;

enum { EPI_PLAIN = 0, EPI_RES = 1, EPI_GLU = 2, EPI_QKV = 3 };

template <typename T>
__device__ __forceinline__ f4 mfma16x16x32(typename fa::MT<T>::x8 a, typename fa::MT<T>::x8 b, f4 c) {
  if constexpr (__is_same(T, bf16)) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// W row fed to MFMA row r of workgroup n-block `blk`
template <int EPI>
__device__ __forceinline__ int64_t w_row(int blk, int r, int N) {
  if constexpr (EPI == EPI_GLU) return r < 8 ? (int64_t)blk * 8 + r : (int64_t)N + blk * 8 + (r - 8);
  else return (int64_t)blk * 16 + r;
}

template <typename T, int WAVES, bool NORM, int EPI, int ACT>
__global__ __launch_bounds__(64 * WAVES) void skinny_gemm_k(const SkinnyArgs p) {
  typedef typename fa::MT<T>::x8 x8;
  constexpr int U = 8;  // k-steps of loads in flight per wave
  __shared__ f4 part[WAVES][64];
  __shared__ float ssq[WAVES][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int M = p.M, N = p.N, K = p.K;
  const T* __restrict__ x = (const T*)p.x;
  const T* __restrict__ w = (const T*)p.w;
  const int kq = K / WAVES, kbeg = wave * kq;
  const int r = lane & 15, kc = 8 * (lane >> 4);  // fragment row / k offset of this lane
  const T* wr = w + w_row<EPI>(blockIdx.x, r, N) * K + kbeg + kc;
  const bool xon = r < M;
  const T* xr = x + (int64_t)(xon ? r : 0) * K + kbeg + kc;
  const int steps = kq / 32;

  float rs = 1.f;  // rstd of X row r (NORM)
  const T* gr = nullptr;
  if constexpr (NORM) {
    gr = (const T*)p.norm_w + kbeg + kc;
    float ss = 0.f;
    for (int s = 0; s < steps; ++s) {
      const x8 v = *reinterpret_cast<const x8*>(xr + 32 * s);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = (float)v[e];
        ss += f * f;
      }
    }
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (lane < 16) ssq[wave][lane] = ss;
    __syncthreads();
    float tot = 0.f;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) tot += ssq[i][r];  // fixed order
    rs = rsqrtf(tot / (float)K + p.eps);
  }
  // B operand: X (or its RMSNorm, rounded like rmsnorm_fwd_k) for k-step s
  auto bop = [&](const x8& v, int s) {
    if constexpr (!NORM) {
      return v;
    } else {
      const x8 g = *reinterpret_cast<const x8*>(gr + 32 * s);
      x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const T xn = (T)((float)v[e] * rs);
        o[e] = (T)((float)xn * (float)g[e]);
      }
      return o;
    }
  };

  f4 acc = {0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + U <= steps; s += U) {
    x8 a[U], bv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = __builtin_nontemporal_load(reinterpret_cast<const x8*>(wr + 32 * (s + u)));
      bv[u] = *reinterpret_cast<const x8*>(xr + 32 * (s + u));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x8 b = bop(bv[u], s + u);
      if (!xon) b = x8{};
      acc = mfma16x16x32<T>(a[u], b, acc);
    }
  }
  for (; s < steps; ++s) {
    const x8 a = __builtin_nontemporal_load(reinterpret_cast<const x8*>(wr + 32 * s));
    x8 b = bop(*reinterpret_cast<const x8*>(xr + 32 * s), s);
    if (!xon) b = x8{};
    acc = mfma16x16x32<T>(a, b, acc);
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave != 0) return;
  f4 t = part[0][lane];
#pragma unroll
  for (int i = 1; i < WAVES; ++i) t += part[i][lane];  // fixed order: deterministic
  // D layout: lane holds column m = lane & 15, rows (features) 4 (lane >> 4) + i
  const int m = lane & 15, nr = 4 * (lane >> 4);
  typename fa::MT<T>::x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (T)t[i];
  T* __restrict__ y = (T*)p.y;
  if constexpr (EPI == EPI_GLU) {
    // lanes 0-31 hold up rows 0-7, lanes 32-63 the gate rows of the same f
    typename fa::MT<T>::x4 gt;
#pragma unroll
    for (int i = 0; i < 4; ++i) gt[i] = (T)__shfl_xor((float)o[i], 32, 64);
    if (lane < 32 && m < M) {
      typename fa::MT<T>::x4 out;
#pragma unroll
      for (int i = 0; i < 4; ++i) out[i] = (T)((float)o[i] * act<ACT>((float)gt[i]));
      *reinterpret_cast<typename fa::MT<T>::x4*>(y + (int64_t)m * p.ldy + blockIdx.x * 8 + nr) = out;
    }
    return;
  }
  if (m >= M) return;
  const int n = blockIdx.x * 16 + nr;
  if constexpr (EPI == EPI_RES) {
    const typename fa::MT<T>::x4 rv =
        *reinterpret_cast<const typename fa::MT<T>::x4*>((const T*)p.res + (int64_t)m * p.ldr + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (T)((float)o[i] + (float)rv[i]);
  }
  if constexpr (EPI == EPI_QKV) {
    const int hd = p.hd, per_g = (p.r + 2) * hd;
    const int g = n / per_g, rem = n - g * per_g, h = rem / hd, d = rem - h * hd;
    if (h <= p.r) {  // q heads and the k head: rotate pairs (d, d+1), (d+2, d+3)
      const int64_t pos = p.pos[(int64_t)m * p.pos_sb];
      const float* cr = p.cos + pos * (hd / 2) + d / 2;
      const float* sr = p.sin + pos * (hd / 2) + d / 2;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float x0 = (float)o[2 * j], x1 = (float)o[2 * j + 1], c = cr[j], sn = sr[j];
        o[2 * j] = (T)(x0 * c - x1 * sn);
        o[2 * j + 1] = (T)(x0 * sn + x1 * c);
      }
    }
    T* dst;
    if (h < p.r) {
      dst = y + (int64_t)m * p.ldy + (int64_t)(g * p.r + h) * hd + d;
    } else {
      const int64_t slot = p.slot_ptr ? *p.slot_ptr : p.slot;
      T* cache = (T*)(h == p.r ? p.kcache : p.vcache);
      dst = cache + slot * p.c_ss + (int64_t)m * p.c_sb + (int64_t)g * hd + d;
    }
    *reinterpret_cast<typename fa::MT<T>::x4*>(dst) = o;
    return;
  }
  *reinterpret_cast<typename fa::MT<T>::x4*>(y + (int64_t)m * p.ldy + n) = o;
}

template <typename T, int WAVES, bool NORM, int EPI, int ACT>
void launch(const SkinnyArgs& p, hipStream_t s) {
  const dim3 grid((unsigned)(EPI == EPI_GLU ? p.N / 8 : p.N / 16));
  hipLaunchKernelGGL((skinny_gemm_k<T, WAVES, NORM, EPI, ACT>), grid, dim3(64 * WAVES), 0, s, p);
}

template <typename T, int WAVES>
void dispatch(const SkinnyArgs& p, int epi, hipStream_t s) {
  const bool nm = p.norm_w != nullptr;
  switch (epi) {
    case EPI_RES:
      nm ? launch<T, WAVES, true, EPI_RES, 0>(p, s) : launch<T, WAVES, false, EPI_RES, 0>(p, s);
      break;
    case EPI_QKV:
      nm ? launch<T, WAVES, true, EPI_QKV, 0>(p, s) : launch<T, WAVES, false, EPI_QKV, 0>(p, s);
      break;
    case EPI_GLU:
      switch (p.act) {
        case 0: nm ? launch<T, WAVES, true, EPI_GLU, 0>(p, s) : launch<T, WAVES, false, EPI_GLU, 0>(p, s); break;
        case 1: nm ? launch<T, WAVES, true, EPI_GLU, 1>(p, s) : launch<T, WAVES, false, EPI_GLU, 1>(p, s); break;
        case 2: nm ? launch<T, WAVES, true, EPI_GLU, 2>(p, s) : launch<T, WAVES, false, EPI_GLU, 2>(p, s); break;
        default: nm ? launch<T, WAVES, true, EPI_GLU, 3>(p, s) : launch<T, WAVES, false, EPI_GLU, 3>(p, s); break;
      }
      break;
    default:
      nm ? launch<T, WAVES, true, EPI_PLAIN, 0>(p, s) : launch<T, WAVES, false, EPI_PLAIN, 0>(p, s);
  }
}

}  // namespace

bool skinny_gemm_supported(int64_t M, int64_t N, int64_t K) {
  return M >= 1 && M <= 16 && N % 16 == 0 && K % 128 == 0 && N > 0 && K > 0 &&
         N * K < ((int64_t)1 << 40);
}

// 8 waves (K split 8 ways) where K allows: twice the loads in flight per CU
// of the 4-wave form, which left the N = 4096 projections (one workgroup per
// CU) latency-bound at ~3.2 TB/s.  EMA_SKINNY_WAVES=4 forces the 4-wave form.
void skinny_gemm_ex(const SkinnyArgs& p, int epi, int dt, hipStream_t s) {
  static const int want = [] {
    const char* e = getenv("EMA_SKINNY_WAVES");
    return e ? atoi(e) : 8;
  }();
  const bool w8 = want == 8 && p.K % 256 == 0;
  if (dt == DT_BF16) w8 ? dispatch<bf16, 8>(p, epi, s) : dispatch<bf16, 4>(p, epi, s);
  else w8 ? dispatch<fp16, 8>(p, epi, s) : dispatch<fp16, 4>(p, epi, s);
}

void skinny_gemm(const void* x, const void* w, void* y, int64_t M, int64_t N, int64_t K, int dt,
                 hipStream_t s) {
  SkinnyArgs p{};
  p.x = x; p.w = w; p.y = y;
  p.M = (int)M; p.N = (int)N; p.K = (int)K; p.ldy = N;
  skinny_gemm_ex(p, EPI_PLAIN, dt, s);
}

}  // namespace ema
