// Weight-streaming GEMM for decode-sized batches on gfx950:
//
//     Y[M, N] = X[M, K] · W[N, K]^T        M <= 16, bf16/fp16, fp32 accumulate
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
// Shapes: M <= 16, N % 16 == 0, K % 128 == 0 (checked by the host).
#include <cstdlib>

#include "common.h"
#include "fa_common.h"
#include "kernels.h"

namespace ema {
namespace {

typedef __attribute__((ext_vector_type(4))) float f4;

template <typename T>
__device__ __forceinline__ f4 mfma16x16x32(typename fa::MT<T>::x8 a, typename fa::MT<T>::x8 b, f4 c) {
  if constexpr (__is_same(T, bf16)) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <typename T, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void skinny_gemm_k(const T* __restrict__ x,
                                                            const T* __restrict__ w,
                                                            T* __restrict__ y, int M, int N, int K) {
  typedef typename fa::MT<T>::x8 x8;
  constexpr int U = 8;  // k-steps of loads in flight per wave
  __shared__ f4 part[WAVES][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const int kq = K / WAVES, kbeg = wave * kq;
  const int r = lane & 15, kc = 8 * (lane >> 4);  // fragment row / k offset of this lane
  const T* wr = w + (int64_t)(n0 + r) * K + kbeg + kc;
  const bool xon = r < M;
  const T* xr = x + (int64_t)(xon ? r : 0) * K + kbeg + kc;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int steps = kq / 32;
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
      if (!xon) bv[u] = x8{};
      acc = mfma16x16x32<T>(a[u], bv[u], acc);
    }
  }
  for (; s < steps; ++s) {
    const x8 a = __builtin_nontemporal_load(reinterpret_cast<const x8*>(wr + 32 * s));
    x8 bv = *reinterpret_cast<const x8*>(xr + 32 * s);
    if (!xon) bv = x8{};
    acc = mfma16x16x32<T>(a, bv, acc);
  }
  part[wave][lane] = acc;
  __syncthreads();
  if (wave == 0) {
    f4 t = part[0][lane];
#pragma unroll
    for (int i = 1; i < WAVES; ++i) t += part[i][lane];  // fixed order: deterministic
    // D layout: lane holds column m = lane & 15, rows 4 (lane >> 4) + i
    const int m = lane & 15, nr = 4 * (lane >> 4);
    if (m < M) {
      typename fa::MT<T>::x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (T)t[i];
      *reinterpret_cast<typename fa::MT<T>::x4*>(y + (int64_t)m * N + n0 + nr) = o;
    }
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
void skinny_gemm(const void* x, const void* w, void* y, int64_t M, int64_t N, int64_t K, int dt,
                 hipStream_t s) {
  static const int want = [] {
    const char* e = getenv("EMA_SKINNY_WAVES");
    return e ? atoi(e) : 8;
  }();
  const bool w8 = want == 8 && K % 256 == 0;
  const dim3 grid((unsigned)(N / 16));
  if (dt == DT_BF16) {
    if (w8)
      hipLaunchKernelGGL((skinny_gemm_k<bf16, 8>), grid, dim3(512), 0, s, (const bf16*)x,
                         (const bf16*)w, (bf16*)y, (int)M, (int)N, (int)K);
    else
      hipLaunchKernelGGL((skinny_gemm_k<bf16, 4>), grid, dim3(256), 0, s, (const bf16*)x,
                         (const bf16*)w, (bf16*)y, (int)M, (int)N, (int)K);
  } else {
    if (w8)
      hipLaunchKernelGGL((skinny_gemm_k<fp16, 8>), grid, dim3(512), 0, s, (const fp16*)x,
                         (const fp16*)w, (fp16*)y, (int)M, (int)N, (int)K);
    else
      hipLaunchKernelGGL((skinny_gemm_k<fp16, 4>), grid, dim3(256), 0, s, (const fp16*)x,
                         (const fp16*)w, (fp16*)y, (int)M, (int)N, (int)K);
  }
}

}  // namespace ema
