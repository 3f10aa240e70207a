// Fused scale -> mask -> softmax (non-flash attention path; reference kernels
// N1-N5, megatron/fused_kernels/scaled_*softmax*).  fp32 math, sk <= 8192.
//   mode 0: no mask;  mode 1: causal (col > row + (sk - sq) masked, written as 0);
//   mode 2: explicit mask [mb, 1, sq, sk], mb = b or 1 (a batch-broadcast mask
//           is indexed with batch stride 0, never expanded); true = masked ->
//           -10000 like the reference; a fully masked row produces zeros.
//
// Layout of the work:
//   * sk <= 1024: one wave64 per row, four rows per 256-thread workgroup; the
//     row's max and sum are two in-wave butterfly reductions (no LDS, no
//     barrier), so short rows do not leave 3/4 of a workgroup idle;
//   * 1024 < sk <= 8192: one 256-thread workgroup per row (LDS reduction);
//   * rows whose length is a multiple of 16 bytes move as 16-byte vectors (8
//     bf16 / fp16, 4 fp32) per lane and per access (CDNA guide G13), the mask
//     as 8 / 4 bytes; other lengths take the element-wise form.
#include "common.h"
#include "kernels.h"

namespace ema {
namespace {

constexpr float kMasked = -10000.f;

// Element e of lane's chunk k: column (k * STRIDE + t) * VN + e (VEC), else
// column k * STRIDE + t (one element per chunk).
template <typename T, int NC, bool VEC, int STRIDE>
struct RowIO {
  static constexpr int VN = VEC ? V16<T>::N : 1;
  float v[NC * VN];

  __device__ __forceinline__ static int col(int k, int e, int t) {
    return VEC ? (k * STRIDE + t) * VN + e : k * STRIDE + t;
  }

  // scaled, masked scores of the row (-inf past sk / causal limit)
  __device__ __forceinline__ void load(const T* xr, const uint8_t* mr, int sk, int limit,
                                       float scale, int t) {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c0 = col(k, 0, t);
      if constexpr (VEC) {
        V16<T> xv;
        uint8_t mv[VN];
        if (c0 < sk) {
          xv = ld16(xr + c0);
          if (mr) {
            if constexpr (VN == 8) *reinterpret_cast<uint2*>(mv) = *reinterpret_cast<const uint2*>(mr + c0);
            else *reinterpret_cast<uint32_t*>(mv) = *reinterpret_cast<const uint32_t*>(mr + c0);
          }
        }
#pragma unroll
        for (int e = 0; e < VN; ++e) {
          const int c = c0 + e;
          float val = -INFINITY;
          if (c < sk && c < limit) {
            val = to_f(xv.v[e]) * scale;
            if (mr && mv[e]) val = kMasked;
          }
          v[k * VN + e] = val;
        }
      } else {
        float val = -INFINITY;
        if (c0 < sk && c0 < limit) {
          val = to_f(xr[c0]) * scale;
          if (mr && mr[c0]) val = kMasked;
        }
        v[k] = val;
      }
    }
  }

  __device__ __forceinline__ void store(T* yr, int sk, float mul, int t) const {
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c0 = col(k, 0, t);
      if (c0 >= sk) continue;
      if constexpr (VEC) {
        V16<T> o;
#pragma unroll
        for (int e = 0; e < VN; ++e) o.v[e] = from_f<T>(v[k * VN + e] * mul);
        st16(yr + c0, o);
      } else {
        yr[c0] = from_f<T>(v[k] * mul);
      }
    }
  }
};

// Row reductions: in-wave (wave per row) or through LDS (workgroup per row).
template <bool WAVE>
__device__ __forceinline__ float row_max(float m, float* red) {
  return WAVE ? wave_max(m) : block_max(m, red);
}
template <bool WAVE>
__device__ __forceinline__ float row_sum(float s, float* red) {
  return WAVE ? wave_sum(s) : block_sum(s, red);
}

// WAVE: row = 4 * block + wave, t = lane; else row = block, t = thread.
template <typename T, int NC, bool VEC, bool WAVE>
__global__ __launch_bounds__(256) void softmax_fwd_k(const T* __restrict__ x,
                                                     const uint8_t* __restrict__ mask,
                                                     int64_t mask_bs, T* __restrict__ y,
                                                     int64_t rows, int64_t NP, int SQ, int SK,
                                                     float scale, int mode) {
  __shared__ float red[16];
  const int64_t row = WAVE ? (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6) : (int64_t)blockIdx.x;
  if (WAVE && row >= rows) return;  // whole wave: no barrier in the wave form
  const int t = WAVE ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  const int q = (int)(row % SQ);
  const int64_t b = row / (NP * SQ);
  const uint8_t* mr = (mode == 2) ? mask + b * mask_bs + (int64_t)q * SK : nullptr;
  const int limit = (mode == 1) ? q + 1 : SK;  // causal: square scores (sq == sk)
  RowIO<T, NC, VEC, WAVE ? 64 : 256> io;
  io.load(x + row * SK, mr, SK, limit, scale, t);
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < NC * io.VN; ++i) m = fmaxf(m, io.v[i]);
  m = row_max<WAVE>(m, red);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NC * io.VN; ++i) {
    const float e = io.v[i] == -INFINITY ? 0.f : __expf(io.v[i] - m);
    io.v[i] = e;
    s += e;
  }
  s = row_sum<WAVE>(s, red);
  const bool all_masked = (mode == 2) && (m == kMasked);
  io.store(y + row * SK, SK, all_masked ? 0.f : 1.f / s, t);
}

template <typename T, int NC, bool VEC, bool WAVE>
__global__ __launch_bounds__(256) void softmax_bwd_k(const T* __restrict__ dy, const T* __restrict__ y,
                                                     T* __restrict__ dx, int64_t rows, int SK,
                                                     float scale) {
  __shared__ float red[16];
  const int64_t row = WAVE ? (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6) : (int64_t)blockIdx.x;
  if (WAVE && row >= rows) return;
  const int t = WAVE ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
  RowIO<T, NC, VEC, WAVE ? 64 : 256> yv, dv;
  yv.load(y + row * SK, nullptr, SK, SK, 1.f, t);
  dv.load(dy + row * SK, nullptr, SK, SK, 1.f, t);
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < NC * yv.VN; ++i) {
    if (yv.v[i] == -INFINITY) yv.v[i] = dv.v[i] = 0.f;  // past the row end
    dot += yv.v[i] * dv.v[i];
  }
  dot = row_sum<WAVE>(dot, red);
#pragma unroll
  for (int i = 0; i < NC * yv.VN; ++i) yv.v[i] = yv.v[i] * (dv.v[i] - dot);
  yv.store(dx + row * SK, SK, scale, t);
}

// (chunks per lane, vector form, wave per row) for a row length; f(NC, VEC, WAVE)
template <typename T, typename F>
void dispatch(int SK, F&& f) {
  constexpr int VN = V16<T>::N;
  const bool vec = SK % VN == 0;
  if (SK <= 1024) {  // wave per row
    const int per_lane = (SK + 63) / 64;
    if (vec) {
      const int nc = (SK + 64 * VN - 1) / (64 * VN);
      if (nc <= 1) f(std::integral_constant<int, 1>{}, std::true_type{}, std::true_type{});
      else if (nc <= 2) f(std::integral_constant<int, 2>{}, std::true_type{}, std::true_type{});
      else f(std::integral_constant<int, 4>{}, std::true_type{}, std::true_type{});  // fp32 rows
    } else if (per_lane <= 2) {
      f(std::integral_constant<int, 2>{}, std::false_type{}, std::true_type{});
    } else if (per_lane <= 4) {
      f(std::integral_constant<int, 4>{}, std::false_type{}, std::true_type{});
    } else if (per_lane <= 8) {
      f(std::integral_constant<int, 8>{}, std::false_type{}, std::true_type{});
    } else {
      f(std::integral_constant<int, 16>{}, std::false_type{}, std::true_type{});
    }
  } else {  // workgroup per row
    if (vec) {
      const int nc = (SK + 256 * VN - 1) / (256 * VN);
      if (nc <= 1) f(std::integral_constant<int, 1>{}, std::true_type{}, std::false_type{});
      else if (nc <= 2) f(std::integral_constant<int, 2>{}, std::true_type{}, std::false_type{});
      else if (nc <= 4) f(std::integral_constant<int, 4>{}, std::true_type{}, std::false_type{});
      else f(std::integral_constant<int, 8>{}, std::true_type{}, std::false_type{});
    } else {
      const int ept = (SK + 255) / 256;
      if (ept <= 8) f(std::integral_constant<int, 8>{}, std::false_type{}, std::false_type{});
      else if (ept <= 16) f(std::integral_constant<int, 16>{}, std::false_type{}, std::false_type{});
      else f(std::integral_constant<int, 32>{}, std::false_type{}, std::false_type{});
    }
  }
}

}  // namespace

void softmax_fwd(const void* x, const uint8_t* mask, int64_t mask_bs, void* y, int64_t B,
                 int64_t NP, int SQ, int SK, float scale, int mode, int dt, hipStream_t s) {
  const int64_t rows = B * NP * SQ;
  EMA_DISPATCH_FLOAT(dt, T, dispatch<T>(SK, [&](auto nc, auto vec, auto wave) {
    constexpr int NC = decltype(nc)::value;
    constexpr bool VEC = decltype(vec)::value, WAVE = decltype(wave)::value;
    const dim3 grid((unsigned)(WAVE ? (rows + 3) / 4 : rows));
    hipLaunchKernelGGL((softmax_fwd_k<T, NC, VEC, WAVE>), grid, dim3(256), 0, s, (const T*)x,
                       mask, mask_bs, (T*)y, rows, NP, SQ, SK, scale, mode);
  }));
}

void softmax_bwd(const void* dy, const void* y, void* dx, int64_t rows, int SK, float scale,
                 int dt, hipStream_t s) {
  EMA_DISPATCH_FLOAT(dt, T, dispatch<T>(SK, [&](auto nc, auto vec, auto wave) {
    constexpr int NC = decltype(nc)::value;
    constexpr bool VEC = decltype(vec)::value, WAVE = decltype(wave)::value;
    const dim3 grid((unsigned)(WAVE ? (rows + 3) / 4 : rows));
    hipLaunchKernelGGL((softmax_bwd_k<T, NC, VEC, WAVE>), grid, dim3(256), 0, s, (const T*)dy,
                       (const T*)y, (T*)dx, rows, SK, scale);
  }));
}

}  // namespace ema
