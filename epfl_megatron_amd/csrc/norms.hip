// RMSNorm / LayerNorm forward + backward for gfx950.
//
// Layout: x[rows, H] row-major.  One wave64 owns one row; the row is held in
// registers as VPL 16-byte vectors per lane (VPL = ceil(H / (64 * 8)) for
// bf16), so x is read from HBM exactly once in forward and once in backward.
// 4 waves (256 threads) per workgroup -> rows/4 workgroups (>> 256 CUs for any
// training shape).  Statistics in fp32.
//
// Weight/bias gradients: each wave accumulates its rows' contribution for all
// H columns in registers, writes one fp32 partial row, and a second kernel
// sums the partials column-wise in a fixed order (deterministic, no atomics).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace ema {
namespace {

constexpr int kWaves = 4;
// backward grid cap: 2 workgroups (8 waves) per CU; more partial rows cost a
// little colsum traffic but keep twice the loads in flight.
constexpr int kBwdBlocks = 512;
constexpr int kLdsDwMaxH = 4096;  // 4 waves x H x fp32 <= 64 KB of LDS

// res != nullptr: the normalised input is s = x + res (rounded to T, as the
// reference's bf16 residual add), and s is written to sum_out (the residual
// stream for the next block) -- one pass instead of an add kernel + a norm.
// PREW (few rows: decode): the weight slices are loaded with x, before the
// row reduction, so the kernel makes one memory round trip instead of two; with
// many rows the extra registers would cost occupancy and w is L2-resident anyway.
template <typename T, int VPL, bool PREW>
__global__ __launch_bounds__(256) void rmsnorm_fwd_k(const T* __restrict__ x,
                                                     const T* __restrict__ res,
                                                     T* __restrict__ sum_out,
                                                     const T* __restrict__ w, T* __restrict__ y,
                                                     float* __restrict__ rstd_out, int64_t rows,
                                                     int H, float eps) {
  constexpr int N = V16<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = H / N;
  const T* xr = x + row * H;
  V16<T> xv[VPL], wpre[PREW ? VPL : 1];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (vi < nvec) {
      xv[i] = ld16(xr + vi * N);
      if constexpr (PREW) wpre[i] = ld16(w + vi * N);
      if (res) {
        const V16<T> rv = ld16(res + row * H + vi * N);
#pragma unroll
        for (int e = 0; e < N; ++e) xv[i].v[e] = from_f<T>(to_f(xv[i].v[e]) + to_f(rv.v[e]));
        st16(sum_out + row * H + vi * N, xv[i]);
      }
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const float f = to_f(xv[i].v[e]);
        ss += f * f;
      }
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)H + eps);
  if (lane == 0) rstd_out[row] = r;
  T* yr = y + row * H;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (vi < nvec) {
      V16<T> wv;
      if constexpr (PREW) wv = wpre[i];
      else wv = ld16(w + vi * N);
      V16<T> o;
#pragma unroll
      for (int e = 0; e < N; ++e) {
        // reference numerics: normalise in fp32, round to T, then multiply by w.
        const T xn = from_f<T>(to_f(xv[i].v[e]) * r);
        o.v[e] = from_f<T>(to_f(xn) * to_f(wv.v[e]));
      }
      st16(yr + vi * N, o);
    }
  }
}

// One wave per row, rows strided by the total wave count; the next row's x/dy
// are loaded before the current row is reduced (software pipeline), so HBM
// requests stay in flight across the wave_sum / store phase.  DRES adds the
// gradient of the residual branch (ds from the next block) into dx:
// dx = rmsnorm'(dy) + dres, saving the separate autograd add kernel.
//
// vmcnt discipline (gfx9 counts loads AND stores in one in-order counter):
// every global access of an iteration is unconditional and issued in the order
// [x,dy(row + nwaves)] [dres(row)] [dx stores(row)], and w / dW live in LDS, so
// phase 1 of a row never waits on the prefetch of the next one.
template <typename T, int VPL, bool R = false>
struct RowRegs {
  V16<T> x[VPL], g[VPL], r[R ? VPL : 1];
};

// R: the row's dres (residual-branch gradient) rides with x / dy, a row ahead
template <typename T, int VPL, bool FULL, bool R = false>
__device__ __forceinline__ void load_row(RowRegs<T, VPL, R>& rr, const T* __restrict__ x,
                                         const T* __restrict__ dy, int64_t row, int H, int lane,
                                         int nvec, const T* __restrict__ dres = nullptr) {
  constexpr int N = V16<T>::N;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (FULL || vi < nvec) {
      rr.x[i] = ld16(x + row * H + vi * N);
      rr.g[i] = ld16(dy + row * H + vi * N);
      if constexpr (R) rr.r[i] = ld16(dres + row * H + vi * N);
    }
  }
}

// w reads as one LLVM vector load.  Through the V16 struct, the DW+FULL
// variants had SROA slice each 16-B read into u16/b64/u16/b32 pieces (4 LDS ops,
// 2-byte aligned -> bank conflicts); a native vector type cannot be sliced.
template <typename T>
using lvec = T __attribute__((ext_vector_type(16 / sizeof(T))));
template <typename T>
__device__ __forceinline__ lvec<T> lds_ld16(const T* p) {
  return *static_cast<const lvec<T>*>(__builtin_assume_aligned(p, 16));
}

// RA: dres prefetched a row ahead with x / dy (EMA_RMS_DRES_AHEAD=0: fetched
// after the row's reduction, the round-4 form)
template <typename T, int VPL, bool DW, bool FULL, bool DRES, bool RA>
__device__ __forceinline__ void rms_bwd_row(const RowRegs<T, VPL, RA>& rr, RowRegs<T, VPL, RA>& nxt,
                                            int64_t nrow, const T* __restrict__ x,
                                            const T* __restrict__ dy, float* __restrict__ acc,
                                            const T* __restrict__ w_lds, float r,
                                            const T* __restrict__ dres, T* __restrict__ dx,
                                            int64_t row, int H, int lane, int nvec) {
  constexpr int N = V16<T>::N;
  static_assert(!RA || DRES, "dres ahead needs dres");
  load_row<T, VPL, FULL, RA>(nxt, x, dy, nrow, H, lane, nvec, dres);
  float dot = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (FULL || vi < nvec) {
      const lvec<T> wv = lds_ld16(w_lds + vi * N);
      float4 a[N / 4];
      if (DW) {
#pragma unroll
        for (int q = 0; q < N / 4; ++q) a[q] = *reinterpret_cast<const float4*>(acc + q * nvec * 4 + vi * 4);
      }
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const float xh = to_f(rr.x[i].v[e]) * r;
        const float g = to_f(rr.g[i].v[e]);
        dot += g * to_f(wv[e]) * xh;
        if (DW) reinterpret_cast<float*>(a)[e] += g * to_f(from_f<T>(xh));
      }
      if (DW) {
#pragma unroll
        for (int q = 0; q < N / 4; ++q) *reinterpret_cast<float4*>(acc + q * nvec * 4 + vi * 4) = a[q];
      }
    }
  }
  // dres is fetched only now (its 32 VGPRs would otherwise overlap the phase-1
  // temporaries and spill); the wait for it also covers the prefetch, which
  // has had all of phase 1 to land.
  V16<T> rv[DRES && !RA ? VPL : 1];
  if (DRES && !RA) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + i * 64;
      if (FULL || vi < nvec) rv[i] = ld16(dres + row * H + vi * N);
    }
  }
  dot = wave_sum(dot) / (float)H;
  T* dxr = dx + row * H;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (FULL || vi < nvec) {
      const lvec<T> wv = lds_ld16(w_lds + vi * N);
      V16<T> o;
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const float xh = to_f(rr.x[i].v[e]) * r;
        float v = r * (to_f(rr.g[i].v[e]) * to_f(wv[e]) - xh * dot);
        if constexpr (RA) v += to_f(rr.r[i].v[e]);
        else if (DRES) v += to_f(rv[i].v[e]);
        o.v[e] = from_f<T>(v);
      }
      st16(dxr + vi * N, o);
    }
  }
}

// LDS: w (H x T) then, with DW, one private fp32 dW row per wave (4 x H x 4 B;
// H <= 4096 -> <= 72 KB per workgroup).  Keeping dW in VGPRs next to the two
// row buffers pinned the kernel at 1 wave/SIMD.  The dW row is stored as N/4
// planes of float4 indexed [q][vi], so a wave's ds_read/write_b128 of it is 64
// consecutive 16-B slots (conflict-free; the natural [vi][q] order put lanes 32
// bytes apart: 2-way conflicts, 4.3 conflict cycles per LDS instruction in
// profiles/r1_llama7b_pmc_step.csv).
template <typename T, int VPL, bool DW, bool FULL, bool DRES, bool RA = false>
__global__ __launch_bounds__(256, DRES ? 1 : 2) void rmsnorm_bwd_k(const T* __restrict__ dy,
                                                        const T* __restrict__ x,
                                                        const T* __restrict__ w,
                                                        const float* __restrict__ rstd,
                                                        const T* __restrict__ dres,
                                                        T* __restrict__ dx,
                                                        float* __restrict__ dw_part, int64_t rows,
                                                        int H) {
  extern __shared__ __attribute__((aligned(16))) float dyn_lds[];
  constexpr int N = V16<T>::N;
  const int lane = threadIdx.x & 63;
  // wave-uniform row bookkeeping in SGPRs (rstd[row] becomes a scalar load)
  const int64_t gw = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
  const int64_t nwaves = (int64_t)gridDim.x * kWaves;
  const int nvec = H / N;
  T* w_lds = reinterpret_cast<T*>(dyn_lds);
  // H is a multiple of N (>= 8), so every wave's dW row starts 16-B aligned;
  // telling the compiler keeps the accesses ds_read/write_b128 (it otherwise
  // falls back to ds_read2_b64 and 2-byte pieces for w).
  float* acc = static_cast<float*>(__builtin_assume_aligned(
      dyn_lds + (H * sizeof(T) + 15) / 16 * 4 + (threadIdx.x >> 6) * H, 16));
  for (int j = threadIdx.x; j < nvec; j += 256)
    *static_cast<uint4*>(__builtin_assume_aligned(w_lds + j * N, 16)) =
        *reinterpret_cast<const uint4*>(w + j * N);
  if (DW) {
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + i * 64;
      if (FULL || vi < nvec)
#pragma unroll
        for (int q = 0; q < N / 4; ++q)
          *reinterpret_cast<float4*>(acc + q * nvec * 4 + vi * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();
  RowRegs<T, VPL, RA> a, b;
  int64_t row = gw;
  if (row < rows) load_row<T, VPL, FULL, RA>(a, x, dy, row, H, lane, nvec, dres);
  // prefetches past the last row re-read row rows-1 (kept unconditional)
  while (row < rows) {
    int64_t nrow = row + nwaves;
    rms_bwd_row<T, VPL, DW, FULL, DRES, RA>(a, b, nrow < rows ? nrow : rows - 1, x, dy, acc, w_lds,
                                        rstd[row], dres, dx, row, H, lane, nvec);
    row = nrow;
    if (row >= rows) break;
    nrow = row + nwaves;
    rms_bwd_row<T, VPL, DW, FULL, DRES, RA>(b, a, nrow < rows ? nrow : rows - 1, x, dy, acc, w_lds,
                                        rstd[row], dres, dx, row, H, lane, nvec);
    row = nrow;
  }
  if (!DW) return;
  // every lane only touches its own slots of acc (same vi mapping as the rows)
  float* part = dw_part + gw * H;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (FULL || vi < nvec)
#pragma unroll
      for (int q = 0; q < N / 4; ++q)
        *reinterpret_cast<float4*>(part + vi * N + 4 * q) =
            *reinterpret_cast<const float4*>(acc + q * nvec * 4 + vi * 4);
  }
}

// One row per workgroup iteration (the row split over the 256 threads, EV
// 16-B vectors each: H = 2048 EV for 16-bit types), rows strided by the grid,
// the next row's x / dy / dres prefetched while the current one is reduced.
// Registers stay ~100 per lane, so ~4 workgroups share a CU and keep 4x the
// loads of the one-wave-per-row kernel (2 waves per SIMD at 256 VGPRs) in
// flight.  The row's dot product crosses the 4 waves through a 2-slot LDS
// pair (one barrier per row); the dW partial of the workgroup's rows stays in
// registers (each thread owns the same columns on every row) and is written
// once as a partial row for the ordered column sum.
template <typename T, int EV, bool DRES>
__global__ __launch_bounds__(256) void rmsnorm_bwd_wg_k(const T* __restrict__ dy,
                                                        const T* __restrict__ x,
                                                        const T* __restrict__ w,
                                                        const float* __restrict__ rstd,
                                                        const T* __restrict__ dres,
                                                        T* __restrict__ dx,
                                                        float* __restrict__ dw_part, int64_t rows,
                                                        int H) {
  constexpr int N = V16<T>::N;
  __shared__ float red[2][4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  struct Row {
    V16<T> x[EV], g[EV], r[DRES ? EV : 1];
  };
  auto load = [&](Row& rr, int64_t row) {
#pragma unroll
    for (int e = 0; e < EV; ++e) {
      const int64_t o = row * H + (int64_t)(tid + 256 * e) * N;
      rr.x[e] = ld16(x + o);
      rr.g[e] = ld16(dy + o);
      if constexpr (DRES) rr.r[e] = ld16(dres + o);
    }
  };
  V16<T> wr[EV];
#pragma unroll
  for (int e = 0; e < EV; ++e) wr[e] = ld16(w + (tid + 256 * e) * N);
  float acc[EV][N];
#pragma unroll
  for (int e = 0; e < EV; ++e)
#pragma unroll
    for (int k = 0; k < N; ++k) acc[e][k] = 0.f;
  const int64_t G = gridDim.x;
  int par = 0;
  auto step = [&](const Row& cur, Row& nxt, int64_t row) {
    const int64_t nrow = row + G;
    if (nrow < rows) load(nxt, nrow);
    const float r = rstd[row];
    float dot = 0.f;
#pragma unroll
    for (int e = 0; e < EV; ++e)
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const float xh = to_f(cur.x[e].v[k]) * r;
        const float g = to_f(cur.g[e].v[k]);
        dot += g * to_f(wr[e].v[k]) * xh;
        acc[e][k] += g * to_f(from_f<T>(xh));
      }
    dot = wave_sum(dot);
    if (lane == 0) red[par][wv] = dot;
    __syncthreads();
    dot = (red[par][0] + red[par][1] + red[par][2] + red[par][3]) / (float)H;
    par ^= 1;
#pragma unroll
    for (int e = 0; e < EV; ++e) {
      V16<T> o;
#pragma unroll
      for (int k = 0; k < N; ++k) {
        const float xh = to_f(cur.x[e].v[k]) * r;
        float v = r * (to_f(cur.g[e].v[k]) * to_f(wr[e].v[k]) - xh * dot);
        if constexpr (DRES) v += to_f(cur.r[e].v[k]);
        o.v[k] = from_f<T>(v);
      }
      st16(dx + row * H + (int64_t)(tid + 256 * e) * N, o);
    }
  };
  Row a, b;
  int64_t row = blockIdx.x;
  if (row < rows) load(a, row);
  while (row < rows) {
    step(a, b, row);
    row += G;
    if (row >= rows) break;
    step(b, a, row);
    row += G;
  }
  float* part = dw_part + (int64_t)blockIdx.x * H;
#pragma unroll
  for (int e = 0; e < EV; ++e)
#pragma unroll
    for (int k = 0; k < N; k += 4)
      *reinterpret_cast<float4*>(part + (tid + 256 * e) * N + k) =
          make_float4(acc[e][k], acc[e][k + 1], acc[e][k + 2], acc[e][k + 3]);
}

template <typename T, int VPL>
__global__ __launch_bounds__(256) void layernorm_fwd_k(const T* __restrict__ x,
                                                       const T* __restrict__ res,
                                                       T* __restrict__ sum_out,
                                                       const T* __restrict__ w,
                                                       const T* __restrict__ b,
                                                       T* __restrict__ y, float* __restrict__ mean_out,
                                                       float* __restrict__ rstd_out, int64_t rows,
                                                       int H, float eps) {
  constexpr int N = V16<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nvec = H / N;
  const T* xr = x + row * H;
  V16<T> xv[VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (vi < nvec) {
      xv[i] = ld16(xr + vi * N);
      if (res) {
        const V16<T> rv = ld16(res + row * H + vi * N);
#pragma unroll
        for (int e = 0; e < N; ++e) xv[i].v[e] = from_f<T>(to_f(xv[i].v[e]) + to_f(rv.v[e]));
        st16(sum_out + row * H + vi * N, xv[i]);
      }
#pragma unroll
      for (int e = 0; e < N; ++e) s += to_f(xv[i].v[e]);
    }
  }
  const float mu = wave_sum(s) / (float)H;
  float var = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (vi < nvec) {
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const float d = to_f(xv[i].v[e]) - mu;
        var += d * d;
      }
    }
  }
  var = wave_sum(var) / (float)H;
  const float r = rsqrtf(var + eps);
  if (lane == 0) {
    mean_out[row] = mu;
    rstd_out[row] = r;
  }
  T* yr = y + row * H;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (vi < nvec) {
      const V16<T> wv = ld16(w + vi * N);
      V16<T> bv;
      if (b) bv = ld16(b + vi * N);
      V16<T> o;
#pragma unroll
      for (int e = 0; e < N; ++e) {
        float v = (to_f(xv[i].v[e]) - mu) * r * to_f(wv.v[e]);
        if (b) v += to_f(bv.v[e]);
        o.v[e] = from_f<T>(v);
      }
      st16(yr + vi * N, o);
    }
  }
}

template <typename T, int VPL, bool DW>
__global__ __launch_bounds__(256) void layernorm_bwd_k(const T* __restrict__ dy,
                                                       const T* __restrict__ x,
                                                       const T* __restrict__ w,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       const T* __restrict__ dres,
                                                       T* __restrict__ dx,
                                                       float* __restrict__ dw_part,
                                                       float* __restrict__ db_part, int64_t rows,
                                                       int H) {
  constexpr int N = V16<T>::N;
  const int lane = threadIdx.x & 63;
  const int64_t gw = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * kWaves;
  const int nvec = H / N;
  float aw[VPL][N], ab[VPL][N];
#pragma unroll
  for (int i = 0; i < VPL; ++i)
#pragma unroll
    for (int e = 0; e < N; ++e) aw[i][e] = ab[i][e] = 0.f;
  for (int64_t row = gw; row < rows; row += nwaves) {
    const float mu = mean[row], r = rstd[row];
    const T* xr = x + row * H;
    const T* dyr = dy + row * H;
    V16<T> xv[VPL], gv[VPL];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + i * 64;
      if (vi < nvec) {
        xv[i] = ld16(xr + vi * N);
        gv[i] = ld16(dyr + vi * N);
        const V16<T> wv = ld16(w + vi * N);
#pragma unroll
        for (int e = 0; e < N; ++e) {
          const float xh = (to_f(xv[i].v[e]) - mu) * r;
          const float g = to_f(gv[i].v[e]);
          const float gw_ = g * to_f(wv.v[e]);
          sg += gw_;
          sgx += gw_ * xh;
          if (DW) {
            aw[i][e] += g * xh;
            ab[i][e] += g;
          }
        }
      }
    }
    sg = wave_sum(sg) / (float)H;
    sgx = wave_sum(sgx) / (float)H;
    T* dxr = dx + row * H;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int vi = lane + i * 64;
      if (vi < nvec) {
        const V16<T> wv = ld16(w + vi * N);
        V16<T> rv;
        if (dres) rv = ld16(dres + row * H + vi * N);
        V16<T> o;
#pragma unroll
        for (int e = 0; e < N; ++e) {
          const float xh = (to_f(xv[i].v[e]) - mu) * r;
          float v = r * (to_f(gv[i].v[e]) * to_f(wv.v[e]) - sg - xh * sgx);
          if (dres) v += to_f(rv.v[e]);
          o.v[e] = from_f<T>(v);
        }
        st16(dxr + vi * N, o);
      }
    }
  }
  if (!DW) return;
  float* pw = dw_part + gw * H;
  float* pb = db_part + gw * H;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int vi = lane + i * 64;
    if (vi < nvec) {
#pragma unroll
      for (int e = 0; e < N; ++e) {
        pw[vi * N + e] = aw[i][e];
        pb[vi * N + e] = ab[i][e];
      }
    }
  }
}

// Column-parallel weight-gradient partials for large H (the fused kernels keep
// the dw accumulator in registers only while VPL <= 8): block (c, p) sums the
// rows of chunk p for 2048 columns; partial rows are reduced by colsum_k.
template <typename T, bool LN>
__global__ __launch_bounds__(256) void norm_dw_k(const T* __restrict__ dy, const T* __restrict__ x,
                                                 const float* __restrict__ mean,
                                                 const float* __restrict__ rstd,
                                                 float* __restrict__ dw_part,
                                                 float* __restrict__ db_part, int64_t rows, int H,
                                                 int64_t rows_per_chunk) {
  constexpr int N = V16<T>::N;
  const int col = (blockIdx.x * 256 + threadIdx.x) * N;
  if (col >= H) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = r0 + rows_per_chunk < rows ? r0 + rows_per_chunk : rows;
  float aw[N], ab[N];
#pragma unroll
  for (int e = 0; e < N; ++e) aw[e] = ab[e] = 0.f;
  for (int64_t row = r0; row < r1; ++row) {
    const float r = rstd[row];
    const float mu = LN ? mean[row] : 0.f;
    const V16<T> xv = ld16(x + row * H + col);
    const V16<T> gv = ld16(dy + row * H + col);
#pragma unroll
    for (int e = 0; e < N; ++e) {
      const float g = to_f(gv.v[e]);
      const float xh = (to_f(xv.v[e]) - mu) * r;
      aw[e] += g * (LN ? xh : to_f(from_f<T>(xh)));
      ab[e] += g;
    }
  }
#pragma unroll
  for (int e = 0; e < N; ++e) {
    dw_part[(int64_t)blockIdx.y * H + col + e] = aw[e];
    if (LN) db_part[(int64_t)blockIdx.y * H + col + e] = ab[e];
  }
}

// Column sums of a [P, H] fp32 partial matrix -> out[H] (type T), fixed order.
// Stage 1: grid (H/64, kSplits), 256 threads = 64 columns x 4 row-lanes; each
// block sums P/kSplits partial rows (coalesced 256-byte row segments) into
// part2[split, H].  Stage 2: one thread per column adds the kSplits values.
// (A one-thread-per-column loop over all P rows left ~4k threads on the whole
// chip and took ~0.5 ms per call in the first MI355X profile.)
constexpr int kSplits = 32;

__global__ __launch_bounds__(256) void colsum_stage1_k(const float* __restrict__ part,
                                                       float* __restrict__ part2, int P, int H) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int per = (P + kSplits - 1) / kSplits;
  const int r0 = blockIdx.y * per;
  const int r1 = r0 + per < P ? r0 + per : P;
  float acc = 0.f;
  if (col < H)
    for (int r = r0 + rg; r < r1; r += 4) acc += part[(int64_t)r * H + col];
  red[rg][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rg == 0 && col < H) {
    const int c = threadIdx.x & 63;
    part2[(int64_t)blockIdx.y * H + col] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// acc != nullptr: the column sums go straight into the parameter's fp32
// main_grad (= when !accumulate, += otherwise) — no bf16 rounding of the
// weight gradient and no separate accumulate kernel.
template <typename T>
__global__ __launch_bounds__(256) void colsum_stage2_k(const float* __restrict__ part2,
                                                       T* __restrict__ out, float* __restrict__ acc,
                                                       int accumulate, int H) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= H) return;
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < kSplits; ++p) s += part2[(int64_t)p * H + j];
  if (acc) acc[j] = accumulate ? acc[j] + s : s;
  else out[j] = from_f<T>(s);
}

// part holds P + kSplits rows: [0, P) stage-1 input, [P, P + kSplits) stage-2 input.
template <typename T>
void colsum(float* part, T* out, float* acc, int accumulate, int P, int H, hipStream_t s) {
  float* part2 = part + (int64_t)P * H;
  hipLaunchKernelGGL(colsum_stage1_k, dim3((H + 63) / 64, kSplits), dim3(256), 0, s, part,
                     part2, P, H);
  hipLaunchKernelGGL((colsum_stage2_k<T>), dim3((H + 255) / 256), dim3(256), 0, s, part2, out,
                     acc, accumulate, H);
}

template <typename T>
int vec_elems() { return 16 / sizeof(T); }

template <typename T>
int pick_vpl(int H) {
  const int per_lane = (H / vec_elems<T>() + 63) / 64;
  if (per_lane <= 1) return 1;
  if (per_lane <= 2) return 2;
  if (per_lane <= 4) return 4;
  if (per_lane <= 8) return 8;
  if (per_lane <= 12) return 12;
  if (per_lane <= 16) return 16;
  if (per_lane <= 32) return 32;
  return -1;
}

#define EMA_VPL_SWITCH(vpl, ...)                \
  switch (vpl) {                                \
    case 1: { constexpr int V = 1; __VA_ARGS__; break; }   \
    case 2: { constexpr int V = 2; __VA_ARGS__; break; }   \
    case 4: { constexpr int V = 4; __VA_ARGS__; break; }   \
    case 8: { constexpr int V = 8; __VA_ARGS__; break; }   \
    case 12: { constexpr int V = 12; __VA_ARGS__; break; } \
    case 16: { constexpr int V = 16; __VA_ARGS__; break; } \
    case 32: { constexpr int V = 32; __VA_ARGS__; break; } \
  }

}  // namespace

int norm_bwd_partials(int64_t rows) {
  int64_t blocks = (rows + kWaves - 1) / kWaves;
  if (blocks > kBwdBlocks) blocks = kBwdBlocks;
  if (blocks < 1) blocks = 1;
  return (int)blocks * kWaves;
}

int norm_bwd_workspace_rows(int64_t rows) { return norm_bwd_partials(rows) + kSplits; }

int norm_max_hidden(int dtype) { return dtype == DT_F32 ? 32 * 64 * 4 : 32 * 64 * 8; }

void rmsnorm_fwd(const void* x, const void* res, void* sum_out, const void* w, void* y,
                 float* rstd, int64_t rows, int H, float eps, int dt, hipStream_t s) {
  const int64_t blocks = (rows + kWaves - 1) / kWaves;
  EMA_DISPATCH_FLOAT(dt, T, {
    const int vpl = pick_vpl<T>(H);
    if (rows <= 64 && vpl <= 8) {
      EMA_VPL_SWITCH(vpl, hipLaunchKernelGGL((rmsnorm_fwd_k<T, V, true>), dim3(blocks), dim3(256), 0,
                                             s, (const T*)x, (const T*)res, (T*)sum_out,
                                             (const T*)w, (T*)y, rstd, rows, H, eps));
    } else {
      EMA_VPL_SWITCH(vpl, hipLaunchKernelGGL((rmsnorm_fwd_k<T, V, false>), dim3(blocks), dim3(256), 0,
                                             s, (const T*)x, (const T*)res, (T*)sum_out,
                                             (const T*)w, (T*)y, rstd, rows, H, eps));
    }
  });
}

template <typename T, int V, bool DW, bool FULL>
void launch_rms_bwd(const void* dy, const void* x, const void* w, const float* rstd,
                    const void* dres, void* dx, float* dw_part, int64_t rows, int H, int blocks,
                    hipStream_t s) {
  const size_t lds = (H * sizeof(T) + 15) / 16 * 16 + (DW ? kWaves * H * sizeof(float) : 0);
  static const bool ahead = [] {
    const char* e = getenv("EMA_RMS_DRES_AHEAD");
    return !(e && e[0] == '0');
  }();
  if (dres && ahead)
    hipLaunchKernelGGL((rmsnorm_bwd_k<T, V, DW, FULL, true, true>), dim3(blocks), dim3(256), lds, s,
                       (const T*)dy, (const T*)x, (const T*)w, rstd, (const T*)dres, (T*)dx,
                       dw_part, rows, H);
  else if (dres)
    hipLaunchKernelGGL((rmsnorm_bwd_k<T, V, DW, FULL, true>), dim3(blocks), dim3(256), lds, s,
                       (const T*)dy, (const T*)x, (const T*)w, rstd, (const T*)dres, (T*)dx,
                       dw_part, rows, H);
  else
    hipLaunchKernelGGL((rmsnorm_bwd_k<T, V, DW, FULL, false>), dim3(blocks), dim3(256), lds, s,
                       (const T*)dy, (const T*)x, (const T*)w, rstd, (const T*)dres, (T*)dx,
                       dw_part, rows, H);
}

// EMA_RMS_BWD_WG=0: the one-wave-per-row backward everywhere (A/B)
bool rms_bwd_wg_on() {
  static const bool on = [] {
    const char* e = getenv("EMA_RMS_BWD_WG");
    return !(e && e[0] == '0');
  }();
  return on;
}

void rmsnorm_bwd(const void* dy, const void* x, const void* w, const float* rstd,
                 const void* dres, void* dx, float* dw_part, void* dw, float* dw_acc,
                 int accumulate, int64_t rows, int H, int dt, hipStream_t s) {
  const int P = norm_bwd_partials(rows);
  const int blocks = P / kWaves;
  // workgroup-per-row form: 16-bit types, H = 2048 EV (EV 1, 2, 4), enough
  // rows to fill the grid; its partial rows (one per workgroup, <= P) go to
  // the same column sum
  const int ev = H % 2048 == 0 ? H / 2048 : 0;
  if (rms_bwd_wg_on() && dt != DT_F32 && (ev == 1 || ev == 2 || ev == 4) && rows >= 4 * 256) {
    // one resident wave of workgroups (registers allow ~5 / 3 / 1 per CU at
    // EV = 1 / 2 / 4): every partial row written once, no second round
    const int per_cu = ev == 1 ? 5 : ev == 2 ? 3 : 1;
    const int G = (int)std::min<int64_t>(std::min<int64_t>(P, 256 * per_cu), rows / 4);
#define EMA_RMS_WG(T_, EV_)                                                                        \
    {                                                                                             \
      if (dres)                                                                                   \
        hipLaunchKernelGGL((rmsnorm_bwd_wg_k<T_, EV_, true>), dim3(G), dim3(256), 0, s,           \
                           (const T_*)dy, (const T_*)x, (const T_*)w, rstd, (const T_*)dres,      \
                           (T_*)dx, dw_part, rows, H);                                            \
      else                                                                                        \
        hipLaunchKernelGGL((rmsnorm_bwd_wg_k<T_, EV_, false>), dim3(G), dim3(256), 0, s,          \
                           (const T_*)dy, (const T_*)x, (const T_*)w, rstd, (const T_*)dres,      \
                           (T_*)dx, dw_part, rows, H);                                            \
      colsum<T_>(dw_part, (T_*)dw, dw_acc, accumulate, G, H, s);                                  \
    }
    if (dt == DT_BF16) {
      if (ev == 1) EMA_RMS_WG(bf16, 1) else if (ev == 2) EMA_RMS_WG(bf16, 2) else EMA_RMS_WG(bf16, 4)
    } else {
      if (ev == 1) EMA_RMS_WG(fp16, 1) else if (ev == 2) EMA_RMS_WG(fp16, 2) else EMA_RMS_WG(fp16, 4)
    }
#undef EMA_RMS_WG
    return;
  }
  EMA_DISPATCH_FLOAT(dt, T, {
    const int vpl = pick_vpl<T>(H);
    const bool full = H == vpl * 64 * (16 / (int)sizeof(T));
    if (vpl <= 8 && H <= kLdsDwMaxH && full) {
      EMA_VPL_SWITCH(vpl, (launch_rms_bwd<T, V, true, true>(dy, x, w, rstd, dres, dx, dw_part,
                                                             rows, H, blocks, s)));
    } else if (vpl <= 8 && H <= kLdsDwMaxH) {
      EMA_VPL_SWITCH(vpl, (launch_rms_bwd<T, V, true, false>(dy, x, w, rstd, dres, dx, dw_part,
                                                              rows, H, blocks, s)));
    } else {
      EMA_VPL_SWITCH(vpl, (launch_rms_bwd<T, V, false, false>(dy, x, w, rstd, dres, dx, dw_part,
                                                               rows, H, blocks, s)));
      const int64_t rpc = (rows + P - 1) / P;
      const int cblocks = (H / (16 / (int)sizeof(T)) + 255) / 256;
      hipLaunchKernelGGL((norm_dw_k<T, false>), dim3(cblocks, P), dim3(256), 0, s, (const T*)dy,
                         (const T*)x, (const float*)nullptr, rstd, dw_part, (float*)nullptr,
                         rows, H, rpc);
    }
    colsum<T>(dw_part, (T*)dw, dw_acc, accumulate, P, H, s);
  });
}

void layernorm_fwd(const void* x, const void* res, void* sum_out, const void* w, const void* b,
                   void* y, float* mean, float* rstd, int64_t rows, int H, float eps, int dt,
                   hipStream_t s) {
  const int64_t blocks = (rows + kWaves - 1) / kWaves;
  EMA_DISPATCH_FLOAT(dt, T, {
    const int vpl = pick_vpl<T>(H);
    EMA_VPL_SWITCH(vpl, hipLaunchKernelGGL((layernorm_fwd_k<T, V>), dim3(blocks), dim3(256), 0, s,
                                           (const T*)x, (const T*)res, (T*)sum_out, (const T*)w,
                                           (const T*)b, (T*)y, mean,
                                           rstd, rows, H, eps));
  });
}

void layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean,
                   const float* rstd, const void* dres, void* dx, float* dw_part, float* db_part, void* dw,
                   void* db, float* dw_acc, float* db_acc, int accumulate_w, int accumulate_b,
                   int64_t rows, int H, int dt, hipStream_t s) {
  const int P = norm_bwd_partials(rows);
  const int blocks = P / kWaves;
  EMA_DISPATCH_FLOAT(dt, T, {
    const int vpl = pick_vpl<T>(H);
    if (vpl <= 8) {
      EMA_VPL_SWITCH(vpl, hipLaunchKernelGGL((layernorm_bwd_k<T, V, true>), dim3(blocks),
                                             dim3(256), 0, s, (const T*)dy, (const T*)x,
                                             (const T*)w, mean, rstd, (const T*)dres, (T*)dx,
                                             dw_part, db_part,
                                             rows, H));
    } else {
      EMA_VPL_SWITCH(vpl, hipLaunchKernelGGL((layernorm_bwd_k<T, V, false>), dim3(blocks),
                                             dim3(256), 0, s, (const T*)dy, (const T*)x,
                                             (const T*)w, mean, rstd, (const T*)dres, (T*)dx,
                                             dw_part, db_part,
                                             rows, H));
      const int64_t rpc = (rows + P - 1) / P;
      const int cblocks = (H / (16 / (int)sizeof(T)) + 255) / 256;
      hipLaunchKernelGGL((norm_dw_k<T, true>), dim3(cblocks, P), dim3(256), 0, s, (const T*)dy,
                         (const T*)x, mean, rstd, dw_part, db_part, rows, H, rpc);
    }
    colsum<T>(dw_part, (T*)dw, dw_acc, accumulate_w, P, H, s);
    colsum<T>(db_part, (T*)db, db_acc, accumulate_b, P, H, s);
  });
}

}  // namespace ema
