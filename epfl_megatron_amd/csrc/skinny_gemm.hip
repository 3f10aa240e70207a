// Weight-streaming GEMM for decode-sized batches on gfx950, with the decode
// step's elementwise work fused into its prologue / epilogue:
//
//     Y[M, N] = f(norm(X)[M, K] · W[N, K]^T)        M <= 32, bf16/fp16, fp32 accumulate
//
// A token-by-token decode step multiplies a handful of rows by every weight
// of the model: the time is the weight stream from HBM.  hipBLASLt's skinny
// tiles reach ~3.2-3.9 TB/s on the Llama-2-7B projections
// (profiles/r2c_serve_decode_b8_kernel_stats.csv); here every CU streams with
// many loads in flight:
//   * workgroup = 8 waves (4 when K % 256 != 0) = 16 output features (rows of
//     W); wave w reduces the K slice [w K/8, (w+1) K/8) with v_mfma_f32_16x16x32 (A = 16 W rows x
//     32 k, B = the <= 16 X rows x 32 k; unused B columns are zero) from a
//     register ring that keeps SKINNY_U k-steps of W / X loads in flight
//     (each slot refilled as soon as its MFMA has consumed it, the first
//     block issued at kernel entry, before the RMSNorm prologue);
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
// Shapes: M <= 32 (17-32 rows: two row blocks per W fragment in the
// per-block kernel), N % 16 == 0, K % 128 == 0 (checked by the host).
//
// Packed weights (p.packed, 8-wave forms, K % 256 == 0).  In row-major W a
// wave's A-operand load (lane L: row L & 15, 8 k at 8 (L >> 4)) touches 16
// rows x 64 B and every 4-lane quad 4 different cache lines; the streams
// topped out at 3.9-4.9 TB/s.  skinny_pack (ops/decode_pack.py) stores each
// (16-row block, wave, k-step) fragment set as one contiguous 1 KiB piece,
// lane L at byte 16 L, read by the identical MFMA schedule: 4.6-6.0 TB/s on
// the Llama-2-7B shapes (scripts/gemv_layout_bench.hip,
// profiles/r4m_gemv_layout.txt).  The k index a lane feeds is unchanged, so X /
// gamma loads and every epilogue are layout-independent.
#include <cstdlib>
#include <type_traits>

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

// Output of one 16-feature block (t = the block's reduced fp32 tile; lane
// holds column m = lane & 15, features 4 (lane >> 4) + i).
// The epilogue's global operands for one block, loaded ahead (before the
// block's k-loop) by the wave that runs the epilogue, so the epilogue does not
// wait out load round trips while the other waves stream the next block: the
// residual tile (EPI_RES) or the rotary cos / sin pairs (EPI_QKV; the token
// positions and the cache slot once per workgroup).
template <typename T, int EPI>
struct EpiPre {
  typename fa::MT<T>::x4 rv{};
  float c[2] = {0.f, 0.f}, s[2] = {0.f, 0.f};
  int pos = 0;       // (32-bit: two row blocks' 64-bit positions and slots spilled)
  int64_t slot = 0;  // uniform: scalar registers
};

template <typename T, int EPI>
__device__ __forceinline__ void epi_init(const SkinnyArgs& p, int lane, EpiPre<T, EPI>& e,
                                         int moff = 0) {
  if constexpr (EPI == EPI_QKV) {
    const int m = (lane & 15) + moff;
    e.pos = m < p.M ? (int)p.pos[(int64_t)m * p.pos_sb] : 0;
    const int64_t sl = p.slot_ptr ? *p.slot_ptr : p.slot;
    e.slot = (int64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(sl & 0xffffffffll)) |
             ((int64_t)__builtin_amdgcn_readfirstlane((int)(sl >> 32)) << 32);
  }
}

template <typename T, int EPI>
__device__ __forceinline__ void epi_prefetch(const SkinnyArgs& p, int blk, int lane, EpiPre<T, EPI>& e,
                                             int moff = 0) {
  const int m = (lane & 15) + moff, n = blk * 16 + 4 * (lane >> 4);
  if (m >= p.M) return;
  if constexpr (EPI == EPI_RES) {
    e.rv = *reinterpret_cast<const typename fa::MT<T>::x4*>((const T*)p.res + (int64_t)m * p.ldr + n);
  }
  if constexpr (EPI == EPI_QKV) {
    const int hd = p.hd, per_g = (p.r + 2) * hd;
    const int d = (n - (n / per_g) * per_g) % hd;
    const float* cr = p.cos + (int64_t)e.pos * (hd / 2) + d / 2;
    const float* sr = p.sin + (int64_t)e.pos * (hd / 2) + d / 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      e.c[j] = cr[j];
      e.s[j] = sr[j];
    }
  }
}

template <typename T, int EPI, int ACT>
__device__ __forceinline__ void epilogue(const SkinnyArgs& p, int blk, const f4& t, int lane,
                                         int half, const EpiPre<T, EPI>& pre, bool use_pre,
                                         int moff = 0) {
  const int M = p.M;
  // D layout: lane holds column m = lane & 15 (+ moff: the row block), rows
  // (features) 4 (lane >> 4) + i
  const int m = (lane & 15) + moff, nr = 4 * (lane >> 4);
  typename fa::MT<T>::x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (T)t[i];
  T* __restrict__ y = (T*)p.y;
  if constexpr (EPI == EPI_GLU) {
    // lanes 0-31 hold up rows 0-7, lanes 32-63 the gate rows of the same f
    typename fa::MT<T>::x4 gt;
#pragma unroll
    for (int i = 0; i < 4; ++i) gt[i] = (T)__shfl_xor((float)o[i], 32, 64);
    // half block (half >= 0): features 4 half .. 4 half + 3 only, in MFMA
    // rows 0-3 / 8-11 (rows 4-7 / 12-15 duplicate them and are not stored)
    if ((half < 0 ? lane < 32 : lane < 16) && m < M) {
      typename fa::MT<T>::x4 out;
#pragma unroll
      for (int i = 0; i < 4; ++i) out[i] = (T)((float)o[i] * act<ACT>((float)gt[i]));
      const int f = blk * 8 + (half < 0 ? nr : 4 * half);
      *reinterpret_cast<typename fa::MT<T>::x4*>(y + (int64_t)m * p.ldy + f) = out;
    }
    return;
  }
  if (m >= M) return;
  const int n = blk * 16 + nr;
  if constexpr (EPI == EPI_RES) {
    const typename fa::MT<T>::x4 rv = use_pre ? pre.rv :
        *reinterpret_cast<const typename fa::MT<T>::x4*>((const T*)p.res + (int64_t)m * p.ldr + n);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (T)((float)o[i] + (float)rv[i]);
  }
  if constexpr (EPI == EPI_QKV) {
    const int hd = p.hd, per_g = (p.r + 2) * hd;
    const int g = n / per_g, rem = n - g * per_g, h = rem / hd, d = rem - h * hd;
    if (h <= p.r) {  // q heads and the k head: rotate pairs (d, d+1), (d+2, d+3)
      const int64_t pos = use_pre ? 0 : p.pos[(int64_t)m * p.pos_sb];
      const float* cr = p.cos + pos * (hd / 2) + d / 2;
      const float* sr = p.sin + pos * (hd / 2) + d / 2;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float x0 = (float)o[2 * j], x1 = (float)o[2 * j + 1];
        const float c = use_pre ? pre.c[j] : cr[j], sn = use_pre ? pre.s[j] : sr[j];
        o[2 * j] = (T)(x0 * c - x1 * sn);
        o[2 * j + 1] = (T)(x0 * sn + x1 * c);
      }
    }
    T* dst;
    if (h < p.r) {
      dst = y + (int64_t)m * p.ldy + (int64_t)(g * p.r + h) * hd + d;
    } else {
      const int64_t slot = use_pre ? pre.slot : p.slot_ptr ? *p.slot_ptr : p.slot;
      T* cache = (T*)(h == p.r ? p.kcache : p.vcache);
      dst = cache + slot * p.c_ss + (int64_t)m * p.c_sb + (int64_t)g * hd + d;
    }
    *reinterpret_cast<typename fa::MT<T>::x4*>(dst) = o;
    return;
  }
  *reinterpret_cast<typename fa::MT<T>::x4*>(y + (int64_t)m * p.ldy + n) = o;
}

#ifndef SKINNY_U
#define SKINNY_U 8  // k-steps of W / X (/ gamma) loads in flight per wave
#endif

// MB: 16-row blocks of X (1: M <= 16; 2: M <= 32 -- every W fragment feeds
// one MFMA per row block, so the weight stream is read once for 32 rows).
template <typename T, int WAVES, bool NORM, int EPI, int ACT, bool PACKED, int MB>
__global__ __launch_bounds__(64 * WAVES) void skinny_gemm_k(const SkinnyArgs p) {
  typedef typename fa::MT<T>::x8 x8;
  // (a 16-deep ring for one row block measured the same: fc2 K = 11008 at
  // 16 rows 23.2 vs 23.0 us, profiles/r4al_skinny_u16.txt)
  // two un-normed row blocks (fc2 at 17-32 rows, K = 11008: 43 k-steps per
  // wave = 3 x 14 + 1): 14 deep, 28.6 / 33.4 us at 24 / 32 rows vs 29.7 / 34.8
  // at 8 (profiles/r4ar_skinny_u14.txt)
  constexpr int U = MB == 2 && !NORM ? 14 : SKINNY_U;
  __shared__ f4 part[WAVES][MB][64];
  __shared__ float ssq[WAVES][16 * MB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int M = p.M, N = p.N, K = p.K;
  const T* __restrict__ x = (const T*)p.x;
  const T* __restrict__ w = (const T*)p.w;
  const int kq = K / WAVES, kbeg = wave * kq;
  const int r = lane & 15, kc = 8 * (lane >> 4);  // fragment row / k offset of this lane
  const int steps = kq / 32;
  // W fragment of k-step s at wr + WS s: row-major rows, or the packed
  // layout's contiguous 1 KiB per (block, wave, step) (skinny_pack)
  constexpr int WS = PACKED ? 512 : 32;
  static_assert(!PACKED || WAVES == 8, "the packed layout is cut for 8 waves");
  const T* wr = PACKED ? w + ((int64_t)blockIdx.x * WAVES + wave) * steps * 512 + 8 * lane
                       : w + w_row<EPI>(blockIdx.x, r, N) * K + kbeg + kc;
  bool xon[MB];
  const T* xr[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    xon[mb] = r + 16 * mb < M;
    xr[mb] = x + (int64_t)(xon[mb] ? r + 16 * mb : 0) * K + kbeg + kc;
  }
  const T* gr = NORM ? (const T*)p.norm_w + kbeg + kc : nullptr;
  const int nblk = steps / U;  // full ring blocks; the < U leftover steps run after them

  // Ring of U k-steps: the W fragment (nontemporal: each weight byte is read
  // once per step), the X fragments and (NORM) the gamma fragment, refilled
  // U steps ahead right after each MFMA consumes its slot, so U k-steps of
  // loads stay in flight through the whole stream.  Issued BEFORE the RMSNorm
  // prologue: the weight stream starts at kernel entry, not after the norm's
  // reduction and barrier.
  x8 a[U], xv[MB][U], gv[U];
  if (nblk > 0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      a[u] = __builtin_nontemporal_load(reinterpret_cast<const x8*>(wr + WS * u));
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) xv[mb][u] = *reinterpret_cast<const x8*>(xr[mb] + 32 * u);
      if constexpr (NORM) gv[u] = *reinterpret_cast<const x8*>(gr + 32 * u);
    }
  }

  float rs[MB];  // rstd of X rows r + 16 mb (NORM)
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) rs[mb] = 1.f;
  if constexpr (NORM) {
    // sum of squares of this wave's X slice: 8 loads issued per round before
    // any is used (a load-then-use loop waits out one L2 round trip per step)
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      float ss = 0.f;
      for (int s0 = 0; s0 < steps; s0 += 8) {
        x8 v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int s = s0 + i < steps ? s0 + i : steps - 1;
          v[i] = *reinterpret_cast<const x8*>(xr[mb] + 32 * s);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float keep = s0 + i < steps ? 1.f : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float f = (float)v[i][e];
            ss += keep * f * f;
          }
        }
      }
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (lane < 16) ssq[wave][16 * mb + lane] = ss;
    }
    __syncthreads();
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      float tot = 0.f;
#pragma unroll
      for (int i = 0; i < WAVES; ++i) tot += ssq[i][16 * mb + r];  // fixed order
      rs[mb] = rsqrtf(tot / (float)K + p.eps);
    }
  }
  // B operand: X (or its RMSNorm, rounded like rmsnorm_fwd_k) of row block mb
  auto bop = [&](const x8& v, const x8& g, int mb) {
    x8 o;
    if constexpr (!NORM) {
      o = v;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const T xn = (T)((float)v[e] * rs[mb]);
        o[e] = (T)((float)xn * (float)g[e]);
      }
    }
    if (!xon[mb]) o = x8{};
    return o;
  };

  f4 acc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) acc[mb] = f4{0.f, 0.f, 0.f, 0.f};
  // one ring block; REFILL: reload each slot U steps ahead once consumed
  auto block = [&](int blk, auto refill_c) {
    constexpr bool REFILL = decltype(refill_c)::value;
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc[mb] = mfma16x16x32<T>(a[u], bop(xv[mb][u], gv[u], mb), acc[mb]);
      if constexpr (REFILL) {
        const int s = (blk + 1) * U + u;
        a[u] = __builtin_nontemporal_load(reinterpret_cast<const x8*>(wr + WS * s));
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) xv[mb][u] = *reinterpret_cast<const x8*>(xr[mb] + 32 * s);
        if constexpr (NORM) gv[u] = *reinterpret_cast<const x8*>(gr + 32 * s);
      }
      // keep {MFMA u, refill u} in program order: hipcc would otherwise
      // cluster the dependent MFMA chain and issue every refill after it,
      // draining the ring (vmcnt(0)) once per block
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  for (int blk = 0; blk + 1 < nblk; ++blk) block(blk, std::true_type{});
  if (nblk > 0) block(nblk - 1, std::false_type{});
  // leftover steps (K / WAVES not a multiple of 32 U): loads first, then MFMAs
  {
    const int s0 = nblk * U, left = steps - s0;
#pragma unroll
    for (int u = 0; u < U - 1; ++u) {
      if (u < left) {
        a[u] = __builtin_nontemporal_load(reinterpret_cast<const x8*>(wr + WS * (s0 + u)));
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) xv[mb][u] = *reinterpret_cast<const x8*>(xr[mb] + 32 * (s0 + u));
        if constexpr (NORM) gv[u] = *reinterpret_cast<const x8*>(gr + 32 * (s0 + u));
      }
    }
#pragma unroll
    for (int u = 0; u < U - 1; ++u)
      if (u < left) {
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb] = mfma16x16x32<T>(a[u], bop(xv[mb][u], gv[u], mb), acc[mb]);
      }
  }
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) part[wave][mb][lane] = acc[mb];
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    f4 t = part[0][mb][lane];
#pragma unroll
    for (int i = 1; i < WAVES; ++i) t += part[i][mb][lane];  // fixed order: deterministic
    epilogue<T, EPI, ACT>(p, blockIdx.x, t, lane, -1, EpiPre<T, EPI>{}, false, 16 * mb);
  }
}

// Persistent form for K = 8 waves x 32 x STEPS (STEPS 16 / 32: the 4096 / 8192
// hidden sizes of Llama-2-7B / 70B), one workgroup per CU walking the output
// blocks blockIdx.x, +grid, ...:
//   * the wave's X slice (RMSNorm applied for NORM) is loaded ONCE into
//     registers (STEPS fragments; rows >= M stay zero and are never loaded)
//     and reused by every block: no per-block X / gamma traffic and one norm
//     prologue per workgroup instead of one per 16 output features (the
//     non-persistent NORM forms spent ~half their time in that prologue:
//     profiles/r3g_decode_b8_kernels.txt);
//   * the W ring runs across block seams: the last U refills of a block load
//     the next block's first U k-steps, so the stream never drains;
//   * per block, the 8 partial tiles meet in a double-buffered LDS slot and
//     wave 0 runs the epilogue while the other waves stream the next block.
template <typename T, bool NORM, int EPI, int ACT, int STEPS, int U, bool PACKED, int MB>
__global__ __launch_bounds__(512) void skinny_pgemm_k(const SkinnyArgs p) {
  typedef typename fa::MT<T>::x8 x8;
  constexpr int WAVES = 8;
  static_assert(STEPS % U == 0, "ring must tile the k-steps");
  static_assert(!NORM || STEPS == 16, "the normed forms keep 64 gamma chunks per wave");
  static_assert(MB == 1 || STEPS == 16, "two row blocks keep 2 x 16 X fragments in registers");
  __shared__ f4 part[2][WAVES][MB][64];
  __shared__ float ssq[WAVES][16 * MB];
  __shared__ x8 gsh[NORM ? WAVES : 1][64];  // NORM: each wave's gamma slice
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int M = p.M, N = p.N, K = p.K;
  const T* __restrict__ x = (const T*)p.x;
  const T* __restrict__ w = (const T*)p.w;
  const int kbeg = wave * STEPS * 32;
  const int r = lane & 15, kc = 8 * (lane >> 4);
  bool xon[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) xon[mb] = r + 16 * mb < M;
  const int nblocks = EPI == EPI_GLU ? N / 8 : N / 16;
  const int G = (int)gridDim.x, wg = blockIdx.x;
  // Work units of this workgroup: blocks wg, wg + G, ...  GLU tail: when the
  // last round has nrem <= G / 2 blocks, they run as 2 nrem HALF blocks (4
  // features each) on 2 nrem workgroups instead of nrem full ones: the
  // round's time halves (Llama-2-7B fc1: 1376 blocks = 5 x 256 + 96 ->
  // at most 5.5 instead of 6 block times per workgroup).  A half block's MFMA
  // rows r and r + 4 read the same W row (one HBM fetch per cache line).
  // PACKED: the nrem tail blocks are stored as half units (skinny_glu_half_tail;
  // ops/decode_pack.py): per (half, wave, k-step) 512 contiguous bytes holding
  // the 4 up + 4 gate rows, which MFMA rows r and r + 4 both read.
  const int nrem = nblocks % G;
  const bool halves = EPI == EPI_GLU && nrem > 0 && 2 * nrem <= G;
  const int rounds = halves ? (nblocks - nrem) / G : 0;
  const int nunits = halves ? rounds + (wg < 2 * nrem ? 1 : 0) : (nblocks - wg + G - 1) / G;
  auto unit_blk = [&](int j) { return j < rounds || !halves ? wg + j * G : nblocks - nrem + wg / 2; };
  auto unit_half = [&](int j) { return j < rounds || !halves ? -1 : (wg & 1); };
  // elements between a lane's consecutive k-steps of unit j
  auto wstr = [&](int j) { return !PACKED ? 32 : unit_half(j) < 0 ? 512 : 256; };
  auto wptr = [&](int j) {
    const int b = unit_blk(j), h = unit_half(j);
    if constexpr (PACKED) {
      if (h < 0) return w + ((int64_t)b * WAVES + wave) * STEPS * 512 + 8 * lane;
      const int64_t tail = (int64_t)(nblocks - nrem) * 16 * K;  // full blocks first
      const int unit = (b - (nblocks - nrem)) * 2 + h, pr = (r & 3) + 4 * (r >> 3);
      return w + tail + ((int64_t)unit * WAVES + wave) * STEPS * 256 + 8 * (kc + pr);
    }
    int64_t row;
    if (h < 0) row = w_row<EPI>(b, r, N);
    else row = (r < 8 ? 0 : (int64_t)N) + (int64_t)b * 8 + 4 * h + (r & 3);
    return w + row * K + kbeg + kc;
  };
  int j = 0, blk = unit_blk(0), half = unit_half(0);
  EpiPre<T, EPI> pre[MB];  // wave 0: the epilogue operands of the current block
  if (wave == 0) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      epi_init<T, EPI>(p, lane, pre[mb], 16 * mb);
      epi_prefetch<T, EPI>(p, blk, lane, pre[mb], 16 * mb);
    }
  }
  const T* wr = wptr(0);
  const T* wn = wptr(nunits > 1 ? 1 : 0);
  int ws = wstr(0), wsn = wstr(nunits > 1 ? 1 : 0);

  // X (and gamma) first, the weight ring right behind them: a wave's loads
  // return in order, so X lands first and the norm prologue runs while the
  // ring's weight loads are in flight (issued the other way round, X came
  // back only after the whole ring and the first MFMA waited for the norm)
  x8 xs[MB][STEPS];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const T* xr = x + (int64_t)(r + 16 * mb) * K + kbeg + kc;
    if (xon[mb]) {
#pragma unroll
      for (int s = 0; s < STEPS; ++s) xs[mb][s] = *reinterpret_cast<const x8*>(xr + 32 * s);
    } else {
#pragma unroll
      for (int s = 0; s < STEPS; ++s) xs[mb][s] = x8{};
    }
  }
  // gamma: the wave's K slice is 64 chunks of 8, one 16-B load per lane,
  // staged through LDS (the per-step fragments would cost 2 x STEPS live
  // registers; loading them after the norm reduction cost two more round trips)
  x8 gl{};
  if constexpr (NORM) gl = *reinterpret_cast<const x8*>((const T*)p.norm_w + kbeg + 8 * lane);
  __builtin_amdgcn_sched_barrier(0);
  x8 a[U];
  // Two normed row blocks keep 2 x 16 X fragments and spill ~0.5 KB per lane
  // in this prologue whatever the order (ring after the norm spills least):
  // the decode layer normalises 17-32 rows with the rmsnorm kernel and calls
  // the un-normed forms instead (models/transformer.py _forward_decode_fused;
  // profiles/r4ai_skinny_mb.txt, r4aj_skinny_mb.txt).
  constexpr bool RING_FIRST = !(NORM && MB == 2);
  if constexpr (RING_FIRST) {
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(reinterpret_cast<const x8*>(wr + ws * u));
  }
  if constexpr (NORM) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      float ss = 0.f;
#pragma unroll
      for (int s = 0; s < STEPS; ++s) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = (float)xs[mb][s][e];
          ss += f * f;
        }
      }
      ss += __shfl_xor(ss, 16, 64);
      ss += __shfl_xor(ss, 32, 64);
      if (lane < 16) ssq[wave][16 * mb + lane] = ss;
    }
    gsh[wave][lane] = gl;
    __syncthreads();
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) {
      float tot = 0.f;
#pragma unroll
      for (int i = 0; i < WAVES; ++i) tot += ssq[i][16 * mb + r];  // fixed order
      const float rs = rsqrtf(tot / (float)K + p.eps);
      // rounded like rmsnorm_fwd_k; step s, lane group q reads chunk 4 s + q
#pragma unroll
      for (int s = 0; s < STEPS; ++s) {
        const x8 g = gsh[wave][4 * s + (lane >> 4)];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const T xn = (T)((float)xs[mb][s][e] * rs);
          xs[mb][s][e] = (T)((float)xn * (float)g[e]);
        }
        if (!xon[mb]) xs[mb][s] = x8{};
      }
    }
  }

  if constexpr (!RING_FIRST) {
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(reinterpret_cast<const x8*>(wr + ws * u));
  }

  // one block's k-steps; LAST: the workgroup's final block, whose last U
  // slots are not refilled (a one-block workgroup would otherwise fetch U of
  // its STEPS k-steps twice)
  struct Acc {
    f4 v[MB];
  };
  auto run_block = [&](auto last_c) {
    constexpr bool LAST = decltype(last_c)::value;
    Acc acc;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) acc.v[mb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) acc.v[mb] = mfma16x16x32<T>(a[s % U], xs[mb][s], acc.v[mb]);
      if (!LAST || s + U < STEPS) {
        const T* src = s + U < STEPS ? wr + ws * (s + U) : wn + wsn * (s + U - STEPS);
        a[s % U] = __builtin_nontemporal_load(reinterpret_cast<const x8*>(src));
      }
      __builtin_amdgcn_sched_barrier(0);  // {MFMA s, refill s} in program order
    }
    return acc;
  };
  for (;; ++j) {
    const bool last = j + 1 >= nunits;
    const Acc acc = last ? run_block(std::true_type{}) : run_block(std::false_type{});
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) part[j & 1][wave][mb][lane] = acc.v[mb];
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        f4 t = part[j & 1][0][mb][lane];
#pragma unroll
        for (int i = 1; i < WAVES; ++i) t += part[j & 1][i][mb][lane];  // fixed order
        epilogue<T, EPI, ACT>(p, blk, t, lane, half, pre[mb], true, 16 * mb);
      }
    }
    if (last) break;
    blk = unit_blk(j + 1);
    half = unit_half(j + 1);
    if (wave == 0) {  // lands during the block's k-loop
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) epi_prefetch<T, EPI>(p, blk, lane, pre[mb], 16 * mb);
    }
    wr = wn;
    ws = wsn;
    wn = wptr(j + 2 < nunits ? j + 2 : nunits - 1);
    wsn = wstr(j + 2 < nunits ? j + 2 : nunits - 1);
  }
}

int num_cus() {
  static const int n = [] {
    int dev = 0, c = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      c = 256;
    return c;
  }();
  return n;
}

// STEPS = 0: one workgroup per output block (skinny_gemm_k); 16 / 32: the
// persistent skinny_pgemm_k on min(blocks, CUs) workgroups.
template <typename T, int WAVES, int STEPS, bool NORM, int EPI, int ACT>
void launch(const SkinnyArgs& p, hipStream_t s) {
  const int nblocks = EPI == EPI_GLU ? p.N / 8 : p.N / 16;
  if constexpr (STEPS == 0) {
    if (p.M > 16) {  // 17-32 rows: two row blocks per W fragment
      if constexpr (WAVES == 8) {
        if (p.packed) {
          hipLaunchKernelGGL((skinny_gemm_k<T, WAVES, NORM, EPI, ACT, true, 2>),
                             dim3((unsigned)nblocks), dim3(64 * WAVES), 0, s, p);
          return;
        }
      }
      hipLaunchKernelGGL((skinny_gemm_k<T, WAVES, NORM, EPI, ACT, false, 2>), dim3((unsigned)nblocks),
                         dim3(64 * WAVES), 0, s, p);
      return;
    }
    if constexpr (WAVES == 8) {
      if (p.packed) {
        hipLaunchKernelGGL((skinny_gemm_k<T, WAVES, NORM, EPI, ACT, true, 1>), dim3((unsigned)nblocks),
                           dim3(64 * WAVES), 0, s, p);
        return;
      }
    }
    hipLaunchKernelGGL((skinny_gemm_k<T, WAVES, NORM, EPI, ACT, false, 1>), dim3((unsigned)nblocks),
                       dim3(64 * WAVES), 0, s, p);
  } else {
    // ring depth (k-steps of weight loads in flight per wave): 16 (batch-1 graph decode
    // 301 -> 308 tok/s over 8, profiles/r3s_skinny_ring_depth.txt); 8 beside the 32
    // register-resident X fragments of K = 8192 (16 spilled 92-204 B per lane)
    constexpr int U = STEPS == 32 ? 8 : 16;
    const int g = nblocks < num_cus() ? nblocks : num_cus();
    if constexpr (STEPS == 16) {
      // 17-32 rows: two row blocks, the ring 8 deep beside 2 x 16 X fragments
      // (16 deep for the un-normed forms measured within noise: o_proj 13.6 /
      // 14.5 vs 13.0 / 14.3 us at 24 / 32 rows, profiles/r4as_pskinny_u16.txt)
      if (p.M > 16) {
        if (p.packed)
          hipLaunchKernelGGL((skinny_pgemm_k<T, NORM, EPI, ACT, STEPS, 8, true, 2>), dim3((unsigned)g),
                             dim3(512), 0, s, p);
        else
          hipLaunchKernelGGL((skinny_pgemm_k<T, NORM, EPI, ACT, STEPS, 8, false, 2>), dim3((unsigned)g),
                             dim3(512), 0, s, p);
        return;
      }
    }
    if (p.packed)
      hipLaunchKernelGGL((skinny_pgemm_k<T, NORM, EPI, ACT, STEPS, U, true, 1>), dim3((unsigned)g),
                         dim3(512), 0, s, p);
    else
      hipLaunchKernelGGL((skinny_pgemm_k<T, NORM, EPI, ACT, STEPS, U, false, 1>), dim3((unsigned)g),
                         dim3(512), 0, s, p);
  }
}

template <typename T, int WAVES, int STEPS>
void dispatch(const SkinnyArgs& p, int epi, hipStream_t s) {
  const bool nm = p.norm_w != nullptr;
  // the bf16 RMSNorm prologue over 32 register-resident k-steps spills: the
  // normed 8192-wide forms keep the one-block-per-workgroup kernel
  constexpr int SN = STEPS == 32 ? 0 : STEPS;
#define EMA_SK(NORM_, EPI_, ACT_) launch<T, WAVES, (NORM_ ? SN : STEPS), NORM_, EPI_, ACT_>(p, s)
  switch (epi) {
    case EPI_RES:
      nm ? EMA_SK(true, EPI_RES, 0) : EMA_SK(false, EPI_RES, 0);
      break;
    case EPI_QKV:
      nm ? EMA_SK(true, EPI_QKV, 0) : EMA_SK(false, EPI_QKV, 0);
      break;
    case EPI_GLU:
      switch (p.act) {
        case 0: nm ? EMA_SK(true, EPI_GLU, 0) : EMA_SK(false, EPI_GLU, 0); break;
        case 1: nm ? EMA_SK(true, EPI_GLU, 1) : EMA_SK(false, EPI_GLU, 1); break;
        case 2: nm ? EMA_SK(true, EPI_GLU, 2) : EMA_SK(false, EPI_GLU, 2); break;
        default: nm ? EMA_SK(true, EPI_GLU, 3) : EMA_SK(false, EPI_GLU, 3); break;
      }
      break;
    default:
      nm ? EMA_SK(true, EPI_PLAIN, 0) : EMA_SK(false, EPI_PLAIN, 0);
  }
#undef EMA_SK
}



}  // namespace


bool skinny_gemm_supported(int64_t M, int64_t N, int64_t K) {
  return M >= 1 && M <= 32 && N % 16 == 0 && K % 128 == 0 && N > 0 && K > 0 &&
         N * K < ((int64_t)1 << 40);
}

// 8 waves (K split 8 ways) where K allows: twice the loads in flight per CU
// of the 4-wave form, which left the N = 4096 projections (one workgroup per
// CU) latency-bound at ~3.2 TB/s.  EMA_SKINNY_WAVES=4 forces the 4-wave form.
// K = 4096 / 8192 (16 / 32 k-steps per wave) take the persistent form
// (EMA_SKINNY_PERSIST=0: the one-block-per-workgroup kernel everywhere).
void skinny_gemm_ex(const SkinnyArgs& p0, int epi, int dt, hipStream_t s) {
  SkinnyArgs p = p0;
  static const int want = [] {
    const char* e = getenv("EMA_SKINNY_WAVES");
    return e ? atoi(e) : 8;
  }();
  static const bool persist = [] {
    const char* e = getenv("EMA_SKINNY_PERSIST");
    return !(e && e[0] == '0');
  }();
  // packed weights are cut for the 8-wave forms (the host checks K % 256 == 0)
  const bool w8 = (want == 8 || p.packed) && p.K % 256 == 0;
  const int steps = w8 ? p.K / 256 : 0;
  // 17-32 rows: the persistent form holds two row blocks of X at K = 4096;
  // at K = 8192 they run the per-block kernel
  if (persist && w8 && (steps == 16 || (steps == 32 && p.M <= 16))) {
    if (dt == DT_BF16) steps == 16 ? dispatch<bf16, 8, 16>(p, epi, s) : dispatch<bf16, 8, 32>(p, epi, s);
    else steps == 16 ? dispatch<fp16, 8, 16>(p, epi, s) : dispatch<fp16, 8, 32>(p, epi, s);
    return;
  }
  if (dt == DT_BF16) w8 ? dispatch<bf16, 8, 0>(p, epi, s) : dispatch<bf16, 4, 0>(p, epi, s);
  else w8 ? dispatch<fp16, 8, 0>(p, epi, s) : dispatch<fp16, 4, 0>(p, epi, s);
}

// GLU blocks of 8 features (F / 8) the persistent kernel runs as half units
// in its last round (0: none / not the persistent form) for an M-row call
// with (norm) or without the RMSNorm prologue.  The decode-packed GLU weight
// stores exactly these tail blocks in the half-unit layout.  The condition
// mirrors skinny_gemm_ex + dispatch: K = 4096 is always persistent; K = 8192
// only un-normed with <= 16 rows (17-32 rows and the normed forms run the
// one-block-per-workgroup kernel, which reads no half units).
int skinny_glu_half_tail(int64_t F, int64_t K, bool norm, int64_t M) {
  static const bool persist = [] {
    const char* e = getenv("EMA_SKINNY_PERSIST");
    return !(e && e[0] == '0');
  }();
  if (K % 256 != 0 || F % 8 != 0) return 0;
  const int64_t steps = K / 256;
  if (!persist || !(steps == 16 || (steps == 32 && !norm && M <= 16))) return 0;
  const int64_t nblocks = F / 8, G = nblocks < num_cus() ? nblocks : num_cus();
  const int64_t nrem = nblocks % G;
  return nrem > 0 && 2 * nrem <= G ? (int)nrem : 0;
}

void skinny_gemm(const void* x, const void* w, void* y, int64_t M, int64_t N, int64_t K, int dt,
                 hipStream_t s) {
  SkinnyArgs p{};
  p.x = x; p.w = w; p.y = y;
  p.M = (int)M; p.N = (int)N; p.K = (int)K; p.ldy = N;
  skinny_gemm_ex(p, EPI_PLAIN, dt, s);
}

}  // namespace ema
