// Forward / data-gradient GEMM for gfx950 (MI355X) with fused GLU epilogues:
//
//     C[M, N] = A[M, K] · B[N, K]^T        A, B bf16/fp16 row-major (K contiguous)
//
// Every product of a linear layer whose reduction dim is contiguous in both
// operands is this "NT" form:
//   * forward  Y  = X · W^T               (A = X,  B = W        [out, in])
//   * dgrad    dX = dY · W = dY · (W^T)^T  (A = dY, B = W^T      [in, out], the
//                                          per-step transposed copy of W)
// and the hand-written kernel replaces hipBLASLt for both, so the MLP's GLU
// passes disappear into the epilogues (reference MLP megatron/model/
// transformer.py:92-123, GLU [up; gate] order megatron/model/
// glu_activations.py:18-21):
//   EPI_STORE   C = A·B^T (bf16)
//   EPI_GLU     fc1 forward.  B = W1 [2F, K]; the tile's 256 B rows are 128
//               "up" rows f0.. and the matching 128 "gate" rows F+f0.., placed
//               so every lane holds x1 and x2 of the same (m, f) in registers.
//               Writes the pre-activation [M, 2F] (saved for backward) and
//               y = x1 * act(x2) [M, F] (the fc2 input).
//   EPI_DGLU    fc2 dgrad.  C = dAct [M, F] is never written: the epilogue reads
//               the saved pre-activation and writes d(pre-act) [M, 2F] =
//               [dAct * act(x2), dAct * x1 * act'(x2)].
// Numerics equal the unfused path's: the fp32 accumulator is rounded to the
// operand dtype once, and the GLU math runs in fp32 on those rounded values.
//
// Structure (the 256x256 ping-pong of gemm_wgrad.hip, K-contiguous operands):
//   * 256 (m) x 256 (n) output tile per workgroup, 8 waves as 2 (m) x 4 (n),
//     each wave 128 x 64 = 8 x 4 tiles of v_mfma_f32_16x16x32, the operands
//     passed as (B-frag, A-frag) so each lane's accumulator holds 4
//     CONSECUTIVE output columns of one row (8-byte epilogue pieces).
//   * K is consumed in subtiles of 32 (one MFMA k-step).  Both [256][32]
//     operand slices go HBM -> LDS by global_load_lds_dwordx4 into a ring of
//     4 subtiles (4 x 32 KiB); subtile p+3's loads issue in phase p and are
//     retired by a counted vmcnt (no vmcnt(0) in the loop).
//   * LDS image: 64-B rows, 16-B chunk c of row r at 16 (c ^ ((-(r >> 2)) & 3)).
//     Every ds_read_b128 of an MFMA fragment (16 rows x 4 chunks) then hits
//     16 distinct 16-B bank slots in each of its 4 lane groups: conflict-free.
//     The swizzle goes through the per-lane DMA SOURCE address (the DMA writes
//     LDS lane-linearly), and fragments differ only by instruction immediates.
//   * Ping-pong: waves 4..7 run one barrier behind waves 0..3, so on every SIMD
//     one wave's 32 MFMAs (s_setprio 1) overlap the other's fragment reads; 3
//     of a subtile's 4 DMA pieces issue in the load section, 1 inside the MFMA
//     section (gemm_wgrad.hip's SCHED 5).
//   * Epilogue through LDS: each wave rounds its 128 x 64 tile to 16 bits into
//     a private 16 KiB region (16-B units XOR-swizzled by row), then moves rows
//     as 16-B pieces (128 B contiguous per 8 lanes).
//   * XCD-aware grouped tile order: each XCD's 32 concurrent workgroups cover
//     an 8 (m) x 4 (n) block, sharing A and B panels in its L2.
// Shapes: K % 32 == 0, N % 8 == 0 (F % 8 for the GLU forms), 16-B aligned rows;
// ragged M and N tails are clamped on load and masked on store.
// Row-group remap (RowMap, STORE / GLU): A rows may be read from, and C rows
// written to, a strided set of row groups of a larger matrix — one chunk of
// the sequence-parallel all-gather / reduce-scatter pipeline
// (parallel/tensor/layers.py) runs as one launch without a copy.
#include <algorithm>
#include <cstdlib>

#include "act_math.h"
#include "fa_common.h"
#include "gemm_plan.h"

namespace ema {
namespace {

using fa::static_for;

typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int TM = 256;               // output rows (m) per tile
constexpr int TN = 256;               // output cols (n) per tile
constexpr int BK = 32;                // reduction depth per subtile = one MFMA k-step
constexpr int OPB = 256 * BK * 2;     // 16 KiB per operand subtile
constexpr int SLOTB = 2 * OPB;        // A + B
constexpr int NSLOT = 4;              // ring depth (3 subtiles ahead)
constexpr int LDSB = NSLOT * SLOTB;   // 128 KiB
constexpr int FA_ = 8, FB_ = 4;       // m and n fragments per wave

enum { EPI_STORE = 0, EPI_GLU = 1, EPI_DGLU = 2 };

// chunk swizzle of row r (see header)
__device__ __forceinline__ int rsw(int r) { return (-(r >> 2)) & 3; }

template <typename T>
__device__ __forceinline__ f32x4 mfma16(typename fa::MT<T>::x8 a, typename fa::MT<T>::x8 b,
                                        f32x4 c) {
  if constexpr (__is_same(T, bf16)) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// ds_read_b128 with a folded immediate, as asm so hipcc inserts no vmcnt(0)
// for the LDS-DMA in flight into other ring slots (consumer waits by hand).
template <int OFF, typename T>
__device__ __forceinline__ typename fa::MT<T>::x8 row_read_imm(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16 bits");
  typename fa::MT<T>::x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "i"(OFF));
  return r;
}

// Grouped tile order: lin -> (tm, tn).  g > 0: groups of g m-tiles x all
// n-tiles, m fastest; g < 0: groups of -g n-tiles x all m-tiles, n fastest.
__device__ __forceinline__ int2 tile_of(int lin, int ntm, int ntn, int g) {
  const bool bym = g > 0;
  const int gg = bym ? g : -g;
  const int nlong = bym ? ntn : ntm, nshort = bym ? ntm : ntn;
  const int grp = lin / (gg * nlong);
  const int first = grp * gg;
  const int gsize = min(gg, nshort - first);
  const int in_grp = lin - grp * gg * nlong;
  const int a = first + in_grp % gsize, b = in_grp / gsize;
  return bym ? int2{a, b} : int2{b, a};
}

struct NtArgs {
  const void* a;      // [M, K]
  const void* b;      // [N, K] (EPI_GLU: [2F, K])
  void* c;            // EPI_STORE: [M, N]; EPI_GLU: pre-activation [M, 2F]; EPI_DGLU: d(pre) [M, 2F]
  void* y;            // EPI_GLU: act output [M, F]
  const void* pre;    // EPI_DGLU: saved pre-activation [M, 2F]
  int64_t lda, ldb, ldc, ldy;
  int M, N, K;        // EPI_GLU / EPI_DGLU: N = F
  int ntm, ntn, gm;
  bool wave4_ok;      // 32-bit per-lane DMA offsets fit (the 4-wave kernel)
  RowMap am, cm;      // row-group remap of A rows (loads) and C rows (stores)
  int ksplit;         // EPI_STORE, persistent kernel: K split this many ways
  float* ws;          // ... fp32 partial tiles [ksplit][tiles][256][256] (ksplit > 1)
};

// logical row q -> physical row (RowMap in kernels.h); q < 2^31
__device__ __forceinline__ int64_t map_row(int64_t q, const RowMap& m) {
  if (m.rows == 0) return q;
  const uint32_t g = (uint32_t)q / (uint32_t)m.rows;
  return (int64_t)g * m.stride + m.offset + (int64_t)((uint32_t)q - g * (uint32_t)m.rows);
}


// ---- epilogue (both kernels) ------------------------------------------------
// A wave's 128 x WNC output tile, rounded to 16 bits, sits in LDS as
// [128 rows][WNC cols] with 16-B unit u of row r stored at unit u ^ (r & (U-1))
// (U = WNC / 8 units per row).  The accumulator of fragment (i, j) holds row
// 16 i + (l & 15), cols 16 j + 4 (l >> 4) .. +3 on lane l.
template <typename T, int FB>
__device__ __forceinline__ void acc_to_lds(const f32x4 (&acc)[8][FB], char* reg, int lane) {
  constexpr int U = 2 * FB, RB = 32 * FB;
  const int r0 = lane & 15, u0 = lane >> 5, h = (lane >> 4) & 1;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j) {
      const int row = 16 * i + r0;
      const int u = 2 * j + u0;
      typename fa::MT<T>::x4 v;
      v[0] = (T)acc[i][j][0]; v[1] = (T)acc[i][j][1];
      v[2] = (T)acc[i][j][2]; v[3] = (T)acc[i][j][3];
      *reinterpret_cast<typename fa::MT<T>::x4*>(reg + row * RB + ((u ^ (row & (U - 1))) << 4) + 8 * h) = v;
    }
}

// Rows of the LDS tile -> global as 16-B pieces.  gm0: first output row of
// the wave; gn0: first output column (STORE / DGLU) or first f (GLU: units
// 0..U/2-1 are up columns f.., units U/2.. the gate columns of the same f).
template <typename T, int EPI, int ACT, int WNC>
__device__ __forceinline__ void epilogue_rows(const NtArgs& p, const char* reg, int lane,
                                              int64_t gm0, int64_t gn0) {
  constexpr int U = WNC / 8, RB = 2 * WNC;
  typedef V16<T> V;
  const int M = p.M, N = p.N;
  auto unit = [&](int row, int u) {
    return *reinterpret_cast<const V*>(reg + row * RB + ((u ^ (row & (U - 1))) << 4));
  };
  if constexpr (EPI == EPI_GLU) {
    constexpr int LPR = U / 2, RPI = 64 / LPR, ITERS = 128 / RPI;
    const int u = lane % LPR;
    const int64_t f = gn0 + 8 * u;
    const bool fok = f < N;
    T* pre = reinterpret_cast<T*>(p.c);
    T* y = reinterpret_cast<T*>(p.y);
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
      const int row = RPI * it + lane / LPR;
      const V x1 = unit(row, u), x2 = unit(row, u + LPR);
      V o;
#pragma unroll
      for (int e = 0; e < V::N; ++e) o.v[e] = from_f<T>(to_f(x1.v[e]) * act<ACT>(to_f(x2.v[e])));
      const int64_t gm = gm0 + row;
      if (fok && gm < M) {
        const int64_t pr = map_row(gm, p.cm);
        st16(pre + pr * p.ldc + f, x1);
        st16(pre + pr * p.ldc + N + f, x2);
        st16(y + pr * p.ldy + f, o);
      }
    }
  } else {
    constexpr int LPR = U, RPI = 64 / LPR, ITERS = 128 / RPI;
    const int u = lane % LPR;
    const int64_t gn = gn0 + 8 * u;
    const bool nok = gn < N;
    if constexpr (EPI == EPI_STORE) {
      T* c = reinterpret_cast<T*>(p.c);
#pragma unroll
      for (int it = 0; it < ITERS; ++it) {
        const int row = RPI * it + lane / LPR;
        const V v = unit(row, u);
        const int64_t gm = gm0 + row;
        if (nok && gm < M) st16(c + map_row(gm, p.cm) * p.ldc + gn, v);
      }
    } else {
      // d(pre) = [g * act(x2), g * x1 * act'(x2)], g = dAct rounded to T
      const T* pre = reinterpret_cast<const T*>(p.pre);
      T* d = reinterpret_cast<T*>(p.c);
      const int64_t gc = nok ? gn : 0;
#pragma unroll
      for (int b8 = 0; b8 < ITERS / 8; ++b8) {  // 8 rows of loads in flight
        V x1[8], x2[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          int64_t gm = gm0 + RPI * (8 * b8 + k) + lane / LPR;
          gm = gm < M ? gm : M - 1;
          x1[k] = ld16(pre + gm * p.ldc + gc);
          x2[k] = ld16(pre + gm * p.ldc + N + gc);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int row = RPI * (8 * b8 + k) + lane / LPR;
          const V g = unit(row, u);
          const int64_t gm = gm0 + row;
          V da, dg;
#pragma unroll
          for (int e = 0; e < V::N; ++e) {
            const float gv = to_f(g.v[e]);
            float av, dv;
            act_dact<ACT>(to_f(x2[k].v[e]), av, dv);
            da.v[e] = from_f<T>(gv * av);
            dg.v[e] = from_f<T>(gv * to_f(x1[k].v[e]) * dv);
          }
          if (nok && gm < M) {
            st16(d + gm * p.ldc + gn, da);
            st16(d + gm * p.ldc + N + gn, dg);
          }
        }
      }
    }
  }
}

template <typename T, int EPI, int ACT>
__global__ void __launch_bounds__(512, 1) gemm_nt_k(NtArgs p) {
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;  // wm is also the ping-pong group

  const int ntiles = p.ntm * p.ntn;
  const int lin = xcd_remap((int)blockIdx.x, ntiles);
  const int2 tt = tile_of(lin, p.ntm, p.ntn, p.gm);
  const int64_t m0 = (int64_t)tt.x * TM;
  // n origin of the tile: output columns (STORE / DGLU) or f (GLU: 128 per tile)
  const int64_t n0 = (int64_t)tt.y * (EPI == EPI_GLU ? TN / 2 : TN);
  const int M = p.M, N = p.N;

  // Per-lane DMA source pointers: wave w stages pieces 2w and 2w+1 (16 rows
  // each) of both operands; lane l lands on row 16 piece + (l >> 2), physical
  // chunk l & 3 = logical chunk (l & 3) ^ rsw(row) (rsw depends on l >> 4 only).
  const T* asrc[2];
  const T* bsrc[2];
  {
    const int c = (lane & 3) ^ ((-(lane >> 4)) & 3);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int tr = 16 * (2 * wave + i) + (lane >> 2);  // tile row 0..255
      int64_t am = m0 + tr;
      am = map_row(am < M ? am : M - 1, p.am);
      asrc[i] = reinterpret_cast<const T*>(p.a) + am * p.lda + 8 * c;
      int64_t bn;
      if constexpr (EPI == EPI_GLU) {
        // tile row -> W1 row: per 64-row wave band, 32 up rows then 32 gate rows
        const int band = tr >> 6, q = tr & 63;
        const int64_t f = n0 + 32 * band + (q & 31);
        bn = f < N ? (q < 32 ? f : N + f) : 0;
      } else {
        bn = n0 + tr;
        bn = bn < N ? bn : N - 1;
      }
      bsrc[i] = reinterpret_cast<const T*>(p.b) + bn * p.ldb + 8 * c;
    }
  }
  char* const ldsp = lds;
  auto stage_piece = [&](int q, int ts) {  // q: 0,1 = A pieces, 2,3 = B pieces
    const int dst = (ts % NSLOT) * SLOTB + (q >= 2 ? OPB : 0) + (2 * wave + (q & 1)) * 1024;
    const T* g = (q >= 2 ? bsrc[q & 1] : asrc[q & 1]) + (int64_t)ts * BK;
    __builtin_amdgcn_global_load_lds((const void*)g,
                                     (__attribute__((address_space(3))) void*)(ldsp + dst), 16, 0, 0);
  };
  auto stage = [&](int ts) {
    static_for<4>([&](auto q) { stage_piece(decltype(q)::value, ts); });
  };

  f32x4 acc[FA_][FB_];
#pragma unroll
  for (int i = 0; i < FA_; ++i)
#pragma unroll
    for (int j = 0; j < FB_; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read bases: row (l & 15) of the wave's band, logical chunk l >> 4
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const uint32_t fr_off = 64u * (lane & 15) + 16u * ((lane >> 4) ^ rsw(lane & 15));
  const uint32_t abase = fr_off + 64u * 128u * wm;
  const uint32_t bbase = OPB + fr_off + 64u * 64u * wn;

  typename fa::MT<T>::x8 fa_[FA_], fb_[FB_];
  auto reads = [&](int t) {
    const uint32_t so = lds_base + (uint32_t)((t % NSLOT) * SLOTB);
    const uint32_t a = so + abase, b = so + bbase;
    static_for<FA_>([&](auto f) {
      constexpr int F = decltype(f)::value;
      fa_[F] = row_read_imm<1024 * F, T>(a);
    });
    static_for<FB_>([&](auto f) {
      constexpr int F = decltype(f)::value;
      fb_[F] = row_read_imm<1024 * F, T>(b);
    });
  };
  const int nt = p.K / BK;
  auto mfmas = [&](int t) {
    __builtin_amdgcn_s_setprio(1);
    static_for<FA_>([&](auto i) {
      constexpr int I = decltype(i)::value;
#pragma unroll
      for (int j = 0; j < FB_; ++j) acc[I][j] = mfma16<T>(fb_[j], fa_[I], acc[I][j]);
      if constexpr (I == 3) {  // the 4th DMA piece of subtile t+3 rides here
        const int ts = t + NSLOT - 1;
        if (ts < nt) {
          __builtin_amdgcn_sched_barrier(0);
          stage_piece(3, ts);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    });
    __builtin_amdgcn_s_setprio(0);
  };

#pragma unroll
  for (int t = 0; t < NSLOT - 1; ++t)
    if (t < nt) stage(t);
  // subtile 0 landed (own DMA): at most min(nt, 3) - 1 subtiles outstanding
  if (nt >= 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (nt == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();               // ... and everyone's
  if (wm == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind

  // Phase t: [reads t][3 DMA pieces of t+3][vmcnt: t+1 landed][lgkmcnt(0)]
  //          BAR_A [32 MFMA + DMA piece 4 of t+3] BAR_B
  // RAW: subtile t+1 is retired by every wave before its BAR_A(t); both
  //      groups read it only after a later barrier.
  // WAR: stage(t+3) overwrites subtile t-1, whose reads every wave retired
  //      (lgkmcnt(0)) before its BAR_A(t-1), a barrier both groups passed.
  for (int t = 0; t < nt; ++t) {
    reads(t);
    if (t + NSLOT - 1 < nt) {
      static_for<3>([&](auto q) { stage_piece(decltype(q)::value, t + NSLOT - 1); });
      asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // t+2 (4) and t+3 (3) may fly
    } else {
      const int ahead = min(t + NSLOT - 2, nt - 1) - (t + 1);  // subtiles allowed in flight
      if (ahead >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    mfmas(t);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // balance the barrier count

  // ---- epilogue: every ring read retired before the last barrier, no DMA in
  // flight: each wave owns a 16 KiB region of the ring
  char* reg = lds + wave * 16384;
  acc_to_lds<T, FB_>(acc, reg, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  epilogue_rows<T, EPI, ACT, 64>(p, reg, lane, m0 + 128 * wm,
                                 n0 + (EPI == EPI_GLU ? 32 : 64) * wn);
}


// ---- 4-wave variant: one wave per SIMD, 128 x 128 per wave, K in steps of 64 --
// 64 accumulator tiles (256 fp32 per lane) pinned in AGPRs by asm MFMAs; the
// MFMA pipe is fed by the wave's own software pipeline instead of a partner
// wave.  A K-step of 64 is two MFMA k-halves; while the 64 MFMAs of one half
// run, the wave reads the next half's 16 fragments into the other register
// set (one ds_read_b128 per 4 MFMAs) and, in the second half, issues the DMA
// of step t+2 (one 1-KiB glds per 4 MFMAs).  Every DMA row is 128 B (a whole
// cache line; the 32-deep 8-wave form fetches half lines, twice the L2
// requests per byte), and half the fragment bytes per MFMA of the 8-wave
// form.  LDS: 2 slots x (A + B) x [256 rows][64 k] = 128 KiB, 16-B chunk c of
// row r at 16 (c ^ ((r >> 1) & 7)) (conflict-free fragment reads for both
// k-halves); one barrier per K-step.
constexpr int BK2 = 64;                     // K per step
constexpr int OPB2 = 256 * BK2 * 2;         // 32 KiB per operand per step
constexpr int SLOTB2 = 2 * OPB2;            // 64 KiB

template <typename T>
__device__ __forceinline__ void mfma_acc(f32x4& acc, typename fa::MT<T>::x8 a,
                                         typename fa::MT<T>::x8 b) {
  if constexpr (__is_same(T, bf16))
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

template <typename T>
__device__ __forceinline__ void mfma_zero(f32x4& acc, typename fa::MT<T>::x8 z) {
  if constexpr (__is_same(T, bf16))
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "=a"(acc) : "v"(z));
  else
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_f16 %0, %1, %1, 0" : "=a"(acc) : "v"(z));
}

template <typename T, int EPI, int ACT>
__global__ void __launch_bounds__(256, 1) gemm_nt4_k(NtArgs p) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * SLOTB2];
  typedef typename fa::MT<T>::x8 X8;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int ntiles = p.ntm * p.ntn;
  const int lin = xcd_remap((int)blockIdx.x, ntiles);
  const int2 tt = tile_of(lin, p.ntm, p.ntn, p.gm);
  const int64_t m0 = (int64_t)tt.x * TM;
  const int64_t n0 = (int64_t)tt.y * (EPI == EPI_GLU ? TN / 2 : TN);
  const int M = p.M, N = p.N;

  // DMA: each operand step is 32 pieces of 1 KiB (8 rows x 128 B); wave w
  // stages pieces 8w..8w+7 of A and of B.  Lane l lands on row 8 piece +
  // (l >> 3), physical chunk l & 7 = logical chunk (l & 7) ^ ((row >> 1) & 7).
  // Source = wave-uniform operand base + K-step byte offset (SGPRs) + a
  // 32-bit per-lane offset (host-checked to fit).
  uint32_t off[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int tr = 8 * (8 * wave + i) + (lane >> 3);  // tile row 0..255
    const int c = (lane & 7) ^ ((tr >> 1) & 7);
    int64_t am = m0 + tr;
    am = map_row(am < M ? am : M - 1, p.am);
    off[i] = (uint32_t)((am * p.lda + 8 * c) * (int64_t)sizeof(T));
    int64_t bn;
    if constexpr (EPI == EPI_GLU) {
      // per 128-row wave band: 64 up rows then the 64 gate rows of the same f
      const int band = tr >> 7, q = tr & 127;
      const int64_t f = n0 + 64 * band + (q & 63);
      bn = f < N ? (q < 64 ? f : N + f) : 0;
    } else {
      bn = n0 + tr;
      bn = bn < N ? bn : N - 1;
    }
    off[8 + i] = (uint32_t)((bn * p.ldb + 8 * c) * (int64_t)sizeof(T));
  }
  const char* const abyte = reinterpret_cast<const char*>(p.a);
  const char* const bbyte = reinterpret_cast<const char*>(p.b);
  char* const ldsp = lds;
  const int nt = p.K / BK2;
  // piece q (0..7 A, 8..15 B) of K-step ts -> LDS slot `slot`
  auto stage_piece = [&](int q, int ts, int slot) {
    const char* base = (q < 8 ? abyte : bbyte) + (int64_t)ts * (BK2 * (int)sizeof(T));
    const int dst = slot * SLOTB2 + (q >= 8 ? OPB2 : 0) + (8 * wave + (q & 7)) * 1024;
    __builtin_amdgcn_global_load_lds((const void*)(base + off[q]),
                                     (__attribute__((address_space(3))) void*)(ldsp + dst), 16, 0, 0);
  };

  f32x4 acc[8][8];  // defined and updated only by asm MFMAs: AGPR-resident

  // fragment bases [k-half]: row (l & 15) of the wave's band, logical chunk
  // (l >> 4) + 4 kh; fragment i adds 2048 i, slot s adds s * SLOTB2
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const int fr = lane & 15, fsw = (fr >> 1) & 7;
  uint32_t abase[2], bbase[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const uint32_t ch = 16u * (uint32_t)(((lane >> 4) + 4 * kh) ^ fsw);
    abase[kh] = lds_base + 128u * (128u * wm + fr) + ch;
    bbase[kh] = lds_base + OPB2 + 128u * (128u * wn + fr) + ch;
  }
  X8 set0[16], set1[16];  // k-half 0 / 1 fragments: [0..7] A (m), [8..15] B (n)
  auto read_frag = [&](X8 (&dst)[16], auto f, auto kh, uint32_t so) {
    constexpr int F = decltype(f)::value, KH = decltype(kh)::value;
    if constexpr (F < 8) dst[F] = row_read_imm<2048 * F, T>(abase[KH] + so);
    else dst[F] = row_read_imm<2048 * (F - 8), T>(bbase[KH] + so);
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  auto mfma4 = [&](X8 (&cur)[16], auto g) {
    constexpr int G = decltype(g)::value;
    static_for<4>([&](auto q) {
      constexpr int IDX = 4 * G + decltype(q)::value, I = IDX / 8, J = IDX % 8;
      mfma_acc<T>(acc[I][J], cur[8 + J], cur[I]);
    });
  };

  // prologue: steps 0 and 1 in flight, acc zeroed meanwhile, k-half (0,0) read
  static_for<16>([&](auto q) { stage_piece(decltype(q)::value, 0, 0); });
  static_for<16>([&](auto q) { stage_piece(decltype(q)::value, min(1, nt - 1), 1); });
  {
    X8 z;
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = (T)0.f;
    static_for<64>([&](auto q) {
      constexpr int I = decltype(q)::value / 8, J = decltype(q)::value % 8;
      mfma_zero<T>(acc[I][J], z);
    });
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // step 0 landed (own DMA)
  __builtin_amdgcn_s_barrier();                      // ... and everyone's
  static_for<16>([&](auto f) { read_frag(set0, f, K0{}, 0u); });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // K-step t (slot t & 1):
  //   half 0: MFMAs on set0 = (t, 0); read (t, 1) -> set1 from slot t
  //           vmcnt(0): step t+1 landed (own DMA, issued in half (t-1, 1))
  //           lgkmcnt(0); BARRIER
  //   half 1: MFMAs on set1; read (t+1, 0) -> set0 from slot t+1;
  //           DMA of step t+2 -> slot t (clamped to the last step past the end)
  //           lgkmcnt(0)
  // RAW: step t+1 is retired by every wave before the barrier, and read only
  //      after it.  WAR: slot t's last reads ((t, 1)) are retired before the
  //      barrier, the DMA into it is issued after.
  for (int t = 0; t < nt; ++t) {
    const uint32_t so = (uint32_t)((t & 1) * SLOTB2), sn = (uint32_t)(SLOTB2 - so);
    static_for<16>([&](auto g) {
      mfma4(set0, g);
      read_frag(set1, g, K1{}, so);
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int ts = min(t + 2, nt - 1), slot = t & 1;
    static_for<16>([&](auto g) {
      mfma4(set1, g);
      read_frag(set0, g, K0{}, sn);
      stage_piece(decltype(g)::value, ts, slot);
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing re-fetches
  __builtin_amdgcn_s_barrier();
  fa::mfma_drain();  // VALU reads of the asm MFMAs' results

  // epilogue: no ring read or DMA is pending
  char* reg = lds + wave * 32768;
  acc_to_lds<T, 8>(acc, reg, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  epilogue_rows<T, EPI, ACT, 128>(p, reg, lane, m0 + 128 * wm,
                                  n0 + (EPI == EPI_GLU ? 64 : 128) * wn);
}

// ---- 4-wave variant, early-refill schedule (variant 5) ---------------------
// Same tile, LDS image and fragment sets as gemm_nt4_k, but each operand's
// half of a ring slot is refilled as soon as every wave has read it, and the
// wait for the next K-step sits three quarters into the current one, so a
// DMA piece has 1.0-1.5 K-steps (not 0.5-1.0) to land.  One K-step = 32
// groups of 4 MFMAs; after group G:
//   G 0-3   read 2 A fragments of (t, k-half 1) -> set1
//   G 5     lgkmcnt(0), BARRIER 1   (A of slot t read by every wave)
//   G 6-13  DMA one A piece of step t+2 -> slot t
//   G 6-9   read 2 B fragments of (t, k-half 1) -> set1
//   G 11    lgkmcnt(0), BARRIER 2   (B of slot t read by every wave)
//   G 12-19 DMA one B piece of step t+2 -> slot t
//   G 23    vmcnt(16), BARRIER 3    (step t+1 landed, own DMA then everyone's)
//   G 24-31 read 2 fragments of (t+1, k-half 0) -> set0 from slot t+1
// then lgkmcnt(0).  Groups 0-15 run on set0 (k-half 0), 16-31 on set1.
template <typename T, int EPI, int ACT>
__global__ void __launch_bounds__(256, 1) gemm_nt5_k(NtArgs p) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * SLOTB2];
  typedef typename fa::MT<T>::x8 X8;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int ntiles = p.ntm * p.ntn;
  const int lin = xcd_remap((int)blockIdx.x, ntiles);
  const int2 tt = tile_of(lin, p.ntm, p.ntn, p.gm);
  const int64_t m0 = (int64_t)tt.x * TM;
  const int64_t n0 = (int64_t)tt.y * (EPI == EPI_GLU ? TN / 2 : TN);
  const int M = p.M, N = p.N;

  uint32_t off[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int tr = 8 * (8 * wave + i) + (lane >> 3);
    const int c = (lane & 7) ^ ((tr >> 1) & 7);
    int64_t am = m0 + tr;
    am = map_row(am < M ? am : M - 1, p.am);
    off[i] = (uint32_t)((am * p.lda + 8 * c) * (int64_t)sizeof(T));
    int64_t bn;
    if constexpr (EPI == EPI_GLU) {
      const int band = tr >> 7, q = tr & 127;
      const int64_t f = n0 + 64 * band + (q & 63);
      bn = f < N ? (q < 64 ? f : N + f) : 0;
    } else {
      bn = n0 + tr;
      bn = bn < N ? bn : N - 1;
    }
    off[8 + i] = (uint32_t)((bn * p.ldb + 8 * c) * (int64_t)sizeof(T));
  }
  const char* const abyte = reinterpret_cast<const char*>(p.a);
  const char* const bbyte = reinterpret_cast<const char*>(p.b);
  char* const ldsp = lds;
  const int nt = p.K / BK2;
  auto stage_piece = [&](int q, int ts, int slot) {
    const char* base = (q < 8 ? abyte : bbyte) + (int64_t)ts * (BK2 * (int)sizeof(T));
    const int dst = slot * SLOTB2 + (q >= 8 ? OPB2 : 0) + (8 * wave + (q & 7)) * 1024;
    __builtin_amdgcn_global_load_lds((const void*)(base + off[q]),
                                     (__attribute__((address_space(3))) void*)(ldsp + dst), 16, 0, 0);
  };

  f32x4 acc[8][8];
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const int fr = lane & 15, fsw = (fr >> 1) & 7;
  uint32_t abase[2], bbase[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const uint32_t ch = 16u * (uint32_t)(((lane >> 4) + 4 * kh) ^ fsw);
    abase[kh] = lds_base + 128u * (128u * wm + fr) + ch;
    bbase[kh] = lds_base + OPB2 + 128u * (128u * wn + fr) + ch;
  }
  X8 set0[16], set1[16];
  auto read_frag = [&](X8 (&dst)[16], auto f, auto kh, uint32_t so) {
    constexpr int F = decltype(f)::value, KH = decltype(kh)::value;
    if constexpr (F < 8) dst[F] = row_read_imm<2048 * F, T>(abase[KH] + so);
    else dst[F] = row_read_imm<2048 * (F - 8), T>(bbase[KH] + so);
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;
  auto mfma4 = [&](X8 (&cur)[16], auto g) {
    constexpr int G = decltype(g)::value;
    static_for<4>([&](auto q) {
      constexpr int IDX = 4 * G + decltype(q)::value, I = IDX / 8, J = IDX % 8;
      mfma_acc<T>(acc[I][J], cur[8 + J], cur[I]);
    });
  };

  static_for<16>([&](auto q) { stage_piece(decltype(q)::value, 0, 0); });
  static_for<16>([&](auto q) { stage_piece(decltype(q)::value, min(1, nt - 1), 1); });
  {
    X8 z;
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = (T)0.f;
    static_for<64>([&](auto q) {
      constexpr int I = decltype(q)::value / 8, J = decltype(q)::value % 8;
      mfma_zero<T>(acc[I][J], z);
    });
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  static_for<16>([&](auto f) { read_frag(set0, f, K0{}, 0u); });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  for (int t = 0; t < nt; ++t) {
    const uint32_t so = (uint32_t)((t & 1) * SLOTB2), sn = (uint32_t)(SLOTB2 - so);
    const int ts = min(t + 2, nt - 1), slot = t & 1;
    static_for<32>([&](auto g) {
      constexpr int G = decltype(g)::value;
      if constexpr (G < 16) mfma4(set0, std::integral_constant<int, G>{});
      else mfma4(set1, std::integral_constant<int, G - 16>{});
      if constexpr (G < 4) {
        read_frag(set1, std::integral_constant<int, 2 * G>{}, K1{}, so);
        read_frag(set1, std::integral_constant<int, 2 * G + 1>{}, K1{}, so);
      }
      if constexpr (G == 5 || G == 11) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
      }
      if constexpr (G >= 6 && G < 14) stage_piece(G - 6, ts, slot);
      if constexpr (G >= 6 && G < 10) {
        read_frag(set1, std::integral_constant<int, 8 + 2 * (G - 6)>{}, K1{}, so);
        read_frag(set1, std::integral_constant<int, 9 + 2 * (G - 6)>{}, K1{}, so);
      }
      if constexpr (G >= 12 && G < 20) stage_piece(8 + G - 12, ts, slot);
      if constexpr (G == 23) {
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
      }
      if constexpr (G >= 24) {
        read_frag(set0, std::integral_constant<int, 2 * (G - 24)>{}, K0{}, sn);
        read_frag(set0, std::integral_constant<int, 2 * (G - 24) + 1>{}, K0{}, sn);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  fa::mfma_drain();

  char* reg = lds + wave * 32768;
  acc_to_lds<T, 8>(acc, reg, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  epilogue_rows<T, EPI, ACT, 128>(p, reg, lane, m0 + 128 * wm,
                                  n0 + (EPI == EPI_GLU ? 64 : 128) * wn);
}

// ---- persistent 4-wave variant (variant 6, EPI_STORE without row maps) ------
// The early-refill K-step of gemm_nt5_k, run as one continuous stream of
// K-steps over all the tiles a workgroup owns (grid = one workgroup per CU,
// tiles dealt round-robin in XCD-grouped order).  The DMA of the next tile's
// first two K-steps rides in the current tile's last two K-steps, so a tile
// starts with its operands already in LDS; the epilogue goes from registers
// straight to global memory (bf16 pack + two permlane swaps give each lane 8
// consecutive columns, one 16-B store per fragment pair), leaving the LDS ring
// to the next tile's data; the first k-half of a tile accumulates onto C = 0.
// Operands are read by buffer_load ... lds through a per-tile descriptor whose
// size ends at the last valid row: rows past M / N read as zeros (no clamping).
template <typename T>
__device__ __forceinline__ void mfma_acc0(f32x4& acc, typename fa::MT<T>::x8 a,
                                          typename fa::MT<T>::x8 b) {
  if constexpr (__is_same(T, bf16))
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

template <typename T>
__device__ __forceinline__ uint2 pack4(f32x4 v) {
  typename fa::MT<T>::x4 h;
  h[0] = (T)v[0]; h[1] = (T)v[1]; h[2] = (T)v[2]; h[3] = (T)v[3];
  return *reinterpret_cast<uint2*>(&h);
}

typedef __amdgpu_buffer_rsrc_t Rsrc;

// Two accumulator fragments (cols 16 j + 4 q' and 16 (j+1) + 4 q' of one row on
// lane group q' = lane >> 4), packed to 16 bits, become 8 CONSECUTIVE columns
// 8 q' .. 8 q' + 7 of the fragment pair on every lane: one permlane32 and one
// permlane16 swap per dword.
__device__ __forceinline__ uint4 pair_to_row8(uint2 x, uint2 y) {
  auto s0 = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
  auto s1 = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
  auto t0 = __builtin_amdgcn_permlane16_swap(s0[0], s0[1], false, false);
  auto t1 = __builtin_amdgcn_permlane16_swap(s1[0], s1[1], false, false);
  return make_uint4(t0[0], t1[0], t0[1], t1[1]);
}

template <typename T>
__device__ __forceinline__ f32x4 unpack4(uint2 v) {
  typename fa::MT<T>::x4 h = *reinterpret_cast<typename fa::MT<T>::x4*>(&v);
  return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
}

// Register epilogue of the persistent kernel: the wave's 128 x 128 accumulator
// tile at (gm0, gn0).  STORE: C; GLU: gn0 is the first f, fragments 0-3 are up,
// 4-7 the gate of the same f (pre-activation and y = up * act(gate) stored);
// DGLU: d(pre) from dAct (rounded to T) and the saved pre-activation.
template <typename T, int EPI, int ACT>
__device__ __forceinline__ void epilogue_regs(const NtArgs& p, const f32x4 (&acc)[8][8], int lane,
                                              int64_t gm0, int64_t gn0) {
  typedef V16<T> V;
  const int M = p.M, N = p.N, q = lane >> 4;
#pragma unroll
  for (int ii = 0; ii < 8; ++ii) {
    const int64_t row = gm0 + 16 * ii + (lane & 15);
    const bool rok = row < M;
    if constexpr (EPI == EPI_STORE) {
      T* c = reinterpret_cast<T*>(p.c);
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const uint4 v = pair_to_row8(pack4<T>(acc[ii][2 * jp]), pack4<T>(acc[ii][2 * jp + 1]));
        const int64_t col = gn0 + 32 * jp + 8 * q;
        if (rok && col < N) *reinterpret_cast<uint4*>(c + map_row(row, p.cm) * p.ldc + col) = v;
      }
    } else if constexpr (EPI == EPI_GLU) {
      T* pre = reinterpret_cast<T*>(p.c);
      T* y = reinterpret_cast<T*>(p.y);
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        uint2 u[2], g[2], yy[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          u[e] = pack4<T>(acc[ii][2 * jp + e]);
          g[e] = pack4<T>(acc[ii][4 + 2 * jp + e]);
          const f32x4 uf = unpack4<T>(u[e]), gf = unpack4<T>(g[e]);
          yy[e] = pack4<T>(f32x4{uf[0] * act<ACT>(gf[0]), uf[1] * act<ACT>(gf[1]),
                                 uf[2] * act<ACT>(gf[2]), uf[3] * act<ACT>(gf[3])});
        }
        const uint4 vu = pair_to_row8(u[0], u[1]), vg = pair_to_row8(g[0], g[1]);
        const uint4 vy = pair_to_row8(yy[0], yy[1]);
        const int64_t f = gn0 + 32 * jp + 8 * q;
        if (rok && f < N) {
          const int64_t pr = map_row(row, p.cm);
          *reinterpret_cast<uint4*>(pre + pr * p.ldc + f) = vu;
          *reinterpret_cast<uint4*>(pre + pr * p.ldc + N + f) = vg;
          *reinterpret_cast<uint4*>(y + pr * p.ldy + f) = vy;
        }
      }
    }
  }
  if constexpr (EPI == EPI_DGLU) {
    // d(pre) from dAct (rounded to T) and the saved pre-activation, software-
    // pipelined over the 8 row groups: the pre loads of D groups are in flight
    // while a group computes and stores (the epilogue was latency-bound: one
    // group's 8 loads at a time)
    const T* pre = reinterpret_cast<const T*>(p.pre);
    T* d = reinterpret_cast<T*>(p.c);
    constexpr int D = 3;
    V x1[D][4], x2[D][4];
    auto load = [&](int ii, V (&a)[4], V (&b)[4]) {
      const int64_t row = gm0 + 16 * ii + (lane & 15);
      const int64_t rr = row < M ? row : M - 1;
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        int64_t f = gn0 + 32 * jp + 8 * q;
        f = f < N ? f : 0;
        a[jp] = ld16(pre + rr * p.ldc + f);
        b[jp] = ld16(pre + rr * p.ldc + N + f);
      }
    };
    static_for<D>([&](auto k) { load(decltype(k)::value, x1[decltype(k)::value], x2[decltype(k)::value]); });
    static_for<8>([&](auto iic) {
      constexpr int ii = decltype(iic)::value, sl = ii % D;
      const int64_t row = gm0 + 16 * ii + (lane & 15);
      const bool rok = row < M;
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const uint4 gv = pair_to_row8(pack4<T>(acc[ii][2 * jp]), pack4<T>(acc[ii][2 * jp + 1]));
        const V g = *reinterpret_cast<const V*>(&gv);
        V da, dg;
#pragma unroll
        for (int e = 0; e < V::N; ++e) {
          const float gf = to_f(g.v[e]);
          float av, dv;
          act_dact<ACT>(to_f(x2[sl][jp].v[e]), av, dv);
          da.v[e] = from_f<T>(gf * av);
          dg.v[e] = from_f<T>(gf * to_f(x1[sl][jp].v[e]) * dv);
        }
        const int64_t f = gn0 + 32 * jp + 8 * q;
        if (rok && f < N) {
          st16(d + row * p.ldc + f, da);
          st16(d + row * p.ldc + N + f, dg);
        }
      }
      if constexpr (ii + D < 8) load(ii + D, x1[sl], x2[sl]);
    });
  }
}

template <typename T, int EPI, int ACT, bool SPK = false>
__global__ void __launch_bounds__(256, 1) gemm_nt6_k(NtArgs p) {
  // (ablation builds of this structure: scripts/lab/gemm_lab.hip, bench-only)
  __shared__ __attribute__((aligned(1024))) char lds[2 * SLOTB2];
  typedef typename fa::MT<T>::x8 X8;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = p.ntm * p.ntn;
  // split-K (EPI_STORE, few tiles): item = (split, tile), split-major; each
  // item runs nt = K / BK2 / ksplit K-steps from K-step ks * nt and stores
  // an fp32 partial tile, summed by gemm_nt_split_reduce_k
  static_assert(!SPK || EPI == EPI_STORE, "split-K: plain products only");
  const int ksplit = SPK ? p.ksplit : 1;
  const int nitems = ntiles * ksplit;
  const int G = gridDim.x, bid = blockIdx.x;
  if (bid >= nitems) return;
  const int nmine = (nitems - 1 - bid) / G + 1;
  const int M = p.M, N = p.N;
  const int nt = p.K / BK2 / ksplit;  // >= 2 (host-checked)

  // per-lane DMA byte offsets inside a tile (fixed for the whole kernel);
  // piece i of the 4 waves = 32 consecutive rows (+1-3 %, profiles/r4h_gemm_ablation.txt)
  uint32_t off[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int pb = 4 * i + wave;  // 8-row block of piece i
    const int tr = 8 * pb + (lane >> 3);
    const int c = (lane & 7) ^ ((tr >> 1) & 7);
    off[i] = (uint32_t)(tr * p.lda + 8 * c) * (uint32_t)sizeof(T);
    int br = tr;  // B row relative to the tile's first row n0
    if constexpr (EPI == EPI_GLU) {
      // per 128-row wave band: 64 up rows f then the 64 gate rows F + f
      const int band = tr >> 7, q = tr & 127;
      br = q < 64 ? 64 * band + q : N + 64 * band + (q - 64);
    }
    off[8 + i] = (uint32_t)(br * p.ldb + 8 * c) * (uint32_t)sizeof(T);
  }
  // tile i of this workgroup -> (m0, n0): n0 = first output column, or first
  // f (EPI_GLU: 128 per tile)
  auto tile_org = [&](int i, int64_t& m0, int64_t& n0, int& ks, int& lt) {
    const int base = i * G, rem = min(G, nitems - base);
    const int item = base + xcd_remap(bid, rem);
    ks = item / ntiles;
    lt = item - ks * ntiles;
    const int2 tt = tile_of(lt, p.ntm, p.ntn, p.gm);
    m0 = (int64_t)tt.x * TM;
    n0 = (int64_t)tt.y * (EPI == EPI_GLU ? TN / 2 : TN);
  };
  // descriptors of tile i (size 0 past the last tile: every load is dropped)
  auto make_rsrc = [&](int i, Rsrc& ra, Rsrc& rb) {
    int64_t m0 = 0, n0 = 0;
    int64_t na = 0, nb = 0;
    int64_t am0 = 0, koff = 0;  // koff: bytes of K before this item's split
    if (i < nmine) {
      int ks, lt;
      tile_org(i, m0, n0, ks, lt);
      koff = (int64_t)ks * nt * BK2 * (int64_t)sizeof(T);
      // a row map's groups hold whole 256-row tiles (host-checked): the tile's
      // physical rows are contiguous from map_row(m0)
      am0 = map_row(m0, p.am);
      const int64_t arows = p.am.rows == 0 ? M - m0 : min((int64_t)TM, (int64_t)M - m0);
      na = arows * p.lda * (int64_t)sizeof(T) - koff;
      nb = (int64_t)((EPI == EPI_GLU ? 2 * (int64_t)N : N) - n0) * p.ldb * (int64_t)sizeof(T) - koff;
    }
    const char* a = reinterpret_cast<const char*>(p.a) + am0 * p.lda * (int64_t)sizeof(T) + koff;
    const char* b = reinterpret_cast<const char*>(p.b) + n0 * p.ldb * (int64_t)sizeof(T) + koff;
    ra = __builtin_amdgcn_make_buffer_rsrc((void*)a, 0, (int)min(na, (int64_t)0x7fffffff), 0x00020000);
    rb = __builtin_amdgcn_make_buffer_rsrc((void*)b, 0, (int)min(nb, (int64_t)0x7fffffff), 0x00020000);
  };
  char* const ldsp = lds;
  auto dma = [&](int q, Rsrc r, uint32_t soff, int slot) {
    const int dst = slot * SLOTB2 + (q >= 8 ? OPB2 : 0) + (4 * (q & 7) + wave) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(ldsp + dst),
                                             16, off[q], soff, 0, 0);
  };

  f32x4 acc[8][8];
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const int fr = lane & 15, fsw = (fr >> 1) & 7;
  uint32_t abase[2], bbase[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) {
    const uint32_t ch = 16u * (uint32_t)(((lane >> 4) + 4 * kh) ^ fsw);
    abase[kh] = lds_base + 128u * (128u * wm + fr) + ch;
    bbase[kh] = lds_base + OPB2 + 128u * (128u * wn + fr) + ch;
  }
  X8 set0[16], set1[16];
  auto read_frag = [&](X8 (&dst)[16], auto f, auto kh, uint32_t so) {
    constexpr int F = decltype(f)::value, KH = decltype(kh)::value;
    if constexpr (F < 8) dst[F] = row_read_imm<2048 * F, T>(abase[KH] + so);
    else dst[F] = row_read_imm<2048 * (F - 8), T>(bbase[KH] + so);
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;

  Rsrc ra_c, rb_c, ra_n, rb_n;  // current / next tile
  make_rsrc(0, ra_c, rb_c);
  make_rsrc(1, ra_n, rb_n);
  static_for<8>([&](auto q) { dma(decltype(q)::value, ra_c, 0u, 0); });
  static_for<8>([&](auto q) { dma(8 + decltype(q)::value, rb_c, 0u, 0); });
  static_for<8>([&](auto q) { dma(decltype(q)::value, ra_c, BK2 * sizeof(T), 1); });
  static_for<8>([&](auto q) { dma(8 + decltype(q)::value, rb_c, BK2 * sizeof(T), 1); });
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  static_for<16>([&](auto f) { read_frag(set0, f, K0{}, 0u); });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  int par = 0;  // LDS slot of K-step 0 of the current tile
  for (int i = 0; i < nmine; ++i) {
    auto kstep = [&](int t, auto zero) {
      const int slot = (t + par) & 1;
      const uint32_t so = (uint32_t)(slot * SLOTB2), sn = (uint32_t)(SLOTB2 - so);
      // source of K-step t+2: this tile, else the next tile's step t+2-nt
      const bool here = t + 2 < nt;
      const Rsrc ra = here ? ra_c : ra_n, rb = here ? rb_c : rb_n;
      const uint32_t soff = (uint32_t)((here ? t + 2 : t + 2 - nt) * BK2 * (int)sizeof(T));
      // One-MFMA slot plan (kNtPlan: events after MFMA index S; +1-5 % over
      // the round-4 plan, profiles/r5e_gemm_lab.txt)
      constexpr int VMW = nt_plan_vmw();
      static_for<128>([&](auto sc) {
        constexpr int S = decltype(sc)::value, IDX = S & 63, I = IDX / 8, J = IDX % 8;
        if constexpr (S < 64) {
          if constexpr (decltype(zero)::value) mfma_acc0<T>(acc[I][J], set0[8 + J], set0[I]);
          else mfma_acc<T>(acc[I][J], set0[8 + J], set0[I]);
        } else {
          mfma_acc<T>(acc[I][J], set1[8 + J], set1[I]);
        }
        static_for<16>([&](auto ec) {
          constexpr int E = decltype(ec)::value;
          if constexpr (kNtPlan.rd1[E] == S) read_frag(set1, std::integral_constant<int, E>{}, K1{}, so);
          if constexpr (kNtPlan.dma[E] == S) dma(E, E < 8 ? ra : rb, soff, slot);
          if constexpr (kNtPlan.rd0[E] == S) read_frag(set0, std::integral_constant<int, E>{}, K0{}, sn);
        });
        if constexpr (S == kNtPlan.b1 || S == kNtPlan.b2) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (S == kNtPlan.w) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VMW) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    kstep(0, std::true_type{});
    for (int t = 1; t < nt; ++t) kstep(t, std::false_type{});

    // epilogue of tile i: registers -> global, while the next tile's first two
    // K-steps are (or have been) landing in LDS
    fa::mfma_drain();
    int64_t m0, n0;
    int ks, lt;
    tile_org(i, m0, n0, ks, lt);
    if constexpr (SPK) {
      // fp32 partial: the wave's 128 x 128 block of the dense 256 x 256 tile
      float* w = p.ws + ((int64_t)ks * ntiles + lt) * (TM * TN) + (128 * wm + (lane & 15)) * TN +
                 128 * wn + 4 * (lane >> 4);
      static_for<8>([&](auto iic) {
        constexpr int ii = decltype(iic)::value;
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
          __builtin_nontemporal_store(acc[ii][jj], reinterpret_cast<f32x4*>(w + 16 * ii * TN + 16 * jj));
        __builtin_amdgcn_sched_barrier(0);  // one row group's accumulators in VGPRs at a time
      });
    } else {
      epilogue_regs<T, EPI, ACT>(p, acc, lane, m0 + 128 * wm, n0 + (EPI == EPI_GLU ? 64 : 128) * wn);
    }
    par ^= nt & 1;
    ra_c = ra_n;
    rb_c = rb_n;
    make_rsrc(i + 2, ra_n, rb_n);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// C[tile] = sum over the K splits of ws[split][tile] (fixed order), rounded
// to T, stored through the C row map; 64 workgroups x 256 threads x 4 per tile
template <typename T>
__global__ __launch_bounds__(256) void gemm_nt_split_reduce_k(NtArgs p) {
  const int ntiles = p.ntm * p.ntn;
  const int lt = blockIdx.x / 64, part = blockIdx.x % 64;
  const int2 tt = tile_of(lt, p.ntm, p.ntn, p.gm);
  const int e = (part * 256 + threadIdx.x) * 4;
  const int row = e / TN, col = e % TN;
  const int64_t m = (int64_t)tt.x * TM + row, n = (int64_t)tt.y * TN + col;
  if (m >= p.M || n >= p.N) return;  // N % 8 == 0: a 4-column piece is all in or all out
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < p.ksplit; ++ks)
    acc += __builtin_nontemporal_load(
        reinterpret_cast<const f32x4*>(p.ws + ((int64_t)ks * ntiles + lt) * (TM * TN) + e));
  *reinterpret_cast<uint2*>(reinterpret_cast<T*>(p.c) + map_row(m, p.cm) * p.ldc + n) = pack4<T>(acc);
}

// K split of a plain / row-mapped product on the persistent kernel: products
// of fewer than half a grid of tiles (TP-sharded narrow outputs: the 70B TP8
// qkv pieces are 80 tiles, the dense dgrad pieces 64) split K so that about
// one item per CU runs; at least 8 K-steps of 64 per item.  EMA_GEMM_NT_SPLITK=0
// disables.
int nt_ksplit(int tiles, int64_t K) {
  static const bool on = [] {
    const char* e = getenv("EMA_GEMM_NT_SPLITK");
    return !(e && e[0] == '0');
  }();
  const int ncu = 256;  // plan independent of the device queried (host tests)
  if (!on || tiles * 2 > ncu || K % BK2 != 0) return 1;
  const int steps = (int)(K / BK2);
  int best = 1;
  for (int sp = 2; sp <= 8; ++sp)
    if (tiles * sp <= ncu && steps % sp == 0 && steps / sp >= 8) best = sp;
  return best;
}

// Tile grouping of the persistent kernel's tile order (tile_of): groups of 4
// m-tiles x all n-tiles.  Measured against the round-4 rule (8 m-tiles, or 8
// n-tiles when M has more tiles) on the 7B shapes, one box
// (profiles/r6t_gemm_group_sweep.txt): fc1 + GLU +3.8 %, fc2 dgrad + dGLU
// +2.7 %, plain products +0.5 %.  EMA_GEMM_GM=<g> overrides (> 0: groups of g
// m-tiles, < 0: groups of -g n-tiles); EMA_GEMM_GM=old restores the old rule.
int group_m(int ntm, int ntn) {
  static const int env = [] {
    const char* e = getenv("EMA_GEMM_GM");
    if (e && e[0] == 'o') return 1 << 20;
    return e ? atoi(e) : 0;
  }();
  if (env == 1 << 20) return ntm <= ntn ? 8 : -8;
  if (env != 0) return env;
  return 4;
}

#define EMA_GLU_KIND2(kind, ...)                              \
  switch (kind) {                                             \
    case 0: { constexpr int A_ = 0; __VA_ARGS__; break; }     \
    case 1: { constexpr int A_ = 1; __VA_ARGS__; break; }     \
    case 2: { constexpr int A_ = 2; __VA_ARGS__; break; }     \
    default: { constexpr int A_ = 3; __VA_ARGS__; break; }    \
  }

// Kernel variant per epilogue: 6 (persistent 4-wave, register epilogue; row
// maps fall back to 5), 5 (one-shot early-refill 4-wave), 4 (one-shot, one
// refill point), 8 (8-wave ping-pong).  Defaults from interleaved same-box
// A/B on the 7B shapes (profiles/r5g_gemm_nt_bench.txt): 6 everywhere (fc1 +
// GLU 1.04x hipBLASLt + glu kernel vs 1.02x on 5; fc2 dgrad + dGLU 1.13x vs
// 1.05x; plain products 0.93-0.99x hipBLASLt, so those stay on hipBLASLt
// in-model unless a row map needs this kernel).
// EMA_GEMM_NT=<v> or gemm_nt_set_variant(v) forces one variant everywhere
// (EMA_GEMM_NT_STORE=<v>: the plain / row-mapped products only)
// (A/B in one process); gemm_nt_set_variant(0) restores the defaults.
int g_var[3] = {6, 6, 6};  // [EPI_STORE, EPI_GLU, EPI_DGLU]
int parse_variant(int v) { return (v == 4 || v == 5 || v == 6 || v == 8) ? v : 0; }
const int g_env_variant = [] {
  const char* e = getenv("EMA_GEMM_NT");
  const int v = e ? parse_variant(atoi(e)) : 0;
  if (v) g_var[0] = g_var[1] = g_var[2] = v;
  const char* es = getenv("EMA_GEMM_NT_STORE");  // plain / row-mapped products only
  const int vs = es ? parse_variant(atoi(es)) : 0;
  if (vs) g_var[0] = vs;
  return v;
}();

int num_cus() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <typename T, int EPI, int ACT>
void launch_one(const NtArgs& p, hipStream_t s) {
  const dim3 grid((unsigned)(p.ntm * p.ntn));
  // (the GeGLU backward's erf-based derivative would spill the accumulators:
  // that form stays on the one-shot kernel)
  if constexpr (!(EPI == EPI_DGLU && ACT == 1)) {
    const int64_t lim = (int64_t)1 << 31;
    const int64_t brows = EPI == EPI_GLU ? 2 * (int64_t)p.N : p.N;
    // row maps: the persistent kernel reads a mapped A tile as one contiguous
    // block, so the map's groups must hold whole 256-row tiles (the SP
    // pipeline's pieces do at the BASELINE sizes: 512-1024 rows)
    const bool maps_ok = (p.am.rows == 0 || p.am.rows % TM == 0) && (p.cm.rows == 0 || p.cm.rows % TM == 0);
    const int64_t a_extent = p.am.rows == 0 ? (int64_t)p.M : (int64_t)TM;  // rows one descriptor spans
    if (g_var[EPI] == 6 && p.K % BK2 == 0 && p.K >= 2 * BK2 && maps_ok &&
        a_extent * p.lda * 2 < lim && brows * p.ldb * 2 < lim) {
      if constexpr (EPI == EPI_STORE) {
        if (p.ws && p.ksplit > 1) {  // few tiles: K split over fp32 partials
          const int g = std::min(p.ntm * p.ntn * p.ksplit, num_cus());
          hipLaunchKernelGGL((gemm_nt6_k<T, EPI, ACT, true>), dim3(g), dim3(256), 0, s, p);
          hipLaunchKernelGGL(gemm_nt_split_reduce_k<T>, dim3((unsigned)(p.ntm * p.ntn * 64)),
                             dim3(256), 0, s, p);
          return;
        }
      }
      NtArgs q = p;
      q.ksplit = 1;
      const int g = std::min(p.ntm * p.ntn, num_cus());
      hipLaunchKernelGGL((gemm_nt6_k<T, EPI, ACT>), dim3(g), dim3(256), 0, s, q);
      return;
    }
  }
  const bool w4 = g_var[EPI] != 8 && p.K % BK2 == 0 && p.wave4_ok;
  if (w4 && g_var[EPI] != 4) hipLaunchKernelGGL((gemm_nt5_k<T, EPI, ACT>), grid, dim3(256), 0, s, p);
  else if (w4) hipLaunchKernelGGL((gemm_nt4_k<T, EPI, ACT>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((gemm_nt_k<T, EPI, ACT>), grid, dim3(512), 0, s, p);
}

template <int EPI>
void launch_nt(NtArgs& p, int kind, int dt, hipStream_t s) {
  const int n_out = EPI == EPI_GLU ? (p.N + TN / 2 - 1) / (TN / 2) : (p.N + TN - 1) / TN;
  p.ntm = (p.M + TM - 1) / TM;
  p.ntn = n_out;
  p.gm = group_m(p.ntm, p.ntn);
  const int64_t brows = EPI == EPI_GLU ? 2 * (int64_t)p.N : p.N;
  // highest A row read (through the remap: groups are increasing in q)
  const int64_t arows = p.am.rows == 0 ? p.M
      : ((int64_t)(p.M - 1) / p.am.rows) * p.am.stride + p.am.offset + (p.M - 1) % p.am.rows + 1;
  p.wave4_ok = arows * p.lda * 2 < ((int64_t)1 << 32) && brows * p.ldb * 2 < ((int64_t)1 << 32);
  if constexpr (EPI == EPI_STORE) {
    if (dt == DT_BF16) launch_one<bf16, EPI, 0>(p, s);
    else launch_one<fp16, EPI, 0>(p, s);
  } else if (dt == DT_BF16) {
    EMA_GLU_KIND2(kind, (launch_one<bf16, EPI, A_>(p, s)));
  } else {
    EMA_GLU_KIND2(kind, (launch_one<fp16, EPI, A_>(p, s)));
  }
}

}  // namespace

void gemm_nt_set_variant(int v) {
  v = parse_variant(v);
  if (v) {
    g_var[0] = g_var[1] = g_var[2] = v;
  } else {
    g_var[0] = 6; g_var[1] = 6; g_var[2] = 6;
  }
}

bool gemm_nt_supported(int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc) {
  return M > 0 && N > 0 && K > 0 && K % BK == 0 && N % 8 == 0 && lda % 8 == 0 && ldb % 8 == 0 &&
         ldc % 8 == 0 && M < ((int64_t)1 << 31) && N < ((int64_t)1 << 30) &&
         ((M + TM - 1) / TM) * ((N + TN / 2 - 1) / (TN / 2)) < ((int64_t)1 << 31);
}

int gemm_nt_ksplit(int64_t M, int64_t N, int64_t K) {
  if (g_var[EPI_STORE] != 6) return 1;
  return nt_ksplit((int)(((M + TM - 1) / TM) * ((N + TN - 1) / TN)), K);
}

int64_t gemm_nt_workspace_floats(int64_t M, int64_t N, int64_t K) {
  if (g_var[EPI_STORE] != 6) return 0;
  const int tiles = (int)(((M + TM - 1) / TM) * ((N + TN - 1) / TN));
  const int sp = nt_ksplit(tiles, K);
  return sp > 1 ? (int64_t)sp * tiles * TM * TN : 0;
}

void gemm_nt(const void* a, const void* b, void* c, int64_t M, int64_t N, int64_t K, int64_t lda,
             int64_t ldb, int64_t ldc, int dt, hipStream_t s, RowMap amap, RowMap cmap, float* ws) {
  NtArgs p{a, b, c, nullptr, nullptr, lda, ldb, ldc, 0, (int)M, (int)N, (int)K, 0, 0, 0, false,
           amap, cmap, 1, nullptr};
  if (ws) {
    p.ksplit = nt_ksplit((int)(((M + TM - 1) / TM) * ((N + TN - 1) / TN)), K);
    p.ws = p.ksplit > 1 ? ws : nullptr;
    if (!p.ws) p.ksplit = 1;
  }
  launch_nt<EPI_STORE>(p, 0, dt, s);
}

void gemm_nt_glu(const void* a, const void* b, void* pre, void* y, int64_t M, int64_t F,
                 int64_t K, int64_t lda, int64_t ldb, int kind, int dt, hipStream_t s,
                 RowMap cmap) {
  NtArgs p{a, b, pre, y, nullptr, lda, ldb, 2 * F, F, (int)M, (int)F, (int)K, 0, 0, 0, false,
           RowMap{}, cmap, 1, nullptr};
  launch_nt<EPI_GLU>(p, kind, dt, s);
}

void gemm_nt_dglu(const void* a, const void* b, const void* pre, void* dpre, int64_t M, int64_t F,
                  int64_t K, int64_t lda, int64_t ldb, int kind, int dt, hipStream_t s) {
  NtArgs p{a, b, dpre, nullptr, pre, lda, ldb, 2 * F, 0, (int)M, (int)F, (int)K, 0, 0, 0, false,
           RowMap{}, RowMap{}, 1, nullptr};
  launch_nt<EPI_DGLU>(p, kind, dt, s);
}

}  // namespace ema
