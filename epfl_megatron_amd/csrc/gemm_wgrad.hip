// Weight-gradient GEMM with fp32 accumulation for gfx950 (MI355X):
//
//     G[N, K] (+)= dY[M, N]^T · X[M, K]          dY, X bf16/fp16 row-major, G fp32
//
// The reference's fused_weight_gradient_dense (wgrad into main_grad, SURVEY N8;
// megatron/fused_kernels/fused_weight_gradient_dense.cu:129-152).  Both operands
// are "reduction-major" (the reduced token index m is the slow dimension): the
// NT case hipBLASLt serves at ~1.0 PF on MI355X whatever the solution
// (profiles/r1_lt_tune.json), 2/3 of its TN rate.  On gfx950 the layout costs
// nothing: ds_read_b64_tr_b16 turns a token-major LDS tile into MFMA operands.
//
// Structure (the 256x256 ping-pong template of the CDNA guide §5, adapted):
//   * 256 (n) x 256 (k) output tile per workgroup, 8 waves as 2 (n) x 4 (k),
//     each wave 128 x 64 = 8 x 4 tiles of v_mfma_f32_16x16x32 (128 fp32 acc;
//     16x16x32 holds a higher clock under load than 32x32x16, MICROARCH (7)).
//   * Tokens are consumed in subtiles of 32 rows (one MFMA k-step).  Both
//     operand slices [32 m][256] go HBM -> LDS by global_load_lds_dwordx4 into
//     a ring of 4 subtiles (4 x 32 KiB); the loads of subtile p+3 are issued in
//     phase p and retired by a COUNTED vmcnt, so ~3 phases (~1.3 us) of
//     latency are hidden and no vmcnt(0) appears in the loop.
//   * LDS image (a) of guide T10 ([32][256] as 8-row x 32-col 512-B subtiles,
//     2-bit XOR inside each 64-B row piece), written lane-linearly by the DMA
//     (the swizzle is applied through the per-lane SOURCE address).  Every
//     transposed fragment read is conflict-free, and the fragments of a wave
//     differ by instruction immediates: 4 base VGPRs per operand.
//   * Ping-pong: waves 4..7 run one barrier behind waves 0..3 (two barriers
//     per phase), so on every SIMD one wave's 32 MFMAs (s_setprio 1) overlap
//     the other wave's fragment reads.  The 4 DMA pieces of subtile p+3 are
//     split between the two sections: dY's two and X's first in the load
//     section after the fragment reads, X's second inside the MFMA section.
//     Each glds costs ~60 issue cycles; the alternatives measured in round 2
//     (and removed since): all four in the load section made it the critical
//     path (fc1 1.09-1.16 PF), all four in the MFMA section stall the MFMA
//     pipe (1.25-1.32 PF), one per alternate MFMA row likewise; splits of 1 / 2
//     / 3 pieces in the load section: 1.31-1.44 / 1.34-1.47 / 1.37-1.48 PF on
//     fc1 / qkv / fc2 (profiles/r2f_wgrad_sched.txt, r2g_wgrad_sched.txt); a
//     non-ping-pong schedule with the reads between the MFMAs: 1.06-1.08 PF.
//   * Epilogue: fp32 read-modify-write of G (beta = 1) or plain store (beta =
//     0: the first micro-batch of a step; main_grad is never zero-filled),
//     transposed through LDS so G moves in 16-B row pieces (+1.5 % on fc1
//     over per-lane 4-B accesses).
//   * XCD-aware tile order: each XCD's consecutive tiles form 8 x 4 blocks
//     (4 or 8 tiles of the shorter output dimension) so concurrently running
//     workgroups share operand panels in L2.
//
//   * Split-K over tokens where whole tiles leave CUs idle (fewer tiles than
//     CUs, or a partial last round of tiles: wgrad_plan): fp32 partials per
//     split, then an ordered reduce into G — deterministic, unlike atomics.
//
// Shapes: N % 8 == 0, K % 8 == 0, M % 32 == 0 (checked by the host); a
// ragged last tile row / column (e.g. the TP=8 shards of Llama-2-7B's FFN,
// 2752 and 1376) clamps its loads and masks its stores.
#include <cstdlib>
#include <stdexcept>

#include "fa_common.h"
#include "gemm_plan.h"

namespace ema {
namespace {

using fa::static_for;

typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int TN = 256;               // output rows (n) per tile
constexpr int TK = 256;               // output cols (k) per tile
constexpr int BM = 32;                // tokens per subtile = one MFMA k-step
constexpr int OPB = BM * TN * 2;      // 16 KiB per operand subtile
constexpr int SLOTB = 2 * OPB;        // dY + X
constexpr int NSLOT = 4;              // ring depth (3 subtiles ahead)
constexpr int LDSB = NSLOT * SLOTB;   // 128 KiB
constexpr int LOADS = 4;              // glds instructions per wave per subtile
constexpr int FA_ = 8, FB_ = 4;       // A (n) and B (k) fragments per wave

// Image (a): byte offset of 16-B chunk `ch` (0..31) of row `row` (0..31).
__device__ __forceinline__ int img_off(int row, int ch) {
  return 4096 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

// Stage the [32 m][256] slice of a row-major [M][ld] matrix (cols c0..c0+255,
// rows m0..m0+31) at LDS byte offset `dst`: 16 pieces of 1 KiB, 2 per wave.
template <typename T, int I0 = 0, int I1 = 2>
__device__ __forceinline__ void stage_op(const T* __restrict__ src, int64_t ld, int64_t m0,
                                         int64_t c0, char* lds, int dst, int wave, int lane) {
  // ld is also the column count: chunks past a ragged last tile's edge re-read
  // the last chunk of the row (their output rows / columns are never stored)
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const int piece = wave * 2 + i;
    const int o = piece * 1024 + lane * 16;  // LDS byte this lane's 16 B land on
    const int rem = o & 4095;
    const int row = 8 * (o >> 12) + ((rem >> 6) & 7);
    const int ch = 4 * (rem >> 9) + (((rem >> 4) & 3) ^ ((row >> 2) & 3));
    int64_t col = c0 + ch * 8;
    col = col < ld ? col : ld - 8;
    const T* g = src + (m0 + row) * ld + col;
    __builtin_amdgcn_global_load_lds(
        (const void*)g, (__attribute__((address_space(3))) void*)(lds + dst + piece * 1024), 16, 0,
        0);
  }
}

// Lane's transposed-read address for the 16-column fragment whose first
// column has (c0 / 16) parity `par` inside a 32-column group, token rows
// 8g + 4u + q (g = lane >> 4): the fragment at column cb + 16 f reads at
// base(par = f & 1, u) + 512 * (f >> 1) (+ the 32-col group of cb).
__device__ __forceinline__ uint32_t frag_base(int cb, int par, int u, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int row = 8 * g + 4 * u + q;
  const int ch = (cb >> 3) + 2 * par + (p >> 1);
  return (uint32_t)(img_off(row, ch) + 8 * (p & 1));
}

// Wait until at most `n` subtiles' DMA of this wave are outstanding
// (wave-uniform; vmcnt takes an immediate).
__device__ __forceinline__ void wait_subtiles(int n) {
  static_assert(LOADS == 4, "vmcnt immediates assume 4 glds per subtile");
  if (n >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Grouped tile order: lin -> (tn, tk) as (x, y).  gn > 0: groups of gn n-tiles
// x all k-tiles, n fastest; gn < 0: groups of -gn k-tiles x all n-tiles, k
// fastest.  Returned by value (out-references were lowered through scratch).
__device__ __forceinline__ int2 tile_of(int lin, int ntn, int ntk, int gn) {
  const bool byn = gn > 0;
  const int g = byn ? gn : -gn;
  const int nlong = byn ? ntk : ntn, nshort = byn ? ntn : ntk;
  const int grp = lin / (g * nlong);
  const int first = grp * g;
  const int gsize = min(g, nshort - first);
  const int in_grp = lin - grp * g * nlong;
  const int a = first + in_grp % gsize, b = in_grp / gsize;
  return byn ? int2{a, b} : int2{b, a};
}

template <typename T>
__device__ __forceinline__ f32x4 mfma16(typename fa::MT<T>::x8 a, typename fa::MT<T>::x8 b,
                                        f32x4 c) {
  if constexpr (__is_same(T, bf16)) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// physical X row of logical token q (TokMap in kernels.h)
__device__ __forceinline__ int64_t tok_row(int64_t q, const TokMap& m) {
  if (m.rows == 0) return q;
  const int64_t grp = q / m.rows;
  return (grp % m.n1) * m.s1 + (grp / m.n1) * m.s2 + (q - grp * m.rows);
}

template <typename T, bool ACCUM>
__global__ void __launch_bounds__(512, 1)
wgrad_k(const T* __restrict__ dy, const T* __restrict__ x, float* __restrict__ g, int M, int N,
        int K, int gn, int msplit, float* __restrict__ ws, int lin0, int nlin, TokMap xm) {
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave >> 2, wk = wave & 3;  // wn is also the ping-pong group

  // tile order: XCD-contiguous, then 8 (n) x 4 (k) groups
  const int ntn = (N + TN - 1) / TN, ntk = (K + TK - 1) / TK;
  const int Nfull = N, Kfull = K;
  // This launch covers tiles [lin0, lin0 + nlin) of the grouped tile order.
  // Split-K over tokens (ws != nullptr): workgroup b takes tile b % nlin of
  // token split b / nlin and stores its fp32 partial as a dense 256 x 256
  // block ws[split][tile] (ACCUM is false); wgrad_split_reduce_k adds the
  // splits in order (deterministic)
  const int split = (int)blockIdx.x / nlin;
  const int lin = lin0 + xcd_remap((int)blockIdx.x - split * nlin, nlin);
  const int2 tt = tile_of(lin, ntn, ntk, gn);
  const int tn = tt.x, tk = tt.y;
  int64_t n0 = (int64_t)tn * TN, k0 = (int64_t)tk * TK;
  int ldg = K;  // row stride of the output
  int64_t xq0 = 0;  // logical token of this workgroup's first X row (split-K offset)
  if (ws) {
    const int m0s = split * msplit;
    M = min(msplit, M - m0s);
    dy += (int64_t)m0s * N;
    xq0 = m0s;
    g = ws + ((int64_t)split * nlin + (lin - lin0)) * (TN * TK);
    ldg = TK;
  }
  // operand panels: rows n0.. of dY^T, k0.. of X^T; output block origin (on, ok)
  const int64_t on = ws ? 0 : n0, ok = ws ? 0 : k0;

  f32x4 acc[FA_][FB_];
#pragma unroll
  for (int i = 0; i < FA_; ++i)
#pragma unroll
    for (int j = 0; j < FB_; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // 4 bases per operand: [parity][u]; B lives OPB after A in a slot
  uint32_t abase[2][2], bbase[2][2];
#pragma unroll
  for (int par = 0; par < 2; ++par)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      abase[par][u] = frag_base(wn * 128, par, u, lane);
      bbase[par][u] = OPB + frag_base(wk * 64, par, u, lane);
    }
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;

  // X rows of subtile t: 32 consecutive physical rows from tok_row(first)
  auto xrow = [&](int t) { return tok_row(xq0 + (int64_t)t * BM, xm); };
  auto stage = [&](int t) {  // slot t % NSLOT <- tokens [t*BM, t*BM + BM)
    const int dst = (t % NSLOT) * SLOTB;
    stage_op<T>(dy, N, (int64_t)t * BM, n0, lds, dst, wave, lane);
    stage_op<T>(x, K, xrow(t), k0, lds, dst + OPB, wave, lane);
  };

  const int nt = M / BM;
  // Each glds costs ~60 issue cycles: 3 of a subtile's 4 DMA pieces (dY 0,
  // dY 1, X 0) issue in the load section, X's second inside the MFMA section
  // after MFMA row 3 (all four in the load section made it the critical path,
  // 1.09-1.16 PF on fc1; all four among the MFMAs stalled the pipe, 1.25-1.32;
  // 3 + 1: 1.37-1.48 PF, profiles/r2f_wgrad_sched.txt, r2g_wgrad_sched.txt)
  constexpr int SPLITL = 3, MROW = 3;
  auto stage_piece = [&](int q, int ts) {
    const int dst = (ts % NSLOT) * SLOTB;
    if (q == 0) stage_op<T, 0, 1>(dy, N, (int64_t)ts * BM, n0, lds, dst, wave, lane);
    else if (q == 1) stage_op<T, 1, 2>(dy, N, (int64_t)ts * BM, n0, lds, dst, wave, lane);
    else if (q == 2) stage_op<T, 0, 1>(x, K, xrow(ts), k0, lds, dst + OPB, wave, lane);
    else stage_op<T, 1, 2>(x, K, xrow(ts), k0, lds, dst + OPB, wave, lane);
  };
  typename fa::MT<T>::x4 fa_[FA_][2], fb_[FB_][2];
  auto reads = [&](int t) {  // all fragments of subtile t (24 transposed reads)
    const uint32_t so = lds_base + (uint32_t)((t % NSLOT) * SLOTB);
    uint32_t a[2][2], b[2][2];
#pragma unroll
    for (int par = 0; par < 2; ++par)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        a[par][u] = so + abase[par][u];
        b[par][u] = so + bbase[par][u];
      }
    static_for<FA_>([&](auto f) {
      constexpr int F = decltype(f)::value;
      fa_[F][0] = fa::tr_read_imm<512 * (F >> 1), T>(a[F & 1][0]);
      fa_[F][1] = fa::tr_read_imm<512 * (F >> 1), T>(a[F & 1][1]);
    });
    static_for<FB_>([&](auto f) {
      constexpr int F = decltype(f)::value;
      fb_[F][0] = fa::tr_read_imm<512 * (F >> 1), T>(b[F & 1][0]);
      fb_[F][1] = fa::tr_read_imm<512 * (F >> 1), T>(b[F & 1][1]);
    });
  };
  auto mfmas = [&](int t) {
    typename fa::MT<T>::x8 av[FA_], bv[FB_];
#pragma unroll
    for (int i = 0; i < FA_; ++i) av[i] = fa::join<T>(fa_[i][0], fa_[i][1]);
#pragma unroll
    for (int j = 0; j < FB_; ++j) bv[j] = fa::join<T>(fb_[j][0], fb_[j][1]);
    __builtin_amdgcn_s_setprio(1);
    static_for<FA_>([&](auto i) {
      constexpr int I = decltype(i)::value;
#pragma unroll
      for (int j = 0; j < FB_; ++j) acc[I][j] = mfma16<T>(av[I], bv[j], acc[I][j]);
      if constexpr (I == MROW) {  // X's second DMA piece of subtile t+3 rides here
        const int ts = t + NSLOT - 1;
        if (ts < nt) {
          __builtin_amdgcn_sched_barrier(0);
          static_for<4 - SPLITL>([&](auto q) { stage_piece(SPLITL + decltype(q)::value, ts); });
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    });
    __builtin_amdgcn_s_setprio(0);
  };

#pragma unroll
  for (int t = 0; t < NSLOT - 1; ++t)
    if (t < nt) stage(t);
  wait_subtiles(min(nt, NSLOT - 1) - 1);  // subtile 0 landed (own DMA)
  __builtin_amdgcn_s_barrier();            // ... and everyone's
  if (wn == 1) __builtin_amdgcn_s_barrier();  // group 1 runs one barrier behind

  // Phase p: [reads p][3 DMA pieces of p+3][vmcnt: p+1 landed][lgkmcnt(0)] BAR_A
  //          [32 MFMA + the 4th DMA piece of p+3] BAR_B
  // Group 0's BAR_A(p) is barrier 2p+1, group 1's is 2p+2 (= group 0's
  // BAR_B(p)): each group's MFMA section overlaps the other's load section.
  // RAW: subtile p+1 is retired by every wave before its BAR_A(p); both
  //      groups read it only after a later barrier.
  // WAR: stage(p+3) overwrites subtile p-1, whose reads every wave retired
  //      (lgkmcnt(0)) before its BAR_A(p-1), a barrier both groups passed.
  for (int t = 0; t < nt; ++t) {
    reads(t);
    if (t + NSLOT - 1 < nt) {
      // the first SPLITL DMA pieces of subtile t+3 here (behind subtile t+2's 4)
      static_for<SPLITL>([&](auto q) { stage_piece(decltype(q)::value, t + NSLOT - 1); });
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(4 + SPLITL) : "memory");
    } else {
      wait_subtiles(min(t + NSLOT - 2, nt - 1) - (t + 1));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    mfmas(t);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
  if (wn == 0) __builtin_amdgcn_s_barrier();  // balance the barrier count

  // Through LDS (free now: every ring read was retired before the last
  // barrier, no DMA is in flight): each wave transposes its 128 x 64 fp32
  // tile in two 64-row halves through a private 16 KiB region, so G moves
  // as 16-B row pieces (256 B contiguous per 16 lanes) instead of 4-B
  // pieces (64 B per 16 lanes).  Region layout: row-major [64][64] fp32
  // with the 16-column group XOR-ed by (row >> 2) & 3 (conflict-free
  // ds_write_b32 of the accumulator layout and ds_read_b128 of rows).
  float* reg = reinterpret_cast<float*>(lds) + wave * 4096;
  const int gq = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FB_; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int lr = 16 * i + 4 * gq + r;  // (lr >> 2) & 3 == gq
          reg[lr * 64 + ((16 * j) ^ (16 * gq)) + cl] = acc[4 * h + i][j][r];
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    f32x4 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int lr = gq + 4 * k, c = 4 * cl;
      v[k] = *reinterpret_cast<const f32x4*>(reg + lr * 64 + (c ^ (16 * ((lr >> 2) & 3))));
    }
    float* gb = g + (on + wn * 128 + 64 * h + gq) * (int64_t)ldg + ok + wk * 64 + 4 * cl;
    // ragged edge (direct stores only; split partials are dense blocks):
    // rows n >= N and 4-float column pieces k >= K are not stored
    const int64_t nrow0 = n0 + wn * 128 + 64 * h + gq;
    const bool full = ws || (n0 + TN <= Nfull && k0 + TK <= Kfull);
    const bool kok = ws || k0 + wk * 64 + 4 * cl < Kfull;
    if (full) {
      if (ACCUM) {
        f32x4 o[16];
#pragma unroll
        for (int k = 0; k < 16; ++k)
          o[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(gb + (int64_t)(4 * k) * ldg));
#pragma unroll
        for (int k = 0; k < 16; ++k)
          __builtin_nontemporal_store(o[k] + v[k], reinterpret_cast<f32x4*>(gb + (int64_t)(4 * k) * ldg));
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k)
          __builtin_nontemporal_store(v[k], reinterpret_cast<f32x4*>(gb + (int64_t)(4 * k) * ldg));
      }
    } else if (kok) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (nrow0 + 4 * k < Nfull) {
          f32x4* q = reinterpret_cast<f32x4*>(gb + (int64_t)(4 * k) * ldg);
          __builtin_nontemporal_store(ACCUM ? __builtin_nontemporal_load(q) + v[k] : v[k], q);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // region reads done before reuse
  }
}

// ---- persistent 4-wave wgrad (the gemm_nt.hip variant-6 structure) ---------
// 256 (n) x 256 (k) tile, 4 waves as 2 x 2, each 128 x 128 = 8 x 8 MFMA
// 16x16x32 accumulators (AGPR-pinned asm MFMAs).  Tokens are consumed 64 per
// K-step: per operand two [32 tok][256] images (a) (one per MFMA k-half) in a
// 64-KiB slot, 2 slots.  Each K-step runs the early-refill schedule of
// gemm_nt6_k (A half refilled after BARRIER 1, B half after BARRIER 2, the
// next step awaited three quarters in), the K-steps of consecutive tiles form
// one stream (the next tile's first two steps load during the current tile's
// last two), and the epilogue adds the accumulators to G straight from
// registers: the MFMA takes (X fragment, dY fragment) so each lane holds 4
// consecutive k of one n row, a 16-B fp32 read-modify-write.
// DMA: buffer_load ... lds; the per-tile descriptor starts at the tile's first
// column and ends at the end of the operand, so a piece is one per-lane VGPR
// (wave parity variant) plus an SGPR offset (token row block + 128-B column
// block), and the last rows of a ragged edge read zeros past the buffer end.
typedef __attribute__((ext_vector_type(4))) float f32x4_;
typedef __amdgpu_buffer_rsrc_t Rsrc;
constexpr int IMG = 32 * 256 * 2;        // one [32][256] 16-bit image (a)
constexpr int OPB2 = 2 * IMG;            // operand per K-step (64 tokens)
constexpr int SLOTB2 = 2 * OPB2;         // dY + X

template <typename T>
__device__ __forceinline__ void wmfma(f32x4_& acc, typename fa::MT<T>::x8 a, typename fa::MT<T>::x8 b) {
  if constexpr (__is_same(T, bf16))
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
template <typename T>
__device__ __forceinline__ void wmfma0(f32x4_& acc, typename fa::MT<T>::x8 a, typename fa::MT<T>::x8 b) {
  if constexpr (__is_same(T, bf16))
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

// Arguments of the persistent 4-wave kernel.  Items: whole tiles [0, nitems)
// over all M tokens, or (SPLIT) token pieces of the tiles [lin0, lin0 + nlin):
// item it = piece (it / nlin) of tile lin0 + it % nlin, msplit tokens each,
// stored as an fp32 block ws[it] for wgrad_split_reduce_k (the 8-wave
// kernel's split-major layout).  TM: X rows through the token map xm (xrows:
// the physical X rows it reaches).
struct W4Args {
  const void* dy;
  const void* x;
  float* g;
  float* ws;
  int M, N, K, msplit, gn, nitems, lin0, nlin, xrows;
  TokMap xm;
};

// 32-bit form of tok_row (the host bounds xrows * K * 2 below 2^31)
__device__ __forceinline__ int tok_row32(int q, const TokMap& m) {
  const int grp = (int)((unsigned)q / (unsigned)m.rows);
  const int n1 = m.n1;
  return (grp % n1) * (int)m.s1 + (grp / n1) * (int)m.s2 + (q - grp * m.rows);
}

template <typename T, bool ACCUM, bool TM, bool SPLIT>
__global__ void __launch_bounds__(256, 1) wgrad4_k(W4Args a) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * SLOTB2];
  typedef typename fa::MT<T>::x8 X8;
  typedef typename fa::MT<T>::x4 X4;
  const T* __restrict__ dy = (const T*)a.dy;
  const T* __restrict__ x = (const T*)a.x;
  const int M = a.M, N = a.N, K = a.K, gn = a.gn, ntiles = a.nitems;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave >> 1, wk = wave & 1;
  const int G = gridDim.x, bid = blockIdx.x;
  if (bid >= ntiles) return;
  const int nmine = (ntiles - 1 - bid) / G + 1;
  const int ntn = (N + TN - 1) / TN, ntk = (K + TK - 1) / TK;
  const int nt = (SPLIT ? a.msplit : M) / 64;  // >= 2 (host-checked)

  // per-lane DMA offset of a piece (rows 8 wave .. of an image, 512 B per row)
  auto lane_off = [&](int ld) {
    const int row = (lane >> 2) & 7;
    const int ch = 4 * (lane >> 5) + ((lane & 3) ^ ((2 * wave + ((lane >> 4) & 1)) & 3));
    return (uint32_t)(row * ld * (int)sizeof(T) + 16 * ch);
  };
  const uint32_t voff_a = lane_off(N), voff_b = lane_off(K);
  const uint32_t srow_a = (uint32_t)(8 * wave * N * (int)sizeof(T));
  const uint32_t srow_b = (uint32_t)(8 * wave * K * (int)sizeof(T));

  // item i of this workgroup: output tile origin, first token, ws block
  auto tile_org = [&](int i, int64_t& n0, int64_t& k0, int& t0, int& blk) {
    const int base = i * G, rem = min(G, ntiles - base);
    const int it = base + xcd_remap(bid, rem);
    const int sp = SPLIT ? it / a.nlin : 0;
    const int lin = SPLIT ? a.lin0 + (it - sp * a.nlin) : it;
    const int2 tt = tile_of(lin, ntn, ntk, gn);
    n0 = (int64_t)tt.x * TN;
    k0 = (int64_t)tt.y * TK;
    t0 = sp * a.msplit;
    blk = it;
  };
  // buffer descriptors of item i (q0: its first logical token, for TM)
  auto make_rsrc = [&](int i, Rsrc& ra, Rsrc& rb, int& q0) {
    int64_t n0 = 0, k0 = 0, na = 0, nb = 0, oa = 0, ob = 0;
    int t0 = 0, blk = 0;
    if (i < nmine) {
      tile_org(i, n0, k0, t0, blk);
      oa = (int64_t)t0 * N + n0;
      ob = TM ? k0 : (int64_t)t0 * K + k0;
      na = ((int64_t)M * N - oa) * (int64_t)sizeof(T);
      nb = ((int64_t)(TM ? a.xrows : M) * K - ob) * (int64_t)sizeof(T);
    }
    q0 = t0;
    ra = __builtin_amdgcn_make_buffer_rsrc((void*)(dy + oa), 0, (int)na, 0x00020000);
    rb = __builtin_amdgcn_make_buffer_rsrc((void*)(x + ob), 0, (int)nb, 0x00020000);
  };
  char* const ldsp = lds;
  // piece i (0..3) of image kh of operand op, K-step s, into slot
  // (xr: TM's byte offsets of the step's two physical X row blocks)
  auto dma = [&](int op, int kh, int i, Rsrc r, int s, int slot, const uint32_t (&xr)[2]) {
    const int ld = op ? K : N;
    const uint32_t rows = (TM && op) ? xr[kh] : (uint32_t)((s * 64 + 32 * kh) * ld * (int)sizeof(T));
    const uint32_t soff = rows + (op ? srow_b : srow_a) + 128u * (uint32_t)i;
    const int dst = slot * SLOTB2 + op * OPB2 + kh * IMG + (4 * wave + i) * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(ldsp + dst),
                                             16, op ? voff_b : voff_a, soff, 0, 0);
  };
  // DMA piece q (0..7 dY, 8..15 X) of a K-step
  auto dmaq = [&](int q, Rsrc ra, Rsrc rb, int s, int slot, const uint32_t (&xr)[2]) {
    const int op = q >> 3, kh = (q >> 2) & 1, i = q & 3;
    dma(op, kh, i, op ? rb : ra, s, slot, xr);
  };
  auto xrows_of = [&](int q0, int s, uint32_t (&xr)[2]) {
    if constexpr (TM) {
      xr[0] = (uint32_t)tok_row32(q0 + 64 * s, a.xm) * (uint32_t)(K * (int)sizeof(T));
      xr[1] = (uint32_t)tok_row32(q0 + 64 * s + 32, a.xm) * (uint32_t)(K * (int)sizeof(T));
    } else {
      xr[0] = xr[1] = 0;
    }
  };

  f32x4_ acc[8][8];
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  uint32_t abase[2][2], bbase[2][2];
#pragma unroll
  for (int par = 0; par < 2; ++par)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      abase[par][u] = lds_base + frag_base(128 * wn, par, u, lane);
      bbase[par][u] = lds_base + OPB2 + frag_base(128 * wk, par, u, lane);
    }
  X8 set0[16], set1[16];  // [0..7] dY (n) fragments, [8..15] X (k) fragments
  auto read_frag = [&](X8 (&dst)[16], auto f, auto kh, uint32_t so) {
    constexpr int F = decltype(f)::value, KH = decltype(kh)::value;
    constexpr int FF = F & 7, OFF = KH * IMG + 512 * (FF >> 1);
    const uint32_t b0 = (F < 8 ? abase[FF & 1][0] : bbase[FF & 1][0]) + so;
    const uint32_t b1 = (F < 8 ? abase[FF & 1][1] : bbase[FF & 1][1]) + so;
    const X4 lo = fa::tr_read_imm<OFF, T>(b0), hi = fa::tr_read_imm<OFF, T>(b1);
    dst[F] = fa::join<T>(lo, hi);
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;

  Rsrc ra_c, rb_c, ra_n, rb_n;
  int q_c, q_n;
  make_rsrc(0, ra_c, rb_c, q_c);
  make_rsrc(1, ra_n, rb_n, q_n);
  {
    uint32_t xr0[2], xr1[2];
    xrows_of(q_c, 0, xr0);
    xrows_of(q_c, 1, xr1);
    static_for<16>([&](auto q) { dmaq(decltype(q)::value, ra_c, rb_c, 0, 0, xr0); });
    static_for<16>([&](auto q) { dmaq(decltype(q)::value, ra_c, rb_c, 1, 1, xr1); });
  }
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  static_for<16>([&](auto f) { read_frag(set0, f, K0{}, 0u); });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  int par = 0;
  for (int i = 0; i < nmine; ++i) {
    auto kstep = [&](int t, auto zero) {
      const int slot = (t + par) & 1;
      const uint32_t so = (uint32_t)(slot * SLOTB2), sn = (uint32_t)(SLOTB2 - so);
      const bool here = t + 2 < nt;
      const Rsrc ra = here ? ra_c : ra_n, rb = here ? rb_c : rb_n;
      const int s2 = here ? t + 2 : t + 2 - nt;
      uint32_t xr[2];
      xrows_of(here ? q_c : q_n, s2, xr);
      // the shared slot plan (gemm_plan.h) with A = dY, B = X: dY's pieces of
      // step t+2 after barrier 1, X's after barrier 2, 13 before the wait
      constexpr int VMW = nt_plan_vmw();
      static_for<128>([&](auto sc) {
        constexpr int S = decltype(sc)::value, IDX = S & 63, I = IDX / 8, J = IDX % 8;
        if constexpr (S < 64) {
          if constexpr (decltype(zero)::value) wmfma0<T>(acc[I][J], set0[8 + J], set0[I]);
          else wmfma<T>(acc[I][J], set0[8 + J], set0[I]);
        } else {
          wmfma<T>(acc[I][J], set1[8 + J], set1[I]);
        }
        static_for<16>([&](auto ec) {
          constexpr int E = decltype(ec)::value;
          if constexpr (kNtPlan.rd1[E] == S) read_frag(set1, std::integral_constant<int, E>{}, K1{}, so);
          if constexpr (kNtPlan.dma[E] == S) dmaq(E, ra, rb, s2, slot, xr);
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

    // epilogue: G[n][k .. k+3] (+)= acc, straight from registers (SPLIT: the
    // item's fp32 block, ragged rows / columns included: the reduce skips them)
    fa::mfma_drain();
    int64_t n0, k0;
    int t0, blk;
    tile_org(i, n0, k0, t0, blk);
    if constexpr (SPLIT) {
      float* wb = a.ws + (int64_t)blk * (TN * TK) + (128 * wn + (lane & 15)) * TK + 128 * wk +
                  4 * (lane >> 4);
#pragma unroll
      for (int ii = 0; ii < 8; ++ii)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          __builtin_nontemporal_store(acc[ii][j], reinterpret_cast<f32x4_*>(wb + 16 * ii * TK + 16 * j));
    } else {
      const int64_t kc = k0 + 128 * wk + 4 * (lane >> 4);
      const int64_t nr = n0 + 128 * wn + (lane & 15);
#pragma unroll
      for (int ii = 0; ii < 8; ++ii) {
        const int64_t n = nr + 16 * ii;
        f32x4_* row = reinterpret_cast<f32x4_*>(a.g + n * K + kc);
        if constexpr (ACCUM) {
#pragma unroll
          for (int jh = 0; jh < 8; jh += 4) {
            f32x4_ o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              o[j] = (n < N && kc + 16 * (jh + j) < K) ? __builtin_nontemporal_load(row + 4 * (jh + j))
                                                        : f32x4_{0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (n < N && kc + 16 * (jh + j) < K)
                __builtin_nontemporal_store(o[j] + acc[ii][jh + j], row + 4 * (jh + j));
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (n < N && kc + 16 * j < K) __builtin_nontemporal_store(acc[ii][j], row + 4 * j);
        }
      }
    }
    par ^= nt & 1;
    ra_c = ra_n;
    rb_c = rb_n;
    q_c = q_n;
    make_rsrc(i + 2, ra_n, rb_n, q_n);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Tile grouping: a few tiles of the SHORTER output dimension x all tiles of
// the longer one, so an XCD's 32 concurrent workgroups form an 8 x 4 block
// (measured on the 7B shapes, profiles/r2_wgrad_ab.txt: +3-5 % on qkv / fc1 /
// lm_head over grouping along n).  EMA_WGRAD_GN overrides (> 0: groups of gn
// n-tiles, < 0: groups of -gn k-tiles).
int tile_group(int ntn, int ntk) {
  static const int env = [] {
    const char* e = getenv("EMA_WGRAD_GN");
    return e ? atoi(e) : 0;
  }();
  if (env != 0) return env;
  return ntn >= ntk ? -4 : 8;
}

// gn: the tile order, shared by every launch of one wgrad_gemm (the main
// rounds and the split tail partition ONE order: both must use the same gn)
template <typename T, bool ACCUM>
void launch(const void* dy, const void* x, float* g, int M, int N, int K, hipStream_t s, int gn,
            int nsplit = 1, float* ws = nullptr, int lin0 = 0, int nlin = -1, TokMap xm = {}) {
  const int ntiles = ((N + TN - 1) / TN) * ((K + TK - 1) / TK);
  if (nlin < 0) nlin = ntiles;
  const int msplit = ((M / nsplit + BM - 1) / BM) * BM;
  hipLaunchKernelGGL((wgrad_k<T, ACCUM>), dim3(nlin * nsplit), dim3(512), 0, s,
                     (const T*)dy, (const T*)x, g, M, N, K, gn, msplit,
                     nsplit > 1 ? ws : nullptr, lin0, nlin, xm);
}

// G[tile] (+)= sum over the token splits of ws[split][tile] (fixed order) for
// tiles [lin0, lin0 + nlin); 64 workgroups x 256 threads x 4 floats per tile
__global__ __launch_bounds__(256) void wgrad_split_reduce_k(const float* __restrict__ ws,
                                                           float* __restrict__ g, int N, int K,
                                                           int gn, int lin0, int nlin, int nsplit,
                                                           int accumulate) {
  const int t = blockIdx.x / 64, part = blockIdx.x % 64;
  const int2 tt = tile_of(lin0 + t, (N + TN - 1) / TN, (K + TK - 1) / TK, gn);
  const int tn = tt.x, tk = tt.y;
  const int e = (part * 256 + threadIdx.x) * 4;  // element of the 256 x 256 block
  const int row = e / TK, col = e % TK;
  if ((int64_t)tn * TN + row >= N || (int64_t)tk * TK + col >= K) return;  // ragged edge
  float* gp = g + ((int64_t)tn * TN + row) * K + (int64_t)tk * TK + col;
  f32x4 acc = accumulate ? *reinterpret_cast<const f32x4*>(gp) : f32x4{0.f, 0.f, 0.f, 0.f};
  for (int sp = 0; sp < nsplit; ++sp)
    acc += __builtin_nontemporal_load(
        reinterpret_cast<const f32x4*>(ws + ((int64_t)sp * nlin + t) * (TN * TK) + e));
  *reinterpret_cast<f32x4*>(gp) = acc;
}

}  // namespace

bool wgrad_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N >= 8 && K >= 8 && M % BM == 0 && N % 8 == 0 && K % 8 == 0 &&
         M <= (int64_t)1 << 30 && ((N + TN - 1) / TN) * ((K + TK - 1) / TK) < (int64_t)1 << 31 &&
         N * K < ((int64_t)1 << 40);
}

// Split planning (wgrad_plan).  One workgroup owns a 256 x 256 output tile,
// so a grid that is not a multiple of the CUs ends in a partial round, and a
// grid of fewer tiles than CUs (TP-sharded projections) leaves CUs idle.  The
// tiles of the partial round (all tiles when there are fewer than CUs) are
// split over the tokens s ways, s picked by a cost model: rounds of tile
// pieces, ceil(t s / CUs) / s tile-times, plus the fp32 partials' round trip
// (t s blocks of 256 KB written and read back by the ordered reduce, ~5 TB/s)
// and ~5 us of ring fill / epilogue per round; a split must win by 5 %.
// At least 2048 tokens per split, at most 4 x CUs pieces (workspace bound).
// E.g. the 7B TP8 shards: qkv / fc2 (96 tiles) 2 ways (was 3: 288 pieces =
// two rounds), fc1 (176 tiles) unsplit (was 2: 352 pieces, two rounds of
// half tiles plus the partials' traffic), dense (32 tiles) 8 ways.
namespace {
int best_split(int t, int64_t M, int ncu) {
  if (t <= 0) return 1;
  const double tile_us = 2.0 * TN * TK * (double)M / (1.3e15 / ncu) * 1e6;
  // per round: the pieces' compute + ~5 us of ring fill / epilogue
  // a split must beat the whole tiles clearly (reduce launch, partial traffic);
  // among the splits the cheapest wins.  Pieces of whole 64-token steps only
  // (the 4-wave kernel's split form) when M allows them.
  const double whole = ((t + ncu - 1) / ncu) * (tile_us + 5.0);
  int best = 1;
  double best_c = whole * 0.95;
  for (int sp = 2; sp <= 16; ++sp) {
    if (M / sp < 2048 || t * sp > 4 * ncu) break;
    if (M % 64 == 0 && M % (64 * sp) != 0) continue;
    const int rounds = (t * sp + ncu - 1) / ncu;
    const double c = rounds * (tile_us / sp + 5.0) +
                     (double)t * sp * TN * TK * 4.0 * 2.0 / 5e12 * 1e6 + 3.0;
    if (c < best_c) {
      best_c = c;
      best = sp;
    }
  }
  return best;
}
}  // namespace

WgradPlan wgrad_plan(int64_t M, int64_t N, int64_t K) {
  const int tiles = (int)(((N + TN - 1) / TN) * ((K + TK - 1) / TK));
  const int ncu = 256;  // the plan must not depend on the device queried (host tests)
  static const bool tail_split = [] {  // EMA_WGRAD_TAIL=0: no split (A/B)
    const char* e = getenv("EMA_WGRAD_TAIL");
    return !(e && e[0] == '0');
  }();
  WgradPlan pl{tiles, tiles, 0, 1};
  if (!tail_split) return pl;
  const int tail = tiles < ncu ? tiles : tiles % ncu;
  const int sp = best_split(tail, M, ncu);
  if (sp > 1) pl = WgradPlan{tiles - tail, tiles - tail, tail, sp};
  return pl;
}

int64_t wgrad_workspace_floats(int64_t M, int64_t N, int64_t K) {
  const WgradPlan pl = wgrad_plan(M, N, K);
  return pl.nsplit > 1 ? (int64_t)pl.nsplit * pl.tail_tiles * TN * TK : 0;
}

// Kernel for the whole-tile rounds: 4 = the persistent 4-wave wgrad4_k
// (default since round 6), 8 = the 8-wave ping-pong wgrad_k (EMA_WGRAD_V=8 /
// wgrad_set_variant: A/B).  Round 4 measured the 4-wave kernel at 0.83-0.95x
// (profiles/r4a_wgrad_variants.txt); with the vendor slot plan it shares with
// gemm_nt6_k since round 5 it is 1.02-1.07x isolated and +1.6 % on the
// headline step (profiles/r7r_wgrad_v4_ab.txt).  It also runs token-mapped X
// (the kept SP gathers) and the split tails whose pieces are whole 64-token
// steps; M % 64 != 0 and > 2 GiB operands stay on wgrad_k.
int g_wvar = [] {
  const char* e = getenv("EMA_WGRAD_V");
  return (e && e[0] == '8') ? 8 : 4;
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

// xrows: the physical X rows (a token map may reach past M)
bool wgrad4_ok(int64_t M, int64_t N, int64_t K, int64_t xrows) {
  const int64_t lim = (int64_t)1 << 31;
  return g_wvar == 4 && M % 64 == 0 && M >= 128 && M * N * 2 < lim && xrows * K * 2 < lim;
}

// Tile grouping of the persistent kernel: groups of 8 n-tiles x all k-tiles on
// every 7B shape (sweep on one box, profiles/r7t_wgrad4_group_sweep.txt: qkv
// +3.2 %, fc1 +4.1 %, lm_head +2.6 % over the 8-wave kernel's rule, dense /
// fc2 within noise); EMA_WGRAD_GN overrides both kernels.
int tile_group4() {
  static const int env = [] {
    const char* e = getenv("EMA_WGRAD_GN");
    return e ? atoi(e) : 0;
  }();
  return env != 0 ? env : 8;
}

template <typename T, bool ACCUM, bool TM, bool SPLIT>
void launch4(const W4Args& a, hipStream_t s) {
  const int grid = a.nitems < num_cus() ? a.nitems : num_cus();
  hipLaunchKernelGGL((wgrad4_k<T, ACCUM, TM, SPLIT>), dim3(grid), dim3(256), 0, s, a);
}

template <typename T>
void launch4_dt(const W4Args& a, bool accumulate, bool split, hipStream_t s) {
  const bool tm = a.xm.rows != 0;
  if (split) {
    if (tm) launch4<T, false, true, true>(a, s);
    else launch4<T, false, false, true>(a, s);
  } else if (accumulate) {
    if (tm) launch4<T, true, true, false>(a, s);
    else launch4<T, true, false, false>(a, s);
  } else {
    if (tm) launch4<T, false, true, false>(a, s);
    else launch4<T, false, false, false>(a, s);
  }
}

void wgrad_gemm(const void* dy, const void* x, float* g, int64_t M, int64_t N, int64_t K,
                bool accumulate, int dt, hipStream_t s, float* ws, TokMap xm) {
  const int iM = (int)M, iN = (int)N, iK = (int)K;
  const WgradPlan pl = wgrad_plan(M, N, K);
  const bool split = pl.nsplit > 1 && ws != nullptr;
  const int main_tiles = split ? pl.main_tiles : pl.main_tiles + pl.tail_tiles;
  if (xm.rows != 0 && xm.rows % BM != 0) throw std::runtime_error("wgrad: token map groups must be 32-row multiples");
  // physical X rows the token map reaches (bindings.cpp checks them against x)
  const int64_t xrows = xm.rows == 0 ? M
                                     : (int64_t)(xm.n1 - 1) * xm.s1 +
                                           (M / ((int64_t)xm.rows * xm.n1) - 1) * xm.s2 + xm.rows;
  const bool v4 = wgrad4_ok(M, N, K, xrows);
  // the split tail runs on the 4-wave kernel when its pieces are whole 64-token steps
  // (EMA_WGRAD_TAIL4=0: the 8-wave kernel, for A/B)
  static const bool tail4 = [] {
    const char* e = getenv("EMA_WGRAD_TAIL4");
    return !(e && e[0] == '0');
  }();
  const bool v4_tail = v4 && tail4 && split && M % (64 * pl.nsplit) == 0 && M / pl.nsplit >= 128;
  const int gn = v4 ? tile_group4() : tile_group((iN + TN - 1) / TN, (iK + TK - 1) / TK);
  W4Args a{dy, x, g, ws, iM, iN, iK, iM, gn, main_tiles, 0, main_tiles, (int)xrows, xm};
  if (main_tiles > 0 && v4) {
    if (dt == DT_BF16) launch4_dt<bf16>(a, accumulate, false, s);
    else if (dt == DT_F16) launch4_dt<fp16>(a, accumulate, false, s);
  } else if (main_tiles > 0) {
    if (dt == DT_BF16) {
      if (accumulate) launch<bf16, true>(dy, x, g, iM, iN, iK, s, gn, 1, nullptr, 0, main_tiles, xm);
      else launch<bf16, false>(dy, x, g, iM, iN, iK, s, gn, 1, nullptr, 0, main_tiles, xm);
    } else if (dt == DT_F16) {
      if (accumulate) launch<fp16, true>(dy, x, g, iM, iN, iK, s, gn, 1, nullptr, 0, main_tiles, xm);
      else launch<fp16, false>(dy, x, g, iM, iN, iK, s, gn, 1, nullptr, 0, main_tiles, xm);
    }
  }
  if (split) {
    if (v4_tail) {
      a.msplit = iM / pl.nsplit;
      a.nitems = pl.tail_tiles * pl.nsplit;
      a.lin0 = pl.tail_lin0;
      a.nlin = pl.tail_tiles;
      if (dt == DT_BF16) launch4_dt<bf16>(a, false, true, s);
      else if (dt == DT_F16) launch4_dt<fp16>(a, false, true, s);
    } else if (dt == DT_BF16) {
      launch<bf16, false>(dy, x, g, iM, iN, iK, s, gn, pl.nsplit, ws, pl.tail_lin0, pl.tail_tiles, xm);
    } else if (dt == DT_F16) {
      launch<fp16, false>(dy, x, g, iM, iN, iK, s, gn, pl.nsplit, ws, pl.tail_lin0, pl.tail_tiles, xm);
    }
    hipLaunchKernelGGL(wgrad_split_reduce_k, dim3((unsigned)(pl.tail_tiles * 64)), dim3(256), 0, s,
                       ws, g, iN, iK, gn, pl.tail_lin0, pl.tail_tiles,
                       pl.nsplit, accumulate ? 1 : 0);
  }
}

void wgrad_set_variant(int v) { g_wvar = v == 8 ? 8 : 4; }

}  // namespace ema
