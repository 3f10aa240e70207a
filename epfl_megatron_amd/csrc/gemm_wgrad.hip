// Weight-gradient GEMM with fp32 accumulation for gfx950 (MI355X):
//
//     G[N, K] (+)= dY[M, N]^T · X[M, K]          dY, X bf16/fp16 row-major, G fp32
//
// This is the reference's fused_weight_gradient_dense (wgrad into main_grad,
// SURVEY N8).  Both operands are "reduction-major" (the reduced token index m
// is the slow dimension), the NT case that hipBLASLt serves at ~1000 TFLOP/s
// on MI355X across all of its solutions (profiles/r1_lt_tune.json).
//
// Design:
//   * 256 x 256 output tile per workgroup, 8 waves (2 along N x 4 along K),
//     each wave 128 x 64 = 4 x 2 tiles of v_mfma_f32_32x32x16 (128 fp32 acc).
//   * Tokens are consumed in slots of BM = 32 rows.  Both operand slices
//     [32 m][256] are staged HBM -> LDS with global_load_lds_dwordx4
//     (lane-linear LDS image, XOR-swizzled through the per-lane SOURCE
//     address) into a ring of 4 slots (4 x 32 KiB = 128 KiB LDS) with 3 slots
//     in flight: the loads of slot t+3 are issued while slot t is consumed and
//     completion is waited with a COUNTED vmcnt (never 0 in the steady state)
//     plus a raw s_barrier — so ~1.3 us of HBM/L2 latency is hidden instead
//     of the one-stage window of a 2-buffer loop (CDNA guide §5 "Pipelining
//     across barriers").
//   * MFMA operands come out of LDS with ds_read_b64_tr_b16 (inline asm, so
//     the compiler cannot drain the LDS-DMA stream in front of them): a 16-lane
//     group reads 4 token rows x 16 columns and receives it column-major —
//     exactly the "8 consecutive k per lane" fragment both MFMA operands need.
//     The swizzle chunk ^= (row & 3) << 2 makes every transposed read of a
//     32-lane half hit 16 distinct 16-byte slots (conflict-free).  Fragment
//     reads of k-step s+1 are issued before the MFMAs of k-step s (counted
//     lgkmcnt).
//   * Epilogue: batched read-modify-write of G in fp32 (beta = 1), or plain
//     store (beta = 0, first micro-batch: main_grad is never zero-filled).
//   * XCD-aware tile order: consecutive tiles of one XCD form 8 (N) x 4 (K)
//     groups so concurrently running workgroups share operand panels in L2.
//
// Shapes: N % 256 == 0, K % 256 == 0, M % 32 == 0 (checked by the host).
#include "fa_common.h"

namespace ema {
namespace {

using fa::MT;
using fa::f32x16;

constexpr int TN = 256;                 // output rows (N) per tile
constexpr int TK = 256;                 // output cols (K) per tile
constexpr int BM = 32;                  // tokens per ring slot
constexpr int ROWB = 512;               // bytes per LDS row (256 x 16-bit)
constexpr int OPB = BM * ROWB;          // 16 KiB per operand slice
constexpr int SLOTB = 2 * OPB;          // A + B
constexpr int NSLOT = 4;                // ring depth (NSLOT - 1 slots in flight)
constexpr int LDSB = NSLOT * SLOTB;     // 128 KiB
constexpr int LOADS = 4;                // glds instructions per wave per slot

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row & 3) << 2); }

// Stage one [32][256] slice of a row-major [M][ld] matrix (cols c0..c0+255,
// rows m0..m0+31) at LDS byte offset `dst`: 8 waves x 2 instructions, each
// instruction = 2 rows x 512 B, lane-linear in LDS.
template <typename T>
__device__ __forceinline__ void stage_op(const T* __restrict__ src, int64_t ld, int64_t m0,
                                         int64_t c0, char* lds, int dst, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int inst = wave * 2 + i;
    const int row = 2 * inst + (lane >> 5);
    const int chunk = swz_chunk(row, lane & 31);  // involution: source chunk for this lane
    const T* g = src + (m0 + row) * ld + c0 + chunk * 8;
    __builtin_amdgcn_global_load_lds(
        (const void*)g, (__attribute__((address_space(3))) void*)(lds + dst + inst * 1024), 16, 0,
        0);
  }
}

// ds_read_b64_tr_b16 as inline asm: invisible to the compiler's LDS-DMA alias
// tracking, so no vmcnt(0) is inserted in front of it.
__device__ __forceinline__ fa::bf16x4 tr_read_asm(uint32_t addr) {
  fa::bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

// Byte address (within a slice) of this lane's transposed read of token rows
// r0+q (q = 0..3 from the lane) for columns c0 + 16*g + 4*p.
__device__ __forceinline__ uint32_t tr_addr(int r0, int c0, int lane) {
  const int i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int col = c0 + ((lane >> 4) & 1) * 16 + 4 * p;
  const int r = r0 + q;
  return (uint32_t)(r * ROWB + swz_chunk(r, col >> 3) * 16 + ((col >> 2) & 1) * 8);
}

// Wait until at most `slots` slots' LDS-DMA loads of this wave are in flight
// (wave-uniform argument; vmcnt needs an immediate).
__device__ __forceinline__ void wait_slots(int slots) {
  static_assert(LOADS == 4, "vmcnt immediates below assume 4 loads per slot");
  if (slots >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (slots == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (slots == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename T, bool ACCUM, int MODE = 0>
__global__ void __launch_bounds__(512, 1)
wgrad_k(const T* __restrict__ dy, const T* __restrict__ x, float* __restrict__ g, int M, int N,
        int K) {
  __shared__ __attribute__((aligned(1024))) char lds[LDSB];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wn = wave >> 2, wk = wave & 3;
  const int h = lane >> 5;

  // tile order: XCD-contiguous, then 8 (N) x 4 (K) groups
  const int ntn = N / TN, ntk = K / TK, ntiles = ntn * ntk;
  const int lin = xcd_remap(blockIdx.x, ntiles);
  constexpr int GN = 8;
  const int grp = lin / (GN * ntk);
  const int first_n = grp * GN;
  const int gsize = min(GN, ntn - first_n);
  const int in_grp = lin - grp * GN * ntk;
  const int tn = first_n + in_grp % gsize;
  const int tk = in_grp / gsize;
  const int64_t n0 = (int64_t)tn * TN, k0 = (int64_t)tk * TK;

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  uint32_t a_off[4], b_off[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) a_off[i] = tr_addr(8 * h, wn * 128 + 32 * i, lane);
#pragma unroll
  for (int j = 0; j < 2; ++j) b_off[j] = tr_addr(8 * h, wk * 64 + 32 * j, lane);
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;

  auto stage = [&](int t) {  // slot t % NSLOT <- tokens [t*BM, t*BM + BM)
    if constexpr (MODE == 2) return;  // experiment: no HBM/L2 traffic in the main loop
    const int dst = (t % NSLOT) * SLOTB;
    stage_op<T>(dy, N, (int64_t)t * BM, n0, lds, dst, wave, lane);
    stage_op<T>(x, K, (int64_t)t * BM, k0, lds, dst + OPB, wave, lane);
  };

  // Fragment registers: two sets, always one k-step (16 tokens) ahead.
  fa::bf16x4 fa_[2][4][2], fb_[2][2][2];
  auto issue = [&](int t, int s, int set) {  // k-step s (0/1) of slot t
    const uint32_t ca = lds_base + (t % NSLOT) * SLOTB + (16 * s) * ROWB, cb = ca + OPB;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int u = 0; u < 2; ++u) fa_[set][i][u] = tr_read_asm(ca + a_off[i] + 4 * u * ROWB);
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int u = 0; u < 2; ++u) fb_[set][j][u] = tr_read_asm(cb + b_off[j] + 4 * u * ROWB);
  };
  auto mfmas = [&](int set) {
    typename MT<T>::x8 a[4], b[2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      a[i] = __builtin_bit_cast(typename MT<T>::x8, fa::join<bf16>(fa_[set][i][0], fa_[set][i][1]));
#pragma unroll
    for (int j = 0; j < 2; ++j)
      b[j] = __builtin_bit_cast(typename MT<T>::x8, fa::join<bf16>(fb_[set][j][0], fb_[set][j][1]));
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = MT<T>::mfma(a[i], b[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nt = M / BM;
#pragma unroll
  for (int t = 0; t < NSLOT - 1; ++t)
    if (t < nt) stage(t);
  wait_slots(min(nt, NSLOT - 1) - 1);  // slot 0 landed, the rest may be in flight
  __builtin_amdgcn_s_barrier();
  issue(0, 0, 0);

  // Per slot t:   [reads (t,1)] [MFMA (t,0)] [wait slot t+1, barrier, stage t+3]
  //               [reads (t+1,0)] [MFMA (t,1)]
  // The barrier sits mid-slot, so the MFMAs of (t,0) cover it and the
  // fragment reads never drain across a slot boundary.  RAW: slot t+1's
  // loads are waited (counted vmcnt) by every wave before the barrier.  WAR:
  // slot t+3 reuses slot t-1, whose reads all completed before the MFMAs of
  // (t-1,1), i.e. before this barrier in every wave.
  for (int t = 0; t < nt; ++t) {
    issue(t, 1, 1);
    asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfmas(0);
    if (t + 1 < nt) {
      // slots issued after t+1 may stay in flight: t+2 .. min(t+NSLOT-2, nt-1)
      wait_slots(min(t + NSLOT - 2, nt - 1) - (t + 1));
      __builtin_amdgcn_s_barrier();
      if (t + NSLOT - 1 < nt) stage(t + NSLOT - 1);
      issue(t + 1, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_sched_barrier(0);
    mfmas(1);
  }

  // epilogue: G[n][k] (+)= acc ; col = lane & 31, row = acc_row(reg, h)
  if constexpr (MODE == 1) {  // experiment: keep acc alive, skip the epilogue traffic
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) s += acc[i][j][0] + acc[i][j][15];
    if (s == 1234567.f) g[threadIdx.x] = s;
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = k0 + wk * 64 + 32 * j + (lane & 31);
      float* base = g + (n0 + wn * 128 + 32 * i) * (int64_t)K + col;
      if (ACCUM) {  // batch the 16 loads, then one wait, then the stores
        float old[16];
#pragma unroll
        for (int r = 0; r < 16; ++r)
          old[r] = __builtin_nontemporal_load(base + (int64_t)fa::acc_row(r, h) * K);
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_nontemporal_store(old[r] + acc[i][j][r],
                                      base + (int64_t)fa::acc_row(r, h) * K);
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          __builtin_nontemporal_store(acc[i][j][r], base + (int64_t)fa::acc_row(r, h) * K);
      }
    }
}

template <typename T, bool ACCUM, int MODE = 0>
void launch(const void* dy, const void* x, float* g, int M, int N, int K, hipStream_t s) {
  const int ntiles = (N / TN) * (K / TK);
  hipLaunchKernelGGL((wgrad_k<T, ACCUM, MODE>), dim3(ntiles), dim3(512), 0, s, (const T*)dy,
                     (const T*)x, g, M, N, K);
}

}  // namespace

// Ablation builds for profiling (bf16, accumulate): 1 = no epilogue traffic,
// 2 = no global loads in the main loop (LDS/MFMA/barrier pipeline only).
void wgrad_gemm_ablation(const void* dy, const void* x, float* g, int64_t M, int64_t N,
                         int64_t K, int mode, hipStream_t s) {
  if (mode == 1) launch<bf16, true, 1>(dy, x, g, (int)M, (int)N, (int)K, s);
  else if (mode == 2) launch<bf16, true, 2>(dy, x, g, (int)M, (int)N, (int)K, s);
  else launch<bf16, true, 0>(dy, x, g, (int)M, (int)N, (int)K, s);
}

bool wgrad_supported(int64_t M, int64_t N, int64_t K) {
  return M > 0 && N > 0 && K > 0 && M % BM == 0 && N % TN == 0 && K % TK == 0 &&
         M <= (int64_t)1 << 30 && (N / TN) * (K / TK) < (int64_t)1 << 31 &&
         N * K < ((int64_t)1 << 40);
}

void wgrad_gemm(const void* dy, const void* x, float* g, int64_t M, int64_t N, int64_t K,
                bool accumulate, int dt, hipStream_t s) {
  if (dt == DT_BF16) {
    if (accumulate) launch<bf16, true>(dy, x, g, (int)M, (int)N, (int)K, s);
    else launch<bf16, false>(dy, x, g, (int)M, (int)N, (int)K, s);
  } else if (dt == DT_F16) {
    if (accumulate) launch<fp16, true>(dy, x, g, (int)M, (int)N, (int)K, s);
    else launch<fp16, false>(dy, x, g, (int)M, (int)N, (int)K, s);
  }
}

}  // namespace ema
