// FlashAttention-2 forward for gfx950 (MI355X), native GQA/MQA, causal.
//
// Workgroup = WAVES waves = a WAVES*32-row query block of one (batch, query
// head); each wave owns 32 query rows (8 waves: two per SIMD sharing every K/V
// tile; 4 waves, two workgroups per CU, at head_dim 64 or on small grids).
// K/V tiles of 64 keys arrive by LDS-DMA (global_load_lds, one 1-KiB piece per
// wave instruction) into the image-(a) layout of the dQ kernel (8-row x 32-col
// subtiles, XOR swizzle produced through the per-lane SOURCE address): no
// staging registers and no ds_write pass; with 8 waves a 3-tile ring with a
// counted vmcnt keeps the DMA two tiles ahead (profiles/r2c_fa_fwd_v5_ab.txt:
// +1-2 % at s=1k, +4-8 % at s=4k, +13 % on TP-rank shapes over the earlier
// register-staged kernel).  One barrier per tile.
//
// Per 32(q) x 64(k) step a wave runs 2 x HD/16 MFMAs for S^T = K Q^T (K read
// by rows) and 2 x 2 x HD/32 MFMAs for O^T += V^T P^T (V^T by
// ds_read_b64_tr_b16, hardware transpose, guide T10), v_mfma_f32_32x32x16.
// S is computed transposed ("swapped QK^T", guide T12) so a query row lives on
// one lane pair (lane, lane^32): the online-softmax max/sum is 31 in-register
// ops + one cross-half shuffle, the O rescale is a per-lane scalar (skipped
// when no lane's max moved), and the P accumulator feeds the PV MFMA as its B
// operand with no LDS round trip.
//
// Query head j reads KV group j / (nq / nkv) directly (no K/V expansion).
// Query blocks are dispatched on a flat grid, heaviest causal blocks of ALL
// heads first.  LSE is written in natural log.
//
// Document mask (p.doc_start set, packed sequences): each query block starts
// at the key tile of its first row's document; keys before a row's document
// start are masked like the causal upper triangle.
//
// Fused RoPE (p.rope_cos set): Q is rotated in registers right after its load
// and written back in place (only this workgroup reads those rows), so the
// backward sees rotated Q; K is rotated by a k-only pre-pass (rope.hip).
#include <cstdlib>

#include "fa_common.h"
#include "kernels.h"

namespace ema {
namespace fa {
namespace {


typedef __attribute__((ext_vector_type(2))) float f2;
typedef __attribute__((ext_vector_type(4))) float f4;

template <typename T, int HD, bool CAUSAL, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 8 / WAVES) void fa_fwd_k(const AttnParams p) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  constexpr int BMW = WAVES * 32, KT = 64;
  constexpr int KS = HD / 16, DT = HD / 32;
  constexpr int ROWB = HD * 2, RG = 8 * ROWB, PIECES = KT * ROWB / 1024, PPW = PIECES / WAVES;
  constexpr int TB = KT * ROWB;  // bytes of one K (or V) tile
  constexpr int NB = WAVES == 8 ? 3 : 2;
  static_assert(PIECES % WAVES == 0, "pieces per wave");
  __shared__ __attribute__((aligned(1024))) char lds[NB * 2 * TB];

  const int tid = threadIdx.x;
  unsigned long long st0 = 0, st1 = 0, st2 = 0;
  if (p.stamps) st0 = fa::wall_stamp();
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nmb = (p.sq + BMW - 1) / BMW;
  const int nhb = p.nq * p.b;
  const int lin = blockIdx.x;
  const int mb = CAUSAL ? (nmb - 1 - lin / nhb) : lin / nhb;
  const int hb = lin % nhb;
  const int head = hb % p.nq, b = hb / p.nq;
  const int r = p.nq / p.nkv, g = head / r;
  const int off = p.coff;

  const T* Q = (const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg + (int64_t)(head % r) * p.q_sh;
  const T* K = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg;
  const T* V = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg;

  const int m0 = mb * BMW + wave * 32;
  const int qrow = m0 + c;
  const int qrow_c = qrow < p.sq ? qrow : p.sq - 1;

  int n_end = p.sk;
  if (CAUSAL) {
    const int lim = mb * BMW + BMW + off;
    n_end = lim < p.sk ? lim : p.sk;
  }
  const int ntiles = n_end > 0 ? (n_end + KT - 1) / KT : 0;
  int wtiles = ntiles;
  if (CAUSAL) {
    const int wl = m0 + 32 + off;
    const int wt = wl > 0 ? (wl + KT - 1) / KT : 0;
    wtiles = wt < ntiles ? wt : ntiles;
  }
  // document mask: the block starts at its first row's document, each wave at
  // its own first row's; keys below a row's document start are masked
  int t0 = 0, wt0 = 0, ds_row = 0, ds_wmax = 0;
  if (CAUSAL && p.doc_start) {
    const int* D = p.doc_start + (int64_t)b * p.sq;
    const int r0 = mb * BMW < p.sq ? mb * BMW : p.sq - 1;
    const int w0 = m0 < p.sq ? m0 : p.sq - 1, w1 = m0 + 31 < p.sq ? m0 + 31 : p.sq - 1;
    t0 = D[r0] / KT;
    wt0 = D[w0] / KT;
    ds_wmax = D[w1];
    ds_row = D[qrow_c];
  }

  int srow[PPW], schunk[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int o = (wave * PPW + i) * 1024 + 16 * lane;
    const int rem = o % RG, rem2 = rem % 512;
    srow[i] = 8 * (o / RG) + rem2 / 64;
    schunk[i] = 4 * (rem / 512) + (((rem2 % 64) / 16) ^ ((srow[i] >> 2) & 3));
  }
  auto prefetch = [&](int t, int slot) {
    char* kl = lds + slot * 2 * TB;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;
      int kr = t * KT + srow[i];
      kr = kr < p.sk ? kr : p.sk - 1;
      __builtin_amdgcn_global_load_lds((const void*)(K + (int64_t)kr * p.k_ss + schunk[i] * 8),
                                       (__attribute__((address_space(3))) void*)(kl + pc * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(V + (int64_t)kr * p.v_ss + schunk[i] * 8),
                                       (__attribute__((address_space(3))) void*)(kl + TB + pc * 1024),
                                       16, 0, 0);
    }
  };
  if (t0 < ntiles) prefetch(t0, t0 % NB);
  if (NB == 3 && t0 + 1 < ntiles) prefetch(t0 + 1, (t0 + 1) % NB);

  x8 qf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) qf[kk] = ld8(Q + (int64_t)qrow_c * p.q_ss + kk * 16 + 8 * h);
  if (p.rope_cos) {
    const float *rc, *rs;
    rope_rows<HD>(p, b, qrow_c, rc, rs);
    rope_rows_fwd<T, KS>(qf, rc, rs, h);  // table loads batched (not one round trip per fragment)
    if (qrow < p.sq) {
      T* Qw = const_cast<T*>(Q) + (int64_t)qrow * p.q_ss + 8 * h;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) *reinterpret_cast<x8*>(Qw + kk * 16) = qf[kk];
    }
  }

  f32x16 o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[d][i] = 0.f;
  float m_i = -INFINITY, l_i = 0.f;
  const float sl2 = p.scale * 1.4426950408889634f;

  int rowb[2], trb[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    rowb[x] = RG * (c >> 3) + 64 * (c & 7) + 16 * ((2 * x + h) ^ ((c >> 2) & 3));
    trb[x] = RG * x + 64 * (4 * h + tq) + 16 * ((2 * ((lane >> 4) & 1) + (tp >> 1)) ^ ((h + 2 * x) & 3)) +
             8 * (tp & 1);
  }
  __syncthreads();  // vmcnt(0) + barrier: tile 0 (and 1) landed
  if (p.stamps) st1 = fa::wall_stamp();

  for (int t = t0; t < ntiles; ++t) {
    // WAR: tile t+NB-1 overwrites the slot of tile t-1, whose reads every wave
    // retired before the barrier that ended tile t-1
    if (t + NB - 1 < ntiles) prefetch(t + NB - 1, (t + NB - 1) % NB);
    if (t < wtiles && t >= wt0) {
      const int n0 = t * KT;
      const char* kl = lds + (t % NB) * 2 * TB;
      const uint32_t trv0 = (uint32_t)(uintptr_t)(kl + trb[0]);
      const uint32_t trv1 = (uint32_t)(uintptr_t)(kl + trb[1]);
      f32x16 s0, s1;
#pragma unroll
      for (int i = 0; i < 16; ++i) s0[i] = s1[i] = 0.f;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const int ko = rowb[kk & 1] + 512 * (kk >> 1);
        const x8 ka0 = *reinterpret_cast<const x8*>(kl + ko);
        const x8 ka1 = *reinterpret_cast<const x8*>(kl + 4 * RG + ko);
        s0 = MT<T>::mfma(ka0, qf[kk], s0);
        s1 = MT<T>::mfma(ka1, qf[kk], s1);
      }
      // V^T fragments of the tile (asm transposed reads: no wait on the DMA
      // in flight; retired by lds_wait before the first PV MFMA)
      x4 vf[2][2][DT][2];
      static_for<2>([&](auto subc) {
        static_for<2>([&](auto scc) {
          static_for<DT>([&](auto dcc) {
            constexpr int vo = TB + decltype(subc)::value * 4 * RG + decltype(scc)::value * 2 * RG +
                               512 * decltype(dcc)::value;
            vf[subc][scc][dcc][0] = tr_read_imm<vo, T>(trv0);
            vf[subc][scc][dcc][1] = tr_read_imm<vo, T>(trv1);
          });
        });
      });
      // (causal: the key-count bound only binds when the diagonal offset
      // reaches past sk, i.e. a context-parallel pair run with coff = sk)
      const bool need_mask = CAUSAL ? (n0 + KT - 1 > m0 + off || n0 < ds_wmax || n0 + KT > p.sk)
                                    : (n0 + KT > p.sk);
      if (need_mask) {
        // element i of s0 is key n0 + acc_row(i, h), of s1 that + 32: with
        // rc = acc_row(i, 0) the tests are rc <= hi and rc >= lo, one compare
        // and one select per element (lo only under a document mask)
        int hi = p.sk - 1 - n0 - 4 * h;
        if (CAUSAL) hi = min(hi, qrow + off - n0 - 4 * h);
        if (CAUSAL && p.doc_start) {
          const int lo = ds_row - n0 - 4 * h;
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rc = (i & 3) + 8 * (i >> 2);
            if (rc > hi || rc < lo) s0[i] = -INFINITY;
            if (rc + 32 > hi || rc + 32 < lo) s1[i] = -INFINITY;
          }
        } else {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int rc = (i & 3) + 8 * (i >> 2);
            if (rc > hi) s0[i] = -INFINITY;
            if (rc + 32 > hi) s1[i] = -INFINITY;
          }
        }
      }
      // row max: 16 three-input max, the lane pair (l, l ^ 32) combined by one
      // permlane32 swap (no LDS round trip)
      float mt = fmaxf(s0[0], s1[0]);
#pragma unroll
      for (int i = 1; i < 16; ++i) mt = fmaxf(fmaxf(mt, s0[i]), s1[i]);
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mt), __float_as_uint(mt),
                                                         false, false);
        mt = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * sl2;
      }
      const float m_new = fmaxf(m_i, mt);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_i - m_use);
      // p = exp2(s * scale * log2e - m): packed fma for the argument, packed
      // adds for the row sum
      const f2 sc2 = {sl2, sl2}, mm2 = {-m_use, -m_use};
      f2 rs2 = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        f2 a = __builtin_elementwise_fma(f2{s0[i], s0[i + 1]}, sc2, mm2);
        f2 b = __builtin_elementwise_fma(f2{s1[i], s1[i + 1]}, sc2, mm2);
        a[0] = __builtin_amdgcn_exp2f(a[0]);
        a[1] = __builtin_amdgcn_exp2f(a[1]);
        b[0] = __builtin_amdgcn_exp2f(b[0]);
        b[1] = __builtin_amdgcn_exp2f(b[1]);
        s0[i] = a[0]; s0[i + 1] = a[1];
        s1[i] = b[0]; s1[i + 1] = b[1];
        rs2 += a;
        rs2 += b;
      }
      float rsum = rs2[0] + rs2[1];
      {
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(rsum),
                                                         __float_as_uint(rsum), false, false);
        rsum = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
      }
      l_i = l_i * alpha + rsum;
      m_i = m_new;
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
        for (int d = 0; d < DT; ++d)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[d][i] *= alpha;
      }
      lds_wait();
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int sc = 0; sc < 2; ++sc) {
          const x8 pf = acc_frag<T>(sub == 0 ? s0 : s1, sc);
#pragma unroll
          for (int dc = 0; dc < DT; ++dc)
            o[dc] = MT<T>::mfma(join<T>(vf[sub][sc][dc][0], vf[sub][sc][dc][1]), pf, o[dc]);
        }
    }
    if (NB == 3 && t + 2 < ntiles) {
      // counted: tile t+1 landed, tile t+2's DMA (2 * PPW instructions) may fly on
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(2 * PPW) : "memory");
      __builtin_amdgcn_s_barrier();
    } else {
      __syncthreads();  // vmcnt(0) + barrier: tile t+1 landed, tile t's reads retired
    }
  }

  if (p.stamps) st2 = fa::wall_stamp();
  if (qrow < p.sq) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    const float lse_j = l_i > 0.f ? (m_i + __log2f(l_i)) * 0.6931471805599453f : -INFINITY;
    float* lp = p.lse + (int64_t)b * p.lse_sb + (int64_t)head * p.lse_sh + qrow;
    if (p.o32) {
      // ring-attention step: combine with the running (O, lse) in place
      float w_old = 0.f, w_new = inv, lse_new = lse_j;
      if (p.merge) {
        const float old = *lp;
        const float mx = fmaxf(old, lse_j);
        if (mx == -INFINITY) {
          w_new = 0.f;
        } else {
          const float eo = __expf(old - mx), en = __expf(lse_j - mx), s = eo + en;
          lse_new = mx + __logf(s);
          w_old = eo / s;
          w_new = inv * (en / s);
        }
      }
      float* O32 = p.o32 + (int64_t)b * p.o32_sb + (int64_t)qrow * p.o32_ss + (int64_t)head * p.o32_sh;
#pragma unroll
      for (int d = 0; d < DT; ++d) {
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          f4* dst = reinterpret_cast<f4*>(O32 + d * 32 + 8 * rg + 4 * h);
          f4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = o[d][4 * rg + e] * w_new;
          if (p.merge) v += *dst * w_old;
          *dst = v;
        }
      }
      if (h == 0) *lp = lse_new;
    } else {
      T* O = (T*)p.o + (int64_t)b * p.o_sb + (int64_t)qrow * p.o_ss + (int64_t)head * p.o_sh;
#pragma unroll
      for (int d = 0; d < DT; ++d) {
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          x4 w;
#pragma unroll
          for (int e = 0; e < 4; ++e) w[e] = (T)(o[d][4 * rg + e] * inv);
          *reinterpret_cast<x4*>(O + d * 32 + 8 * rg + 4 * h) = w;
        }
      }
      if (h == 0) *lp = lse_j;
    }
  }
  if (p.stamps) {  // diagnostics (scripts/fa_stamps.py)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores done
    __syncthreads();
    if (tid == 0 && (int64_t)lin * 8 + 8 <= p.stamps_n) {
      unsigned long long* so = p.stamps + (int64_t)lin * 8;
      so[0] = st0; so[1] = st1; so[2] = st2; so[3] = fa::wall_stamp();
      so[4] = __smid(); so[5] = fa::xcc_id();
    }
  }
}


// ---- forward v2 (head_dim 128): 4 waves, 64 query rows per wave ------------
// Each wave owns two 32-row sub-blocks A (rows 0-31 of its 64) and B (32-63)
// and runs them half a K/V tile apart, so one sub-block's softmax (VALU)
// issues between the other's MFMAs on the same SIMD (one wave per SIMD: the
// MFMA and VALU pipes are separate, and an in-order wave keeps both busy
// when the two instruction streams are independent).  Per 32-key tile t:
//   slot P(t):  MFMA  PV_B(t-1), QK_B(t)        VALU  softmax_A(t)
//   [tile t+1 landed (own DMA), barrier, DMA of tile t+3]
//   slot Q(t):  MFMA  PV_A(t),   QK_A(t+1)      VALU  softmax_B(t)
// (QK_X(t) = S^T = K_t Q_X^T into X's 16 score VGPRs, PV_X(t) = O_X^T +=
// V_t^T P_X(t)^T from X's bf16 P fragments: 8 MFMAs each).  Registers: O in
// AGPRs and Q read from AGPRs by the asm MFMAs; scores, P and one tile's K / V
// fragments in arch VGPRs.  The O rescale of the online softmax is lazy
// (guide T13): a row's running max moves only when a tile's max exceeds it by
// more than kFaThr (log2 units; P <= 2^kFaThr), so the rescale (an AGPR round
// trip) runs on a few early tiles, not every tile.  LDS: a 4-tile ring of
// image-(a) K / V tiles by LDS-DMA, refilled at the mid-tile barrier two
// tiles ahead.  Fully masked tiles of one sub-block (diagonal) run the same
// code with p = 0.
// Reference: megatron/model/transformer.py:514-522 (flash_attn_func).
constexpr float kFaThr = 8.f;

template <typename T, int NOP = 0>
__device__ __forceinline__ void mfma_kq(f32x16& acc, typename MT<T>::x8 k, typename MT<T>::x8 q) {
  // S^T += K Q^T with Q held in AGPRs (operand B)
  if constexpr (__is_same(T, bf16)) {
    if constexpr (NOP) asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "a"(q));
    else asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "a"(q));
  } else {
    if constexpr (NOP) asm("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "a"(q));
    else asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(k), "a"(q));
  }
}
template <typename T>
__device__ __forceinline__ void mfma_kq0(f32x16& acc, typename MT<T>::x8 k, typename MT<T>::x8 q) {
  if constexpr (__is_same(T, bf16))
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(k), "a"(q));
  else
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(k), "a"(q));
}

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fa_fwd2_k(const AttnParams p) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  constexpr int HD = 128, BMW = 256, KT = 32, KS = HD / 16, DT = HD / 32;
  constexpr int ROWB = HD * 2, RG = 8 * ROWB, TB = KT * ROWB;  // 256 B rows, 8 KiB tiles
  constexpr int PIECES = TB / 1024, PPW = PIECES / 4;          // 8 pieces, 2 per wave
  constexpr int NB = 4;
  __shared__ __attribute__((aligned(1024))) char lds[NB * 2 * TB];  // 64 KiB

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, c = lane & 31;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nmb = (p.sq + BMW - 1) / BMW;
  const int nhb = p.nq * p.b;
  const int lin = blockIdx.x;
  const int mb = CAUSAL ? (nmb - 1 - lin / nhb) : lin / nhb;
  const int hb = lin % nhb;
  const int head = hb % p.nq, b = hb / p.nq;
  const int r = p.nq / p.nkv, g = head / r;
  const int off = p.coff;

  const T* Q = (const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg + (int64_t)(head % r) * p.q_sh;
  const T* K = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg;
  const T* V = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg;

  // sub-block X in {A, B}: query rows mX .. mX + 31, this lane's row mX + c
  const int mA = mb * BMW + wave * 64, mB = mA + 32;
  const int qrowA = mA + c, qrowB = mB + c;
  const int qA_c = qrowA < p.sq ? qrowA : p.sq - 1, qB_c = qrowB < p.sq ? qrowB : p.sq - 1;

  int n_end = p.sk;
  if (CAUSAL) {
    const int lim = mb * BMW + BMW + off;
    n_end = lim < p.sk ? lim : p.sk;
  }
  const int ntiles = n_end > 0 ? (n_end + KT - 1) / KT : 0;
  // the wave's tiles [wlo, whi): the union of its two sub-blocks' ranges
  int whi = ntiles;
  if (CAUSAL) {
    const int wl = mB + 32 + off;
    const int wt = wl > 0 ? (wl + KT - 1) / KT : 0;
    whi = wt < ntiles ? wt : ntiles;
  }
  int t0 = 0, wlo = 0, dsA_row = 0, dsB_row = 0, dsA_max = 0, dsB_max = 0;
  if (CAUSAL && p.doc_start) {
    const int* D = p.doc_start + (int64_t)b * p.sq;
    const int rb = mb * BMW < p.sq ? mb * BMW : p.sq - 1;
    const int ra = mA < p.sq ? mA : p.sq - 1;
    const int ra31 = mA + 31 < p.sq ? mA + 31 : p.sq - 1, rb31 = mB + 31 < p.sq ? mB + 31 : p.sq - 1;
    t0 = D[rb] / KT;
    wlo = D[ra] / KT;
    dsA_max = D[ra31];
    dsB_max = D[rb31];
    dsA_row = D[qA_c];
    dsB_row = D[qB_c];
  }
  if (wlo < t0) wlo = t0;

  int srow[PPW], schunk[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int o = (wave * PPW + i) * 1024 + 16 * lane;
    const int rem = o % RG, rem2 = rem % 512;
    srow[i] = 8 * (o / RG) + rem2 / 64;
    schunk[i] = 4 * (rem / 512) + (((rem2 % 64) / 16) ^ ((srow[i] >> 2) & 3));
  }
  auto prefetch = [&](int t) {
    char* kl = lds + (t % NB) * 2 * TB;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;
      int kr = t * KT + srow[i];
      kr = kr < p.sk ? kr : p.sk - 1;
      __builtin_amdgcn_global_load_lds((const void*)(K + (int64_t)kr * p.k_ss + schunk[i] * 8),
                                       (__attribute__((address_space(3))) void*)(kl + pc * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(V + (int64_t)kr * p.v_ss + schunk[i] * 8),
                                       (__attribute__((address_space(3))) void*)(kl + TB + pc * 1024),
                                       16, 0, 0);
    }
  };
#pragma unroll
  for (int k = 0; k < NB - 1; ++k)
    if (t0 + k < ntiles) prefetch(t0 + k);

  x8 qa[KS], qb[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    qa[kk] = ld8(Q + (int64_t)qA_c * p.q_ss + kk * 16 + 8 * h);
    qb[kk] = ld8(Q + (int64_t)qB_c * p.q_ss + kk * 16 + 8 * h);
  }
  if (p.rope_cos) {
    const float *rc, *rs;
    rope_rows<HD>(p, b, qA_c, rc, rs);
    rope_rows_fwd<T, KS>(qa, rc, rs, h);
    rope_rows<HD>(p, b, qB_c, rc, rs);
    rope_rows_fwd<T, KS>(qb, rc, rs, h);
    T* Qw = const_cast<T*>(Q);
    if (qrowA < p.sq)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) *reinterpret_cast<x8*>(Qw + (int64_t)qrowA * p.q_ss + kk * 16 + 8 * h) = qa[kk];
    if (qrowB < p.sq)
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) *reinterpret_cast<x8*>(Qw + (int64_t)qrowB * p.q_ss + kk * 16 + 8 * h) = qb[kk];
  }

  // Q lives in AGPRs for the whole block (operand B of the asm score MFMAs):
  // defined there once through an empty asm with an AGPR output
  x8 qaa[KS], qba[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    asm volatile("; q -> agpr" : "=a"(qaa[kk]) : "0"(qa[kk]));
    asm volatile("; q -> agpr" : "=a"(qba[kk]) : "0"(qb[kk]));
  }

  f32x16 oa[DT], ob[DT];  // AGPR-resident (asm MFMAs only, zeroed by an MFMA with C = 0)
  f32x16 sa, sb;          // S^T of the current tile: keys acc_row(i, h), query c
  x8 pa[2], pb[2];        // bf16 P fragments (k-steps of 16 keys)
  float ma = -INFINITY, la = 0.f, mbx = -INFINITY, lb = 0.f;
  const float sl2 = p.scale * 1.4426950408889634f;
  {
    x8 z;
#pragma unroll
    for (int e = 0; e < 8; ++e) z[e] = (T)0.f;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      mfma_agpr0_init<T>(oa[d], z);
      mfma_agpr0_init<T>(ob[d], z);
    }
  }

  // lane's LDS read bases (image (a)): K rows (row = key c), V^T transposed
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  uint32_t rowb[2], trb[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    rowb[x] = lds_base + RG * (c >> 3) + 64 * (c & 7) + 16 * ((2 * x + h) ^ ((c >> 2) & 3));
    trb[x] = lds_base + RG * x + 64 * (4 * h + tq) +
             16 * ((2 * ((lane >> 4) & 1) + (tp >> 1)) ^ ((h + 2 * x) & 3)) + 8 * (tp & 1);
  }

  x8 kf[KS];          // K fragments of one tile (AGPRs: ds_read_b128 -> MFMA operand A)
  x4 vf[2][DT][2];    // V^T fragments of one tile [k-step][d-tile][half]
  auto read_k = [&](int t) {
    const uint32_t so = (uint32_t)((t % NB) * 2 * TB);
    const uint32_t b0 = rowb[0] + so, b1 = rowb[1] + so;
    static_for<KS>([&](auto kc) {
      constexpr int KK = decltype(kc)::value, O = 512 * (KK >> 1);
      kf[KK] = row_read_imm_a<O, T>((KK & 1) ? b1 : b0);
    });
  };
  // V^T fragments of tile t, part P of 4 (k-step P / 2, d-tiles 2 (P % 2) and
  // 2 (P % 2) + 1): issued between the MFMAs of the slot before their use
  auto read_v = [&](int t, auto pc) {
    constexpr int P = decltype(pc)::value, SC = P / 2;
    const uint32_t so = (uint32_t)((t % NB) * 2 * TB);
    const uint32_t v0 = trb[0] + so, v1 = trb[1] + so;
    static_for<2>([&](auto dd) {
      constexpr int DC = 2 * (P % 2) + decltype(dd)::value;
      constexpr int vo = TB + SC * 2 * RG + 512 * DC;
      vf[SC][DC][0] = tr_read_imm<vo, T>(v0);
      vf[SC][DC][1] = tr_read_imm<vo, T>(v1);
    });
  };
  // ---- MFMA steps (asm volatile: issued in source order, so the VALU
  // placed between them below interleaves the two sub-blocks' streams)
  auto qk_step = [&](const x8 (&q)[KS], f32x16& sc, auto kc) {
    constexpr int KK = decltype(kc)::value;
    if constexpr (KK == 0) {
      if constexpr (__is_same(T, bf16))
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(sc) : "a"(kf[0]), "a"(q[0]));
      else
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(sc) : "a"(kf[0]), "a"(q[0]));
    } else {
      if constexpr (__is_same(T, bf16))
        asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(sc) : "a"(kf[KK]), "a"(q[KK]));
      else
        asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(sc) : "a"(kf[KK]), "a"(q[KK]));
    }
  };
  auto pv_step = [&](const x8 (&pf)[2], f32x16 (&o)[DT], auto jc) {
    constexpr int J = decltype(jc)::value, SC = J / DT, DC = J % DT;
    const x8 vv = join<T>(vf[SC][DC][0], vf[SC][DC][1]);
    // (P fragments were written by VALU a slot earlier: no s_nop needed)
    if constexpr (__is_same(T, bf16))
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o[DC]) : "v"(vv), "v"(pf[SC]));
    else
      asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(o[DC]) : "v"(vv), "v"(pf[SC]));
  };
  // ---- softmax pieces of one sub-block's tile
  auto mask = [&](f32x16& sc, int t, int m0, int qrow, int ds_row, int ds_max) {
    const int n0 = t * KT;
    const bool need_mask = CAUSAL ? (n0 + KT - 1 > m0 + off || n0 < ds_max || n0 + KT > p.sk)
                                  : (n0 + KT > p.sk);
    if (need_mask) {
      int hi = p.sk - 1 - n0 - 4 * h;
      if (CAUSAL) hi = min(hi, qrow + off - n0 - 4 * h);
      const int lo = (CAUSAL && p.doc_start) ? ds_row - n0 - 4 * h : -KT;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int rc = (i & 3) + 8 * (i >> 2);
        if (rc > hi || rc < lo) sc[i] = -INFINITY;
      }
    }
  };
  // lazy rescale (guide T13): rare after a block's first tile
  auto rescale = [&](float mt, float& m_i, float& l_i, f32x16 (&o)[DT]) {
    const bool grow = mt > m_i + kFaThr;
    if (__builtin_amdgcn_ballot_w64(grow)) {
      // (a lane that does not grow keeps alpha = 1: its m_i may still be -inf
      // under a document mask, and -inf - -inf would poison O and l)
      const float m_new = grow ? fmaxf(m_i, mt) : m_i;
      const float alpha = grow ? __builtin_amdgcn_exp2f(m_i - m_new) : 1.f;
      fa::mfma_drain();
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        f32x16 v;
        asm volatile("; o -> vgpr" : "=v"(v) : "0"(o[d]));
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] *= alpha;
        asm volatile("; vgpr -> o" : "=a"(o[d]) : "0"(v));
      }
      l_i *= alpha;
      m_i = m_new;
    }
  };
  // One slot: 8 "first" MFMAs (fa) interleaved with the row max of sub-block
  // X's scores, the rescale decision, 8 "second" MFMAs (fb) interleaved with
  // the exponentials / row sum / bf16 P fragments of X.
  auto slot = [&](f32x16& sc, float& m_i, float& l_i, f32x16 (&o)[DT], x8 (&pf)[2], auto fa_,
                  auto fb_, auto pre_b, auto rd_) {
    float mt = -INFINITY;
    static_for<8>([&](auto jc) {
      constexpr int J = decltype(jc)::value;
      fa_(jc);
      mt = fmaxf(fmaxf(mt, sc[2 * J]), sc[2 * J + 1]);
      __builtin_amdgcn_sched_barrier(0);
    });
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(mt), __float_as_uint(mt),
                                                       false, false);
      mt = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * sl2;
    }
    rescale(mt, m_i, l_i, o);
    const float m_use = m_i == -INFINITY ? 0.f : m_i;
    float rs = 0.f;
    pre_b();
    static_for<8>([&](auto jc) {
      constexpr int J = decltype(jc)::value;
      fb_(jc);
      rd_(jc);
      sc[2 * J] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[2 * J], sl2, -m_use));
      sc[2 * J + 1] = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[2 * J + 1], sl2, -m_use));
      rs += sc[2 * J] + sc[2 * J + 1];
      if constexpr (J == 4) pf[0] = acc_frag<T>(sc, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    pf[1] = acc_frag<T>(sc, 1);
    {
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(rs), __float_as_uint(rs),
                                                       false, false);
      rs = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    l_i += rs;
  };
  auto none = [&](auto) {};

  // tiles t0 .. t0 + NB - 2 landed (own DMA), then everyone's
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  // mid-tile sync of tile t: tile t+1 landed (own DMA; tile t+2's may fly),
  // then everyone's; tile t-1's ring slot is free: refill it with tile t+3
  auto mid = [&](int t) {
    if (t + 2 < ntiles) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t + NB - 1 < ntiles) prefetch(t + NB - 1);
  };
  // Fragment registers: slot Q(t-1) leaves K_t in kf and V_{t-1} in vf, which
  // are exactly slot P(t)'s MFMA operands, so slot P starts without an LDS
  // round trip; it reads V_t between its QK_B MFMAs (after its PV_B MFMAs
  // consumed V_{t-1}).  Slot Q(t) reads K_{t+1} (landed at the mid barrier)
  // under its PV_A(t) MFMAs and waits for it only before QK_A(t+1).
  auto rd_v = [&](int t) {
    return [&, t](auto jc) {
      constexpr int J = decltype(jc)::value;
      if constexpr (J < 4) read_v(t, jc);
    };
  };
  auto lds_wait_fn = [&]() { lds_wait(); };
  auto nothing = [&]() {};
  // slot P(t): PV_B(t-1), QK_B(t) | softmax_A(t)
  auto slot_p = [&](int t, auto first) {
    if constexpr (decltype(first)::value) {  // prologue: S_A of the wave's first tile
      read_k(t);
      lds_wait();
      static_for<KS>([&](auto kc) { qk_step(qaa, sa, kc); });
    }
    fa::mfma_drain();
    mask(sa, t, mA, qrowA, dsA_row, dsA_max);
    if constexpr (decltype(first)::value)
      slot(sa, ma, la, oa, pa, none, [&](auto kc) { qk_step(qba, sb, kc); }, nothing, rd_v(t));
    else
      slot(sa, ma, la, oa, pa, [&](auto jc) { pv_step(pb, ob, jc); },
           [&](auto kc) { qk_step(qba, sb, kc); }, nothing, rd_v(t));
  };
  // slot Q(t): PV_A(t), QK_A(t+1) | softmax_B(t); on the wave's last tile
  // (no QK_A(t+1)) its final PV_B(t) follows, while V_t is still in registers
  auto slot_q = [&](int t, auto last) {
    if constexpr (!decltype(last)::value) read_k(t + 1);
    fa::mfma_drain();
    mask(sb, t, mB, qrowB, dsB_row, dsB_max);
    if constexpr (decltype(last)::value) {
      slot(sb, mbx, lb, ob, pb, [&](auto jc) { pv_step(pa, oa, jc); }, none, nothing, none);
      static_for<8>([&](auto jc) { pv_step(pb, ob, jc); });
    } else {
      slot(sb, mbx, lb, ob, pb, [&](auto jc) { pv_step(pa, oa, jc); },
           [&](auto kc) { qk_step(qaa, sa, kc); }, lds_wait_fn, none);
    }
  };

  int t = t0;
  const int lo_ = wlo < ntiles ? wlo : ntiles;
  for (; t < lo_; ++t) mid(t);  // tiles before this wave's rows' documents
  if (wlo < whi) {
    slot_p(t, std::true_type{});
    mid(t);
    if (t + 1 == whi) slot_q(t, std::true_type{});
    else slot_q(t, std::false_type{});
    ++t;
    for (; t + 1 < whi; ++t) {  // steady state: no branch but the rare rescale / mask
      slot_p(t, std::false_type{});
      mid(t);
      slot_q(t, std::false_type{});
    }
    if (t < whi) {
      slot_p(t, std::false_type{});
      mid(t);
      slot_q(t, std::true_type{});
      ++t;
    }
  }
  for (; t < ntiles; ++t) mid(t);  // tiles past this wave's causal limit
  fa::mfma_drain();

  // epilogue: O / l, 16-bit, and the log-sum-exp, per sub-block
  auto store = [&](const f32x16 (&o)[DT], float m_i, float l_i, int qrow) {
    if (qrow >= p.sq) return;
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    const float lse_j = l_i > 0.f ? (m_i + __log2f(l_i)) * 0.6931471805599453f : -INFINITY;
    float* lp = p.lse + (int64_t)b * p.lse_sb + (int64_t)head * p.lse_sh + qrow;
    T* O = (T*)p.o + (int64_t)b * p.o_sb + (int64_t)qrow * p.o_ss + (int64_t)head * p.o_sh;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (T)(o[d][4 * rg + e] * inv);
        *reinterpret_cast<x4*>(O + d * 32 + 8 * rg + 4 * h) = w;
      }
    }
    if (h == 0) *lp = lse_j;
  };
  store(oa, ma, la, qrowA);
  store(ob, mbx, lb, qrowB);
}

template <typename T, int HD, int WAVES>
void launch_fwd(const AttnParams& p, hipStream_t s) {
  const int bmw = 32 * WAVES;
  dim3 grid(((p.sq + bmw - 1) / bmw) * p.nq * p.b);
  if (p.causal)
    hipLaunchKernelGGL((fa_fwd_k<T, HD, true, WAVES>), grid, dim3(64 * WAVES), 0, s, p);
  else
    hipLaunchKernelGGL((fa_fwd_k<T, HD, false, WAVES>), grid, dim3(64 * WAVES), 0, s, p);
}

}  // namespace
}  // namespace fa

bool flash_attn_supported(int hd, int dt) {
  return (hd == 64 || hd == 128) && (dt == DT_BF16 || dt == DT_F16);
}

int flash_attn_waves(int b, int sq, int nq, int hd) {
  static const int forced = [] {
    const char* e = getenv("EMA_FA_WAVES");
    return e ? atoi(e) : 0;
  }();
  if (forced == 4 || forced == 8) return forced;
  const long blocks8 = (long)((sq + 255) / 256) * nq * b;
  return (hd == 64 || blocks8 < 512) ? 4 : 8;
}

// Forward v2 (fa_fwd2_k) for head_dim 128 without the ring-attention merge,
// opt-in while it is slower than the 8 / 4-wave kernel (EMA_FA_FWD=2;
// profiles/r7f_fa_v2_ab.txt).
bool fa_fwd_v2(const AttnParams& p) {
  const char* e = getenv("EMA_FA_FWD");  // (read per launch: tests switch it)
  return e && e[0] == '2' && p.hd == 128 && p.o32 == nullptr;
}

void flash_attn_fwd(const AttnParams& p, int dt, hipStream_t s) {
  if (fa_fwd_v2(p)) {
    const dim3 grid(((p.sq + 255) / 256) * p.nq * p.b);
    if (dt == DT_BF16) {
      if (p.causal) hipLaunchKernelGGL((fa::fa_fwd2_k<bf16, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((fa::fa_fwd2_k<bf16, false>), grid, dim3(256), 0, s, p);
    } else {
      if (p.causal) hipLaunchKernelGGL((fa::fa_fwd2_k<fp16, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((fa::fa_fwd2_k<fp16, false>), grid, dim3(256), 0, s, p);
    }
    return;
  }
  const bool w4 = flash_attn_waves(p.b, p.sq, p.nq, p.hd) == 4;
  if (dt == DT_BF16) {
    if (p.hd == 128) w4 ? fa::launch_fwd<bf16, 128, 4>(p, s) : fa::launch_fwd<bf16, 128, 8>(p, s);
    else w4 ? fa::launch_fwd<bf16, 64, 4>(p, s) : fa::launch_fwd<bf16, 64, 8>(p, s);
  } else {
    if (p.hd == 128) w4 ? fa::launch_fwd<fp16, 128, 4>(p, s) : fa::launch_fwd<fp16, 128, 8>(p, s);
    else w4 ? fa::launch_fwd<fp16, 64, 4>(p, s) : fa::launch_fwd<fp16, 64, 8>(p, s);
  }
}

}  // namespace ema
