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

// KV2 (WAVES = 8): the 128 query rows of a 4-wave block on 8 waves, waves
// 4..7 repeating waves 0..3's rows over the second half of the block's key
// tiles; each half keeps its own online softmax and 2-slot ring (every wave
// loads pieces of both halves' tiles), and the halves' (m, l, O) merge through
// LDS at the end.  For grids of at most one 4-wave block per CU (Llama-2-70B's
// 8 heads per TP-8 rank: 256 causal blocks of 1..32 key tiles), where the
// heaviest block sets the kernel time and one wave per SIMD hides no latency.
template <typename T, int HD, bool CAUSAL, int WAVES, bool KV2 = false>
__global__ __launch_bounds__(WAVES * 64, 8 / WAVES) void fa_fwd_k(const AttnParams p) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  static_assert(!KV2 || WAVES == 8, "KV2: two 4-wave halves");
  constexpr int RW = KV2 ? 4 : WAVES;  // waves holding distinct query rows
  constexpr int BMW = RW * 32, KT = 64;
  constexpr int KS = HD / 16, DT = HD / 32;
  constexpr int ROWB = HD * 2, RG = 8 * ROWB, PIECES = KT * ROWB / 1024, PPW = PIECES / WAVES;
  constexpr int TB = KT * ROWB;  // bytes of one K (or V) tile
  constexpr int NB = (WAVES == 8 && !KV2) ? 3 : 2;
  constexpr int NG = KV2 ? 2 : 1;  // key halves, each with its own ring
  static_assert(PIECES % WAVES == 0, "pieces per wave");
  __shared__ __attribute__((aligned(1024))) char lds[NG * NB * 2 * TB];

  const int tid = threadIdx.x;
  unsigned long long st0 = 0, st1 = 0, st2 = 0;
  if (p.stamps) st0 = fa::wall_stamp();
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int grp = KV2 ? (wave >> 2) : 0, rw = KV2 ? (wave & 3) : wave;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nmb = (p.sq + BMW - 1) / BMW;
  const int nhb = p.nq * p.b;
  int lin = blockIdx.x;
  if (CAUSAL && p.pair_ncu > 0 && lin >= p.pair_ncu) lin = 3 * p.pair_ncu - 1 - lin;
  const int mb = CAUSAL ? (nmb - 1 - lin / nhb) : lin / nhb;
  const int hb = lin % nhb;
  const int head = hb % p.nq, b = hb / p.nq;
  const int r = p.nq / p.nkv, g = head / r;
  const int off = p.coff;

  const T* Q = (const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg + (int64_t)(head % r) * p.q_sh;
  const T* K = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg;
  const T* V = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg;

  const int m0 = mb * BMW + rw * 32;
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
  auto prefetch = [&](int t, int slot, int g) {
    char* kl = lds + (g * NB + slot) * 2 * TB;
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
  // this wave's key tiles [gs, ge) over niter barrier-synchronous iterations
  // (KV2: the halves [t0, t0 + half) and [t0 + half, ntiles))
  const int ntot = ntiles > t0 ? ntiles - t0 : 0;
  const int half = KV2 ? (ntot + 1) / 2 : ntot;
  const int niter = half;
  const int gs = t0 + (grp ? half : 0), ge = KV2 && grp == 0 ? t0 + half : ntiles;
  if constexpr (KV2) {
    if (half > 0) prefetch(t0, 0, 0);
    if (t0 + half < ntiles) prefetch(t0 + half, 0, 1);
  } else {
    if (t0 < ntiles) prefetch(t0, t0 % NB, 0);
    if (NB == 3 && t0 + 1 < ntiles) prefetch(t0 + 1, (t0 + 1) % NB, 0);
  }

  x8 qf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) qf[kk] = ld8(Q + (int64_t)qrow_c * p.q_ss + kk * 16 + 8 * h);
  if (p.rope_cos) {
    const float *rc, *rs;
    rope_rows<HD>(p, b, qrow_c, rc, rs);
    rope_rows_fwd<T, KS>(qf, rc, rs, h);  // table loads batched (not one round trip per fragment)
    // (KV2: written back after the merge -- the other half reads these rows now)
    if (!KV2 && qrow < p.sq) {
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

  for (int it = 0; it < niter; ++it) {
    const int t = gs + it;
    // WAR: tile t+NB-1 overwrites the slot of tile t-1, whose reads every wave
    // retired before the barrier that ended tile t-1
    if constexpr (KV2) {
      if (it + 1 < niter) {
        prefetch(t0 + it + 1, (it + 1) & 1, 0);
        if (t0 + half + it + 1 < ntiles) prefetch(t0 + half + it + 1, (it + 1) & 1, 1);
      }
    } else {
      if (t + NB - 1 < ntiles) prefetch(t + NB - 1, (t + NB - 1) % NB, 0);
    }
    if (t < ge && t < wtiles && t >= wt0) {
      const int n0 = t * KT;
      const char* kl = lds + (KV2 ? grp * NB + (it & 1) : t % NB) * 2 * TB;
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

  if constexpr (KV2) {
    // merge the second half's (m, l, O) into the first's (the loop ended on a
    // barrier: the rings are drained); lane-contiguous floats, conflict-free
    float* ml = reinterpret_cast<float*>(lds);
    float* ob = ml + 4 * 2 * 64;
    if (grp == 1) {
      ml[(rw * 2) * 64 + lane] = m_i;
      ml[(rw * 2 + 1) * 64 + lane] = l_i;
#pragma unroll
      for (int d = 0; d < DT; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) ob[((rw * DT + d) * 16 + i) * 64 + lane] = o[d][i];
    }
    __syncthreads();
    if (grp == 0) {
      const float mB = ml[(rw * 2) * 64 + lane], lB = ml[(rw * 2 + 1) * 64 + lane];
      const float m = fmaxf(m_i, mB);
      if (m != -INFINITY) {
        const float aA = __builtin_amdgcn_exp2f(m_i - m), aB = __builtin_amdgcn_exp2f(mB - m);
        l_i = l_i * aA + lB * aB;
#pragma unroll
        for (int d = 0; d < DT; ++d)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[d][i] = o[d][i] * aA + ob[((rw * DT + d) * 16 + i) * 64 + lane] * aB;
        m_i = m;
      }
      if (p.rope_cos && qrow < p.sq) {
        T* Qw = const_cast<T*>(Q) + (int64_t)qrow * p.q_ss + 8 * h;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) *reinterpret_cast<x8*>(Qw + kk * 16) = qf[kk];
      }
    }
  }
  if (p.stamps) st2 = fa::wall_stamp();
  if ((!KV2 || grp == 0) && qrow < p.sq) {
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


template <typename T, int HD, int WAVES, bool KV2 = false>
void launch_fwd(const AttnParams& p0, hipStream_t s) {
  const int bmw = 32 * (KV2 ? 4 : WAVES);
  dim3 grid(((p0.sq + bmw - 1) / bmw) * p0.nq * p0.b);
  AttnParams p = p0;
  p.pair_ncu = KV2 ? 0 : fa_pair_ncu(p.causal, grid.x, WAVES, HD);
  if (p.causal)
    hipLaunchKernelGGL((fa_fwd_k<T, HD, true, WAVES, KV2>), grid, dim3(64 * WAVES), 0, s, p);
  else
    hipLaunchKernelGGL((fa_fwd_k<T, HD, false, WAVES, KV2>), grid, dim3(64 * WAVES), 0, s, p);
}

}  // namespace
}  // namespace fa

namespace {
// an environment default read on first use (function-local static), which a
// setter overrides (tests / A/B in one process)
bool env_on(const char* name) {
  const char* e = getenv(name);
  return !(e && e[0] == '0');
}
int g_fa_pairing_set = -1;  // -1: EMA_FA_PAIR
int g_fa_kv2_set = -1;      // -1: EMA_FA_KV2
bool fa_pairing_on() {
  static const bool env = env_on("EMA_FA_PAIR");
  return g_fa_pairing_set >= 0 ? g_fa_pairing_set != 0 : env;
}
bool fa_kv2_on() {
  static const bool env = env_on("EMA_FA_KV2");
  return g_fa_kv2_set >= 0 ? g_fa_kv2_set != 0 : env;
}
}  // namespace

void fa_set_pairing(bool on) { g_fa_pairing_set = on ? 1 : 0; }

// Causal balance of a fully resident grid (kernels.h AttnParams::pair_ncu).
// Only the 4-wave head_dim-128 blocks run exactly two per CU (64 KiB of LDS
// each); fa_stamps.py showed the pairs (k, k + ncu) on one CU: heavy-first
// order alone gave the 7B TP8 rank (4 heads x 4 x 4096 tokens, 512 blocks)
// CUs that ran query blocks 15 + 31 next to CUs that ran 0 + 16 (CU ends
// 62-119 us).
static int fa_ncu() {
  static const int ncu = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 0;
    return n;
  }();
  return ncu;
}

int fa_pair_ncu(int causal, long grid, int waves, int hd) {
  const int ncu = fa_ncu();
  return (fa_pairing_on() && causal && waves == 4 && hd == 128 && ncu > 0 && grid == 2L * ncu) ? ncu : 0;
}

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

void fa_set_kv2(bool on) { g_fa_kv2_set = on ? 1 : 0; }

// The split-key forward and dQ (fa_fwd_k / fa_bwd_dq2_k KV2) for head_dim-128
// grids of at most one 4-wave block per CU
bool flash_attn_kv2(int b, int sq, int nq, int hd) {
  const long blocks4 = (long)((sq + 127) / 128) * nq * b;
  const int ncu = fa_ncu();
  return fa_kv2_on() && hd == 128 && ncu > 0 && blocks4 <= ncu;
}

void flash_attn_fwd(const AttnParams& p, int dt, hipStream_t s) {
  if (flash_attn_kv2(p.b, p.sq, p.nq, p.hd)) {
    if (dt == DT_BF16) fa::launch_fwd<bf16, 128, 8, true>(p, s);
    else fa::launch_fwd<fp16, 128, 8, true>(p, s);
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
