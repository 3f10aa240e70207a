// FlashAttention-2 backward for gfx950 (MI355X), native GQA/MQA, causal.
//
// Two MFMA kernels after a delta = rowsum(dO * O) pre-pass; neither needs
// atomics or an fp32 workspace:
//
// fa_bwd_dkdv_k -- workgroup = 4 waves = 128 keys of one (batch, KV group);
//   each wave keeps its 32 keys' K and V fragments in registers and
//   accumulates dK^T / dV^T over ALL query heads of the group and all query
//   tiles (GQA reduced inside the workgroup).  Per 32-row query tile (Q, dO
//   double-buffered in LDS, one barrier per tile):
//     S  = Q K^T, P = exp2(S*scale*log2e - LSE*log2e)
//     dP = dO V^T (acc pre-loaded with -delta),  dS = P * (dP - delta)
//     dV^T += dO^T P,  dK^T += Q^T dS   (P / dS accumulators used directly as
//                                        the B operand; dO^T / Q^T via
//                                        ds_read_b64_tr_b16)
// fa_bwd_dq_k -- workgroup = 128 query rows of one head, 64-key tiles of K/V
//   streamed through double-buffered LDS; recomputes S^T / dP^T with the
//   query on the MFMA lane and accumulates dQ^T = K^T dS^T in registers.
//
// The previous single-kernel design added dQ with fp32 atomics from every
// key block (~0.6 GB of atomic traffic per Llama-7B layer backward); the
// recompute costs 3 extra 32x32 MFMA products per tile pair instead.
#include <cstdio>
#include <vector>

#include "fa_common.h"
#include "kernels.h"

namespace ema {
namespace fa {
namespace {

typedef __attribute__((ext_vector_type(4))) float f4;

// Diagnostic-build cycle stamps (EMA_FA_STAMPS=1 launches the STAMP=true
// instantiation; the production kernels contain none).
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define EMA_STAMP(k)                  \
  if constexpr (STAMP) {              \
    const uint64_t now_ = stamp();    \
    seg[k] += now_ - last_;           \
    last_ = now_;                     \
  }

constexpr int BNK = 128;  // keys per dK/dV workgroup
constexpr int BQ = 32;    // query rows per dK/dV step
constexpr int BMQ = 128;  // query rows per dQ workgroup
constexpr int KT = 64;    // keys per dQ step

template <typename T, int HD>
__global__ __launch_bounds__(256) void fa_delta_k(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)p.b * p.nq * p.sq;
  if (t >= total) return;
  const int q = (int)(t % p.sq);
  const int head = (int)((t / p.sq) % p.nq);
  const int b = (int)(t / ((int64_t)p.sq * p.nq));
  const int64_t off = (int64_t)b * p.o_sb + (int64_t)q * p.o_ss + (int64_t)head * p.o_sh;
  const T* o = (const T*)p.o + off;
  const T* d = (const T*)P.dout + off;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < HD; c += 8) {
    const typename MT<T>::x8 a = ld8(o + c);
    const typename MT<T>::x8 g = ld8(d + c);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += (float)a[e] * (float)g[e];
  }
  P.delta[t] = s;
  P.ndelta[t] = -s;
  P.lse2[t] = p.lse[t] * 1.4426950408889634f;
}

template <typename T, int HD, bool CAUSAL, int OCC, bool STAMP = false>
__global__ __launch_bounds__(256, OCC) void fa_bwd_dkdv_k(const AttnBwdParams P) {
  uint64_t seg[6] = {0, 0, 0, 0, 0, 0}, last_ = 0;
  if constexpr (STAMP) last_ = stamp();
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  const AttnParams& p = P.f;
  constexpr int KS = HD / 16, DT = HD / 32, CPR = HD / 8;
  // double-buffered query-tile images (one barrier per step)
  __shared__ __attribute__((aligned(16))) T q_lds[2][BQ * HD];
  __shared__ __attribute__((aligned(16))) T do_lds[2][BQ * HD];
  __shared__ __attribute__((aligned(16))) float lse_lds[2][BQ];
  __shared__ __attribute__((aligned(16))) float dl_lds[2][BQ];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nb = blockIdx.x, g = blockIdx.y, b = blockIdx.z;
  const int r = p.nq / p.nkv;
  const int off = p.sk - p.sq;
  const int kbase = nb * BNK + wave * 32;
  const int key = kbase + c;
  const int key_c = key < p.sk ? key : p.sk - 1;
  const float sl2 = p.scale * 1.4426950408889634f;

  const T* K = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg;
  const T* V = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg;

  // K / V fragments of this wave's 32 keys, register-resident for the whole
  // sweep (B operands of S and dP: B[k = d][col = key])
  x8 kf[KS], vf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    kf[kk] = ld8(K + (int64_t)key_c * p.k_ss + kk * 16 + 8 * h);
    vf[kk] = ld8(V + (int64_t)key_c * p.v_ss + kk * 16 + 8 * h);
  }

  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[d][i] = dv[d][i] = 0.f;

  int q_first = 0;
  if (CAUSAL) {
    q_first = nb * BNK - off;
    q_first = q_first < 0 ? 0 : (q_first / BQ) * BQ;
  }
  constexpr int QCH = 2 * BQ * CPR / 256;  // Q + dO chunks staged per thread

  // Flat (head, query-tile) step loop; the next step's Q / dO / LSE / delta
  // are register-staged while this step computes (CDNA guide T14).
  const int nsteps_q = p.sq > q_first ? (p.sq - q_first + BQ - 1) / BQ : 0;
  const int nsteps = r * nsteps_q;
  x8 qst[QCH];
  float lse_st = 0.f, dl_st = 0.f;
  auto prefetch = [&](int step) {
    const int hh = step / nsteps_q;
    const int q0 = q_first + (step - hh * nsteps_q) * BQ;
    const int head = g * r + hh;
    const T* Q = (const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg + (int64_t)hh * p.q_sh;
    const T* DO = (const T*)P.dout + (int64_t)b * p.o_sb + (int64_t)head * p.o_sh;
#pragma unroll
    for (int i = 0; i < QCH; ++i) {
      const bool is_do = i >= QCH / 2;  // chunks [0, QCH/2): Q, then dO
      const int rem = tid + 256 * (i - (is_do ? QCH / 2 : 0));
      const int row = rem / CPR, ch = rem % CPR;
      int qr = q0 + row;
      qr = qr < p.sq ? qr : p.sq - 1;
      qst[i] = is_do ? ld8(DO + (int64_t)qr * p.o_ss + ch * 8)
                     : ld8(Q + (int64_t)qr * p.q_ss + ch * 8);
    }
    if (tid < BQ) {
      const int qr = q0 + tid;
      const int64_t rb = ((int64_t)b * p.nq + head) * p.sq;
      lse_st = qr < p.sq ? p.lse[rb + qr] * 1.4426950408889634f : 0.f;
      dl_st = qr < p.sq ? P.delta[rb + qr] : 0.f;
    }
  };
  if (nsteps > 0) prefetch(0);

  for (int step = 0; step < nsteps; ++step) {
    EMA_STAMP(0)
    const int hh = step / nsteps_q;
    const int q0 = q_first + (step - hh * nsteps_q) * BQ;
    const int buf = step & 1;
    T* ql = q_lds[buf];
    T* dl = do_lds[buf];
    // buffer `buf` was last read two steps ago; every wave has since passed
    // the previous step's barrier, so it can be overwritten without waiting
#pragma unroll
    for (int i = 0; i < QCH; ++i) {
      const bool is_do = i >= QCH / 2;
      const int rem = tid + 256 * (i - (is_do ? QCH / 2 : 0));
      const int row = rem / CPR, ch = rem % CPR;
      *reinterpret_cast<x8*>((is_do ? dl : ql) + sw_off<HD>(row, ch * 8)) = qst[i];
    }
    if (tid < BQ) {
      lse_lds[buf][tid] = lse_st;
      dl_lds[buf][tid] = dl_st;
    }
    if (step + 1 < nsteps && !(P.ablate & 1)) prefetch(step + 1);
    EMA_STAMP(1)
    __syncthreads();
    EMA_STAMP(2)
    // No early-out for a query tile entirely before this wave's keys (at most
    // 3 per head for waves 1..3): the mask zeroes it, and a skip branch would
    // split the accumulators' live ranges into per-iteration AGPR copies.

    // Every LDS read of the S / dP phase is issued up front (row constants
    // as 16-byte vectors), then the two MFMA chains; the transposed reads of
    // the dV / dK phase do not depend on P and are issued before the softmax
    // VALU so their latency hides behind it (one wave per SIMD: nothing else
    // would cover a per-MFMA LDS wait).
    f4 lse4[4], dl4[4];
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      lse4[rg] = *reinterpret_cast<const f4*>(&lse_lds[buf][8 * rg + 4 * h]);
      dl4[rg] = *reinterpret_cast<const f4*>(&dl_lds[buf][8 * rg + 4 * h]);
    }
    f32x16 sacc, dpacc;
#pragma unroll
    for (int i = 0; i < 16; ++i) dpacc[i] = -dl4[i >> 2][i & 3];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      x8 qa[KS / 2], da[KS / 2];
#pragma unroll
      for (int j = 0; j < KS / 2; ++j) {
        const int col = (half * KS / 2 + j) * 16 + 8 * h;
        qa[j] = *reinterpret_cast<const x8*>(ql + sw_off<HD>(c, col));
        da[j] = *reinterpret_cast<const x8*>(dl + sw_off<HD>(c, col));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < KS / 2; ++j) {
        const int kk = half * KS / 2 + j;
        if (kk == 0) {
          sacc = mfma_vgpr0<T>(qa[0], kf[0]);
          mfma_vgpr<T, 1>(dpacc, da[0], vf[0]);  // C just written by VALU
        } else {
          mfma_vgpr<T>(sacc, qa[j], kf[kk]);
          mfma_vgpr<T>(dpacc, da[j], vf[kk]);
        }
      }
    }
    x8 doa[2][DT], qta[2][DT];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int qrow = 16 * s + 4 * h + tq;
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        const int col = d * 32 + (lane & 16) + 4 * tp;
        doa[s][d] = join<T>(MT<T>::tr_read(dl + sw_off<HD>(qrow, col)),
                            MT<T>::tr_read(dl + sw_off<HD>(qrow + 8, col)));
        qta[s][d] = join<T>(MT<T>::tr_read(ql + sw_off<HD>(qrow, col)),
                            MT<T>::tr_read(ql + sw_off<HD>(qrow + 8, col)));
      }
    }
    mfma_drain();
    EMA_STAMP(3)
    // P and dS (rows = q, col = key)
    const bool need_mask = (q0 + BQ > p.sq) || (kbase + 32 > p.sk) ||
                           (CAUSAL && (kbase + 31 > q0 + off));
#pragma unroll
    for (int i = 0; i < 16; ++i)
      sacc[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[i], sl2, -lse4[i >> 2][i & 3]));
    if (need_mask) {  // wave-uniform; per-element selects, no exec branches
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = q0 + acc_row(i, h);
        const bool ok = (qr < p.sq) & (key < p.sk) & (!CAUSAL | (key <= qr + off));
        sacc[i] = ok ? sacc[i] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) dpacc[i] = sacc[i] * dpacc[i];
    EMA_STAMP(4)
    // dV^T += dO^T P ;  dK^T += Q^T dS
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const x8 pf = acc_frag<T>(sacc, s);
      const x8 sf = acc_frag<T>(dpacc, s);
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        if (d == 0) {  // pf / sf just converted by VALU
          mfma_agpr<T, 1>(dv[d], doa[s][d], pf);
        } else {
          mfma_agpr<T>(dv[d], doa[s][d], pf);
        }
        mfma_agpr<T>(dk[d], qta[s][d], sf);
      }
    }
  }

  if constexpr (STAMP) {
    EMA_STAMP(5)
    if (lane == 0) {
      uint64_t* o = P.stamps + ((((int64_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x +
                                 blockIdx.x) * 4 + wave) * 8;
#pragma unroll
      for (int k = 0; k < 6; ++k) o[k] = seg[k];
      o[6] = nsteps;
    }
  }
  mfma_drain();
  // write dK (scaled) and dV for this wave's 32 keys
  if (key < p.sk) {
    T* DK = (T*)P.dk + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg + (int64_t)key * p.k_ss;
    T* DV = (T*)P.dv + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg + (int64_t)key * p.v_ss;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        x4 wk, wv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          wk[e] = (T)(dk[d][4 * rg + e] * p.scale);
          wv[e] = (T)dv[d][4 * rg + e];
        }
        *reinterpret_cast<x4*>(DK + d * 32 + 8 * rg + 4 * h) = wk;
        *reinterpret_cast<x4*>(DV + d * 32 + 8 * rg + 4 * h) = wv;
      }
    }
  }
}

// dQ = scale * dS K, one workgroup per (128 query rows, query head); loops
// over 64-key tiles (K / V double-buffered in LDS, register-staged one tile
// ahead).  Transposed formulation so the query is the MFMA column (lane):
//   S^T = K Q^T, dP^T = V dO^T   (Q / dO fragments register-resident; the
//                                 lane's LSE / delta are scalars)
//   dQ^T += K^T dS^T             (dS^T accumulator used directly as B operand,
//                                 K^T via ds_read_b64_tr_b16)
// Every dQ element is produced by exactly one lane: no atomics, no fp32
// workspace, and the result is written straight into dq's layout.
template <typename T, int HD, bool CAUSAL, int OCC>
__global__ __launch_bounds__(256, OCC) void fa_bwd_dq_k(const AttnBwdParams P) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  const AttnParams& p = P.f;
  constexpr int KS = HD / 16, DT = HD / 32, CPR = HD / 8;
  constexpr int CH = KT * CPR / 256;  // 16-byte chunks per thread per tile, per tensor
  __shared__ __attribute__((aligned(16))) T k_lds[2][KT * HD];
  __shared__ __attribute__((aligned(16))) T v_lds[2][KT * HD];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nqb = (p.sq + BMQ - 1) / BMQ;
  const int qb = nqb - 1 - (int)blockIdx.x;  // most keys (causal) first
  const int head = blockIdx.y, b = blockIdx.z;
  const int r = p.nq / p.nkv, g = head / r, hh = head - g * r;
  const int off = p.sk - p.sq;
  const int q0w = qb * BMQ + wave * 32;
  const int qrow = q0w + c;
  const int qrow_c = qrow < p.sq ? qrow : p.sq - 1;
  const float sl2 = p.scale * 1.4426950408889634f;

  const T* Q = (const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg + (int64_t)hh * p.q_sh;
  const T* DO = (const T*)P.dout + (int64_t)b * p.o_sb + (int64_t)head * p.o_sh;
  const T* K = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg;
  const T* V = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg;

  // Q / dO as B operands: B[k = d][col = q]
  x8 qf[KS], df[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    qf[kk] = ld8(Q + (int64_t)qrow_c * p.q_ss + kk * 16 + 8 * h);
    df[kk] = ld8(DO + (int64_t)qrow_c * p.o_ss + kk * 16 + 8 * h);
  }
  const int64_t rb = ((int64_t)b * p.nq + head) * p.sq;
  const float lse2 = p.lse[rb + qrow_c] * 1.4426950408889634f;
  const float dlt = P.delta[rb + qrow_c];

  int kend = p.sk;
  if (CAUSAL) {
    const int last = qb * BMQ + BMQ + off;  // one past the block's last visible key
    kend = last < kend ? last : kend;
  }
  const int ntiles = kend > 0 ? (kend + KT - 1) / KT : 0;

  f32x16 dq[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[d][i] = 0.f;

  x8 kst[CH], vst[CH];
  auto prefetch = [&](int t) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / CPR, ch = idx % CPR;
      int kr = t * KT + row;
      kr = kr < p.sk ? kr : p.sk - 1;
      kst[i] = ld8(K + (int64_t)kr * p.k_ss + ch * 8);
      vst[i] = ld8(V + (int64_t)kr * p.v_ss + ch * 8);
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int idx = tid + 256 * i;
      const int row = idx / CPR, ch = idx % CPR;
      *reinterpret_cast<x8*>(k_lds[buf] + sw_off<HD>(row, ch * 8)) = kst[i];
      *reinterpret_cast<x8*>(v_lds[buf] + sw_off<HD>(row, ch * 8)) = vst[i];
    }
  };
  if (ntiles > 0) {
    prefetch(0);
    commit(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles && !(P.ablate & 1)) prefetch(t + 1);
    const T* kl = k_lds[buf];
    const T* vl = v_lds[buf];
#pragma unroll
    for (int sub = 0; sub < KT / 32; ++sub) {
      const int kb = t * KT + sub * 32;
      // no skip of sub-tiles past this wave's causal horizon (<= 3 per
      // workgroup): masked to zero instead, keeping dq's live range unsplit
      f32x16 sacc, dpacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) dpacc[i] = -dlt;
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        x8 ka[KS / 2], va[KS / 2];
#pragma unroll
        for (int j = 0; j < KS / 2; ++j) {
          const int col = (half * KS / 2 + j) * 16 + 8 * h;
          ka[j] = *reinterpret_cast<const x8*>(kl + sw_off<HD>(sub * 32 + c, col));
          va[j] = *reinterpret_cast<const x8*>(vl + sw_off<HD>(sub * 32 + c, col));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < KS / 2; ++j) {
          if (half == 0 && j == 0) {
            sacc = mfma_vgpr0<T>(ka[0], qf[0]);
            mfma_vgpr<T, 1>(dpacc, va[0], df[0]);
          } else {
            mfma_vgpr<T>(sacc, ka[j], qf[half * KS / 2 + j]);
            mfma_vgpr<T>(dpacc, va[j], df[half * KS / 2 + j]);
          }
        }
      }
      // K^T operands of the dQ product, issued ahead of the softmax VALU
      x8 kt[2][DT];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int krow = sub * 32 + 16 * s + 4 * h + tq;
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          const int col = d * 32 + (lane & 16) + 4 * tp;
          kt[s][d] = join<T>(MT<T>::tr_read(kl + sw_off<HD>(krow, col)),
                             MT<T>::tr_read(kl + sw_off<HD>(krow + 8, col)));
        }
      }
      mfma_drain();
      const bool need_mask = (kb + 32 > p.sk) || (q0w + 32 > p.sq) ||
                             (CAUSAL && kb + 31 > q0w + off);
#pragma unroll
      for (int i = 0; i < 16; ++i)
        sacc[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[i], sl2, -lse2));
      if (need_mask) {  // wave-uniform; per-element selects, no exec branches
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int kr = kb + acc_row(i, h);
          const bool ok = (kr < p.sk) & (qrow < p.sq) & (!CAUSAL | (kr <= qrow + off));
          sacc[i] = ok ? sacc[i] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) sacc[i] = sacc[i] * dpacc[i];  // dS^T [key][q]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const x8 sf = acc_frag<T>(sacc, s);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          if (d == 0) mfma_agpr<T, 1>(dq[d], kt[s][d], sf);  // sf just converted
          else mfma_agpr<T>(dq[d], kt[s][d], sf);
        }
      }
    }
    if (t + 1 < ntiles) commit(buf ^ 1);
    __syncthreads();
  }

  mfma_drain();
  if (qrow < p.sq) {
    T* DQ = (T*)P.dq + (int64_t)b * p.q_sb + (int64_t)qrow * p.q_ss + (int64_t)g * p.q_sg +
            (int64_t)hh * p.q_sh;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (T)(dq[d][4 * rg + e] * p.scale);
        *reinterpret_cast<x4*>(DQ + d * 32 + 8 * rg + 4 * h) = w;
      }
    }
  }
}

// dK/dV, v2: the same per-wave math as fa_bwd_dkdv_k (4 waves x 32 keys, K/V
// fragments and dK^T/dV^T accumulators register-resident), but each step
// covers 64 query rows (two 32-row sub-slices: half the barriers per unit of
// work) and the Q / dO / LSE / delta tiles arrive by LDS-DMA into a 2-deep
// ring (issued one step ahead; the lane-linear image takes the sw_off swizzle
// through the per-lane SOURCE address) — no staging registers and no
// ds_write pass, which together cost more than the step's MFMAs in the
// round-1 kernel (profiles/r1_fa_bwd_split.txt).  Transposed reads are inline
// asm so hipcc does not drain the in-flight DMA in front of them.
constexpr int BQ2 = 64;

template <typename T, int HD, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv2_k(const AttnBwdParams P) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  const AttnParams& p = P.f;
  constexpr int KS = HD / 16, DT = HD / 32;
  constexpr int ROWB = HD * 2;                   // bytes per Q / dO row
  constexpr int RG = 8 * ROWB;                   // bytes per 8-row group (image (a))
  constexpr int TILEB = BQ2 * ROWB;              // one Q (or dO) tile
  constexpr int BUFB = 2 * TILEB + 2 * BQ2 * 4;  // Q, dO, lse2, -delta
  constexpr int PIECES = TILEB / 1024, PPW = PIECES / 4;
  static_assert(PIECES % 4 == 0, "pieces per wave");
  __shared__ __attribute__((aligned(1024))) char lds[2 * BUFB];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3, l4 = (lane >> 4) & 1;
  // blockIdx.y = KV group * kv_split + split: split takes query heads
  // [split * r_per, (split + 1) * r_per) of the group
  const int S = P.kv_split > 1 ? P.kv_split : 1;
  const int nb = blockIdx.x, g = blockIdx.y / S, split = blockIdx.y % S, b = blockIdx.z;
  const int r = p.nq / p.nkv, r_per = r / S, h0 = split * r_per;
  const int off = p.sk - p.sq;
  const int kbase = nb * BNK + wave * 32;
  const int key = kbase + c;
  const int key_c = key < p.sk ? key : p.sk - 1;
  const float sl2 = p.scale * 1.4426950408889634f;

  const T* K = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg;
  const T* V = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg;

  int q_first = 0;
  if (CAUSAL) {
    q_first = nb * BNK - off;
    q_first = q_first < 0 ? 0 : (q_first / BQ2) * BQ2;
  }
  const int nsteps_q = p.sq > q_first ? (p.sq - q_first + BQ2 - 1) / BQ2 : 0;
  const int nsteps = r_per * nsteps_q;

  // LDS-DMA source offsets of this lane's pieces (image (a) through the source)
  int srow[PPW], schunk[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int o = (wave * PPW + i) * 1024 + 16 * lane;
    const int rem = o % RG, rem2 = rem % 512;
    srow[i] = 8 * (o / RG) + rem2 / 64;
    schunk[i] = 4 * (rem / 512) + (((rem2 % 64) / 16) ^ ((srow[i] >> 2) & 3));
  }
  auto prefetch = [&](int step, int buf) {
    const int hl = step / nsteps_q, hh = h0 + hl;
    const int q0 = q_first + (step - hl * nsteps_q) * BQ2;
    const int head = g * r + hh;
    const T* Q = (const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg + (int64_t)hh * p.q_sh;
    const T* DO = (const T*)P.dout + (int64_t)b * p.o_sb + (int64_t)head * p.o_sh;
    char* base = lds + buf * BUFB;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;
      int qr = q0 + srow[i];
      qr = qr < p.sq ? qr : p.sq - 1;
      __builtin_amdgcn_global_load_lds((const void*)(Q + (int64_t)qr * p.q_ss + schunk[i] * 8),
                                       (__attribute__((address_space(3))) void*)(base + pc * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (const void*)(DO + (int64_t)qr * p.o_ss + schunk[i] * 8),
          (__attribute__((address_space(3))) void*)(base + TILEB + pc * 1024), 16, 0, 0);
    }
    if (wave < 2) {  // 64 rows x 4 B: one dword-wide piece each for lse2 and -delta
      int qr = q0 + lane;
      qr = qr < p.sq ? qr : p.sq - 1;
      const int64_t rb = ((int64_t)b * p.nq + head) * p.sq;
      const float* src = wave == 0 ? P.lse2 + rb + qr : P.ndelta + rb + qr;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(base + 2 * TILEB + wave * BQ2 * 4), 4, 0, 0);
    }
  };
  if (nsteps > 0) prefetch(0, 0);

  // loop-invariant LDS read offsets (the rest are immediates)
  int rowb[2], trb[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    rowb[x] = RG * (c >> 3) + 64 * (c & 7) + 16 * ((2 * x + h) ^ ((c >> 2) & 3));
    trb[x] = RG * x + 64 * (4 * h + tq) + 16 * ((2 * l4 + (tp >> 1)) ^ ((h + 2 * x) & 3)) +
             8 * (tp & 1);
  }
  const int cstb = 2 * TILEB + 4 * (4 * h);

  x8 kf[KS], vf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    kf[kk] = ld8(K + (int64_t)key_c * p.k_ss + kk * 16 + 8 * h);
    vf[kk] = ld8(V + (int64_t)key_c * p.v_ss + kk * 16 + 8 * h);
  }
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) dk[d][i] = dv[d][i] = 0.f;
  __syncthreads();  // vmcnt(0) + barrier: step 0 landed

  for (int step = 0; step < nsteps; ++step) {
    const int hs = step / nsteps_q;
    const int q0 = q_first + (step - hs * nsteps_q) * BQ2;
    const int buf = step & 1;
    if (step + 1 < nsteps) prefetch(step + 1, buf ^ 1);
    const char* bb = lds + buf * BUFB;
    const uint32_t trv0 = (uint32_t)(uintptr_t)(bb + trb[0]);
    const uint32_t trv1 = (uint32_t)(uintptr_t)(bb + trb[1]);
    static_for<BQ2 / 32>([&](auto s2c) {
      constexpr int s2 = decltype(s2c)::value;
      const char* qb = bb + s2 * 4 * RG;  // 32 rows = 4 row groups
      const float* cst = reinterpret_cast<const float*>(bb + cstb) + 32 * s2;
      const int q0s = q0 + 32 * s2;
      f4 l24[4], nd4[4];
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        l24[rg] = *reinterpret_cast<const f4*>(cst + 8 * rg);
        nd4[rg] = *reinterpret_cast<const f4*>(cst + BQ2 + 8 * rg);
      }
      // dP accumulator starts at -delta (row constant): dS = P * (dP - delta)
      f32x16 dpacc = __builtin_shufflevector(__builtin_shufflevector(nd4[0], nd4[1], 0, 1, 2, 3, 4, 5, 6, 7),
                                             __builtin_shufflevector(nd4[2], nd4[3], 0, 1, 2, 3, 4, 5, 6, 7),
                                             0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
      f32x16 sacc;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const int o = rowb[kk & 1] + 512 * (kk >> 1);
        const x8 qa = *reinterpret_cast<const x8*>(qb + o);
        const x8 da = *reinterpret_cast<const x8*>(qb + TILEB + o);
        if (kk == 0) {
          sacc = mfma_vgpr0<T>(qa, kf[0]);
          mfma_vgpr<T, 1>(dpacc, da, vf[0]);
        } else {
          mfma_vgpr<T>(sacc, qa, kf[kk]);
          mfma_vgpr<T>(dpacc, da, vf[kk]);
        }
      }
      x4 doa[2][DT][2], qta[2][DT][2];
      static_for<2>([&](auto sc) {
        static_for<DT>([&](auto dc) {
          constexpr int o = s2 * 4 * RG + decltype(sc)::value * 2 * RG + 512 * decltype(dc)::value;
          doa[sc][dc][0] = tr_read_imm<TILEB + o, T>(trv0);
          doa[sc][dc][1] = tr_read_imm<TILEB + o, T>(trv1);
          qta[sc][dc][0] = tr_read_imm<o, T>(trv0);
          qta[sc][dc][1] = tr_read_imm<o, T>(trv1);
        });
      });
      mfma_drain();
      const bool need_mask = (q0s + 32 > p.sq) || (kbase + 32 > p.sk) ||
                             (CAUSAL && (kbase + 31 > q0s + off));
#pragma unroll
      for (int i = 0; i < 16; ++i)
        sacc[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[i], sl2, -l24[i >> 2][i & 3]));
      if (need_mask) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qr = q0s + acc_row(i, h);
          const bool ok = (qr < p.sq) & (key < p.sk) & (!CAUSAL | (key <= qr + off));
          sacc[i] = ok ? sacc[i] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) dpacc[i] = sacc[i] * dpacc[i];
      lds_wait();  // the asm transposed reads above
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const x8 pf = acc_frag<T>(sacc, s);
        const x8 sf = acc_frag<T>(dpacc, s);
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          if (d == 0) mfma_agpr<T, 1>(dv[d], join<T>(doa[s][d][0], doa[s][d][1]), pf);
          else mfma_agpr<T>(dv[d], join<T>(doa[s][d][0], doa[s][d][1]), pf);
          mfma_agpr<T>(dk[d], join<T>(qta[s][d][0], qta[s][d][1]), sf);
        }
      }
    });
    __syncthreads();  // vmcnt(0) + barrier: step+1 landed, this step's reads retired
  }

  mfma_drain();
  if (S > 1) {  // fp32 partial sums; fa_dkv_reduce_k adds the splits in order
    if (key < p.sk) {
      float* W = P.dkv_ws + ((((int64_t)split * p.b + b) * p.nkv + g) * p.sk + key) * 2 * HD;
#pragma unroll
      for (int d = 0; d < DT; ++d)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          f4 wk, wv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            wk[e] = dk[d][4 * rg + e];
            wv[e] = dv[d][4 * rg + e];
          }
          *reinterpret_cast<f4*>(W + d * 32 + 8 * rg + 4 * h) = wk;
          *reinterpret_cast<f4*>(W + HD + d * 32 + 8 * rg + 4 * h) = wv;
        }
    }
    return;
  }
  if (key < p.sk) {
    T* DK = (T*)P.dk + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg + (int64_t)key * p.k_ss;
    T* DV = (T*)P.dv + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg + (int64_t)key * p.v_ss;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        x4 wk, wv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          wk[e] = (T)(dk[d][4 * rg + e] * p.scale);
          wv[e] = (T)dv[d][4 * rg + e];
        }
        *reinterpret_cast<x4*>(DK + d * 32 + 8 * rg + 4 * h) = wk;
        *reinterpret_cast<x4*>(DV + d * 32 + 8 * rg + 4 * h) = wv;
      }
    }
  }
}

// dK = scale * sum_s dK_s, dV = sum_s dV_s over the kv_split partial sums of
// fa_bwd_dkdv2_k (fixed order: deterministic).  One thread = 4 elements.
template <typename T, int HD>
__global__ __launch_bounds__(256) void fa_dkv_reduce_k(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  const int64_t per = (int64_t)p.b * p.nkv * p.sk * (2 * HD / 4);
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= per) return;
  const int c4 = (int)(t % (2 * HD / 4));
  const int64_t row = t / (2 * HD / 4);  // (b, g, key)
  const int key = (int)(row % p.sk), g = (int)((row / p.sk) % p.nkv), b = (int)(row / ((int64_t)p.sk * p.nkv));
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < P.kv_split; ++s)
    acc += *reinterpret_cast<const f4*>(P.dkv_ws + ((int64_t)s * per + t) * 4);
  const bool is_v = c4 * 4 >= HD;
  const int col = c4 * 4 - (is_v ? HD : 0);
  typename MT<T>::x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (T)(is_v ? acc[e] : acc[e] * p.scale);
  T* dst = is_v ? (T*)P.dv + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg + (int64_t)key * p.v_ss
                : (T*)P.dk + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg + (int64_t)key * p.k_ss;
  *reinterpret_cast<typename MT<T>::x4*>(dst + col) = o;
}

// dQ, v2: WAVES x 32 query rows of one head per workgroup (WAVES = 8: 512
// threads sharing every K/V tile; two waves per SIMD), K/V double-buffered in
// LDS with ONE barrier per 64-key tile (next tile's loads issued before the
// MFMAs, written to the other buffer after them), flat grid with the query
// blocks holding the most keys (causal) dispatched first.  Same math as
// fa_bwd_dq_k.
template <typename T, int HD, bool CAUSAL, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 8 / WAVES) void fa_bwd_dq2_k(const AttnBwdParams P) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  const AttnParams& p = P.f;
  constexpr int NT = WAVES * 64, BMW = WAVES * 32;
  constexpr int KS = HD / 16, DT = HD / 32, CPR = HD / 8;
  __shared__ __attribute__((aligned(16))) T lds[2 * 2 * KT * HD];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nqb = (p.sq + BMW - 1) / BMW;
  const int nhb = p.nq * p.b;
  const int lin = blockIdx.x;
  const int qb = CAUSAL ? (nqb - 1 - lin / nhb) : lin / nhb;
  const int head = (lin % nhb) % p.nq, b = (lin % nhb) / p.nq;
  const int r = p.nq / p.nkv, g = head / r, hh = head - g * r;
  const int off = p.sk - p.sq;
  const int q0w = qb * BMW + wave * 32;
  const int qrow = q0w + c;
  const int qrow_c = qrow < p.sq ? qrow : p.sq - 1;
  const float sl2 = p.scale * 1.4426950408889634f;

  const T* Q = (const T*)p.q + (int64_t)b * p.q_sb + (int64_t)g * p.q_sg + (int64_t)hh * p.q_sh;
  const T* DO = (const T*)P.dout + (int64_t)b * p.o_sb + (int64_t)head * p.o_sh;
  const T* K = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg;
  const T* V = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg;

  int kend = p.sk;
  if (CAUSAL) {
    const int last = qb * BMW + BMW + off;
    kend = last < kend ? last : kend;
  }
  const int ntiles = kend > 0 ? (kend + KT - 1) / KT : 0;
  int wtiles = ntiles;  // this wave's causal horizon
  if (CAUSAL) {
    const int wl = q0w + 32 + off;
    const int wt = wl > 0 ? (wl + KT - 1) / KT : 0;
    wtiles = wt < ntiles ? wt : ntiles;
  }

  // K / V tiles arrive by LDS-DMA (global_load_lds_dwordx4: lane-linear LDS
  // image; the image-(a) layout (ia_off) is produced through the per-lane
  // SOURCE address): no staging registers, no ds_write pass.  One 1-KiB
  // piece per wave-instruction.  All LDS reads are base VGPR + immediate.
  constexpr int ROWB = HD * 2, RG = 8 * ROWB, PIECES = KT * ROWB / 1024, PPW = PIECES / WAVES;
  static_assert(PIECES % WAVES == 0, "pieces per wave");
  int srow[PPW], schunk[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int o = (wave * PPW + i) * 1024 + 16 * lane;
    const int rem = o % RG, rem2 = rem % 512;
    srow[i] = 8 * (o / RG) + rem2 / 64;
    schunk[i] = 4 * (rem / 512) + (((rem2 % 64) / 16) ^ ((srow[i] >> 2) & 3));
  }
  auto prefetch = [&](int t, int buf) {
    char* kl = reinterpret_cast<char*>(lds + buf * 2 * KT * HD);
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = wave * PPW + i;
      const int row = srow[i], chunk = schunk[i];
      int kr = t * KT + row;
      kr = kr < p.sk ? kr : p.sk - 1;
      __builtin_amdgcn_global_load_lds(
          (const void*)(K + (int64_t)kr * p.k_ss + chunk * 8),
          (__attribute__((address_space(3))) void*)(kl + pc * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds(
          (const void*)(V + (int64_t)kr * p.v_ss + chunk * 8),
          (__attribute__((address_space(3))) void*)(kl + KT * ROWB + pc * 1024), 16, 0, 0);
    }
  };
  if (ntiles > 0) prefetch(0, 0);

  x8 qf[KS], df[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    qf[kk] = ld8(Q + (int64_t)qrow_c * p.q_ss + kk * 16 + 8 * h);
    df[kk] = ld8(DO + (int64_t)qrow_c * p.o_ss + kk * 16 + 8 * h);
  }
  const int64_t rb = ((int64_t)b * p.nq + head) * p.sq;
  const float lse2 = p.lse[rb + qrow_c] * 1.4426950408889634f;
  const float dlt = P.delta[rb + qrow_c];

  f32x16 dq[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[d][i] = 0.f;

  int rowb[2], trb[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    rowb[x] = RG * (c >> 3) + 64 * (c & 7) + 16 * ((2 * x + h) ^ ((c >> 2) & 3));
    trb[x] = RG * x + 64 * (4 * h + tq) + 16 * ((2 * ((lane >> 4) & 1) + (tp >> 1)) ^ ((h + 2 * x) & 3)) +
             8 * (tp & 1);
  }
  __syncthreads();  // vmcnt(0) + barrier: tile 0 landed

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1;
    if (t + 1 < ntiles) prefetch(t + 1, buf ^ 1);
    const char* kl = reinterpret_cast<const char*>(lds + buf * 2 * KT * HD);
    const char* vl = kl + KT * ROWB;
    const uint32_t trv0 = (uint32_t)(uintptr_t)(kl + trb[0]);
    const uint32_t trv1 = (uint32_t)(uintptr_t)(kl + trb[1]);
    if (t < wtiles) {
      static_for<KT / 32>([&](auto subc) {
        constexpr int sub = decltype(subc)::value;
        const int kb = t * KT + sub * 32;
        f32x16 sacc, dpacc;
#pragma unroll
        for (int i = 0; i < 16; ++i) dpacc[i] = -dlt;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int o = sub * 4 * RG + rowb[kk & 1] + 512 * (kk >> 1);
          const x8 ka = *reinterpret_cast<const x8*>(kl + o);
          const x8 va = *reinterpret_cast<const x8*>(vl + o);
          if (kk == 0) {
            sacc = mfma_vgpr0<T>(ka, qf[0]);
            mfma_vgpr<T, 1>(dpacc, va, df[0]);
          } else {
            mfma_vgpr<T>(sacc, ka, qf[kk]);
            mfma_vgpr<T>(dpacc, va, df[kk]);
          }
        }
        mfma_drain();
        const bool need_mask = (kb + 32 > p.sk) || (q0w + 32 > p.sq) ||
                               (CAUSAL && kb + 31 > q0w + off);
#pragma unroll
        for (int i = 0; i < 16; ++i)
          sacc[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[i], sl2, -lse2));
        if (need_mask) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int kr = kb + acc_row(i, h);
            const bool ok = (kr < p.sk) & (qrow < p.sq) & (!CAUSAL | (kr <= qrow + off));
            sacc[i] = ok ? sacc[i] : 0.f;
          }
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = sacc[i] * dpacc[i];
        static_for<2>([&](auto sc) {
          const x8 sf = acc_frag<T>(sacc, decltype(sc)::value);
          static_for<DT>([&](auto dc) {
            constexpr int o = sub * 4 * RG + decltype(sc)::value * 2 * RG + 512 * decltype(dc)::value;
            const typename MT<T>::x4 k0 = tr_read_imm<o, T>(trv0);
            const typename MT<T>::x4 k1 = tr_read_imm<o, T>(trv1);
            lds_wait();
            mfma_vgpr<T, 1>(dq[dc], join<T>(k0, k1), sf);
          });
        });
      });
    }
    __syncthreads();  // vmcnt(0) + barrier: tile t+1 landed, tile t's reads retired
  }

  mfma_drain();
  if (qrow < p.sq) {
    T* DQ = (T*)P.dq + (int64_t)b * p.q_sb + (int64_t)qrow * p.q_ss + (int64_t)g * p.q_sg +
            (int64_t)hh * p.q_sh;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (T)(dq[d][4 * rg + e] * p.scale);
        *reinterpret_cast<x4*>(DQ + d * 32 + 8 * rg + 4 * h) = w;
      }
    }
  }
}

bool stamps_on() {
  static const bool on = getenv("EMA_FA_STAMPS") != nullptr;
  return on;
}

template <typename T, int HD>
void launch_bwd(const AttnBwdParams& P0, hipStream_t s) {
  static const int ablate = [] {
    const char* e = getenv("EMA_FA_ABLATE");
    return e ? atoi(e) : 0;
  }();
  AttnBwdParams P = P0;
  P.ablate = ablate;
  const AttnParams& p = P.f;
  const int64_t rows = (int64_t)p.b * p.nq * p.sq;
  hipLaunchKernelGGL((fa_delta_k<T, HD>), dim3((rows + 255) / 256), dim3(256), 0, s, P);
  // dK/dV kernel: EMA_FA_DKDV = 1 (round-1 kernel) or 2 (64-row steps, LDS-DMA, default)
  static const int kvv = [] {
    const char* e = getenv("EMA_FA_DKDV");
    return e ? atoi(e) : 2;
  }();
  if (kvv != 2 || stamps_on()) P.kv_split = 1;  // only the v2 kernel splits query heads
  const dim3 gkv((p.sk + BNK - 1) / BNK, p.nkv * (P.kv_split > 1 ? P.kv_split : 1), p.b);
  const dim3 gq((p.sq + BMQ - 1) / BMQ, p.nq, p.b);
  // occupancy variants (waves/SIMD) for tuning: EMA_FA_BWD_OCC = "<dkdv><dq>", default "11"
  static const int occ = [] {
    const char* e = getenv("EMA_FA_BWD_OCC");
    return e ? atoi(e) : 11;
  }();
  const bool kv2 = occ / 10 == 2, q2 = occ % 10 == 2;
  const int64_t kvred = (int64_t)p.b * p.nkv * p.sk * (2 * HD / 4);
  // dQ kernel: EMA_FA_DQ = 1 (round-1 4-wave kernel) or 8 (8-wave, default)
  static const int dqv = [] {
    const char* e = getenv("EMA_FA_DQ");
    return e ? atoi(e) : 8;
  }();
  const dim3 gq2(((p.sq + 255) / 256) * p.nq * p.b);
#define EMA_FA_BWD(C)                                                                     \
  {                                                                                       \
    if (kvv == 2) {                                                                       \
      hipLaunchKernelGGL((fa_bwd_dkdv2_k<T, HD, C>), gkv, dim3(256), 0, s, P);            \
      if (P.kv_split > 1)                                                                 \
        hipLaunchKernelGGL((fa_dkv_reduce_k<T, HD>), dim3((unsigned)((kvred + 255) / 256)), \
                           dim3(256), 0, s, P);                                           \
    }                                                                                     \
    else if (kv2) hipLaunchKernelGGL((fa_bwd_dkdv_k<T, HD, C, 2>), gkv, dim3(256), 0, s, P); \
    else hipLaunchKernelGGL((fa_bwd_dkdv_k<T, HD, C, 1>), gkv, dim3(256), 0, s, P);       \
    if (dqv == 8) hipLaunchKernelGGL((fa_bwd_dq2_k<T, HD, C, 8>), gq2, dim3(512), 0, s, P); \
    else if (q2) hipLaunchKernelGGL((fa_bwd_dq_k<T, HD, C, 2>), gq, dim3(256), 0, s, P);  \
    else hipLaunchKernelGGL((fa_bwd_dq_k<T, HD, C, 1>), gq, dim3(256), 0, s, P);          \
  }
  const bool stamps = stamps_on();
  if (stamps && p.causal) {  // diagnostic: per-segment cycle shares of the dK/dV loop
    const size_t nw = (size_t)gkv.x * gkv.y * gkv.z * 4;
    uint64_t* d = nullptr;
    (void)hipMalloc(&d, nw * 8 * sizeof(uint64_t));
    (void)hipMemsetAsync(d, 0, nw * 8 * sizeof(uint64_t), s);
    P.stamps = d;
    hipLaunchKernelGGL((fa_bwd_dkdv_k<T, HD, true, 1, true>), gkv, dim3(256), 0, s, P);
    std::vector<uint64_t> h(nw * 8);
    (void)hipMemcpyAsync(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    (void)hipFree(d);
    double tot[6] = {0, 0, 0, 0, 0, 0}, steps = 0;
    for (size_t w = 0; w < nw; ++w) {
      for (int k = 0; k < 6; ++k) tot[k] += (double)h[w * 8 + k];
      steps += (double)h[w * 8 + 6];
    }
    fprintf(stderr, "[fa_bwd_dkdv stamps] cycles/step: dVdK-issue %.0f  write+prefetch %.0f  "
            "barrier %.0f  S,dP+reads %.0f  softmax %.0f  tail %.0f\n", tot[0] / steps,
            tot[1] / steps, tot[2] / steps, tot[3] / steps, tot[4] / steps, tot[5] / steps);
    hipLaunchKernelGGL((fa_bwd_dq_k<T, HD, true, 1>), gq, dim3(256), 0, s, P);
    return;
  }
  if (p.causal) EMA_FA_BWD(true) else EMA_FA_BWD(false)
#undef EMA_FA_BWD
}

}  // namespace
}  // namespace fa

void flash_attn_bwd(const AttnBwdParams& p, int dt, hipStream_t s) {
  if (dt == DT_BF16) {
    if (p.f.hd == 128) fa::launch_bwd<bf16, 128>(p, s);
    else fa::launch_bwd<bf16, 64>(p, s);
  } else {
    if (p.f.hd == 128) fa::launch_bwd<fp16, 128>(p, s);
    else fa::launch_bwd<fp16, 64>(p, s);
  }
}

}  // namespace ema
