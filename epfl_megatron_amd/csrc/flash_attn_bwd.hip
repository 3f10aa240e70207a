// FlashAttention-2 backward for gfx950 (MI355X), native GQA/MQA, causal.
//
// Workgroup = 4 waves = 128 keys of one (batch, KV group); each wave keeps its
// 32 keys' K and V fragments in registers and accumulates dK^T / dV^T for
// them over ALL query heads of the group and all query tiles, so dK and dV
// need no cross-workgroup reduction (GQA handled natively: the r = nq/nkv
// query heads of a group are summed inside the workgroup).
//
// Per 32-row query tile (Q, dO staged in LDS, shared by the 4 waves):
//   S  = Q K^T        (acc pre-loaded with -LSE/scale => P = exp2(S * scale*log2e))
//   dP = dO V^T       (acc pre-loaded with -delta    => dP - delta)
//   dS = P * (dP - delta)
//   dV^T += dO^T P,  dK^T += Q^T dS   (P / dS accumulators used directly as
//                                      the B operand; dO^T / Q^T via
//                                      ds_read_b64_tr_b16 from one LDS image)
//   dQ  += dS K      (dS^T staged through LDS once; each wave owns a 32-wide
//                     d slice; fp32 atomics in two 128-B rows per instruction,
//                     the full-rate shape on MI355X)
// Key on the MFMA lane everywhere (CDNA guide, attention backward).
// Pre-pass: delta = rowsum(dO * O); post-pass: dQ = scale * dq_acc -> dtype.
#include "fa_common.h"
#include "kernels.h"

namespace ema {
namespace fa {
namespace {

constexpr int BNK = 128;  // keys per workgroup
constexpr int BQ = 32;    // query rows per step

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
}

template <typename T, int HD, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fa_bwd_k(const AttnBwdParams P) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  const AttnParams& p = P.f;
  constexpr int KS = HD / 16, DT = HD / 32, CPR = HD / 8;
  __shared__ __attribute__((aligned(16))) T q_lds[BQ * HD];
  __shared__ __attribute__((aligned(16))) T do_lds[BQ * HD];
  __shared__ __attribute__((aligned(16))) T k_lds[BNK * HD];
  __shared__ __attribute__((aligned(16))) T ds_lds[BNK * BQ];  // dS^T [key][q]
  __shared__ float lse_lds[BQ];
  __shared__ float dl_lds[BQ];

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
  const float inv_scale = 1.f / p.scale;

  const T* K = (const T*)p.k + (int64_t)b * p.k_sb + (int64_t)g * p.k_sg;
  const T* V = (const T*)p.v + (int64_t)b * p.v_sb + (int64_t)g * p.v_sg;

  // K / V fragments as B operands: B[k = d][col = key]
  x8 kf[KS], vf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    kf[kk] = ld8(K + (int64_t)key_c * p.k_ss + kk * 16 + 8 * h);
    vf[kk] = ld8(V + (int64_t)key_c * p.v_ss + kk * 16 + 8 * h);
  }
  // whole 128-key K tile in LDS (B operand of dQ = dS K via transposed reads)
#pragma unroll
  for (int i = 0; i < BNK * CPR / 256; ++i) {
    const int idx = tid + 256 * i;
    const int row = idx / CPR, ch = idx % CPR;
    int kr = nb * BNK + row;
    kr = kr < p.sk ? kr : p.sk - 1;
    *reinterpret_cast<x8*>(k_lds + sw_off<HD>(row, ch * 8)) =
        ld8(K + (int64_t)kr * p.k_ss + ch * 8);
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

  // Flat (head, query-tile) step loop.  The next step's Q / dO / LSE / delta
  // are register-staged (issued right after this step's LDS image is written)
  // so their HBM latency hides behind this step's 40 MFMAs instead of
  // stalling the single wave per SIMD every step (CDNA guide T14).
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
      lse_st = qr < p.sq ? p.lse[rb + qr] : 0.f;
      dl_st = qr < p.sq ? P.delta[rb + qr] : 0.f;
    }
  };
  if (nsteps > 0) prefetch(0);

  for (int step = 0; step < nsteps; ++step) {
    const int hh = step / nsteps_q;
    const int q0 = q_first + (step - hh * nsteps_q) * BQ;
    const int head = g * r + hh;
    float* DQ = P.dq_acc + ((int64_t)b * p.nq + head) * (int64_t)p.sq * HD;
    {
      __syncthreads();  // previous step finished reading LDS
#pragma unroll
      for (int i = 0; i < QCH; ++i) {
        const bool is_do = i >= QCH / 2;
        const int rem = tid + 256 * (i - (is_do ? QCH / 2 : 0));
        const int row = rem / CPR, ch = rem % CPR;
        *reinterpret_cast<x8*>((is_do ? do_lds : q_lds) + sw_off<HD>(row, ch * 8)) = qst[i];
      }
      if (tid < BQ) {
        lse_lds[tid] = lse_st;
        dl_lds[tid] = dl_st;
      }
      if (step + 1 < nsteps) prefetch(step + 1);
      __syncthreads();

      f32x16 sacc, dpacc;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qr = acc_row(i, h);
        sacc[i] = -lse_lds[qr] * inv_scale;
        dpacc[i] = -dl_lds[qr];
      }
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const x8 qa = *reinterpret_cast<const x8*>(q_lds + sw_off<HD>(c, kk * 16 + 8 * h));
        const x8 da = *reinterpret_cast<const x8*>(do_lds + sw_off<HD>(c, kk * 16 + 8 * h));
        sacc = MT<T>::mfma(qa, kf[kk], sacc);
        dpacc = MT<T>::mfma(da, vf[kk], dpacc);
      }
      // P and dS (rows = q, col = key)
      const bool need_mask = (q0 + BQ > p.sq) || (kbase + 32 > p.sk) ||
                             (CAUSAL && (kbase + 31 > q0 + off));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float pv = exp2f(sacc[i] * sl2);
        if (need_mask) {
          const int qr = q0 + acc_row(i, h);
          bool ok = (qr < p.sq) && (key < p.sk);
          if (CAUSAL) ok = ok && (key <= qr + off);
          if (!ok) pv = 0.f;
        }
        sacc[i] = pv;
        dpacc[i] = pv * dpacc[i];
      }
      // dV^T += dO^T P ;  dK^T += Q^T dS
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const x8 pf = acc_frag<T>(sacc, s);
        const x8 sf = acc_frag<T>(dpacc, s);
        const int qrow = 16 * s + 4 * h + tq;
#pragma unroll
        for (int d = 0; d < DT; ++d) {
          const int col = d * 32 + (lane & 16) + 4 * tp;
          const x8 doa = join<T>(MT<T>::tr_read(do_lds + sw_off<HD>(qrow, col)),
                                 MT<T>::tr_read(do_lds + sw_off<HD>(qrow + 8, col)));
          dv[d] = MT<T>::mfma(doa, pf, dv[d]);
          const x8 qa = join<T>(MT<T>::tr_read(q_lds + sw_off<HD>(qrow, col)),
                                MT<T>::tr_read(q_lds + sw_off<HD>(qrow + 8, col)));
          dk[d] = MT<T>::mfma(qa, sf, dk[d]);
        }
      }
      // stage dS^T [key][q] (bf16) for the dQ product
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (T)dpacc[4 * rg + e];
        *reinterpret_cast<x4*>(ds_lds + (wave * 32 + c) * BQ + 8 * rg + 4 * h) = w;
      }
      __syncthreads();
      // dQ[q][d-slice of this wave] = sum over the 128 keys dS[q][key] K[key][d]
      if (wave < DT) {
        f32x16 dq;
#pragma unroll
        for (int i = 0; i < 16; ++i) dq[i] = 0.f;
#pragma unroll
        for (int kk = 0; kk < BNK / 16; ++kk) {
          const int krow = kk * 16 + 8 * h + tq;
          const x8 a = join<T>(MT<T>::tr_read(ds_lds + krow * BQ + (lane & 16) + 4 * tp),
                               MT<T>::tr_read(ds_lds + (krow + 4) * BQ + (lane & 16) + 4 * tp));
          const int col = wave * 32 + (lane & 16) + 4 * tp;
          const x8 bk = join<T>(MT<T>::tr_read(k_lds + sw_off<HD>(krow, col)),
                                MT<T>::tr_read(k_lds + sw_off<HD>(krow + 4, col)));
          dq = MT<T>::mfma(a, bk, dq);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qr = q0 + acc_row(i, h);
          if (qr < p.sq) atomicAdd(DQ + (int64_t)qr * HD + wave * 32 + c, dq[i]);
        }
      }
    }
  }

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

template <typename T, int HD>
__global__ __launch_bounds__(256) void fa_dq_convert_k(const AttnBwdParams P) {
  const AttnParams& p = P.f;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // one per 8 elements
  const int64_t total = (int64_t)p.b * p.nq * p.sq * (HD / 8);
  if (t >= total) return;
  const int c8 = (int)(t % (HD / 8));
  const int64_t row = t / (HD / 8);  // (b, head, q)
  const int q = (int)(row % p.sq);
  const int head = (int)((row / p.sq) % p.nq);
  const int b = (int)(row / ((int64_t)p.sq * p.nq));
  const int r = p.nq / p.nkv;
  const float* src = P.dq_acc + row * HD + c8 * 8;
  const float4 a = *reinterpret_cast<const float4*>(src);
  const float4 bb = *reinterpret_cast<const float4*>(src + 4);
  typename MT<T>::x8 o;
  o[0] = (T)(a.x * p.scale); o[1] = (T)(a.y * p.scale); o[2] = (T)(a.z * p.scale); o[3] = (T)(a.w * p.scale);
  o[4] = (T)(bb.x * p.scale); o[5] = (T)(bb.y * p.scale); o[6] = (T)(bb.z * p.scale); o[7] = (T)(bb.w * p.scale);
  T* dst = (T*)P.dq + (int64_t)b * p.q_sb + (int64_t)q * p.q_ss + (int64_t)(head / r) * p.q_sg +
           (int64_t)(head % r) * p.q_sh + c8 * 8;
  *reinterpret_cast<typename MT<T>::x8*>(dst) = o;
}

template <typename T, int HD>
void launch_bwd(const AttnBwdParams& P, hipStream_t s) {
  const AttnParams& p = P.f;
  const int64_t rows = (int64_t)p.b * p.nq * p.sq;
  (void)hipMemsetAsync(P.dq_acc, 0, rows * HD * sizeof(float), s);
  hipLaunchKernelGGL((fa_delta_k<T, HD>), dim3((rows + 255) / 256), dim3(256), 0, s, P);
  dim3 grid((p.sk + BNK - 1) / BNK, p.nkv, p.b);
  if (p.causal)
    hipLaunchKernelGGL((fa_bwd_k<T, HD, true>), grid, dim3(256), 0, s, P);
  else
    hipLaunchKernelGGL((fa_bwd_k<T, HD, false>), grid, dim3(256), 0, s, P);
  const int64_t n8 = rows * (HD / 8);
  hipLaunchKernelGGL((fa_dq_convert_k<T, HD>), dim3((n8 + 255) / 256), dim3(256), 0, s, P);
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
