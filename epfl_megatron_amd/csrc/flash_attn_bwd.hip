// FlashAttention-2 backward for gfx950 (MI355X), native GQA/MQA, causal.
//
// Two MFMA kernels, dQ first (it also produces delta = rowsum(dO * O) and
// the LSE in log2 units for the dK/dV kernel); neither needs atomics:
//
// fa_bwd_dkdv2_k -- workgroup = 4 waves = 128 keys of one (batch, KV group);
//   each wave keeps its 32 keys' K and V fragments in registers and
//   accumulates dK^T / dV^T over the query heads of the group and all query
//   tiles (GQA reduced inside the workgroup).  Per 64-row query step (Q, dO,
//   LSE, delta by LDS-DMA into a 2-deep ring, one barrier per step):
//     S  = Q K^T, P = exp2(S*scale*log2e - LSE*log2e)
//     dP = dO V^T (acc pre-loaded with -delta),  dS = P * (dP - delta)
//     dV^T += dO^T P,  dK^T += Q^T dS   (P / dS accumulators used directly as
//                                        the B operand; dO^T / Q^T via
//                                        ds_read_b64_tr_b16)
//   With few KV heads per rank the group's query heads are split over
//   kv_split workgroups (fp32 partials, fa_dkv_reduce_k adds them in order).
// fa_bwd_dq2_k -- workgroup = 8 waves = 256 query rows of one head, 64-key
//   tiles of K/V through double-buffered LDS; recomputes S^T / dP^T with the
//   query on the MFMA lane and accumulates dQ^T = K^T dS^T in registers.
//
// Document mask (optional, p.doc_start != nullptr): the dQ kernel starts each
// query block at its first document's first key tile; the dK/dV kernel ends
// each key block's query range at its last key's document end and masks
// queries whose document starts after the key (doc starts streamed with LSE).
//
// RoPE (optional, p.rope_cos != nullptr): the forward rotated Q and K, so dQ
// and dK come out in the rotated basis; both kernels apply R^T to them in
// their epilogue (fp32, before the bf16 store), replacing a separate
// read-modify-write pass over dQ/dK.
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

typedef __attribute__((ext_vector_type(2))) float f2;


typedef __attribute__((ext_vector_type(4))) float f4;

constexpr int BNK = 128;  // keys per dK/dV workgroup
constexpr int KT = 64;    // keys per dQ step
#ifndef DQ_RING
#define DQ_RING 3  // K/V ring depth of the 8-wave dQ kernel (A/B: -DDQ_RING=2)
#endif


// dK/dV: 4 waves x 32 keys, K/V fragments and dK^T/dV^T accumulators
// register-resident; each step covers 64 query rows (two 32-row sub-slices)
// and the Q / dO / LSE / delta tiles arrive by LDS-DMA into a 2-deep ring
// (issued one step ahead; the lane-linear image takes the swizzle through the
// per-lane SOURCE address) — no staging registers and no ds_write pass, which
// together cost more than the step's MFMAs in the round-1 register-staged
// kernel (profiles/r1_fa_bwd_split.txt).  Transposed reads are inline asm so
// hipcc does not drain the in-flight DMA in front of them.
constexpr int BQ2 = 64;

// Persistent form: a flat grid of min(items, CUs) workgroups walks the
// (key block, KV group x split, batch) items, listed heaviest-first, in a
// snake order (round k: item k*G + w, or k*G + G-1-w for odd k), so under the
// causal mask every workgroup gets a balanced sum of work.  Across an item seam the next item's K/V rows (LDS-DMA into a
// staging image, read into registers at the item start) and its first Q/dO
// step are loaded during the current item's steps, so the per-item prologue
// (≈ 4-5 steps' worth of load latency at s = 1024) is hidden.
template <typename T, int HD, bool CAUSAL>
__global__ __launch_bounds__(256, 1) void fa_bwd_dkdv2_k(const AttnBwdParams P) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  const AttnParams& p = P.f;
  constexpr int KS = HD / 16, DT = HD / 32, CH = HD / 8;
  constexpr int ROWB = HD * 2;                   // bytes per Q / dO / K / V row
  constexpr int RG = 8 * ROWB;                   // bytes per 8-row group (image (a))
  constexpr int TILEB = BQ2 * ROWB;              // one Q (or dO) tile
  constexpr int BUFB = 2 * TILEB + 3 * BQ2 * 4;  // Q, dO, lse2, -delta, doc start
  constexpr int PIECES = TILEB / 1024, PPW = PIECES / 4;
  constexpr int KVB = BNK * ROWB;                // K (or V) rows of one item
  constexpr int KVPW = KVB / 1024 / 4;           // 1-KiB DMA pieces per wave for K (and V)
  static_assert(PIECES % 4 == 0 && (KVB / 1024) % 4 == 0, "pieces per wave");
  __shared__ __attribute__((aligned(1024))) char lds[2 * BUFB + 2 * KVB];
  char* const kvs = lds + 2 * BUFB;  // staging: K rows then V rows, chunk ^ (row % CH)

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3, l4 = (lane >> 4) & 1;
  const int S = P.kv_split > 1 ? P.kv_split : 1;
  const int r = p.nq / p.nkv, r_per = r / S;
  const int off = p.coff;
  const float sl2 = p.scale * 1.4426950408889634f;
  const int ngs = p.nkv * S;
  const int nitems = ((p.sk + BNK - 1) / BNK) * ngs * p.b;

  // item -> key block (heaviest first), KV group, query-head split, batch
  struct Item {
    int nb, g, split, b, h0, q_first, nsteps_q, nsteps;
  };
  auto decode = [&](int it, Item& I) {
    I.nb = it / (ngs * p.b);
    const int rem = it - I.nb * (ngs * p.b);
    const int gs = rem % ngs;
    I.b = rem / ngs;
    I.g = gs / S;
    I.split = gs % S;
    I.h0 = I.split * r_per;
    int qf = 0;
    if (CAUSAL) {
      qf = I.nb * BNK - off;
      qf = qf < 0 ? 0 : (qf / BQ2) * BQ2;
    }
    I.q_first = qf;
    int q_end = p.sq;
    if (CAUSAL && p.doc_end) {  // no query past the last key's document sees this block
      const int kl = I.nb * BNK + BNK - 1 < p.sk ? I.nb * BNK + BNK - 1 : p.sk - 1;
      q_end = p.doc_end[(int64_t)I.b * p.sq + kl];
    }
    I.nsteps_q = q_end > qf ? (q_end - qf + BQ2 - 1) / BQ2 : 0;
    I.nsteps = r_per * I.nsteps_q;
  };

  // LDS-DMA source offsets of this lane's Q/dO pieces (image (a) through the source)
  int srow[PPW], schunk[PPW];
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int o = (wave * PPW + i) * 1024 + 16 * lane;
    const int rem = o % RG, rem2 = rem % 512;
    srow[i] = 8 * (o / RG) + rem2 / 64;
    schunk[i] = 4 * (rem / 512) + (((rem2 % 64) / 16) ^ ((srow[i] >> 2) & 3));
  }
  auto prefetch = [&](const Item& I, int step, int buf) {
    const int hl = step / I.nsteps_q, hh = I.h0 + hl;
    const int q0 = I.q_first + (step - hl * I.nsteps_q) * BQ2;
    const int head = I.g * r + hh;
    const T* Q = (const T*)p.q + (int64_t)I.b * p.q_sb + (int64_t)I.g * p.q_sg + (int64_t)hh * p.q_sh;
    const T* DO = (const T*)P.dout + (int64_t)I.b * p.o_sb + (int64_t)head * p.o_sh;
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
      const int64_t rb = ((int64_t)I.b * p.nq + head) * p.sq;
      const float* src = wave == 0 ? P.lse2 + rb + qr : P.ndelta + rb + qr;
      __builtin_amdgcn_global_load_lds(
          (const void*)src,
          (__attribute__((address_space(3))) void*)(base + 2 * TILEB + wave * BQ2 * 4), 4, 0, 0);
    } else if (wave == 2 && CAUSAL && p.doc_start) {  // the rows' document starts
      int qr = q0 + lane;
      qr = qr < p.sq ? qr : p.sq - 1;
      __builtin_amdgcn_global_load_lds(
          (const void*)(p.doc_start + (int64_t)I.b * p.sq + qr),
          (__attribute__((address_space(3))) void*)(base + 2 * TILEB + 2 * BQ2 * 4), 4, 0, 0);
    }
  };
  // K / V rows of an item into the staging image: piece byte o holds row
  // o / ROWB, physical chunk (o % ROWB) / 16 = logical chunk ^ (row % CH).
  auto kv_prefetch = [&](const Item& I) {
    const T* K = (const T*)p.k + (int64_t)I.b * p.k_sb + (int64_t)I.g * p.k_sg;
    const T* V = (const T*)p.v + (int64_t)I.b * p.v_sb + (int64_t)I.g * p.v_sg;
    // lane index made opaque: the piece addresses are recomputed here (twice
    // per item) instead of being hoisted and held in 32 VGPRs across the loop
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int i = 0; i < KVPW; ++i) {
      const int pc = wave * KVPW + i;
      const int o = pc * 1024 + 16 * ln;
      const int row = o / ROWB, ch = ((o % ROWB) / 16) ^ (row % CH);
      int kr = I.nb * BNK + row;
      kr = kr < p.sk ? kr : p.sk - 1;
      __builtin_amdgcn_global_load_lds((const void*)(K + (int64_t)kr * p.k_ss + ch * 8),
                                       (__attribute__((address_space(3))) void*)(kvs + pc * 1024),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(V + (int64_t)kr * p.v_ss + ch * 8),
                                       (__attribute__((address_space(3))) void*)(kvs + KVB + pc * 1024),
                                       16, 0, 0);
    }
  };

  // loop-invariant LDS read offsets (the rest are immediates)
  int rowb[2], trb[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    rowb[x] = RG * (c >> 3) + 64 * (c & 7) + 16 * ((2 * x + h) ^ ((c >> 2) & 3));
    trb[x] = RG * x + 64 * (4 * h + tq) + 16 * ((2 * l4 + (tp >> 1)) ^ ((h + 2 * x) & 3)) +
             8 * (tp & 1);
  }
  const int cstb = 2 * TILEB + 4 * (4 * h);
  const int krow = wave * 32 + c;  // this lane's key within the item

  // round k of workgroup w takes item k*G + (k odd ? G-1-w : w): a snake over the
  // heaviest-first list, so every workgroup's sum of causal work is balanced
  const int G = (int)gridDim.x, w = (int)blockIdx.x;
  auto item_of = [&](int k) { return k * G + ((k & 1) ? G - 1 - w : w); };
  int k = 0, it = item_of(0);
  if (it >= nitems) return;  // whole workgroup (grid <= items; defensive)
  Item cur;
  decode(it, cur);
  kv_prefetch(cur);
  if (cur.nsteps > 0) prefetch(cur, 0, 0);
  int gstep = 0;  // ring parity runs across items
  __syncthreads();  // vmcnt(0) + barrier: K/V rows and step 0 landed

  while (true) {
    const int kbase = cur.nb * BNK + wave * 32;
    const int key = kbase + c;
    x8 kf[KS], vf[KS];
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int so = krow * ROWB + 16 * ((2 * kk + h) ^ (krow % CH));
      kf[kk] = *reinterpret_cast<const x8*>(kvs + so);
      vf[kk] = *reinterpret_cast<const x8*>(kvs + KVB + so);
    }
    f32x16 dk[DT], dv[DT];
#pragma unroll
    for (int d = 0; d < DT; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) dk[d][i] = dv[d][i] = 0.f;
    const int nit = item_of(k + 1);
    const bool has_next = nit < nitems;
    const int nsteps = cur.nsteps;

    for (int step = 0; step < nsteps; ++step) {
      const int hs = step / cur.nsteps_q;
      const int q0 = cur.q_first + (step - hs * cur.nsteps_q) * BQ2;
      const int buf = gstep & 1;
      if (step + 1 < nsteps) {
        prefetch(cur, step + 1, buf ^ 1);
      } else if (has_next) {  // (next item decoded where used: fewer live registers)
        Item nx;
        decode(nit, nx);
        if (nx.nsteps > 0) prefetch(nx, 0, buf ^ 1);
      }
      // the staging image was read at the item start, before step 0's barrier
      if (step == 1 && has_next) {
        Item nx;
        decode(nit, nx);
        kv_prefetch(nx);
      }
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
        const bool docs = CAUSAL && p.doc_start;
        const bool need_mask = (q0s + 32 > p.sq) || (kbase + 32 > p.sk) ||
                               (CAUSAL && (kbase + 31 > q0s + off)) || docs;
        // P = exp2(S scale log2e - lse log2e), the argument by packed fma
        const f2 sc2 = {sl2, sl2};
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f2 a = __builtin_elementwise_fma(
              f2{sacc[i], sacc[i + 1]}, sc2, -f2{l24[i >> 2][i & 3], l24[i >> 2][(i & 3) + 1]});
          sacc[i] = __builtin_amdgcn_exp2f(a[0]);
          sacc[i + 1] = __builtin_amdgcn_exp2f(a[1]);
        }
        if (need_mask) {
          if (docs) {
            typedef __attribute__((ext_vector_type(4))) int i4;
            i4 ds4[4];
            const int* dsl = reinterpret_cast<const int*>(cst + 2 * BQ2);
#pragma unroll
            for (int rg = 0; rg < 4; ++rg) ds4[rg] = *reinterpret_cast<const i4*>(dsl + 8 * rg);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int qr = q0s + acc_row(i, h);
              const bool ok = (qr < p.sq) & (key < p.sk) & (key <= qr + off) &
                              (key >= ds4[i >> 2][i & 3]);
              sacc[i] = ok ? sacc[i] : 0.f;
            }
          } else {
            // row rc = acc_row(i, 0) of the block is kept iff lo <= rc <= hi
            int hi = p.sq - 1 - q0s - 4 * h;
            if (key >= p.sk) hi = -1;
            const int lo = CAUSAL ? key - off - q0s - 4 * h : -(1 << 30);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int rc = (i & 3) + 8 * (i >> 2);
              if (rc > hi || rc < lo) sacc[i] = 0.f;
            }
          }
        }
        // dS = P (dP - delta): packed multiplies
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f2 d = f2{sacc[i], sacc[i + 1]} * f2{dpacc[i], dpacc[i + 1]};
          dpacc[i] = d[0];
          dpacc[i + 1] = d[1];
        }
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
      __syncthreads();  // vmcnt(0) + barrier: next step (or item) landed, this step's reads retired
      ++gstep;
    }
    // items with < 2 steps: nothing of the next item was loaded in the loop
    if (has_next && nsteps <= 1) {
      Item nx;
      decode(nit, nx);
      if (nsteps == 0 && nx.nsteps > 0) prefetch(nx, 0, gstep & 1);
      kv_prefetch(nx);
    }

    mfma_drain();
    if (key < p.sk) {
      if (S > 1) {  // fp32 partial sums; fa_dkv_reduce_k adds the splits in order
        float* W = P.dkv_ws + ((((int64_t)cur.split * p.b + cur.b) * p.nkv + cur.g) * p.sk + key) * 2 * HD;
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
      } else {
        T* DK = (T*)P.dk + (int64_t)cur.b * p.k_sb + (int64_t)cur.g * p.k_sg + (int64_t)key * p.k_ss;
        T* DV = (T*)P.dv + (int64_t)cur.b * p.v_sb + (int64_t)cur.g * p.v_sg + (int64_t)key * p.v_ss;
        const float *rc = nullptr, *rs = nullptr;
        rf2 rcc[DT][4], rsn[DT][4];
        if (p.rope_cos) {
          rope_rows<HD>(p, cur.b, key, rc, rs);
          rope_inv_tables<DT>(rcc, rsn, rc, rs, h);
        }
#pragma unroll
        for (int d = 0; d < DT; ++d) {
#pragma unroll
          for (int rg = 0; rg < 4; ++rg) {
            float f[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) f[e] = dk[d][4 * rg + e] * p.scale;
            if (rc) rope_inv4v(f, rcc[d][rg], rsn[d][rg]);
            x4 wk, wv;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              wk[e] = (T)f[e];
              wv[e] = (T)dv[d][4 * rg + e];
            }
            *reinterpret_cast<x4*>(DK + d * 32 + 8 * rg + 4 * h) = wk;
            *reinterpret_cast<x4*>(DV + d * 32 + 8 * rg + 4 * h) = wv;
          }
        }
      }
    }
    if (!has_next) break;
    if (nsteps <= 1) __syncthreads();  // the loads issued after the loop landed
    ++k;
    it = nit;
    decode(it, cur);
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
  float f[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) f[e] = is_v ? acc[e] : acc[e] * p.scale;
  if (!is_v && p.rope_cos) {
    const float *rc, *rs;
    rope_rows<HD>(p, b, key, rc, rs);
    rope_inv4(f, rc, rs, col / 2);
  }
  typename MT<T>::x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (T)f[e];
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
// KV2 (WAVES = 8): the split-key form of the forward's fa_fwd_k KV2 -- the 128
// rows of a 4-wave block on 8 waves, waves 4..7 over the second half of the
// key tiles; their dQ partials are added through LDS at the end.
template <typename T, int HD, bool CAUSAL, int WAVES, bool KV2 = false>
__global__ __launch_bounds__(WAVES * 64, 8 / WAVES) void fa_bwd_dq2_k(const AttnBwdParams P) {
  typedef typename MT<T>::x8 x8;
  typedef typename MT<T>::x4 x4;
  const AttnParams& p = P.f;
  static_assert(!KV2 || WAVES == 8, "KV2: two 4-wave halves");
  constexpr int RW = KV2 ? 4 : WAVES;  // waves holding distinct query rows
  constexpr int NT = WAVES * 64, BMW = RW * 32;
  constexpr int KS = HD / 16, DT = HD / 32, CPR = HD / 8;
  // K/V ring depth: 3 tiles (two in flight behind the one being read) for the
  // one-block-per-CU 8-wave form; 2 for the 4-wave form (two blocks per CU)
  // and for each half of the split-key form
  constexpr int NB = (WAVES == 8 && !KV2) ? DQ_RING : 2;
  constexpr int NG = KV2 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) T lds[NG * NB * 2 * KT * HD];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int grp = KV2 ? (wave >> 2) : 0, rw = KV2 ? (wave & 3) : wave;
  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nqb = (p.sq + BMW - 1) / BMW;
  const int nhb = p.nq * p.b;
  int lin = blockIdx.x;
  if (CAUSAL && p.pair_ncu > 0 && lin >= p.pair_ncu) lin = 3 * p.pair_ncu - 1 - lin;  // kernels.h
  const int qb = CAUSAL ? (nqb - 1 - lin / nhb) : lin / nhb;
  const int head = (lin % nhb) % p.nq, b = (lin % nhb) / p.nq;
  const int r = p.nq / p.nkv, g = head / r, hh = head - g * r;
  const int off = p.coff;
  const int q0w = qb * BMW + rw * 32;
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
  // document mask (as in the forward): start at the first row's document
  int t0 = 0, wt0 = 0, ds_row = 0, ds_wmax = 0;
  if (CAUSAL && p.doc_start) {
    const int* D = p.doc_start + (int64_t)b * p.sq;
    const int r0 = qb * BMW < p.sq ? qb * BMW : p.sq - 1;
    const int w0 = q0w < p.sq ? q0w : p.sq - 1, w1 = q0w + 31 < p.sq ? q0w + 31 : p.sq - 1;
    t0 = D[r0] / KT;
    wt0 = D[w0] / KT;
    ds_wmax = D[w1];
    ds_row = D[qrow_c];
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
  auto prefetch = [&](int t, int buf, int g) {
    char* kl = reinterpret_cast<char*>(lds + (g * NB + buf) * 2 * KT * HD);
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
  // this wave's key tiles [gs, ge) over niter barrier-synchronous iterations
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

  x8 qf[KS], df[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    qf[kk] = ld8(Q + (int64_t)qrow_c * p.q_ss + kk * 16 + 8 * h);
    df[kk] = ld8(DO + (int64_t)qrow_c * p.o_ss + kk * 16 + 8 * h);
  }
  // delta = rowsum(dO * O) for this lane's row (the row's two halves live on
  // lanes c and c + 32); the row constants the dK/dV kernel (launched after
  // this one) streams in are written here: no separate delta pass.
  const int64_t rb = ((int64_t)b * p.nq + head) * p.sq;
  const float lse2 = p.lse[rb + qrow_c] * 1.4426950408889634f;
  float dlt = 0.f;
  {
    const T* O = (const T*)p.o + (int64_t)b * p.o_sb + (int64_t)qrow_c * p.o_ss + (int64_t)head * p.o_sh;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const x8 ov = ld8(O + kk * 16 + 8 * h);
#pragma unroll
      for (int e = 0; e < 8; ++e) dlt += (float)ov[e] * (float)df[kk][e];
    }
    dlt += __shfl_xor(dlt, 32, 64);
    if (h == 0 && qrow < p.sq && grp == 0) {
      P.ndelta[rb + qrow] = -dlt;
      P.lse2[rb + qrow] = lse2;
    }
  }

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

  for (int it = 0; it < niter; ++it) {
    const int t = gs + it;
    const int buf = KV2 ? grp * NB + (it & 1) : t % NB;
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
    const char* kl = reinterpret_cast<const char*>(lds + buf * 2 * KT * HD);
    const char* vl = kl + KT * ROWB;
    const uint32_t trv0 = (uint32_t)(uintptr_t)(kl + trb[0]);
    const uint32_t trv1 = (uint32_t)(uintptr_t)(kl + trb[1]);
    if (t < ge && t < wtiles && t >= wt0) {
      static_for<KT / 32>([&](auto subc) {
        constexpr int sub = decltype(subc)::value;
        const int kb = t * KT + sub * 32;
        f32x16 sacc, dpacc;
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int o = sub * 4 * RG + rowb[kk & 1] + 512 * (kk >> 1);
          const x8 ka = *reinterpret_cast<const x8*>(kl + o);
          const x8 va = *reinterpret_cast<const x8*>(vl + o);
          if (kk == 0) {
            sacc = mfma_vgpr0<T>(ka, qf[0]);
            dpacc = mfma_vgpr0<T>(va, df[0]);
          } else {
            mfma_vgpr<T>(sacc, ka, qf[kk]);
            mfma_vgpr<T>(dpacc, va, df[kk]);
          }
        }
        // K^T fragments of this 32-key sub-block (asm transposed reads), issued
        // before the softmax VALU so their latency hides under it (retired by
        // one lds_wait before the dS K MFMAs, as the dK/dV kernel does)
        typename MT<T>::x4 kt[2][DT][2];
        static_for<2>([&](auto sc) {
          static_for<DT>([&](auto dc) {
            constexpr int o = sub * 4 * RG + decltype(sc)::value * 2 * RG + 512 * decltype(dc)::value;
            kt[sc][dc][0] = tr_read_imm<o, T>(trv0);
            kt[sc][dc][1] = tr_read_imm<o, T>(trv1);
          });
        });
        mfma_drain();
        const bool need_mask = (kb + 32 > p.sk) || (q0w + 32 > p.sq) ||
                               (CAUSAL && (kb + 31 > q0w + off || kb < ds_wmax));
        const f2 sc2 = {sl2, sl2}, ml2 = {-lse2, -lse2}, nd2 = {-dlt, -dlt};
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f2 a = __builtin_elementwise_fma(f2{sacc[i], sacc[i + 1]}, sc2, ml2);
          sacc[i] = __builtin_amdgcn_exp2f(a[0]);
          sacc[i + 1] = __builtin_amdgcn_exp2f(a[1]);
        }
        if (need_mask) {
          // key rc = acc_row(i, 0) of the block is kept iff lo <= rc <= hi
          int hi = p.sk - 1 - kb - 4 * h;
          if (CAUSAL) hi = min(hi, qrow + off - kb - 4 * h);
          if (qrow >= p.sq) hi = -1;
          if (CAUSAL && p.doc_start) {
            const int lo = ds_row - kb - 4 * h;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int rc = (i & 3) + 8 * (i >> 2);
              if (rc > hi || rc < lo) sacc[i] = 0.f;
            }
          } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int rc = (i & 3) + 8 * (i >> 2);
              if (rc > hi) sacc[i] = 0.f;
            }
          }
        }
        // dS = P (dP - delta): packed add and multiply
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f2 d = f2{sacc[i], sacc[i + 1]} * (f2{dpacc[i], dpacc[i + 1]} + nd2);
          sacc[i] = d[0];
          sacc[i + 1] = d[1];
        }
        lds_wait();  // the K^T reads above
        static_for<2>([&](auto sc) {
          const x8 sf = acc_frag<T>(sacc, decltype(sc)::value);
          static_for<DT>([&](auto dc) {
            mfma_vgpr<T, 1>(dq[dc], join<T>(kt[sc][dc][0], kt[sc][dc][1]), sf);
          });
        });
      });
    }
    if (NB == 3 && t + 2 < ntiles) {
      // counted: tile t+1 landed, tile t+2's DMA (2 * PPW instructions) may fly on
      asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"i"(2 * PPW) : "memory");
      __builtin_amdgcn_s_barrier();
    } else {
      __syncthreads();  // vmcnt(0) + barrier: tile t+1 landed, tile t's reads retired
    }
  }

  mfma_drain();
  if constexpr (KV2) {
    // add the second half's dQ partials (the loop ended on a barrier: the rings
    // are drained); lane-contiguous floats, conflict-free
    float* ob = reinterpret_cast<float*>(lds);
    if (grp == 1) {
#pragma unroll
      for (int d = 0; d < DT; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) ob[((rw * DT + d) * 16 + i) * 64 + lane] = dq[d][i];
    }
    __syncthreads();
    if (grp == 0) {
#pragma unroll
      for (int d = 0; d < DT; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) dq[d][i] += ob[((rw * DT + d) * 16 + i) * 64 + lane];
    }
  }
  if ((!KV2 || grp == 0) && qrow < p.sq) {
    T* DQ = (T*)P.dq + (int64_t)b * p.q_sb + (int64_t)qrow * p.q_ss + (int64_t)g * p.q_sg +
            (int64_t)hh * p.q_sh;
    const float *rc = nullptr, *rs = nullptr;
    rf2 rcc[DT][4], rsn[DT][4];
    if (p.rope_cos) {
      rope_rows<HD>(p, b, qrow, rc, rs);
      rope_inv_tables<DT>(rcc, rsn, rc, rs, h);
    }
#pragma unroll
    for (int d = 0; d < DT; ++d) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        float f[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) f[e] = dq[d][4 * rg + e] * p.scale;
        if (rc) rope_inv4v(f, rcc[d][rg], rsn[d][rg]);
        x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (T)f[e];
        *reinterpret_cast<x4*>(DQ + d * 32 + 8 * rg + 4 * h) = w;
      }
    }
  }
}

template <typename T, int HD>
void launch_bwd(const AttnBwdParams& P0, hipStream_t s) {
  AttnBwdParams P = P0;
  const AttnParams& p = P.f;
  // dK/dV: persistent, min(items, CUs) workgroups (EMA_FA_DKDV_GRID=full: one per item)
  static const int ncu = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    const char* e = getenv("EMA_FA_DKDV_GRID");
    return (e && e[0] == 'f') ? (1 << 30) : n;
  }();
  const long kv_items = (long)((p.sk + BNK - 1) / BNK) * p.nkv * (P.kv_split > 1 ? P.kv_split : 1) * p.b;
  const dim3 gkv((unsigned)(kv_items < ncu ? kv_items : ncu));
  const int64_t kvred = (int64_t)p.b * p.nkv * p.sk * (2 * HD / 4);
  const int wv = flash_attn_waves(p.b, p.sq, p.nq, HD);
  const dim3 gq(((p.sq + 255) / 256) * p.nq * p.b);
  const dim3 gq4(((p.sq + 127) / 128) * p.nq * p.b);
  // dQ blocks in the forward's causal pairing; the dK/dV kernel reads none
  // the split-key dQ on the grids the forward runs split-key
  const bool kv2 = HD == 128 && flash_attn_kv2(p.b, p.sq, p.nq, HD);
  P.f.pair_ncu = kv2 ? 0 : fa_pair_ncu(p.causal, wv == 4 ? gq4.x : gq.x, wv, HD);
#define EMA_FA_BWD(C)                                                                     \
  {                                                                                       \
    if (kv2) hipLaunchKernelGGL((fa_bwd_dq2_k<T, HD, C, 8, true>), gq4, dim3(512), 0, s, P); \
    else if (wv == 4) hipLaunchKernelGGL((fa_bwd_dq2_k<T, HD, C, 4>), gq4, dim3(256), 0, s, P); \
    else hipLaunchKernelGGL((fa_bwd_dq2_k<T, HD, C, 8>), gq, dim3(512), 0, s, P);         \
    hipLaunchKernelGGL((fa_bwd_dkdv2_k<T, HD, C>), gkv, dim3(256), 0, s, P);              \
    if (P.kv_split > 1)                                                                   \
      hipLaunchKernelGGL((fa_dkv_reduce_k<T, HD>), dim3((unsigned)((kvred + 255) / 256)), \
                         dim3(256), 0, s, P);                                             \
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
