// FlashAttention-2 forward for gfx950 (MI355X), native GQA/MQA, causal.
//
// Workgroup = 8 waves = a 256-row query block of one (batch, query head); each
// wave owns 32 query rows, two waves per SIMD share every K/V tile.  K/V tiles
// of 64 keys stream through double-buffered LDS, register-staged: the next
// tile's global loads are issued before the current tile's MFMAs and written
// to the other buffer after them (CDNA guide T14), one barrier per tile.
//
// Per 32(q) x 64(k) step a wave runs 2 x HD/16 MFMAs for S^T = K Q^T and
// 2 x 2 x HD/32 MFMAs for O^T += V^T P^T (v_mfma_f32_32x32x16).  S is computed
// transposed ("swapped QK^T", guide T12) so a query row lives on one lane pair
// (lane, lane^32): the online-softmax max/sum is 31 in-register ops + one
// cross-half shuffle, the O rescale is a per-lane scalar, and the P
// accumulator feeds the PV MFMA as its B operand with no LDS round trip.  V is
// read from LDS with ds_read_b64_tr_b16 (hardware transpose, guide T10) from a
// row-padded image (conflict-free); K uses an XOR-swizzled image (T2).
//
// Query head j reads KV group j / (nq / nkv) directly (no K/V expansion).
// Query blocks are dispatched on a flat grid, heaviest causal blocks of ALL
// heads first.  LSE is written in natural log.
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

constexpr int BN = 64;
constexpr int VPAD = 32;  // elements of padding per V row (64 B) -> conflict-free tr reads

template <typename T, int HD, bool CAUSAL, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 8 / WAVES) void fa_fwd2_k(const AttnParams p) {
  typedef typename MT<T>::x8 x8;
  constexpr int NT = WAVES * 64;
  constexpr int BMW = WAVES * 32;
  constexpr int KS = HD / 16;
  constexpr int DT = HD / 32;
  constexpr int CPR = HD / 8;
  constexpr int VST = HD + VPAD;
  constexpr int KCH = (BN * CPR + NT - 1) / NT;  // chunks of K (and of V) per thread
  constexpr int KTILE = BN * HD, VTILE = BN * VST;
  __shared__ __attribute__((aligned(16))) T lds[2 * (KTILE + VTILE)];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, h = lane >> 5, c = lane & 31;
  const int nmb = (p.sq + BMW - 1) / BMW;
  // flat grid: lin -> (query block, head, batch); heavy blocks first
  const int nhb = p.nq * p.b;
  const int lin = blockIdx.x;
  const int mb = CAUSAL ? (nmb - 1 - lin / nhb) : lin / nhb;
  const int hb = lin % nhb;
  const int head = hb % p.nq, b = hb / p.nq;
  const int r = p.nq / p.nkv, g = head / r;
  const int off = p.sk - p.sq;

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
  const int ntiles = n_end > 0 ? (n_end + BN - 1) / BN : 0;
  // this wave's own last useful tile (causal): later tiles are fully masked
  int wtiles = ntiles;
  if (CAUSAL) {
    const int wl = m0 + 32 + off;
    const int wt = wl > 0 ? (wl + BN - 1) / BN : 0;
    wtiles = wt < ntiles ? wt : ntiles;
  }

  x8 kst[KCH], vst[KCH];
  int krow[KCH];
  bool kact[KCH];
  int64_t koff[KCH], voff[KCH];
#pragma unroll
  for (int i = 0; i < KCH; ++i) {
    const int idx = tid + NT * i;
    kact[i] = idx < BN * CPR;
    krow[i] = (idx / CPR) % BN;
    koff[i] = (int64_t)krow[i] * p.k_ss + (idx % CPR) * 8;
    voff[i] = (int64_t)krow[i] * p.v_ss + (idx % CPR) * 8;
  }
  auto load_tile = [&](int n0) {
    const T* kt = K + (int64_t)n0 * p.k_ss;
    const T* vt = V + (int64_t)n0 * p.v_ss;
    if (n0 + BN <= p.sk) {
#pragma unroll
      for (int i = 0; i < KCH; ++i)
        if (kact[i]) {
          kst[i] = ld8(kt + koff[i]);
          vst[i] = ld8(vt + voff[i]);
        }
    } else {
#pragma unroll
      for (int i = 0; i < KCH; ++i)
        if (kact[i]) {
          const int64_t back = (n0 + krow[i] < p.sk) ? 0 : (int64_t)(n0 + krow[i] - (p.sk - 1));
          kst[i] = ld8(kt + koff[i] - back * p.k_ss);
          vst[i] = ld8(vt + voff[i] - back * p.v_ss);
        }
    }
  };
  auto store_tile = [&](int buf) {
    T* kl = lds + buf * (KTILE + VTILE);
    T* vl = kl + KTILE;
#pragma unroll
    for (int i = 0; i < KCH; ++i)
      if (kact[i]) {
        const int idx = tid + NT * i;
        const int row = idx / CPR, ch = idx % CPR;
        *reinterpret_cast<x8*>(kl + sw_off<HD>(row, ch * 8)) = kst[i];
        *reinterpret_cast<x8*>(vl + row * VST + ch * 8) = vst[i];
      }
  };

  if (ntiles > 0) load_tile(0);
  x8 qf[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) qf[kk] = ld8(Q + (int64_t)qrow_c * p.q_ss + kk * 16 + 8 * h);
  if (p.rope_cos) {
    const float *rc, *rs;
    rope_rows<HD>(p, b, qrow_c, rc, rs);
    T* Qw = const_cast<T*>(Q) + (int64_t)qrow * p.q_ss + 8 * h;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      qf[kk] = rope_fwd8<T>(qf[kk], rc, rs, kk * 8 + 4 * h);
      if (qrow < p.sq) *reinterpret_cast<x8*>(Qw + kk * 16) = qf[kk];
    }
  }

  f32x16 o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int i = 0; i < 16; ++i) o[d][i] = 0.f;
  float m_i = -INFINITY, l_i = 0.f;
  const float sl2 = p.scale * 1.4426950408889634f;

  if (ntiles > 0) store_tile(0);
  __syncthreads();

  const int gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  for (int t = 0; t < ntiles; ++t) {
    const int n0 = t * BN;
    const int cur = t & 1;
    if (t + 1 < ntiles) load_tile(n0 + BN);
    const T* kl = lds + cur * (KTILE + VTILE);
    const T* vl = kl + KTILE;

    if (t < wtiles) {
      f32x16 s0, s1;
#pragma unroll
      for (int i = 0; i < 16; ++i) s0[i] = s1[i] = 0.f;
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) {
        const x8 ka0 = *reinterpret_cast<const x8*>(kl + sw_off<HD>(c, kk * 16 + 8 * h));
        const x8 ka1 = *reinterpret_cast<const x8*>(kl + sw_off<HD>(32 + c, kk * 16 + 8 * h));
        s0 = MT<T>::mfma(ka0, qf[kk], s0);
        s1 = MT<T>::mfma(ka1, qf[kk], s1);
      }
      const bool need_mask = CAUSAL ? (n0 + BN - 1 > m0 + off) : (n0 + BN > p.sk);
      if (need_mask) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int k0 = n0 + acc_row(i, h), k1 = k0 + 32;
          bool ok0 = k0 < p.sk, ok1 = k1 < p.sk;
          if (CAUSAL) {
            ok0 = ok0 && (k0 <= qrow + off);
            ok1 = ok1 && (k1 <= qrow + off);
          }
          if (!ok0) s0[i] = -INFINITY;
          if (!ok1) s1[i] = -INFINITY;
        }
      }
      float mt = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; i += 2)
        mt = fmaxf(mt, fmaxf(fmaxf(s0[i], s0[i + 1]), fmaxf(s1[i], s1[i + 1])));
      mt = fmaxf(mt, __shfl_xor(mt, 32, 64)) * sl2;
      const float m_new = fmaxf(m_i, mt);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = __builtin_amdgcn_exp2f(m_i - m_use);
      float rs0 = 0.f, rs1 = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s0[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s0[i], sl2, -m_use));
        s1[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s1[i], sl2, -m_use));
        rs0 += s0[i];
        rs1 += s1[i];
      }
      float rs = rs0 + rs1;
      rs += __shfl_xor(rs, 32, 64);
      l_i = l_i * alpha + rs;
      m_i = m_new;
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
        for (int d = 0; d < DT; ++d)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[d][i] *= alpha;
      }
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const x8 pf = acc_frag<T>(sub == 0 ? s0 : s1, s);
          const int kr = sub * 32 + 16 * s + 4 * h + tq;
#pragma unroll
          for (int d = 0; d < DT; ++d) {
            const int col = d * 32 + (lane & 16) + 4 * tp;
            const typename MT<T>::x4 va = MT<T>::tr_read(vl + kr * VST + col);
            const typename MT<T>::x4 vb = MT<T>::tr_read(vl + (kr + 8) * VST + col);
            o[d] = MT<T>::mfma(join<T>(va, vb), pf, o[d]);
          }
        }
      }
    }
    if (t + 1 < ntiles) store_tile(cur ^ 1);
    __syncthreads();
  }

  if (qrow < p.sq) {
    const float inv = l_i > 0.f ? 1.f / l_i : 0.f;
    T* O = (T*)p.o + (int64_t)b * p.o_sb + (int64_t)qrow * p.o_ss + (int64_t)head * p.o_sh;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        typename MT<T>::x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) w[e] = (T)(o[d][4 * rg + e] * inv);
        *reinterpret_cast<typename MT<T>::x4*>(O + d * 32 + 8 * rg + 4 * h) = w;
      }
    }
    if (h == 0) {
      const float lse = l_i > 0.f ? (m_i + __log2f(l_i)) * 0.6931471805599453f : -INFINITY;
      p.lse[((int64_t)b * p.nq + head) * p.sq + qrow] = lse;
    }
  }
}

template <typename T, int HD, int WAVES>
void launch_fwd2(const AttnParams& p, hipStream_t s) {
  const int bmw = 32 * WAVES;
  dim3 grid(((p.sq + bmw - 1) / bmw) * p.nq * p.b);
  if (p.causal)
    hipLaunchKernelGGL((fa_fwd2_k<T, HD, true, WAVES>), grid, dim3(64 * WAVES), 0, s, p);
  else
    hipLaunchKernelGGL((fa_fwd2_k<T, HD, false, WAVES>), grid, dim3(64 * WAVES), 0, s, p);
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

void flash_attn_fwd(const AttnParams& p, int dt, hipStream_t s) {
  const bool w4 = flash_attn_waves(p.b, p.sq, p.nq, p.hd) == 4;
  if (dt == DT_BF16) {
    if (p.hd == 128) w4 ? fa::launch_fwd2<bf16, 128, 4>(p, s) : fa::launch_fwd2<bf16, 128, 8>(p, s);
    else w4 ? fa::launch_fwd2<bf16, 64, 4>(p, s) : fa::launch_fwd2<bf16, 64, 8>(p, s);
  } else {
    if (p.hd == 128) w4 ? fa::launch_fwd2<fp16, 128, 4>(p, s) : fa::launch_fwd2<fp16, 128, 8>(p, s);
    else w4 ? fa::launch_fwd2<fp16, 64, 4>(p, s) : fa::launch_fwd2<fp16, 64, 8>(p, s);
  }
}

}  // namespace ema
