// Bench-only GEMM experiments (not used by the model): C = A · B^T, bf16,
// the persistent 4-wave 256x256 structure of gemm_nt.hip (variant 6) with the
// LDS image selectable at compile time, so a layout change is A/B-timed in one
// process against the production kernel and hipBLASLt
// (scripts/gemm_lab.py).  Ablation builds live here, not in the production
// translation units.
//
// LAYOUT 0 (production gemm_nt.hip): [256 rows][128 B] per operand and K-step,
//   16-B chunk c of row r at 16 (c ^ ((r >> 1) & 7)); the XOR is applied
//   through the per-lane DMA SOURCE address (lanes of one 8-lane row group
//   fetch the row's 8 chunks in permuted order).
// LAYOUT 1 (linear source, padded blocks): the operand's 256 rows form 32
//   blocks of 8 rows; block b holds rows b, b + 32, .., b + 224 (128 B each,
//   the DMA's lane-linear image of ONE instruction: lanes 8s..8s+7 fetch row
//   b + 32 s chunks 0..7 in order) at byte 1056 b (1 KiB + 32 B pad).  A
//   fragment (16 consecutive rows r0 + x) then sits in 16 distinct blocks of
//   one row slot: bank slot 2 (x & 7) + c + const, conflict-free for every
//   ds_read_b128 lane group, and the DMA never permutes a row's chunks.
// LAYOUT 2 / 3 (the vendor kernel's image): block b = 8 CONSECUTIVE rows
//   8b..8b+7 at byte BLK b (BLK = 1040 (2, the vendor's 16-B pad) or 1056
//   (3, conflict-free)), chunks in order; MFMA fragment j takes rows 8x + j of
//   the wave's band (x = lane & 15), so a lane's accumulators hold one row's
//   32 consecutive columns per A fragment (epilogue without lane shuffles);
//   MFMAs iterate the B fragment outermost (the A operand register changes
//   every MFMA, the B operand every 8).
#include <algorithm>

#include "fa_common.h"

namespace ema {
namespace {

using fa::static_for;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef fa::MT<bf16>::x8 X8;

constexpr int TM = 256, TN = 256, BK = 64;

template <int LAYOUT>
struct Lay {
  static constexpr int BLK = LAYOUT == 1 || LAYOUT == 3 ? 1056 : LAYOUT == 2 ? 1040 : 1024;  // bytes per 8-row DMA block
  static constexpr int OPB = 32 * BLK;                   // one operand, one K-step
  static constexpr int SLOTB = 2 * OPB;
};

__device__ __forceinline__ void mfma_acc(f32x4& acc, X8 a, X8 b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_acc0(f32x4& acc, X8 a, X8 b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}
template <int OFF>
__device__ __forceinline__ X8 row_read_imm(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16 bits");
  X8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "i"(OFF));
  return r;
}
__device__ __forceinline__ uint2 pack4(f32x4 v) {
  fa::MT<bf16>::x4 h;
  h[0] = (bf16)v[0]; h[1] = (bf16)v[1]; h[2] = (bf16)v[2]; h[3] = (bf16)v[3];
  return *reinterpret_cast<uint2*>(&h);
}
__device__ __forceinline__ uint4 pair_to_row8(uint2 x, uint2 y) {
  auto s0 = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
  auto s1 = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
  auto t0 = __builtin_amdgcn_permlane16_swap(s0[0], s0[1], false, false);
  auto t1 = __builtin_amdgcn_permlane16_swap(s1[0], s1[1], false, false);
  return make_uint4(t0[0], t1[0], t0[1], t1[1]);
}
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

struct LabArgs {
  const bf16* a;
  const bf16* b;
  bf16* c;
  int M, N, K, ntm, ntn, gm;
};

// Byte offset, inside an operand's K-step image, of 16-B chunk c of tile row r.
template <int LAYOUT>
__device__ __forceinline__ int img(int r, int c) {
  if constexpr (LAYOUT == 1) return (r & 31) * Lay<1>::BLK + 128 * (r >> 5) + 16 * c;
  else return 128 * r + 16 * (c ^ ((r >> 1) & 7));
}

// Vendor-style slot plans (SCHED 1 / 2): events after MFMA index S of a
// K-step, [parity][event]; parity = SIMD id bit 0 for SCHED 2 (the two SIMDs
// of one LDS/TA half run orders shifted by one MFMA), 0 for every wave in
// SCHED 1.  Operand X = A (read k-half 1 before barrier 1, refilled after it),
// Y = B (read between the barriers, refilled after barrier 2).
struct VPlan {
  int rd1[16];   // k-half-1 reads: 0..7 A frags, 8..15 B frags
  int dma[16];   // DMA pieces: 0..7 A, 8..15 B
  int rd0[16];   // next step's k-half-0 reads
  int b1, b2, w;
};
constexpr VPlan kVPlan[7] = {
    {{0, 2, 4, 6, 8, 10, 12, 14, 24, 27, 30, 33, 36, 38, 40, 42},
     {22, 25, 28, 31, 34, 52, 55, 58, 61, 64, 85, 87, 89, 96, 100, 124},
     {93, 94, 95, 97, 98, 102, 103, 104, 105, 106, 109, 112, 114, 117, 120, 123},
     20, 50, 91},
    {{0, 2, 4, 6, 8, 10, 12, 14, 22, 25, 28, 31, 34, 38, 40, 42},
     {23, 26, 29, 32, 35, 53, 56, 59, 62, 65, 84, 86, 88, 95, 99, 123},
     {93, 94, 96, 97, 98, 102, 103, 104, 105, 106, 109, 112, 114, 117, 120, 122},
     20, 51, 91},
    // 2: all 16 pieces before a later wait (slot 107), k-half-0 reads packed after it
    {{0, 2, 4, 6, 8, 10, 12, 14, 24, 27, 30, 33, 36, 38, 40, 42},
     {22, 25, 28, 31, 34, 52, 55, 58, 61, 64, 85, 87, 89, 92, 96, 100},
     {108, 109, 110, 111, 112, 113, 114, 115, 116, 117, 118, 119, 120, 121, 122, 123},
     20, 50, 107},
    // 3: dense bursts right after each refill barrier, wait at 91
    {{0, 2, 4, 6, 8, 10, 12, 14, 24, 27, 30, 33, 36, 38, 40, 42},
     {21, 23, 25, 27, 29, 31, 33, 35, 51, 53, 55, 57, 59, 61, 63, 65},
     {93, 94, 95, 97, 98, 102, 103, 104, 105, 106, 109, 112, 114, 117, 120, 123},
     20, 50, 91},
    // 4: the vendor plan with its wait (and the reads behind it) 8 MFMAs later
    {{0, 2, 4, 6, 8, 10, 12, 14, 24, 27, 30, 33, 36, 38, 40, 42},
     {22, 25, 28, 31, 34, 52, 55, 58, 61, 64, 85, 87, 89, 104, 108, 124},
     {101, 102, 103, 105, 106, 108, 109, 110, 111, 112, 113, 115, 116, 118, 120, 123},
     20, 50, 99},
    // 5: two barriers per K-step: all 16 k-half-1 reads before barrier 1, all
    //    16 pieces after it (every 4 MFMAs), wait at 95
    {{0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20, 22, 24, 26, 28, 30},
     {34, 38, 42, 46, 50, 54, 58, 62, 66, 70, 74, 78, 82, 86, 90, 94},
     {96, 98, 100, 102, 104, 106, 108, 110, 112, 114, 116, 118, 120, 122, 124, 126},
     32, -1, 95},
    // 6: as 5 with the pieces every 3 MFMAs (34..79)
    {{0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20, 22, 24, 26, 28, 30},
     {34, 37, 40, 43, 46, 49, 52, 55, 58, 61, 64, 67, 70, 73, 76, 79},
     {96, 98, 100, 102, 104, 106, 108, 110, 112, 114, 116, 118, 120, 122, 124, 126},
     32, -1, 95},
};
constexpr int vplan_vmw(int par) {
  int n = 0;
  for (int q = 0; q < 16; ++q) n += kVPlan[par].dma[q] <= kVPlan[par].w;
  return n;
}

// ADDR 1 (LAYOUT 0 only): the vendor's DMA addressing, one per-lane offset
// VGPR per operand (the piece's lane pattern is the same for every piece) and
// the piece's row block in the SGPR soffset.
template <int LAYOUT, int SCHED = 0, int ADDR = 0>
__global__ void __launch_bounds__(256, 1) lab_nt_k(LabArgs p) {
  typedef Lay<LAYOUT> L;
  __shared__ __attribute__((aligned(1024))) char lds[2 * L::SLOTB];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = p.ntm * p.ntn;
  const int G = gridDim.x, bid = blockIdx.x;
  if (bid >= ntiles) return;
  const int nmine = (ntiles - 1 - bid) / G + 1;
  const int M = p.M, N = p.N;
  const int nt = p.K / BK;

  // DMA piece i (0..7) of this wave: 8 rows x 128 B, lane-linear in LDS at
  // byte dst_of(i); lane l fetches tile row row_of(i, l), chunk chunk_of(l).
  uint32_t off[16];
  int dsti[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    int tr, c;
    if constexpr (LAYOUT == 1) {
      const int b = 4 * i + wave;  // block
      tr = b + 32 * (lane >> 3);
      c = lane & 7;
      dsti[i] = b * L::BLK;
    } else if constexpr (LAYOUT >= 2) {
      const int b = 4 * i + wave;  // block = 8 consecutive rows
      tr = 8 * b + (lane >> 3);
      c = lane & 7;
      dsti[i] = b * L::BLK;
    } else {
      const int pb = 4 * i + wave;  // 8-row block of piece i
      tr = 8 * pb + (lane >> 3);
      c = (lane & 7) ^ ((tr >> 1) & 7);
      dsti[i] = pb * 1024;
    }
    off[i] = (uint32_t)(tr * p.K + 8 * c) * 2u;
    off[8 + i] = (uint32_t)(tr * p.K + 8 * c) * 2u;
  }
  auto tile_org = [&](int i, int64_t& m0, int64_t& n0) {
    const int base = i * G, rem = min(G, ntiles - base);
    const int lin = base + xcd_remap(bid, rem);
    const int2 tt = tile_of(lin, p.ntm, p.ntn, p.gm);
    m0 = (int64_t)tt.x * TM;
    n0 = (int64_t)tt.y * TN;
  };
  auto make_rsrc = [&](int i, Rsrc& ra, Rsrc& rb) {
    int64_t m0 = 0, n0 = 0, na = 0, nb = 0;
    if (i < nmine) {
      tile_org(i, m0, n0);
      na = (int64_t)(M - m0) * p.K * 2;
      nb = (int64_t)(N - n0) * p.K * 2;
    }
    ra = __builtin_amdgcn_make_buffer_rsrc((void*)(p.a + m0 * p.K), 0, (int)min(na, (int64_t)0x7fffffff), 0x00020000);
    rb = __builtin_amdgcn_make_buffer_rsrc((void*)(p.b + n0 * p.K), 0, (int)min(nb, (int64_t)0x7fffffff), 0x00020000);
  };
  char* const ldsp = lds;
  const uint32_t piece_stride = (uint32_t)(32 * p.K * 2);  // 32 rows, bytes
  auto dma = [&](int q, Rsrc r, uint32_t soff, int slot) {
    const int dst = slot * L::SLOTB + (q >= 8 ? L::OPB : 0) + dsti[q & 7];
    if constexpr (ADDR == 1 && LAYOUT == 0) {
      const uint32_t so2 = __builtin_amdgcn_readfirstlane(soff + (uint32_t)(q & 7) * piece_stride);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(ldsp + dst),
                                               16, off[0], so2, 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(ldsp + dst),
                                               16, off[q], soff, 0, 0);
    }
  };

  f32x4 acc[8][8];
  const uint32_t lds_base = (uint32_t)(uintptr_t)lds;
  const int fr = lane & 15, fc = lane >> 4;
  // fragment F (16 rows 16 F .. of the wave's 128-row band), k-half KH:
  // lane base + compile-time immediate
  uint32_t abase, bbase;
  if constexpr (LAYOUT == 1) {
    abase = lds_base + fr * L::BLK + 16 * fc + 512 * wm;
    bbase = lds_base + L::OPB + fr * L::BLK + 16 * fc + 512 * wn;
  } else if constexpr (LAYOUT >= 2) {
    // fragment j, lane x: row 8 x + j of the band (block 16 band + x, slot j)
    abase = lds_base + (16 * wm + fr) * L::BLK + 16 * fc;
    bbase = lds_base + L::OPB + (16 * wn + fr) * L::BLK + 16 * fc;
  } else {
    abase = lds_base + 128u * (128u * wm + fr);
    bbase = lds_base + L::OPB + 128u * (128u * wn + fr);
  }
  // LAYOUT 0: the chunk XOR depends on the lane; two bases per k-half
  uint32_t xo[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh) xo[kh] = 16u * (uint32_t)((fc + 4 * kh) ^ ((fr >> 1) & 7));
  X8 set0[16], set1[16];
  auto read_frag = [&](X8 (&dst)[16], auto f, auto kh, uint32_t so) {
    constexpr int F = decltype(f)::value, KH = decltype(kh)::value, FF = F & 7;
    const uint32_t base = (F < 8 ? abase : bbase) + so;
    if constexpr (LAYOUT == 1) {
      constexpr int OFF = 16 * Lay<1>::BLK * (FF & 1) + 128 * (FF >> 1) + 64 * KH;
      dst[F] = row_read_imm<OFF>(base);
    } else if constexpr (LAYOUT >= 2) {
      dst[F] = row_read_imm<128 * FF + 64 * KH>(base);
    } else {
      dst[F] = row_read_imm<2048 * FF>(base + xo[KH]);
    }
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;

  Rsrc ra_c, rb_c, ra_n, rb_n;
  make_rsrc(0, ra_c, rb_c);
  make_rsrc(1, ra_n, rb_n);
  static_for<8>([&](auto q) { dma(decltype(q)::value, ra_c, 0u, 0); });
  static_for<8>([&](auto q) { dma(8 + decltype(q)::value, rb_c, 0u, 0); });
  static_for<8>([&](auto q) { dma(decltype(q)::value, ra_c, BK * 2, 1); });
  static_for<8>([&](auto q) { dma(8 + decltype(q)::value, rb_c, BK * 2, 1); });
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  static_for<16>([&](auto f) { read_frag(set0, f, K0{}, 0u); });
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  int simd_par = 0;
  if constexpr (SCHED == 2) {
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID, 4, 1)" : "=s"(simd_par));
  }
  auto run = [&](auto parc) {
  constexpr int PAR = SCHED >= 3 ? SCHED - 1 : decltype(parc)::value;
  int par = 0;
  for (int i = 0; i < nmine; ++i) {
    auto kstep = [&](int t, auto zero) {
      const int slot = (t + par) & 1;
      const uint32_t so = (uint32_t)(slot * L::SLOTB), sn = (uint32_t)(L::SLOTB - so);
      const bool here = t + 2 < nt;
      const Rsrc ra = here ? ra_c : ra_n, rb = here ? rb_c : rb_n;
      const uint32_t soff = (uint32_t)((here ? t + 2 : t + 2 - nt) * BK * 2);
      if constexpr (SCHED == 0) {
      // the production slot plan of gemm_nt6_k (MODE 0)
      constexpr int B1 = 17, B2 = 35, DA = B1 + 2, SA1 = 4, DB = B2 + 2, SB1 = 8, W = 95;
      auto cnt = [](int d, int st, int w) constexpr {
        int n = 0;
        for (int k = 0; k < 8; ++k) n += d + st * k <= w;
        return n;
      };
      constexpr int VMW = cnt(DA, SA1, W) + cnt(DB, SB1, W);
      static_for<128>([&](auto sc) {
        constexpr int S = decltype(sc)::value, IDX = S & 63;
        // acc[I][J]: I = A (m) fragment, J = B (n) fragment
        constexpr int I = LAYOUT >= 2 ? IDX % 8 : IDX / 8, J = LAYOUT >= 2 ? IDX / 8 : IDX % 8;
        if constexpr (S < 64) {
          if constexpr (decltype(zero)::value) mfma_acc0(acc[I][J], set0[8 + J], set0[I]);
          else mfma_acc(acc[I][J], set0[8 + J], set0[I]);
        } else {
          mfma_acc(acc[I][J], set1[8 + J], set1[I]);
        }
        if constexpr (S < 16 && S % 2 == 0) read_frag(set1, std::integral_constant<int, S / 2>{}, K1{}, so);
        if constexpr (S == B1 || S == B2) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (S > B1 && S <= B1 + 15 && (S - B1 - 1) % 2 == 0)
          read_frag(set1, std::integral_constant<int, 8 + (S - B1 - 1) / 2>{}, K1{}, so);
        if constexpr (S >= DA && (S - DA) % SA1 == 0 && (S - DA) / SA1 < 8) dma((S - DA) / SA1, ra, soff, slot);
        if constexpr (S >= DB && (S - DB) % SB1 == 0 && (S - DB) / SB1 < 8) dma(8 + (S - DB) / SB1, rb, soff, slot);
        if constexpr (S == W) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VMW) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (S > W && S < 127) {
          static_for<16>([&](auto kc) {
            constexpr int Kr = decltype(kc)::value;
            if constexpr (W + 1 + (Kr * (126 - W)) / 16 == S)
              read_frag(set0, std::integral_constant<int, Kr>{}, K0{}, sn);
          });
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      } else {
      constexpr VPlan P = kVPlan[PAR];
      constexpr int VMW = vplan_vmw(PAR);
      static_for<128>([&](auto sc) {
        constexpr int S = decltype(sc)::value, IDX = S & 63;
        constexpr int I = LAYOUT >= 2 ? IDX % 8 : IDX / 8, J = LAYOUT >= 2 ? IDX / 8 : IDX % 8;
        if constexpr (S < 64) {
          if constexpr (decltype(zero)::value) mfma_acc0(acc[I][J], set0[8 + J], set0[I]);
          else mfma_acc(acc[I][J], set0[8 + J], set0[I]);
        } else {
          mfma_acc(acc[I][J], set1[8 + J], set1[I]);
        }
        static_for<16>([&](auto ec) {
          constexpr int E = decltype(ec)::value;
          if constexpr (P.rd1[E] == S) read_frag(set1, std::integral_constant<int, E>{}, K1{}, so);
          if constexpr (P.dma[E] == S) dma(E, E < 8 ? ra : rb, soff, slot);
          if constexpr (P.rd0[E] == S) read_frag(set0, std::integral_constant<int, E>{}, K0{}, sn);
        });
        if constexpr (S == P.b1 || S == P.b2) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (S == P.w) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"i"(VMW) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    kstep(0, std::true_type{});
    for (int t = 1; t < nt; ++t) kstep(t, std::false_type{});

    fa::mfma_drain();
    int64_t m0, n0;
    tile_org(i, m0, n0);
    const int q = lane >> 4;
    if constexpr (LAYOUT >= 2) {
      // acc[a][b] lane l: row 8 (l & 15) + a, cols 32 q + 8 e + b (e = element):
      // 16-B piece e of the lane's 32 columns = {acc[a][0..7][e]}
#pragma unroll
      for (int a = 0; a < 8; ++a) {
        const int64_t row = m0 + 128 * wm + 8 * (lane & 15) + a;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          fa::MT<bf16>::x8 v;
#pragma unroll
          for (int b = 0; b < 8; ++b) v[b] = (bf16)acc[a][b][e];
          const int64_t col = n0 + 128 * wn + 32 * q + 8 * e;
          if (row < M && col < N) *reinterpret_cast<fa::MT<bf16>::x8*>(p.c + row * N + col) = v;
        }
      }
    } else {
#pragma unroll
    for (int ii = 0; ii < 8; ++ii) {
      const int64_t row = m0 + 128 * wm + 16 * ii + (lane & 15);
#pragma unroll
      for (int jp = 0; jp < 4; ++jp) {
        const uint4 v = pair_to_row8(pack4(acc[ii][2 * jp]), pack4(acc[ii][2 * jp + 1]));
        const int64_t col = n0 + 128 * wn + 32 * jp + 8 * q;
        if (row < M && col < N) *reinterpret_cast<uint4*>(p.c + row * N + col) = v;
      }
    }
    }
    par ^= nt & 1;
    ra_c = ra_n;
    rb_c = rb_n;
    make_rsrc(i + 2, ra_n, rb_n);
  }
  };
  if (simd_par) run(std::integral_constant<int, SCHED == 2 ? 1 : 0>{});
  else run(std::integral_constant<int, 0>{});
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int num_cus_lab() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

}  // namespace

// variant: 0 = production layout, 1 = linear-source padded layout.
// Host-checked by the binding: bf16, contiguous, K % 64 == 0, K >= 128,
// M * K * 2 and N * K * 2 < 2^31.
void gemm_lab(const void* a, const void* b, void* c, int64_t M, int64_t N, int64_t K, int variant,
              hipStream_t s) {
  LabArgs p{(const bf16*)a, (const bf16*)b, (bf16*)c, (int)M, (int)N, (int)K, 0, 0, 0};
  p.ntm = (p.M + TM - 1) / TM;
  p.ntn = (p.N + TN - 1) / TN;
  p.gm = p.ntm <= p.ntn ? 8 : -8;
  const int g = std::min(p.ntm * p.ntn, num_cus_lab());
  if (variant == 7) hipLaunchKernelGGL((lab_nt_k<0, 1, 1>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 8) hipLaunchKernelGGL((lab_nt_k<2, 1>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 10) hipLaunchKernelGGL((lab_nt_k<0, 3>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 11) hipLaunchKernelGGL((lab_nt_k<0, 4>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 12) hipLaunchKernelGGL((lab_nt_k<0, 5>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 13) hipLaunchKernelGGL((lab_nt_k<0, 6>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 14) hipLaunchKernelGGL((lab_nt_k<0, 7>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 9) hipLaunchKernelGGL((lab_nt_k<3, 1>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 4) hipLaunchKernelGGL((lab_nt_k<0, 1>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 5) hipLaunchKernelGGL((lab_nt_k<0, 2>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 6) hipLaunchKernelGGL((lab_nt_k<3, 2>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 1) hipLaunchKernelGGL((lab_nt_k<1>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 2) hipLaunchKernelGGL((lab_nt_k<2>), dim3(g), dim3(256), 0, s, p);
  else if (variant == 3) hipLaunchKernelGGL((lab_nt_k<3>), dim3(g), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((lab_nt_k<0>), dim3(g), dim3(256), 0, s, p);
}

}  // namespace ema
