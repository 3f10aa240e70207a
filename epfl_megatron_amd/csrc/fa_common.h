// Shared pieces of the gfx950 FlashAttention-2 forward/backward kernels.
//
// MFMA: v_mfma_f32_32x32x16_{bf16,f16}.  Fragment maps (CDNA guide §3):
//   A[row = lane&31][k = 8*(lane>>5) + j],  B[k = 8*(lane>>5) + j][col = lane&31]
//   C/D: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5), reg = 0..15.
// An accumulator used as the next MFMA's B operand: registers 8s..8s+7 form
// k-step s with k = 16s + 8(j>>2) + 4h + (j&3) (j = element, h = lane>>5).
#pragma once
#include <utility>

#include "common.h"

namespace ema {
namespace fa {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

template <typename T>
struct MT;
template <>
struct MT<bf16> {
  typedef bf16x8 x8;
  typedef bf16x4 x4;
  static __device__ __forceinline__ f32x16 mfma(x8 a, x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ x4 tr_read(const bf16* lds) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        (__attribute__((address_space(3))) x4*)(lds));
  }
};
template <>
struct MT<fp16> {
  typedef f16x8 x8;
  typedef f16x4 x4;
  static __device__ __forceinline__ f32x16 mfma(x8 a, x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ x4 tr_read(const fp16* lds) {
    typedef __attribute__((ext_vector_type(4))) short s4;
    const s4 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s4*)(lds));
    return __builtin_bit_cast(x4, r);
  }
};

// Inline-asm MFMAs with the accumulator's register class pinned: "+a" for
// loop-carried accumulators that only ever feed further MFMAs (dK/dV/dQ),
// "+v" for short-lived ones read by VALU right after (S, dP).  Left to the
// register allocator, a 1-wave/SIMD kernel with saturated arch VGPRs gets
// its accumulators shuttled AGPR <-> VGPR around every MFMA.
// hipcc pads no hazard inside an asm string (CDNA guide §5.7):
//   * NOP = 1: an operand (A, B or C) was just written by VALU -> s_nop 1;
//   * back-to-back MFMAs accumulating into the same registers need nothing;
//   * VALU / stores reading an MFMA result need 18 wait states: mfma_drain().
template <typename T, int NOP = 0>
__device__ __forceinline__ void mfma_agpr(f32x16& acc, typename MT<T>::x8 a,
                                          typename MT<T>::x8 b) {
  if constexpr (__is_same(T, bf16)) {
    if constexpr (NOP) asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
    else asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  } else {
    if constexpr (NOP) asm("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
    else asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  }
}
template <typename T, int NOP = 0>
__device__ __forceinline__ void mfma_vgpr(f32x16& acc, typename MT<T>::x8 a,
                                          typename MT<T>::x8 b) {
  if constexpr (__is_same(T, bf16)) {
    if constexpr (NOP) asm("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
    else asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  } else {
    if constexpr (NOP) asm("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
    else asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
  }
}
// acc = A * B (C = 0), VGPR destination
template <typename T>
__device__ __forceinline__ f32x16 mfma_vgpr0(typename MT<T>::x8 a, typename MT<T>::x8 b) {
  f32x16 acc;
  if constexpr (__is_same(T, bf16))
    asm("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
  else
    asm("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
  return acc;
}

// Wait states between an asm MFMA and any VALU / store reading its result
// (16-pass XDL op: 18 states, padded to 24).
__device__ __forceinline__ void mfma_drain() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <typename T>
__device__ __forceinline__ typename MT<T>::x8 ld8(const T* p) {
  return *reinterpret_cast<const typename MT<T>::x8*>(p);
}

template <typename T>
__device__ __forceinline__ typename MT<T>::x8 join(typename MT<T>::x4 a, typename MT<T>::x4 b) {
  typename MT<T>::x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}

// ds_read_b64_tr_b16 as inline asm: invisible to hipcc's LDS-DMA alias
// tracking, so no vmcnt(0) is inserted in front of it while a
// global_load_lds into ANOTHER buffer is in flight.  The result is NOT
// tracked either: the consumer must follow lds_wait() (lgkmcnt + a
// sched_barrier so no MFMA is hoisted above the wait, CDNA guide rule 18).
template <typename T>
__device__ __forceinline__ typename MT<T>::x4 tr_read_asm(const T* lds) {
  typename MT<T>::x4 r;
  const uint32_t a = (uint32_t)(uintptr_t)lds;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
// The same with a compile-time byte offset folded into the instruction.
template <int OFF, typename T>
__device__ __forceinline__ typename MT<T>::x4 tr_read_imm(uint32_t base) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset is 16 bits");
  typename MT<T>::x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(base), "i"(OFF));
  return r;
}
// Compile-time loop: f(std::integral_constant<int, i>) for i in [0, N).
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
__device__ __forceinline__ void lds_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Registers 8s..8s+7 of an fp32 accumulator -> operand fragment of k-step s.
template <typename T>
__device__ __forceinline__ typename MT<T>::x8 acc_frag(const f32x16& acc, int s) {
  typename MT<T>::x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (T)acc[8 * s + j];
  return r;
}

// Diagnostics (AttnParams::stamps): 10-ns wall clock, CU and XCD of the wave.
__device__ __forceinline__ unsigned long long wall_stamp() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

__device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// ---- fused RoPE (Meta-Llama interleaved pairs (x[2j], x[2j+1]), fp32) ------
typedef __attribute__((ext_vector_type(2))) float rf2;
typedef __attribute__((ext_vector_type(4))) float rf4;

// Table rows (cos, sin) of sequence row `row` of batch `b`.
template <int HD>
__device__ __forceinline__ void rope_rows(const AttnParams& p, int b, int row, const float*& c,
                                          const float*& s) {
  const int64_t pos = p.rope_pos ? p.rope_pos[(int64_t)b * p.rope_pos_sb + row] : (int64_t)row;
  c = p.rope_cos + pos * (HD / 2);
  s = p.rope_sin + pos * (HD / 2);
}
// R^T on 4 consecutive fp32 elements with their 2 (cos, sin) pairs given.
__device__ __forceinline__ void rope_inv4v(float (&x)[4], rf2 cc, rf2 sn) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float x0 = x[2 * i], x1 = x[2 * i + 1];
    x[2 * i] = x0 * cc[i] + x1 * sn[i];
    x[2 * i + 1] = x1 * cc[i] - x0 * sn[i];
  }
}
// R^T on 4 consecutive fp32 elements starting at head-dim index 2*j0 (j0 even).
__device__ __forceinline__ void rope_inv4(float (&x)[4], const float* c, const float* s, int j0) {
  rope_inv4v(x, *reinterpret_cast<const rf2*>(c + j0), *reinterpret_cast<const rf2*>(s + j0));
}
// The (cos, sin) pairs of an accumulator-layout epilogue row (element groups
// (d, rg) at head-dim d*32 + 8*rg + 4*h), all loaded before any is used: the
// per-group load-then-use form waits out 2 DT 4 L2 round trips, each behind
// the stores already issued (profiles: the dQ epilogue).
template <int DT>
__device__ __forceinline__ void rope_inv_tables(rf2 (&cc)[DT][4], rf2 (&sn)[DT][4], const float* c,
                                                const float* s, int h) {
#pragma unroll
  for (int d = 0; d < DT; ++d)
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int j0 = (d * 32 + 8 * rg + 4 * h) / 2;
      cc[d][rg] = *reinterpret_cast<const rf2*>(c + j0);
      sn[d][rg] = *reinterpret_cast<const rf2*>(s + j0);
    }
}
// R on an 8-element 16-bit fragment with the 4 (cos, sin) pairs given.
template <typename T>
__device__ __forceinline__ typename MT<T>::x8 rope_fwd8v(typename MT<T>::x8 v, rf4 cc, rf4 sn) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = (float)v[2 * i], x1 = (float)v[2 * i + 1];
    v[2 * i] = (T)(x0 * cc[i] - x1 * sn[i]);
    v[2 * i + 1] = (T)(x0 * sn[i] + x1 * cc[i]);
  }
  return v;
}
// R on an 8-element 16-bit fragment starting at head-dim index 2*j0 (j0 % 4 == 0).
template <typename T>
__device__ __forceinline__ typename MT<T>::x8 rope_fwd8(typename MT<T>::x8 v, const float* c,
                                                        const float* s, int j0) {
  return rope_fwd8v<T>(v, *reinterpret_cast<const rf4*>(c + j0), *reinterpret_cast<const rf4*>(s + j0));
}
// R on the KS fragments of one query row (fragment kk at head-dim 16 kk + 8 h):
// every table load issued before any is used (a load-use pair per fragment
// would wait out KS L2 round trips), half of the fragments at a time.
template <typename T, int KS>
__device__ __forceinline__ void rope_rows_fwd(typename MT<T>::x8 (&qf)[KS], const float* c,
                                              const float* s, int h) {
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    rf4 cc[KS / 2], sn[KS / 2];
#pragma unroll
    for (int i = 0; i < KS / 2; ++i) {
      const int j0 = (half * (KS / 2) + i) * 8 + 4 * h;
      cc[i] = *reinterpret_cast<const rf4*>(c + j0);
      sn[i] = *reinterpret_cast<const rf4*>(s + j0);
    }
#pragma unroll
    for (int i = 0; i < KS / 2; ++i) qf[half * (KS / 2) + i] = rope_fwd8v<T>(qf[half * (KS / 2) + i], cc[i], sn[i]);
  }
}

// 16-byte-chunk XOR swizzle for [rows][HD] tiles that are read both by rows
// (ds_read_b128 A/B fragments) and transposed (ds_read_b64_tr_b16): CDNA guide
// T10 image (b) for 256-byte rows; a 3-bit analogue for 128-byte rows.
template <int HD>
__device__ __forceinline__ int swz(int row) {
  if constexpr (HD == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return ((row & 3) << 1) | ((row >> 2) & 1);
}

// Element offset of (row, col) in a swizzled [rows][HD] tile (col multiple of 4).
template <int HD>
__device__ __forceinline__ int sw_off(int row, int col) {
  return row * HD + (((col >> 3) ^ swz<HD>(row)) << 3) + (col & 7);
}

// Image (a) of CDNA guide T10 for [rows][HD] 16-bit tiles: 8-row x 32-column
// (512-B) subtiles with a 2-bit XOR inside each 64-B row piece.  Byte offset
// of 16-B chunk `ch` of row `row`.  Every 32x32x16 row read (ds_read_b128) and
// transposed read (ds_read_b64_tr_b16) of it is conflict-free, and reads that
// differ only in the k-step / d-tile / row-group differ by a lane-independent
// constant (an instruction immediate), so a handful of address VGPRs serve a
// whole tile.
template <int HD>
__device__ __forceinline__ int ia_off(int row, int ch) {
  constexpr int RG = 8 * HD * 2;
  return RG * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}

}  // namespace fa
}  // namespace ema
