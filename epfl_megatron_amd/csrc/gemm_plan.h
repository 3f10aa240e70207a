// Shared K-step slot plan of the persistent 4-wave 256x256 GEMMs
// (gemm_nt.hip gemm_nt6_k, gemm_wgrad.hip wgrad4_k): one K-step = 128 MFMAs
// per wave over two register fragment sets (k-half 0 / 1), two LDS slots.
#pragma once

namespace ema {

// K-step slot plan of the persistent kernel: the event lists say after which
// MFMA (0..127) of a K-step each fragment read / DMA piece / barrier issues.
//   rd1: the 16 k-half-1 fragments (0..7 A, 8..15 B) from the current slot:
//        A before barrier b1, B between b1 and b2;
//   dma: the 16 pieces of step t+2 into the current slot: A after b1 (every
//        wave has read A's k-half 1), B after b2; 13 of them before w;
//   w:   vmcnt(13) + barrier: step t+1 landed (own DMA, then everyone's);
//   rd0: the next step's k-half-0 fragments from the other slot, after w.
// (the vendor 256x256 kernel's placement, measured in scripts/gemm_lab.py:
// one load burst right after each refill barrier, B's last three pieces
// after the wait)
struct NtPlan {
  int rd1[16], dma[16], rd0[16];
  int b1, b2, w;
};
inline constexpr NtPlan kNtPlan = {
    {0, 2, 4, 6, 8, 10, 12, 14, 24, 27, 30, 33, 36, 38, 40, 42},
    {22, 25, 28, 31, 34, 52, 55, 58, 61, 64, 85, 87, 89, 96, 100, 124},
    {93, 94, 95, 97, 98, 102, 103, 104, 105, 106, 109, 112, 114, 117, 120, 123},
    20, 50, 91};
inline constexpr int nt_plan_vmw() {
  int n = 0;
  for (int q = 0; q < 16; ++q) n += kNtPlan.dma[q] <= kNtPlan.w;
  return n;
}
static_assert(nt_plan_vmw() == 13, "pieces issued before the step-t+1 wait");

}  // namespace ema
