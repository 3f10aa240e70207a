// 2-D transpose of 16-bit matrices through LDS (gfx950, wave64).
//
// Used to keep a K-contiguous copy W^T of every linear weight so the
// input-gradient GEMM dX = dY W runs in hipBLASLt's fastest ("TN") operand
// layout: profiles/r1_gemm_layouts_hipblaslt.json measures dY @ (W^T)^T at
// 1544-1612 TFLOP/s against 1343-1405 for dY @ W on the Llama-2-7B shapes.
// The copy is refreshed once per optimizer step, so its cost (one read + one
// write of the bf16 weights) is amortised over every micro-batch.  The same
// kernel can transpose activations for a TN weight-gradient GEMM.
//
// Tile 64 x 64 elements per 256-thread block: each lane loads 16 bytes
// (8 consecutive columns) of two source rows, scatters them into a padded LDS
// tile (pitch 65 halves -> conflict-free column reads), then gathers 8
// consecutive source rows of one column and stores them as one 16-byte vector
// of the destination row.  Global traffic is 16 B/lane in both directions.
// Host code guarantees rows % 64 == 0 and cols % 64 == 0.
#include "common.h"

namespace ema {
namespace {

constexpr int TT = 64;       // tile edge
constexpr int TP = TT + 1;   // LDS pitch (halves)

__global__ void __launch_bounds__(256) transpose16_k(const uint16_t* __restrict__ src,
                                                     uint16_t* __restrict__ dst, int64_t rows,
                                                     int64_t cols) {
  __shared__ uint16_t tile[TT * TP];
  const int tiles_c = (int)(cols / TT);
  const int nwg = gridDim.x;
  const int t_id = xcd_remap((int)blockIdx.x, nwg);
  const int64_t r0 = (int64_t)(t_id / tiles_c) * TT;
  const int64_t c0 = (int64_t)(t_id % tiles_c) * TT;
  const int tid = threadIdx.x;
  // load: 64 rows x 8 vectors; thread handles rows (tid / 8) and (tid / 8 + 32)
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int r = (tid >> 3) + it * 32;
    const int c = (tid & 7) * 8;
    const V16<uint16_t> v = ld16(src + (r0 + r) * cols + c0 + c);
#pragma unroll
    for (int i = 0; i < 8; ++i) tile[r * TP + c + i] = v.v[i];
  }
  __syncthreads();
  // store: destination row = source column (tid % 64), 8 source rows per vector
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = tid & 63;
    const int rg = ((tid >> 6) + it * 4) * 8;
    V16<uint16_t> v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v.v[i] = tile[(rg + i) * TP + c];
    st16(dst + (c0 + c) * rows + r0 + rg, v);
  }
}

}  // namespace

bool transpose16_supported(int64_t rows, int64_t cols) {
  return rows > 0 && cols > 0 && rows % TT == 0 && cols % TT == 0 &&
         (rows / TT) * (cols / TT) < (int64_t)0x7fffffff;
}

void transpose16(const void* src, void* dst, int64_t rows, int64_t cols, hipStream_t stream) {
  const int64_t n = (rows / TT) * (cols / TT);
  hipLaunchKernelGGL(transpose16_k, dim3((unsigned)n), dim3(256), 0, stream,
                     (const uint16_t*)src, (uint16_t*)dst, rows, cols);
}

}  // namespace ema
