// Weight-stream layout experiment for the decode GEMV.
//
// Question: does the address pattern of the MFMA A-operand loads limit the
// skinny GEMM's HBM rate?  With W row-major [N, K] and the 16x16x32 operand
// layout (lane L: row L & 15, 8 k at 8 (L >> 4)), every 4-lane quad of a
// global_load_dwordx4 touches 4 different rows and a 16-lane quarter 16
// different cache lines.  A pre-packed W (each wave-instruction's 1 KiB
// contiguous, lane L at byte 16 L) is read by the same MFMA schedule.
//
//   mode 0: row-major W, the production lane map (16 rows x 64 B per instr)
//   mode 1: packed W (1 KiB contiguous per instr, same ring / MFMAs)
//   mode 2: packed W, plain (temporal) loads
//   mode 3: row-major W, plain loads
//   mode 4: packed W, no MFMA (pure stream, xor-reduce)
// N x K bf16, 8 waves x U loads in flight, persistent grid = CUs; the
// buffer rotates over NB copies (> the 256 MiB MALL) so every pass is HBM.
// Build: hipcc -O3 --offload-arch=gfx950 -o gemv_layout_bench gemv_layout_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf8;
typedef __attribute__((ext_vector_type(4))) float f4;
typedef __attribute__((ext_vector_type(4))) unsigned u4;

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                \
    }                                                                         \
  } while (0)

template <int MODE, int U>
__global__ __launch_bounds__(512) void gemv_k(const __bf16* __restrict__ w, const __bf16* __restrict__ x,
                                              float* __restrict__ y, int N, int K) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int steps = K / 256;  // k-steps of 32 per wave (K split over 8 waves)
  const int nblk = N / 16;
  const int r = lane & 15, q = lane >> 4;
  bf8 xv = *reinterpret_cast<const bf8*>(x + wave * steps * 32 + 8 * q);
  f4 acc = {0, 0, 0, 0};
  u4 xr = {0, 0, 0, 0};
  for (int b = blockIdx.x; b < nblk; b += gridDim.x) {
    const __bf16* base;
    int64_t stride;
    if constexpr (MODE == 0 || MODE == 3) {
      base = w + ((int64_t)b * 16 + r) * K + wave * steps * 32 + 8 * q;
      stride = 32;
    } else {
      // packed: block b, wave, step s -> 1 KiB at ((b * 8 + wave) * steps + s) KiB
      base = w + ((int64_t)b * 8 + wave) * steps * 512 + 8 * lane;
      stride = 512;
    }
    bf8 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u >= steps) {  // ring deeper than the wave's k-steps: never read past them
        a[u] = bf8{};
        continue;
      }
      if constexpr (MODE == 2 || MODE == 3) a[u] = *reinterpret_cast<const bf8*>(base + stride * u);
      else a[u] = __builtin_nontemporal_load(reinterpret_cast<const bf8*>(base + stride * u));
    }
    for (int s0 = 0; s0 < steps; s0 += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (MODE == 4) {
          xr ^= __builtin_bit_cast(u4, a[u]);
        } else {
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], xv, acc, 0, 0, 0);
        }
        const int s = s0 + U + u;
        if (s < steps) {
          if constexpr (MODE == 2 || MODE == 3) a[u] = *reinterpret_cast<const bf8*>(base + stride * s);
          else a[u] = __builtin_nontemporal_load(reinterpret_cast<const bf8*>(base + stride * s));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  if (MODE == 4) acc[0] = (float)(xr[0] ^ xr[1] ^ xr[2] ^ xr[3]);
  y[blockIdx.x * 512 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int MODE, int U = 16>
float run(const std::vector<__bf16*>& bufs, const __bf16* x, float* y, int N, int K, int cus) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 40;
  for (int i = 0; i < 8; ++i)
    hipLaunchKernelGGL((gemv_k<MODE, U>), dim3(cus), dim3(512), 0, 0, bufs[i % bufs.size()], x, y, N, K);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; ++i)
    hipLaunchKernelGGL((gemv_k<MODE, U>), dim3(cus), dim3(512), 0, 0, bufs[i % bufs.size()], x, y, N, K);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  int cus = 256;
  int dev = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  struct Shape { const char* name; int N, K; };
  const Shape shapes[] = {{"qkv", 12288, 4096}, {"o", 4096, 4096}, {"fc1", 22016, 4096}, {"fc2", 4096, 11008 / 256 * 256}};
  float* y;
  __bf16* x;
  CK(hipMalloc(&y, (size_t)4 * cus * 512 * 4));  // grids up to 4 x CUs
  CK(hipMalloc(&x, 16384 * 2));
  CK(hipMemset(x, 0, 16384 * 2));
  for (const Shape& sh : shapes) {
    const size_t bytes = (size_t)sh.N * sh.K * 2;
    const int nb = (int)((1536ull << 20) / bytes) + 1;  // > 1.5 GiB rotating
    std::vector<__bf16*> bufs(nb);
    for (auto& b : bufs) {
      CK(hipMalloc(&b, bytes));
      CK(hipMemset(b, 0, bytes));
    }
    float t[9];
    t[0] = run<0>(bufs, x, y, sh.N, sh.K, cus);
    t[1] = run<1>(bufs, x, y, sh.N, sh.K, cus);
    t[2] = run<2>(bufs, x, y, sh.N, sh.K, cus);
    t[3] = run<3>(bufs, x, y, sh.N, sh.K, cus);
    t[4] = run<4>(bufs, x, y, sh.N, sh.K, cus);
    t[5] = run<1, 8>(bufs, x, y, sh.N, sh.K, cus);
    t[6] = run<1, 32>(bufs, x, y, sh.N, sh.K, cus);
    t[7] = run<1>(bufs, x, y, sh.N, sh.K, 2 * cus);
    t[8] = run<1, 8>(bufs, x, y, sh.N, sh.K, 2 * cus);
    printf("%-4s N=%5d K=%5d %6.1f MB:\n", sh.name, sh.N, sh.K, bytes / 1e6);
    const char* names[] = {"rowmajor_nt", "packed_nt", "packed_plain", "rowmajor_plain", "packed_nomfma",
                           "packed_nt_U8", "packed_nt_U32", "packed_nt_2wg", "packed_nt_U8_2wg"};
    for (int m = 0; m < 9; ++m) printf("    %-18s %6.2f us %5.2f TB/s\n", names[m], t[m] * 1e3, bytes / (t[m] * 1e-3) / 1e12);
    for (auto& b : bufs) CK(hipFree(b));
  }
  return 0;
}
