// Diagnostic (not product): global store throughput of the GEMM epilogue's 16-byte store layout
// vs a line-contiguous layout, at different numbers of active CUs (one 8-wave workgroup per CU),
// writing 256 x 256 fp16 tiles into an M x 3072 fp16 matrix (the FFN1 output shape).
//   hipcc --offload-arch=gfx950 -O3 tools/diag/store_rate.hip -o tools/diag/store_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
constexpr int LDY = 3072, TN = LDY / 256;

template <int LAYOUT>
__global__ __launch_bounds__(512) void k(_Float16* __restrict__ Y, int tiles_per_wg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wn = wave >> 2, wm = wave & 3, g = lane >> 4, odd = g & 1;
  h8 v = (h8)(_Float16)(lane * 0.001f);
  for (int k = 0; k < tiles_per_wg; ++k) {
    const int t = blockIdx.x + k * gridDim.x;
    const long m0 = (long)(t / TN) * 256, n0 = (long)(t % TN) * 256;
    if (LAYOUT == 0) {  // the wide epilogue: 16 rows x 64 B per store instruction
      const long nl = n0 + wn * 128 + 16 * odd + 4 * (g & 2);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const long m = m0 + wm * 64 + j * 16 + (lane & 15);
          *reinterpret_cast<h8*>(Y + m * LDY + nl + 32 * p) = v;
        }
    } else {  // line-contiguous: each instruction writes 2 rows x 512 B (whole 128-B lines)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = wave * 32 + i * 2 + (lane >> 5);
        *reinterpret_cast<h8*>(Y + (m0 + r) * LDY + n0 + (lane & 31) * 8) = v;
      }
    }
    v += (h8)(_Float16)1.f;
  }
}

int main() {
  const int tiles_total = 24576;  // M = 524288 rows x 3072 columns (3.2 GB)
  _Float16* Y;
  hipMalloc(&Y, (size_t)tiles_total / TN * 256 * LDY * 2);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int layout = 0; layout < 2; ++layout)
    for (int G : {8, 32, 64, 128, 256}) {
      const int per = 64;                      // tiles per workgroup (8 MiB)
      auto launch = [&] {
        if (layout == 0) hipLaunchKernelGGL(k<0>, dim3(G), dim3(512), 0, 0, Y, per);
        else hipLaunchKernelGGL(k<1>, dim3(G), dim3(512), 0, 0, Y, per);
      };
      launch();
      hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double bytes = 5.0 * G * per * 256.0 * 256 * 2;
      printf("layout %s G=%3d: %8.1f GB/s total, %6.2f GB/s per WG (%.2f B/clk at 1.7 GHz)\n",
             layout ? "lines   " : "epilogue", G, bytes / ms / 1e6, bytes / ms / 1e6 / G,
             bytes / ms / 1e6 / G / 1.7);
    }
  hipFree(Y);
  return 0;
}
