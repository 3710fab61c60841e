// Diagnostic (not product): issue rate of v_mfma_f32_16x16x32_f16 vs
// v_mfma_scale_f32_16x16x128_f8f6f4 (fp8) vs v_mfma_f32_16x16x128_f8f6f4-free fp8 16x16x32:
// 8 independent accumulator chains per wave, 4 waves per SIMD-less block, timed with events;
// and v_mfma_f32_32x32x16_f16 with 4 chains.
//   hipcc --offload-arch=gfx950 -O3 tools/diag/mfma_rate.hip -o tools/diag/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef int i8v __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef long l1;

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
  f4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  h8 a = (h8)(_Float16)(threadIdx.x * 1e-3f), b = (h8)(_Float16)1.f;
  i8v ia = (i8v)(int)(threadIdx.x | 0x38383838), ib = (i8v)0x38383838;
  long la = 0x3838383838383838l, lb = la + threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (MODE == 0) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[i], 0, 0, 0);
      else if constexpr (MODE == 1)
        acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(ia, ib, acc[i], 0, 0, 0, 127, 0, 127);
      else acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(la, lb, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 32x32x16 f16 (MODE 3): 4 independent 16-float accumulator chains per wave
__global__ __launch_bounds__(256) void k32(float* out, int iters) {
  f16v acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = (f16v)0.f;
  h8 a = (h8)(_Float16)(threadIdx.x * 1e-3f), b = (h8)(_Float16)1.f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

double run32(float* d, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8;
  hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)blocks * 4 * iters * 4 * (32.0 * 32 * 16 * 2);
  return flops / (ms * 1e-3) / 1e12;
}

template <int MODE>
double run(float* d, int iters, double flop_per) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8;  // 8 waves-of-4 per CU -> 8 waves per SIMD
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double flops = (double)blocks * 4 * iters * 8 * flop_per;
  return flops / (ms * 1e-3) / 1e12;
}

int main() {
  float* d;
  (void)hipMalloc(&d, 256 * 8 * 256 * 4);
  const int iters = 4000;
  printf("f16 16x16x32        : %.0f TF/s\n", run<0>(d, iters, 16.0 * 16 * 32 * 2));
  printf("mx fp8 16x16x128    : %.0f TF/s\n", run<1>(d, iters, 16.0 * 16 * 128 * 2));
  printf("fp8 16x16x32        : %.0f TF/s\n", run<2>(d, iters, 16.0 * 16 * 32 * 2));
  printf("f16 32x32x16        : %.0f TF/s\n", run32(d, iters));
  printf("f16 16x16x32 (again): %.0f TF/s\n", run<0>(d, iters, 16.0 * 16 * 32 * 2));
  return 0;
}
