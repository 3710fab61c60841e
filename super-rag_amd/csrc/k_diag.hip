// Diagnostic kernels (libsrmi_diag.so only, SR_WITH_DIAG): the MFMA issue-rate peak the GEMM
// rooflines are read against ("the MFMA peak measured on the box").
//
// mfma_rate: every CU runs 8 waves (2 per SIMD, the product GEMMs' occupancy), each with 8
// independent accumulator chains of the product's MFMA shape (f16: v_mfma_f32_16x16x32_f16; fp8:
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 scales) fed by 4 + 4 operand registers of
// hashed random data (full-range f16 below 2, e4m3 bytes without NaN: the multipliers toggle as on
// real operands -- zero or constant operands let the chip hold a higher clock,
// cdna_hip_programming.md §5.4 rule 25).  No memory traffic in the loop.  Wave 0 of every block
// stamps s_memtime (shader clock) and s_memrealtime (100 MHz) around its loop; the clock it held
// is d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md: the in-kernel clock recipe).
#include "sr_common.h"
#include "sr_kernels.h"

#if SR_WITH_DIAG
namespace sr {

namespace {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef int i8vv __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

template <bool F8>
__global__ __launch_bounds__(512) void mfma_rate_kernel(float* __restrict__ sink, uint64_t* __restrict__ stamps,
                                                        int iters) {
  const uint32_t seed = (blockIdx.x * 512u + threadIdx.x) * 0x9e3779b9u;
  f4v acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = f4v{0.f, 0.f, 0.f, 0.f};
  h8v a16[4], b16[4];
  i8vv a8[4], b8[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t ha = mix32(seed + 131u * r + 17u * e), hb = mix32(seed ^ (0x51ed27u + 977u * r + 29u * e));
      if constexpr (F8) {
        a8[r][e] = (int)(ha & 0xF7F7F7F7u);  // e4m3 bytes, lowest exponent bit clear: never NaN
        b8[r][e] = (int)(hb & 0xF7F7F7F7u);
      } else {
        a16[r][e] = __builtin_bit_cast(_Float16, (unsigned short)(ha & 0xBFFFu));  // |x| < 2
        b16[r][e] = __builtin_bit_cast(_Float16, (unsigned short)(hb & 0xBFFFu));
      }
    }
  }
  uint64_t t0 = 0, r0 = 0;
  if (threadIdx.x == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if constexpr (F8)
        acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8[i & 3], b8[(i >> 1) & 3], acc[i], 0, 0, 0, 127,
                                                                   0, 127);
      else
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a16[i & 3], b16[(i >> 1) & 3], acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  if (threadIdx.x == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    stamps[2 * blockIdx.x] = t1 - t0;       // (vector stores from lane 0)
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
  sink[blockIdx.x * 512 + threadIdx.x] = s;
}

}  // namespace

// FLOP of one launch: blocks x 8 waves x iters x 8 MFMAs x (16 x 16 x K x 2), K = 32 (f16) / 128 (fp8)
void launch_mfma_rate(int f8, int blocks, int iters, float* sink, uint64_t* stamps, hipStream_t st) {
  SR_CHECK(blocks > 0 && iters > 0, "mfma_rate: blocks and iters must be positive");
  if (f8)
    hipLaunchKernelGGL((mfma_rate_kernel<true>), dim3(blocks), dim3(512), 0, st, sink, stamps, iters);
  else
    hipLaunchKernelGGL((mfma_rate_kernel<false>), dim3(blocks), dim3(512), 0, st, sink, stamps, iters);
  SR_LAUNCH_CHECK();
}

}  // namespace sr
#endif
