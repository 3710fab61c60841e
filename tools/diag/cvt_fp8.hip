// Diagnostic (not product): v_cvt_pk_fp8_f32 (gfx950, OCP e4m3) vs the software e4m3_rne of
// sr_common.h on 2^24 floats spread over the e4m3 range (incl. subnormals, ties, +-448).
//   hipcc --offload-arch=gfx950 -O2 -I super-rag_amd/csrc tools/diag/cvt_fp8.hip -o tools/diag/cvt_fp8
#include <hip/hip_runtime.h>
#include <cstdio>
#include "sr_common.h"

__global__ void k(unsigned* bad, unsigned* first) {
  const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  // a float from the bits: exponents 2^-12 .. 2^9, any mantissa, both signs
  const unsigned e = 115 + (i >> 20) % 22, m = (i * 2654435761u) & 0x7fffff, s = (i & 1) << 31;
  float v = __uint_as_float(s | (e << 23) | m);
  v = fminf(fmaxf(v, -448.f), 448.f);
  const unsigned hw = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(v, 0.f, 0, false) & 0xffu;
  const unsigned sw = sr::e4m3_rne(v) & 0xffu;
  if (hw != sw) {
    const unsigned n = atomicAdd(bad, 1u);
    if (n == 0) { first[0] = __float_as_uint(v); first[1] = hw; first[2] = sw; }
  }
}

int main() {
  unsigned *d, h[4] = {0, 0, 0, 0};
  (void)hipMalloc(&d, 16);
  (void)hipMemset(d, 0, 16);
  hipLaunchKernelGGL(k, dim3(1 << 16), dim3(256), 0, 0, d, d + 1);
  (void)hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
  printf("mismatches %u of %u", h[0], 1u << 24);
  if (h[0]) {
    float f;
    memcpy(&f, &h[1], 4);
    printf("  first: %.9g hw 0x%02x sw 0x%02x", f, h[2], h[3]);
  }
  printf("\n");
  return h[0] ? 1 : 0;
}
