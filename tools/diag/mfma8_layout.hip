// Diagnostic (not product): checks the gfx950 block-scaled fp8 MFMA the K1-fp8 scan relies on,
// with exact small-integer data: v_mfma_scale_f32_16x16x128_f8f6f4 (fmt 0 = OCP e4m3fn), lane l
// supplying row l & 15 and the 32 K-bytes {16 g .. 16 g + 15} u {64 + 16 g .. 64 + 16 g + 15},
// g = l >> 4 (the two 16-byte LDS fragments the f16 pipe kernel already reads per K-step), the
// same map for A and B; E8M0 scale bytes (127 = 2^0).  C/D: col = lane & 15, row = 4 (l >> 4) + r.
//   hipcc --offload-arch=gfx950 -O2 tools/diag/mfma8_layout.hip -o tools/diag/mfma8_layout
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

static unsigned char e4m3(int v) {  // small integers -8..8, exact in e4m3fn
  if (v == 0) return 0;
  const unsigned s = v < 0 ? 0x80 : 0;
  int a = v < 0 ? -v : v;
  int e = 0;
  while ((1 << (e + 1)) <= a) ++e;
  const int m = ((a << 3) >> e) & 7;  // 3 mantissa bits
  return (unsigned char)(s | ((e + 7) << 3) | m);
}

__global__ void k(const unsigned char* A, const unsigned char* B, float* C, int sa, int sb) {
  const int l = threadIdx.x, row = l & 15, g = l >> 4;
  v8i a, b;
  unsigned char* pa = reinterpret_cast<unsigned char*>(&a);
  unsigned char* pb = reinterpret_cast<unsigned char*>(&b);
  for (int j = 0; j < 16; ++j) {
    pa[j] = A[row * 128 + 16 * g + j];
    pa[16 + j] = A[row * 128 + 64 + 16 * g + j];
    pb[j] = B[row * 128 + 16 * g + j];
    pb[16 + j] = B[row * 128 + 64 + 16 * g + j];
  }
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
  for (int r = 0; r < 4; ++r) C[(4 * g + r) * 16 + row] = c[r];
}

int main() {
  int Ai[16 * 128], Bi[16 * 128];
  unsigned char A[16 * 128], B[16 * 128];
  srand(1);
  for (int i = 0; i < 16 * 128; ++i) {
    Ai[i] = rand() % 17 - 8;
    Bi[i] = rand() % 17 - 8;
    A[i] = e4m3(Ai[i]);
    B[i] = e4m3(Bi[i]);
  }
  unsigned char *dA, *dB;
  float* dC;
  hipMalloc(&dA, sizeof(A));
  hipMalloc(&dB, sizeof(B));
  hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
  hipMemcpy(dB, B, sizeof(B), hipMemcpyHostToDevice);
  int fails = 0;
  const int scales[3][2] = {{127, 127}, {128, 127}, {126, 129}};
  for (int t = 0; t < 3; ++t) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, scales[t][0], scales[t][1]);
    float C[256];
    hipMemcpy(C, dC, sizeof(C), hipMemcpyDeviceToHost);
    const float f = ldexpf(1.f, scales[t][0] - 127 + scales[t][1] - 127);
    int bad = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        int ref = 0;
        for (int kk = 0; kk < 128; ++kk) ref += Ai[i * 128 + kk] * Bi[j * 128 + kk];
        if (C[i * 16 + j] != f * ref) {
          if (bad < 3) printf("  scale %d/%d: C[%d][%d] = %g, want %g\n", scales[t][0], scales[t][1], i, j, C[i * 16 + j], f * ref);
          ++bad;
        }
      }
    printf("scales %d/%d: %s (%d mismatches)\n", scales[t][0], scales[t][1], bad ? "FAIL" : "PASS", bad);
    fails += bad;
  }
  return fails ? 1 : 0;
}
