// Diagnostic (not product): the GEMM main loop (no epilogue) with v_mfma_f32_32x32x16_f16 vs
// v_mfma_f32_16x16x32_f16 under one identical structure, to size the re-tiling of K4:
//   256 x 256 tile per 8-wave workgroup, wave tile 128 (W rows) x 64 (X rows), K-step 64,
//   two LDS stages (XOR-swizzled 16-byte chunks, LDS-DMA staging), per K-step: wait + barrier,
//   read all fragments of the step, issue the next step's staging, then the MFMAs.
// Both variants hold 128 fp32 accumulators and 96 fragment VGPRs per lane.
//   hipcc --offload-arch=gfx950 -O3 tools/diag/mfma_mainloop.hip -o tools/diag/mfma_mainloop
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef _Float16 half_t;
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

#define LDSP(p) ((__attribute__((address_space(3))) void*)(p))
#define WAITCNT(vm, lgkm) \
  __builtin_amdgcn_s_waitcnt(((vm) & 15) | (7 << 4) | (((lgkm) & 15) << 8) | (((vm) >> 4) << 14))

constexpr int BK = 64;           // halfs per K-step (128-byte rows)
constexpr int STAGE = 512 * BK;  // 256 W rows + 256 X rows

__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }

__device__ __forceinline__ h8 frag(const half_t* t, int row, int chunk) {
  return *reinterpret_cast<const h8*>(t + row * BK + swz(row, chunk) * 8);
}

template <bool MF32>
__global__ __launch_bounds__(512) void mainloop(const half_t* __restrict__ W, const half_t* __restrict__ X,
                                                float* __restrict__ out, int N, int K) {
  __shared__ __attribute__((aligned(16))) half_t lds[2 * STAGE];
  const int tiles_n = N / 256;
  const int n0 = (blockIdx.x % tiles_n) * 256, m0 = (blockIdx.x / tiles_n) * 256;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 2, wm = wave & 3;
  const int nk = K / BK;

  // staging: 64 pieces of 8 rows x 128 B per K-step (pieces 0..31 = W rows, 32..63 = X rows);
  // wave w issues pieces w, w + 8, ..., lane l -> row (l >> 3), stored chunk (l & 7)
  auto stage = [&](int kt, half_t* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int piece = wave + 8 * i;
      const int r = piece * 8 + (lane >> 3);  // 0..511
      const int lc = swz(r, lane & 7);        // logical chunk stored at position (lane & 7)
      const half_t* src = r < 256 ? W + (size_t)(n0 + r) * K : X + (size_t)(m0 + r - 256) * K;
      __builtin_amdgcn_global_load_lds((const void*)(src + kt * BK + lc * 8), LDSP(dst + piece * 8 * BK),
                                       16, 0, 0);
    }
  };

  f16v acc32[MF32 ? 4 : 1][MF32 ? 2 : 1];
  f4 acc16[MF32 ? 1 : 8][MF32 ? 1 : 4];
  if constexpr (MF32) {
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 2; ++j) acc32[i][j] = (f16v)0.f;
  } else {
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j) acc16[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  }

  stage(0, lds);
  for (int kt = 0; kt < nk; ++kt) {
    const half_t* cur = lds + (kt & 1) * STAGE;
    WAITCNT(0, 0);
    __builtin_amdgcn_s_barrier();
    if constexpr (MF32) {
      // A: W rows wn*128 + 32i + (l & 31), k 16ks + 8(l >> 5) .. +7 ; B: X rows wm*64 + 32j + ...
      h8 a[4][4], b[2][4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i][ks] = frag(cur, wn * 128 + 32 * i + (lane & 31), 2 * ks + (lane >> 5));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          b[j][ks] = frag(cur + 256 * BK, wm * 64 + 32 * j + (lane & 31), 2 * ks + (lane >> 5));
      }
      WAITCNT(63, 0);
      if (kt + 1 < nk) stage(kt + 1, lds + ((kt + 1) & 1) * STAGE);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][ks], b[j][ks], acc32[i][j], 0, 0, 0);
    } else {
      h8 a[8][2], b[4][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i][s] = frag(cur, wn * 128 + 16 * i + (lane & 15), 4 * s + (lane >> 4));
#pragma unroll
        for (int j = 0; j < 4; ++j)
          b[j][s] = frag(cur + 256 * BK, wm * 64 + 16 * j + (lane & 15), 4 * s + (lane >> 4));
      }
      WAITCNT(63, 0);
      if (kt + 1 < nk) stage(kt + 1, lds + ((kt + 1) & 1) * STAGE);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc16[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][s], b[j][s], acc16[i][j], 0, 0, 0);
    }
  }
  float sum = 0.f;
  if constexpr (MF32) {
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 2; ++j)
        for (int r = 0; r < 16; ++r) sum += acc32[i][j][r];
  } else {
    for (int i = 0; i < 8; ++i)
      for (int j = 0; j < 4; ++j)
        for (int r = 0; r < 4; ++r) sum += acc16[i][j][r];
  }
  out[(size_t)blockIdx.x * 512 + tid] = sum;
}

template <bool MF32>
static double run(const half_t* W, const half_t* X, float* out, int M, int N, int K, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const dim3 grid((M / 256) * (N / 256)), block(512);
  hipLaunchKernelGGL(mainloop<MF32>, grid, block, 0, 0, W, X, out, N, K);
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(mainloop<MF32>, grid, block, 0, 0, W, X, out, N, K);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return 2.0 * M * (double)N * K * reps / (ms * 1e-3) / 1e12;
}

// elements are multiples of 1/16 in [-0.5, 0.5]: every product, partial sum and the per-lane
// sums are exact in fp32, so both variants must give the same total (checked exactly)
static double total(const float* d_out, int M, int N) {
  const size_t n = (size_t)(M / 256) * (N / 256) * 512;
  float* h = (float*)malloc(n * sizeof(float));
  (void)hipMemcpy(h, d_out, n * sizeof(float), hipMemcpyDeviceToHost);
  double s = 0.0;
  for (size_t i = 0; i < n; ++i) s += h[i];
  free(h);
  return s;
}

int main() {
  const int M = 131072, shapes[4][2] = {{3072, 768}, {2304, 768}, {768, 768}, {768, 3072}};
  half_t *W, *X;
  float* out;
  (void)hipMalloc(&W, (size_t)3072 * 3072 * 2);
  (void)hipMalloc(&X, (size_t)M * 3072 * 2);
  (void)hipMalloc(&out, (size_t)(M / 256) * 12 * 512 * 4);
  {
    const size_t nx = (size_t)M * 3072, nw = (size_t)3072 * 3072;
    half_t* h = (half_t*)malloc(nx * 2);
    uint32_t x = 12345u;
    for (size_t i = 0; i < nx; ++i) {
      x = x * 1664525u + 1013904223u;
      h[i] = (half_t)((float)((int)((x >> 24) % 17) - 8) / 16.0f);
    }
    (void)hipMemcpy(X, h, nx * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(W, h, nw * 2, hipMemcpyHostToDevice);
    free(h);
  }
  for (auto& s : shapes) {
    const int N = s[0], K = s[1];
    const double t16 = run<false>(W, X, out, M, N, K, 10);
    const double s16 = total(out, M, N);
    const double t32 = run<true>(W, X, out, M, N, K, 10);
    const double s32 = total(out, M, N);
    printf("M=%d N=%d K=%d  16x16x32: %7.1f TF/s   32x32x16: %7.1f TF/s   totals %s (%.6g)\n", M, N, K,
           t16, t32, s16 == s32 ? "equal" : "DIFFER", s16);
  }
  return 0;
}
