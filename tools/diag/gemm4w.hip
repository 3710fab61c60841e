// Diagnostic (not product): GEMM main-loop structures for K4 on gfx950, no epilogue.
//   V0  the shipped structure: 8 waves (2 per SIMD), wave tile 128 (W rows) x 64 (X rows),
//       LDS-DMA staging, 2 stages, one barrier per K-step
//   V1  4 waves (1 per SIMD, up to 512 registers), wave tile 128 x 128, LDS-DMA staging issued by
//       every wave right after the barrier
//   V2  4 waves, wave tile 128 x 128, register staging: global_load_dwordx4 of K-step kt+2 and
//       ds_write_b128 of kt+1 (loaded a K-step earlier) spread over the MFMA phases of kt
// All: 256 x 256 x 64 per K-step, v_mfma_f32_16x16x32_f16, XOR-swizzled 128-B rows (chunk c of row
// r at c ^ ((r >> 1) & 7)), operands multiples of 1/16 so the per-lane sums are exact and every
// variant must return the same total.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/diag/gemm4w.hip -o tools/diag/gemm4w
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef _Float16 half_t;
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef int i4 __attribute__((ext_vector_type(4)));

#define LDSP(p) ((__attribute__((address_space(3))) void*)(p))
#define WAITCNT(vm, lgkm) \
  __builtin_amdgcn_s_waitcnt(((vm) & 15) | (7 << 4) | (((lgkm) & 15) << 8) | (((vm) >> 4) << 14))

constexpr int BK = 64;           // halfs per K-step (128-byte rows)
constexpr int STAGE = 512 * BK;  // 256 W rows + 256 X rows

__device__ __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }
__device__ __forceinline__ h8 frag(const half_t* t, int row, int chunk) {
  return *reinterpret_cast<const h8*>(t + row * BK + swz(row, chunk) * 8);
}

// tile of workgroup b: XCD-contiguous ranges, n fastest (W column tiles re-served from L2)
__device__ __forceinline__ void tile_of(int b, int nwg, int tiles_n, int& n0, int& m0) {
  const int xcd = b & 7, q = nwg >> 3, rem = nwg & 7;
  const int lo = xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
  const int t = lo + (b >> 3);
  n0 = (t % tiles_n) * 256;
  m0 = (t / tiles_n) * 256;
}

// ---- V0: 8 waves --------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void v0(const half_t* __restrict__ W, const half_t* __restrict__ X,
                                          float* __restrict__ out, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) half_t lds[2 * STAGE];
  int n0, m0;
  tile_of(blockIdx.x, gridDim.x, N / 256, n0, m0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 2, wm = wave & 3;
  const int nk = K / BK;
  auto stage = [&](int kt, half_t* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int piece = wave + 8 * i;
      const int r = piece * 8 + (lane >> 3);
      const int lc = swz(r, lane & 7);
      const half_t* src = r < 256 ? W + (size_t)(n0 + r) * K : X + (size_t)(m0 + r - 256) * K;
      __builtin_amdgcn_global_load_lds((const void*)(src + kt * BK + lc * 8), LDSP(dst + piece * 8 * BK), 16, 0, 0);
    }
  };
  f4 acc[8][4];
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  stage(0, lds);
  for (int kt = 0; kt < nk; ++kt) {
    const half_t* cur = lds + (kt & 1) * STAGE;
    WAITCNT(0, 0);
    __builtin_amdgcn_s_barrier();
    h8 a[8][2], b[4][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i][s] = frag(cur, wn * 128 + 16 * i + (lane & 15), 4 * s + (lane >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j][s] = frag(cur + 256 * BK, wm * 64 + 16 * j + (lane & 15), 4 * s + (lane >> 4));
    }
    WAITCNT(63, 0);
    if (kt + 1 < nk) stage(kt + 1, lds + ((kt + 1) & 1) * STAGE);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
  }
  float sum = 0.f;
  for (int i = 0; i < 8; ++i)
    for (int j = 0; j < 4; ++j)
      for (int r = 0; r < 4; ++r) sum += acc[i][j][r];
  out[(size_t)blockIdx.x * 512 + tid] = sum;
}

// ---- V1 / V2: 4 waves, 128 x 128 wave tiles --------------------------------------------------------
// wave w: W rows wn*128 .. +127 (wn = w >> 1), X rows wm*128 .. +127 (wm = w & 1).
// Staging: the 64 pieces (8 rows x 128 B) of a K-step, wave w owns pieces 16w .. 16w + 15:
// piece p = rows 8p .. 8p + 7 of the 512-row stage, lane l -> row 8p + (l >> 3), stored chunk l & 7.
// A K-step = 4 phases of 32 MFMAs: phase q = (k half h = q >> 1, W row group g = q & 1):
// acc[4g + i][j] += A_h[g][i] x B_h[j], i < 4, j < 8.  The next phase's operands are read during
// the current one (A group: 4 reads; at q = 1 also the next half's 8 B reads; at q = 3 the next
// K-step's A and B of half 0, after the barrier).
template <int VAR>
__global__ __launch_bounds__(256, 1) void v4(const half_t* __restrict__ W, const half_t* __restrict__ X,
                                             float* __restrict__ out, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) half_t lds[2 * STAGE];
  int n0, m0;
  tile_of(blockIdx.x, gridDim.x, N / 256, n0, m0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 1, wm = wave & 1;
  const int nk = K / BK;
  const int arow = wn * 128 + (lane & 15), brow = 256 + wm * 128 + (lane & 15), c0 = lane >> 4;
  // staging addresses: wave w loads pieces 16w .. 16w + 15 (waves 0, 1: W rows; 2, 3: X rows);
  // a piece's lane offset depends on the piece only through its row block (uniform soffset) and
  // the swizzle parity (i & 1), so a lane keeps two 32-bit offsets
  const half_t* base = wave < 2 ? W + (size_t)n0 * K : X + (size_t)m0 * K;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 256 * K * 2, 0x00020000);
  int voff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par)
    voff[par] = ((lane >> 3) * K + ((lane & 7) ^ ((4 * par + (lane >> 4)) & 7)) * 8) * 2;
  const int wrow0 = (wave & 1) * 16;   // first piece of the wave within its operand (8-row blocks)
  auto dma = [&](int kt, half_t* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDSP(dst + (wave * 16 + i) * 8 * BK), 16, voff[i & 1],
                                               (8 * (wrow0 + i) * K + kt * BK) * 2, 0, 0);
  };
  i4 stg[16];
  auto gload = [&](int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      stg[i] = __builtin_bit_cast(i4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff[i & 1], (8 * (wrow0 + i) * K + kt * BK) * 2, 0));
  };
  auto swrite = [&](half_t* dst, int i) __attribute__((always_inline)) {
    *reinterpret_cast<i4*>(dst + (wave * 16 + i) * 8 * BK + lane * 8) = stg[i];
  };

  f4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

  // prologue: K-step 0 in stage 0 (V2: and K-step 1 loaded into registers)
  if constexpr (VAR == 1) {
    dma(0, lds);
  } else {
    gload(0);
#pragma unroll
    for (int i = 0; i < 16; ++i) swrite(lds, i);
    if (nk > 1) gload(1);
  }
  WAITCNT(VAR == 1 ? 0 : 16, 0);
  __builtin_amdgcn_s_barrier();
  h8 A[2][4], B[2][8];   // [buffer][...]: current / next operands
#pragma unroll
  for (int i = 0; i < 4; ++i) A[0][i] = frag(lds, arow + 16 * i, c0);
#pragma unroll
  for (int j = 0; j < 8; ++j) B[0][j] = frag(lds, brow + 16 * j, c0);

  for (int kt = 0; kt < nk; ++kt) {
    const half_t* cur = lds + (kt & 1) * STAGE;
    half_t* nxt = lds + ((kt + 1) & 1) * STAGE;
    const bool more = kt + 1 < nk;
    if constexpr (VAR == 1) {
      if (more) dma(kt + 1, nxt);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int h = q >> 1, g = q & 1;
      // operands of phase q + 1 into the other buffers
      if (q < 3) {
        const int h1 = (q + 1) >> 1, g1 = (q + 1) & 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) A[(q + 1) & 1][i] = frag(cur, arow + 64 * g1 + 16 * i, c0 + 4 * h1);
        if (q == 1) {
#pragma unroll
          for (int j = 0; j < 8; ++j) B[1][j] = frag(cur, brow + 16 * j, c0 + 4);
        }
      }
      if constexpr (VAR == 2) {
        // V2: the 16 staging writes of K-step kt+1 over phases 0..2 (6, 5, 5), then the loads of
        // kt+2 into the freed registers; all before phase 2's barrier
        if (q < 3 && more) {
          const int w0 = q == 0 ? 0 : (q == 1 ? 6 : 11), w1 = q == 0 ? 6 : (q == 1 ? 11 : 16);
#pragma unroll
          for (int i = w0; i < w1; ++i) swrite(nxt, i);
        }
        if (q == 2 && kt + 2 < nk) gload(kt + 2);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[4 * g + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[q & 1][i], B[h][j], acc[4 * g + i][j], 0, 0, 0);
      if (q == 2) {
        // all of this K-step's LDS reads are issued; the next stage is complete once every wave
        // passes here: staging (V1 vmcnt, V2 lgkmcnt) + barrier before phase 3's reads of kt+1
        if constexpr (VAR == 1)
          WAITCNT(0, 0);
        else
          WAITCNT(63, 0);
        __builtin_amdgcn_s_barrier();
      }
      if (q == 3 && more) {
#pragma unroll
        for (int i = 0; i < 4; ++i) A[0][i] = frag(nxt, arow + 16 * i, c0);
#pragma unroll
        for (int j = 0; j < 8; ++j) B[0][j] = frag(nxt, brow + 16 * j, c0);
      }
    }
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum += acc[i][j][r];
  // two of these lanes' sums per v0 lane: write into the 512-slot layout of v0 as pairs
  out[(size_t)blockIdx.x * 512 + tid] = sum;
  out[(size_t)blockIdx.x * 512 + 256 + tid] = 0.f;
}

// ---- V3: 8 waves, wave tile 256 (W rows) x 32 (X rows), X straight into registers ----------------
// Only W is staged by LDS-DMA (32 pieces per K-step, 4 per wave, 3-stage ring of 32 KiB); every
// wave's 32 X rows are exclusive to it, so their B fragments are loaded with buffer_load_dwordx4
// into a 3-K-step register ring (4 loads per wave and K-step).  A K-step = 8 phases of 4 W blocks
// x 2 X blocks (8 MFMAs); phase q + 1's A fragments are read during phase q; the barrier sits
// before phase 7, after which the next K-step's phase-0 fragments are read and the DMA of K-step
// kt + 2 is issued.
template <int XD>
__global__ __launch_bounds__(512) void v3(const half_t* __restrict__ W, const half_t* __restrict__ X,
                                          float* __restrict__ out, int M, int N, int K) {
  constexpr int WST = 256 * BK;
  __shared__ __attribute__((aligned(16))) half_t lds[3 * WST];
  int n0, m0;
  tile_of(blockIdx.x, gridDim.x, N / 256, n0, m0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nk = K / BK;
  const int c = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)(W + (size_t)n0 * K), (short)0, 256 * K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (size_t)(m0 + 32 * wave) * K), (short)0, 32 * K * 2, 0x00020000);
  int voff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par)
    voff[par] = ((lane >> 3) * K + ((lane & 7) ^ ((4 * par + (lane >> 4)) & 7)) * 8) * 2;
  const int xoff = (c * K + 8 * g) * 2;
  auto dma = [&](int kt) __attribute__((always_inline)) {
    half_t* dst = lds + (kt % 3) * WST;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = wave * 4 + i;  // rows 8p .. 8p + 7; swizzle parity p & 1 = i & 1
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, LDSP(dst + p * 8 * BK), 16, voff[i & 1], (8 * p * K + kt * BK) * 2, 0, 0);
    }
  };
  h8 xb[XD][2][2];  // [ring slot][X block][k half]
  auto xload = [&](int slot, int kt) __attribute__((always_inline)) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        xb[slot][mb][h] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(rx, xoff, (mb * 16 * K + kt * BK + 32 * h) * 2, 0));
  };
  f4 acc[16][2];
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // phase q: W blocks 4 (q & 3) .. + 3, k half q >> 2
  auto afrag = [&](const half_t* st, int q, int i) __attribute__((always_inline)) {
    return frag(st, 16 * (4 * (q & 3) + i) + c, 4 * (q >> 2) + g);
  };
  dma(0);
  if (nk > 1) dma(1);
#pragma unroll
  for (int d = 0; d < XD; ++d) xload(d, d);
  WAITCNT(0, 0);
  __builtin_amdgcn_s_barrier();
  h8 A[2][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) A[0][i] = afrag(lds, 0, i);
  for (int kt0 = 0; kt0 < nk; kt0 += 6) {
#pragma unroll
    for (int u6 = 0; u6 < 6; ++u6) {
      const int kt = kt0 + u6;  // (nk % 6 == 0: K = 768 / 3072)
      const int u = u6 % 3, xs = u6 % XD;
      const half_t* cur = lds + u * WST;
#pragma unroll
      for (int q = 0; q < 7; ++q) {
        if (q < 6) {
#pragma unroll
          for (int i = 0; i < 4; ++i) A[(q + 1) & 1][i] = afrag(cur, q + 1, i);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) A[1][i] = afrag(cur, 7, i);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[4 * (q & 3) + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[q & 1][i], xb[xs][j][q >> 2], acc[4 * (q & 3) + i][j], 0, 0, 0);
      }
      // K-step kt + 1's W stage has landed (younger: X(kt - 1 + XD) only) -> barrier
      if (kt - 1 + XD < nk)
        WAITCNT(4, 0);
      else
        WAITCNT(0, 0);
      __builtin_amdgcn_s_barrier();
      if (kt + 2 < nk) dma(kt + 2);
      const half_t* nxt = lds + ((u + 1) % 3) * WST;
      if (kt + 1 < nk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) A[0][i] = afrag(nxt, 0, i);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[12 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[1][i], xb[xs][j][1], acc[12 + i][j], 0, 0, 0);
      if (kt + XD < nk) xload(xs, kt + XD);
    }
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sum += acc[i][j][r];
  out[(size_t)blockIdx.x * 512 + tid] = sum;
}

template <class Kern>
static double run(Kern k, int threads, const half_t* W, const half_t* X, float* out, int M, int N, int K,
                  int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const dim3 grid((M / 256) * (N / 256)), block(threads);
  hipLaunchKernelGGL(k, grid, block, 0, 0, W, X, out, M, N, K);
  (void)hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, grid, block, 0, 0, W, X, out, M, N, K);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return 2.0 * M * (double)N * K * reps / (ms * 1e-3) / 1e12;
}

static double total(const float* d_out, int M, int N) {
  const size_t n = (size_t)(M / 256) * (N / 256) * 512;
  float* h = (float*)malloc(n * sizeof(float));
  (void)hipMemcpy(h, d_out, n * sizeof(float), hipMemcpyDeviceToHost);
  double s = 0.0;
  for (size_t i = 0; i < n; ++i) s += h[i];
  free(h);
  return s;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 131072;
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  const int shapes[4][2] = {{3072, 768}, {2304, 768}, {768, 768}, {768, 3072}};
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
    for (size_t i = 0; i < nw; ++i) {
      x = x * 1664525u + 1013904223u;
      h[i] = (half_t)((float)((int)((x >> 24) % 17) - 8) / 16.0f);
    }
    (void)hipMemcpy(W, h, nw * 2, hipMemcpyHostToDevice);
    free(h);
  }
  for (auto& s : shapes) {
    const int N = s[0], K = s[1];
    const double t0 = run(v0, 512, W, X, out, M, N, K, reps);
    const double s0 = total(out, M, N);
    const double t1 = run(v4<1>, 256, W, X, out, M, N, K, reps);
    const double s1 = total(out, M, N);
    const double t2 = run(v4<2>, 256, W, X, out, M, N, K, reps);
    const double s2 = total(out, M, N);
    const double t3 = run(v3<3>, 512, W, X, out, M, N, K, reps);
    const double s3 = total(out, M, N);
    const double t4 = run(v3<2>, 512, W, X, out, M, N, K, reps);
    const double s4 = total(out, M, N);
    printf("M=%d N=%d K=%d  V0 8w: %7.1f  V1 4w dma: %7.1f  V2 4w reg: %7.1f  V3 8w Xreg3: %7.1f  Xreg2: %7.1f TF/s  totals %s %s %s %s\n", M, N,
           K, t0, t1, t2, t3, t4, s0 == s1 ? "eq" : "DIFF", s0 == s2 ? "eq" : "DIFF", s0 == s3 ? "eq" : "DIFF",
           s0 == s4 ? "eq" : "DIFF");
    fflush(stdout);
  }
  return 0;
}
