// K4: MFMA GEMM with fused epilogues for the encoder projections (QKV, O, FFN1, FFN2, cls dense).
//
//   Y[m][n] = epi( sum_k X[m][k] * W[n][k] + bias[n] (+ R[m][n]) )
//
// X is the activation (M x K, fp16, row stride lda), W the PyTorch-layout weight (N x K, fp16).
// Both operands are K-contiguous, so each MFMA fragment is one 16-byte LDS read.
// The MFMA computes the transposed tile D = W_tile . X_tile^T (A = W rows, B = X rows): a lane
// then owns 4 consecutive output columns n of one row m, which makes the bias / residual / store
// of the epilogue a single 8- or 16-byte access per 16x16 tile.
//
// Tiling: 128 (n) x 128 (m) x 64 (k) per workgroup of 4 waves (2 x 2), each wave 64 x 64 =
// 4 x 4 tiles of v_mfma_f32_16x16x32_f16.  Global -> LDS staging uses global_load_lds_dwordx4
// (16 B per lane) into a double-buffered, XOR-swizzled LDS image (conflict-free ds_read_b128,
// checked by simulation: the 16-byte chunk c of row r is stored at chunk c ^ ((r >> 1) & 7)).
// Workgroups are remapped so each XCD owns a contiguous range of m-panels (L2 reuse of X).
#include "sr_common.h"
#include "sr_kernels.h"

namespace sr {

namespace {

constexpr int GBM = 128;  // m per workgroup
constexpr int GBN = 128;  // n per workgroup
constexpr int GBK = 64;   // k per stage
constexpr int GTHREADS = 256;

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Issue the glds for one 128 x 64 fp16 tile: 16 wave-instructions of 1 KiB (8 rows x 128 B),
// 4 per wave.  Lane l of an instruction lands at LDS byte l*16 of the 1 KiB piece, i.e. row
// (l >> 3), stored chunk (l & 7); it therefore loads the global chunk that belongs there.
__device__ __forceinline__ void stage_tile(const half_t* __restrict__ g, int64_t ld, int row0,
                                           int row_max, int k0, half_t* lds_tile, int wave,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = wave * 32 + i * 8 + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    int gr = row0 + r;
    gr = gr < row_max ? gr : row_max - 1;
    const half_t* src = g + (int64_t)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, SR_LDS(lds_tile + (wave * 32 + i * 8) * GBK),
                                     16, 0, 0);
  }
}

__device__ __forceinline__ half8 read_frag(const half_t* lds_tile, int row, int chunk) {
  const int off = row * GBK + swz_chunk(row, chunk) * 8;
  return *reinterpret_cast<const half8*>(lds_tile + off);
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

template <int EPI>
__global__ __launch_bounds__(GTHREADS, 2) void gemm_f16_kernel(
    const half_t* __restrict__ X, int64_t lda, const half_t* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ R, int64_t ldr, void* __restrict__ Y,
    int64_t ldy, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) half_t lds[2 * 2 * GBM * GBK];  // 64 KiB

  const int tiles_n = N / GBN;
  const int tiles_m = (M + GBM - 1) / GBM;
  const int nwg = tiles_n * tiles_m;
  // XCD-aware bijective remap: blocks b and b+8 share an XCD; give each XCD a contiguous range.
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, rem = nwg & 7;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (orig >> 3);
  const int tm = wg / tiles_n, tn = wg - tm * tiles_n;
  const int m0 = tm * GBM, n0 = tn * GBN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (LDS-DMA base in M0)
  const int wn = wave >> 1, wm = wave & 1;

  float4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GBK;
  // stage buffer b: W tile at lds + b*2*GBM*GBK, X tile right after it.
  stage_tile(W, K, n0, N, 0, lds, wave, lane);
  stage_tile(X, lda, m0, M, 0, lds + GBM * GBK, wave, lane);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    half_t* As = lds + cur * (2 * GBM * GBK);
    half_t* Bs = As + GBM * GBK;
    if (kt + 1 < nk) {
      half_t* An = lds + (cur ^ 1) * (2 * GBM * GBK);
      stage_tile(W, K, n0, N, (kt + 1) * GBK, An, wave, lane);
      stage_tile(X, lda, m0, M, (kt + 1) * GBK, An + GBM * GBK, wave, lane);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      half8 a[4], b[4];
      const int chunk = (lane >> 4) + 4 * s;
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = read_frag(As, wn * 64 + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = read_frag(Bs, wm * 64 + j * 16 + (lane & 15), chunk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // Epilogue: lane owns D[n = n0 + 64wn + 16i + 4(lane>>4) + r][m = m0 + 64wm + 16j + (lane&15)].
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = n0 + wn * 64 + i * 16 + 4 * (lane >> 4);
    const float4v bv = *reinterpret_cast<const float4v*>(bias + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wm * 64 + j * 16 + (lane & 15);
      if (m >= M) continue;
      float4v v = acc[i][j] + bv;
      if constexpr (EPI == EPI_BIAS_RES_F32) {
        const float4v rv = *reinterpret_cast<const float4v*>(R + (int64_t)m * ldr + n);
        v += rv;
        *reinterpret_cast<float4v*>(reinterpret_cast<float*>(Y) + (int64_t)m * ldy + n) = v;
      } else if constexpr (EPI == EPI_BIAS_TANH_F32) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = tanhf(v[r]);
        *reinterpret_cast<float4v*>(reinterpret_cast<float*>(Y) + (int64_t)m * ldy + n) = v;
      } else {
        if constexpr (EPI == EPI_BIAS_GELU_F16) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
        }
        half4 h = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
        *reinterpret_cast<half4*>(reinterpret_cast<half_t*>(Y) + (int64_t)m * ldy + n) = h;
      }
    }
  }
}

}  // namespace

static const char* epi_name(int epi) {
  switch (epi) {
    case EPI_BIAS_F16: return "gemm_f16_bias";
    case EPI_BIAS_GELU_F16: return "gemm_f16_bias_gelu";
    case EPI_BIAS_RES_F32: return "gemm_f16_bias_residual";
    default: return "gemm_f16_bias_tanh";
  }
}

void launch_gemm(int epi, const half_t* X, int64_t lda, const half_t* W, const float* bias,
                 const float* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K,
                 hipStream_t stream) {
  SR_CHECK(K % GBK == 0, "gemm: K must be a multiple of 64");
  SR_CHECK(N % GBN == 0, "gemm: N must be a multiple of 128");
  SR_CHECK(lda % 8 == 0 && ldy % 4 == 0, "gemm: leading dimensions must keep 16-byte rows");
  if (M <= 0) return;
  const int64_t tiles = (int64_t)(N / GBN) * ceil_div(M, GBM);
  SR_CHECK(tiles < (1ll << 31), "gemm: too many tiles");
  const double out_b = (epi == EPI_BIAS_RES_F32 || epi == EPI_BIAS_TANH_F32) ? 4.0 : 2.0;
  const double bytes = 2.0 * ((double)M * K + (double)N * K) + out_b * (double)M * N +
                       (epi == EPI_BIAS_RES_F32 ? 4.0 * M * N : 0.0);
  ProfScope prof(epi_name(epi), stream, 2.0 * M * (double)N * K, bytes);
  dim3 grid((unsigned)tiles), block(GTHREADS);
  switch (epi) {
    case EPI_BIAS_F16:
      hipLaunchKernelGGL(gemm_f16_kernel<EPI_BIAS_F16>, grid, block, 0, stream, X, lda, W, bias, R,
                         ldr, Y, ldy, M, N, K);
      break;
    case EPI_BIAS_GELU_F16:
      hipLaunchKernelGGL(gemm_f16_kernel<EPI_BIAS_GELU_F16>, grid, block, 0, stream, X, lda, W,
                         bias, R, ldr, Y, ldy, M, N, K);
      break;
    case EPI_BIAS_RES_F32:
      hipLaunchKernelGGL(gemm_f16_kernel<EPI_BIAS_RES_F32>, grid, block, 0, stream, X, lda, W,
                         bias, R, ldr, Y, ldy, M, N, K);
      break;
    case EPI_BIAS_TANH_F32:
      hipLaunchKernelGGL(gemm_f16_kernel<EPI_BIAS_TANH_F32>, grid, block, 0, stream, X, lda, W,
                         bias, R, ldr, Y, ldy, M, N, K);
      break;
    default: SR_CHECK(false, "gemm: unknown epilogue");
  }
  SR_LAUNCH_CHECK();
}

}  // namespace sr
