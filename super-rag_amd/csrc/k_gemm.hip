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
// Tiles (BN x BM x 64, v_mfma_f32_16x16x32_f16, fp32 accumulation):
//   big   256 (n) x 256 (m), 8 waves as 2 (n) x 4 (m), 128 x 64 per wave, 128 KiB LDS, 1 WG/CU
//   small 128 (n) x 128 (m), 4 waves as 2 x 2,        64 x 64 per wave,  64 KiB LDS, 2 WG/CU
// The big tile halves the L2->LDS bytes per FLOP (128 flop/B vs 64): at 128x128 the operand
// stream alone needs ~39 TB/s of L2 bandwidth at the 2.5 PF MFMA peak, more than the ~34 TB/s
// the L2s deliver.  Global -> LDS staging is global_load_lds_dwordx4 (16 B per lane) into a
// double-buffered, XOR-swizzled LDS image (conflict-free ds_read_b128, checked by simulation:
// 16-byte chunk c of row r is stored at chunk c ^ ((r >> 1) & 7)); the next K-step's loads are
// issued before the current step's MFMAs (2-phase pipeline), MFMA clusters run at s_setprio 1.
// Workgroups are remapped so each XCD owns a contiguous range of tiles, n fastest: the X panel
// of an m-tile is read from HBM once per XCD and re-served from that XCD's L2.
#include <cstdlib>

#include "sr_common.h"
#include "sr_kernels.h"

namespace sr {

namespace {

constexpr int GBK = 64;  // k per stage

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Issue NI glds wave-instructions of one tile: instruction i of this wave fills LDS rows
// prow..prow+7 (1 KiB = 8 rows x 128 B); lane l lands at byte l*16 of the piece, i.e. row
// (l >> 3), stored chunk (l & 7), and therefore loads the global chunk that belongs there.
template <int NI>
__device__ __forceinline__ void stage_tile(const half_t* __restrict__ g, int64_t ld, int row0,
                                           int row_max, int k0, half_t* lds_tile, int wave,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int prow = (wave * NI + i) * 8;
    const int r = prow + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    int gr = row0 + r;
    gr = gr < row_max ? gr : row_max - 1;
    const half_t* src = g + (int64_t)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, SR_LDS(lds_tile + prow * GBK), 16, 0, 0);
  }
}

__device__ __forceinline__ half8 read_frag(const half_t* lds_tile, int row, int chunk) {
  const int off = row * GBK + swz_chunk(row, chunk) * 8;
  return *reinterpret_cast<const half8*>(lds_tile + off);
}

__device__ __forceinline__ float gelu_erf(float x) {
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
}

template <int EPI, int BN, int BM, int WN, int WM>
__global__ __launch_bounds__(64 * WN * WM, 2) void gemm_f16_kernel(
    const half_t* __restrict__ X, int64_t lda, const half_t* __restrict__ W,
    const float* __restrict__ bias, const void* __restrict__ R, int64_t ldr,
    void* __restrict__ Y, int64_t ldy, int M, int N, int K) {
  constexpr int WAVES = WN * WM;
  constexpr int FN = BN / WN / 16, FM = BM / WM / 16;  // 16x16 tiles per wave
  constexpr int NIA = BN / 8 / WAVES, NIB = BM / 8 / WAVES;
  constexpr int STAGE = (BN + BM) * GBK;  // halfs per stage
  static_assert(NIA * WAVES * 8 == BN && NIB * WAVES * 8 == BM, "tile/wave mismatch");
  __shared__ __attribute__((aligned(16))) half_t lds[2 * STAGE];

  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m;
  // XCD-aware bijective remap: blocks b and b+8 share an XCD; give each XCD a contiguous range.
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q = nwg >> 3, rem = nwg & 7;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (orig >> 3);
  const int tm = wg / tiles_n, tn = wg - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (LDS-DMA base in M0)
  const int wn = wave / WM, wm = wave % WM;

  float4v acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  const int nk = K / GBK;
  // stage buffer b: W tile (BN rows) at lds + b*STAGE, X tile (BM rows) right after it.
  stage_tile<NIA>(W, K, n0, N, 0, lds, wave, lane);
  stage_tile<NIB>(X, lda, m0, M, 0, lds + BN * GBK, wave, lane);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const half_t* As = lds + cur * STAGE;
    const half_t* Bs = As + BN * GBK;
    if (kt + 1 < nk) {
      half_t* An = lds + (cur ^ 1) * STAGE;
      stage_tile<NIA>(W, K, n0, N, (kt + 1) * GBK, An, wave, lane);
      stage_tile<NIB>(X, lda, m0, M, (kt + 1) * GBK, An + BN * GBK, wave, lane);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      half8 a[FN], b[FM];
      const int chunk = (lane >> 4) + 4 * s;
#pragma unroll
      for (int i = 0; i < FN; ++i) a[i] = read_frag(As, wn * (BN / WN) + i * 16 + (lane & 15), chunk);
#pragma unroll
      for (int j = 0; j < FM; ++j) b[j] = read_frag(Bs, wm * (BM / WM) + j * 16 + (lane & 15), chunk);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
  }

  // Epilogue: lane owns D[n = n0 + wn*BN/WN + 16i + 4(lane>>4) + r][m = m0 + wm*BM/WM + 16j + (lane&15)].
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n0 + wn * (BN / WN) + i * 16 + 4 * (lane >> 4);
    const float4v bv = *reinterpret_cast<const float4v*>(bias + n);
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * (BM / WM) + j * 16 + (lane & 15);
      if (m >= M) continue;
      float4v v = acc[i][j] + bv;
      if constexpr (EPI == EPI_BIAS_RES_F32) {
        v += *reinterpret_cast<const float4v*>(reinterpret_cast<const float*>(R) + (int64_t)m * ldr + n);
        *reinterpret_cast<float4v*>(reinterpret_cast<float*>(Y) + (int64_t)m * ldy + n) = v;
      } else if constexpr (EPI == EPI_BIAS_TANH_F32) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = tanhf(v[r]);
        *reinterpret_cast<float4v*>(reinterpret_cast<float*>(Y) + (int64_t)m * ldy + n) = v;
      } else {
        if constexpr (EPI == EPI_BIAS_GELU_F16) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
        } else if constexpr (EPI == EPI_BIAS_RES_F16) {
          const half4 rv =
              *reinterpret_cast<const half4*>(reinterpret_cast<const half_t*>(R) + (int64_t)m * ldr + n);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += (float)rv[r];
        }
        half4 h = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
        *reinterpret_cast<half4*>(reinterpret_cast<half_t*>(Y) + (int64_t)m * ldy + n) = h;
      }
    }
  }
}

template <int BN, int BM, int WN, int WM>
void launch_tile(int epi, dim3 grid, hipStream_t stream, const half_t* X, int64_t lda,
                 const half_t* W, const float* bias, const void* R, int64_t ldr, void* Y,
                 int64_t ldy, int M, int N, int K) {
  const dim3 block(64 * WN * WM);
  switch (epi) {
    case EPI_BIAS_F16:
      hipLaunchKernelGGL((gemm_f16_kernel<EPI_BIAS_F16, BN, BM, WN, WM>), grid, block, 0, stream,
                         X, lda, W, bias, R, ldr, Y, ldy, M, N, K);
      break;
    case EPI_BIAS_GELU_F16:
      hipLaunchKernelGGL((gemm_f16_kernel<EPI_BIAS_GELU_F16, BN, BM, WN, WM>), grid, block, 0,
                         stream, X, lda, W, bias, R, ldr, Y, ldy, M, N, K);
      break;
    case EPI_BIAS_RES_F32:
      hipLaunchKernelGGL((gemm_f16_kernel<EPI_BIAS_RES_F32, BN, BM, WN, WM>), grid, block, 0,
                         stream, X, lda, W, bias, R, ldr, Y, ldy, M, N, K);
      break;
    case EPI_BIAS_RES_F16:
      hipLaunchKernelGGL((gemm_f16_kernel<EPI_BIAS_RES_F16, BN, BM, WN, WM>), grid, block, 0,
                         stream, X, lda, W, bias, R, ldr, Y, ldy, M, N, K);
      break;
    case EPI_BIAS_TANH_F32:
      hipLaunchKernelGGL((gemm_f16_kernel<EPI_BIAS_TANH_F32, BN, BM, WN, WM>), grid, block, 0,
                         stream, X, lda, W, bias, R, ldr, Y, ldy, M, N, K);
      break;
    default: SR_CHECK(false, "gemm: unknown epilogue");
  }
}

}  // namespace

static const char* epi_name(int epi) {
  switch (epi) {
    case EPI_BIAS_F16: return "gemm_f16_bias";
    case EPI_BIAS_GELU_F16: return "gemm_f16_bias_gelu";
    case EPI_BIAS_RES_F32: return "gemm_f16_bias_residual";
    case EPI_BIAS_RES_F16: return "gemm_f16_bias_residual16";
    default: return "gemm_f16_bias_tanh";
  }
}

// Tile override for parity tests: SR_GEMM_TILE=small|big (read per launch), or gemm_force_tile().
static int g_force_tile = -1;
void gemm_force_tile(int t) { g_force_tile = t; }
static int forced_tile() {
  if (g_force_tile >= 0) return g_force_tile;
  const char* e = std::getenv("SR_GEMM_TILE");
  if (!e) return -1;
  return std::strcmp(e, "big") == 0 ? 1 : (std::strcmp(e, "small") == 0 ? 0 : -1);
}

void launch_gemm(int epi, const half_t* X, int64_t lda, const half_t* W, const float* bias,
                 const void* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K,
                 hipStream_t stream) {
  SR_CHECK(K % GBK == 0, "gemm: K must be a multiple of 64");
  SR_CHECK(N % 128 == 0, "gemm: N must be a multiple of 128");
  SR_CHECK(lda % 8 == 0 && ldy % 4 == 0, "gemm: leading dimensions must keep 16-byte rows");
  if (M <= 0) return;
  const double out_b = (epi == EPI_BIAS_RES_F32 || epi == EPI_BIAS_TANH_F32) ? 4.0 : 2.0;
  const double res_b = epi == EPI_BIAS_RES_F32 ? 4.0 : (epi == EPI_BIAS_RES_F16 ? 2.0 : 0.0);
  const double bytes = 2.0 * ((double)M * K + (double)N * K) + (out_b + res_b) * (double)M * N;
  ProfScope prof(epi_name(epi), stream, 2.0 * M * (double)N * K, bytes);
  const int64_t big_tiles = (N % 256 == 0) ? (int64_t)(N / 256) * ceil_div(M, 256) : 0;
  const int force = forced_tile();
  const bool big = force >= 0 ? (force == 1 && N % 256 == 0) : big_tiles >= 512;
  if (big) {
    SR_CHECK(big_tiles < (1ll << 31), "gemm: too many tiles");
    launch_tile<256, 256, 2, 4>(epi, dim3((unsigned)big_tiles), stream, X, lda, W, bias, R, ldr,
                                Y, ldy, M, N, K);
  } else {
    const int64_t tiles = (int64_t)(N / 128) * ceil_div(M, 128);
    SR_CHECK(tiles < (1ll << 31), "gemm: too many tiles");
    launch_tile<128, 128, 2, 2>(epi, dim3((unsigned)tiles), stream, X, lda, W, bias, R, ldr, Y,
                                ldy, M, N, K);
  }
  SR_LAUNCH_CHECK();
}

}  // namespace sr
