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
#include <string>
#include <vector>
#include <type_traits>

#include "sr_common.h"
#include "sr_kernels.h"

// Store cache policy of the FFN1 line stores: nt (streaming; the output is read once, by the next
// GEMM).  Measured against 0 / sc0 / sc0 sc1 / sc1 in rounds 4-5 (profiles/r05_store_policy/):
// within +-0.5 %.  The wide epilogues' line stores use the default policy (0).
constexpr int kFfn1StoreAux = 2;

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

// fp8 fragment of a 128-byte K-step row: the lane's two 16-byte chunks c and c + 4 (the same two
// reads as the f16 K-step's two halves) as ONE 32-byte operand of the block-scaled fp8 MFMA.  The
// MFMA pairs A and B elements by their (lane group, byte) slot, so any slot -> k map shared by A
// and B is exact (checked with integer data: tools/diag/mfma8_layout.hip).
typedef int int8v __attribute__((ext_vector_type(8)));
typedef int int4v_ __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int8v read_frag8(const half_t* lds_tile, int row, int chunk) {
  const int4v_ lo = __builtin_bit_cast(int4v_, read_frag(lds_tile, row, chunk));
  const int4v_ hi = __builtin_bit_cast(int4v_, read_frag(lds_tile, row, chunk + 4));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// Unit vectors are stored / staged as e4m3(256 x): |256 x_i| <= 256 < 448 never saturates and the
// E8M0 block scales 119 = 2^-8 on A and B undo the factor inside the MFMA (exact power of two), so
// the accumulators are plain cosines.
__device__ __forceinline__ float4v mfma8(int8v a, int8v b, float4v c, int sa, int sb) {
  // fmt 0 / 0 = fp8 e4m3 (OCP); E8M0 block scales of A (lane's row) and B
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
}

// Exact-GELU x * Phi(x) with erf from Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below
// the fp16 rounding of the output): branch-free, one v_rcp + one v_exp + 7 FMA per element,
// about a third of the instructions of the library erff in this VALU-heavy epilogue.
__device__ __forceinline__ float gelu_erf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = 1.0f - p * __expf(-z * z);   // erf(|x| / sqrt 2)
  return 0.5f * x * (1.0f + copysignf(e, x));
}

// 2 * GELU(x) = x + |x| erf(|x| / sqrt 2) with the same erf (A&S 7.1.26): no copysign and no final
// halving (the consumer's weight carries the 0.5, exact in fp16), 4 VALU fewer per element than
// gelu_erf.  Used by the LayerNorm-folded FFN1 epilogue (EPI_LNF_GELU_F16).
__device__ __forceinline__ float gelu2_erf(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float w = __builtin_amdgcn_exp2f(x * (x * -0.72134752044448170f));  // exp(-x^2 / 2)
  return fmaf(ax, fmaf(-p, w, 1.0f), x);
}

// The lane id re-read by an asm the compiler may not hoist: epilogue addresses derived from it are
// recomputed where used instead of being hoisted out of the persistent tile loop (at 256 VGPRs
// hoisted lane-dependent offsets spill).
__device__ __forceinline__ int lane_id_here() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0" : "=v"(l));
  asm volatile("v_mbcnt_hi_u32_b32 %0, -1, %0" : "+v"(l));
  return l;
}

// Packed-fp32 forms of the epilogue math for the wide (8-column) layout: every FMA / MUL / ADD of
// two neighbouring columns is ONE v_pk_*_f32 (2 lanes of math per issue; the scalar forms issue at
// half that rate), only the transcendentals stay per element.  Same operations in the same order
// as gelu_erf / gelu2_erf, so the outputs are bit-identical to the scalar epilogue's.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v splat2(float x) { return f2v{x, x}; }

__device__ __forceinline__ f2v gelu2_erf2(f2v x) {
  const f2v ax = __builtin_elementwise_abs(x);
  const f2v d = pk_fma(splat2(0.3275911f * 0.70710678118654752f), ax, splat2(1.0f));
  const f2v t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f2v p = pk_fma(splat2(1.061405429f), t, splat2(-1.453152027f));
  p = pk_fma(p, t, splat2(1.421413741f));
  p = pk_fma(p, t, splat2(-0.284496736f));
  p = pk_fma(p, t, splat2(0.254829592f));
  p *= t;
  const f2v e = x * (x * splat2(-0.72134752044448170f));
  const f2v w = {__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
  return pk_fma(ax, pk_fma(-p, w, splat2(1.0f)), x);
}

// 2 GELU(x) = x * T(x), T(x) = 1 + erf(x / sqrt 2) = erfc(-x / sqrt 2), linearly interpolated
// from an LDS table of GELU_NT + 1 nodes x_i = -XMAX + i h over [-XMAX, XMAX] (XMAX = 4 sqrt 2,
// h = 2 XMAX / GELU_NT; entries (T(x_i), T(x_i+1) - T(x_i))); x outside the range takes the end
// nodes (T(-XMAX) = 1.5e-8, T(XMAX) = 2 - 1.5e-8).  |T error| <= h^2 / 8 max|T''| = 7.4e-6 (1.5 %
// of an fp16 ulp of the output x T; 1,025 entries = 8 KiB beside the FFN1 line scratch).  Per
// element: v_fma + v_med3 (index space, clamped), v_cvt_u32 + v_fract, one address op, one
// ds_read_b64, v_fma + v_mul: 7 VALU against gelu2_lut's 9-10 (and no abs / sign handling).
constexpr int GELU_LOG2_NT = 10;
constexpr int GELU_NT = 1 << GELU_LOG2_NT;
constexpr float GELU_XMAX = 5.6568542494923802f;  // 4 sqrt 2
// (index space through [0, 1] (the clamp modifier) and an exact ldexp)
__device__ __forceinline__ float gelu2_t(float x, const float2* __restrict__ tab) {
  const float zc = __builtin_amdgcn_fmed3f(fmaf(x, 1.0f / (2.0f * GELU_XMAX), 0.5f), 0.0f, 1.0f);
  const float az = __builtin_amdgcn_ldexpf(zc, GELU_LOG2_NT);
  const float2 t = tab[(uint32_t)az];
  return x * fmaf(__builtin_amdgcn_fractf(az), t.y, t.x);
}
__device__ __forceinline__ void gelu_t_tab_init(float2* __restrict__ tab, int tid, int nthreads) {
  constexpr float h = 2.0f * GELU_XMAX / (float)GELU_NT;
  for (int i = tid; i <= GELU_NT; i += nthreads) {
    const double x0 = -(double)GELU_XMAX + (double)i * (double)h;
    const float t0 = (float)erfc(-x0 * 0.70710678118654752);
    const float t1 = i < GELU_NT ? (float)erfc(-(x0 + (double)h) * 0.70710678118654752) : t0;
    tab[i] = make_float2(t0, t1 - t0);
  }
}

// The e4m3-output FFN1 epilogue (fp8 modes) reads T at the NEAREST of GELU_NT8 + 1 nodes over the
// same range (one fp32 entry each, 16 KiB): per element v_fma + v_med3 (index space + 0.5,
// clamped), v_cvt_u32, one address op, one ds_read_b32, v_mul -- 5 VALU against the interpolated
// form's 7.  |T error| <= h8 / 2 max|T'| = 1.1e-3 (x > 0: <= 0.11 % of x T; x = -2: 0.33 %), against
// e4m3's relative half-step of 3.1 %.
constexpr int GELU_NT8 = 4096;
__device__ __forceinline__ void gelu_t8_tab_init(float* __restrict__ tab, int tid, int nthreads) {
  constexpr double h = 2.0 * (double)GELU_XMAX / (double)GELU_NT8;
  for (int i = tid; i <= GELU_NT8; i += nthreads)
    tab[i] = (float)erfc(-(-(double)GELU_XMAX + (double)i * h) * 0.70710678118654752);
}

// W-row order of the wide epilogues (PERMW): inside each 32-row block, LDS row k holds W row
// perm32(k), so that MFMA tile 2p's rows 4g .. 4g+3 (lane group g) and tile 2p+1's rows 4g ..
// 4g+3 are the 8 CONSECUTIVE output columns 32p + 16(g & 1) + 4(g & 2) + 0..7 -- the layout the
// permlane16_swap exchange used to build (one swap per two outputs, no longer issued).
__device__ __forceinline__ int perm32(int k) {
  const int h = k >> 4, g = (k >> 2) & 3, r = k & 3;
  return 16 * (g & 1) + 4 * (g & 2) + 4 * h + r;
}
// the piece-dependent (uniform) part of perm32 for staging piece i (rows 8i + lane / 8 of a band)
__host__ __device__ constexpr int perm_row_off(int i) { return 32 * (i >> 2) + 8 * (i & 1) + 4 * ((i >> 1) & 1); }
// The e4m3-output FFN1 (P64): inside each 64-row block LDS row k = 16 t + 4 g + r (tile t of the
// quad, lane group g, row r) holds W row 16 g + 4 t + r, so lane group g's rows of the quad's 4 tiles
// are the 16 CONSECUTIVE output columns 16 g .. 16 g + 15: one 16-byte e4m3 store per (quad, row
// group).  The lane part of the staging offset, 16 (l3 >> 2) + (l3 & 3), is perm32's; the piece part:
__host__ __device__ constexpr int perm64_row_off(int i) { return 32 * (i & 1) + 4 * (i >> 1); }

__device__ __forceinline__ f2v gelu_erf2(f2v x) {
  const f2v z = __builtin_elementwise_abs(x) * splat2(0.70710678118654752f);
  const f2v d = pk_fma(splat2(0.3275911f), z, splat2(1.0f));
  const f2v t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f2v p = pk_fma(splat2(1.061405429f), t, splat2(-1.453152027f));
  p = pk_fma(p, t, splat2(1.421413741f));
  p = pk_fma(p, t, splat2(-0.284496736f));
  p = pk_fma(p, t, splat2(0.254829592f));
  p *= t;
  const f2v zz = -z * z;
  const f2v e = splat2(1.0f) - p * f2v{__expf(zz.x), __expf(zz.y)};
  const f2v s = {copysignf(e.x, x.x), copysignf(e.y, x.y)};
  return splat2(0.5f) * x * (splat2(1.0f) + s);
}

struct NoPre {
  __device__ __forceinline__ void operator()() const {}
};

// Epilogue: lane owns D[n = nw0 + 16i + 4(lane>>4) + r][m = mw0 + 16j + (lane&15)] of the wave's
// FN x FM 16x16 tiles; bias (+ residual) (+ activation), one 8/16-byte store per tile.
template <int EPI, int FN, int FM>
__device__ __forceinline__ void store_tile(float4v (&acc)[FN][FM], int nw0, int mw0, int lane, int M,
                                           const float* __restrict__ bias,
                                           const void* __restrict__ R, int64_t ldr,
                                           void* __restrict__ Y, int64_t ldy) {
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = nw0 + i * 16 + 4 * (lane >> 4);
    const float4v bv = *reinterpret_cast<const float4v*>(bias + n);
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = mw0 + j * 16 + (lane & 15);
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

// ---- "pipe" variant: 256 x 256 x 64, register-pipelined fragments, one barrier per K-step -------
// A K-step is four MFMA phases of 16 MFMAs each (wave tile 128 n x 64 m = 8 x 4 16x16 tiles):
//   p0: A[0..3]  x B  (k 0..31)     p1: A[4..7] x B (k 0..31)
//   p2: A[0..3]  x B' (k 32..63)    p3: A[4..7] x B' (k 32..63)
// The LDS fragments of phase p+1 are read while phase p's MFMAs run (two register sets, 64
// VGPRs), so the LDS latency is hidden behind 16 MFMAs instead of exposed at every K-half.
// Between p2 and p3 one raw s_barrier (behind vmcnt(0) lgkmcnt(0)) publishes K-step kt+1 (its
// glds were issued a K-step earlier) and frees buffer kt&1, into which the glds of kt+2 are issued
// before p3; p3 already reads K-step kt+1's first fragments from the other buffer.
template <int EPI, bool CHECK, int FN, int FM>
__device__ __forceinline__ void store_tile_fast(float4v (&acc)[FN][FM], int nw0, int mw0, int lane,
                                                int M, const float* __restrict__ bias,
                                                const void* __restrict__ R, int64_t ldr,
                                                void* __restrict__ Y, int64_t ldy) {
  constexpr bool RES32 = EPI == EPI_BIAS_RES_F32, RES16 = EPI == EPI_BIAS_RES_F16;
  constexpr bool OUT32 = EPI == EPI_BIAS_RES_F32 || EPI == EPI_BIAS_TANH_F32;
  const int ng = nw0 + 4 * (lane >> 4);
  float4v bv[FN];
#pragma unroll
  for (int i = 0; i < FN; ++i) bv[i] = *reinterpret_cast<const float4v*>(bias + ng + i * 16);
#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int m = mw0 + j * 16 + (lane & 15);
    if (CHECK && m >= M) continue;
    // the residual row segment first (all loads of the row group issued before its stores)
    float4v r32[RES32 ? FN : 1];
    half4 r16[RES16 ? FN : 1];
    if constexpr (RES32) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
        r32[i] = *reinterpret_cast<const float4v*>(reinterpret_cast<const float*>(R) + (int64_t)m * ldr + ng + i * 16);
    }
    if constexpr (RES16) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
        r16[i] = *reinterpret_cast<const half4*>(reinterpret_cast<const half_t*>(R) + (int64_t)m * ldr + ng + i * 16);
    }
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      float4v v = acc[i][j] + bv[i];
      if constexpr (RES32) v += r32[i];
      if constexpr (RES16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)r16[i][r];
      }
      if constexpr (EPI == EPI_BIAS_TANH_F32) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = tanhf(v[r]);
      }
      if constexpr (EPI == EPI_BIAS_GELU_F16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_erf(v[r]);
      }
      if constexpr (OUT32) {
        *reinterpret_cast<float4v*>(reinterpret_cast<float*>(Y) + (int64_t)m * ldy + ng + i * 16) = v;
      } else {
        half4 h = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
        *reinterpret_cast<half4*>(reinterpret_cast<half_t*>(Y) + (int64_t)m * ldy + ng + i * 16) = h;
      }
    }
  }
}

// fp16-output epilogue with 16-byte stores: tiles i = 2p and 2p + 1 of a row group are combined
// with v_permlane16_swap (rows of 16 lanes: even row g keeps its 4 columns of tile 2p and takes
// the odd partner's 4 columns of tile 2p, the odd row gets tile 2p + 1), so a lane owns 8
// consecutive columns nb .. nb+7 and every store / residual load is one dwordx4 (half the store
// instructions of the 8-byte layout; the store tail is issue-bound).
//
// LayerNorm folding (EPI_LNF_* / EPI_LNR16_STATS / EPI_RES16_STATS): (mu, rstd) of a row come
// from mr (launch_ln_stats_finalize of the producer's partials).  The *_STATS epilogues write the
// Chan partials of their own fp16-rounded outputs: per 128-column wave span the sum over the 4
// lane groups (xor-shuffles 16 / 32), then M2 around that span's mean.
// The *_STATS epilogues' (sum, M2) partials of a row's 128-value span, exact without any
// data-dependent form: M2 = sq - (sum - 128 c)^2 / 128 with sq = sum (x - c)^2 taken in fp32 around
// the pivot c = fp16(the mean of the span's first 64 values, column groups 0 and 1):
//   * x - c is EXACT in fp32 (x and c are fp16 values: their difference needs at most 24 bits for
//     any exponent gap under 13), so no bit of the deviation is lost, centred row or not;
//   * the squares and sums round once each in fp32 (2^-24 relative);
//   * cancellation: sum (x - c)^2 = M2 + 128 (mean - c)^2, and since c is the mean of one half,
//     128 (mean - c)^2 = 32 (mean_1 - mean_2)^2 <= M2 (the between-halves part of M2): at most a
//     factor 2, for every row.
// Each half span (16 values per lane) is summed per lane and reduced over the row's 4 lane groups
// on its own (half_span_stats), the halves then added (span_stats): the persistent residual
// epilogue (store_tile_res) parks the first half's three results in one lane group per row group
// instead of holding four of each per lane.  The sums of x stay on v_dot2c_f32_f16 (exact
// products); the deviations are one v_dot2_f32_f16 each (f16x2_minus) and the squares v_fmac_f32:
// one VALU per value more than an fp16 difference.  Against two-pass fp64 M2 of the same fp16
// outputs: tests/test_gpu_gemm.py (gate 2e-4).  (Rounds 4-5: x - c rounded to fp16 with c = the
// span's first value when three samples looked far from zero, else 0: up to 5.3e-4 on centred
// rows, ~3e-3 in the e4m3-copy epilogue that skipped the test; round 6's first try, the fp16
// difference around the half-span pivot: 3.9e-4 on centred rows, profiles/r06a/.)
// d = x - c in fp32 for the two fp16 values of a packed pair (nc = -c), each as ONE v_dot2_f32_f16
// of the pair with (1, 0) / (0, 1) and nc as the accumulator: exact (x * 1 and x * 0 are exact, the
// sum rounds once and fits 24 bits), reading the pair from the register it already sits in (a
// separate v_cvt_f32_f16 per value needed a temporary each, and at 256 VGPRs the residual epilogue
// spilled; the spill's reload waited vmcnt(0) inside the K-loop)
__device__ __forceinline__ void f16x2_minus(_Float16 x0, _Float16 x1, float nc, float& lo, float& hi) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  lo = __builtin_amdgcn_fdot2(h2{x0, x1}, h2{(_Float16)1.f, (_Float16)0.f}, nc, false);
  hi = __builtin_amdgcn_fdot2(h2{x0, x1}, h2{(_Float16)0.f, (_Float16)1.f}, nc, false);
}

// The 4 lane groups (lane >> 4) of a row hold its 4 column groups: the row's total in every lane.
__device__ __forceinline__ float row_reduce4(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// One half span (column groups 2h, 2h + 1: 16 values per lane) of the statistics: the lane's sum
// (v_dot2c) and, around the pivot nc = -c, the lane's sum of squared deviations (f16x2_minus +
// v_fmac), each reduced over the row's 4 lane groups (row_reduce4).  h = 0 derives the pivot from
// its own sum first (c = fp16(half sum / 64)).
template <bool FIRST>
__device__ __forceinline__ void half_span_stats(const half8& x0, const half8& x1, float& nc, float& sum, float& sq) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  const h2 one2 = {(_Float16)1.f, (_Float16)1.f};
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < 8; r += 2) s = __builtin_amdgcn_fdot2(h2{x0[r], x0[r + 1]}, one2, s, false);
#pragma unroll
  for (int r = 0; r < 8; r += 2) s = __builtin_amdgcn_fdot2(h2{x1[r], x1[r + 1]}, one2, s, false);
  sum = row_reduce4(s);
  if constexpr (FIRST) nc = -(float)(_Float16)(sum * (1.f / 64.f));
  float q = 0.f;
#pragma unroll
  for (int r = 0; r < 8; r += 2) {
    float d0, d1;
    f16x2_minus(x0[r], x0[r + 1], nc, d0, d1);
    q = fmaf(d0, d0, q);
    q = fmaf(d1, d1, q);
  }
#pragma unroll
  for (int r = 0; r < 8; r += 2) {
    float d0, d1;
    f16x2_minus(x1[r], x1[r + 1], nc, d0, d1);
    q = fmaf(d0, d0, q);
    q = fmaf(d1, d1, q);
  }
  sq = row_reduce4(q);
}

// The span's (sum, M2) from its two halves' reduced sums (pivot -nc): M2 = sq - (sum - 128 c)^2 / 128.
__device__ __forceinline__ float2 span_stats(float nc, float s0, float q0, float s1, float q1) {
  const float sum = s0 + s1, sq = q0 + q1;
  const float sp = fmaf(128.f, nc, sum);
  return float2{sum, fmaxf(fmaf(-sp * (1.f / 128.f), sp, sq), 0.f)};
}

// pre(): called once the epilogue's constant loads (bias, column sums / LayerNorm weight, row
// statistics) are issued: the persistent kernel stages the next tile's first K-steps there, so
// those loads are older than the staging pieces and their wait (vmcnt counts in order) does not
// also wait for the staging.
template <int EPI, bool CHECK, bool LINE_ST = false, bool GLUT = false, bool PERM = false,
          class Pre = NoPre>
__device__ __forceinline__ void store_tile_wide(float4v (&acc)[8][4], int nw0, int mw0, int lane,
                                                int M, int N, const float* __restrict__ bias,
                                                const void* __restrict__ R, int64_t ldr,
                                                void* __restrict__ Y, int64_t ldy,
                                                const LnFold& lf, half_t* __restrict__ scr = nullptr,
                                                const float2* __restrict__ gtab = nullptr,
                                                const Pre& pre = Pre{}) {
  constexpr bool OUT8 = EPI == EPI_LNF_GELU_F8;  // e4m3 bytes instead of fp16
  constexpr bool Y8 = EPI == EPI_RES16_STATS_Y8 || EPI == EPI_LNR16_STATS_Y8;  // + e4m3 copy
  constexpr bool LNF = EPI == EPI_LNF_F16 || EPI == EPI_LNF_GELU_F16 || OUT8;
  constexpr bool RESN = EPI == EPI_BIAS_RES_F16 || EPI == EPI_RES16_STATS || EPI == EPI_RES16_STATS_Y8;
  constexpr bool LNR = EPI == EPI_LNR16_STATS || EPI == EPI_LNR16_STATS_Y8;
  constexpr bool STATS = (RESN && EPI != EPI_BIAS_RES_F16) || LNR;
  constexpr bool GELU = EPI == EPI_BIAS_GELU_F16;
  constexpr bool GELU2 = EPI == EPI_LNF_GELU_F16 || OUT8;  // stores 2 * GELU (consumer weight halved)
  // packed fp32 math (f2v) for the LN-folded / GELU epilogues; the residual + statistics
  // epilogues keep the scalar form (packing them raised EPI_LNR16_STATS's spills 12 -> 112 B)
  constexpr bool PACK = !(RESN || LNR);
  // LINE: the fp16 rows of a 16-row group go through the wave's 4 KiB LDS scratch `scr` and leave
  // as whole 256-B row segments (4 rows x 256 B per store instruction) instead of 16 rows x 64 B:
  // 71 vs 19 B/clk of store throughput per CU (tools/diag/store_rate.hip)
  // (not for the GELU epilogues: there the exchange measured slower, FFN1 932 -> 881 TF/s, while
  // QKV gained 1005 -> 1044 and the residual + statistics GEMMs 1072 -> 1078, ab_line3)
  // (Y8: the e4m3 copy leaves from the line read-back too, as whole 128-B row segments)
  constexpr bool LINE = LINE_ST && !OUT8 && !GELU && !GELU2;
  static_assert(EPI == EPI_BIAS_F16 || GELU || GELU2 || RESN || LNF || LNR, "wide epilogue: fp16 outputs");
  const int g = lane >> 4, odd = g & 1;
  const int nlane = nw0 + 16 * odd + 4 * (g & 2);  // + 32 p
  float4v b0[4], b1[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    b0[p] = *reinterpret_cast<const float4v*>(bias + nlane + 32 * p);
    b1[p] = *reinterpret_cast<const float4v*>(bias + nlane + 32 * p + 4);
  }
  // LNF: column sums c[n]; LNR: the residual's LayerNorm weight (its beta is in the bias)
  float4v c0[(LNF || LNR) ? 4 : 1], c1[(LNF || LNR) ? 4 : 1];
  if constexpr (LNF || LNR) {
    const float* cv = LNF ? lf.colsum : lf.gamma;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      c0[p] = *reinterpret_cast<const float4v*>(cv + nlane + 32 * p);
      c1[p] = *reinterpret_cast<const float4v*>(cv + nlane + 32 * p + 4);
    }
  }
  float2 mrj[(LNF || LNR) ? 4 : 1];
  if constexpr (LNF || LNR) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int m = mw0 + j * 16 + (lane & 15);
      m = (CHECK && m >= M) ? M - 1 : m;
      mrj[j] = *reinterpret_cast<const float2*>(lf.mr + (int64_t)m * lf.stat_ld * 2);
    }
  }
  if constexpr (!std::is_same<Pre, NoPre>::value) {
    __builtin_amdgcn_sched_barrier(0);
    pre();
    __builtin_amdgcn_sched_barrier(0);
  }
  // BUFST (LINE): lane-constant byte offsets -- the residual read of the lane's row
  // in a 16-row group (+ 64 B per column group p: an immediate), the scratch write (column group p
  // is offset ^ 64 p: chunk 4p + k0 XOR-swizzled by the row), the scratch read (rows 4q + lane /
  // 16: offset ^ 64 q, + 1 KiB q) and the store offset within the row group (+ 8 ldy q bytes) --
  // against buffer resources whose base is the row group's first element and whose range ends
  // at row M (checked tiles: rows past M read zeros and are not stored)
  // (recomputed per row group from a fresh lane id: hoisted over the whole epilogue, the four
  // offsets spilled the residual epilogues at 256 VGPRs)
  constexpr bool BUFST = LINE;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t bo_res = 0, bo_wr = 0, bo_rd = 0, bo_st = 0;
    if constexpr (BUFST) {
      const int ln0 = lane_id_here(), l16 = ln0 & 15, l4 = ln0 >> 4;
      bo_res = (uint32_t)((l16 * (int)ldr + 16 * (l4 & 1) + 4 * (l4 & 2)) * 2);
      bo_wr = (uint32_t)(l16 * 256 + (((2 * (l4 & 1) + (l4 >> 1)) ^ l16) << 4));
      bo_rd = (uint32_t)(l4 * 256 + ((l16 ^ l4) << 4));
      bo_st = (uint32_t)((l4 * (int)ldy + l16 * 8) * 2);
    }
    (void)bo_res; (void)bo_wr; (void)bo_rd; (void)bo_st;
    const int m_row = mw0 + j * 16 + (lane & 15);
    // LINE: every lane takes part in the scratch exchange; rows past M compute on row M - 1's
    // operands and are never stored
    if (!LINE && CHECK && m_row >= M) continue;
    const int m = (LINE && CHECK && m_row >= M) ? M - 1 : m_row;
    half8 r16[(RESN || LNR) ? 4 : 1];
    if constexpr ((RESN || LNR) && BUFST) {
      const int row0 = mw0 + j * 16;
      const int64_t nb = CHECK ? (int64_t)max(0, min(16, M - row0)) * ldr * 2 : (int64_t)16 * ldr * 2;
      const auto rr = panel_rsrc(reinterpret_cast<const half_t*>(R) + (int64_t)row0 * ldr + nw0, nb);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
#if defined(__HIP_DEVICE_COMPILE__)
        r16[p] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rr, bo_res + 64 * p, 0, 0));
#else
        (void)rr;
#endif
      }
    } else if constexpr (RESN || LNR) {
#pragma unroll
      for (int p = 0; p < 4; ++p)
        r16[p] = *reinterpret_cast<const half8*>(reinterpret_cast<const half_t*>(R) + (int64_t)m * ldr + nlane + 32 * p);
    }
    float mu = 0.f, rstd = 1.f;
    if constexpr (LNF || LNR) {
      mu = mrj[j].x;
      rstd = mrj[j].y;
    }
    half8 hv[4];
    if constexpr (PACK) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // columns nb .. nb+7 as 4 packed pairs: x[q] = (col 2q, col 2q + 1)
      f2v x[4];
      if constexpr (PERM) {  // W rows staged in perm32 order: the lane's 8 columns as they are
        x[0] = f2v{acc[2 * p][j][0], acc[2 * p][j][1]};
        x[1] = f2v{acc[2 * p][j][2], acc[2 * p][j][3]};
        x[2] = f2v{acc[2 * p + 1][j][0], acc[2 * p + 1][j][1]};
        x[3] = f2v{acc[2 * p + 1][j][2], acc[2 * p + 1][j][3]};
      } else {
#pragma unroll
      for (int r = 0; r < 4; r += 2) {
        const auto s0 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * p][j][r]),
                                                         __float_as_uint(acc[2 * p + 1][j][r]), false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * p][j][r + 1]),
                                                         __float_as_uint(acc[2 * p + 1][j][r + 1]), false, false);
        x[r / 2] = f2v{__uint_as_float(s0[0]), __uint_as_float(s1[0])};
        x[2 + r / 2] = f2v{__uint_as_float(s0[1]), __uint_as_float(s1[1])};
      }
      }
      const f2v bb[4] = {b0[p].xy, b0[p].zw, b1[p].xy, b1[p].zw};
      if constexpr (LNF) {
        const f2v cc[4] = {c0[p].xy, c0[p].zw, c1[p].xy, c1[p].zw};
#pragma unroll
        for (int q = 0; q < 4; ++q)
          x[q] = pk_fma(splat2(rstd), pk_fma(splat2(-mu), cc[q], x[q]), bb[q]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] += bb[q];
      }
      if constexpr (RESN) {
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] += f2v{(float)r16[p][2 * q], (float)r16[p][2 * q + 1]};
      }
      if constexpr (LNR) {
        const f2v cc[4] = {c0[p].xy, c0[p].zw, c1[p].xy, c1[p].zw};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f2v rn = (f2v{(float)r16[p][2 * q], (float)r16[p][2 * q + 1]} - splat2(mu)) * splat2(rstd);
          x[q] = pk_fma(rn, cc[q], x[q]);
        }
      }
      if constexpr (GELU) {
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = gelu_erf2(x[q]);
      }
      if constexpr (GELU2) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if constexpr (GLUT)
            x[q] = f2v{gelu2_t(x[q].x, gtab), gelu2_t(x[q].y, gtab)};
          else
            x[q] = gelu2_erf2(x[q]);
        }
      }
      if constexpr (OUT8) {
        uint2 q8;
        q8.x = e4m3x4(x[0].x, x[0].y, x[1].x, x[1].y);
        q8.y = e4m3x4(x[2].x, x[2].y, x[3].x, x[3].y);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(Y) + (int64_t)m * ldy + nlane + 32 * p) = q8;
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          hv[p][2 * q] = (half_t)x[q].x;
          hv[p][2 * q + 1] = (half_t)x[q].y;
        }
        if constexpr (BUFST)
          *reinterpret_cast<half8*>(reinterpret_cast<char*>(scr) + (bo_wr ^ (uint32_t)(p << 6))) = hv[p];
        else
          *reinterpret_cast<half8*>(reinterpret_cast<half_t*>(Y) + (int64_t)m * ldy + nlane + 32 * p) = hv[p];
        if constexpr (Y8 && !LINE) {  // e4m3 copy of the stored fp16 values for the next fp8 GEMM
          {
            uint2 q8;
            q8.x = e4m3x4((float)hv[p][0], (float)hv[p][1], (float)hv[p][2], (float)hv[p][3]);
            q8.y = e4m3x4((float)hv[p][4], (float)hv[p][5], (float)hv[p][6], (float)hv[p][7]);
            *reinterpret_cast<uint2*>(lf.y8 + (int64_t)m * ldy + nlane + 32 * p) = q8;
          }
        }
      }
    }
    } else {
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (PERM) {
          v[r] = acc[2 * p][j][r];
          v[4 + r] = acc[2 * p + 1][j][r];
        } else {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * p][j][r]),
                                                           __float_as_uint(acc[2 * p + 1][j][r]), false, false);
          v[r] = __uint_as_float(sw[0]);
          v[4 + r] = __uint_as_float(sw[1]);
        }
      }
      if constexpr (LNF) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = fmaf(rstd, v[r] - mu * c0[p][r], b0[p][r]);
          v[4 + r] = fmaf(rstd, v[4 + r] - mu * c1[p][r], b1[p][r]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] += b0[p][r];
          v[4 + r] += b1[p][r];
        }
      }
      if constexpr (RESN) {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] += (float)r16[p][r];
      }
      if constexpr (LNR) {
        // (r - mu) rstd as one FMA with -mu rstd (one VALU per output fewer than sub + mul)
        const float nmr = -mu * rstd;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = fmaf(fmaf((float)r16[p][r], rstd, nmr), c0[p][r], v[r]);
          v[4 + r] = fmaf(fmaf((float)r16[p][4 + r], rstd, nmr), c1[p][r], v[4 + r]);
        }
      }
      if constexpr (GELU) {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = gelu_erf(v[r]);
      }
      if constexpr (GELU2) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          if constexpr (GLUT)
            v[r] = gelu2_t(v[r], gtab);
          else
            v[r] = gelu2_erf(v[r]);
        }
      }
      if constexpr (OUT8) {
        uint2 q8;
        q8.x = e4m3x4(v[0], v[1], v[2], v[3]);
        q8.y = e4m3x4(v[4], v[5], v[6], v[7]);
        *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(Y) + (int64_t)m * ldy + nlane + 32 * p) = q8;
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) hv[p][r] = (half_t)v[r];
        if constexpr (BUFST)
          *reinterpret_cast<half8*>(reinterpret_cast<char*>(scr) + (bo_wr ^ (uint32_t)(p << 6))) = hv[p];
        else
          *reinterpret_cast<half8*>(reinterpret_cast<half_t*>(Y) + (int64_t)m * ldy + nlane + 32 * p) = hv[p];
        if constexpr (Y8 && !LINE) {  // e4m3 copy of the stored fp16 values for the next fp8 GEMM
          {
            uint2 q8;
            q8.x = e4m3x4((float)hv[p][0], (float)hv[p][1], (float)hv[p][2], (float)hv[p][3]);
            q8.y = e4m3x4((float)hv[p][4], (float)hv[p][5], (float)hv[p][6], (float)hv[p][7]);
            *reinterpret_cast<uint2*>(lf.y8 + (int64_t)m * ldy + nlane + 32 * p) = q8;
          }
        }
      }
    }
    }
    if constexpr (BUFST) {
      const int row0 = mw0 + j * 16;
      const int64_t nr = CHECK ? (int64_t)max(0, min(16, M - row0)) : 16;
      const auto ry = panel_rsrc(reinterpret_cast<const half_t*>(Y) + (int64_t)row0 * ldy + nw0, nr * ldy * 2);
      const auto r8 = panel_rsrc(reinterpret_cast<const half_t*>(Y8 ? lf.y8 + (int64_t)row0 * ldy + nw0 : nullptr),
                                 Y8 ? nr * ldy : 0);
      (void)r8;
      typedef int v2i __attribute__((ext_vector_type(2)));
      v2i keep8 = {0, 0};  // Y8: the e4m3 bytes of the even q, paired with the odd q's below
      (void)keep8;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const half8 o = *reinterpret_cast<const half8*>(reinterpret_cast<const char*>(scr) +
                                                        (bo_rd ^ (uint32_t)(q << 6)) + q * 1024);
#if defined(__HIP_DEVICE_COMPILE__)
        typedef int v4i __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, o), ry, bo_st + q * (uint32_t)(8 * ldy), 0, 0);
        if constexpr (Y8) {  // e4m3 copy of the stored fp16 values for the next fp8 GEMM
          const v2i q8 = {(int)e4m3x4((float)o[0], (float)o[1], (float)o[2], (float)o[3]),
                          (int)e4m3x4((float)o[4], (float)o[5], (float)o[6], (float)o[7])};
          if ((q & 1) == 0) {
            keep8 = q8;
          } else {
            // 16-byte copy stores (half the store instructions: the epilogue is store-issue
            // bound): the lanes of a chunk pair (2k, 2k + 1: the same row) trade 8 bytes -- the
            // even lane sends its odd-q chunk, the odd lane its even-q chunk -- so the even lane
            // stores chunks 2k, 2k + 1 of row 4 (q - 1) + lane / 16, the odd lane those of row
            // 4 q + lane / 16
            const int odd = lane_id_here() & 1;
            const v2i send = odd ? keep8 : q8;
            const v2i recv = {__shfl_xor(send.x, 1, 64), __shfl_xor(send.y, 1, 64)};
            const v4i w = odd ? v4i{recv.x, recv.y, q8.x, q8.y} : v4i{keep8.x, keep8.y, recv.x, recv.y};
            __builtin_amdgcn_raw_buffer_store_b128(w, r8, (bo_st >> 1) - 8 * odd + (uint32_t)(q - 1 + odd) * (uint32_t)(4 * ldy),
                                                   0, 0);
          }
        }
#else
        (void)o;
        (void)ry;
#endif
      }
    }
    if constexpr (STATS) {
      // partner lanes (xor 16 / 32) share the row m, so they are active together; the two half
      // spans in store_tile_res's order and arithmetic (the same partials bit for bit)
      float nc, s0, q0, s1, q1;
      half_span_stats<true>(hv[0], hv[1], nc, s0, q0);
      half_span_stats<false>(hv[2], hv[3], nc, s1, q1);
      const float2 sm = span_stats(nc, s0, q0, s1, q1);
      const float sum = sm.x, m2 = sm.y;
      if (g == 0 && (!CHECK || m_row < M)) {
        float2 st;
        st.x = sum;
        st.y = m2;
        *reinterpret_cast<float2*>(lf.stat_out + ((int64_t)m * (N >> 7) + (nw0 >> 7)) * 2) = st;
      }
    }
  }
}

// The LayerNorm-folded FFN1 epilogues (EPI_LNF_GELU_F16 / _F8): 2 GELU(x) = x T(x) from the LDS
// table (gelu2_t), x = rstd (acc - mu c) + b.  Per 8 outputs of one row (column group p, row
// group j): 16 fma of the LayerNorm fold, 7 VALU + one ds_read_b64 each of the GELU.
//   fp16 (scr != nullptr): half-tile outer -- the bias / column sums of column
//     groups 2h, 2h + 1 live at a time (32 VGPRs) -- and per row group the 16 rows x 64 columns
//     pass through the wave's 2 KiB LDS scratch and leave as WHOLE 128-byte lines (8 rows x 128 B
//     per dwordx4 store instead of 16 rows x 64 B): the per-CU store path moves whole lines ~3.7x
//     faster (tools/diag/store_rate.hip) and the FFN1 tile writes 128 KiB.
//   fp8, the W tile staged in perm64 order (PERM, the product): quad outer -- the bias / column
//     sums of the lane's 16 consecutive columns of quad q live at a time (32 VGPRs) -- and ONE
//     16-byte store per (quad, row group): 8 stores per wave, 16 rows x 64 B each (the perm32 form
//     stored 16 x 8 B, 16 rows x 32 B each; whole lines through a 1 KiB scratch measured slower).
//   fallback (diagnostic variants without PERMW): column-group outer, one 8- / 16-byte store per
//     (p, j), 16 per wave.
// DMODE (timing diagnostics, wrong results): 5 = the math (and the scratch exchange) without the
// global stores, 6 = the stores of the raw accumulators without the math.
// CST: the tile's bias / column sums / row statistics come from the LDS table the K-loop staged
// (cst: [256 bias][256 colsum][256 x (mu, rstd)] of the tile; ln0 / lm0 = the wave's column / row
// offset in the tile) instead of global loads: no vmcnt wait inside the epilogue, so its line
// stores drain while the next row groups compute.
template <int EPI, bool CHECK, bool PERM, class Pre = NoPre, int DMODE = 0, bool CST = false>
__device__ __forceinline__ void store_tile_gelu(float4v (&acc)[8][4], int nw0, int mw0, int lane,
                                                int M, const float* __restrict__ bias,
                                                void* __restrict__ Y, int64_t ldy, const LnFold& lf,
                                                const float2* __restrict__ gtab, half_t* __restrict__ scr,
                                                const Pre& pre = Pre{}, const float* __restrict__ cst = nullptr,
                                                int ln0 = 0, int lm0 = 0) {
  constexpr bool OUT8 = EPI == EPI_LNF_GELU_F8;
  static_assert(EPI == EPI_LNF_GELU_F16 || OUT8, "store_tile_gelu: LN-folded FFN1 epilogues");
  const int g = lane >> 4, odd = g & 1;
  const int nlane = nw0 + 16 * odd + 4 * (g & 2);  // + 32 p
  const int clane = ln0 + 16 * odd + 4 * (g & 2);  // CST: the same column in the tile's table
  (void)clane;
  float2 mrj[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if constexpr (CST) {
      // (the table address from a fresh lane id: hoisted out of the tile loop, it spilled at 256
      // VGPRs in the fp8 kernel and its reload waited vmcnt(0) -- the next tile's staging -- here)
      mrj[j] = *reinterpret_cast<const float2*>(cst + 512 + 2 * (lm0 + j * 16 + (lane_id_here() & 15)));
    } else {
      int m = mw0 + j * 16 + (lane & 15);
      m = (CHECK && m >= M) ? M - 1 : m;
      mrj[j] = *reinterpret_cast<const float2*>(lf.mr + (int64_t)m * lf.stat_ld * 2);
    }
  }
  auto load_consts = [&](float4v (&d)[4], int p) __attribute__((always_inline)) {
    if constexpr (CST) {
      d[0] = *reinterpret_cast<const float4v*>(cst + clane + 32 * p);
      d[1] = *reinterpret_cast<const float4v*>(cst + clane + 32 * p + 4);
      d[2] = *reinterpret_cast<const float4v*>(cst + 256 + clane + 32 * p);
      d[3] = *reinterpret_cast<const float4v*>(cst + 256 + clane + 32 * p + 4);
    } else {
      d[0] = *reinterpret_cast<const float4v*>(bias + nlane + 32 * p);
      d[1] = *reinterpret_cast<const float4v*>(bias + nlane + 32 * p + 4);
      d[2] = *reinterpret_cast<const float4v*>(lf.colsum + nlane + 32 * p);
      d[3] = *reinterpret_cast<const float4v*>(lf.colsum + nlane + 32 * p + 4);
    }
  };
  // the 8 outputs of (column group p, row group j): columns nlane + 32 p + 0..7 of row j
  auto gelu8 = [&](float (&v)[8], int p, int j, const float4v (&cst)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (PERM) {
        v[r] = acc[2 * p][j][r];
        v[4 + r] = acc[2 * p + 1][j][r];
      } else {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * p][j][r]),
                                                         __float_as_uint(acc[2 * p + 1][j][r]), false, false);
        v[r] = __uint_as_float(sw[0]);
        v[4 + r] = __uint_as_float(sw[1]);
      }
    }
    if constexpr (DMODE == 6) return;
    const float mu = mrj[j].x, rstd = mrj[j].y;
    // (each value through an empty asm: kept scalar -- SLP packing it into v_pk_fma_f32 cost two
    // v_mov per packed pair here, and packed f32 VALU issues no faster than two scalar ops)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = fmaf(rstd, fmaf(-mu, cst[2][r], v[r]), cst[0][r]);
      v[4 + r] = fmaf(rstd, fmaf(-mu, cst[3][r], v[4 + r]), cst[1][r]);
      asm("" : "+v"(v[r]));
      asm("" : "+v"(v[4 + r]));
    }
    // the 8 table reads issued together, consumed after a scheduling fence (left to the
    // scheduler, each read was awaited right behind its own issue)
    if constexpr (OUT8) {  // nearest node of the 4,097-entry fp32 table
      const float* const t8 = reinterpret_cast<const float*>(gtab);
      float tn[8];
#pragma unroll
      for (int r = 0; r < 8; ++r)
        tn[r] = t8[(uint32_t)__builtin_amdgcn_fmed3f(
            fmaf(v[r], (float)GELU_NT8 / (2.0f * GELU_XMAX), 0.5f * (float)GELU_NT8 + 0.5f), 0.0f, (float)GELU_NT8)];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        // e4m3: 2 GELU >= -0.34, so only the upper saturation bound can apply (e4m3x4's clamp)
        v[r] = fminf(v[r] * tn[r], 448.f);
        asm("" : "+v"(v[r]));
      }
      return;
    }
    float fr[8];
    float2 tv[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const float az = __builtin_amdgcn_ldexpf(
          __builtin_amdgcn_fmed3f(fmaf(v[r], 1.0f / (2.0f * GELU_XMAX), 0.5f), 0.0f, 1.0f), GELU_LOG2_NT);
      fr[r] = __builtin_amdgcn_fractf(az);
      tv[r] = gtab[(uint32_t)az];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      v[r] *= fmaf(fr[r], tv[r].y, tv[r].x);
      asm("" : "+v"(v[r]));
    }
  };
  if constexpr (!OUT8) {
    // ---- fp16, whole-line stores through the 2 KiB scratch (16 rows x 128 B, chunk k of row r
    // at k ^ (r & 7): conflict-free b128 writes and reads) --------------------------------------
    // Every address is a lane constant computed once: the scratch write of pp = 0 (pp = 1 writes
    // chunk k + 4, i.e. byte offset ^ 64: k < 4 and the swizzle XORs 3 bits), the scratch read
    // (rows 8q + lane / 8, chunk lane & 7: q = 1 is + 1 KiB) and the row-group store offset
    // (rows (lane / 8) (+ 8 q) x ldy, 16 B chunk lane & 7) against a buffer resource whose base is
    // the row group's first output (SGPRs) and whose size ends at row M: rows past M are dropped by
    // the range check (no compare / exec mask).  The per-store 64-bit address arithmetic and the
    // recomputed swizzles were ~4 VALU per output, about a third of the epilogue's VALU.
    float4v bc[2][4];  // bias / colsum of column groups 2h, 2h + 1
    load_consts(bc[0], 0);
    load_consts(bc[1], 1);
    if constexpr (!std::is_same<Pre, NoPre>::value) {
      __builtin_amdgcn_sched_barrier(0);
      pre();
      __builtin_amdgcn_sched_barrier(0);
    }
    char* const sb = reinterpret_cast<char*>(scr);
    const int ln0 = lane_id_here();
    const uint32_t wofs = (uint32_t)((ln0 & 15) * 128 +
                                     (((2 * ((ln0 >> 4) & 1) + (ln0 >> 5)) ^ (ln0 & 7)) << 4));
    const uint32_t rofs = (uint32_t)((ln0 >> 3) * 128 + (((ln0 & 7) ^ (ln0 >> 3)) << 4));
    const uint32_t gofs = (uint32_t)(((ln0 >> 3) * (int)ldy + (ln0 & 7) * 8) * 2);
    const uint32_t g8 = (uint32_t)(8 * ldy * 2);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1) {
        load_consts(bc[0], 2);
        load_consts(bc[1], 3);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          float v[8];
          gelu8(v, 2 * h + pp, j, bc[pp]);
          half8 hv;
#pragma unroll
          for (int r = 0; r < 8; ++r) hv[r] = (half_t)v[r];
          *reinterpret_cast<half8*>(sb + (wofs ^ (uint32_t)(pp << 6))) = hv;
        }
        const int row0 = mw0 + j * 16;
        const int64_t nb = CHECK ? (int64_t)max(0, min(16, M - row0)) * ldy * 2 : (int64_t)16 * ldy * 2;
        const auto ry = panel_rsrc(reinterpret_cast<const half_t*>(Y) + (int64_t)row0 * ldy + nw0 + 64 * h, nb);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const half8 o = *reinterpret_cast<const half8*>(sb + rofs + q * 1024);
          if constexpr (DMODE == 5) {
            if ((float)o[0] == 12345.f) reinterpret_cast<half_t*>(Y)[ln0] = o[1];
          } else {
#if defined(__HIP_DEVICE_COMPILE__)
            typedef int v4i __attribute__((ext_vector_type(4)));
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, o), ry, gofs + q * g8, 0, kFfn1StoreAux);
#else
            (void)ry;
            (void)gofs;
            (void)g8;
#endif
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // the second half's constant loads stay here
    }
  } else if constexpr (OUT8 && PERM) {
    // ---- fp8, perm64 tile: lane group g owns columns 64 q + 16 g .. + 15 of quad q ----------------
    auto load16 = [&](float4v (&d)[4], int q, int hh) __attribute__((always_inline)) {
      const int col = 64 * q + 16 * g + 8 * hh;  // the 8 columns of gelu8's p = 2 q + hh
      if constexpr (CST) {
        d[0] = *reinterpret_cast<const float4v*>(cst + ln0 + col);
        d[1] = *reinterpret_cast<const float4v*>(cst + ln0 + col + 4);
        d[2] = *reinterpret_cast<const float4v*>(cst + 256 + ln0 + col);
        d[3] = *reinterpret_cast<const float4v*>(cst + 256 + ln0 + col + 4);
      } else {
        d[0] = *reinterpret_cast<const float4v*>(bias + nw0 + col);
        d[1] = *reinterpret_cast<const float4v*>(bias + nw0 + col + 4);
        d[2] = *reinterpret_cast<const float4v*>(lf.colsum + nw0 + col);
        d[3] = *reinterpret_cast<const float4v*>(lf.colsum + nw0 + col + 4);
      }
    };
    float4v bc[2][4];
    load16(bc[0], 0, 0);
    load16(bc[1], 0, 1);
    if constexpr (!std::is_same<Pre, NoPre>::value) {
      __builtin_amdgcn_sched_barrier(0);
      pre();
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (q == 1) {
        load16(bc[0], 1, 0);
        load16(bc[1], 1, 1);
      }
      // (lane-constant byte offset of the lane's 16 bytes in a row group; rows past M are dropped
      // by the buffer resource's range)
      const int ln = lane_id_here();
      const uint32_t bo = (uint32_t)((ln & 15) * (int)ldy + 64 * q + 16 * (ln >> 4));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v0[8], v1[8];
        gelu8(v0, 2 * q, j, bc[0]);
        gelu8(v1, 2 * q + 1, j, bc[1]);
        if constexpr (DMODE == 5) {
          float z = 0.f;
#pragma unroll
          for (int r = 0; r < 8; ++r) z += v0[r] + v1[r];
          if (z == 12345.678f) reinterpret_cast<float*>(Y)[lane] = z;
        } else {
          typedef int v4i __attribute__((ext_vector_type(4)));
          const v4i o = {__builtin_amdgcn_cvt_pk_fp8_f32(v0[2], v0[3], __builtin_amdgcn_cvt_pk_fp8_f32(v0[0], v0[1], 0, false), true),
                         __builtin_amdgcn_cvt_pk_fp8_f32(v0[6], v0[7], __builtin_amdgcn_cvt_pk_fp8_f32(v0[4], v0[5], 0, false), true),
                         __builtin_amdgcn_cvt_pk_fp8_f32(v1[2], v1[3], __builtin_amdgcn_cvt_pk_fp8_f32(v1[0], v1[1], 0, false), true),
                         __builtin_amdgcn_cvt_pk_fp8_f32(v1[6], v1[7], __builtin_amdgcn_cvt_pk_fp8_f32(v1[4], v1[5], 0, false), true)};
          const int row0 = mw0 + j * 16;
          const int64_t nb = CHECK ? (int64_t)max(0, min(16, M - row0)) * ldy : (int64_t)16 * ldy;
          const auto ry = panel_rsrc(reinterpret_cast<const half_t*>(reinterpret_cast<const uint8_t*>(Y) +
                                                                     (int64_t)row0 * ldy + nw0), nb);
#if defined(__HIP_DEVICE_COMPILE__)
          __builtin_amdgcn_raw_buffer_store_b128(o, ry, bo, 0, 0);
#else
          (void)o;
          (void)ry;
          (void)bo;
#endif
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // the second quad's constant loads stay here
    }
  } else {
    // ---- column-group outer, one 8- / 16-byte store per (p, j) -----------------------------------
    float4v bc[2][4];  // [buffer][b0, b1, c0, c1] of column group p
    load_consts(bc[0], 0);
    if constexpr (!std::is_same<Pre, NoPre>::value) {
      __builtin_amdgcn_sched_barrier(0);
      pre();
      __builtin_amdgcn_sched_barrier(0);
    }
    // fp8 (BUFST8): the e4m3 rows leave through a range-checked buffer resource per row group
    // (rows past M dropped by the bounds check, no exec mask) at one lane offset per column group
    constexpr bool B8 = OUT8 && DMODE == 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p < 3) load_consts(bc[(p + 1) & 1], p + 1);
      uint32_t bo8 = 0;
      if constexpr (B8) {
        const int ln0 = lane_id_here(), g0 = ln0 >> 4;
        bo8 = (uint32_t)((ln0 & 15) * (int)ldy + 16 * (g0 & 1) + 4 * (g0 & 2) + 32 * p);
      }
      (void)bo8;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mw0 + j * 16 + (lane & 15);
        if (!B8 && CHECK && m >= M) continue;
        float v[8];
        gelu8(v, p, j, bc[p & 1]);
        if constexpr (DMODE == 5) {
          float z = 0.f;
#pragma unroll
          for (int r = 0; r < 8; ++r) z += v[r];
          if (z == 12345.678f) reinterpret_cast<float*>(Y)[lane] = z;
        } else if constexpr (OUT8) {
          uint2 q8;
          q8.x = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(
              v[2], v[3], __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false), true);
          q8.y = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(
              v[6], v[7], __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false), true);
          if constexpr (B8) {
            const int row0 = mw0 + j * 16;
            const int64_t nb = CHECK ? (int64_t)max(0, min(16, M - row0)) * ldy : (int64_t)16 * ldy;
            const auto ry = panel_rsrc(reinterpret_cast<const half_t*>(reinterpret_cast<const uint8_t*>(Y) +
                                                                       (int64_t)row0 * ldy + nw0), nb);
#if defined(__HIP_DEVICE_COMPILE__)
            typedef int v2i __attribute__((ext_vector_type(2)));
            __builtin_amdgcn_raw_buffer_store_b64(v2i{(int)q8.x, (int)q8.y}, ry, bo8, 0, 0);
#else
            (void)ry;
#endif
          } else {
            *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(Y) + (int64_t)m * ldy + nlane + 32 * p) = q8;
          }
        } else {
          half8 hv;
#pragma unroll
          for (int r = 0; r < 8; ++r) hv[r] = (half_t)v[r];
          *reinterpret_cast<half8*>(reinterpret_cast<half_t*>(Y) + (int64_t)m * ldy + nlane + 32 * p) = hv;
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the next groups' constant loads where they are
    }
  }
}

// The persistent residual + statistics epilogues (EPI_RES16_STATS / EPI_LNR16_STATS and their
// e4m3-copy forms) in half-tile order, the FFN1 epilogue's layout:
//   * bias, the residual's LayerNorm weight and the tile's row statistics come from the LDS table
//     the K-loop staged (cst: [256 bias][256 gamma][256 x (mu, rstd)]), no global constant loads;
//   * half h (column groups 2h, 2h + 1) outer, row group j inner: the 16 rows x 64 columns pass
//     through the wave's 2 KiB line scratch and leave as whole 128-B lines (2 stores per (h, j));
//   * the residual of step s + 1 = (h, j) + 1 is loaded before step s's stores, so its wait (vmcnt
//     counts in issue order) does not also wait for those stores; step 0's is loaded before the
//     next tile's staging burst (pre), so the first wait does not wait for the 16 pieces either;
//   * the row's sum / M2 partials accumulate over both halves in the order of store_tile_wide
//     (same fp16 outputs, same partials bit for bit).
// Register budget: the tile's 128 accumulators + 32 constants of one half + 2 x 8 residual.
template <int EPI, bool CHECK, bool PERM, class Pre = NoPre>
__device__ __forceinline__ void store_tile_res(float4v (&acc)[8][4], int nw0, int mw0, int lane, int M, int N,
                                               const void* __restrict__ R, int64_t ldr,
                                               void* __restrict__ Y, int64_t ldy, const LnFold& lf,
                                               half_t* __restrict__ scr, const Pre& pre,
                                               const float* __restrict__ cst, int ln0, int lm0) {
  constexpr bool Y8 = EPI == EPI_RES16_STATS_Y8 || EPI == EPI_LNR16_STATS_Y8;
  constexpr bool LNR = EPI == EPI_LNR16_STATS || EPI == EPI_LNR16_STATS_Y8;
  static_assert(LNR || EPI == EPI_RES16_STATS || EPI == EPI_RES16_STATS_Y8, "store_tile_res: residual epilogues");
  static_assert(PERM, "store_tile_res: the W tile staged in perm32 order (8 consecutive columns per lane)");
  // (the lane recomputed here: the caller's copy, live across the K-loop, was spilled at 256 VGPRs
  // and its reload's vmcnt(0) waited for the epilogue's residual loads)
  (void)lane;
  const int lid = lane_id_here();
  const int g = lid >> 4, odd = g & 1;
  const int clane = ln0 + 16 * odd + 4 * (g & 2);  // the lane's column in the tile's table (+ 32 p)
  // lane-constant byte offsets: the residual segment of row (lid & 15) (+ 64 B per column group),
  // the scratch write / read-back and the row-group store offsets of store_tile_gelu
  const uint32_t bo_res = (uint32_t)(((lid & 15) * (int)ldr + 16 * ((lid >> 4) & 1) + 4 * ((lid >> 4) & 2)) * 2);
  const uint32_t wofs = (uint32_t)((lid & 15) * 128 + (((2 * ((lid >> 4) & 1) + (lid >> 5)) ^ (lid & 7)) << 4));
  const uint32_t rofs = (uint32_t)((lid >> 3) * 128 + (((lid & 7) ^ (lid >> 3)) << 4));
  const uint32_t gofs = (uint32_t)(((lid >> 3) * (int)ldy + (lid & 7) * 8) * 2);
  const uint32_t g8 = (uint32_t)(8 * ldy * 2);
  char* const sb = reinterpret_cast<char*>(scr);
  auto load_res = [&](half8 (&r)[2], int st) __attribute__((always_inline)) {
    const int h = st >> 2, row0 = mw0 + (st & 3) * 16;
    const int64_t nb = CHECK ? (int64_t)max(0, min(16, M - row0)) * ldr * 2 : (int64_t)16 * ldr * 2;
    const auto rr = panel_rsrc(reinterpret_cast<const half_t*>(R) + (int64_t)row0 * ldr + nw0, nb);
#if defined(__HIP_DEVICE_COMPILE__)
    r[0] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rr, bo_res + 128 * h, 0, 0));
    r[1] = __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(rr, bo_res + 128 * h + 64, 0, 0));
#else
    (void)rr;
#endif
  };
  half8 rA[2], rB[2];
  load_res(rA, 0);
  if constexpr (!std::is_same<Pre, NoPre>::value) {
    __builtin_amdgcn_sched_barrier(0);
    pre();
    __builtin_amdgcn_sched_barrier(0);
  }
  float4v bc[2][2], gc[2][2];  // bias / gamma of column groups 2h, 2h + 1
  // the first half's reduced row sums, squared deviations and pivots, parked one row group per lane
  // group: lane group g keeps row group g's (3 VGPRs; four of each per lane spilled at 256 VGPRs)
  float park_s = 0.f, park_q = 0.f, park_nc = 0.f;
#pragma unroll
  for (int st = 0; st < 8; ++st) {
    const int h = st >> 2, j = st & 3;
    if (j == 0) {
#pragma unroll
      for (int pp = 0; pp < 2; ++pp) {
        const int p = 2 * h + pp;
        bc[pp][0] = *reinterpret_cast<const float4v*>(cst + clane + 32 * p);
        bc[pp][1] = *reinterpret_cast<const float4v*>(cst + clane + 32 * p + 4);
        if constexpr (LNR) {
          gc[pp][0] = *reinterpret_cast<const float4v*>(cst + 256 + clane + 32 * p);
          gc[pp][1] = *reinterpret_cast<const float4v*>(cst + 256 + clane + 32 * p + 4);
        }
      }
    }
    half8 (&rc)[2] = (st & 1) ? rB : rA;
    if (st < 7) load_res((st & 1) ? rA : rB, st + 1);
    float mu = 0.f, rstd = 1.f;
    if constexpr (LNR) {
      const float2 mr = *reinterpret_cast<const float2*>(cst + 512 + 2 * (lm0 + j * 16 + (lid & 15)));
      mu = mr.x;
      rstd = mr.y;
    }
    half8 hv[2];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int p = 2 * h + pp;
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[2 * p][j][r] + bc[pp][0][r];
        v[4 + r] = acc[2 * p + 1][j][r] + bc[pp][1][r];
      }
      if constexpr (LNR) {
        const float nmr = -mu * rstd;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = fmaf(fmaf((float)rc[pp][r], rstd, nmr), gc[pp][0][r], v[r]);
          v[4 + r] = fmaf(fmaf((float)rc[pp][4 + r], rstd, nmr), gc[pp][1][r], v[4 + r]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] += (float)rc[pp][r];
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) hv[pp][r] = (half_t)v[r];
      *reinterpret_cast<half8*>(sb + (wofs ^ (uint32_t)(pp << 6))) = hv[pp];
    }
    // statistics of this half span (store_tile_wide's arithmetic: the same partials bit for bit);
    // the first half parks its results in lane group j, the second fetches them back
    float nc, hs, hq;
    if (h == 0) {
      half_span_stats<true>(hv[0], hv[1], nc, hs, hq);
      const bool mine = g == j;
      park_s = mine ? hs : park_s;
      park_q = mine ? hq : park_q;
      park_nc = mine ? nc : park_nc;
    } else {
      nc = __shfl(park_nc, (lid & 15) + 16 * j, 64);
      half_span_stats<false>(hv[0], hv[1], nc, hs, hq);
    }
    // read back as 8 rows x 128 B per instruction and store (rows past M dropped by the range)
    const int row0 = mw0 + j * 16;
    const int64_t nr = CHECK ? (int64_t)max(0, min(16, M - row0)) : 16;
    const auto ry = panel_rsrc(reinterpret_cast<const half_t*>(Y) + (int64_t)row0 * ldy + nw0 + 64 * h, nr * ldy * 2);
    const auto r8 = panel_rsrc(reinterpret_cast<const half_t*>(Y8 ? lf.y8 + (int64_t)row0 * ldy + nw0 + 64 * h : nullptr),
                               Y8 ? nr * ldy : 0);
    (void)r8;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const half8 o = *reinterpret_cast<const half8*>(sb + rofs + q * 1024);
#if defined(__HIP_DEVICE_COMPILE__)
      typedef int v4i __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, o), ry, gofs + q * g8, 0, 0);
      if constexpr (Y8) {  // e4m3 copy of the stored fp16 values for the next fp8 GEMM
        typedef int v2i __attribute__((ext_vector_type(2)));
        const v2i q8 = {(int)e4m3x4((float)o[0], (float)o[1], (float)o[2], (float)o[3]),
                        (int)e4m3x4((float)o[4], (float)o[5], (float)o[6], (float)o[7])};
        __builtin_amdgcn_raw_buffer_store_b64(q8, r8, (gofs >> 1) + q * (g8 >> 1), 0, 0);
      }
#else
      (void)o;
      (void)ry;
#endif
    }
    if (h == 1) {
      const float2 sm = span_stats(nc, __shfl(park_s, (lid & 15) + 16 * j, 64), __shfl(park_q, (lid & 15) + 16 * j, 64),
                                   hs, hq);
      const float sum = sm.x, m2 = sm.y;
      const int m_row = row0 + (lid & 15);
      if (g == 0 && (!CHECK || m_row < M)) {
        float2 stv;
        stv.x = sum;
        stv.y = m2;
        *reinterpret_cast<float2*>(lf.stat_out + ((int64_t)m_row * (N >> 7) + (nw0 >> 7)) * 2) = stv;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One epilogue for the pipelined kernels; NSTORE = global store instructions per wave on the
// unchecked path (the persistent kernel's counted vmcnt relies on it: extra stores, such as the
// statistics of the *_STATS epilogues, only make its waits stricter).
template <int EPI>
struct PipeEpi {
  static constexpr bool WIDE = !(EPI == EPI_BIAS_RES_F32 || EPI == EPI_BIAS_TANH_F32);
  // (the fp8-output FFN1 epilogue through its scratch: 8 x 16-B stores, 16 rows x 64 B each)
  static constexpr int NSTORE = WIDE ? 16 : 32;
  template <bool CHECK, bool LINE = false, bool GLUT = false, bool PERM = false, class Pre = NoPre,
            bool CST = false>
  __device__ __forceinline__ static void run(float4v (&acc)[8][4], int nw0, int mw0, int lane, int M,
                                             int N, const float* __restrict__ bias,
                                             const void* __restrict__ R, int64_t ldr,
                                             void* __restrict__ Y, int64_t ldy, const LnFold& lf,
                                             half_t* __restrict__ scr = nullptr,
                                             const float2* __restrict__ gtab = nullptr,
                                             const Pre& pre = Pre{}, const float* __restrict__ cst = nullptr,
                                             int ln0 = 0, int lm0 = 0) {
    if constexpr (WIDE && GLUT && (EPI == EPI_LNF_GELU_F16 || EPI == EPI_LNF_GELU_F8))
      store_tile_gelu<EPI, CHECK, PERM, Pre, 0, CST>(acc, nw0, mw0, lane, M, bias, Y, ldy, lf, gtab, scr, pre,
                                                     cst, ln0, lm0);
    else if constexpr (WIDE && CST && (EPI == EPI_RES16_STATS || EPI == EPI_LNR16_STATS ||
                                       EPI == EPI_RES16_STATS_Y8 || EPI == EPI_LNR16_STATS_Y8))
      store_tile_res<EPI, CHECK, PERM, Pre>(acc, nw0, mw0, lane, M, N, R, ldr, Y, ldy, lf, scr, pre, cst, ln0, lm0);
    else if constexpr (WIDE)
      store_tile_wide<EPI, CHECK, LINE, GLUT, PERM, Pre>(acc, nw0, mw0, lane, M, N, bias, R, ldr, Y, ldy, lf, scr, gtab, pre);
    else
    {
      pre();
      store_tile_fast<EPI, CHECK, 8, 4>(acc, nw0, mw0, lane, M, bias, R, ldr, Y, ldy);
    }
  }
};

// EPI_SCAN epilogue (K1 threshold mode on the GEMM main loop): lane owns
// sim(row n = nw0 + 16i + 4(lane>>4) + r, query q = mw0 + 16j + (lane&15)) of the chunk; keys of
// rows with sim >= tau[q] are appended to q's candidate list (cap entries, overflow counted).
// Reading the rows' live flags here cost a load per row per tile on the critical path (and VGPRs
// the fp8 main loop needs): the selection filters tombstoned rows instead.
// tau of the lane's 4 query columns from the workgroup's LDS copy (written once per launch by
// scan_tau_table; q >= B holds +inf).  Loading them from global memory in the epilogue made the
// wait (vmcnt counts in order) also wait for the next tile's 32 in-flight staging pieces, and
// holding them in VGPRs across the last K-step spilled.
__device__ __forceinline__ void scan_tau(float (&t)[4], int mw0, int lane, const float* tau_lds) {
#pragma unroll
  for (int j = 0; j < 4; ++j) t[j] = tau_lds[mw0 + 16 * j + (lane & 15)];
}

__device__ __forceinline__ void scan_epilogue(float4v (&acc)[8][4], const float (&t)[4], int nw0,
                                              int mw0, int lane, int nrows,
                                              uint64_t* __restrict__ cand, int cap, const LnFold& lf) {
  // Fast rejection: almost every tile of a threshold chunk has no key above tau, and testing the
  // 128 values one by one cost a compare + exec-mask branch each (~3k cycles per wave per tile,
  // as long as the fp8 tile's main loop).  A v_max3 tree per query column decides it in ~45 VALU;
  // only lanes holding a hit take the exact per-value path below (same keys).  Rows past nrows
  // (zero-padded by the staging; only in a chunk's last tile) are masked out of the maxima.
  bool hit = false;
  if (nw0 + 128 <= nrows) {  // wave-uniform
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float mx = acc[0][j][0];
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = (i == 0 ? 1 : 0); r < 4; ++r) mx = fmaxf(mx, acc[i][j][r]);
      hit |= mx >= t[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int nb = nw0 + 16 * i + 4 * (lane_id_here() >> 4);
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, nb + r < nrows ? acc[i][j][r] : -INFINITY);
      }
      hit |= mx >= t[j];
    }
  }
  if (__builtin_amdgcn_ballot_w64(hit) == 0) return;  // wave-uniform: no key in this wave's tile
  // lane-derived offsets re-derived here (kept live from the kernel's prologue, the fp8 kernel
  // spilled one and its reload waited vmcnt(0) on the next tile's staging every tile)
  lane = lane_id_here();
  const int g = lane >> 4;
  int* const cnt = reinterpret_cast<int*>(lf.stat_out);
  // Slot reservation: one returning atomic per (query column, wave) instead of one per key.  In
  // the early threshold chunks (tau still loose) most tiles hold keys, and the per-key atomics,
  // each awaited before its store, serialised on the 256 shared counters (a 65k-row chunk took
  // 200 us for one tile per CU).  The 4 lanes of a query column (lane & 15 equal, g = 0..3) add
  // their counts by two xor-shuffles; lane g = 0 reserves the column's range; each lane writes its
  // keys from base + (keys of the lanes g' < g).  Counts, overflow and the key set are unchanged.
  int c[4], pre[4], base[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int nb = nw0 + 16 * i + 4 * g;
#pragma unroll
      for (int r = 0; r < 4; ++r) c[j] += (nb + r < nrows && acc[i][j][r] >= t[j]) ? 1 : 0;
    }
    const int x1 = __shfl_xor(c[j], 16, 64);
    const int s2 = c[j] + x1;
    const int x2 = __shfl_xor(s2, 32, 64);
    pre[j] = ((g & 1) ? x1 : 0) + ((g & 2) ? x2 : 0);
    c[j] = s2 + x2;  // the column's total from here on
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // the 4 reservations in flight together
    base[j] = 0;
    if (g == 0 && c[j] > 0) base[j] = atomicAdd(cnt + mw0 + 16 * j + (lane & 15), c[j]);
  }
  // (no live flags here: tombstoned rows' keys are dropped by the selection, topk_select)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (c[j] == 0) continue;  // no key in this column (any lane): skip the broadcast too
    const int q = mw0 + 16 * j + (lane & 15);
    int pos = __shfl(base[j], lane & 15, 64) + pre[j];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int nb = nw0 + 16 * i + 4 * g;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float sim = acc[i][j][r];
        if (nb + r < nrows && sim >= t[j]) {  // false for padded queries (t = inf)
          if (pos < cap) cand[(int64_t)q * cap + pos] = make_key(sim, (uint32_t)(lf.stat_ld + nb + r));
          ++pos;
        }
      }
    }
  }
}

// Buffer-resource LDS-DMA staging (buffer_load_dwordx4 ... lds, panel_rsrc in sr_common.h): the
// tile's panel base lives in the SGPR descriptor, the K offset in soffset, so a lane keeps ONE
// 32-bit VGPR offset per instruction for the whole kernel; rows past num_records read as zero.
template <int NI>
__device__ __forceinline__ void stage_buf(__amdgpu_buffer_rsrc_t rs, const uint32_t (&voff)[NI],
                                          int soff, half_t* lds_tile, int wave) {
#if defined(__HIP_DEVICE_COMPILE__)  // device-only builtin: its host-pass instantiation made hipcc
                                     // drop the host launch stubs of the kernel templates using it
#pragma unroll
  for (int i = 0; i < NI; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, SR_LDS(lds_tile + (wave * NI + i) * 8 * GBK), 16,
                                             voff[i], soff, 0, 0);
#endif
}
template <int NI>
__device__ __forceinline__ void stage_offsets(uint32_t (&voff)[NI], int64_t ld, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = (wave * NI + i) * 8 + (lane >> 3);
    voff[i] = (uint32_t)(((int64_t)r * ld + swz_chunk(r, lane & 7) * 8) * 2);
  }
}

// Scheduling pin for one phase: R LDS fragment reads spread among its 16 MFMAs (the MFMAs of the
// phase go first so the wait for the phase's own operands does not also wait for these reads).
#define SR_INTERLEAVE(R)                                                   \
  do {                                                                     \
    _Pragma("unroll") for (int _r = 0; _r < (R); ++_r) {                   \
      __builtin_amdgcn_sched_group_barrier(0x008, 16 / (R) / 2 > 0 ? 16 / (R) / 2 : 1, 0); \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                   \
    }                                                                      \
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);                    \
    __builtin_amdgcn_sched_barrier(0);                                     \
  } while (0)

// The same for a phase of 8 (fp8) MFMAs: R reads after the first MFMAs, about one per MFMA.
#define SR_INTERLEAVE8(R)                                                  \
  do {                                                                     \
    _Pragma("unroll") for (int _r = 0; _r < 8; ++_r) {                     \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                   \
      __builtin_amdgcn_sched_group_barrier(0x100, ((R) + 7) / 8, 0);       \
    }                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                     \
  } while (0)

// PERSIST: one workgroup per CU walks a contiguous per-XCD tile range.  The next tile's first two
// K-steps are staged (glds) right after the last K-step's barrier, before the epilogue, and the
// epilogue's stores are left in flight: the next tile's first waits count them (vmcnt(8 + 32) /
// vmcnt(32): the unchecked epilogue issues exactly FN * FM = 32 global stores per wave, checked in
// the ISA; 16 dwordx4 stores for the fp16 outputs), so the store drain overlaps the next tile's
// MFMAs instead of stalling the CU.
// DIAG (timing experiments only, wrong results): 1 = no glds inside the K-loop (LDS re-read),
// 2 = no epilogue (one masked store per lane keeps the accumulators live).
template <int EPI, bool PERSIST, int DIAG = 0, bool F8IN = false>
__global__ __launch_bounds__(512, 2) void gemm_pipe_kernel(
    const half_t* __restrict__ X, int64_t lda, const half_t* __restrict__ W,
    const float* __restrict__ bias, const void* __restrict__ R, int64_t ldr,
    void* __restrict__ Y, int64_t ldy, int M, int N, int K, const LnFold lf) {
  constexpr int BN = 256, BM = 256;
  constexpr int STAGE = (BN + BM) * GBK;  // halfs per buffer (64 KiB)
  // fp8 operands (EPI_SCAN8): K, lda count 2-byte units, so the staging below moves the same
  // 128-byte K-step rows; a K-step then holds 128 fp8 elements
  constexpr bool F8W = F8IN;  // fp8 activations x fp8 weights (row exponents in lf.wexp)
  constexpr bool F8 = EPI == EPI_SCAN8 || F8W;
  constexpr bool SCAN = EPI == EPI_SCAN || EPI == EPI_SCAN8;
  constexpr int EPI_OUT = EPI;
  // whole-line epilogue stores: a 4 KiB LDS scratch per wave after the two 64 KiB stages (one
  // array: a second __shared__ object made the compiler wait vmcnt(0) before the K-loop's reads)
  // (the e4m3-output epilogues never take the line path: no scratch for them)
  // (DIAG 9 = the product epilogue with stamps: the residual epilogues' line path too)
  constexpr bool LINE = PipeEpi<EPI>::WIDE && !SCAN && (DIAG == 0 || DIAG == 9) && EPI != EPI_LNF_GELU_F8 &&
                        EPI != EPI_BIAS_GELU_F16 && EPI != EPI_LNF_GELU_F16;
  // (EPI_SCAN / EPI_SCAN8: a 1 KiB tau table of the <= 256 queries past the stages)
  // GLUT: the FFN1 epilogues' 8 KiB erfc table (gelu2_t) past the stages / line scratch
  // STAMP (diagnostic library: sr_diag_ffn1 diag 9 = the product epilogue, 10 = its math without
  // the stores): per-wave s_memtime phase sums of every tile -- K-step 0, K-step 1, the rest of
  // the K-loop, the epilogue, the tile transition -- stored once at the end (lf.y8 as uint64 [8]
  // per wave); the stamps themselves cost a lgkmcnt(0) right behind a barrier
  constexpr bool STAMP = DIAG == 9 || DIAG == 10 || DIAG == 11;  // (11: 9 without the next tile's staging)
  constexpr bool GLUT = (DIAG == 0 || DIAG == 5 || DIAG == 6 || DIAG == 7 || STAMP) &&
                        (EPI == EPI_LNF_GELU_F16 || EPI == EPI_LNF_GELU_F8);
  // float2 entries (the fp8 FFN1's nearest-node table: GELU_NT8 + 1 floats)
  constexpr int GTAB = (EPI == EPI_LNF_GELU_F8) ? (GELU_NT8 + 2) / 2 : GELU_NT + 1;
  // PERMW: the W tile's rows are staged in perm32 order (wide epilogues only: the scan epilogue
  // and the 32-bit-output epilogues index the rows as staged)
  constexpr bool PERMW = PipeEpi<EPI>::WIDE && !SCAN && (DIAG == 0 || DIAG >= 5);
  // P64: the e4m3-output FFN1 stages its W rows in perm64 order instead (store_tile_gelu: one
  // 16-byte store per quad and row group, 8 per wave)
  constexpr bool P64 = PERMW && EPI == EPI_LNF_GELU_F8;
  // global store instructions per wave the epilogue leaves in flight (the diagnostics without
  // stores leave none: their waits must not let the next tile's staging loads through)
  constexpr int NST = (DIAG == 5 || DIAG == 10) ? 0 : P64 ? 8 : PipeEpi<EPI>::NSTORE;
  // GLINE: the fp16 FFN1 epilogue's 2 KiB per-wave line scratch (store_tile_gelu)
  constexpr bool GLINE = GLUT && EPI == EPI_LNF_GELU_F16;
  // CSTL: the FFN1 epilogue's per-tile constants -- bias and column sums of the tile's 256 columns,
  // (mu, rstd) of its 256 rows: 4 KiB -- reach LDS by LDS-DMA during the tile's K-loop (group 1,
  // with its K-step 3 burst) instead of as global loads inside the epilogue: vmcnt is in order, so
  // the epilogue's constant loads made it wait for the next tile's in-flight K-step 0 / 1 pieces,
  // and the second half's for the first half's 8 line STORES (write completion, the whole chip
  // storing at once) -- measured in-kernel as an epilogue of 11.2k cycles with stores vs 4.4k
  // without (profiles/r05c/ffn1_stamps.log)
  constexpr bool CSTL = GLUT;
  // RHALF: the persistent residual + statistics epilogues in half-tile order (store_tile_res): a
  // 2 KiB line scratch per wave and the same 4 KiB constants table ([256 bias][256 gamma][256 x
  // (mu, rstd)]; RES16: the bias only), the next tile's staging issued from inside the epilogue
  constexpr bool RLNR = EPI == EPI_LNR16_STATS || EPI == EPI_LNR16_STATS_Y8;
  // (EPI_LNR16_STATS on fp16 operands only.  Round 5: the RES16 and fp8-operand instantiations
  // spilled 12-36 B in this form, profiles/r05_res_half/, r05_wexp_lds/.  Round 6: with the parked
  // statistics the RES16 and the e4m3-copy LNR (fp8 mode 3's O-projection) fit with no spills, and
  // measured the same as the old epilogue: config 5 619.6-622.4 vs 620.5-621.0 q/s, config 4
  // 500.5 vs 500.5 q/s, one box (profiles/r06_res_half_y8/); left as they were.)
  constexpr bool RHALF = EPI == EPI_LNR16_STATS && !F8IN && LINE && PERSIST;
  constexpr bool CSTX = CSTL || RHALF;              // an epilogue constants table in LDS
  constexpr int NCST = CSTL ? 4 : RHALF ? (RLNR ? 4 : 1) : 0;  // its 1 KiB pieces (one per wave)
  constexpr int LSCR = LINE ? (RHALF ? 8 * 1024 : 8 * 2048) : 0;
  constexpr int LDS_BASE = 2 * STAGE + LSCR + (GLINE ? 8 * 1024 : 0) + (CSTX ? 2048 : 0) + (SCAN ? 512 : 0) +
                           (GLUT ? 4 * GTAB : 0);
  __shared__ __attribute__((aligned(16))) half_t lds[LDS_BASE];
  float* const cst = reinterpret_cast<float*>(lds + 2 * STAGE + LSCR + (GLINE ? 8 * 1024 : 0));
  (void)cst;
  float2* const gtab = reinterpret_cast<float2*>(lds + 2 * STAGE + LSCR + (GLINE ? 8 * 1024 : 0) +
                                                 (CSTX ? 2048 : 0));
  // LATE: the next tile's first two K-steps are staged from inside the epilogue, right after its
  // first residual load (store_tile_res's pre hook) instead of at the last K-step's barrier (for
  // the other epilogues measured -0.3 % end to end, profiles/r03_gemm_epilogue_ab/)
  constexpr bool LATE = RHALF && PERSIST && !SCAN && (DIAG == 0 || DIAG == 9) && PipeEpi<EPI>::WIDE;

  const int tiles_n = (N + BN - 1) / BN;  // N % 256 == 0 except for EPI_SCAN (corpus chunk rows)
  const int nwg = tiles_n * ((M + BM - 1) / BM);
  int t, t_end, t_step;
  {
    const int xcd = blockIdx.x & 7, q = nwg >> 3, rem = nwg & 7;
    const int lo = xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
    t = lo + (blockIdx.x >> 3);
    if constexpr (PERSIST) {  // grid = 8 x G (host-checked), so every XCD group has G >= 1 walkers
      t_end = lo + q + (xcd < rem ? 1 : 0);
      t_step = gridDim.x >> 3;
    } else {
      t_end = t + 1;
      t_step = 1;
    }
  }
  if (t >= t_end || t_step <= 0) return;
  // tile walk: n fastest, or groups of lf.group_m m-panels with m fastest inside a group (a window
  // of concurrent tiles then shares fewer W column tiles in the XCD's L2)
  const int gm = lf.group_m, tiles_m = (M + BM - 1) / BM;
  // (only called for tt < nwg; gsz is clamped to >= 1 so no argument can divide by zero)
  auto tile_m = [&](int tt) __attribute__((always_inline)) {
    if (gm <= 1) return tt / tiles_n;
    const int first = (tt / (gm * tiles_n)) * gm, gsz = max(1, min(gm, tiles_m - first));
    return first + (tt - first * tiles_n) % gsz;
  };
  auto tile_n = [&](int tt) __attribute__((always_inline)) {
    if (gm <= 1) return tt % tiles_n;
    const int first = (tt / (gm * tiles_n)) * gm, gsz = max(1, min(gm, tiles_m - first));
    return (tt - first * tiles_n) / gsz;
  };
  int m0 = tile_m(t) * BM, n0 = tile_n(t) * BN;


  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 2, wm = wave & 3;
  // the epilogue's per-wave scratch: LINE 4 KiB / GLINE 2 KiB (nothing else uses it)
  half_t* const escr = lds + 2 * STAGE + wave * ((GLINE || RHALF) ? 1024 : 2048);
  half_t* const gscr = GLINE ? escr : nullptr;
  (void)gscr;
  const int nk = K / GBK;
  const int kxs = lf.x_k > 0 ? lf.x_k / GBK : nk;  // K-steps of the X operand (split weights)
  (void)kxs;
  const int arow = wn * 128 + (lane & 15), brow = wm * 64 + (lane & 15), c0 = lane >> 4;

  // LDS-DMA staging is split by K-step parity: the 4 waves of group (s & 1) issue all 64 pieces
  // (8 rows x 128 B each, 16 per wave) of K-step s, the other group none.  A piece costs its wave
  // ~60-180 issue cycles; with both halves loading in lockstep the two waves of every SIMD stalled
  // together, now one wave per SIMD loads while its partner keeps the matrix pipe busy.
  // Piece p's lane offset depends on p only through p * 8 rows (uniform, in soffset) and the
  // swizzle parity p & 1, so a lane keeps 2 offsets per operand.
  const int grp = wave >> 2, w4 = wave & 3;
  (void)w4;
  // PERMW: piece i of a wave fills LDS rows 8i + (lane >> 3) of its 64-row band, i.e. row
  // k = 8 (i & 3) + l3 (l3 = lane >> 3) of the band's 32-row block i >> 2, which takes W row
  // perm32(k) = [16 (l3 >> 2) + (l3 & 3)] + 8 (i & 1) + 4 ((i >> 1) & 1): the lane part stays in
  // the 2 offsets per operand, the piece part joins the uniform soffset (perm_row_off)
  uint32_t vbw[2], vbx[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int ch = (lane & 7) ^ ((lane >> 4) + 4 * par);
    const int l3 = lane >> 3;
    const int wr = PERMW ? 16 * (l3 >> 2) + (l3 & 3) : l3;
    vbw[par] = (uint32_t)(((int64_t)wr * K + ch * 8) * 2);
    vbx[par] = (uint32_t)(((int64_t)l3 * lda + ch * 8) * 2);
  }
  // tile panels: W rows [nn, nn+256) and X rows [mm, min(M, mm+256)) (a lambda may not carry the
  // buffer-resource type through its signature: hipcc then drops the host stubs of this template)
  auto stage = [&](int kt, half_t* s, int mm, int nn) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto rw = panel_rsrc(W + (int64_t)nn * K, (int64_t)(N - nn < BN ? N - nn : BN) * K * 2);
    const auto rx = panel_rsrc(X + (int64_t)mm * lda, (int64_t)(M - mm < BM ? M - mm : BM) * lda * 2);
    // row-group offsets advanced in place (an opaque running value: precomputed per piece and
    // hoisted, the 32 soffsets would exhaust the SGPRs)
    const int kx = kt >= kxs ? kt - kxs : kt;   // split weights: X's K-steps repeat
    int sw = w4 * 8 * 16 * K + kt * GBK * 2, sx = w4 * 8 * 16 * (int)lda + kx * GBK * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      asm volatile("" : "+s"(sw));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, SR_LDS(s + (w4 * 8 + i) * 8 * GBK), 16,
                                               vbw[i & 1], sw, 0, 0);
      // next piece's row offset (bytes = rows x 2K): PERMW rows 0 8 4 12 32 40 36 44
      if (i < 7)
        sw += (P64 ? perm64_row_off(i + 1) - perm64_row_off(i) : PERMW ? perm_row_off(i + 1) - perm_row_off(i) : 8) * 2 * K;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      asm volatile("" : "+s"(sx));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, SR_LDS(s + BN * GBK + (w4 * 8 + i) * 8 * GBK), 16,
                                               vbx[i & 1], sx, 0, 0);
      sx += 16 * (int)lda;
    }
#endif
  };

  // CSTL: group 1's 4 waves stage the tile's epilogue constants, one 1 KiB piece each: bias and
  // column sums of columns [nn, nn + 256), (mu, rstd) of rows [mm, mm + 256) (two pieces; rows past
  // M read as zero and are never stored).  Issued at the top of every tile (the previous tile's
  // epilogue, the last reader, ended before the transition barrier), younger than group 1's
  // K-step 1 pieces and epilogue stores: K-step 0's lenient wait counts the wave's piece too, the end
  // of K-step 1 (vmcnt(0)) awaits them, the epilogue reads them 10+ K-steps later (persistent FFN1
  // launches keep nk >= 4, host-checked).  (Issued from inside the K-step loop under a runtime kt
  // test, the staging code spilled 12-96 B at 256 VGPRs.)
  auto stage_cst = [&](int mm, int nn) __attribute__((always_inline)) {
#if defined(__HIP_DEVICE_COMPILE__)
    // (the lane offset re-derived here: a hoisted one stayed live through the K-loop and spilled)
    const uint32_t lo = (uint32_t)lane_id_here() * 16u;
    if (w4 >= NCST) {
    } else if (w4 < 2) {  // bias; column sums (FFN1) or the residual's LayerNorm weight (RHALF)
      const float* src = w4 == 0 ? bias : CSTL ? lf.colsum : lf.gamma;
      const auto r = panel_rsrc(reinterpret_cast<const half_t*>(src + nn), 1024);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, SR_LDS(cst + 256 * w4), 16, lo, 0, 0, 0);
    } else {
      const int r0 = mm + 128 * (w4 - 2);
      // (wave-uniform, kept scalar: a VALU clamp put the descriptor in VGPRs, spilled at 256 VGPRs
      // and its reload's vmcnt(0) waited for the epilogue's stores at every tile's top)
      const int nrow = __builtin_amdgcn_readfirstlane(max(0, min(128, M - r0)));
      const auto r = panel_rsrc(reinterpret_cast<const half_t*>(lf.mr + (int64_t)r0 * 2), (int64_t)nrow * 8);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(r, SR_LDS(cst + 512 + 256 * (w4 - 2)), 16, lo, 0, 0, 0);
    }
#endif
  };

  float4v acc[8][4];
  half8 aX[4], aY[4], bX[4], bY[4];
  int8v f0[2], f1[2], fb[4];  // fp8 path: A row pairs (ping-pong) and B
  int sa[8];                  // fp8 weights: E8M0 exponent of each A (W) fragment row
#pragma unroll
  for (int i = 0; i < 8; ++i) sa[i] = 119;  // the scan: 2^-8 on both operands

  if (PERSIST && lf.stagger != 0) {  // de-phase the walkers of an XCD (> 0) or the XCDs (< 0)
    const int n_sleep = lf.stagger > 0 ? ((blockIdx.x >> 3) & 7) * lf.stagger : (blockIdx.x & 7) * -lf.stagger;
    for (int i = 0; i < n_sleep; ++i) __builtin_amdgcn_s_sleep(8);
  }
  float* const tau_lds = reinterpret_cast<float*>(lds + 2 * STAGE);
  if constexpr (SCAN) {  // tau table (bias = tau, M = B <= 256, host-checked); the prologue's
                         // barrier publishes it
    for (int q = tid; q < 256; q += blockDim.x) tau_lds[q] = q < M ? bias[q] : INFINITY;
  }
  if constexpr (GLUT) {  // published by the prologue's barrier
    if constexpr (EPI == EPI_LNF_GELU_F8)
      gelu_t8_tab_init(reinterpret_cast<float*>(gtab), tid, blockDim.x);
    else
      gelu_t_tab_init(gtab, tid, blockDim.x);
  }
  // prologue of the first tile: group 0 stages K-step 0 (and waits for it), group 1 K-step 1
  if (grp == 0) {
    stage(0, lds, m0, n0);
    SR_WAITCNT(0, 15);
  } else if (nk > 1) {
    stage(1, lds + STAGE, m0, n0);
  }
  __builtin_amdgcn_s_barrier();
  bool stores_pending = false;  // 32 unchecked epilogue stores of the previous tile in flight
  // STAMP: last stamp and the phase sums, 32-bit (wave-uniform: readfirstlane keeps them in SGPRs)
  uint32_t st_t0 = 0, st_sum[6] = {0, 0, 0, 0, 0, 0};
  if constexpr (STAMP) st_t0 = (uint32_t)__builtin_amdgcn_s_memtime();
  auto stamp = [&](int phase) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const uint32_t t1 = (uint32_t)__builtin_amdgcn_s_memtime();
      st_sum[phase] = __builtin_amdgcn_readfirstlane(st_sum[phase] + (t1 - st_t0));
      st_t0 = t1;
    }
  };

  // One K-step.  SN: 0 none, 1 stage kt+2 of this tile, 2 stage K-steps 0/1 of tile (mn, nn).
  // RN: read kt+1's p0 fragments.  The barrier waits vmcnt(0), or vmcnt(32) when `lenient` (the
  // only younger VMEM ops are the previous tile's epilogue stores).
  // (a plain lambda with constant arguments, force-inlined: a generic lambda inside this kernel
  // template made hipcc drop the host stubs of the other instantiations)
  auto kstep = [&](int kt, const int SN, const bool RN, bool lenient, int mn, int nn,
                   bool more_) __attribute__((always_inline)) {
    half_t* cur = lds + (kt & 1) * STAGE;
    const half_t* nxt = lds + ((kt + 1) & 1) * STAGE;
    const half_t* Bc = cur + BN * GBK;
    // p0: A[0..3] x B (k 0..31); reads A[4..7] (k 0..31)
#pragma unroll
    for (int i = 0; i < 4; ++i) aX[i] = read_frag(cur, arow + 16 * (4 + i), c0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aY[i], bX[j], acc[i][j], 0, 0, 0);
    SR_INTERLEAVE(4);
    // p1: A[4..7] x B (k 0..31); reads A[0..3], B (k 32..63)
#pragma unroll
    for (int i = 0; i < 4; ++i) aY[i] = read_frag(cur, arow + 16 * i, c0 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) bY[j] = read_frag(Bc, brow + 16 * j, c0 + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aX[i], bX[j], acc[4 + i][j], 0, 0, 0);
    SR_INTERLEAVE(8);
    // p2: A[0..3] x B' (k 32..63); reads A[4..7] (k 32..63)
#pragma unroll
    for (int i = 0; i < 4; ++i) aX[i] = read_frag(cur, arow + 16 * (4 + i), c0 + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aY[i], bY[j], acc[i][j], 0, 0, 0);
    SR_INTERLEAVE(4);
    // K-step kt+1 landed (all waves) and buffer kt&1 is no longer read: restage it
    if (lenient) {
      if (NCST && grp == 1 && w4 < NCST)  // (+ the wave's one constant piece issued at the tile's top)
        SR_WAITCNT(NST + 1, 0);
      else
        SR_WAITCNT(NST, 0);
    } else
      SR_WAITCNT(0, 0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (STAMP) {
      if (kt <= 1) stamp(kt);  // phase 0: tile start -> K-step 0's barrier; 1: -> K-step 1's
      __builtin_amdgcn_sched_barrier(0);
    }
    // (group (kt & 1) stages K-step kt + 2 in one burst while the partner wave of every SIMD,
    // from the other group, runs its MFMAs)
    // (interleaving the 16 pieces one per p3 MFMA instead measured -2.3 % on the main loop and
    // -3.5 % end to end: profiles/r05_stage_ilv/)
    if (SN == 1 && DIAG != 1 && grp == (kt & 1)) stage(kt + 2, cur, m0, n0);
    if (SN == 2 && !LATE && DIAG != 11) {
      if (more_) {
        if (grp == 0)
          stage(0, lds, mn, nn);
        else
          stage(1, lds + STAGE, mn, nn);
      }
    }
    // p3: A[4..7] x B' (k 32..63); reads K-step kt+1's p0 operands
    if (RN) {
#pragma unroll
      for (int i = 0; i < 4; ++i) aY[i] = read_frag(nxt, arow + 16 * i, c0);
#pragma unroll
      for (int j = 0; j < 4; ++j) bX[j] = read_frag(nxt + BN * GBK, brow + 16 * j, c0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aX[i], bY[j], acc[4 + i][j], 0, 0, 0);
    if (RN) {
      SR_INTERLEAVE(8);
    }
    __builtin_amdgcn_sched_barrier(0);
  };

  // fp8 K-step (128 elements): four phases of 8 block-scaled MFMAs (each covers a 16 x 16 x 128
  // block, twice the f16 MFMA's time), A row pairs ping-ponging between f0 / f1: q0 A[0,1] x B
  // (reads A[2,3]), q1 A[2,3] (reads A[4,5]), q2 A[4,5] (reads A[6,7]), barrier + staging as in
  // the f16 K-step, q3 A[6,7] (reads K-step kt+1's A[0,1] and B, in two halves).
  auto kstep8 = [&](int kt, const int SN, const bool RN, bool lenient, int mn, int nn,
                    bool more_) __attribute__((always_inline)) {
    half_t* cur = lds + (kt & 1) * STAGE;
    const half_t* nxt = lds + ((kt + 1) & 1) * STAGE;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      int8v (&use)[2] = (q & 1) ? f1 : f0;
      int8v (&fill)[2] = (q & 1) ? f0 : f1;
#pragma unroll
      for (int i = 0; i < 2; ++i) fill[i] = read_frag8(cur, arow + 16 * (2 * q + 2 + i), c0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[2 * q + i][j] = mfma8(use[i], fb[j], acc[2 * q + i][j], sa[2 * q + i], F8W ? 127 : 119);
      SR_INTERLEAVE8(4);
    }
    // (the fp8 K-step waits for everything, the previous tile's epilogue stores included: a
    // lenient first K-step -- a runtime choice, or a peeled constant one -- spilled 48-112 B in
    // every fp8 kernel at 256 VGPRs)
    (void)lenient;
    SR_WAITCNT(0, 0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (SN == 1 && grp == (kt & 1)) stage(kt + 2, cur, m0, n0);
    if (SN == 2 && !LATE) {
      if (more_) {
        if (grp == 0)
          stage(0, lds, mn, nn);
        else
          stage(1, lds + STAGE, mn, nn);
      }
    }
    // q3 in two halves so B needs no second register set: A[6,7] x B[0,1], then K-step kt+1's
    // A[0,1] and B[0,1] are read into the freed registers while A[6,7] x B[2,3] runs, then its
    // B[2,3] (consumed last in the next q0)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[6 + i][j] = mfma8(f1[i], fb[j], acc[6 + i][j], sa[6 + i], F8W ? 127 : 119);
    if (RN) {
#pragma unroll
      for (int i = 0; i < 2; ++i) f0[i] = read_frag8(nxt, arow + 16 * i, c0);
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = read_frag8(nxt + BN * GBK, brow + 16 * j, c0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 2; j < 4; ++j) acc[6 + i][j] = mfma8(f1[i], fb[j], acc[6 + i][j], sa[6 + i], F8W ? 127 : 119);
    if (RN) {
#pragma unroll
      for (int j = 2; j < 4; ++j) fb[j] = read_frag8(nxt + BN * GBK, brow + 16 * j, c0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto step = [&](int kt, const int SN, const bool RN, bool lenient, int mn, int nn,
                  bool more_) __attribute__((always_inline)) {
    if constexpr (F8)
      kstep8(kt, SN, RN, lenient, mn, nn, more_);
    else
      kstep(kt, SN, RN, lenient, mn, nn, more_);
  };

  for (;;) {
    if (NCST && grp == 1) stage_cst(m0, n0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    if constexpr (F8W) {
      const uint8_t* wexp = lf.wexp;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int n = P64     ? n0 + wn * 128 + 64 * (i >> 2) + 16 * ((lane & 15) >> 2) + 4 * (i & 3) + (lane & 3)
                      : PERMW ? n0 + wn * 128 + 32 * (i >> 1) + 4 * (i & 1) + perm32(lane & 15)
                              : n0 + arow + 16 * i;
        // (from an LDS copy staged with the tile's first K-step instead: fp8 FFN1 1,572 -> 1,540
        // TF/s, spills 8 -> 20 B, profiles/r05_wexp_lds/)
        sa[i] = wexp[n < N ? n : N - 1];
      }
    }
    if constexpr (F8) {
#pragma unroll
      for (int i = 0; i < 2; ++i) f0[i] = read_frag8(lds, arow + 16 * i, c0);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag8(lds + BN * GBK, brow + 16 * j, c0);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) aY[i] = read_frag(lds, arow + 16 * i, c0);
#pragma unroll
      for (int j = 0; j < 4; ++j) bX[j] = read_frag(lds + BN * GBK, brow + 16 * j, c0);
    }

    const int t_next = t + t_step;
    const bool more = PERSIST && t_next < t_end && nk > 1;
    const int t_walk = more ? t_next : t;   // the next tile's coordinates only when it exists
    const int m0n = tile_m(t_walk) * BM, n0n = tile_n(t_walk) * BN;
    int kt = 0;
    bool lenient = stores_pending;
    for (; kt + 2 < nk; ++kt) {
      step(kt, 1, true, lenient, 0, 0, false);
      lenient = false;
    }
    if (kt + 1 < nk) {
      step(kt++, 0, true, lenient, 0, 0, false);
      lenient = false;
    }
    if constexpr (PERSIST)
      step(kt, 2, false, lenient, m0n, n0n, more);
    else
      step(kt, 0, false, lenient, 0, 0, false);

    // (EPI_SCAN issues a data-dependent number of atomics / stores: never counted as pending)
    const bool full = !SCAN && m0 + BM <= M;
    stamp(2);  // phase 2: the rest of the K-loop
    if constexpr (DIAG == 7) {  // the FFN1 epilogue with every tile's stores folded onto tile (0, 0)
      store_tile_gelu<EPI, false, PERMW, NoPre, 0, CSTL>(acc, wn * 128, wm * 64, lane, M, bias, Y, ldy, lf, gtab, gscr,
                                                        NoPre{}, cst, wn * 128, wm * 64);
    } else if constexpr (DIAG == 5 || DIAG == 6 || DIAG == 10) {  // FFN1 epilogue without its stores / its math
      static_assert(GLUT, "DIAG 5 / 6: the FFN1 epilogue");
      constexpr int DM = DIAG == 10 ? 5 : DIAG;
      if (full)
        store_tile_gelu<EPI, false, PERMW, NoPre, DM, CSTL>(acc, n0 + wn * 128, m0 + wm * 64, lane, M, bias, Y, ldy, lf,
                                                            gtab, gscr, NoPre{}, cst, wn * 128, wm * 64);
      else
        store_tile_gelu<EPI, true, PERMW, NoPre, DM, CSTL>(acc, n0 + wn * 128, m0 + wm * 64, lane, M, bias, Y, ldy, lf,
                                                           gtab, gscr, NoPre{}, cst, wn * 128, wm * 64);
    } else if constexpr (DIAG == 4) {  // stores only: acc -> fp16, wide layout, no bias / activation
      const int g = lane >> 4, odd = g & 1;
      const int nl = n0 + wn * 128 + 16 * odd + 4 * (g & 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = m0 + wm * 64 + j * 16 + (lane & 15);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          half8 h;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * p][j][r]),
                                                             __float_as_uint(acc[2 * p + 1][j][r]), false, false);
            h[r] = (half_t)__uint_as_float(sw[0]);
            h[4 + r] = (half_t)__uint_as_float(sw[1]);
          }
          if (m < M) *reinterpret_cast<half8*>(reinterpret_cast<half_t*>(Y) + (int64_t)m * ldy + nl + 32 * p) = h;
        }
      }
    } else if constexpr (DIAG == 3) {  // epilogue math (bias + GELU, wide layout), no stores
      const int g = lane >> 4, odd = g & 1;
      const int nl = n0 + wn * 128 + 16 * odd + 4 * (g & 2);
      float sacc = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float4v b0 = *reinterpret_cast<const float4v*>(bias + nl + 32 * p);
          const float4v b1 = *reinterpret_cast<const float4v*>(bias + nl + 32 * p + 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * p][j][r]),
                                                             __float_as_uint(acc[2 * p + 1][j][r]), false, false);
            sacc += (float)(half_t)gelu_erf(__uint_as_float(sw[0]) + b0[r]);
            sacc += (float)(half_t)gelu_erf(__uint_as_float(sw[1]) + b1[r]);
          }
        }
      if (sacc == 12345.678f) reinterpret_cast<float*>(Y)[tid] = sacc;
    } else if constexpr (DIAG == 2) {
      float sacc = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) sacc += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (sacc == 12345.678f) reinterpret_cast<float*>(Y)[tid] = sacc;
    } else if constexpr (SCAN) {
      float tq[4];
      scan_tau(tq, m0 + wm * 64, lane, tau_lds);
      scan_epilogue(acc, tq, n0 + wn * 128, m0 + wm * 64, lane, N, reinterpret_cast<uint64_t*>(Y),
                    (int)ldy, lf);
    } else if constexpr (LATE) {
      auto pre = [&]() __attribute__((always_inline)) {
        if (more) {
          if (grp == 0)
            stage(0, lds, m0n, n0n);
          else
            stage(1, lds + STAGE, m0n, n0n);
        }
      };
      if (full)
        PipeEpi<EPI_OUT>::template run<false, LINE, GLUT, PERMW, decltype(pre), CSTX>(
            acc, n0 + wn * 128, m0 + wm * 64, lane, M, N, bias, R, ldr, Y, ldy, lf, escr, gtab, pre, cst, wn * 128,
            wm * 64);
      else
        PipeEpi<EPI_OUT>::template run<true, LINE, GLUT, PERMW, decltype(pre), CSTX>(
            acc, n0 + wn * 128, m0 + wm * 64, lane, M, N, bias, R, ldr, Y, ldy, lf, escr, gtab, pre, cst, wn * 128,
            wm * 64);
    } else if (full) {
      PipeEpi<EPI_OUT>::template run<false, LINE, GLUT, PERMW, NoPre, CSTL>(
          acc, n0 + wn * 128, m0 + wm * 64, lane, M, N, bias, R, ldr, Y, ldy, lf, escr, gtab, NoPre{}, cst, wn * 128,
          wm * 64);
    } else {
      PipeEpi<EPI_OUT>::template run<true, LINE, GLUT, PERMW, NoPre, CSTL>(
          acc, n0 + wn * 128, m0 + wm * 64, lane, M, N, bias, R, ldr, Y, ldy, lf, escr, gtab, NoPre{}, cst, wn * 128,
          wm * 64);
    }
    stamp(3);  // phase 3: the epilogue (math, scratch, store issue)
    if (!more) break;
    // next tile: K-step 0 (group 0's 16 glds) landed; younger: the epilogue's NSTORE stores
    // (group 1: its K-step 1 glds too, awaited in K-step 0).  Unchecked tiles: wait for all.
    if (!full)
      SR_WAITCNT(0, 15);
    else if (grp == 0)  // (group 1: its K-step 1 glds too, awaited in K-step 0)
      SR_WAITCNT(NST, 15);
    else
      SR_WAITCNT(NST + 16, 15);
    __builtin_amdgcn_s_barrier();
    stamp(4);  // phase 4: the tile transition (the next tile's K-step 0 wait + barrier)
    if constexpr (STAMP) st_sum[5] = __builtin_amdgcn_readfirstlane(st_sum[5] + 1);
    stores_pending = full;
    t = t_next;
    m0 = m0n;
    n0 = n0n;
  }
  if constexpr (STAMP) {  // [transitions, K-step 0, K-step 1, rest of K-loop, epilogue, transition, 0, 0]
    if (lane == 0 && lf.y8) {
      uint64_t* o = reinterpret_cast<uint64_t*>(lf.y8) + ((int64_t)blockIdx.x * 8 + wave) * 8;
      o[0] = st_sum[5];
      for (int i = 0; i < 5; ++i) o[1 + i] = (uint64_t)st_sum[i];
      o[6] = (uint64_t)nk;
      o[7] = 0;
    }
  }
}

// PERSIST: a grid of 8 * G blocks walks the tiles; XCD group x = blockIdx & 7 owns a contiguous
// tile range (X panels stay in that XCD's L2) and the next tile's first K-step is staged by
// LDS-DMA while the current tile's epilogue runs, hiding the per-tile load latency.
// ---- "pp" variant: 4-wave workgroups, 256 (n) x 128 (m) tile, K-step 32, 3-slot LDS ring ----------
// 72 KiB of LDS and <= 256 VGPRs, so TWO workgroups share a CU: one's epilogue (bias / GELU /
// LayerNorm VALU work and the output stores) runs beside the other's MFMA main loop instead of
// idling the matrix pipe (the 256 x 256 single-workgroup kernels stall on every epilogue).
// Per wave 128 x 64 outputs as before.  K-step kt: p0 = A[0..3] x B while A[4..7] is read;
// vmcnt (step kt+1 landed; kt+2 stays in flight) + raw s_barrier; the glds of kt+3 go into the
// slot just consumed; p1 = A[4..7] x B while kt+1's A[0..3] / B are read.  Rows are 64 B: 16-byte
// chunk c of row r lives at c ^ ((r >> 2) & 2) (conflict-free ds_read_b128, simulated).
__device__ __forceinline__ int swz_pp(int r, int c) { return c ^ ((r >> 2) & 2); }

__device__ __forceinline__ half8 read_frag_pp(const half_t* t, int row, int chunk) {
  return *reinterpret_cast<const half8*>(t + row * 32 + swz_pp(row, chunk) * 8);
}

template <int NI>
__device__ __forceinline__ void pp_offsets(uint32_t (&voff)[NI], int64_t ld, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r = (wave * NI + i) * 16 + (lane >> 2);
    voff[i] = (uint32_t)(((int64_t)r * ld + swz_pp(r, lane & 3) * 8) * 2);
  }
}

template <int NI>
__device__ __forceinline__ void pp_stage(__amdgpu_buffer_rsrc_t rs, const uint32_t (&voff)[NI],
                                         int soff, half_t* lds_tile, int wave) {
#if defined(__HIP_DEVICE_COMPILE__)  // (see stage_buf)
#pragma unroll
  for (int i = 0; i < NI; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, SR_LDS(lds_tile + (wave * NI + i) * 16 * 32), 16,
                                             voff[i], soff, 0, 0);
#endif
}

template <int EPI>
__global__ __launch_bounds__(256, 2) void gemm_pp_kernel(
    const half_t* __restrict__ X, int64_t lda, const half_t* __restrict__ W,
    const float* __restrict__ bias, const void* __restrict__ R, int64_t ldr,
    void* __restrict__ Y, int64_t ldy, int M, int N, int K, const LnFold lf) {
  constexpr int BN = 256, BM = 128, KS = 32, NSLOT = 3;
  constexpr int SLOT = (BN + BM) * KS;  // halfs (24 KiB)
  __shared__ __attribute__((aligned(16))) half_t lds[NSLOT * SLOT];

  const int tiles_n = N / BN;
  const int nwg = tiles_n * ((M + BM - 1) / BM);
  const int xcd = blockIdx.x & 7, q = nwg >> 3, rem = nwg & 7;
  const int wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (blockIdx.x >> 3);
  const int m0 = (wg / tiles_n) * BM, n0 = (wg % tiles_n) * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 1, wm = wave & 1;
  const int nk = K / KS;

  const int arow = wn * 128 + (lane & 15), brow = wm * 64 + (lane & 15), ch = lane >> 4;

  uint32_t vw[4], vx[2];
  pp_offsets<4>(vw, K, wave, lane);
  pp_offsets<2>(vx, lda, wave, lane);
  const __amdgpu_buffer_rsrc_t rw = panel_rsrc(W + (int64_t)n0 * K, (int64_t)BN * K * 2);
  const __amdgpu_buffer_rsrc_t rx =
      panel_rsrc(X + (int64_t)m0 * lda, (int64_t)(M - m0 < BM ? M - m0 : BM) * lda * 2);
  auto stage = [&](int kt) {
    half_t* sl = lds + (kt % NSLOT) * SLOT;
    pp_stage<4>(rw, vw, kt * KS * 2, sl, wave);
    pp_stage<2>(rx, vx, kt * KS * 2, sl + BN * KS, wave);
  };

  float4v acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
  half8 aX[4], aY[4], bX[4], bY[4];

  stage(0);
  if (nk > 1) stage(1);
  if (nk > 2) stage(2);
  if (nk > 2)
    SR_WAITCNT(12, 15);
  else if (nk > 1)
    SR_WAITCNT(6, 15);
  else
    SR_WAITCNT(0, 15);
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int i = 0; i < 4; ++i) aY[i] = read_frag_pp(lds, arow + 16 * i, ch);
#pragma unroll
  for (int j = 0; j < 4; ++j) bX[j] = read_frag_pp(lds + BN * KS, brow + 16 * j, ch);

  // K-step with fragments (a0 = A[0..3], b) in registers; reads the next step's into (a0n, bn)
  auto kstep = [&](int kt, half8 (&a0)[4], half8 (&b)[4], half8 (&a0n)[4], half8 (&bn)[4],
                   const bool st, const bool rd) __attribute__((always_inline)) {
    const half_t* cur = lds + (kt % NSLOT) * SLOT;
    const half_t* nxt = lds + ((kt + 1) % NSLOT) * SLOT;
#pragma unroll
    for (int i = 0; i < 4; ++i) aX[i] = read_frag_pp(cur, arow + 16 * (4 + i), ch);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[i], b[j], acc[i][j], 0, 0, 0);
    SR_INTERLEAVE(4);
    if (kt + 2 < nk)
      SR_WAITCNT(6, 0);
    else
      SR_WAITCNT(0, 0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (st) stage(kt + 3);
    if (rd) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a0n[i] = read_frag_pp(nxt, arow + 16 * i, ch);
#pragma unroll
      for (int j = 0; j < 4; ++j) bn[j] = read_frag_pp(nxt + BN * KS, brow + 16 * j, ch);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aX[i], b[j], acc[4 + i][j], 0, 0, 0);
    if (st && rd) {
#pragma unroll
      for (int r = 0; r < 6; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // steady state (every step stages kt+3 and reads kt+1: no branches inside), then the tail;
  // aY is consumed by p0 before p1 re-reads it, the B set alternates bX / bY
  int kt = 0;
  for (; kt + 4 < nk; kt += 2) {
    kstep(kt, aY, bX, aY, bY, true, true);
    kstep(kt + 1, aY, bY, aY, bX, true, true);
  }
  while (kt < nk) {
    kstep(kt, aY, bX, aY, bY, kt + 3 < nk, kt + 1 < nk);
    if (++kt >= nk) break;
    kstep(kt, aY, bY, aY, bX, kt + 3 < nk, kt + 1 < nk);
    ++kt;
  }

  const int nw0 = n0 + wn * 128, mw0 = m0 + wm * 64;
  if (m0 + BM <= M)
    PipeEpi<EPI>::template run<false>(acc, nw0, mw0, lane, M, N, bias, R, ldr, Y, ldy, lf);
  else
    PipeEpi<EPI>::template run<true>(acc, nw0, mw0, lane, M, N, bias, R, ldr, Y, ldy, lf);
}

// K-chunked accumulation of the 128 x 128 kernel (GEMM_SMALL, the embedders' GEMMs): the K-steps
// form chunks of KCHUNK, each chunk's MFMA chain starts from zero and the chunk sums are added in
// chunk order into an fp32 total.  With few tiles (a short M: the query embeddings of drop-in
// requests, M = 32-1,024 rows, where one tile's serial K-loop of up to 96 K-steps was the whole
// GEMM's time) the chunks run in separate workgroups (split-K, blockIdx.y = a group of cpg
// chunks) that store their partial tiles to `part`, and gemm_chunk_reduce_kernel adds them in the
// same order before the same epilogue: the outputs are bit-identical either way, so an embedding
// never depends on the batch it was coalesced into.
constexpr int KCHUNK = 6;
constexpr int64_t kSplitMaxTiles = 128;  // split only below half a workgroup per CU slot pair

template <int EPI, int BN, int BM, int WN, int WM, bool PERSIST>
__global__ __launch_bounds__(64 * WN * WM, (WN * WM > 8) ? (WN * WM) / 4 : 2) void gemm_f16_kernel(
    const half_t* __restrict__ X, int64_t lda, const half_t* __restrict__ W,
    const float* __restrict__ bias, const void* __restrict__ R, int64_t ldr,
    void* __restrict__ Y, int64_t ldy, int M, int N, int K, int kxs, float4v* __restrict__ part,
    int cpg, int kchunk) {
  constexpr int WAVES = WN * WM;
  constexpr int FN = BN / WN / 16, FM = BM / WM / 16;  // 16x16 tiles per wave
  // (the 256 x 256 form keeps one chain: a second 128-VGPR set does not fit; host: no split)
  constexpr bool CHUNKED = FN * FM <= 16 && !PERSIST;
  constexpr int NIA = BN / 8 / WAVES, NIB = BM / 8 / WAVES;
  constexpr int STAGE = (BN + BM) * GBK;  // halfs per stage
  static_assert(NIA * WAVES * 8 == BN && NIB * WAVES * 8 == BM, "tile/wave mismatch");
  __shared__ __attribute__((aligned(16))) half_t lds[2 * STAGE];

  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_n * tiles_m;
  int t, t_end, t_step;
  {
    // blocks b and b+8 share an XCD: give each XCD a contiguous range of tiles (n fastest).
    const int xcd = blockIdx.x & 7, q = nwg >> 3, rem = nwg & 7;
    const int lo = xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
    if constexpr (PERSIST) {
      t = lo + (blockIdx.x >> 3);
      t_end = lo + q + (xcd < rem ? 1 : 0);
      t_step = gridDim.x >> 3;
    } else {
      t = lo + (blockIdx.x >> 3);
      t_end = t + 1;
      t_step = 1;
    }
  }
  int m0 = (t / tiles_n) * BM, n0 = (t % tiles_n) * BN;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (LDS-DMA base in M0)
  const int wn = wave / WM, wm = wave % WM;
  // K-steps [kb, ke) of this workgroup: all of them, or chunks [cpg y, cpg (y + 1)) (split);
  // kchunk = 0: one chunk (the callers that did not ask for chunked sums: plain accumulation)
  int kb = 0, ke = K / GBK;
  if (CHUNKED && part != nullptr) {
    kb = (int)blockIdx.y * cpg * kchunk;
    ke = min(ke, kb + cpg * kchunk);
  }
  const int kstride = CHUNKED && kchunk > 0 ? kchunk : ke;

  // stage buffer b: W tile (BN rows) at lds + b*STAGE, X tile (BM rows) right after it.
  if (t < t_end) {
    const int kx = kb >= kxs ? kb - kxs : kb;
    stage_tile<NIA>(W, K, n0, N, kb * GBK, lds, wave, lane);
    stage_tile<NIB>(X, lda, m0, M, kx * GBK, lds + BN * GBK, wave, lane);
  }
  __syncthreads();

  for (; t < t_end; t += t_step) {
  float4v acc[FN][FM], tot[CHUNKED ? FN : 1][CHUNKED ? FM : 1];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};

  // (chunks as an outer loop: the chunk-end work stays out of the K-step loop's body)
  for (int c0 = kb; c0 < ke; c0 += kstride) {
    const int c1 = min(ke, c0 + kstride);
    for (int kt = c0; kt < c1; ++kt) {
      const int cur = (kt - kb) & 1;
      const half_t* As = lds + cur * STAGE;
      const half_t* Bs = As + BN * GBK;
      if (kt + 1 < ke) {
        half_t* An = lds + (cur ^ 1) * STAGE;
        const int kx = kt + 1 >= kxs ? kt + 1 - kxs : kt + 1;   // split weights: X repeats
        stage_tile<NIA>(W, K, n0, N, (kt + 1) * GBK, An, wave, lane);
        stage_tile<NIB>(X, lda, m0, M, kx * GBK, An + BN * GBK, wave, lane);
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
    if constexpr (CHUNKED) {  // a chunk ends: into the total, or stored (split)
      if (part != nullptr) {
        const int c = c0 / kchunk;
        float4v* pt = part + ((int64_t)(c * (int)(gridDim.x) + t) * WAVES + wave) * (FN * FM * 64) + lane;
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) pt[(i * FM + j) * 64] = acc[i][j];
      } else if (c0 == kb) {  // (the first chunk is copied: kchunk = 0 stays plain accumulation)
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) tot[i][j] = acc[i][j];
      } else {
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int j = 0; j < FM; ++j) tot[i][j] += acc[i][j];
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
    }
  }
  if (CHUNKED && part != nullptr) return;  // (split: gemm_chunk_reduce_kernel runs the epilogue)

  // Next tile: its first K-step lands in buffer 0 while this tile's epilogue runs (every LDS read
  // of this tile finished before the K-loop's last barrier).
  const int tn_next = t + t_step;
  const int m0_next = (tn_next / tiles_n) * BM, n0_next = (tn_next % tiles_n) * BN;
  if (PERSIST && tn_next < t_end) {
    stage_tile<NIA>(W, K, n0_next, N, 0, lds, wave, lane);
    stage_tile<NIB>(X, lda, m0_next, M, 0, lds + BN * GBK, wave, lane);
  }

  if constexpr (CHUNKED)
    store_tile<EPI, FN, FM>(tot, n0 + wn * (BN / WN), m0 + wm * (BM / WM), lane, M, bias, R, ldr, Y,
                            ldy);
  else
    store_tile<EPI, FN, FM>(acc, n0 + wn * (BN / WN), m0 + wm * (BM / WM), lane, M, bias, R, ldr, Y,
                            ldy);
  if constexpr (PERSIST) {
    __syncthreads();  // next tile's first K-step has landed in buffer 0
    m0 = m0_next;
    n0 = n0_next;
  }
  }  // tile loop
}

// The split-K epilogue of the 128 x 128 kernel: tile blockIdx.x's chunk partials summed in chunk
// order (the unsplit kernel's total, operation for operation), then its epilogue.
template <int EPI>
__global__ __launch_bounds__(256) void gemm_chunk_reduce_kernel(
    const float4v* __restrict__ part, int nchunk, const float* __restrict__ bias,
    const void* __restrict__ R, int64_t ldr, void* __restrict__ Y, int64_t ldy, int M, int N) {
  const int t = blockIdx.x, tiles_n = N / 128;
  const int m0 = (t / tiles_n) * 128, n0 = (t % tiles_n) * 128;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float4v acc[4][4];
  const float4v* p0 = part + ((int64_t)t * 4 + wave) * (16 * 64) + lane;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = p0[(i * 4 + j) * 64];
  for (int c = 1; c < nchunk; ++c) {
    const float4v* pt = part + ((int64_t)(c * (int)gridDim.x + t) * 4 + wave) * (16 * 64) + lane;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += pt[(i * 4 + j) * 64];
  }
  store_tile<EPI, 4, 4>(acc, n0 + (wave >> 1) * 64, m0 + (wave & 1) * 64, lane, M, bias, R, ldr, Y, ldy);
}

template <int BN, int BM, int WN, int WM, bool PERSIST>
void launch_tile(int epi, dim3 grid, hipStream_t stream, const half_t* X, int64_t lda,
                 const half_t* W, const float* bias, const void* R, int64_t ldr, void* Y,
                 int64_t ldy, int M, int N, int K, int kxs, float4v* part = nullptr, int cpg = 0,
                 int kchunk = 0) {
  const dim3 block(64 * WN * WM);
#define SR_GEMM_CASE(E)                                                                        \
  case E:                                                                                      \
    hipLaunchKernelGGL((gemm_f16_kernel<E, BN, BM, WN, WM, PERSIST>), grid, block, 0, stream, \
                       X, lda, W, bias, R, ldr, Y, ldy, M, N, K, kxs, part, cpg, kchunk);      \
    if (part != nullptr)                                                                       \
      hipLaunchKernelGGL((gemm_chunk_reduce_kernel<E>), dim3(grid.x), dim3(256), 0, stream,    \
                         part, (int)ceil_div(K / GBK, KCHUNK), bias, R, ldr, Y, ldy, M, N);     \
    break;
  switch (epi) {
    SR_GEMM_CASE(EPI_BIAS_F16)
    SR_GEMM_CASE(EPI_BIAS_GELU_F16)
    SR_GEMM_CASE(EPI_BIAS_RES_F32)
    SR_GEMM_CASE(EPI_BIAS_RES_F16)
    SR_GEMM_CASE(EPI_BIAS_TANH_F32)
    default: SR_CHECK(false, "gemm: unknown epilogue");
  }
#undef SR_GEMM_CASE
}

}  // namespace

static const char* epi_name(int epi) {
  switch (epi) {
    case EPI_BIAS_F16: return "gemm_f16_bias";
    case EPI_BIAS_GELU_F16: return "gemm_f16_bias_gelu";
    case EPI_BIAS_RES_F32: return "gemm_f16_bias_residual";
    case EPI_BIAS_RES_F16: return "gemm_f16_bias_residual16";
    case EPI_LNF_F16: return "gemm_f16_lnfold";
    case EPI_LNF_GELU_F16: return "gemm_f16_lnfold_gelu";
    case EPI_RES16_STATS: return "gemm_f16_residual16_stats";
    case EPI_LNR16_STATS: return "gemm_f16_lnres16_stats";
    case EPI_LNF_GELU_F8: return "gemm_f16_lnfold_gelu_out8";
    case EPI_RES16_STATS_Y8: return "gemm_f16_residual16_stats_y8";
    case EPI_LNR16_STATS_Y8: return "gemm_f16_lnres16_stats_y8";
    default: return "gemm_f16_bias_tanh";
  }
}

// Tile override for parity tests: SR_GEMM_TILE=small|big (read per launch), or gemm_force_tile().
void launch_cosine_scan_gemm(const half_t* corpus, int64_t ldc, const uint8_t* live, int64_t r0,
                             int64_t r1, const half_t* Q, int B, const float* tau, uint64_t* cand,
                             int* cnt, int cap, hipStream_t s) {
  SR_CHECK(B > 0 && B <= 256, "cosine_scan_gemm: 1..256 queries");
  SR_CHECK(ldc % GBK == 0 && ldc >= 2 * GBK, "cosine_scan_gemm: padded dim must be a multiple of 64, >= 128");
  if (r1 <= r0) return;
  const int64_t n = r1 - r0;
  SR_CHECK(n < (1ll << 31), "cosine_scan_gemm: chunk too large");
  const double rows = (double)n;
  ProfScope prof("cosine_scan", s, 2.0 * rows * ldc * B, rows * ldc * 2.0 + (double)B * ldc * 2.0);
  LnFold lf;
  lf.stat_out = reinterpret_cast<float*>(cnt);  // (EPI_SCAN field re-use, see LnFold)
  lf.stat_ld = r0;
  const int64_t tiles = ceil_div(n, 256);
  const dim3 grid((unsigned)(8 * std::min<int64_t>(32, ceil_div(tiles, 8)))), block(512);
  auto kern = gemm_pipe_kernel<EPI_SCAN, true>;
#if SR_WITH_DIAG
  static const bool diag_noepi = diag_getenv("SR_SCAN_DIAG_NOEPI") != nullptr;  // timing only
  if (diag_noepi) kern = gemm_pipe_kernel<EPI_SCAN, true, 2>;
#endif
  hipLaunchKernelGGL(kern, grid, block, 0, s, Q, ldc,
                     corpus + r0 * ldc, tau, (const void*)(live ? live + r0 : nullptr), (int64_t)0,
                     (void*)cand, (int64_t)cap, B, (int)n, (int)ldc, lf);
  SR_LAUNCH_CHECK();
}

void launch_cosine_scan_gemm8(const uint8_t* corpus8, int64_t ld8, const uint8_t* live, int64_t r0,
                              int64_t r1, const uint8_t* Q8, int B, const float* tau, uint64_t* cand,
                              int* cnt, int cap, hipStream_t s) {
  SR_CHECK(B > 0 && B <= 256, "cosine_scan_gemm8: 1..256 queries");
  SR_CHECK(ld8 % 128 == 0 && ld8 >= 256, "cosine_scan_gemm8: row bytes must be a multiple of 128, >= 256");
  if (r1 <= r0) return;
  const int64_t n = r1 - r0;
  SR_CHECK(n < (1ll << 31), "cosine_scan_gemm8: chunk too large");
  const double rows = (double)n;
  ProfScope prof("cosine_scan8", s, 2.0 * rows * ld8 * B, rows * ld8 + (double)B * ld8);
  LnFold lf;
  lf.stat_out = reinterpret_cast<float*>(cnt);  // (EPI_SCAN field re-use, see LnFold)
  lf.stat_ld = r0;
  const int64_t tiles = ceil_div(n, 256);
  const dim3 grid((unsigned)(8 * std::min<int64_t>(32, ceil_div(tiles, 8)))), block(512);
  // operands as 2-byte units: K = ld8 / 2 (the staging moves bytes)
  auto kern = gemm_pipe_kernel<EPI_SCAN8, true>;
#if SR_WITH_DIAG
  static const bool diag_noepi = diag_getenv("SR_SCAN_DIAG_NOEPI") != nullptr;  // timing only
  if (diag_noepi) kern = gemm_pipe_kernel<EPI_SCAN8, true, 2>;
#endif
  hipLaunchKernelGGL(kern, grid, block, 0, s,
                     reinterpret_cast<const half_t*>(Q8), ld8 / 2,
                     reinterpret_cast<const half_t*>(corpus8 + r0 * ld8), tau,
                     (const void*)(live ? live + r0 : nullptr), (int64_t)0, (void*)cand, (int64_t)cap,
                     B, (int)n, (int)(ld8 / 2), lf);
  SR_LAUNCH_CHECK();
}

void launch_gemm_f8w(int epi, const uint8_t* X8, int64_t lda, const uint8_t* W8, const float* bias,
                     const void* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K,
                     hipStream_t stream, const LnFold* lf) {
  SR_CHECK(epi == EPI_LNF_F16 || epi == EPI_LNF_GELU_F8 || epi == EPI_RES16_STATS ||
               epi == EPI_LNR16_STATS || epi == EPI_RES16_STATS_Y8 || epi == EPI_LNR16_STATS_Y8,
           "gemm_f8w: unsupported epilogue");
  const bool y8 = epi == EPI_RES16_STATS_Y8 || epi == EPI_LNR16_STATS_Y8;
  const bool lnr = epi == EPI_LNR16_STATS || epi == EPI_LNR16_STATS_Y8;
  const bool stats = lnr || epi == EPI_RES16_STATS || epi == EPI_RES16_STATS_Y8;
  SR_CHECK(K % 128 == 0 && K >= 256, "gemm_f8w: K must be a multiple of 128, >= 256");
  SR_CHECK(N % 256 == 0, "gemm_f8w: N must be a multiple of 256");
  SR_CHECK(lda % 16 == 0 && ldy % 8 == 0 && ldr % 8 == 0, "gemm_f8w: 16-byte rows");
  SR_CHECK(lf && lf->wexp, "gemm_f8w: the weight rows' exponents (LnFold.wexp)");
  SR_CHECK((stats && !lnr) || lf->mr, "gemm_f8w: LN-folded operand needs its row statistics");
  SR_CHECK(stats || lf->colsum, "gemm_f8w: LNF needs colsum");
  SR_CHECK(epi != EPI_LNF_GELU_F8 || lf->stat_ld == 1, "gemm_f8w: FFN1 reads consecutive row statistics");
  SR_CHECK(!lnr || lf->gamma, "gemm_f8w: LNR needs the LayerNorm weight");
  SR_CHECK(!stats || lf->stat_out, "gemm_f8w: stat_out");
  SR_CHECK(!y8 || lf->y8, "gemm_f8w: the e4m3-copy epilogues need LnFold.y8");
  if (M <= 0) return;
  const char* name = epi == EPI_LNF_F16 ? "gemm_f8_lnfold" : epi == EPI_LNF_GELU_F8 ? "gemm_f8_lnfold_gelu_out8"
                     : !stats ? "gemm_f8" : !lnr ? (y8 ? "gemm_f8_residual16_stats_y8" : "gemm_f8_residual16_stats")
                     : (y8 ? "gemm_f8_lnres16_stats_y8" : "gemm_f8_lnres16_stats");
  const double out_b = epi == EPI_LNF_GELU_F8 ? 1.0 : 2.0, res_b = stats ? 2.0 : 0.0;
  ProfScope prof(name, stream, 2.0 * M * (double)N * K,
                 (double)M * K + (double)N * K + (out_b + res_b + (y8 ? 1.0 : 0.0)) * (double)M * N);
  const LnFold lfv = *lf;
  const int64_t tiles = (int64_t)(N / 256) * ceil_div(M, 256);
  // (the FFN1 epilogue's constants are staged during K-step 1 of a persistent tile: nk >= 4)
  const bool persist = tiles >= 512 && (epi != EPI_LNF_GELU_F8 || K / 2 >= 4 * 64);
  const dim3 grid(persist ? (unsigned)(8 * std::min<int64_t>(32, ceil_div(tiles, 8))) : (unsigned)tiles);
  // operands as 2-byte units: K / 2, lda / 2 (the staging moves bytes)
  const half_t* x = reinterpret_cast<const half_t*>(X8);
  const half_t* w = reinterpret_cast<const half_t*>(W8);
#define SR_F8_CASE(E)                                                                            \
  case E:                                                                                        \
    if (persist)                                                                                 \
      hipLaunchKernelGGL((gemm_pipe_kernel<E, true, 0, true>), grid, dim3(512), 0, stream, x,     \
                         lda / 2, w, bias, R, ldr, Y, ldy, M, N, K / 2, lfv);                    \
    else                                                                                         \
      hipLaunchKernelGGL((gemm_pipe_kernel<E, false, 0, true>), grid, dim3(512), 0, stream, x,    \
                         lda / 2, w, bias, R, ldr, Y, ldy, M, N, K / 2, lfv);                    \
    break;
  switch (epi) {
    SR_F8_CASE(EPI_LNF_F16)
    SR_F8_CASE(EPI_LNF_GELU_F8)
    SR_F8_CASE(EPI_RES16_STATS)
    SR_F8_CASE(EPI_LNR16_STATS)
    SR_F8_CASE(EPI_RES16_STATS_Y8)
    SR_F8_CASE(EPI_LNR16_STATS_Y8)
    default: break;
  }
#undef SR_F8_CASE
  SR_LAUNCH_CHECK();
}

#if SR_WITH_DIAG
void launch_ffn1_diag(int diag, bool f8, const void* X, int64_t lda, const void* W, const uint8_t* wexp,
                      const float* bias, const float* colsum, const float* mr, void* Y, int64_t ldy,
                      int M, int N, int K, hipStream_t stream, uint64_t* stamps) {
  SR_CHECK(diag == 0 || diag == 2 || (diag >= 5 && diag <= 7) || (diag >= 9 && diag <= 11),
           "ffn1_diag: diag must be 0, 2, 5, 6, 7, 9, 10 or 11");
  SR_CHECK(N % 256 == 0 && M > 0, "ffn1_diag: N % 256 == 0, M > 0");
  // diag 7 stores every tile unchecked onto rows 0..255 of Y
  SR_CHECK(diag != 7 || (M >= 256 && ldy >= N), "ffn1_diag: diag 7 needs M >= 256, ldy >= N");
  SR_CHECK(diag < 9 || (stamps && !f8), "ffn1_diag: diag 9 / 10 / 11 need a stamp buffer (fp16)");
  LnFold lf;
  lf.mr = mr;
  lf.colsum = colsum;
  lf.wexp = wexp;
  lf.y8 = reinterpret_cast<uint8_t*>(stamps);  // (STAMP diagnostics only; FFN1 has no e4m3 copy)
  if (diag == 0) {
    if (f8)
      launch_gemm_f8w(EPI_LNF_GELU_F8, reinterpret_cast<const uint8_t*>(X), lda,
                      reinterpret_cast<const uint8_t*>(W), bias, nullptr, 0, Y, ldy, M, N, K, stream, &lf);
    else
      launch_gemm(EPI_LNF_GELU_F16, reinterpret_cast<const half_t*>(X), lda,
                  reinterpret_cast<const half_t*>(W), bias, nullptr, 0, Y, ldy, M, N, K, stream, &lf);
    return;
  }
  SR_CHECK(!f8 || (wexp && K % 128 == 0), "ffn1_diag: fp8 needs wexp, K % 128 == 0");
  SR_CHECK((f8 ? K / 2 : K) >= 4 * 64, "ffn1_diag: the persistent FFN1 needs >= 4 K-steps");
  const int64_t tiles = (int64_t)(N / 256) * ceil_div(M, 256);
  // SR_FFN1_DIAG_WALKERS = walkers per XCD (1..32; default 32 = every CU): with fewer CUs storing
  // at once, a store cost that is the chip's write bandwidth shrinks, a per-CU one does not
  static const int walkers = [] {
    const char* e = diag_getenv("SR_FFN1_DIAG_WALKERS");
    const int w = e ? std::atoi(e) : 32;
    return w < 1 ? 1 : (w > 32 ? 32 : w);
  }();
  const dim3 grid((unsigned)(8 * std::min<int64_t>(walkers, ceil_div(tiles, 8)))), block(512);
  lf.group_m = K <= 1024 ? (N >= 2048 ? 8 : 4) : 0;  // the product walk
  {  // the product's walker de-phasing (SR_GEMM_STAGGER, launch_gemm)
    const char* e = diag_getenv("SR_GEMM_STAGGER");
    const int st = e ? std::atoi(e) : 0;
    lf.stagger = st > 0 ? std::max(1, st * K / 768) : st < 0 ? std::min(-1, st * K / 768) : 0;
  }
  ProfScope prof(f8 ? "ffn1_diag_f8" : "ffn1_diag", stream, 2.0 * M * (double)N * K, 0.0);
  const half_t* x = reinterpret_cast<const half_t*>(X);
  const half_t* w = reinterpret_cast<const half_t*>(W);
  const int64_t la = f8 ? lda / 2 : lda;
  const int kk = f8 ? K / 2 : K;
#define SR_FD(D)                                                                                  \
  if (f8)                                                                                         \
    hipLaunchKernelGGL((gemm_pipe_kernel<EPI_LNF_GELU_F8, true, D, true>), grid, block, 0, stream, \
                       x, la, w, bias, nullptr, 0, Y, ldy, M, N, kk, lf);                        \
  else                                                                                            \
    hipLaunchKernelGGL((gemm_pipe_kernel<EPI_LNF_GELU_F16, true, D>), grid, block, 0, stream, x,  \
                       la, w, bias, nullptr, 0, Y, ldy, M, N, kk, lf);
  if (diag == 2) {
    SR_FD(2)
  } else {
    if (diag == 5) {
      SR_FD(5)
    } else if (diag == 6) {
      SR_FD(6)
    } else if (diag == 9) {
      SR_FD(9)
    } else if (diag == 10) {
      SR_FD(10)
    } else if (diag == 11) {
      SR_FD(11)
    } else {
      SR_FD(7)
    }
  }
#undef SR_FD
  SR_LAUNCH_CHECK();
}

// Stamped product launch of the residual + statistics GEMM (EPI_LNR16_STATS: FFN2 / O-projection,
// the persistent kernel with its half-tile epilogue) -- sr_diag_gemm_lnr_stats_stamps: per-wave
// s_memtime phase sums into stamps (the FFN1 stamps' layout, tools/lnr_stamps.py)
void launch_lnr_stats_stamps(const half_t* X, int64_t lda, const half_t* W, const float* bias, const void* R,
                             int64_t ldr, const float* mr, const float* gamma, void* Y, int64_t ldy, int M,
                             int N, int K, float* stat_out, uint64_t* stamps, hipStream_t stream) {
  SR_CHECK(N % 256 == 0 && M > 0 && K % GBK == 0 && K >= 2 * GBK, "lnr_stamps: N % 256, K % 64, K >= 128");
  SR_CHECK(ldy % 8 == 0 && ldr % 8 == 0 && lda % 8 == 0, "lnr_stamps: 16-byte rows");
  LnFold lf;
  lf.mr = mr;
  lf.gamma = gamma;
  lf.stat_out = stat_out;
  lf.y8 = reinterpret_cast<uint8_t*>(stamps);  // (the non-Y8 epilogue has no e4m3 copy)
  lf.group_m = K <= 1024 ? (N >= 2048 ? 8 : 4) : 0;  // the product walk
  const int64_t tiles = (int64_t)(N / 256) * ceil_div(M, 256);
  const dim3 grid((unsigned)(8 * std::min<int64_t>(32, ceil_div(tiles, 8)))), block(512);
  hipLaunchKernelGGL((gemm_pipe_kernel<EPI_LNR16_STATS, true, 9>), grid, block, 0, stream, X, lda, W, bias, R, ldr,
                     Y, ldy, M, N, K, lf);
  SR_LAUNCH_CHECK();
}
#endif  // SR_WITH_DIAG

__device__ __forceinline__ float e4m3_decode(uint32_t b) {
  const uint32_t e = (b >> 3) & 15u, m = b & 7u;
  const float v = e ? ldexpf(1.f + (float)m * 0.125f, (int)e - 7) : ldexpf((float)m, -9);
  return (b & 0x80u) ? -v : v;
}

__global__ void colsum_fp8_kernel(const uint8_t* __restrict__ W8, const uint8_t* __restrict__ wexp,
                                  int N, int K, float* __restrict__ colsum) {
  const int n = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  float acc = 0.f;
  for (int k = lane; k < K; k += 64) acc += e4m3_decode(W8[(int64_t)n * K + k]);
  acc = wave_sum(acc);
  if (lane == 0) colsum[n] = ldexpf(acc, (int)wexp[n] - 127);
}

void launch_colsum_fp8(const uint8_t* W8, const uint8_t* wexp, int N, int K, float* colsum,
                       hipStream_t s) {
  if (N <= 0) return;
  hipLaunchKernelGGL(colsum_fp8_kernel, dim3((unsigned)ceil_div(N, 4)), dim3(256), 0, s, W8, wexp,
                     N, K, colsum);
  SR_LAUNCH_CHECK();
}

__global__ void quantize_rows_fp8_exp_kernel(const half_t* __restrict__ W, int N, int K,
                                             uint8_t* __restrict__ W8, uint8_t* __restrict__ wexp) {
  const int n = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (n >= N) return;
  const half_t* w = W + (int64_t)n * K;
  float amax = 0.f;
  for (int k = lane; k < K; k += 64) amax = fmaxf(amax, fabsf((float)w[k]));
  amax = wave_max(amax);
  int e = 0;
  if (amax > 0.f) {
    int ex;
    (void)frexpf(448.f / amax, &ex);
    e = ex - 1;
    while (ldexpf(amax, e + 1) <= 448.f) ++e;
    while (ldexpf(amax, e) > 448.f) --e;
  }
  e = e > 127 ? 127 : (e < -127 ? -127 : e);
  for (int k = lane; k < K; k += 64) W8[(int64_t)n * K + k] = (uint8_t)e4m3_rne(ldexpf((float)w[k], e));
  if (lane == 0) wexp[n] = (uint8_t)(127 - e);
}

void launch_quantize_rows_fp8(const half_t* W, int N, int K, uint8_t* W8, uint8_t* wexp,
                              hipStream_t s) {
  if (N <= 0) return;
  hipLaunchKernelGGL(quantize_rows_fp8_exp_kernel, dim3((unsigned)ceil_div(N, 4)), dim3(256), 0, s,
                     W, N, K, W8, wexp);
  SR_LAUNCH_CHECK();
}

static int g_force_tile = -1;
void gemm_force_tile(int t) { g_force_tile = t; }
static int forced_tile() {
  if (g_force_tile >= 0) return g_force_tile;
  const char* e = std::getenv("SR_GEMM_TILE");
  if (!e) return -1;
  if (std::strcmp(e, "small") == 0) return GEMM_SMALL;
  if (std::strcmp(e, "big") == 0) return GEMM_BIG;
  if (std::strcmp(e, "pipe") == 0) return GEMM_PIPE;
  if (std::strcmp(e, "pipe_persist") == 0) return GEMM_PIPE_PERSIST;
  if (std::strcmp(e, "pp") == 0) return GEMM_PP;
  return -1;
}

void launch_gemm(int epi, const half_t* X, int64_t lda, const half_t* W, const float* bias,
                 const void* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K,
                 hipStream_t stream, const LnFold* lf) {
  launch_gemm_variant(-1, epi, X, lda, W, bias, R, ldr, Y, ldy, M, N, K, stream, lf);
}

void launch_gemm_variant(int variant, int epi, const half_t* X, int64_t lda, const half_t* W,
                         const float* bias, const void* R, int64_t ldr, void* Y, int64_t ldy,
                         int M, int N, int K, hipStream_t stream, const LnFold* lf) {
  SR_CHECK(K % GBK == 0, "gemm: K must be a multiple of 64");
  SR_CHECK(N % 128 == 0, "gemm: N must be a multiple of 128");
  SR_CHECK(lda % 8 == 0 && ldy % 4 == 0, "gemm: leading dimensions must keep 16-byte rows");
  const bool fold = epi >= EPI_LNF_F16;
  SR_CHECK((epi >= 0 && epi <= EPI_LNR16_STATS) || epi == EPI_LNF_GELU_F8 ||
               epi == EPI_RES16_STATS_Y8 || epi == EPI_LNR16_STATS_Y8, "gemm: unknown epilogue");
  SR_CHECK(!(epi == EPI_RES16_STATS_Y8 || epi == EPI_LNR16_STATS_Y8) || (lf && lf->y8),
           "gemm: the e4m3-copy epilogues need LnFold.y8");
  SR_CHECK(!fold || (lf && N % 256 == 0), "gemm: LayerNorm-folded epilogues need LnFold, N % 256");
  SR_CHECK(!(epi == EPI_LNF_F16 || epi == EPI_LNF_GELU_F16 || epi == EPI_LNF_GELU_F8 ||
             epi == EPI_LNR16_STATS || epi == EPI_LNR16_STATS_Y8) || lf->mr,
           "gemm: LN-folded operand needs its row statistics");
  SR_CHECK(!(epi == EPI_LNF_F16 || epi == EPI_LNF_GELU_F16 || epi == EPI_LNF_GELU_F8) || lf->colsum,
           "gemm: LNF needs colsum");
  SR_CHECK(!(epi == EPI_LNF_GELU_F16 || epi == EPI_LNF_GELU_F8) || lf->stat_ld == 1,
           "gemm: the FFN1 epilogues read consecutive row statistics (stat_ld 1)");
  SR_CHECK(!(epi == EPI_LNR16_STATS || epi == EPI_LNR16_STATS_Y8) || lf->gamma,
           "gemm: LNR needs the LayerNorm weight");
  SR_CHECK(!(epi == EPI_RES16_STATS || epi == EPI_LNR16_STATS || epi == EPI_RES16_STATS_Y8 ||
             epi == EPI_LNR16_STATS_Y8) || lf->stat_out,
           "gemm: *_STATS epilogue needs stat_out");
  const int x_k = lf && lf->x_k > 0 ? lf->x_k : K;
  SR_CHECK(x_k == K || (K == 2 * x_k && x_k % GBK == 0 && epi < EPI_LNF_GELU_F8),
           "gemm: split weights need K == 2 x_k (x_k % 64 == 0, fp16 operands)");
  if (M <= 0) return;
  const bool out32 = epi == EPI_BIAS_RES_F32 || epi == EPI_BIAS_TANH_F32;
  const double out_b = out32 ? 4.0 : epi == EPI_LNF_GELU_F8 ? 1.0 : 2.0;
  const double res_b = epi == EPI_BIAS_RES_F32 ? 4.0
                       : (epi == EPI_BIAS_RES_F16 || epi == EPI_RES16_STATS || epi == EPI_LNR16_STATS ||
                          epi == EPI_RES16_STATS_Y8 || epi == EPI_LNR16_STATS_Y8) ? 2.0
                                                                                                     : 0.0;
  const double bytes = 2.0 * ((double)M * x_k + (double)N * K) + (out_b + res_b) * (double)M * N;
  ProfScope prof(epi_name(epi), stream, 2.0 * M * (double)N * K, bytes);
  const int64_t big_tiles = (N % 256 == 0) ? (int64_t)(N / 256) * ceil_div(M, 256) : 0;
  SR_CHECK(big_tiles < (1ll << 31), "gemm: too many tiles");
  int v = variant >= 0 ? variant : forced_tile();
  if (v < 0) v = big_tiles >= 512 ? GEMM_PIPE_PERSIST : GEMM_SMALL;
  if (v != GEMM_SMALL && N % 256 != 0) v = GEMM_SMALL;
  if (v == GEMM_PP && (K % 32 != 0 || epi >= EPI_LNF_GELU_F8 || x_k != K)) v = GEMM_PIPE;
  if (x_k != K && v >= GEMM_DIAG_NOLOAD && v != GEMM_PP) v = GEMM_PIPE;  // diagnostics: plain K
  SR_CHECK(SR_WITH_DIAG || !(v == GEMM_DIAG_NOLOAD || v == GEMM_DIAG_NOEPI ||
                             (v >= GEMM_DIAG_P_NOEPI && v <= GEMM_DIAG_P_STOREONLY)),
           "gemm: timing-only variants are in the diagnostic library (libsrmi_diag.so)");
  if (fold && (v == GEMM_SMALL || v == GEMM_BIG)) v = big_tiles >= 512 ? GEMM_PIPE_PERSIST : GEMM_PIPE;
  const bool wide = (v == GEMM_PIPE || v == GEMM_PIPE_PERSIST || v == GEMM_PP) && !out32;
  SR_CHECK(!wide || (ldy % 8 == 0 && ldr % 8 == 0), "gemm: fp16 outputs need ldy, ldr % 8 == 0");
  SR_CHECK(epi < EPI_LNF_GELU_F8 || v == GEMM_PIPE || v == GEMM_PIPE_PERSIST,
           "gemm: the e4m3-output epilogues run on the pipelined kernels");
  LnFold lfv = lf ? *lf : LnFold{};
  // Short-K GEMMs (K <= 1024: QKV, FFN1, O-proj) walk groups of 8 (N >= 2048) or 4 m-panels;
  // FFN2 (K = 3072) stays n fastest.  Same-box A/B of the full bench: 422.8 / 424.0 -> 429.8 /
  // 431.0 q/s (profiles/r01_gemm_group_m.log).  SR_GEMM_GROUP_M overrides (diagnostic).
  // (diagnostic) SR_GEMM_GROUP_M = "G" for every shape, or "N:G,N:G,..." per output width N
  static const std::vector<std::pair<int, int>> group_m_env = [] {
    std::vector<std::pair<int, int>> v;
    const char* e = diag_getenv("SR_GEMM_GROUP_M");
    if (!e) return v;
    std::string str(e);
    if (str.find(':') == std::string::npos) {
      v.emplace_back(-1, std::atoi(e));
      return v;
    }
    size_t pos = 0;
    while (pos < str.size()) {
      const size_t end = std::min(str.find(',', pos), str.size());
      const std::string item = str.substr(pos, end - pos);
      const size_t c = item.find(':');
      if (c != std::string::npos) v.emplace_back(std::atoi(item.c_str()), std::atoi(item.c_str() + c + 1));
      pos = end + 1;
    }
    return v;
  }();
  lfv.group_m = K <= 1024 ? (N >= 2048 ? 8 : 4) : 0;
  for (const auto& [n_env, g_env] : group_m_env)
    if (n_env < 0 || n_env == N) lfv.group_m = g_env;
  lfv.x_k = x_k == K ? 0 : x_k;
  // de-phasing of the persistent walkers: phase step ~1/16 of a tile (K / 96 x 512 cycles);
  // SR_GEMM_STAGGER = units of 512 cycles per phase (0 = off): > 0 de-phases the walkers inside
  // each XCD (their L2 working set spreads), < 0 the 8 XCDs against each other (diagnostic)
  static const int stagger_env = [] {
    const char* e = diag_getenv("SR_GEMM_STAGGER");
    return e ? std::atoi(e) : 0;
  }();
  lfv.stagger = stagger_env > 0 ? std::max(1, stagger_env * K / 768)
                : stagger_env < 0 ? std::min(-1, stagger_env * K / 768) : 0;
  if (v == GEMM_BIG) {
    launch_tile<256, 256, 2, 4, false>(epi, dim3((unsigned)big_tiles), stream, X, lda, W, bias, R,
                                       ldr, Y, ldy, M, N, K, x_k / GBK);
#if SR_WITH_DIAG
  } else if (v >= GEMM_DIAG_P_NOEPI && v <= GEMM_DIAG_P_STOREONLY) {
    const int64_t g = 8 * std::min<int64_t>(32, ceil_div(big_tiles, 8));
    const dim3 grid((unsigned)g), block(512);
    if (v == GEMM_DIAG_P_NOEPI)
      hipLaunchKernelGGL((gemm_pipe_kernel<EPI_BIAS_F16, true, 2>), grid, block, 0, stream, X, lda,
                         W, bias, R, ldr, Y, ldy, M, N, K, lfv);
    else if (v == GEMM_DIAG_P_MATHONLY)
      hipLaunchKernelGGL((gemm_pipe_kernel<EPI_BIAS_F16, true, 3>), grid, block, 0, stream, X, lda,
                         W, bias, R, ldr, Y, ldy, M, N, K, lfv);
    else
      hipLaunchKernelGGL((gemm_pipe_kernel<EPI_BIAS_F16, true, 4>), grid, block, 0, stream, X, lda,
                         W, bias, R, ldr, Y, ldy, M, N, K, lfv);
  } else if (v == GEMM_DIAG_NOLOAD || v == GEMM_DIAG_NOEPI) {
    const dim3 grid((unsigned)big_tiles), block(512);
    if (v == GEMM_DIAG_NOLOAD)
      hipLaunchKernelGGL((gemm_pipe_kernel<EPI_BIAS_F16, false, 1>), grid, block, 0, stream, X, lda,
                         W, bias, R, ldr, Y, ldy, M, N, K, lfv);
    else
      hipLaunchKernelGGL((gemm_pipe_kernel<EPI_BIAS_F16, false, 2>), grid, block, 0, stream, X, lda,
                         W, bias, R, ldr, Y, ldy, M, N, K, lfv);
#endif
  } else if (v == GEMM_PP) {
    const int64_t tiles = (int64_t)(N / 256) * ceil_div(M, 128);
    const dim3 grid((unsigned)tiles), block(256);
#define SR_PP_CASE(E)                                                                            \
  case E:                                                                                        \
    hipLaunchKernelGGL((gemm_pp_kernel<E>), grid, block, 0, stream, X, lda, W, bias, R, ldr, Y,  \
                       ldy, M, N, K, lfv);                                                       \
    break;
    switch (epi) {
      SR_PP_CASE(EPI_BIAS_F16)
      SR_PP_CASE(EPI_BIAS_GELU_F16)
      SR_PP_CASE(EPI_BIAS_RES_F32)
      SR_PP_CASE(EPI_BIAS_RES_F16)
      SR_PP_CASE(EPI_BIAS_TANH_F32)
      SR_PP_CASE(EPI_LNF_F16)
      SR_PP_CASE(EPI_LNF_GELU_F16)
      SR_PP_CASE(EPI_RES16_STATS)
      SR_PP_CASE(EPI_LNR16_STATS)
      default: SR_CHECK(false, "gemm: unknown epilogue");
    }
#undef SR_PP_CASE
  } else if (v == GEMM_PIPE || v == GEMM_PIPE_PERSIST) {
    // (the FFN1 epilogues stage their constants during K-step 1 of a persistent tile: nk >= 4)
    // (the persistent LNR epilogues stage consecutive row statistics: stat_ld 1)
    const bool persist = v == GEMM_PIPE_PERSIST && K >= 2 * GBK &&
                         ((epi != EPI_LNF_GELU_F16 && epi != EPI_LNF_GELU_F8) || K >= 4 * GBK) &&
                         !(epi == EPI_LNR16_STATS && lfv.stat_ld != 1);
    // persistent: 8 XCD groups x G walkers (one 8-wave workgroup per CU, 128 KiB LDS)
    const int64_t g = persist ? 8 * std::min<int64_t>(32, ceil_div(big_tiles, 8)) : big_tiles;
    SR_CHECK(!persist || (g % 8 == 0 && g >= 8), "gemm: persistent grid must be a multiple of 8");
    const dim3 grid((unsigned)g), block(512);
#define SR_PIPE_CASE(E)                                                                          \
  case E:                                                                                        \
    if (persist)                                                                                 \
      hipLaunchKernelGGL((gemm_pipe_kernel<E, true>), grid, block, 0, stream, X, lda, W, bias, R, \
                         ldr, Y, ldy, M, N, K, lfv);                                             \
    else                                                                                         \
      hipLaunchKernelGGL((gemm_pipe_kernel<E, false>), grid, block, 0, stream, X, lda, W, bias, R,\
                         ldr, Y, ldy, M, N, K, lfv);                                             \
    break;
    switch (epi) {
      SR_PIPE_CASE(EPI_BIAS_F16)
      SR_PIPE_CASE(EPI_BIAS_GELU_F16)
      SR_PIPE_CASE(EPI_BIAS_RES_F32)
      SR_PIPE_CASE(EPI_BIAS_RES_F16)
      SR_PIPE_CASE(EPI_BIAS_TANH_F32)
      SR_PIPE_CASE(EPI_LNF_F16)
      SR_PIPE_CASE(EPI_LNF_GELU_F16)
      SR_PIPE_CASE(EPI_RES16_STATS)
      SR_PIPE_CASE(EPI_LNR16_STATS)
      SR_PIPE_CASE(EPI_LNF_GELU_F8)
      SR_PIPE_CASE(EPI_RES16_STATS_Y8)
      SR_PIPE_CASE(EPI_LNR16_STATS_Y8)
      default: SR_CHECK(false, "gemm: unknown epilogue");
    }
#undef SR_PIPE_CASE
  } else {
    const int64_t tiles = (int64_t)(N / 128) * ceil_div(M, 128);
    SR_CHECK(tiles < (1ll << 31), "gemm: too many tiles");
    // split-K over the K chunks (see KCHUNK) when the tiles alone leave the CUs idle and the
    // caller lent a workspace for the partial tiles (64 KiB per tile and chunk): chunk groups of
    // cpg chunks, about 512 workgroups in all
    const int64_t nchunk = ceil_div(K / GBK, KCHUNK);
    int64_t groups = 1, cpg = 0;
    if (lf && lf->chunk_ws && nchunk >= 2 && tiles <= kSplitMaxTiles &&
        nchunk * tiles * 65536 <= lf->chunk_ws_bytes) {
      cpg = ceil_div(nchunk, std::min<int64_t>(nchunk, ceil_div(512, tiles)));
      groups = ceil_div(nchunk, cpg);
    }
    // (chunked sums only for the callers that lent a workspace: the same chunks split or not)
    launch_tile<128, 128, 2, 2, false>(epi, dim3((unsigned)tiles, (unsigned)groups), stream, X, lda, W,
                                       bias, R, ldr, Y, ldy, M, N, K, x_k / GBK,
                                       cpg ? reinterpret_cast<float4v*>(lf->chunk_ws) : nullptr, (int)cpg,
                                       lf && lf->chunk_ws ? KCHUNK : 0);
  }
  SR_LAUNCH_CHECK();
}

}  // namespace sr
