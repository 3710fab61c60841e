/* super_rag_mi355x_diag.h -- the diagnostic surface of the MI355X hot-path library.
 *
 * Exported by libsrmi_diag.so only (make -C super-rag_amd: the product sources built again with
 * SR_WITH_DIAG=1), never by the product library libsrmi.so.  These entry points drive ONE kernel
 * on device buffers for single-kernel parity tests (tests/test_gpu_gemm.py, test_gpu_attention.py,
 * test_gpu_ffn1_epilogue.py), microbenchmarks (tools/) and the measured peaks of bench.py; the
 * timing-only variants return wrong results by design.  The diagnostic library also honours the
 * A/B environment knobs of DESIGN.md §4 (SR_GEMM_GROUP_M, SR_GEMM_STAGGER, SR_SCAN_CHUNK,
 * SR_SCAN_GROWTH, SR_SCAN_LEGACY, SR_SCAN_DIAG_NOEPI, SR_QA_DIAG, SR_FFN1_DIAG_WALKERS), which the
 * product library ignores.  No reference counterpart (the reference has no kernels).
 */
#ifndef SUPER_RAG_MI355X_DIAG_H
#define SUPER_RAG_MI355X_DIAG_H

#include "super_rag_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#pragma GCC visibility push(default)
#endif

/* ------------------------------------------------------------------------------------------------
 * Diagnostics (microbenchmarks / parity tests of a single kernel; not used by the product path)
 * ---------------------------------------------------------------------------------------------- */
/* One encoder GEMM Y = epi(X W^T + bias (+R)) on device buffers: X M x K fp16 (row stride lda),
 * W N x K fp16, bias N fp32, R residual (epi 2: fp32, epi 4: fp16, row stride ldr), Y row stride
 * ldy (fp16 for epi 0/1/4, fp32 for 2/3).  epi: 0 bias, 1 bias+GELU, 2 bias+residual fp32,
 * 3 bias+tanh (fp32 out), 4 bias+residual fp16.  variant: -1 auto, 0 128x128, 1 256x256 (8 waves,
 * 2-stage), 4 pipelined 256x256, 5 persistent pipelined 256x256 (6 / 7: timing-only diagnostics
 * with wrong results); variant | 0x100 = split weights: W is [hi | lo] (N x K) over an X of K / 2
 * columns (the embedders' precision mode). */
int sr_diag_gemm(int variant, int epi, const void* X, int64_t lda, const void* W, const float* bias,
                 const void* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K, int device,
                 void* stream);

/* Diagnostic: the LayerNorm-folded FFN1 GEMM Y = 2 GELU(rstd_m (X W^T - mu_m colsum) + bias) on
 * device buffers (the cross-encoders' FFN1 epilogue), fp16 (f8 = 0: X M x K, W N x K fp16, Y fp16)
 * or fp8 (f8 = 1: X, W OCP e4m3 bytes, wexp the E8M0 exponent byte of each W row, Y e4m3 bytes);
 * mr = (mu, rstd) per X row, colsum / bias N fp32.  diag: 0 the product kernel, 2 the main loop
 * without an epilogue, 5 the epilogue math without its stores, 6 the stores of the raw
 * accumulators without the math, 7 the product epilogue with every tile's stores folded onto the
 * first tile (L2-resident) (2 / 5 / 6 / 7: timing only, wrong results). */
int sr_diag_ffn1(int diag, int f8, const void* X, int64_t lda, const void* W, const uint8_t* wexp,
                 const float* bias, const float* colsum, const float* mr, void* Y, int64_t ldy, int M,
                 int N, int K, int device, void* stream);

/* Diagnostic: the residual + row-statistics GEMM epilogue (EPI_RES16_STATS, the encoders'
 * O-projection / FFN2 of layer 0) on device buffers: Y = fp16(X W^T + bias + R) (X M x K fp16, W
 * N x K fp16, bias N fp32, R / Y M x N fp16, row strides ldr / ldy, N % 256 == 0) and per row m and
 * 128-column span s the partials stat_out[(m * N / 128 + s) * 2 + {0, 1}] = (sum, M2) of the fp16
 * outputs of that span (the LayerNorm statistics ln_stats_finalize combines). */
int sr_diag_gemm_stats(const void* X, int64_t lda, const void* W, const float* bias, const void* R,
                       int64_t ldr, void* Y, int64_t ldy, int M, int N, int K, float* stat_out,
                       int device, void* stream);

/* Diagnostic: the FFN2 / O-projection GEMM of the LN-folded encoders, EPI_LNR16_STATS:
 * Y = X W^T + bias + ((R - mu) rstd) gamma per row (R un-normalised, mr = (mu, rstd) per row,
 * consecutive), fp16 Y, and the (sum, M2) partials of every 128-column span of Y as
 * sr_diag_gemm_stats. */
int sr_diag_gemm_lnr_stats(const void* X, int64_t lda, const void* W, const float* bias, const void* R,
                           int64_t ldr, const float* mr, const float* gamma, void* Y, int64_t ldy, int M,
                           int N, int K, float* stat_out, int device, void* stream);

/* Diagnostic: the e4m3-copy statistics epilogues (fp8 mode 3's O-projection: EPI_LNR16_STATS_Y8
 * when lnr != 0, as sr_diag_gemm_lnr_stats; EPI_RES16_STATS_Y8 otherwise, as sr_diag_gemm_stats,
 * mr / gamma unused): fp16 Y, its e4m3 copy y8 (bytes, row stride ldy) and the (sum, M2) partials. */
int sr_diag_gemm_stats_y8(int lnr, const void* X, int64_t lda, const void* W, const float* bias,
                          const void* R, int64_t ldr, const float* mr, const float* gamma, void* Y,
                          int64_t ldy, uint8_t* y8, int M, int N, int K, float* stat_out, int device,
                          void* stream);

/* Diagnostic: the MFMA issue-rate peak on this box (k_diag.hip).  blocks workgroups of 8 waves,
 * each wave 8 independent accumulator chains x iters of the product's MFMA (f8 = 0: f16
 * 16x16x32; f8 = 1: block-scaled fp8 16x16x128) on random operands; FLOP = blocks x 8 x iters x 8 x
 * 16 x 16 x K x 2 (K = 32 / 128).  sink: device float [blocks x 512]; stamps: device uint64
 * [blocks x 2] = (d s_memtime, d s_memrealtime) of each block's loop (clock = ratio x 100 MHz). */
int sr_diag_mfma_rate(int f8, int blocks, int iters, float* sink, uint64_t* stamps, int device, void* stream);

/* Diagnostic: sr_diag_gemm_lnr_stats's persistent kernel with in-kernel s_memtime phase stamps
 * (stamps: device uint64 [grid x 8 waves x 8], sr_diag_ffn1_stamps' layout; grid = 8 x min(32,
 * ceil(tiles / 8))). */
int sr_diag_gemm_lnr_stats_stamps(const void* X, int64_t lda, const void* W, const float* bias, const void* R,
                                  int64_t ldr, const float* mr, const float* gamma, void* Y, int64_t ldy, int M,
                                  int N, int K, float* stat_out, uint64_t* stamps, int device, void* stream);

/* Diagnostic: K5c (fused QKV projection + attention, LN-folded: X un-normalised rows, W the folded
 * [Q; K; V] weight (3d x d), bias the folded bias, colsum its row sums, mr (mu, rstd) per row; S ==
 * 128, head dim 64) with in-kernel s_memtime phase stamps.  stamps: device uint64 [grid x 8 waves
 * x 8] = per wave [tiles, cycles of: the K-loop, the epilogue into the LDS images, the attention,
 * the tile transition, 0, 0, 0]; grid = 8 x min(32, ceil(B S / 256 x heads / 8)). */
int sr_diag_qkv_attention_stamps(const void* X, int64_t lda, const void* W, const float* bias,
                                 const float* colsum, const float* mr, const int32_t* mask, void* ctx, int B,
                                 int S, int d, int heads, uint64_t* stamps, int device, void* stream);

/* Diagnostic: the fp16 FFN1 of sr_diag_ffn1 with in-kernel s_memtime phase stamps (diag 9: the
 * product epilogue, 10: its math without the global stores, 11: the product epilogue without the
 * next tile's staging in its shadow -- timing only, wrong results).  stamps: device uint64 [grid x 8
 * waves x 8] = per wave [tile transitions, cycles of: K-step 0 (tile start -> its barrier),
 * K-step 1, the rest of the K-loop, the epilogue, the transition wait + barrier, K-steps per
 * tile, 0] (grid = 8 x min(32, tiles / 8) persistent workgroups). */
int sr_diag_ffn1_stamps(int diag, const void* X, int64_t lda, const void* W, const float* bias,
                        const float* colsum, const float* mr, void* Y, int64_t ldy, int M, int N,
                        int K, uint64_t* stamps, int device, void* stream);

/* Diagnostic: device-to-device copy of `bytes` (multiple of 16) with 16-byte lanes, the HBM
 * yardstick bench.py reports beside the spec peak (no reference counterpart). */
int sr_diag_copy(const void* src, void* dst, int64_t bytes, int device, void* stream);

/* Diagnostic: one attention launch (K5) on device pointers.  qkv: [B*S, 3d] fp16 (Q | K | V),
 * mask: [B, S] int32 (0 = padding key), ctx: [B*Sq, d] fp16 (first Sq query rows of every
 * sequence).  variant: -1 auto, 0 the 64-key-tile kernel, 1 the whole-head-in-LDS kernel with 4
 * waves per workgroup, 2 the same with 8 waves, 3 auto but the per-workgroup K5b STREAM form instead
 * of the persistent K5d at S_pad = 512 (variants 1-3: d/heads must be 64 and S <= 512). */
int sr_diag_attention(int variant, const void* qkv, const int32_t* mask, void* ctx, int B, int S,
                      int Sq, int d, int heads, int device, void* stream);

#if defined(__GNUC__) || defined(__clang__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif

#endif /* SUPER_RAG_MI355X_DIAG_H */
