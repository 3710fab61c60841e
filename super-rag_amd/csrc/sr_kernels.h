// Host-side launchers of the HIP kernels (one declaration per kernel family).
#pragma once

#include "sr_common.h"

namespace sr {

enum Epilogue {
  EPI_BIAS_F16 = 0,       // y = acc + b                 -> fp16
  EPI_BIAS_GELU_F16 = 1,  // y = gelu_erf(acc + b)       -> fp16
  EPI_BIAS_RES_F32 = 2,   // y = acc + b + R (fp32)      -> fp32
  EPI_BIAS_TANH_F32 = 3,  // y = tanh(acc + b)           -> fp32 (classifier head)
  EPI_BIAS_RES_F16 = 4,   // y = acc + b + R (fp16)      -> fp16
  // LayerNorm folded into the GEMMs around it (fp16 residual stream; pipelined 256x256 kernels,
  // N % 256 == 0).  The A operand / residual is the UN-normalised row u with LN(u) =
  // (u - mu) * rstd * gamma + beta; mu / rstd come from per-row partial statistics written by the
  // producing GEMM's epilogue (LnFold below).
  EPI_LNF_F16 = 5,        // y = rstd * (acc - mu * c[n]) + b'[n], W' = W . diag(gamma) -> fp16
  EPI_LNF_GELU_F16 = 6,   // y = 2 gelu(same) (the FFN2 weight carries the 0.5)          -> fp16
  EPI_RES16_STATS = 7,    // y = acc + b + R (fp16, already normalised) -> fp16 + row statistics
  EPI_LNR16_STATS = 8,    // y = acc + b + LN(R) (R un-normalised)      -> fp16 + row statistics
  // K1 on the GEMM main loop (internal: launch_cosine_scan_gemm): W = corpus rows, X = queries,
  // epilogue = threshold filter appending (sim, row) keys to per-query candidate lists
  EPI_SCAN = 9,
  // the same on OCP fp8-e4m3 operands e4m3(256 x) of unit vectors (block-scaled MFMA
  // v_mfma_scale_f32_16x16x128_f8f6f4, E8M0 block scales 2^-8 undo the factor)
  EPI_SCAN8 = 10,
  // EPI_LNF_GELU_F16 storing OCP e4m3(2 GELU) bytes (the fp8 FFN1; its consumer runs fp8)
  EPI_LNF_GELU_F8 = 11,
  // EPI_RES16_STATS / EPI_LNR16_STATS that also store an e4m3 copy of their fp16 output to
  // LnFold.y8 (the next fp8 GEMM's A operand; separate codes keep the fp16 kernels' registers)
  EPI_RES16_STATS_Y8 = 12,
  EPI_LNR16_STATS_Y8 = 13
};

// Per-row statistics hand-over between GEMMs (Chan-combinable partials over 128-column spans):
// stat[row][part] = (sum, M2 = sum (x - sum/128)^2) of the fp16-rounded outputs in that span.
// launch_ln_stats_finalize turns them into mr[row] = (mu, rstd), which the folded epilogues read.
struct LnFold {
  const float* mr = nullptr;       // (mu, rstd) of the A rows (LNF) / residual rows (LNR)
  int64_t stat_ld = 1;             // row r of the operand reads mr row r * stat_ld
  const float* colsum = nullptr;   // LNF: c[n] = sum_k W'[n][k] (fp32 sum of the fp16 W')
  const float* gamma = nullptr;    // LNR: LayerNorm weight of the residual rows (its beta is
                                   //      pre-added to the GEMM bias)
  float* stat_out = nullptr;       // *_STATS: [M][N / 128] partials of the output rows
  const uint8_t* wexp = nullptr;   // fp8 operands (launch_gemm_f8w): E8M0 exponent per weight row
  uint8_t* y8 = nullptr;           // *_STATS: optional e4m3 copy of the fp16 output (row stride
                                   //          ldy bytes), the next fp8 GEMM's A operand
  int group_m = 0;                 // pipelined kernels: tile t walks groups of group_m m-panels
                                   // (m fastest inside a group); 0 / 1 = n fastest
  int stagger = 0;                 // persistent pipelined kernels (diagnostic): > 0: walker w of
                                   // an XCD starts (w & 7) x stagger x 512 cycles late; < 0: the
                                   // walkers of XCD x start x |stagger| x 512 cycles late
                                   // (de-phasing the epilogue store bursts)
  int x_k = 0;                     // split weights: X has x_k columns and K = 2 x_k; the K-steps
                                   // past x_k re-read X from k = 0, so W = [W_hi | W_lo] (N x 2 x_k)
                                   // gives X W_hi^T + X W_lo^T in one fp32 accumulation (0 = K)
  float* chunk_ws = nullptr;        // GEMM_SMALL (128 x 128, short M): workspace for split-K
  int64_t chunk_ws_bytes = 0;      // partial tiles (k_gemm.hip KCHUNK); null: never split
  // EPI_SCAN(8) re-uses the fields (kernel-argument SGPRs are scarce in the persistent kernels):
  // stat_out = per-query candidate counts (int*), stat_ld = global row id of the chunk's first
  // row; bias = tau[B], R = live flags of the chunk, Y = candidate keys [B][cap] (ldy = cap).
};

// k_gemm.hip — Y = epi(X . W^T + bias (+ R)); K % 64 == 0, N % 128 == 0.
void launch_gemm(int epi, const half_t* X, int64_t lda, const half_t* W, const float* bias,
                 const void* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K,
                 hipStream_t stream, const LnFold* lf = nullptr);
enum GemmVariant { GEMM_SMALL = 0, GEMM_BIG = 1, GEMM_PIPE = 4, GEMM_PIPE_PERSIST = 5,
                   GEMM_DIAG_NOLOAD = 6, GEMM_DIAG_NOEPI = 7 /* timing only */, GEMM_PP = 8,
                   GEMM_DIAG_P_NOEPI = 9, GEMM_DIAG_P_MATHONLY = 10, GEMM_DIAG_P_STOREONLY = 11 };
void launch_gemm_variant(int variant, int epi, const half_t* X, int64_t lda, const half_t* W,
                         const float* bias, const void* R, int64_t ldr, void* Y, int64_t ldy,
                         int M, int N, int K, hipStream_t stream, const LnFold* lf = nullptr);
void gemm_force_tile(int t);  // test hook: -1 auto, else a GemmVariant
// K1 for large query blocks (B in (128, 256]) on the pipelined GEMM: rows [r0, r1) of the corpus
// against B queries; non-dense threshold mode only (same contract as launch_cosine_scan).
// Y = epi(X8 . W8^T) on OCP e4m3 operands: X8 [M][K] bytes (lda bytes), W8 [N][K] bytes with
// per-row E8M0 exponents lf->wexp[N] (W = W8 * 2^(wexp - 127)); K % 128 == 0, K >= 256;
// epi in {EPI_LNF_F16, EPI_LNF_GELU_F8, EPI_RES16_STATS(_Y8), EPI_LNR16_STATS(_Y8)}.
#if SR_WITH_DIAG
// Diagnostic FFN1 launches (sr_diag_ffn1): diag 0 product, 2 no epilogue, 5 math only, 6 stores only.
void launch_ffn1_diag(int diag, bool f8, const void* X, int64_t lda, const void* W, const uint8_t* wexp,
                      const float* bias, const float* colsum, const float* mr, void* Y, int64_t ldy,
                      int M, int N, int K, hipStream_t stream, uint64_t* stamps = nullptr);
// MFMA issue-rate peak (k_diag.hip): blocks x 8 waves x iters x 8 independent MFMAs of the
// product's f16 (f8 = 0) or block-scaled fp8 (f8 = 1) shape on random operands; stamps[2 b] /
// [2 b + 1] = d(s_memtime) / d(s_memrealtime) of block b's wave 0 around its loop.
void launch_mfma_rate(int f8, int blocks, int iters, float* sink, uint64_t* stamps, hipStream_t st);
// The persistent EPI_LNR16_STATS GEMM with in-kernel phase stamps (k_gemm.hip; diagnostic)
void launch_lnr_stats_stamps(const half_t* X, int64_t lda, const half_t* W, const float* bias, const void* R,
                             int64_t ldr, const float* mr, const float* gamma, void* Y, int64_t ldy, int M,
                             int N, int K, float* stat_out, uint64_t* stamps, hipStream_t stream);
#endif
void launch_gemm_f8w(int epi, const uint8_t* X8, int64_t lda, const uint8_t* W8, const float* bias,
                     const void* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K,
                     hipStream_t stream, const LnFold* lf);
// colsum[n] = sum_k W8[n][k] * 2^(wexp[n] - 127) (the LN fold's column sums of an e4m3 weight)
void launch_colsum_fp8(const uint8_t* W8, const uint8_t* wexp, int N, int K, float* colsum,
                       hipStream_t s);
// W [N][K] fp16 -> W8 [N][K] e4m3 of W * 2^e_n (largest power of two with max|W_n| 2^e_n <= 448),
// wexp[n] = 127 - e_n
void launch_quantize_rows_fp8(const half_t* W, int N, int K, uint8_t* W8, uint8_t* wexp,
                              hipStream_t s);
// fp8 rows e4m3(256 x) (ld8 bytes, a multiple of 128, >= 256) of unit vectors; sims are cosines.
void launch_cosine_scan_gemm8(const uint8_t* corpus8, int64_t ld8, const uint8_t* live, int64_t r0,
                              int64_t r1, const uint8_t* Q8, int B, const float* tau, uint64_t* cand,
                              int* cnt, int cap, hipStream_t s);
// fp8 K1 for B <= 64 (k_search.hip): the small-block scan kernel on e4m3 rows (ld8 bytes each)
void launch_cosine_scan8(bool dense, const uint8_t* corpus8, int64_t ld8, const uint8_t* live,
                         int64_t r0, int64_t r1, const uint8_t* Q8, int B, const float* tau,
                         uint64_t* cand, int* cnt, int cap, hipStream_t s);
void launch_cosine_scan_gemm(const half_t* corpus, int64_t ldc, const uint8_t* live, int64_t r0,
                             int64_t r1, const half_t* Q, int B, const float* tau, uint64_t* cand,
                             int* cnt, int cap, hipStream_t s);

// k_attention.hip — ctx = MHA(qkv, key padding mask) for the first Sq query rows of each
// sequence; ctx rows are laid out [B][Sq][d].
// K5c (k_attention.hip): ctx = attention(epi(X . Wqkv^T)) without the QKV activation in HBM;
// epi = EPI_BIAS_F16 or EPI_LNF_F16 (lf: row statistics mr, column sums colsum).  S == 128, d_h == 64.
// ctx8 != nullptr: ctx is written there as OCP e4m3 bytes instead ([B*S, d], fp8 mode 5).
bool qkv_attention_supported(int S, int d, int heads);
void launch_qkv_attention(int epi, const half_t* X, int64_t lda, const half_t* W, const float* bias,
                          const LnFold* lf, const int32_t* mask, half_t* ctx, int B, int S, int d,
                          int heads, hipStream_t stream, uint8_t* ctx8 = nullptr,
                          uint64_t* stamps = nullptr);
void launch_attention(const half_t* qkv, const int32_t* mask, half_t* ctx, int B, int S, int Sq,
                      int d, int heads, hipStream_t stream);
void attention_force_variant(int v);  // test hook: -1 auto, 0 = 64-key-tile kernel, 1 = K5b, 2 = K5b with 8 waves

// k_encoder_misc.hip
void launch_positions(const int32_t* ids, int32_t* pos, int B, int S, int offset, hipStream_t s);
// h32 may be null (fp16 residual stream): then only the fp16 copy is written.
void launch_embed_ln(const int32_t* ids, const int32_t* pos, const int32_t* types,
                     const half_t* wemb, const half_t* pemb, const half_t* temb,
                     const float* gamma, const float* beta, float eps, int M, int d, int vocab,
                     int max_pos, int type_vocab, half_t* h16, float* h32, hipStream_t s);
// y is fp32 (y_f16 = false) or fp16; h32 may be null.
void launch_layernorm(const void* y, bool y_f16, const float* gamma, const float* beta, float eps,
                      int M, int d, half_t* h16, float* h32, hipStream_t s);
void launch_pool_l2(const void* h, bool h_f16, const int32_t* mask, int B, int S, int d, int pool,
                    void* out, int out_dtype, int ld_out, hipStream_t s);
void launch_cls_logits(const float* t, const float* w, const float* bias, int P, int d,
                       int labels, float* out, hipStream_t s);
void launch_normalize_rows(const void* x, int dtype, int64_t n, int dim, half_t* out, int ld,
                           hipStream_t s);
void launch_convert_f32_f16(const float* in, half_t* out, int64_t n, hipStream_t s);
// LayerNorm folding of a [N][K] fp32 weight behind LN(gamma, beta): w16 = fp16(W . diag(gamma)),
// colsum[n] = sum_k float(w16[n][k]), bias_out[n] = sum_k W[n][k] beta[k] + bias[n].
void launch_fold_ln_weight(const float* w32, const float* gamma, const float* beta,
                           const float* bias, int N, int K, half_t* w16, float* colsum,
                           float* bias_out, hipStream_t s);
// mr[r] = (mu, rstd) of row r from its nparts Chan partials (n = 128 each), rstd = 1/sqrt(var+eps).
void launch_ln_stats_finalize(const float* stat, int nparts, float eps, int M, float* mr,
                              hipStream_t s);
// h16 = LayerNorm(u) with (mu, rstd) from mr (no re-reduction).
void launch_ln_apply(const half_t* u, int64_t ldu, const float* mr, const float* gamma,
                     const float* beta, int M, int d, half_t* h16, hipStream_t s);
void launch_vec_add(const float* a, const float* b, float* out, int n, hipStream_t s);
// fp8 mode 4: e4m3 copy of the normalised rows (u - mu) rstd (k_encoder_misc.hip)
void launch_quantize_norm_fp8(const half_t* u, int64_t ldu, const float* mr, int M, int d, uint8_t* x8,
                              hipStream_t s);
// K/V-free CLS-only last layer (k_encoder_misc.hip): block-diagonal K / V weights from the folded
// QKV weight, and per sequence scores + softmax + z' = sum_j p_j rstd_j (u_j - mu_j)
bool cls_attn_fold_supported(int S, int D, int H);
void launch_kv_blockdiag(const half_t* wqkv_f, int D, int H, half_t* wk_bd, half_t* wv_bd,
                         hipStream_t s);
void launch_cls_attn_fold(const half_t* w, const half_t* U, const float* mr, const int32_t* mask,
                          int B, int S, int D, int H, half_t* z, hipStream_t s);
void launch_scale_f16(const half_t* in, float scale, half_t* out, int64_t n, hipStream_t s);

// k_search.hip
int scan_query_tiles(int B);
int select_capacity();
void launch_cosine_scan(bool dense, const half_t* corpus, int64_t ldc, const uint8_t* live,
                        int64_t r0, int64_t r1, const half_t* Q, int B, const float* tau,
                        uint64_t* cand, int* cnt, int cap, hipStream_t s);
void launch_topk_select(uint64_t* cand, int* cnt, int cap, float* tau, int B, int k,
                        int* overflow, bool final_pass, float* out_sim, int64_t* out_rows,
                        int64_t row_offset, hipStream_t s,
                        const uint8_t* live = nullptr);
void launch_topk_merge(const float* sims, const int64_t* rows, int P, int B, int k, int k_out,
                       float* out_sim, int64_t* out_rows, hipStream_t s);
void launch_fill_int(int* p, int n, int v, hipStream_t s);
void launch_copy16(const void* src, void* dst, int64_t bytes, hipStream_t s);  // diagnostic
void launch_fill_float(float* p, int n, float v, hipStream_t s);
void launch_build_pairs(const int32_t* q_tok, const int32_t* q_len, int lq_max,
                        const int32_t* p_tok, const int32_t* p_len, int lp_max,
                        const int64_t* cand_rows, int B, int K, int S, int style, int bos, int eos,
                        int pad, int32_t* out_ids, int32_t* out_mask, int32_t* out_type,
                        hipStream_t s);
void launch_rerank_select(const float* logits, int B, int K, int k_out, int32_t* out_index,
                          hipStream_t s);

// k_lex.hip — reciprocal-rank fusion of two ranked row lists per query (-1 padded), fp64 scores.
void launch_rrf_fuse(const int64_t* rows_a, int ka, const int64_t* rows_b, int kb, int B,
                     int rank_const, double min_score, int k_out, double* out_score,
                     int64_t* out_rows, hipStream_t s);

}  // namespace sr
