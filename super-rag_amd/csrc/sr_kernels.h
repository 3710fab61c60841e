// Host-side launchers of the HIP kernels (one declaration per kernel family).
#pragma once

#include "sr_common.h"

namespace sr {

enum Epilogue {
  EPI_BIAS_F16 = 0,       // y = acc + b                 -> fp16
  EPI_BIAS_GELU_F16 = 1,  // y = gelu_erf(acc + b)       -> fp16
  EPI_BIAS_RES_F32 = 2,   // y = acc + b + R (fp32)      -> fp32
  EPI_BIAS_TANH_F32 = 3,  // y = tanh(acc + b)           -> fp32 (classifier head)
  EPI_BIAS_RES_F16 = 4    // y = acc + b + R (fp16)      -> fp16
};

// k_gemm.hip — Y = epi(X . W^T + bias (+ R)); K % 64 == 0, N % 128 == 0.
void launch_gemm(int epi, const half_t* X, int64_t lda, const half_t* W, const float* bias,
                 const void* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K,
                 hipStream_t stream);
enum GemmVariant { GEMM_SMALL = 0, GEMM_BIG = 1, GEMM_BIG_PERSIST = 2, GEMM_DEEP = 3, GEMM_PIPE = 4, GEMM_PIPE_PERSIST = 5,
                   GEMM_DIAG_NOLOAD = 6, GEMM_DIAG_NOEPI = 7 /* timing only */ };
void launch_gemm_variant(int variant, int epi, const half_t* X, int64_t lda, const half_t* W,
                         const float* bias, const void* R, int64_t ldr, void* Y, int64_t ldy,
                         int M, int N, int K, hipStream_t stream);
void gemm_force_tile(int t);  // test hook: -1 auto, else a GemmVariant

// k_attention.hip — ctx = MHA(qkv, key padding mask) for the first Sq query rows of each
// sequence; ctx rows are laid out [B][Sq][d].
void launch_attention(const half_t* qkv, const int32_t* mask, half_t* ctx, int B, int S, int Sq,
                      int d, int heads, hipStream_t stream);
void attention_force_variant(int v);  // test hook: -1 auto, 0 = 64-key-tile kernel, 1 = K5b

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

// k_search.hip
int scan_query_tiles(int B);
int select_capacity();
void launch_cosine_scan(bool dense, const half_t* corpus, int64_t ldc, const uint8_t* live,
                        int64_t r0, int64_t r1, const half_t* Q, int B, const float* tau,
                        uint64_t* cand, int* cnt, int cap, hipStream_t s);
void launch_topk_select(uint64_t* cand, int* cnt, int cap, float* tau, int B, int k,
                        int* overflow, bool final_pass, float* out_sim, int64_t* out_rows,
                        int64_t row_offset, hipStream_t s);
void launch_topk_merge(const float* sims, const int64_t* rows, int P, int B, int k, int k_out,
                       float* out_sim, int64_t* out_rows, hipStream_t s);
void launch_fill_int(int* p, int n, int v, hipStream_t s);
void launch_fill_float(float* p, int n, float v, hipStream_t s);
void launch_build_pairs(const int32_t* q_tok, const int32_t* q_len, int lq_max,
                        const int32_t* p_tok, const int32_t* p_len, int lp_max,
                        const int64_t* cand_rows, int B, int K, int S, int style, int bos, int eos,
                        int pad, int32_t* out_ids, int32_t* out_mask, int32_t* out_type,
                        hipStream_t s);
void launch_rerank_select(const float* logits, int B, int K, int k_out, int32_t* out_index,
                          hipStream_t s);

}  // namespace sr
