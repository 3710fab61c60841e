/*
 * super_rag_mi355x.h — C-ABI of the MI355X (gfx950) embed -> retrieve -> rerank hot path.
 *
 * This library replaces the arithmetic that promoteAI/super-rag sends out of process:
 *   - the SeekDB HNSW cosine search behind
 *       super_rag/vectorstore/seekdb_connector.py:98-115  (SeekDBVectorStoreConnector.search)
 *       super_rag/vectorstore/seekdb_connector.py:56-96   (create_collection / add / delete)
 *     -> sr_store_*  (in-HBM exact cosine top-k, fp16 rows, MFMA scan + fused threshold filter)
 *   - the remote embedding server reached by litellm.embedding() at
 *       super_rag/llm/embed/embedding_service.py:153-194  (EmbeddingService._embed_batch)
 *     -> sr_encoder_forward*  (BERT / XLM-R encoder, CLS or masked-mean pool, L2 normalise)
 *   - the remote cross-encoder reached by litellm.arerank() at
 *       super_rag/llm/rerank/rerank_service.py:87-153    (RerankService._rank_texts)
 *     -> sr_cross_score*  (XLM-R encoder + RoBERTa classification head -> one logit per pair)
 *
 * Conventions
 *   - Every int-returning entry point returns SR_OK (0) on success and a negative SR_ERR_* code on
 *     failure; the message is available from sr_last_error() (thread-local, valid until the next
 *     call on the same thread).
 *   - Host pointers are caller-owned and only read/written during the call.  Device pointers
 *     (the *_dev entry points) must live on the object's device; `stream` is a hipStream_t used
 *     as given (NULL = the HIP null stream, which is what PyTorch reports for its default
 *     stream) and the call is asynchronous on it unless stated.  Host-pointer entry points run
 *     on the object's own stream and are blocking.
 *   - Objects are internally locked: every entry point is safe to call from several host threads.
 *     The Python binding calls through ctypes.CDLL, which releases the GIL for the duration.
 *   - Scores follow SeekDB's cosine semantics: dist = 1 - cos(q, x)  (lower is better,
 *     seekdb_connector.py:143 passes the distance through as DocumentWithScore.score).
 *     Ties are broken by ascending row id.  Missing results (k > live rows) are reported as
 *     row = -1, dist = +inf.
 */
#ifndef SUPER_RAG_MI355X_H
#define SUPER_RAG_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#pragma GCC visibility push(default)
#endif

#define SR_OK 0
#define SR_ERR_INVALID (-1)   /* bad argument / shape                                   */
#define SR_ERR_HIP (-2)       /* HIP runtime or kernel launch failure                    */
#define SR_ERR_OOM (-3)       /* device allocation failed                                */
#define SR_ERR_IO (-4)        /* snapshot read/write failure                             */
#define SR_ERR_STATE (-5)     /* object not ready (e.g. encoder weights missing)         */

#define SR_DTYPE_F32 0
#define SR_DTYPE_F16 1
#define SR_DTYPE_FP8_E4M3 2   /* OCP e4m3fn (scan copy of the store, sr_store_set_scan_dtype)  */

#define SR_POOL_CLS 0         /* BGE models: hidden state of the first token             */
#define SR_POOL_MEAN 1        /* attention-mask weighted mean over tokens                */

#define SR_MAX_TOPK 1024

typedef struct sr_store sr_store;
typedef struct sr_encoder sr_encoder;

const char* sr_last_error(void);
int sr_version(void);
/* Number of visible HIP devices (0 on a host without a GPU; never fails on such a host). */
int sr_device_count(int* out);
/* Copy `bytes` between host and device memory of `device` (kind: 0 = H2D, 1 = D2H, 2 = D2D). */
int sr_memcpy(void* dst, const void* src, int64_t bytes, int kind, int device);

/* ------------------------------------------------------------------------------------------------
 * Vector store  (replaces SeekDBVectorStoreConnector, seekdb_connector.py:31-155)
 * Rows are L2-normalised on insertion and kept as fp16 in HBM, row-major, dim padded to 64.
 * ---------------------------------------------------------------------------------------------- */

/* create_collection(vector_size=dim) — seekdb_connector.py:56-66 (HNSW, distance="cosine"). */
int sr_store_create(int dim, int device, int64_t initial_capacity, sr_store** out);
/* add(nodes) — seekdb_connector.py:68-85: n host fp32 rows (n x dim); out_rows[i] = row id. */
int sr_store_add(sr_store* s, const float* vecs, int64_t n, int64_t* out_rows);
/* Same, rows already on the device (dtype SR_DTYPE_F32 or SR_DTYPE_F16, n x dim, row-major).
 * Row ids are first_row .. first_row + n - 1. */
int sr_store_add_dev(sr_store* s, const void* vecs, int dtype, int64_t n, int64_t* first_row,
                     void* stream);
/* delete(ids=...) — seekdb_connector.py:90-96: tombstones rows (ignored ids are an error). */
int sr_store_remove(sr_store* s, const int64_t* rows, int64_t n);
int sr_store_count(sr_store* s, int64_t* n_rows, int64_t* n_live);
int sr_store_dim(sr_store* s, int* dim);
/* Read back stored (normalised, fp16-rounded) rows as fp32, for with_vectors / parity checks. */
int sr_store_get(sr_store* s, const int64_t* rows, int64_t n, float* out);
/* search(QueryWithEmbedding) — seekdb_connector.py:98-115 (collection.query n_results=top_k).
 * q: B x dim host fp32 (normalised internally).  out_dist / out_rows: B x k host buffers, each
 * query's results sorted by (dist asc, row asc).  Blocking. */
int sr_store_search(sr_store* s, const float* q, int B, int k, float* out_dist, int64_t* out_rows);
/* Filtered search (the score_threshold / filter kwargs the reference passes and SeekDB's
 * connector ignores, context/context.py:37-47, :74-111): only rows with
 * allow[row] != 0 (host, n_rows bytes) compete, so a query still gets its k best ELIGIBLE rows.
 * The eligibility mask (allow & live) is kept on the device and reused while mask_key (non-zero)
 * and the store contents are unchanged; mask_key 0 uploads it every call. */
int sr_store_search_masked(sr_store* s, const float* q, int B, int k, const uint8_t* allow,
                           int64_t mask_key, float* out_dist, int64_t* out_rows);
/* sr_store_search / sr_store_search_masked (allow may be NULL) returning the similarities
 * (descending, -inf when missing) instead of 1 - sim: for callers that merge several stores' lists
 * (two neighbouring fp32 similarities can round to one fp32 distance). */
int sr_store_search_sim(sr_store* s, const float* q, int B, int k, const uint8_t* allow,
                        int64_t mask_key, float* out_sim, int64_t* out_rows);
/* Device variant: q is B x dim on the device (SR_DTYPE_F32 or SR_DTYPE_F16), out_sim/out_rows
 * device buffers of B x k (similarity = 1 - dist, rows int64; -1 / -inf when missing).
 * row_offset is added to every returned row (global row id of a shard).  Synchronises `stream`
 * once at the end to check the candidate-overflow flag (and reruns the exact slow path if set). */
int sr_store_search_dev(sr_store* s, const void* q, int q_dtype, int B, int k, float* out_sim,
                        int64_t* out_rows, int64_t row_offset, void* stream);
/* Scan precision (BASELINE config 5 "fp8 MFMA GEMM path"): SR_DTYPE_F16 (default) or
 * SR_DTYPE_FP8_E4M3: an fp8 copy of the rows (per-row power-of-two scale) is scanned with the
 * block-scaled fp8 MFMA (half the HBM bytes of the fp16 scan), the top max(2k, k + 32) candidates
 * are re-scored exactly on the fp16 rows, and the exact top k is returned (same result as the fp16
 * scan whenever the fp8 stage keeps the true top k among its candidates; recall measured in
 * tests/test_gpu_store.py and bench).  Quantises every row when switched on. */
int sr_store_set_scan_dtype(sr_store* s, int dtype);
/* Snapshot (checkpoint/resume of the corpus; SeekDB persisted rows server-side). */
int sr_store_save(sr_store* s, const char* path);
int sr_store_load(const char* path, int device, sr_store** out);
/* Drop tombstoned rows; old_to_new (host, n_rows entries, may be NULL) receives the new row id
 * of every old row (-1 for removed rows). */
int sr_store_compact(sr_store* s, int64_t* old_to_new);
void sr_store_destroy(sr_store* s);

/* ------------------------------------------------------------------------------------------------
 * Multi-device collection: SURVEY §8(b)'s sr_store_create(dim, dtype, devices, n_dev) — the
 * reference configures one vector DB per deployment (super_rag/config.py:65-67, adaptor
 * vectorstore/connector.py:4-15); here a collection is row-sharded over the listed devices (the
 * same device may repeat).  Global row ids are the insertion order across shards (each add batch
 * goes to the shard with the fewest rows), so every result equals one sr_store's bit for bit:
 * shards are searched concurrently (K1 + K2 on each device) and merged by (dist asc, row asc).
 * dtype: SR_DTYPE_F16, or SR_DTYPE_FP8_E4M3 for the fp8 scan copy (sr_store_set_scan_dtype).
 * Snapshots, compaction and the device-buffer entry points stay per shard (sr_store_*; the Python
 * connector's ShardedStore composes them). */
typedef struct sr_store_set sr_store_set;
int sr_store_set_create(int dim, int dtype, const int* devices, int n_dev, sr_store_set** out);
int sr_store_set_add(sr_store_set* s, const float* vecs, int64_t n, int64_t* out_rows);
int sr_store_set_remove(sr_store_set* s, const int64_t* rows, int64_t n);
int sr_store_set_count(sr_store_set* s, int64_t* n_rows, int64_t* n_live, int* n_shards);
int sr_store_set_get(sr_store_set* s, const int64_t* rows, int64_t n, float* out);
/* sr_store_search semantics; allow (host, n_rows bytes) may be NULL, else as sr_store_search_masked. */
int sr_store_set_search(sr_store_set* s, const float* q, int B, int k, const uint8_t* allow,
                        int64_t mask_key, float* out_dist, int64_t* out_rows);
int sr_store_set_set_scan_dtype(sr_store_set* s, int dtype);
void sr_store_set_destroy(sr_store_set* s);

/* Merge P per-shard top-k lists (device buffers P x B x k of similarity and global row, as written
 * by sr_store_search_dev) into one B x k_out list per query, on `device`. */
int sr_topk_merge_dev(const float* sims, const int64_t* rows, int P, int B, int k, int k_out,
                      float* out_sim, int64_t* out_rows, int device, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Lexical (BM25) index and hybrid dense + lexical retrieval  (BASELINE config 5)
 * The reference declares a `fulltext_search` node type (schema/view_models.py:276-283,
 * FulltextSearchParams{topk, keywords} at :1043-1047) and a merge slot for its output
 * (nodeflow/runners/merge.py:18-20) but ships no backend for them; these entry points are that
 * backend.  Rows are the same row ids as the companion sr_store (the connector adds both in step).
 * Scoring is Okapi BM25 with Lucene's idf ln(1 + (N - df + 0.5) / (df + 0.5)) over LIVE rows,
 * accumulated in 2^-16 fixed point (exact, order-independent); see DESIGN.md "Hybrid retrieval".
 * ---------------------------------------------------------------------------------------------- */
typedef struct sr_lex sr_lex;

int sr_lex_create(int device, float k1, float b, sr_lex** out);
/* Append n documents: document i has the DISTINCT term ids terms[off[i] .. off[i+1]) with
 * frequencies tf[...] (>= 1) and length dl[i] (tokens); off[0] == 0.  first_row receives the row
 * id of document 0 (rows are consecutive). */
int sr_lex_add(sr_lex* x, const int64_t* off, const int32_t* terms, const int32_t* tf,
               const int32_t* dl, int64_t n, int64_t* first_row);
int sr_lex_remove(sr_lex* x, const int64_t* rows, int64_t n);
int sr_lex_stats(sr_lex* x, int64_t* n_rows, int64_t* n_live, int64_t* n_postings,
                 int64_t* vocab, double* avgdl);
/* BM25 top-k: query b is the term ids qterms[qoff[b] .. qoff[b+1]) (a repeated term counts once
 * per occurrence; unknown ids are ignored).  out_score / out_rows: B x k host buffers sorted by
 * (score desc, row asc); -inf / -1 past the matching rows.  allow (optional, n_rows bytes) as in
 * sr_store_search_masked. */
int sr_lex_search(sr_lex* x, const int64_t* qoff, const int32_t* qterms, int B, int k,
                  const uint8_t* allow, int64_t mask_key, float* out_score, int64_t* out_rows);
/* Corpus-wide statistics of a row-sharded lexical corpus, so every shard scores with the same N,
 * avgdl and document frequencies (then per-shard results merge into exactly one index's):
 * n_live / sum_dl summed over the shards (sr_lex_totals), df[i] of terms[i] summed (sr_lex_df)
 * for every term of the queries. */
typedef struct sr_lex_global {
  int64_t n_live;
  int64_t sum_dl;
  const int32_t* terms;
  const int64_t* df;
  int n_terms;
} sr_lex_global;
int sr_lex_totals(sr_lex* x, int64_t* n_live, int64_t* sum_dl);
/* sr_lex_search scored with the corpus-wide statistics of a row-sharded collection (one shard of a
 * multi-device fulltext / hybrid collection; global NULL = sr_lex_search). */
int sr_lex_search_global(sr_lex* x, const int64_t* qoff, const int32_t* qterms, int B, int k,
                         const uint8_t* allow, int64_t mask_key, const sr_lex_global* global,
                         float* out_score, int64_t* out_rows);
/* The same with the exact 2^-16 fixed-point scores too (out_fixed, B x k uint32; score =
 * out_fixed / 65536, 0 past the matches): fp32 rounds scores above 256, so a row-sharded
 * collection merges its shards' lists on these to keep one index's (score, row) order. */
int sr_lex_search_global_fixed(sr_lex* x, const int64_t* qoff, const int32_t* qterms, int B, int k,
                               const uint8_t* allow, int64_t mask_key, const sr_lex_global* global,
                               float* out_score, int64_t* out_rows, uint32_t* out_fixed);
int sr_lex_df(sr_lex* x, const int32_t* terms, int n, int64_t* out_df);
/* Device outputs (B x k on the index's device, score fp32 / row int64 + row_offset; -inf / -1 past
 * the matches), asynchronous on `stream` after the host-side term preparation; global may be NULL
 * (this index's own statistics). */
int sr_lex_search_dev(sr_lex* x, const int64_t* qoff, const int32_t* qterms, int B, int k,
                      const sr_lex_global* global, float* out_score, int64_t* out_rows,
                      int64_t row_offset, void* stream);
/* Device-resident queries (the batched hybrid pipeline: query tokens already in HBM, no host copy
 * of the queries).  Asynchronous on `stream` when the batch fits one worst-case query group
 * (B x Lq x max df keys within the 2 GiB key budget, B <= 1024); a larger batch is grouped by the
 * queries' actual candidate caps, computed on the device and read back ONCE (one blocking
 * hipStreamSynchronize on `stream`, which also waits for work queued before it).  tok: B x Lq int32 device (row stride Lq), qlen: B int32 device.
 * sr_lex_query_stats_dev writes out_stats[0] = live rows, [1] = summed document length, [2 + q Lq +
 * i] = live df of query q's i-th token (0 past qlen[q]): 2 + B Lq int64 on the device, the vector a
 * row-sharded corpus sums over its shards (one all-reduce).  sr_lex_search_tok_dev = sr_lex_search_dev
 * for those queries, scored with the summed vector gstats (device, NULL = this index's own
 * statistics); same results bit for bit. */
int sr_lex_query_stats_dev(sr_lex* x, const int32_t* tok, const int32_t* qlen, int B, int Lq,
                           int64_t* out_stats, void* stream);
int sr_lex_search_tok_dev(sr_lex* x, const int32_t* tok, const int32_t* qlen, int B, int Lq, int k,
                          const int64_t* gstats, float* out_score, int64_t* out_rows,
                          int64_t row_offset, void* stream);
int sr_lex_save(sr_lex* x, const char* path);
int sr_lex_load(const char* path, int device, sr_lex** out);
int sr_lex_compact(sr_lex* x, int64_t* old_to_new);
void sr_lex_destroy(sr_lex* x);

/* Reciprocal-rank fusion of two ranked row lists per query (B x ka and B x kb, -1 padded), as
 * graphiti rrf (graphiti_core/search/search_utils.py:1762-1778): score = sum 1 / (rank +
 * rank_const) in fp64, order (score desc, first appearance), rows with score < min_score
 * dropped.  Host buffers; computed on `device`. */
int sr_rrf_fuse(const int64_t* rows_a, int ka, const int64_t* rows_b, int kb, int B,
                int rank_const, double min_score, int k_out, double* out_score,
                int64_t* out_rows, int device);
/* Same on device buffers, asynchronous on `stream` of `device`. */
int sr_rrf_fuse_dev(const int64_t* rows_a, int ka, const int64_t* rows_b, int kb, int B,
                    int rank_const, double min_score, int k_out, double* out_score,
                    int64_t* out_rows, int device, void* stream);
/* Hybrid retrieval on one device: dense top-k_each (sr_store_search semantics) and BM25
 * top-k_each of the same queries, fused on the device by rrf into B x k (out_score = rrf score).
 * q: B x dim host fp32; the lexical query as in sr_lex_search; allow optional (mask_key as in
 * sr_store_search_masked). */
int sr_hybrid_search(sr_store* s, sr_lex* x, const float* q, const int64_t* qoff,
                     const int32_t* qterms, int B, int k, int k_each, int rank_const,
                     double min_score, const uint8_t* allow, int64_t mask_key,
                     double* out_score, int64_t* out_rows);

/* ------------------------------------------------------------------------------------------------
 * Transformer encoder (BERT / XLM-R family: bge-small/base-en, bge-m3, bge-reranker-*)
 * Weights are set by Hugging Face tensor name without the model prefix, e.g.
 * "embeddings.word_embeddings.weight", "encoder.layer.3.attention.self.query.weight",
 * "classifier.dense.weight", "classifier.out_proj.bias".  Matrices are stored fp16 in HBM,
 * biases / LayerNorm parameters fp32.  Activations are fp16 GEMM operands with an fp32
 * residual stream; accumulation is fp32 everywhere.
 * ---------------------------------------------------------------------------------------------- */
typedef struct sr_encoder_config {
  int vocab_size;
  int hidden;           /* d                                         */
  int layers;           /* L                                         */
  int heads;            /* d / heads must be 32 or 64               */
  int intermediate;     /* FFN width                                 */
  int max_position;
  int type_vocab;       /* token-type rows (1 for XLM-R, 2 for BERT) */
  float ln_eps;         /* 1e-12 BERT, 1e-5 XLM-R                    */
  int position_offset;  /* 0: BERT (pos = index); >0: XLM-R padding_idx (pos = cumsum(mask)+pad) */
  int classifier;       /* 0: none; 1: RoBERTa classification head (dense+tanh+out_proj)       */
  int num_labels;       /* classifier outputs (1 for bge-reranker)                             */
  int max_tokens;       /* workspace size in tokens per launch chunk (0 = default 262144)      */
  int residual_fp16;    /* 0: fp32 residual stream (embeddings, <= 1e-3 rel error);
                           1: fp16 residual stream (cross-encoders: ~2.5x less LayerNorm and
                              epilogue traffic, ranking-level fidelity)                         */
} sr_encoder_config;

int sr_encoder_create(const sr_encoder_config* cfg, int device, sr_encoder** out);
int sr_encoder_set_weight(sr_encoder* e, const char* name, const float* data, int64_t numel);
/* Returns SR_OK when every weight has been set, SR_ERR_STATE (message lists a missing one) else. */
int sr_encoder_ready(sr_encoder* e);
/* Sentence embeddings: ids/mask/type_ids are B x S int32 host arrays (type_ids may be NULL);
 * out: B x hidden fp32, L2-normalised (EmbeddingService.embed_documents result rows). Blocking. */
int sr_encoder_forward(sr_encoder* e, const int32_t* ids, const int32_t* mask,
                       const int32_t* type_ids, int B, int S, int pool, float* out);
/* Device variant; out dtype SR_DTYPE_F32 (B x hidden) or SR_DTYPE_F16 (B x ld_out, row-major,
 * ld_out >= hidden, zero-padded to ld_out so it can be fed to sr_store_search_dev). */
int sr_encoder_forward_dev(sr_encoder* e, const int32_t* ids, const int32_t* mask,
                           const int32_t* type_ids, int B, int S, int pool, void* out,
                           int out_dtype, int ld_out, void* stream);
/* Cross-encoder relevance: P (query, passage) pairs already packed as token ids (P x S);
 * out_logits: P x num_labels fp32 raw logits (bge-reranker scores = logits, sigmoid optional). */
int sr_cross_score(sr_encoder* e, const int32_t* ids, const int32_t* mask,
                   const int32_t* type_ids, int P, int S, float* out_logits);
int sr_cross_score_dev(sr_encoder* e, const int32_t* ids, const int32_t* mask,
                       const int32_t* type_ids, int P, int S, float* out_logits, void* stream);
/* fp8 precision modes (BASELINE config 5 "fp8 MFMA GEMM path"; LN-folded fp16-residual encoders,
 * e.g. the cross-encoders).  1: FFN1 stores OCP e4m3 activations and FFN2 runs the block-scaled
 * fp8 MFMA against an e4m3 copy of its weight (per-row power-of-two scales); 2: also FFN1 and the
 * QKV GEMMs of layers >= 1 on e4m3 copies of the residual sums (written by the residual
 * epilogues) and of the folded weights; 3: FFN1 and FFN2 as in mode 2, the QKV projection and
 * attention stay fp16 (fused).  0 (default): fp16.  Opt-in: logits move by the fp8 rounding
 * (tests/test_gpu_encoder.py; ranking fidelity per mode: tests/test_gpu_rerank_fidelity.py). */
int sr_encoder_set_fp8(sr_encoder* e, int mode);
void sr_encoder_destroy(sr_encoder* e);

/* ------------------------------------------------------------------------------------------------
 * Device pipeline helpers for the batched search path (embed -> top-K -> pairs -> rerank)
 * ---------------------------------------------------------------------------------------------- */
/* Pack cross-encoder inputs for every (query b, candidate j):
 *   style 0 (RoBERTa/XLM-R):  <s> q </s> </s> p </s>      style 1 (BERT): [CLS] q [SEP] p [SEP]
 * q_tok: B x lq_max content tokens (no specials), q_len: B;  p_tok: N x lp_max, p_len: N;
 * cand_rows: B x K (int64; rows < 0 give an all-padding pair).  The passage is truncated first,
 * then the query.  out_ids / out_mask / out_type: (B*K) x S int32 (out_type may be NULL). */
int sr_build_pairs_dev(const int32_t* q_tok, const int32_t* q_len, int lq_max,
                       const int32_t* p_tok, const int32_t* p_len, int lp_max,
                       const int64_t* cand_rows, int B, int K, int S, int style,
                       int bos_id, int eos_id, int pad_id,
                       int32_t* out_ids, int32_t* out_mask, int32_t* out_type,
                       int device, void* stream);
/* Per query: order the K candidates by (logit desc, candidate index asc) and keep k_out.
 * logits: B x K fp32; out_index: B x k_out int32 positions into the candidate list. */
int sr_rerank_select_dev(const float* logits, int B, int K, int k_out, int32_t* out_index,
                         int device, void* stream);

/* ------------------------------------------------------------------------------------------------
 * Profiling: per-kernel HIP-event timing of every launch on the library's streams.
 * ---------------------------------------------------------------------------------------------- */
typedef struct sr_kernel_stat {
  char name[64];        /* kernel family, e.g. "gemm_f16_gelu", "cosine_scan"              */
  int64_t launches;
  double total_ms;      /* sum of HIP-event durations                                        */
  double flops;         /* algorithmic FLOPs over all launches                               */
  double bytes;         /* algorithmic HBM bytes over all launches                           */
} sr_kernel_stat;

int sr_profile_enable(int on);              /* clears the table when turned on                  */
/* Fills up to max entries (synchronises the recorded events); *n receives the number written. */
int sr_profile_read(sr_kernel_stat* out, int max, int* n);

/* The kernel-level diagnostics (sr_diag_*: single-kernel parity entry points, timing-only
 * variants, the HBM copy yardstick) are not part of this library: they live in the separate
 * libsrmi_diag.so, declared in super_rag_mi355x_diag.h. */

#if defined(__GNUC__) || defined(__clang__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif

#endif /* SUPER_RAG_MI355X_H */
