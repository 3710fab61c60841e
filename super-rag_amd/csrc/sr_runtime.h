// Host runtime objects behind the C-ABI: the in-HBM vector store and the transformer encoder.
#pragma once

#include <memory>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include <fcntl.h>
#include <unistd.h>

#include "sr_common.h"

namespace sr {

// Flush a written file's data to stable storage before it is renamed into place (snapshot
// writers: a commit must never name a base whose bytes are still only in the page cache).
inline bool fsync_path(const std::string& path) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  const bool ok = ::fsync(fd) == 0;
  return (::close(fd) == 0) && ok;
}

// RAII device allocation.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) {
    o.p = nullptr;
    o.bytes = 0;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  // Grow to at least n bytes (contents are NOT preserved).
  void reserve(size_t n) {
    if (n <= bytes) return;
    release();
    SR_HIP(hipMalloc(&p, n));
    bytes = n;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

// Scoped device selection (restores the caller's current device).
struct DeviceGuard {
  int prev = 0;
  explicit DeviceGuard(int dev) {
    SR_HIP(hipGetDevice(&prev));
    if (prev != dev) SR_HIP(hipSetDevice(dev));
  }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

// ------------------------------------------------------------------------------------------------
class Store {
 public:
  Store(int dim, int device, int64_t capacity);
  ~Store();

  int dim() const { return dim_; }
  int ld() const { return ld_; }
  int device() const { return device_; }
  int64_t rows() const { return n_rows_; }
  int64_t live() const { return n_live_; }

  void add_host(const float* vecs, int64_t n, int64_t* out_rows);
  int64_t add_dev(const void* vecs, int dtype, int64_t n, hipStream_t s);
  void remove(const int64_t* rows, int64_t n);
  void get(const int64_t* rows, int64_t n, float* out);
  // allow: optional host eligibility mask (n_rows bytes), cached on the device per mask_key
  // raw_sim: out_dist receives the similarities (descending) instead of 1 - sim, for callers
  // that merge lists (1 - sim in fp32 can merge two neighbouring similarities into one distance)
  void search_host(const float* q, int B, int k, float* out_dist, int64_t* out_rows,
                   const uint8_t* allow = nullptr, int64_t mask_key = 0, bool raw_sim = false);
  void search_dev(const void* q, int q_dtype, int B, int k, float* out_sim, int64_t* out_rows,
                  int64_t row_offset, hipStream_t s, const uint8_t* elig = nullptr);
  // device eligibility mask live & allow (cached per mask_key and store version); null for null
  const uint8_t* eligibility(const uint8_t* allow, int64_t mask_key);
  // scan dtype: SR_DTYPE_F16 (default) or SR_DTYPE_FP8_E4M3 (fp8 copy + exact fp16 re-scoring)
  void set_scan_dtype(int dtype);
  int scan_dtype() const { return fp8_ ? SR_DTYPE_FP8_E4M3 : SR_DTYPE_F16; }
  void save(const char* path);
  static Store* load(const char* path, int device);
  void compact(int64_t* old_to_new);

  std::mutex mu;

 private:
  // Cross-stream ordering: every operation first makes its stream wait for the previous
  // operation's completion event, and records the event when it has enqueued its work, so calls
  // on different streams (the object's own stream, torch's stream, the null stream) never race
  // on the corpus or the shared workspaces.
  void begin(hipStream_t s) { SR_HIP(hipStreamWaitEvent(s, done_, 0)); }
  void end(hipStream_t s) { SR_HIP(hipEventRecord(done_, s)); }
  void ensure_capacity(int64_t rows);
  void ensure_query_ws(int B);
  // Runs the chunked scan/select schedule for one block of <= 256 normalised queries.
  void search_block(const half_t* qn, int B, int k, float* out_sim, int64_t* out_rows,
                    int64_t row_offset, hipStream_t s, bool safe, const uint8_t* live);
  void search_block8(const half_t* qn, int B, int k, float* out_sim, int64_t* out_rows,
                     int64_t row_offset, hipStream_t s, bool safe, const uint8_t* live);
  int ld8() const;
  void grow_fp8();
  void quantize_rows(int64_t r0, int64_t n, hipStream_t s);

  int dim_, ld_, device_;
  int64_t n_rows_ = 0, n_live_ = 0, capacity_ = 0;
  DevBuf corpus_, live_;
  std::vector<uint8_t> live_host_;
  hipStream_t stream_ = nullptr;
  hipEvent_t done_ = nullptr;
  // search workspace
  DevBuf qbuf_, qstage_, cand_, cnt_, tau_, overflow_, osim_, orows_, scratch_;
  int ws_queries_ = 0;
  // fp8 scan: e4m3(256 x) copy of the rows (ld8 bytes each), query staging, fp8-stage candidates
  bool fp8_ = false;
  DevBuf corpus8_, q8_, approx_;
  // filtered search: device eligibility mask (live & allow) and what it was built from
  DevBuf mask_;
  int64_t version_ = 0, mask_key_ = 0, mask_version_ = -1, mask_rows_ = -1;
};

// One collection row-sharded over several devices (store_set.cpp; C-ABI sr_store_set_*).
class StoreSet {
 public:
  StoreSet(int dim, int dtype, const int* devices, int n_dev);
  int dim() const { return dim_; }
  int shards() const { return (int)shards_.size(); }
  int64_t rows() const;
  int64_t live() const;
  void add_host(const float* vecs, int64_t n, int64_t* out_rows);
  void remove(const int64_t* rows, int64_t n);
  void get(const int64_t* rows, int64_t n, float* out);
  void search_host(const float* q, int B, int k, float* out_dist, int64_t* out_rows,
                   const uint8_t* allow = nullptr, int64_t mask_key = 0);
  void set_scan_dtype(int dtype);

  std::mutex mu;

 private:
  // rows -> per-shard local rows and their positions in the argument
  void split(const int64_t* rows, int64_t n, std::vector<std::vector<int64_t>>& local,
             std::vector<std::vector<int64_t>>& pos) const;
  int dim_;
  std::vector<std::unique_ptr<Store>> shards_;
  std::vector<std::vector<int64_t>> tables_;  // per shard: local row -> global row
  std::vector<int32_t> shard_of_;             // global row -> shard
  std::vector<int64_t> local_of_;             // global row -> local row
};

// ------------------------------------------------------------------------------------------------
class Encoder {
 public:
  Encoder(const sr_encoder_config& cfg, int device);
  ~Encoder();

  void set_weight(const std::string& name, const float* data, int64_t numel);
  std::string missing() const;  // empty when every weight is set

  // mode 0: pooled embeddings to `out` (dtype/ld_out); mode 1: classifier logits (fp32).
  void forward_dev(const int32_t* ids, const int32_t* mask, const int32_t* types, int B, int S,
                   int mode, int pool, void* out, int out_dtype, int ld_out, hipStream_t s);
  void forward_host(const int32_t* ids, const int32_t* mask, const int32_t* types, int B, int S,
                    int mode, int pool, float* out);

  const sr_encoder_config& config() const { return cfg_; }
  // fp8 modes (LN-folded encoders): 1 = FFN (FFN1 stores e4m3(2 GELU), FFN2 on the block-scaled
  // fp8 MFMA with an e4m3 copy of its weight); 2 = also FFN1 and the QKV GEMMs of layers >= 1 on
  // e4m3 copies of the residual sums written by the *_STATS epilogues; 0 = fp16
  void set_fp8(int mode);
  int device() const { return device_; }
  std::mutex mu;

 private:
  struct Target {
    void* ptr;
    int64_t numel;
    bool f16;
    float* master = nullptr;  // fp32 copy kept for LayerNorm folding (QKV / FFN1 weights)
    int64_t split_k = 0;      // split weights: rows of split_k fp32 -> [fp16 hi | fp16 lo]
  };
  struct Layer {
    DevBuf wqkv, bqkv, wo, bo, ln1g, ln1b, w1, b1, w2, b2, ln2g, ln2b;
    // LayerNorm folding (fp16 residual stream): fp32 masters and the folded copies
    DevBuf wqkv32, w132, wqkv_f, cqkv, dqkv, w1_f, c1, d1, bo_f, b2_f, w2h;
    // fp8 modes: e4m3 copies of w2h (FFN) and of the folded w1_f / wqkv_f (all), their per-row
    // exponents and the folded column sums of the quantised weights
    DevBuf w2_8, w2e, w1_8, w1e, c1_8, wqkv8, wqkve, cqkv8;
    DevBuf wo_8, woe;  // fp8 mode 5: e4m3 rows of the O-projection weight + their E8M0 exponents
    // K/V-free CLS-only last layer: block-diagonal K / V weights, zero bias (H*D)
    DevBuf wk_bd, wv_bd, zb;
  };
  bool fold_enabled() const;
  void prepare_fold(hipStream_t s);
  void begin(hipStream_t s) { SR_HIP(hipStreamWaitEvent(s, done_, 0)); }
  void end(hipStream_t s) { SR_HIP(hipEventRecord(done_, s)); }
  void register_target(const std::string& name, DevBuf& buf, int64_t numel, bool f16,
                       int64_t offset_elems = 0, int64_t total_elems = -1, int64_t split_k = 0);
  void ensure_ws(int64_t tokens, int B);

  sr_encoder_config cfg_;
  int device_;
  hipStream_t stream_ = nullptr;
  hipEvent_t done_ = nullptr;
  int64_t max_tokens_;
  DevBuf wemb_, pemb_, temb_, embg_, embb_, wc_, bc_, wout_, bout_;
  std::vector<Layer> layers_;
  std::map<std::string, Target> targets_;
  std::map<std::string, bool> is_set_;
  // workspace
  DevBuf ids_, mask_, types_, pos_, h16_, h32_, qkv_, ctx_, y32_, ffn_, clst_, hostio_;
  DevBuf statA_, statB_, mrA_, mrB_;  // per-row LayerNorm partials / (mu, rstd) (folded path)
  bool fold_ready_ = false;  // folded weights match the current weights
  int fp8_ = 0;
  // split weights (fp32-residual encoders, i.e. the embedders): each layer matrix W is held as
  // [fp16(W) | fp16(W - fp16(W))] and the GEMMs run K = 2 K_x over the repeated activation, which
  // removes the fp16 weight rounding (~9e-4 of the 1.1e-3 embedding error of 24-layer bge-m3)
  bool split_ = false;
  DevBuf u8_;  // e4m3 copy of the residual sums (fp8 modes 2 / 3) or normalised rows (mode 4)
  DevBuf unit_mr_;  // (mu, rstd) = (0, 1): fp8 mode 4 QKV statistics (stat_ld 0)
  static constexpr size_t kChunkWsBytes = size_t(64) << 20;
  DevBuf chunk_ws_;  // split-K partial tiles of the unfolded (embedder) GEMMs at short M
  int64_t ws_tokens_ = 0;
};

// ------------------------------------------------------------------------------------------------
// BM25 lexical index over the rows of a store (k_lex.hip).
class LexIndex {
 public:
  LexIndex(int device, float k1, float b);
  ~LexIndex();

  // n documents: terms[off[i] .. off[i+1]) distinct term ids with frequencies tf, length dl[i]
  void add(const int64_t* off, const int32_t* terms, const int32_t* tf, const int32_t* dl,
           int64_t n, int64_t* first_row);
  void remove(const int64_t* rows, int64_t n);
  void compact(int64_t* old_to_new);
  // query b: terms qterms[qoff[b] .. qoff[b+1]) (repeats count); outputs on the device (search_dev,
  // on stream s) or the host
  void search_dev(const int64_t* qoff, const int32_t* qterms, int B, int k, const uint8_t* allow,
                  int64_t mask_key, float* out_score, int64_t* out_rows, hipStream_t s,
                  const sr_lex_global* glob = nullptr, int64_t row_offset = 0,
                  uint32_t* out_fixed = nullptr);
  // device-resident queries: tok [B, Lq] int32 (row stride Lq), qlen [B] int32, both in HBM.
  // query_stats_dev writes [n_live, sum_dl, df of every (query, position)] (2 + B Lq int64, the
  // vector a row-sharded corpus sums over its shards); search_tok_dev scores with those summed
  // statistics (gstats, device) or this index's own (null).  No host synchronisation.
  void query_stats_dev(const int32_t* tok, const int32_t* qlen, int B, int Lq, int64_t* out,
                       hipStream_t s);
  void search_tok_dev(const int32_t* tok, const int32_t* qlen, int B, int Lq, int k,
                      const int64_t* gstats, float* out_score, int64_t* out_rows, hipStream_t s,
                      int64_t row_offset);
  void totals(int64_t* n_live, int64_t* sum_dl) const;
  void df(const int32_t* terms, int n, int64_t* out);
  void search_host(const int64_t* qoff, const int32_t* qterms, int B, int k, const uint8_t* allow,
                   int64_t mask_key, float* out_score, int64_t* out_rows,
                   const sr_lex_global* glob = nullptr, uint32_t* out_fixed = nullptr);
  void stats(int64_t* rows, int64_t* live, int64_t* postings, int64_t* vocab, double* avgdl);
  void save(const char* path);
  static LexIndex* load(const char* path, int device);
  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }
  void begin(hipStream_t s) { SR_HIP(hipStreamWaitEvent(s, done_, 0)); }
  void end(hipStream_t s) { SR_HIP(hipEventRecord(done_, s)); }

  std::mutex mu;

 private:
  void rebuild(hipStream_t s);
  const uint8_t* eligibility(const uint8_t* allow, int64_t mask_key, hipStream_t s);
  static float idf(int64_t df, int64_t n_live);
  static float avgdl(int64_t sum_dl, int64_t n_live);
  void forward(std::vector<int32_t>& fterm, std::vector<uint64_t>& fval);
  void load_rows(const std::vector<int32_t>& dl, const std::vector<uint8_t>& live,
                 const std::vector<int32_t>& ft, const std::vector<uint64_t>& fv);

  int device_;
  float k1_, b_;
  hipStream_t stream_ = nullptr;
  hipEvent_t done_ = nullptr;
  int64_t rows_ = 0, live_n_ = 0, P_ = 0, vocab_ = 0, nnz_ = 0, sum_dl_ = 0, max_df_ = 0;
  bool dirty_ = true;
  // device: forward index, per-row data, inverted index, workspaces
  DevBuf fterm_, fval_, dlen_, live_, off_, post_, ws_, out_, mask_, caps_;
  // host mirrors
  std::vector<int32_t> dl_host_, df_host_;
  std::vector<uint8_t> live_host_;
  std::vector<int64_t> off_host_;
  int64_t version_ = 0, mask_key_ = 0, mask_version_ = -1;
};

}  // namespace sr
