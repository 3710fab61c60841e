// C-ABI entry points (include/super_rag_mi355x.h): argument checks, exception -> error-code
// mapping, per-object locking, and the HIP-event profiler.
#include <algorithm>
#include <map>
#include <mutex>
#include <vector>

#include "sr_kernels.h"
#include "sr_runtime.h"

struct sr_store {
  sr::Store* impl;
};
struct sr_encoder {
  sr::Encoder* impl;
};
struct sr_lex {
  sr::LexIndex* impl;
};
struct sr_store_set {
  sr::StoreSet* impl;
};

namespace sr {

static thread_local std::string t_last_error;
void set_last_error(const std::string& msg) { t_last_error = msg; }

// ---- profiler --------------------------------------------------------------------------------
namespace {
struct ProfRecord {
  std::string name;
  hipEvent_t ev0, ev1;
  double flops, bytes;
};
struct ProfAgg {
  int64_t launches = 0;
  double ms = 0, flops = 0, bytes = 0;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRecord> g_prof_pending;
std::vector<hipEvent_t> g_event_pool;
std::map<std::string, ProfAgg> g_prof_agg;

hipEvent_t take_event() {
  if (!g_event_pool.empty()) {
    hipEvent_t e = g_event_pool.back();
    g_event_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  SR_HIP(hipEventCreate(&e));
  return e;
}

void drain_pending_locked() {
  for (auto& r : g_prof_pending) {
    (void)hipEventSynchronize(r.ev1);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, r.ev0, r.ev1) == hipSuccess) {
      ProfAgg& a = g_prof_agg[r.name];
      a.launches += 1;
      a.ms += ms;
      a.flops += r.flops;
      a.bytes += r.bytes;
    }
    g_event_pool.push_back(r.ev0);
    g_event_pool.push_back(r.ev1);
  }
  g_prof_pending.clear();
}
}  // namespace

ProfScope::ProfScope(const char* n, hipStream_t s, double f, double b)
    : name(n), flops(f), bytes(b), stream(s) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (!g_prof_on) return;
  ev0 = take_event();
  ev1 = take_event();
  if (hipEventRecord(ev0, stream) != hipSuccess) {
    g_event_pool.push_back(ev0);
    g_event_pool.push_back(ev1);
    ev0 = ev1 = nullptr;
  }
}

ProfScope::~ProfScope() {
  if (!ev0) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  if (hipEventRecord(ev1, stream) == hipSuccess) {
    g_prof_pending.push_back(ProfRecord{name, ev0, ev1, flops, bytes});
    if (g_prof_pending.size() > 65536) drain_pending_locked();
  } else {
    g_event_pool.push_back(ev0);
    g_event_pool.push_back(ev1);
  }
}

}  // namespace sr

#define SR_API_BEGIN try {
#define SR_API_END                           \
  return SR_OK;                              \
  }                                          \
  catch (const sr::Error& e) {               \
    sr::set_last_error(e.what());            \
    return e.code;                           \
  }                                          \
  catch (const std::bad_alloc&) {            \
    sr::set_last_error("host out of memory"); \
    return SR_ERR_OOM;                       \
  }                                          \
  catch (const std::exception& e) {          \
    sr::set_last_error(e.what());            \
    return SR_ERR_INVALID;                   \
  }

#define SR_NONNULL(p)                                                   \
  do {                                                                  \
    if (!(p)) throw sr::Error(SR_ERR_INVALID, "null argument: " #p);    \
  } while (0)

extern "C" {

const char* sr_last_error(void) { return sr::t_last_error.c_str(); }
int sr_version(void) { return 100; }

int sr_device_count(int* out) {
  SR_API_BEGIN
  SR_NONNULL(out);
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *out = n;
  SR_API_END
}

int sr_memcpy(void* dst, const void* src, int64_t bytes, int kind, int device) {
  SR_API_BEGIN
  SR_NONNULL(dst);
  SR_NONNULL(src);
  sr::DeviceGuard g(device);
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                          : kind == 1 ? hipMemcpyDeviceToHost
                                      : hipMemcpyDeviceToDevice;
  SR_HIP(hipMemcpy(dst, src, (size_t)bytes, k));
  SR_API_END
}

// ---- store -----------------------------------------------------------------------------------
int sr_store_create(int dim, int device, int64_t initial_capacity, sr_store** out) {
  SR_API_BEGIN
  SR_NONNULL(out);
  *out = nullptr;
  auto* s = new sr_store{new sr::Store(dim, device, initial_capacity)};
  *out = s;
  SR_API_END
}

int sr_store_add(sr_store* s, const float* vecs, int64_t n, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->add_host(vecs, n, out_rows);
  SR_API_END
}

int sr_store_add_dev(sr_store* s, const void* vecs, int dtype, int64_t n, int64_t* first_row,
                     void* stream) {
  SR_API_BEGIN
  SR_NONNULL(s);
  SR_NONNULL(vecs);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  const int64_t first = s->impl->add_dev(vecs, dtype, n, reinterpret_cast<hipStream_t>(stream));
  if (first_row) *first_row = first;
  SR_API_END
}

int sr_store_remove(sr_store* s, const int64_t* rows, int64_t n) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->remove(rows, n);
  SR_API_END
}

int sr_store_count(sr_store* s, int64_t* n_rows, int64_t* n_live) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  if (n_rows) *n_rows = s->impl->rows();
  if (n_live) *n_live = s->impl->live();
  SR_API_END
}

int sr_store_dim(sr_store* s, int* dim) {
  SR_API_BEGIN
  SR_NONNULL(s);
  SR_NONNULL(dim);
  *dim = s->impl->dim();
  SR_API_END
}

int sr_store_get(sr_store* s, const int64_t* rows, int64_t n, float* out) {
  SR_API_BEGIN
  SR_NONNULL(s);
  if (n > 0) {
    SR_NONNULL(rows);
    SR_NONNULL(out);
  }
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->get(rows, n, out);
  SR_API_END
}

int sr_store_search(sr_store* s, const float* q, int B, int k, float* out_dist, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->search_host(q, B, k, out_dist, out_rows);
  SR_API_END
}

int sr_store_search_masked(sr_store* s, const float* q, int B, int k, const uint8_t* allow,
                           int64_t mask_key, float* out_dist, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(s);
  SR_NONNULL(allow);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->search_host(q, B, k, out_dist, out_rows, allow, mask_key);
  SR_API_END
}

int sr_store_search_sim(sr_store* s, const float* q, int B, int k, const uint8_t* allow,
                        int64_t mask_key, float* out_sim, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->search_host(q, B, k, out_sim, out_rows, allow, allow ? mask_key : 0, true);
  SR_API_END
}

int sr_store_search_dev(sr_store* s, const void* q, int q_dtype, int B, int k, float* out_sim,
                        int64_t* out_rows, int64_t row_offset, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(s);
  if (B > 0) {
    SR_NONNULL(q);
    SR_NONNULL(out_sim);
    SR_NONNULL(out_rows);
  }
  SR_CHECK(q_dtype == SR_DTYPE_F32 || q_dtype == SR_DTYPE_F16, "search: q dtype must be f32/f16");
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->search_dev(q, q_dtype, B, k, out_sim, out_rows, row_offset,
                      reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_store_set_scan_dtype(sr_store* s, int dtype) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->set_scan_dtype(dtype);
  SR_API_END
}

int sr_store_save(sr_store* s, const char* path) {
  SR_API_BEGIN
  SR_NONNULL(s);
  SR_NONNULL(path);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->save(path);
  SR_API_END
}

int sr_store_load(const char* path, int device, sr_store** out) {
  SR_API_BEGIN
  SR_NONNULL(path);
  SR_NONNULL(out);
  *out = nullptr;
  sr::Store* st = sr::Store::load(path, device);
  *out = new sr_store{st};
  SR_API_END
}

int sr_store_compact(sr_store* s, int64_t* old_to_new) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->compact(old_to_new);
  SR_API_END
}

void sr_store_destroy(sr_store* s) {
  if (!s) return;
  delete s->impl;
  delete s;
}

// ---- multi-device collection (SURVEY 8(b) sr_store_create(dim, dtype, devices, n_dev)) ---------
int sr_store_set_create(int dim, int dtype, const int* devices, int n_dev, sr_store_set** out) {
  SR_API_BEGIN
  SR_NONNULL(out);
  SR_NONNULL(devices);
  *out = nullptr;
  *out = new sr_store_set{new sr::StoreSet(dim, dtype, devices, n_dev)};
  SR_API_END
}

int sr_store_set_add(sr_store_set* s, const float* vecs, int64_t n, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->add_host(vecs, n, out_rows);
  SR_API_END
}

int sr_store_set_remove(sr_store_set* s, const int64_t* rows, int64_t n) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->remove(rows, n);
  SR_API_END
}

int sr_store_set_count(sr_store_set* s, int64_t* n_rows, int64_t* n_live, int* n_shards) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  if (n_rows) *n_rows = s->impl->rows();
  if (n_live) *n_live = s->impl->live();
  if (n_shards) *n_shards = s->impl->shards();
  SR_API_END
}

int sr_store_set_get(sr_store_set* s, const int64_t* rows, int64_t n, float* out) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->get(rows, n, out);
  SR_API_END
}

int sr_store_set_search(sr_store_set* s, const float* q, int B, int k, const uint8_t* allow,
                        int64_t mask_key, float* out_dist, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->search_host(q, B, k, out_dist, out_rows, allow, allow ? mask_key : 0);
  SR_API_END
}

int sr_store_set_set_scan_dtype(sr_store_set* s, int dtype) {
  SR_API_BEGIN
  SR_NONNULL(s);
  std::lock_guard<std::mutex> lk(s->impl->mu);
  s->impl->set_scan_dtype(dtype);
  SR_API_END
}

void sr_store_set_destroy(sr_store_set* s) {
  if (!s) return;
  delete s->impl;
  delete s;
}

int sr_topk_merge_dev(const float* sims, const int64_t* rows, int P, int B, int k, int k_out,
                      float* out_sim, int64_t* out_rows, int device, void* stream) {
  SR_API_BEGIN
  SR_CHECK(P >= 1 && B >= 0 && k >= 1, "merge: bad shape");
  if (B > 0) {
    SR_NONNULL(sims);
    SR_NONNULL(rows);
    SR_NONNULL(out_sim);
    SR_NONNULL(out_rows);
  }
  sr::DeviceGuard g(device);
  sr::launch_topk_merge(sims, rows, P, B, k, k_out, out_sim, out_rows,
                        reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

// ---- encoder ---------------------------------------------------------------------------------
// ---- lexical index / hybrid ------------------------------------------------------------------
int sr_lex_create(int device, float k1, float b, sr_lex** out) {
  SR_API_BEGIN
  SR_NONNULL(out);
  *out = nullptr;
  *out = new sr_lex{new sr::LexIndex(device, k1, b)};
  SR_API_END
}

int sr_lex_add(sr_lex* x, const int64_t* off, const int32_t* terms, const int32_t* tf,
               const int32_t* dl, int64_t n, int64_t* first_row) {
  SR_API_BEGIN
  SR_NONNULL(x);
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->add(off, terms, tf, dl, n, first_row);
  SR_API_END
}

int sr_lex_remove(sr_lex* x, const int64_t* rows, int64_t n) {
  SR_API_BEGIN
  SR_NONNULL(x);
  if (n > 0) SR_NONNULL(rows);
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->remove(rows, n);
  SR_API_END
}

int sr_lex_stats(sr_lex* x, int64_t* n_rows, int64_t* n_live, int64_t* n_postings, int64_t* vocab,
                 double* avgdl) {
  SR_API_BEGIN
  SR_NONNULL(x);
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->stats(n_rows, n_live, n_postings, vocab, avgdl);
  SR_API_END
}

int sr_lex_search(sr_lex* x, const int64_t* qoff, const int32_t* qterms, int B, int k,
                  const uint8_t* allow, int64_t mask_key, float* out_score, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(x);
  if (B > 0) {
    SR_NONNULL(qoff);
    SR_NONNULL(out_score);
    SR_NONNULL(out_rows);
    if (qoff[B] > 0) SR_NONNULL(qterms);
  }
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->search_host(qoff, qterms, B, k, allow, mask_key, out_score, out_rows);
  SR_API_END
}

int sr_lex_search_global(sr_lex* x, const int64_t* qoff, const int32_t* qterms, int B, int k,
                         const uint8_t* allow, int64_t mask_key, const sr_lex_global* global,
                         float* out_score, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(x);
  if (B > 0) {
    SR_NONNULL(qoff);
    SR_NONNULL(out_score);
    SR_NONNULL(out_rows);
    if (qoff[B] > 0) SR_NONNULL(qterms);
  }
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->search_host(qoff, qterms, B, k, allow, mask_key, out_score, out_rows, global);
  SR_API_END
}

int sr_lex_search_global_fixed(sr_lex* x, const int64_t* qoff, const int32_t* qterms, int B, int k,
                               const uint8_t* allow, int64_t mask_key, const sr_lex_global* global,
                               float* out_score, int64_t* out_rows, uint32_t* out_fixed) {
  SR_API_BEGIN
  SR_NONNULL(x);
  if (B > 0) {
    SR_NONNULL(qoff);
    SR_NONNULL(out_score);
    SR_NONNULL(out_rows);
    SR_NONNULL(out_fixed);
    if (qoff[B] > 0) SR_NONNULL(qterms);
  }
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->search_host(qoff, qterms, B, k, allow, mask_key, out_score, out_rows, global, out_fixed);
  SR_API_END
}

int sr_lex_totals(sr_lex* x, int64_t* n_live, int64_t* sum_dl) {
  SR_API_BEGIN
  SR_NONNULL(x);
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->totals(n_live, sum_dl);
  SR_API_END
}

int sr_lex_df(sr_lex* x, const int32_t* terms, int n, int64_t* out_df) {
  SR_API_BEGIN
  SR_NONNULL(x);
  SR_CHECK(n >= 0, "lex.df: negative count");
  if (n > 0) {
    SR_NONNULL(terms);
    SR_NONNULL(out_df);
  }
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->df(terms, n, out_df);
  SR_API_END
}

int sr_lex_search_dev(sr_lex* x, const int64_t* qoff, const int32_t* qterms, int B, int k,
                      const sr_lex_global* global, float* out_score, int64_t* out_rows,
                      int64_t row_offset, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(x);
  if (B > 0) {
    SR_NONNULL(qoff);
    SR_NONNULL(out_score);
    SR_NONNULL(out_rows);
    if (qoff[B] > 0) SR_NONNULL(qterms);
  }
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->search_dev(qoff, qterms, B, k, nullptr, 0, out_score, out_rows,
                      reinterpret_cast<hipStream_t>(stream), global, row_offset);
  SR_API_END
}

int sr_lex_query_stats_dev(sr_lex* x, const int32_t* tok, const int32_t* qlen, int B, int Lq,
                           int64_t* out_stats, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(x);
  SR_NONNULL(out_stats);
  SR_CHECK(B >= 0 && Lq >= 0, "lex.query_stats: negative shape");
  if ((int64_t)B * Lq > 0) {
    SR_NONNULL(tok);
    SR_NONNULL(qlen);
  }
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->query_stats_dev(tok, qlen, B, Lq, out_stats, reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_lex_search_tok_dev(sr_lex* x, const int32_t* tok, const int32_t* qlen, int B, int Lq, int k,
                          const int64_t* gstats, float* out_score, int64_t* out_rows,
                          int64_t row_offset, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(x);
  if (B > 0) {
    SR_NONNULL(qlen);
    SR_NONNULL(out_score);
    SR_NONNULL(out_rows);
    if (Lq > 0) SR_NONNULL(tok);
  }
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->search_tok_dev(tok, qlen, B, Lq, k, gstats, out_score, out_rows,
                          reinterpret_cast<hipStream_t>(stream), row_offset);
  SR_API_END
}

int sr_lex_save(sr_lex* x, const char* path) {
  SR_API_BEGIN
  SR_NONNULL(x);
  SR_NONNULL(path);
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->save(path);
  SR_API_END
}

int sr_lex_load(const char* path, int device, sr_lex** out) {
  SR_API_BEGIN
  SR_NONNULL(path);
  SR_NONNULL(out);
  *out = nullptr;
  sr::LexIndex* li = sr::LexIndex::load(path, device);
  *out = new sr_lex{li};
  SR_API_END
}

int sr_lex_compact(sr_lex* x, int64_t* old_to_new) {
  SR_API_BEGIN
  SR_NONNULL(x);
  std::lock_guard<std::mutex> lk(x->impl->mu);
  x->impl->compact(old_to_new);
  SR_API_END
}

void sr_lex_destroy(sr_lex* x) {
  if (!x) return;
  delete x->impl;
  delete x;
}

int sr_rrf_fuse(const int64_t* rows_a, int ka, const int64_t* rows_b, int kb, int B,
                int rank_const, double min_score, int k_out, double* out_score,
                int64_t* out_rows, int device) {
  SR_API_BEGIN
  SR_CHECK(B >= 0, "rrf: negative batch");
  if (B == 0) return SR_OK;
  SR_NONNULL(out_score);
  SR_NONNULL(out_rows);
  if (ka > 0) SR_NONNULL(rows_a);
  if (kb > 0) SR_NONNULL(rows_b);
  sr::DeviceGuard g(device);
  const size_t ba = (size_t)B * ka * 8, bb = (size_t)B * kb * 8, bo = (size_t)B * k_out * 8;
  sr::DevBuf ws;
  ws.reserve(ba + bb + 2 * bo + 8);
  char* w = ws.as<char>();
  int64_t* da = reinterpret_cast<int64_t*>(w);
  int64_t* db = reinterpret_cast<int64_t*>(w + ba);
  double* ds = reinterpret_cast<double*>(w + ba + bb);
  int64_t* dr = reinterpret_cast<int64_t*>(w + ba + bb + bo);
  hipStream_t st = nullptr;
  SR_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  try {
    if (ba) SR_HIP(hipMemcpyAsync(da, rows_a, ba, hipMemcpyHostToDevice, st));
    if (bb) SR_HIP(hipMemcpyAsync(db, rows_b, bb, hipMemcpyHostToDevice, st));
    sr::launch_rrf_fuse(da, ka, db, kb, B, rank_const, min_score, k_out, ds, dr, st);
    SR_HIP(hipMemcpyAsync(out_score, ds, bo, hipMemcpyDeviceToHost, st));
    SR_HIP(hipMemcpyAsync(out_rows, dr, bo, hipMemcpyDeviceToHost, st));
    SR_HIP(hipStreamSynchronize(st));
  } catch (...) {
    (void)hipStreamSynchronize(st);
    (void)hipStreamDestroy(st);
    throw;
  }
  SR_HIP(hipStreamDestroy(st));
  SR_API_END
}

int sr_rrf_fuse_dev(const int64_t* rows_a, int ka, const int64_t* rows_b, int kb, int B,
                    int rank_const, double min_score, int k_out, double* out_score,
                    int64_t* out_rows, int device, void* stream) {
  SR_API_BEGIN
  SR_CHECK(B >= 0, "rrf: negative batch");
  if (B == 0) return SR_OK;
  SR_NONNULL(out_score);
  SR_NONNULL(out_rows);
  sr::DeviceGuard g(device);
  sr::launch_rrf_fuse(rows_a, ka, rows_b, kb, B, rank_const, min_score, k_out, out_score, out_rows,
                      reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_hybrid_search(sr_store* s, sr_lex* x, const float* q, const int64_t* qoff,
                     const int32_t* qterms, int B, int k, int k_each, int rank_const,
                     double min_score, const uint8_t* allow, int64_t mask_key,
                     double* out_score, int64_t* out_rows) {
  SR_API_BEGIN
  SR_NONNULL(s);
  SR_NONNULL(x);
  SR_CHECK(B >= 0, "hybrid: negative batch");
  if (B == 0) return SR_OK;
  SR_NONNULL(q);
  SR_NONNULL(qoff);
  SR_NONNULL(out_score);
  SR_NONNULL(out_rows);
  SR_CHECK(k_each >= 1 && k_each <= SR_MAX_TOPK, "hybrid: k_each must be in [1, 1024]");
  SR_CHECK(k >= 1 && k <= 2 * k_each, "hybrid: k must be in [1, 2 * k_each]");
  std::scoped_lock lk(s->impl->mu, x->impl->mu);
  sr::Store& st = *s->impl;
  sr::LexIndex& lx = *x->impl;
  SR_CHECK(st.device() == lx.device(), "hybrid: store and lexical index on different devices");
  int64_t lrows = 0;
  lx.stats(&lrows, nullptr, nullptr, nullptr, nullptr);
  SR_CHECK(lrows == st.rows(), "hybrid: store and lexical index hold different row counts");
  sr::DeviceGuard g(st.device());
  hipStream_t sm = lx.stream();
  const size_t bq = (size_t)B * st.dim() * 4, be = (size_t)B * k_each * 8, bo = (size_t)B * k * 8;
  sr::DevBuf ws;
  ws.reserve(bq + 4 * be + 2 * bo + 64);
  char* w = ws.as<char>();
  float* dq = reinterpret_cast<float*>(w);
  float* dsim = reinterpret_cast<float*>(w + bq);
  int64_t* drow = reinterpret_cast<int64_t*>(w + bq + be);
  float* lsc = reinterpret_cast<float*>(w + bq + 2 * be);
  int64_t* lrow = reinterpret_cast<int64_t*>(w + bq + 3 * be);
  double* os = reinterpret_cast<double*>(w + bq + 4 * be);
  int64_t* orow = reinterpret_cast<int64_t*>(w + bq + 4 * be + bo);
  const uint8_t* elig = st.eligibility(allow, mask_key);
  lx.begin(sm);
  SR_HIP(hipMemcpyAsync(dq, q, bq, hipMemcpyHostToDevice, sm));
  st.search_dev(dq, SR_DTYPE_F32, B, k_each, dsim, drow, 0, sm, elig);
  lx.search_dev(qoff, qterms, B, k_each, allow, mask_key, lsc, lrow, sm);
  sr::launch_rrf_fuse(drow, k_each, lrow, k_each, B, rank_const, min_score, k, os, orow, sm);
  SR_HIP(hipMemcpyAsync(out_score, os, bo, hipMemcpyDeviceToHost, sm));
  SR_HIP(hipMemcpyAsync(out_rows, orow, bo, hipMemcpyDeviceToHost, sm));
  lx.end(sm);
  SR_HIP(hipStreamSynchronize(sm));
  SR_API_END
}

int sr_encoder_create(const sr_encoder_config* cfg, int device, sr_encoder** out) {
  SR_API_BEGIN
  SR_NONNULL(cfg);
  SR_NONNULL(out);
  *out = nullptr;
  auto* e = new sr_encoder{new sr::Encoder(*cfg, device)};
  *out = e;
  SR_API_END
}

int sr_encoder_set_weight(sr_encoder* e, const char* name, const float* data, int64_t numel) {
  SR_API_BEGIN
  SR_NONNULL(e);
  SR_NONNULL(name);
  std::lock_guard<std::mutex> lk(e->impl->mu);
  e->impl->set_weight(name, data, numel);
  SR_API_END
}

int sr_encoder_ready(sr_encoder* e) {
  SR_API_BEGIN
  SR_NONNULL(e);
  std::lock_guard<std::mutex> lk(e->impl->mu);
  const std::string m = e->impl->missing();
  if (!m.empty()) throw sr::Error(SR_ERR_STATE, "encoder: weight not set: " + m);
  SR_API_END
}

int sr_encoder_forward(sr_encoder* e, const int32_t* ids, const int32_t* mask,
                       const int32_t* type_ids, int B, int S, int pool, float* out) {
  SR_API_BEGIN
  SR_NONNULL(e);
  std::lock_guard<std::mutex> lk(e->impl->mu);
  e->impl->forward_host(ids, mask, type_ids, B, S, 0, pool, out);
  SR_API_END
}

int sr_encoder_forward_dev(sr_encoder* e, const int32_t* ids, const int32_t* mask,
                           const int32_t* type_ids, int B, int S, int pool, void* out,
                           int out_dtype, int ld_out, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(e);
  if (B > 0) {
    SR_NONNULL(ids);
    SR_NONNULL(mask);
    SR_NONNULL(out);
  }
  std::lock_guard<std::mutex> lk(e->impl->mu);
  e->impl->forward_dev(ids, mask, type_ids, B, S, 0, pool, out, out_dtype, ld_out,
                       reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_cross_score(sr_encoder* e, const int32_t* ids, const int32_t* mask, const int32_t* type_ids,
                   int P, int S, float* out_logits) {
  SR_API_BEGIN
  SR_NONNULL(e);
  std::lock_guard<std::mutex> lk(e->impl->mu);
  e->impl->forward_host(ids, mask, type_ids, P, S, 1, SR_POOL_CLS, out_logits);
  SR_API_END
}

int sr_cross_score_dev(sr_encoder* e, const int32_t* ids, const int32_t* mask,
                       const int32_t* type_ids, int P, int S, float* out_logits, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(e);
  if (P > 0) {
    SR_NONNULL(ids);
    SR_NONNULL(mask);
    SR_NONNULL(out_logits);
  }
  std::lock_guard<std::mutex> lk(e->impl->mu);
  e->impl->forward_dev(ids, mask, type_ids, P, S, 1, SR_POOL_CLS, out_logits, SR_DTYPE_F32,
                       e->impl->config().hidden, reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_encoder_set_fp8(sr_encoder* e, int mode) {
  SR_API_BEGIN
  SR_NONNULL(e);
  std::lock_guard<std::mutex> lk(e->impl->mu);
  e->impl->set_fp8(mode);
  SR_API_END
}

void sr_encoder_destroy(sr_encoder* e) {
  if (!e) return;
  delete e->impl;
  delete e;
}

// ---- pipeline helpers ------------------------------------------------------------------------
int sr_build_pairs_dev(const int32_t* q_tok, const int32_t* q_len, int lq_max, const int32_t* p_tok,
                       const int32_t* p_len, int lp_max, const int64_t* cand_rows, int B, int K,
                       int S, int style, int bos_id, int eos_id, int pad_id, int32_t* out_ids,
                       int32_t* out_mask, int32_t* out_type, int device, void* stream) {
  SR_API_BEGIN
  SR_CHECK(B >= 0 && K >= 1 && lq_max >= 1 && lp_max >= 1, "build_pairs: bad shape");
  if (B > 0) {
    SR_NONNULL(q_tok);
    SR_NONNULL(q_len);
    SR_NONNULL(p_tok);
    SR_NONNULL(p_len);
    SR_NONNULL(cand_rows);
    SR_NONNULL(out_ids);
    SR_NONNULL(out_mask);
  }
  sr::DeviceGuard g(device);
  sr::launch_build_pairs(q_tok, q_len, lq_max, p_tok, p_len, lp_max, cand_rows, B, K, S, style,
                         bos_id, eos_id, pad_id, out_ids, out_mask, out_type,
                         reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_rerank_select_dev(const float* logits, int B, int K, int k_out, int32_t* out_index,
                         int device, void* stream) {
  SR_API_BEGIN
  if (B > 0) {
    SR_NONNULL(logits);
    SR_NONNULL(out_index);
  }
  sr::DeviceGuard g(device);
  sr::launch_rerank_select(logits, B, K, k_out, out_index, reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

// ---- diagnostics (libsrmi_diag.so only: include/super_rag_mi355x_diag.h) --------------------
#if SR_WITH_DIAG
int sr_diag_gemm(int variant, int epi, const void* X, int64_t lda, const void* W, const float* bias,
                 const void* R, int64_t ldr, void* Y, int64_t ldy, int M, int N, int K, int device,
                 void* stream) {
  SR_API_BEGIN
  SR_NONNULL(X);
  SR_NONNULL(W);
  SR_NONNULL(bias);
  SR_NONNULL(Y);
  SR_CHECK(epi >= 0 && epi <= 4, "diag_gemm: epi must be 0..4");
  SR_CHECK((epi != 2 && epi != 4) || R, "diag_gemm: residual epilogue needs R");
  sr::DeviceGuard g(device);
  sr::LnFold lf;  // variant | 0x100: split weights, W = [hi | lo] with K = 2 x_k
  if (variant >= 0 && (variant & 0x100)) {
    SR_CHECK(K % 128 == 0, "diag_gemm: split weights need K % 128 == 0");
    lf.x_k = K / 2;
    variant &= 0xff;
  }
  sr::launch_gemm_variant(variant, epi, reinterpret_cast<const sr::half_t*>(X), lda,
                          reinterpret_cast<const sr::half_t*>(W), bias, R, ldr, Y, ldy, M, N, K,
                          reinterpret_cast<hipStream_t>(stream), &lf);
  SR_API_END
}

int sr_diag_gemm_stats(const void* X, int64_t lda, const void* W, const float* bias, const void* R,
                       int64_t ldr, void* Y, int64_t ldy, int M, int N, int K, float* stat_out,
                       int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(X);
  SR_NONNULL(W);
  SR_NONNULL(bias);
  SR_NONNULL(R);
  SR_NONNULL(Y);
  SR_NONNULL(stat_out);
  SR_CHECK(N % 256 == 0, "diag_gemm_stats: N % 256 == 0");
  sr::DeviceGuard g(device);
  sr::LnFold lf;
  lf.stat_out = stat_out;
  sr::launch_gemm(sr::EPI_RES16_STATS, reinterpret_cast<const sr::half_t*>(X), lda,
                  reinterpret_cast<const sr::half_t*>(W), bias, R, ldr, Y, ldy, M, N, K,
                  reinterpret_cast<hipStream_t>(stream), &lf);
  SR_API_END
}

int sr_diag_gemm_lnr_stats(const void* X, int64_t lda, const void* W, const float* bias, const void* R,
                           int64_t ldr, const float* mr, const float* gamma, void* Y, int64_t ldy, int M,
                           int N, int K, float* stat_out, int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(X);
  SR_NONNULL(W);
  SR_NONNULL(bias);
  SR_NONNULL(R);
  SR_NONNULL(mr);
  SR_NONNULL(gamma);
  SR_NONNULL(Y);
  SR_NONNULL(stat_out);
  SR_CHECK(N % 256 == 0, "diag_gemm_lnr_stats: N % 256 == 0");
  sr::DeviceGuard g(device);
  sr::LnFold lf;
  lf.mr = mr;
  lf.gamma = gamma;
  lf.stat_out = stat_out;
  sr::launch_gemm(sr::EPI_LNR16_STATS, reinterpret_cast<const sr::half_t*>(X), lda,
                  reinterpret_cast<const sr::half_t*>(W), bias, R, ldr, Y, ldy, M, N, K,
                  reinterpret_cast<hipStream_t>(stream), &lf);
  SR_API_END
}

int sr_diag_gemm_stats_y8(int lnr, const void* X, int64_t lda, const void* W, const float* bias,
                          const void* R, int64_t ldr, const float* mr, const float* gamma, void* Y,
                          int64_t ldy, uint8_t* y8, int M, int N, int K, float* stat_out, int device,
                          void* stream) {
  SR_API_BEGIN
  SR_NONNULL(X);
  SR_NONNULL(W);
  SR_NONNULL(bias);
  SR_NONNULL(R);
  SR_NONNULL(Y);
  SR_NONNULL(y8);
  SR_NONNULL(stat_out);
  SR_CHECK(N % 256 == 0, "diag_gemm_stats_y8: N % 256 == 0");
  SR_CHECK(!lnr || (mr && gamma), "diag_gemm_stats_y8: the LNR form needs mr and gamma");
  sr::DeviceGuard g(device);
  sr::LnFold lf;
  lf.mr = lnr ? mr : nullptr;
  lf.gamma = lnr ? gamma : nullptr;
  lf.stat_out = stat_out;
  lf.y8 = y8;
  sr::launch_gemm(lnr ? sr::EPI_LNR16_STATS_Y8 : sr::EPI_RES16_STATS_Y8, reinterpret_cast<const sr::half_t*>(X),
                  lda, reinterpret_cast<const sr::half_t*>(W), bias, R, ldr, Y, ldy, M, N, K,
                  reinterpret_cast<hipStream_t>(stream), &lf);
  SR_API_END
}

int sr_diag_mfma_rate(int f8, int blocks, int iters, float* sink, uint64_t* stamps, int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(sink);
  SR_NONNULL(stamps);
  sr::DeviceGuard g(device);
  sr::launch_mfma_rate(f8, blocks, iters, sink, stamps, reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_diag_gemm_lnr_stats_stamps(const void* X, int64_t lda, const void* W, const float* bias, const void* R,
                                  int64_t ldr, const float* mr, const float* gamma, void* Y, int64_t ldy, int M,
                                  int N, int K, float* stat_out, uint64_t* stamps, int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(X);
  SR_NONNULL(W);
  SR_NONNULL(bias);
  SR_NONNULL(R);
  SR_NONNULL(mr);
  SR_NONNULL(gamma);
  SR_NONNULL(Y);
  SR_NONNULL(stat_out);
  SR_NONNULL(stamps);
  sr::DeviceGuard g(device);
  sr::launch_lnr_stats_stamps(reinterpret_cast<const sr::half_t*>(X), lda, reinterpret_cast<const sr::half_t*>(W),
                              bias, R, ldr, mr, gamma, Y, ldy, M, N, K, stat_out, stamps,
                              reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_diag_ffn1(int diag, int f8, const void* X, int64_t lda, const void* W, const uint8_t* wexp,
                 const float* bias, const float* colsum, const float* mr, void* Y, int64_t ldy, int M,
                 int N, int K, int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(X);
  SR_NONNULL(W);
  SR_NONNULL(bias);
  SR_NONNULL(colsum);
  SR_NONNULL(mr);
  SR_NONNULL(Y);
  SR_CHECK(!f8 || wexp, "diag_ffn1: fp8 needs wexp");
  sr::DeviceGuard g(device);
  sr::launch_ffn1_diag(diag, f8 != 0, X, lda, W, wexp, bias, colsum, mr, Y, ldy, M, N, K,
                       reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_diag_ffn1_stamps(int diag, const void* X, int64_t lda, const void* W, const float* bias,
                        const float* colsum, const float* mr, void* Y, int64_t ldy, int M, int N,
                        int K, uint64_t* stamps, int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(X);
  SR_NONNULL(W);
  SR_NONNULL(bias);
  SR_NONNULL(colsum);
  SR_NONNULL(mr);
  SR_NONNULL(Y);
  SR_NONNULL(stamps);
  sr::DeviceGuard g(device);
  sr::launch_ffn1_diag(diag, false, X, lda, W, nullptr, bias, colsum, mr, Y, ldy, M, N, K,
                       reinterpret_cast<hipStream_t>(stream), stamps);
  SR_API_END
}

int sr_diag_copy(const void* src, void* dst, int64_t bytes, int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(src);
  SR_NONNULL(dst);
  SR_CHECK(bytes >= 0 && bytes % 16 == 0, "diag_copy: bytes must be a non-negative multiple of 16");
  sr::DeviceGuard g(device);
  sr::launch_copy16(src, dst, bytes, reinterpret_cast<hipStream_t>(stream));
  SR_API_END
}

int sr_diag_qkv_attention_stamps(const void* X, int64_t lda, const void* W, const float* bias,
                                 const float* colsum, const float* mr, const int32_t* mask, void* ctx, int B,
                                 int S, int d, int heads, uint64_t* stamps, int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(X);
  SR_NONNULL(W);
  SR_NONNULL(bias);
  SR_NONNULL(colsum);
  SR_NONNULL(mr);
  SR_NONNULL(mask);
  SR_NONNULL(ctx);
  SR_NONNULL(stamps);
  sr::DeviceGuard g(device);
  sr::LnFold lf;
  lf.mr = mr;
  lf.colsum = colsum;
  sr::launch_qkv_attention(sr::EPI_LNF_F16, reinterpret_cast<const sr::half_t*>(X), lda,
                           reinterpret_cast<const sr::half_t*>(W), bias, &lf, mask,
                           reinterpret_cast<sr::half_t*>(ctx), B, S, d, heads,
                           reinterpret_cast<hipStream_t>(stream), nullptr, stamps);
  SR_API_END
}

int sr_diag_attention(int variant, const void* qkv, const int32_t* mask, void* ctx, int B, int S,
                      int Sq, int d, int heads, int device, void* stream) {
  SR_API_BEGIN
  SR_NONNULL(qkv);
  SR_NONNULL(mask);
  SR_NONNULL(ctx);
  SR_CHECK(variant >= -1 && variant <= 3, "diag_attention: variant must be -1 .. 3");
  SR_CHECK(variant < 1 || (heads > 0 && d == 64 * heads && S <= 512),
           "diag_attention: variants 1-3 need head dim 64 and S <= 512");
  sr::DeviceGuard g(device);
  sr::attention_force_variant(variant);
  try {
    sr::launch_attention(reinterpret_cast<const sr::half_t*>(qkv), mask,
                         reinterpret_cast<sr::half_t*>(ctx), B, S, Sq, d, heads,
                         reinterpret_cast<hipStream_t>(stream));
  } catch (...) {
    sr::attention_force_variant(-1);
    throw;
  }
  sr::attention_force_variant(-1);
  SR_API_END
}
#endif  // SR_WITH_DIAG

// ---- profiling -------------------------------------------------------------------------------
int sr_profile_enable(int on) {
  SR_API_BEGIN
  std::lock_guard<std::mutex> lk(sr::g_prof_mu);
  if (on) {
    sr::drain_pending_locked();
    sr::g_prof_agg.clear();
  }
  sr::g_prof_on = on != 0;
  SR_API_END
}

int sr_profile_read(sr_kernel_stat* out, int max, int* n) {
  SR_API_BEGIN
  SR_NONNULL(n);
  std::lock_guard<std::mutex> lk(sr::g_prof_mu);
  sr::drain_pending_locked();
  int i = 0;
  for (const auto& kv : sr::g_prof_agg) {
    if (i >= max || !out) break;
    sr_kernel_stat& st = out[i++];
    std::memset(&st, 0, sizeof(st));
    std::strncpy(st.name, kv.first.c_str(), sizeof(st.name) - 1);
    st.launches = kv.second.launches;
    st.total_ms = kv.second.ms;
    st.flops = kv.second.flops;
    st.bytes = kv.second.bytes;
  }
  *n = i;
  SR_API_END
}

}  // extern "C"
