// In-HBM exact cosine vector store (replaces SeekDB's HNSW collection,
// super_rag/vectorstore/seekdb_connector.py:31-155).
//
// Layout in HBM: corpus = capacity x ld fp16 rows (ld = dim rounded up to 64, zero padded),
// every row L2-normalised on insertion; live = capacity bytes (1 = live, 0 = tombstoned).
// Search runs K1 (cosine_scan) over geometrically growing row chunks, each followed by K2
// (topk_select) that keeps the exact top-k and raises the per-query threshold tau:
//   chunk 0: DENSE scan of min(n, 8192) rows (seeds tau), then chunks growing by up to 8x.
// A per-query candidate list holds at most select_capacity() keys; if any list overflows (an
// adversarial row order), the whole block is re-run in "safe" mode with chunks of
// capacity - k rows, which can never overflow.  Results are exact either way.
#include <cstdlib>
#include <fstream>

#include "sr_kernels.h"
#include "sr_runtime.h"

namespace sr {

// Threshold-chunk growth cap of the K1 schedule (chunk = rows scanned so far x growth, growth <=
// (cap - k) / 2k so the expected keys fit the candidate lists).  SR_SCAN_GROWTH overrides the cap
// (schedule experiments).
static int64_t scan_fixed_chunk() {  // SR_SCAN_CHUNK: fixed threshold-chunk rows (experiments)
  static const int64_t c = [] {
    const char* e = diag_getenv("SR_SCAN_CHUNK");
    const long v = e ? std::strtol(e, nullptr, 10) : 0;
    return (int64_t)(v > 0 ? v : 0);
  }();
  return c;
}
static int64_t scan_growth_max() {
  static const int64_t g = [] {
    const char* e = diag_getenv("SR_SCAN_GROWTH");
    const long v = e ? std::strtol(e, nullptr, 10) : 0;
    return (int64_t)(v > 0 ? v : 8);
  }();
  return g;
}

namespace {
constexpr int kDenseRows = 8192;
constexpr int kQueryBlock = 256;
constexpr int64_t kAddChunk = 1 << 16;

__global__ void clear_flags_kernel(uint8_t* live, const int64_t* rows, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) live[rows[i]] = 0;
}
__global__ void gather_rows_kernel(const half_t* __restrict__ src, int ld,
                                   const int64_t* __restrict__ rows, int64_t n,
                                   half_t* __restrict__ dst) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  const half8* s = reinterpret_cast<const half8*>(src + rows[r] * ld);
  half8* d = reinterpret_cast<half8*>(dst + r * ld);
  for (int c = threadIdx.x; c < ld / 8; c += blockDim.x) d[c] = s[c];
}
// fp16 unit rows (ld halfs) -> e4m3(256 x) rows (ld8 bytes, zero padded): |256 x| <= 256 < 448, so
// one fixed power of two serves every row and query (the scan MFMA's E8M0 scales undo it).
__global__ void quantize_rows_fp8_kernel(const half_t* __restrict__ src, int ld, int dim,
                                         int64_t n, uint8_t* __restrict__ dst, int ld8) {
  const int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n) return;
  const half_t* x = src + r * ld;
  uint8_t* d = dst + r * ld8;
  for (int c = lane; c < ld8; c += 64)
    d[c] = c < dim ? (uint8_t)e4m3_rne((float)x[c] * 256.f) : (uint8_t)0;
}

// exact fp16 re-scoring of a query's fp8-stage candidates: key (sim, row) per candidate slot
// (0 = empty), count = kk
__global__ void rescore_kernel(const half_t* __restrict__ corpus, int ld, int dim,
                               const half_t* __restrict__ qn, const int64_t* __restrict__ rows,
                               int kk, uint64_t* __restrict__ cand, int cap, int* __restrict__ cnt) {
  const int q = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const half_t* qv = qn + (int64_t)q * ld;
  for (int c = wave; c < kk; c += blockDim.x >> 6) {
    const int64_t row = rows[(int64_t)q * kk + c];
    float acc = 0.f;
    if (row >= 0) {
      const half_t* x = corpus + row * ld;
      for (int i = lane; i < dim; i += 64) acc = fmaf((float)qv[i], (float)x[i], acc);
    }
    acc = wave_sum(acc);
    if (lane == 0) cand[(int64_t)q * cap + c] = row >= 0 ? make_key(acc, (uint32_t)row) : 0ull;
  }
  if (threadIdx.x == 0) cnt[q] = kk;
}

__global__ void f16_to_f32_rows_kernel(const half_t* __restrict__ src, int ld,
                                       const int64_t* __restrict__ rows, int64_t n, int dim,
                                       float* __restrict__ out) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  for (int c = threadIdx.x; c < dim; c += blockDim.x) out[r * dim + c] = (float)src[rows[r] * ld + c];
}
}  // namespace

Store::Store(int dim, int device, int64_t capacity) : dim_(dim), device_(device) {
  SR_CHECK(dim > 0 && dim <= 8192, "store: dim must be in [1, 8192]");
  ld_ = (int)round_up(dim, 64);
  DeviceGuard g(device_);
  SR_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  SR_HIP(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  ensure_capacity(capacity > 0 ? capacity : 1024);
}

Store::~Store() {
  (void)hipSetDevice(device_);
  if (done_) {
    (void)hipEventSynchronize(done_);
    (void)hipEventDestroy(done_);
  }
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    (void)hipStreamDestroy(stream_);
  }
}

void Store::ensure_capacity(int64_t rows) {
  if (rows <= capacity_) return;
  int64_t cap = std::max<int64_t>(rows, capacity_ + capacity_ / 2);
  cap = round_up(cap, 256);
  DevBuf nc, nl;
  nc.reserve((size_t)cap * ld_ * sizeof(half_t));
  nl.reserve((size_t)cap);
  SR_HIP(hipMemsetAsync(nl.p, 0, (size_t)cap, stream_));
  if (n_rows_ > 0) {
    SR_HIP(hipMemcpyAsync(nc.p, corpus_.p, (size_t)n_rows_ * ld_ * sizeof(half_t),
                          hipMemcpyDeviceToDevice, stream_));
    SR_HIP(hipMemcpyAsync(nl.p, live_.p, (size_t)n_rows_, hipMemcpyDeviceToDevice, stream_));
  }
  SR_HIP(hipStreamSynchronize(stream_));
  std::swap(corpus_.p, nc.p);
  std::swap(corpus_.bytes, nc.bytes);
  std::swap(live_.p, nl.p);
  std::swap(live_.bytes, nl.bytes);
  capacity_ = cap;
  live_host_.resize((size_t)cap, 0);
  if (fp8_) grow_fp8();
}

int Store::ld8() const { return (int)round_up(dim_, 128) < 256 ? 256 : (int)round_up(dim_, 128); }

void Store::grow_fp8() {
  DevBuf nc;
  nc.reserve((size_t)capacity_ * ld8());
  if (n_rows_ > 0 && corpus8_.p)
    SR_HIP(hipMemcpyAsync(nc.p, corpus8_.p, (size_t)n_rows_ * ld8(), hipMemcpyDeviceToDevice, stream_));
  SR_HIP(hipStreamSynchronize(stream_));
  std::swap(corpus8_.p, nc.p);
  std::swap(corpus8_.bytes, nc.bytes);
}

void Store::quantize_rows(int64_t r0, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(quantize_rows_fp8_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, s,
                     corpus_.as<half_t>() + r0 * ld_, ld_, dim_, n, corpus8_.as<uint8_t>() + r0 * ld8(),
                     ld8());
  SR_LAUNCH_CHECK();
}

void Store::set_scan_dtype(int dtype) {
  SR_CHECK(dtype == SR_DTYPE_F16 || dtype == SR_DTYPE_FP8_E4M3, "store: scan dtype must be f16 or fp8");
  DeviceGuard g(device_);
  begin(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  if (dtype == SR_DTYPE_F16) {
    fp8_ = false;
    corpus8_.release();
  } else if (!fp8_) {
    SR_CHECK(ld8() <= 2048, "store: the fp8 scan supports dim <= 2048");
    fp8_ = true;
    grow_fp8();
    quantize_rows(0, n_rows_, stream_);
  }
  end(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
}

void Store::add_host(const float* vecs, int64_t n, int64_t* out_rows) {
  SR_CHECK(n >= 0 && (n == 0 || vecs), "store.add: null vectors");
  DeviceGuard g(device_);
  begin(stream_);
  ensure_capacity(n_rows_ + n);
  for (int64_t off = 0; off < n; off += kAddChunk) {
    const int64_t m = std::min(kAddChunk, n - off);
    scratch_.reserve((size_t)m * dim_ * sizeof(float));
    SR_HIP(hipMemcpyAsync(scratch_.p, vecs + off * dim_, (size_t)m * dim_ * sizeof(float),
                          hipMemcpyHostToDevice, stream_));
    const int64_t first = add_dev(scratch_.p, SR_DTYPE_F32, m, stream_);
    if (out_rows)
      for (int64_t i = 0; i < m; ++i) out_rows[off + i] = first + i;
  }
  SR_HIP(hipStreamSynchronize(stream_));
}

int64_t Store::add_dev(const void* vecs, int dtype, int64_t n, hipStream_t s) {
  SR_CHECK(dtype == SR_DTYPE_F32 || dtype == SR_DTYPE_F16, "store.add: dtype must be f32 or f16");
  DeviceGuard g(device_);
  const int64_t first = n_rows_;
  if (n <= 0) return first;
  begin(s);
  if (n_rows_ + n > capacity_) {
    SR_HIP(hipStreamSynchronize(s));
    ensure_capacity(n_rows_ + n);
  }
  launch_normalize_rows(vecs, dtype, n, dim_, corpus_.as<half_t>() + first * ld_, ld_, s);
  if (fp8_) quantize_rows(first, n, s);
  SR_HIP(hipMemsetAsync(live_.as<uint8_t>() + first, 1, (size_t)n, s));
  end(s);
  std::fill(live_host_.begin() + first, live_host_.begin() + first + n, 1);
  n_rows_ += n;
  n_live_ += n;
  ++version_;
  return first;
}

void Store::remove(const int64_t* rows, int64_t n) {
  SR_CHECK(n > 0 && rows, "store.delete: ids is required");
  for (int64_t i = 0; i < n; ++i)
    SR_CHECK(rows[i] >= 0 && rows[i] < n_rows_ && live_host_[rows[i]],
             "store.delete: unknown or already deleted row " + std::to_string(rows[i]));
  DeviceGuard g(device_);
  begin(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  scratch_.reserve((size_t)n * sizeof(int64_t));
  SR_HIP(hipMemcpyAsync(scratch_.p, rows, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, stream_));
  hipLaunchKernelGGL(clear_flags_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, stream_,
                     live_.as<uint8_t>(), scratch_.as<int64_t>(), n);
  SR_LAUNCH_CHECK();
  end(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  for (int64_t i = 0; i < n; ++i) {
    if (live_host_[rows[i]]) {
      live_host_[rows[i]] = 0;
      --n_live_;
    }
  }
  ++version_;
}

void Store::get(const int64_t* rows, int64_t n, float* out) {
  if (n <= 0) return;
  for (int64_t i = 0; i < n; ++i)
    SR_CHECK(rows[i] >= 0 && rows[i] < n_rows_, "store.get: row out of range");
  DeviceGuard g(device_);
  begin(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  scratch_.reserve((size_t)n * (sizeof(int64_t) + dim_ * sizeof(float)));
  int64_t* drows = scratch_.as<int64_t>();
  float* dout = reinterpret_cast<float*>(drows + n);
  SR_HIP(hipMemcpyAsync(drows, rows, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, stream_));
  hipLaunchKernelGGL(f16_to_f32_rows_kernel, dim3((unsigned)n), dim3(256), 0, stream_,
                     corpus_.as<half_t>(), ld_, drows, n, dim_, dout);
  SR_LAUNCH_CHECK();
  SR_HIP(hipMemcpyAsync(out, dout, (size_t)n * dim_ * sizeof(float), hipMemcpyDeviceToHost, stream_));
  end(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
}

void Store::ensure_query_ws(int B) {
  const int nq = (int)round_up(std::max(B, 1), kQueryBlock);
  if (nq <= ws_queries_) return;
  SR_HIP(hipEventSynchronize(done_));  // the previous search may still use the old workspace
  const int cap = select_capacity();
  qbuf_.reserve((size_t)nq * ld_ * sizeof(half_t));
  SR_HIP(hipMemsetAsync(qbuf_.p, 0, qbuf_.bytes, stream_));
  cand_.reserve((size_t)kQueryBlock * cap * sizeof(uint64_t));
  cnt_.reserve(kQueryBlock * sizeof(int));
  tau_.reserve(kQueryBlock * sizeof(float));
  overflow_.reserve(sizeof(int));
  q8_.reserve((size_t)kQueryBlock * 2048);
  approx_.reserve((size_t)round_up((int64_t)kQueryBlock * SR_MAX_TOPK * 4, 256) +
                  (size_t)kQueryBlock * SR_MAX_TOPK * 8);
  SR_HIP(hipStreamSynchronize(stream_));
  ws_queries_ = nq;
}

// fp8 scan (set_scan_dtype(SR_DTYPE_FP8_E4M3)): the same chunk / threshold schedule on the fp8 rows
// (half the bytes, block-scaled MFMA) keeps the top kk = min(max(2k, k + 32), 1024) by the
// fp8-stage similarity; those candidates are re-scored exactly on the fp16 rows and the top k of
// the exact scores returned.  Exact whenever the fp8 stage's top kk contains the true top k.
void Store::search_block8(const half_t* qn, int B, int k, float* out_sim, int64_t* out_rows,
                          int64_t row_offset, hipStream_t s, bool safe, const uint8_t* live) {
  const int cap = select_capacity();
  const int kk = std::min(std::min(std::max(2 * k, k + 32), SR_MAX_TOPK), cap / 4);
  uint64_t* cand = cand_.as<uint64_t>();
  int* cnt = cnt_.as<int>();
  float* tau = tau_.as<float>();
  int* ovf = overflow_.as<int>();
  const int64_t n = n_rows_;
  uint8_t* q8 = q8_.as<uint8_t>();
  hipLaunchKernelGGL(quantize_rows_fp8_kernel, dim3((unsigned)ceil_div(B, 4)), dim3(256), 0, s, qn,
                     ld_, dim_, (int64_t)B, q8, ld8());
  SR_LAUNCH_CHECK();
  float* asim = approx_.as<float>();
  int64_t* arow = reinterpret_cast<int64_t*>(approx_.as<char>() + round_up((int64_t)kQueryBlock * SR_MAX_TOPK * 4, 256));
  launch_fill_int(cnt, B, 0, s);
  launch_fill_float(tau, B, -INFINITY, s);
  if (n == 0) {
    launch_topk_select(cand, cnt, cap, tau, B, kk, ovf, true, asim, arow, 0, s, live);
  } else {
    // B <= 64: the small-block fp8 kernel (dense first chunk, then threshold chunks); larger
    // blocks: the 256 x 256 fp8 GEMM main loop (its first chunk in threshold mode at tau = -inf)
    const bool small = B <= 64;   // (at 128 queries the GEMM main loop is faster: 4.4 ms vs ~3.7)
    const int64_t dense = std::min<int64_t>(n, safe ? (int64_t)(cap - kk) : kDenseRows);
    if (small) {
      launch_cosine_scan8(true, corpus8_.as<uint8_t>(), ld8(), live, 0, dense, q8, B, tau, cand,
                          cnt, cap, s);
      launch_fill_int(cnt, B, (int)dense, s);
    } else {
      launch_cosine_scan_gemm8(corpus8_.as<uint8_t>(), ld8(), live, 0, dense, q8, B, tau, cand, cnt,
                               cap, s);
    }
    launch_topk_select(cand, cnt, cap, tau, B, kk, ovf, dense == n, asim, arow, 0, s, live);
    const int64_t growth = std::max<int64_t>(1, std::min<int64_t>(scan_growth_max(), (cap - kk) / (2 * kk)));
    int64_t r = dense;
    while (r < n) {
      const int64_t step = safe ? (int64_t)(cap - kk) : std::max<int64_t>(r * growth, kDenseRows);
      const int64_t next = std::min(n, r + step);
      if (small)
        launch_cosine_scan8(false, corpus8_.as<uint8_t>(), ld8(), live, r, next, q8, B, tau, cand,
                            cnt, cap, s);
      else
        launch_cosine_scan_gemm8(corpus8_.as<uint8_t>(), ld8(), live, r, next, q8, B, tau, cand, cnt,
                                 cap, s);
      launch_topk_select(cand, cnt, cap, tau, B, kk, ovf, next == n, asim, arow, 0, s, live);
      r = next;
    }
  }
  {
    ProfScope prof("rescore", s, 2.0 * B * kk * dim_, (double)B * kk * ld_ * 2.0);
    hipLaunchKernelGGL(rescore_kernel, dim3(B), dim3(256), 0, s, corpus_.as<half_t>(), ld_, dim_, qn,
                       arow, kk, cand, cap, cnt);
    SR_LAUNCH_CHECK();
  }
  launch_topk_select(cand, cnt, cap, tau, B, k, ovf, true, out_sim, out_rows, row_offset, s, live);
}

void Store::search_block(const half_t* qn, int B, int k, float* out_sim, int64_t* out_rows,
                         int64_t row_offset, hipStream_t s, bool safe, const uint8_t* live) {
  if (fp8_) {
    search_block8(qn, B, k, out_sim, out_rows, row_offset, s, safe, live);
    return;
  }
  const int cap = select_capacity();
  uint64_t* cand = cand_.as<uint64_t>();
  int* cnt = cnt_.as<int>();
  float* tau = tau_.as<float>();
  int* ovf = overflow_.as<int>();
  const half_t* C = corpus_.as<half_t>();
  const int64_t n = n_rows_;
  if (n == 0) {
    launch_fill_int(cnt, B, 0, s);
    launch_topk_select(cand, cnt, cap, tau, B, k, ovf, true, out_sim, out_rows, row_offset, s, live);
    return;
  }
  const int64_t dense = std::min<int64_t>(n, safe ? (int64_t)(cap - k) : kDenseRows);
  launch_cosine_scan(true, C, ld_, live, 0, dense, qn, B, tau, cand, cnt, cap, s);
  launch_fill_int(cnt, B, (int)dense, s);
  launch_topk_select(cand, cnt, cap, tau, B, k, ovf, dense == n, out_sim, out_rows, row_offset, s, live);
  const int64_t growth = std::max<int64_t>(1, std::min<int64_t>(scan_growth_max(), (cap - k) / (2 * k)));
  int64_t r = dense;
  while (r < n) {
    const int64_t step = safe ? (int64_t)(cap - k)
                              : (scan_fixed_chunk() ? scan_fixed_chunk() : std::max<int64_t>(r * growth, kDenseRows));
    const int64_t next = std::min(n, r + step);
    launch_cosine_scan(false, C, ld_, live, r, next, qn, B, tau, cand, cnt, cap, s);
    launch_topk_select(cand, cnt, cap, tau, B, k, ovf, next == n, out_sim, out_rows, row_offset, s, live);
    r = next;
  }
}

void Store::search_dev(const void* q, int q_dtype, int B, int k, float* out_sim,
                       int64_t* out_rows, int64_t row_offset, hipStream_t s, const uint8_t* elig) {
  // elig: per-row eligibility (device, n_rows bytes; live & filter), or null for the live flags
  const uint8_t* live = elig ? elig : live_.as<uint8_t>();
  SR_CHECK(B >= 0, "store.search: negative batch");
  SR_CHECK(k >= 1 && k <= SR_MAX_TOPK, "store.search: top_k must be in [1, 1024]");
  SR_CHECK(k <= select_capacity() / 4, "store.search: top_k too large");
  if (B == 0) return;
  DeviceGuard g(device_);
  // s == nullptr is the HIP null stream (what torch reports for its default stream): use as-is.
  begin(s);
  ensure_query_ws(B);
  half_t* qn = qbuf_.as<half_t>();
  launch_normalize_rows(q, q_dtype, B, dim_, qn, ld_, s);
  SR_HIP(hipMemsetAsync(overflow_.p, 0, sizeof(int), s));
  for (int b0 = 0; b0 < B; b0 += kQueryBlock) {
    const int bb = std::min(kQueryBlock, B - b0);
    search_block(qn + (int64_t)b0 * ld_, bb, k, out_sim + (int64_t)b0 * k,
                 out_rows + (int64_t)b0 * k, row_offset, s, false, live);
  }
  int ovf = 0;
  SR_HIP(hipMemcpyAsync(&ovf, overflow_.p, sizeof(int), hipMemcpyDeviceToHost, s));
  end(s);
  SR_HIP(hipStreamSynchronize(s));
  if (ovf) {
    // Rare: a candidate list overflowed (row order adversarial to the threshold).  Redo exactly.
    for (int b0 = 0; b0 < B; b0 += kQueryBlock) {
      const int bb = std::min(kQueryBlock, B - b0);
      search_block(qn + (int64_t)b0 * ld_, bb, k, out_sim + (int64_t)b0 * k,
                   out_rows + (int64_t)b0 * k, row_offset, s, true, live);
    }
    end(s);
  }
}

const uint8_t* Store::eligibility(const uint8_t* allow, int64_t mask_key) {
  if (!allow) return nullptr;
  // eligibility = live & allow, uploaded once per (mask_key, store version)
  if (mask_key == 0 || mask_key != mask_key_ || mask_version_ != version_ || mask_rows_ != n_rows_) {
    std::vector<uint8_t> m((size_t)std::max<int64_t>(n_rows_, 1));
    for (int64_t r = 0; r < n_rows_; ++r) m[(size_t)r] = (live_host_[(size_t)r] && allow[r]) ? 1 : 0;
    mask_.reserve(m.size());
    begin(stream_);
    SR_HIP(hipMemcpyAsync(mask_.p, m.data(), (size_t)n_rows_, hipMemcpyHostToDevice, stream_));
    SR_HIP(hipStreamSynchronize(stream_));
    end(stream_);
    mask_key_ = mask_key;
    mask_version_ = version_;
    mask_rows_ = n_rows_;
  }
  return mask_.as<uint8_t>();
}

void Store::search_host(const float* q, int B, int k, float* out_dist, int64_t* out_rows,
                        const uint8_t* allow, int64_t mask_key, bool raw_sim) {
  SR_CHECK(B >= 0 && (B == 0 || (q && out_dist && out_rows)), "store.search: null buffer");
  if (B == 0) return;
  DeviceGuard g(device_);
  const uint8_t* elig = eligibility(allow, mask_key);
  const size_t qb = (size_t)B * dim_ * sizeof(float);
  const size_t ob = (size_t)B * k * (sizeof(float) + sizeof(int64_t));
  qstage_.reserve(qb + ob);
  float* dq = qstage_.as<float>();
  float* dsim = reinterpret_cast<float*>(qstage_.as<char>() + qb);
  int64_t* drows = reinterpret_cast<int64_t*>(dsim + (size_t)B * k);
  SR_HIP(hipMemcpyAsync(dq, q, qb, hipMemcpyHostToDevice, stream_));
  search_dev(dq, SR_DTYPE_F32, B, k, dsim, drows, 0, stream_, elig);
  SR_HIP(hipMemcpyAsync(out_dist, dsim, (size_t)B * k * sizeof(float), hipMemcpyDeviceToHost, stream_));
  SR_HIP(hipMemcpyAsync(out_rows, drows, (size_t)B * k * sizeof(int64_t), hipMemcpyDeviceToHost, stream_));
  SR_HIP(hipStreamSynchronize(stream_));
  if (raw_sim) return;
  for (int64_t i = 0; i < (int64_t)B * k; ++i)
    out_dist[i] = out_rows[i] >= 0 ? 1.0f - out_dist[i] : INFINITY;
}

// Snapshot format (little endian): "SRMISTO1", int32 dim, int64 n_rows, n_rows x dim fp16
// (normalised rows, unpadded), n_rows bytes of live flags.  Written to "<path>.tmp", fsync'd and
// renamed over <path>, so a crash mid-save leaves the previous snapshot intact.
void Store::save(const char* path) {
  DeviceGuard g(device_);
  begin(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  const std::string tmp = std::string(path) + ".tmp";
  std::ofstream f(tmp, std::ios::binary | std::ios::trunc);
  if (!f) throw Error(SR_ERR_IO, std::string("store.save: cannot open ") + tmp);
  f.write("SRMISTO1", 8);
  const int32_t d = dim_;
  f.write(reinterpret_cast<const char*>(&d), 4);
  f.write(reinterpret_cast<const char*>(&n_rows_), 8);
  std::vector<half_t> buf;
  const int64_t chunk = 1 << 16;
  for (int64_t r = 0; r < n_rows_; r += chunk) {
    const int64_t m = std::min(chunk, n_rows_ - r);
    buf.resize((size_t)m * dim_);
    SR_HIP(hipMemcpy2D(buf.data(), dim_ * sizeof(half_t), corpus_.as<half_t>() + r * ld_,
                       ld_ * sizeof(half_t), dim_ * sizeof(half_t), (size_t)m,
                       hipMemcpyDeviceToHost));
    f.write(reinterpret_cast<const char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(half_t)));
  }
  f.write(reinterpret_cast<const char*>(live_host_.data()), (std::streamsize)n_rows_);
  f.flush();
  if (!f) throw Error(SR_ERR_IO, std::string("store.save: write failed for ") + tmp);
  f.close();
  if (!fsync_path(tmp)) throw Error(SR_ERR_IO, std::string("store.save: fsync failed for ") + tmp);
  if (std::rename(tmp.c_str(), path) != 0)
    throw Error(SR_ERR_IO, std::string("store.save: cannot rename ") + tmp + " to " + path);
}

Store* Store::load(const char* path, int device) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error(SR_ERR_IO, std::string("store.load: cannot open ") + path);
  char magic[8];
  f.read(magic, 8);
  if (!f || std::memcmp(magic, "SRMISTO1", 8) != 0)
    throw Error(SR_ERR_IO, std::string("store.load: not a store snapshot: ") + path);
  int32_t d = 0;
  int64_t n = 0;
  f.read(reinterpret_cast<char*>(&d), 4);
  f.read(reinterpret_cast<char*>(&n), 8);
  if (!f || d <= 0 || d > (1 << 16) || n < 0 || n > (int64_t(1) << 40))
    throw Error(SR_ERR_IO, "store.load: corrupt header");
  // the exact size the header implies, checked before anything is allocated: a corrupt count
  // must not size a device allocation (or read past the rows into the live flags)
  const std::streamoff here = f.tellg();
  f.seekg(0, std::ios::end);
  const std::streamoff size = f.tellg();
  f.seekg(here);
  if (!f || size != (std::streamoff)(20 + n * (int64_t)d * 2 + n))
    throw Error(SR_ERR_IO, "store.load: file size does not match the header (truncated or corrupt)");
  Store* s = new Store(d, device, std::max<int64_t>(n, 1024));
  try {
    DeviceGuard g(device);
    std::vector<half_t> buf;
    const int64_t chunk = 1 << 16;
    for (int64_t r = 0; r < n; r += chunk) {
      const int64_t m = std::min(chunk, n - r);
      buf.resize((size_t)m * d);
      f.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(buf.size() * sizeof(half_t)));
      if (!f) throw Error(SR_ERR_IO, "store.load: truncated rows");
      SR_HIP(hipMemcpy2D(s->corpus_.as<half_t>() + r * s->ld_, s->ld_ * sizeof(half_t), buf.data(),
                         d * sizeof(half_t), d * sizeof(half_t), (size_t)m, hipMemcpyHostToDevice));
    }
    if (s->ld_ > d && n > 0)
      SR_HIP(hipMemset2D(s->corpus_.as<half_t>() + d, s->ld_ * sizeof(half_t), 0,
                         (s->ld_ - d) * sizeof(half_t), (size_t)n));
    f.read(reinterpret_cast<char*>(s->live_host_.data()), (std::streamsize)n);
    if (!f) throw Error(SR_ERR_IO, "store.load: truncated live flags");
    SR_HIP(hipMemcpy(s->live_.p, s->live_host_.data(), (size_t)n, hipMemcpyHostToDevice));
    s->n_rows_ = n;
    s->n_live_ = 0;
    for (int64_t i = 0; i < n; ++i) s->n_live_ += s->live_host_[i] ? 1 : 0;
  } catch (...) {
    delete s;
    throw;
  }
  return s;
}

void Store::compact(int64_t* old_to_new) {
  DeviceGuard g(device_);
  begin(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  std::vector<int64_t> keep;
  keep.reserve((size_t)n_live_);
  for (int64_t r = 0; r < n_rows_; ++r) {
    if (live_host_[r]) {
      if (old_to_new) old_to_new[r] = (int64_t)keep.size();
      keep.push_back(r);
    } else if (old_to_new) {
      old_to_new[r] = -1;
    }
  }
  const int64_t m = (int64_t)keep.size();
  DevBuf nc, rows;
  nc.reserve((size_t)std::max<int64_t>(capacity_, 1) * ld_ * sizeof(half_t));
  if (m > 0) {
    rows.reserve((size_t)m * sizeof(int64_t));
    SR_HIP(hipMemcpyAsync(rows.p, keep.data(), (size_t)m * sizeof(int64_t), hipMemcpyHostToDevice, stream_));
    hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)m), dim3(64), 0, stream_,
                       corpus_.as<half_t>(), ld_, rows.as<int64_t>(), m, nc.as<half_t>());
    SR_LAUNCH_CHECK();
  }
  SR_HIP(hipMemsetAsync(live_.p, 0, (size_t)capacity_, stream_));
  if (m > 0) SR_HIP(hipMemsetAsync(live_.p, 1, (size_t)m, stream_));
  end(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  std::swap(corpus_.p, nc.p);
  std::swap(corpus_.bytes, nc.bytes);
  std::fill(live_host_.begin(), live_host_.end(), 0);
  std::fill(live_host_.begin(), live_host_.begin() + m, 1);
  n_rows_ = m;
  n_live_ = m;
  ++version_;
  if (fp8_) {
    quantize_rows(0, m, stream_);
    SR_HIP(hipStreamSynchronize(stream_));
  }
}

}  // namespace sr
