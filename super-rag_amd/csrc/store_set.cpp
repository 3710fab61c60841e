// Multi-device collection behind one C-ABI handle (sr_store_set_*): SURVEY §8(b)'s
// sr_store_create(dim, dtype, devices, n_dev) — one collection row-sharded over several devices
// (the reference configures its vector DB per deployment, super_rag/config.py:65-67, adaptor
// super_rag/vectorstore/connector.py:4-15; the connector ctx key "devices" maps here).
//
// Rows: one Store (corpus in that device's HBM) per listed device.  Global row ids are the
// insertion order across all shards — exactly the ids one Store would hand out — so every result
// equals a single store's: an add batch goes to the shard with the fewest rows (ties: lowest
// index) and a per-shard table maps its local rows to global rows.  A search runs K1 + K2 on every
// shard concurrently (one host thread per shard, each shard on its own device and stream), maps
// local rows to global rows and merges the B x k lists by (similarity desc, global row asc), the
// order sr_store_search returns (merged on the similarities, not on 1 - sim: two neighbouring
// fp32 similarities can round to one fp32 distance).  A row's similarity does not depend on its
// shard (same fp16 row, same query, same MFMA accumulation order), so the merged lists are
// bit-identical to one store's.
#include <algorithm>
#include <cmath>
#include <numeric>
#include <thread>

#include "sr_runtime.h"

namespace sr {

StoreSet::StoreSet(int dim, int dtype, const int* devices, int n_dev) : dim_(dim) {
  SR_CHECK(n_dev >= 1 && devices, "store_set: at least one device");
  SR_CHECK(dtype == SR_DTYPE_F16 || dtype == SR_DTYPE_FP8_E4M3,
           "store_set: dtype must be SR_DTYPE_F16 or SR_DTYPE_FP8_E4M3 (fp8 scan copy)");
  for (int i = 0; i < n_dev; ++i) {
    shards_.emplace_back(new Store(dim, devices[i], 0));
    if (dtype == SR_DTYPE_FP8_E4M3) shards_.back()->set_scan_dtype(dtype);
    tables_.emplace_back();
  }
}

int64_t StoreSet::rows() const { return (int64_t)shard_of_.size(); }

int64_t StoreSet::live() const {
  int64_t n = 0;
  for (const auto& s : shards_) n += s->live();
  return n;
}

void StoreSet::add_host(const float* vecs, int64_t n, int64_t* out_rows) {
  SR_CHECK(n >= 0 && (n == 0 || vecs), "store_set.add: null vectors");
  if (n == 0) return;
  size_t s = 0;
  for (size_t i = 1; i < shards_.size(); ++i)
    if (tables_[i].size() < tables_[s].size()) s = i;
  std::vector<int64_t> local((size_t)n);
  {
    std::lock_guard<std::mutex> lk(shards_[s]->mu);
    shards_[s]->add_host(vecs, n, local.data());
  }
  SR_CHECK(local[0] == (int64_t)tables_[s].size(), "store_set.add: shard row numbering out of step");
  const int64_t first = rows();
  for (int64_t i = 0; i < n; ++i) {
    tables_[s].push_back(first + i);
    shard_of_.push_back((int32_t)s);
    local_of_.push_back(local[(size_t)i]);
    if (out_rows) out_rows[i] = first + i;
  }
}

void StoreSet::split(const int64_t* rows, int64_t n, std::vector<std::vector<int64_t>>& local,
                     std::vector<std::vector<int64_t>>& pos) const {
  local.assign(shards_.size(), {});
  pos.assign(shards_.size(), {});
  for (int64_t i = 0; i < n; ++i) {
    SR_CHECK(rows[i] >= 0 && rows[i] < this->rows(), "store_set: row out of range");
    const int s = shard_of_[(size_t)rows[i]];
    local[(size_t)s].push_back(local_of_[(size_t)rows[i]]);
    pos[(size_t)s].push_back(i);
  }
}

void StoreSet::remove(const int64_t* rows, int64_t n) {
  SR_CHECK(n >= 0 && (n == 0 || rows), "store_set.remove: null rows");
  std::vector<std::vector<int64_t>> local, pos;
  split(rows, n, local, pos);
  for (size_t s = 0; s < shards_.size(); ++s)
    if (!local[s].empty()) {
      std::lock_guard<std::mutex> lk(shards_[s]->mu);
      shards_[s]->remove(local[s].data(), (int64_t)local[s].size());
    }
}

void StoreSet::get(const int64_t* rows, int64_t n, float* out) {
  SR_CHECK(n >= 0 && (n == 0 || (rows && out)), "store_set.get: null buffer");
  std::vector<std::vector<int64_t>> local, pos;
  split(rows, n, local, pos);
  std::vector<float> buf;
  for (size_t s = 0; s < shards_.size(); ++s) {
    if (local[s].empty()) continue;
    buf.resize(local[s].size() * (size_t)dim_);
    {
      std::lock_guard<std::mutex> lk(shards_[s]->mu);
      shards_[s]->get(local[s].data(), (int64_t)local[s].size(), buf.data());
    }
    for (size_t i = 0; i < local[s].size(); ++i)
      std::copy(buf.begin() + i * dim_, buf.begin() + (i + 1) * dim_, out + pos[s][i] * dim_);
  }
}

void StoreSet::set_scan_dtype(int dtype) {
  for (auto& s : shards_) {
    std::lock_guard<std::mutex> lk(s->mu);
    s->set_scan_dtype(dtype);
  }
}

void StoreSet::search_host(const float* q, int B, int k, float* out_dist, int64_t* out_rows,
                           const uint8_t* allow, int64_t mask_key) {
  SR_CHECK(B >= 0 && (B == 0 || (q && out_dist && out_rows)), "store_set.search: null buffer");
  SR_CHECK(k >= 1 && k <= SR_MAX_TOPK, "store.search: top_k must be in [1, 1024]");
  if (B == 0) return;
  const size_t P = shards_.size(), bk = (size_t)B * k;
  std::vector<std::vector<float>> dist(P, std::vector<float>(bk));
  std::vector<std::vector<int64_t>> loc(P, std::vector<int64_t>(bk));
  // per-shard eligibility: the global mask gathered through the shard's row table (the shard
  // caches its device copy per mask_key and store version, as a single store does)
  std::vector<std::vector<uint8_t>> lallow(allow ? P : 0);
  for (size_t s = 0; s < lallow.size(); ++s) {
    lallow[s].resize(std::max<size_t>(tables_[s].size(), 1));
    for (size_t i = 0; i < tables_[s].size(); ++i) lallow[s][i] = allow[tables_[s][i]];
  }
  std::vector<std::string> err(P);
  std::vector<int> code(P, SR_OK);
  auto run = [&](size_t s) {
    try {
      std::lock_guard<std::mutex> lk(shards_[s]->mu);
      shards_[s]->search_host(q, B, k, dist[s].data(), loc[s].data(),
                              allow ? lallow[s].data() : nullptr, allow ? mask_key : 0, true);
    } catch (const Error& e) {
      code[s] = e.code;
      err[s] = e.what();
    } catch (const std::exception& e) {
      code[s] = SR_ERR_HIP;
      err[s] = e.what();
    }
  };
  std::vector<std::thread> th;
  for (size_t s = 1; s < P; ++s) th.emplace_back(run, s);  // shards scan concurrently
  run(0);
  for (auto& t : th) t.join();
  for (size_t s = 0; s < P; ++s)
    if (code[s] != SR_OK) throw Error(code[s], "store_set shard " + std::to_string(s) + ": " + err[s]);
  // merge: per query the P lists by (similarity desc, global row asc); missing entries (-1) last
  std::vector<std::pair<float, int64_t>> cand;  // (-similarity, global row): ascending order
  for (int b = 0; b < B; ++b) {
    cand.clear();
    for (size_t s = 0; s < P; ++s)
      for (int j = 0; j < k; ++j) {
        const int64_t r = loc[s][(size_t)b * k + j];
        if (r >= 0) cand.emplace_back(-dist[s][(size_t)b * k + j], tables_[s][(size_t)r]);
      }
    const size_t m = std::min(cand.size(), (size_t)k);
    std::partial_sort(cand.begin(), cand.begin() + m, cand.end());
    for (int j = 0; j < k; ++j) {
      const bool ok = (size_t)j < m;
      out_dist[(size_t)b * k + j] = ok ? 1.0f - (-cand[(size_t)j].first) : INFINITY;
      out_rows[(size_t)b * k + j] = ok ? cand[(size_t)j].second : -1;
    }
  }
}

}  // namespace sr
