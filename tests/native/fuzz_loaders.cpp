// Host-side robustness driver for the C-ABI (SURVEY §5 sanitizers), built by
// `make -C super-rag_amd asan` with AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code
// only (host-only objects: no GPU code, no GPU needed) and run by tests/test_native_asan.py:
//   * sr_store_load / sr_lex_load on every truncation of a valid snapshot and on corrupted headers,
//     counts, document lengths and postings: each must return SR_ERR_IO before anything is
//     allocated (a valid snapshot gets past the parser and fails only at the missing device);
//   * argument validation of the entry points (null handles / arrays, negative or absurd sizes):
//     each must return an SR_ERR_* code.
// Any out-of-bounds access, overflow or misaligned load aborts the run with a sanitizer report.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>
#include <utility>
#include <string>
#include <vector>

#include "super_rag_mi355x_diag.h"  // (the ASan build is the diagnostic superset)

static int g_cases = 0, g_fail = 0;

static void expect(bool ok, const std::string& what, int rc) {
  ++g_cases;
  if (!ok) {
    ++g_fail;
    std::fprintf(stderr, "FAIL: %s (rc %d, last error: %s)\n", what.c_str(), rc, sr_last_error());
  }
}

template <class T>
static void put(std::vector<uint8_t>& b, T v) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
  b.insert(b.end(), p, p + sizeof(T));
}

static void write_file(const std::string& path, const std::vector<uint8_t>& bytes) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) {
    std::perror(path.c_str());
    std::exit(2);
  }
  if (!bytes.empty()) std::fwrite(bytes.data(), 1, bytes.size(), f);
  std::fclose(f);
}

// "SRMISTO1", int32 dim, int64 n, n x dim fp16, n live bytes (store.hip Store::save)
static std::vector<uint8_t> store_snapshot(int32_t d, int64_t n) {
  std::vector<uint8_t> b;
  const char* m = "SRMISTO1";
  b.insert(b.end(), m, m + 8);
  put(b, d);
  put(b, n);
  for (int64_t i = 0; i < n * d; ++i) put<uint16_t>(b, (uint16_t)(0x3c00 + (i % 7)));  // ~1.0
  for (int64_t i = 0; i < n; ++i) b.push_back((uint8_t)(i % 3 != 1));
  return b;
}

struct Lex {
  float k1 = 1.2f, b = 0.75f;
  std::vector<int32_t> dl, ft;
  std::vector<uint8_t> live;
  std::vector<uint64_t> fv;
};

// "SRMILEX1", float k1, float b, int64 rows, int64 P, dl, live, terms, (row << 32 | tf) (k_lex.hip)
static std::vector<uint8_t> lex_snapshot(const Lex& x) {
  std::vector<uint8_t> b;
  const char* m = "SRMILEX1";
  b.insert(b.end(), m, m + 8);
  put(b, x.k1);
  put(b, x.b);
  put<int64_t>(b, (int64_t)x.dl.size());
  put<int64_t>(b, (int64_t)x.ft.size());
  for (int32_t v : x.dl) put(b, v);
  for (uint8_t v : x.live) b.push_back(v);
  for (int32_t v : x.ft) put(b, v);
  for (uint64_t v : x.fv) put(b, v);
  return b;
}

static Lex lex_valid() {
  Lex x;
  x.dl = {3, 0, 5};
  x.live = {1, 1, 0};
  // row 0: terms 7 (tf 2), 9 (tf 1); row 2: terms 7 (tf 1), 11 (tf 4)
  x.ft = {7, 9, 7, 11};
  x.fv = {(0ull << 32) | 2, (0ull << 32) | 1, (2ull << 32) | 1, (2ull << 32) | 4};
  return x;
}

static int load_store(const std::string& p) {
  sr_store* s = nullptr;
  const int rc = sr_store_load(p.c_str(), 0, &s);
  if (s) sr_store_destroy(s);
  return rc;
}
static int load_lex(const std::string& p) {
  sr_lex* x = nullptr;
  const int rc = sr_lex_load(p.c_str(), 0, &x);
  if (x) sr_lex_destroy(x);
  return rc;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  const std::string sp = dir + "/fuzz.srmi", lp = dir + "/fuzz.srlex";
  int ndev = -1;
  expect(sr_device_count(&ndev) == SR_OK && ndev >= 0, "sr_device_count", 0);
  const bool gpu = ndev > 0;

  // ---- store snapshots ------------------------------------------------------------------------
  const std::vector<uint8_t> st = store_snapshot(8, 5);
  write_file(sp, st);
  int rc = load_store(sp);
  expect(gpu ? rc == SR_OK : (rc != SR_OK && rc != SR_ERR_IO), "store: valid snapshot parses", rc);
  for (size_t len = 0; len < st.size(); ++len) {  // every truncation
    write_file(sp, std::vector<uint8_t>(st.begin(), st.begin() + len));
    rc = load_store(sp);
    expect(rc == SR_ERR_IO, "store: truncated at " + std::to_string(len), rc);
  }
  {
    std::vector<uint8_t> ext = st;
    ext.push_back(0);
    write_file(sp, ext);
    rc = load_store(sp);
    expect(rc == SR_ERR_IO, "store: trailing byte", rc);
  }
  const struct { int32_t d; int64_t n; } bad_hdr[] = {
      {0, 5}, {-1, 5}, {8, -1}, {1 << 20, 5}, {0x7fffffff, 1}, {8, int64_t(1) << 62},
      {8, (int64_t(1) << 40) + 1}, {8, 6}, {8, 4}, {16, 5}, {4, 5}};
  for (auto h : bad_hdr) {
    std::vector<uint8_t> b = st;
    std::memcpy(b.data() + 8, &h.d, 4);
    std::memcpy(b.data() + 12, &h.n, 8);
    write_file(sp, b);
    rc = load_store(sp);
    expect(rc == SR_ERR_IO, "store: header d=" + std::to_string(h.d) + " n=" + std::to_string(h.n), rc);
  }
  {
    std::vector<uint8_t> b = st;
    b[3] ^= 0x20;  // magic
    write_file(sp, b);
    expect(load_store(sp) == SR_ERR_IO, "store: bad magic", 0);
  }
  expect(load_store(dir + "/does_not_exist.srmi") == SR_ERR_IO, "store: missing file", 0);
  write_file(sp, {});
  expect(load_store(sp) == SR_ERR_IO, "store: empty file", 0);

  // ---- lexical snapshots ------------------------------------------------------------------------
  const Lex lv = lex_valid();
  const std::vector<uint8_t> lx = lex_snapshot(lv);
  write_file(lp, lx);
  rc = load_lex(lp);
  expect(gpu ? rc == SR_OK : (rc != SR_OK && rc != SR_ERR_IO), "lex: valid snapshot parses", rc);
  for (size_t len = 0; len < lx.size(); ++len) {
    write_file(lp, std::vector<uint8_t>(lx.begin(), lx.begin() + len));
    rc = load_lex(lp);
    expect(rc == SR_ERR_IO, "lex: truncated at " + std::to_string(len), rc);
  }
  const int64_t hdr_rows[] = {-1, 2, 4, int64_t(1) << 31, int64_t(1) << 62};
  for (int64_t r : hdr_rows) {
    std::vector<uint8_t> b = lx;
    std::memcpy(b.data() + 16, &r, 8);
    write_file(lp, b);
    rc = load_lex(lp);
    expect(rc == SR_ERR_IO, "lex: header rows=" + std::to_string(r), rc);
  }
  const int64_t hdr_p[] = {-1, 3, 5, int64_t(1) << 40, int64_t(1) << 61};
  for (int64_t P : hdr_p) {
    std::vector<uint8_t> b = lx;
    std::memcpy(b.data() + 24, &P, 8);
    write_file(lp, b);
    rc = load_lex(lp);
    expect(rc == SR_ERR_IO, "lex: header P=" + std::to_string(P), rc);
  }
  auto lex_case = [&](const std::string& what, auto mutate) {
    Lex x = lex_valid();
    mutate(x);
    write_file(lp, lex_snapshot(x));
    const int r = load_lex(lp);
    expect(r == SR_ERR_IO, "lex: " + what, r);
  };
  lex_case("posting row past n_rows", [](Lex& x) { x.fv[3] = (3ull << 32) | 1; });
  lex_case("posting row 2^31", [](Lex& x) { x.fv[3] = (0x80000000ull << 32) | 1; });
  lex_case("postings out of row order", [](Lex& x) { std::swap(x.fv[1], x.fv[2]); });
  lex_case("zero term frequency", [](Lex& x) { x.fv[0] = 0; });
  lex_case("negative term id", [](Lex& x) { x.ft[1] = -5; });
  // a term id sizes the device offset table (vocab + 1 int64): near 2^31 it asked for ~16 GiB
  lex_case("huge term id", [](Lex& x) { x.ft[1] = 0x7ffffff0; });
  lex_case("term id 2^26", [](Lex& x) { x.ft[2] = 1 << 26; });
  lex_case("negative document length", [](Lex& x) { x.dl[1] = -1; });
  lex_case("k1 NaN", [](Lex& x) { x.k1 = std::numeric_limits<float>::quiet_NaN(); });
  lex_case("b infinite", [](Lex& x) { x.b = std::numeric_limits<float>::infinity(); });
  {
    std::vector<uint8_t> b = lx;
    b.push_back(1);
    write_file(lp, b);
    expect(load_lex(lp) == SR_ERR_IO, "lex: trailing byte", 0);
  }
  expect(load_lex(dir + "/does_not_exist.srlex") == SR_ERR_IO, "lex: missing file", 0);

  // random byte flips in the headers: never a crash, never a success without a device
  std::mt19937 rng(1234);
  for (int it = 0; it < 400; ++it) {
    const bool is_lex = it & 1;
    std::vector<uint8_t> b = is_lex ? lx : st;
    const size_t hdr = is_lex ? 32 : 20;
    const int flips = 1 + (int)(rng() % 3);
    for (int f = 0; f < flips; ++f) b[rng() % hdr] ^= (uint8_t)(1u << (rng() % 8));
    write_file(is_lex ? lp : sp, b);
    rc = is_lex ? load_lex(lp) : load_store(sp);
    expect(rc <= 0 && (gpu || rc != SR_OK), "random header flip " + std::to_string(it), rc);
  }

  // ---- argument validation -------------------------------------------------------------------
  auto neg = [&](const std::string& what, int r) { expect(r < 0, what, r); };
  sr_store* sn = nullptr;
  sr_lex* xn = nullptr;
  sr_encoder* en = nullptr;
  neg("store_create(out=NULL)", sr_store_create(8, 0, 16, nullptr));
  neg("store_create(dim=0)", sr_store_create(0, 0, 16, &sn));
  neg("store_create(dim<0)", sr_store_create(-3, 0, 16, &sn));
  neg("store_add(NULL)", sr_store_add(nullptr, nullptr, 4, nullptr));
  neg("store_search(NULL)", sr_store_search(nullptr, nullptr, 2, 10, nullptr, nullptr));
  neg("store_remove(NULL)", sr_store_remove(nullptr, nullptr, 3));
  neg("store_count(NULL)", sr_store_count(nullptr, nullptr, nullptr));
  neg("store_save(NULL)", sr_store_save(nullptr, sp.c_str()));
  neg("store_load(path NULL)", sr_store_load(nullptr, 0, &sn));
  neg("store_load(out NULL)", sr_store_load(sp.c_str(), 0, nullptr));
  neg("store_set_create(devices NULL)", sr_store_set_create(8, SR_DTYPE_F16, nullptr, 2, nullptr));
  {
    const int devs[2] = {0, 0};
    sr_store_set* ss = nullptr;
    neg("store_set_create(dim 0)", sr_store_set_create(0, SR_DTYPE_F16, devs, 2, &ss));
    neg("store_set_create(n_dev 0)", sr_store_set_create(8, SR_DTYPE_F16, devs, 0, &ss));
  }
  neg("lex_create(out NULL)", sr_lex_create(0, 1.2f, 0.75f, nullptr));
  neg("lex_create(b > 1)", sr_lex_create(0, 1.2f, 1.5f, &xn));
  neg("lex_add(NULL)", sr_lex_add(nullptr, nullptr, nullptr, nullptr, nullptr, 3, nullptr));
  neg("lex_search(NULL)", sr_lex_search(nullptr, nullptr, nullptr, 2, 5, nullptr, 0, nullptr, nullptr));
  neg("lex_load(path NULL)", sr_lex_load(nullptr, 0, &xn));
  neg("encoder_create(cfg NULL)", sr_encoder_create(nullptr, 0, &en));
  {
    sr_encoder_config c;
    std::memset(&c, 0, sizeof c);
    c.hidden = 768;
    c.heads = 7;  // d / heads not 32 or 64
    c.layers = 1;
    neg("encoder_create(bad heads)", sr_encoder_create(&c, 0, &en));
    c.heads = 12;
    c.hidden = -768;
    neg("encoder_create(negative hidden)", sr_encoder_create(&c, 0, &en));
  }
  neg("encoder_forward(NULL)", sr_encoder_forward(nullptr, nullptr, nullptr, nullptr, 2, 8, 0, nullptr));
  neg("cross_score(NULL)", sr_cross_score(nullptr, nullptr, nullptr, nullptr, 2, 8, nullptr));
  neg("encoder_set_weight(NULL)", sr_encoder_set_weight(nullptr, "x", nullptr, 4));
  neg("rrf_fuse(B < 0)", sr_rrf_fuse(nullptr, 1, nullptr, 1, -1, 1, 0.0, 1, nullptr, nullptr, 0));
  {
    int64_t ra[2] = {1, 2};
    double sc[2];
    int64_t ro[2];
    neg("rrf_fuse(out NULL)", sr_rrf_fuse(ra, 2, ra, 2, 1, 1, 0.0, 2, nullptr, ro, 0));
    neg("rrf_fuse(rows_b NULL)", sr_rrf_fuse(ra, 2, nullptr, 2, 1, 1, 0.0, 2, sc, ro, 0));
  }
  neg("memcpy(NULL)", sr_memcpy(nullptr, nullptr, 16, 0, 0));
  {
    char buf[32] = {0};
    neg("diag_copy(odd size)", sr_diag_copy(buf, buf + 16, 15, 0, nullptr));
  }
  expect(sr_last_error() != nullptr, "last_error after failures", 0);

  std::printf("fuzz_loaders: %d cases, %d failures (%s)\n", g_cases, g_fail,
              gpu ? "with a device" : "no device: parsers and validation only");
  return g_fail ? 1 : 0;
}
