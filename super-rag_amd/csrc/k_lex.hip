// BM25 lexical index over the store's rows and the reciprocal-rank fusion of a dense and a lexical
// ranking ("dense + BM25 fusion"; the reference's fulltext index is a no-op and its
// node slot `fulltext_search_docs` (nodeflow/runners/merge.py:18-20) is empty, so the scoring
// below is this library's own definition, documented in DESIGN.md, and the fusion follows the
// reference's only precedent, graphiti rrf, super_rag/graphiti/graphiti_core/search/search_utils.py:1762-1778).
//
// Layout in HBM
//   forward index (append-only, row order): fterm[P] int32, fval[P] u64 = row << 32 | tf;
//   dlen[rows] int32 (document length in tokens), live[rows] u8;
//   inverted index (CSR by term over LIVE documents, rebuilt on the device when dirty):
//   off[T + 1] int64, post[nnz] u64 = row << 32 | tf, rows ascending inside a term (stable radix
//   sort of the row-ordered forward index by term id, dead rows keyed past the vocabulary; off by a
//   binary search per term over the sorted keys).
//
// Scoring (one block of queries):
//   L0 lex_bounds: for every (query term, 8192-row block) the first posting of that block
//      (binary search: postings are row-sorted inside a term).
//   L1 lex_score: one workgroup per (row block, query).  The query's postings of the block are
//      contiguous in each term's list (streaming 8-byte loads); each posting's Okapi weight
//      w = idf * (tf * (k1 + 1)) / (tf + k1 * ((1 - b) + b * (dl / avgdl)))   (fp32, no FMA
//      contraction, so a numpy float32 restatement reproduces it bit for bit) is quantised to
//      q = max(1, rint(w * 2^16)) x (query multiplicity) and added with an LDS atomic into the
//      block.s 32 KiB accumulator.  Non-zero entries are then appended to the query's candidate
//      keys (score << 32 | ~row; one counter atomic per wave).  Integer sums make the result
//      independent of the atomic order: bit-exact against the oracle.
//   L2 lex_select: one workgroup per query: exact top-k of the candidate keys: a score histogram
//      pass, then a pass collecting the keys of the top bins into LDS for the block radix select
//      (sr_topk.h).
// Fusion:
//   F1 rrf_fuse: one workgroup per query: rrf score of a row = sum over the lists of
//      1 / (rank + rank_const) in fp64 (list a first, as graphiti accumulates), ordered by score
//      descending with ties by first appearance (a's ranks, then b's new rows in b order), as
//      Python's stable sort over the insertion-ordered dict does; rows below min_score dropped.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "sr_kernels.h"
#include "sr_runtime.h"
#include "sr_topk.h"

namespace sr {

constexpr int LEX_RB = 8192;           // rows per accumulation block (32 KiB of LDS; 16384: -20 %)
constexpr int LEX_THREADS = 512;
constexpr float LEX_SCALE = 65536.f;   // fixed-point unit of the accumulated score
constexpr int64_t LEX_KEY_BUDGET = (int64_t)1 << 28;  // candidate keys per query block (2 GiB)
// term ids are dense vocabulary indices (lexical.Vocab, or a model's token ids: <= 250,002); the
// device offset table holds vocab + 1 int64, so 2^26 ids bound it at 512 MiB
constexpr int32_t kLexMaxVocab = (int32_t)1 << 26;

struct LexTerm {  // one distinct term of one query
  int64_t start;  // first posting of the term
  int32_t len;    // its document frequency (postings)
  float idf;
  int32_t mult;   // multiplicity of the term in the query
  int32_t pad;
};

// ---- rebuild ------------------------------------------------------------------------------------
// sort key of every forward posting: its term, or dead_key (= vocabulary size, sorts last) for a
// tombstoned row
__global__ void lex_keys_kernel(const int32_t* __restrict__ fterm, const uint64_t* __restrict__ fval,
                                const uint8_t* __restrict__ live, int64_t P, uint32_t dead_key,
                                uint32_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P) return;
  const uint32_t row = (uint32_t)(fval[i] >> 32);
  keys[i] = live[row] ? (uint32_t)fterm[i] : dead_key;
}

// off[t] = first sorted posting with key >= t, t in [0, T] (so off[T] = live postings); a binary
// search per term instead of a histogram (whose atomics serialise on the Zipf head terms)
__global__ void lex_offsets_kernel(const uint32_t* __restrict__ keys, int64_t P, int64_t T,
                                   int64_t* __restrict__ off) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t > T) return;
  int64_t lo = 0, hi = P;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)keys[mid] < t) lo = mid + 1;
    else hi = mid;
  }
  off[t] = lo;
}

// ---- L1 -----------------------------------------------------------------------------------------
// (no FMA contraction anywhere below: the BM25 weight and the fp64 rrf sums are restated in numpy
// / Python, which round every operation)
#pragma clang fp contract(off)
__device__ __forceinline__ uint32_t bm25_fixed(float idf, float tf, float dl, float avgdl, float k1,
                                               float b, float one_minus_b, float k1p1) {
  const float t1 = __fdiv_rn(dl, avgdl);
  const float norm = k1 * (one_minus_b + b * t1);
  const float w = idf * __fdiv_rn(tf * k1p1, tf + norm);
  const float q = rintf(w * LEX_SCALE);
  return q < 1.f ? 1u : (uint32_t)q;
}

// bnd[t][blk] = first posting of term slot t whose row is >= blk * LEX_RB (postings are sorted by
// row inside a term, and a posting's u64 orders by row first), blk in [0, NB]
__global__ void lex_bounds_kernel(const LexTerm* __restrict__ terms, int nslots, int NB,
                                  const uint64_t* __restrict__ post, int32_t* __restrict__ bnd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)nslots * (NB + 1)) return;
  const int t = (int)(i / (NB + 1)), blk = (int)(i % (NB + 1));
  const LexTerm e = terms[t];
  const uint64_t target = ((uint64_t)blk * LEX_RB) << 32;
  int lo = 0, hi = e.len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (post[e.start + mid] < target) lo = mid + 1;
    else hi = mid;
  }
  bnd[i] = lo;
}

// One workgroup per (query, row block): the query's postings whose rows fall in the block are
// accumulated with LDS atomics into a 8192-row fixed-point accumulator, then every non-zero
// entry is appended to the query's candidate keys (score << 32 | ~row), one counter atomic per
// wave.  Postings of a block are contiguous in each term's list: streaming 8-byte loads.
__global__ __launch_bounds__(LEX_THREADS) void lex_score_kernel(
    const LexTerm* __restrict__ terms, const int* __restrict__ slot_off, const int32_t* __restrict__ bnd,
    int NB, const uint64_t* __restrict__ post, const int32_t* __restrict__ dlen,
    const uint8_t* __restrict__ elig, int64_t rows, const float* __restrict__ avgdl_p, float k1,
    float b, int* __restrict__ kcnt, const int64_t* __restrict__ koff, uint64_t* __restrict__ keys) {
  extern __shared__ __attribute__((aligned(16))) uint32_t acc[];
  const int q = blockIdx.x, blk = blockIdx.y, tid = threadIdx.x, lane = tid & 63;
  const int s0 = slot_off[q], s1 = slot_off[q + 1];
  // The query's terms are handled in batches of 64 slots: their block ranges [lo, hi) come in with
  // one parallel load into LDS, and the batch's postings are processed as ONE flat range (a term
  // has few postings per 8192-row block: a loop per term left most threads idle and chained a
  // dependent load per term).
  constexpr int TB = 64;
  __shared__ int s_lo[TB], s_pre[TB + 1], s_total;
  __shared__ LexTerm s_term[TB];
  if (tid == 0) s_total = 0;
  __syncthreads();
  int mine_total = 0;
  for (int t = s0 + tid; t < s1; t += LEX_THREADS)
    mine_total += bnd[(int64_t)t * (NB + 1) + blk + 1] - bnd[(int64_t)t * (NB + 1) + blk];
  mine_total = (int)wave_sum((float)mine_total);  // exact: counts < 2^24 per workgroup
  if (lane == 0 && mine_total) atomicAdd(&s_total, mine_total);
  __syncthreads();
  if (s_total == 0) return;  // uniform: no posting of this query in this row block
  for (int i = tid; i < LEX_RB; i += LEX_THREADS) acc[i] = 0u;
  const float avgdl = *avgdl_p;  // (host path: uploaded; device path: lex_qprep_kernel)
  const float one_minus_b = 1.f - b, k1p1 = k1 + 1.f;
  const int64_t r0 = (int64_t)blk * LEX_RB;
  for (int tb = s0; tb < s1; tb += TB) {
    const int nt = s1 - tb < TB ? s1 - tb : TB;
    __syncthreads();  // previous batch done with s_*
    if (tid < nt) {
      const int t = tb + tid;
      const int lo = bnd[(int64_t)t * (NB + 1) + blk], hi = bnd[(int64_t)t * (NB + 1) + blk + 1];
      s_lo[tid] = lo;
      s_pre[tid + 1] = hi - lo;
      s_term[tid] = terms[t];
    }
    __syncthreads();
    if (tid == 0) {
      s_pre[0] = 0;
      for (int i = 0; i < nt; ++i) s_pre[i + 1] += s_pre[i];
    }
    __syncthreads();
    const int tot = s_pre[nt];
    for (int p = tid; p < tot; p += LEX_THREADS) {
      int lo_t = 0, hi_t = nt - 1;  // term of flat posting p: last t with s_pre[t] <= p
      while (lo_t < hi_t) {
        const int mid = (lo_t + hi_t + 1) >> 1;
        if (s_pre[mid] <= p) lo_t = mid;
        else hi_t = mid - 1;
      }
      const LexTerm& e = s_term[lo_t];
      const uint64_t v = post[e.start + s_lo[lo_t] + (p - s_pre[lo_t])];
      const uint32_t row = (uint32_t)(v >> 32);
      if (elig && !elig[row]) continue;
      const float tf = (float)(uint32_t)v;
      const float dl = (float)dlen[row];
      const uint32_t sc = bm25_fixed(e.idf, tf, dl, avgdl, k1, b, one_minus_b, k1p1) * (uint32_t)e.mult;
      atomicAdd(&acc[row - r0], sc);
    }
  }
  __syncthreads();
  // wave w owns the contiguous entries [w * SPAN, (w + 1) * SPAN): count, one global atomic per
  // workgroup (the per-query counter is shared by all NB workgroups of the query), then write
  constexpr int SPAN = LEX_RB / (LEX_THREADS / 64);
  __shared__ int wave_cnt[LEX_THREADS / 64];
  __shared__ int wg_base;
  const int wave = tid >> 6;
  const uint32_t* mine = acc + wave * SPAN;
  int cnt = 0;
  for (int i = lane; i < SPAN; i += 64) cnt += __popcll(__ballot(mine[i] != 0u));
  if (lane == 0) wave_cnt[wave] = cnt;
  __syncthreads();
  if (tid == 0) {
    int tot = 0;
    for (int w = 0; w < LEX_THREADS / 64; ++w) {
      const int c = wave_cnt[w];
      wave_cnt[w] = tot;
      tot += c;
    }
    wg_base = atomicAdd(&kcnt[q], tot);
  }
  __syncthreads();
  uint64_t* kl = keys + koff[q] + wg_base + wave_cnt[wave];
  for (int i = lane; i < SPAN; i += 64) {
    const uint32_t sc = mine[i];
    const bool hit = sc != 0u;
    const uint64_t bal = __ballot(hit);
    if (hit) {
      const uint32_t row = (uint32_t)(r0 + wave * SPAN + i);
      kl[__popcll(bal & ((1ull << lane) - 1ull))] = ((uint64_t)sc << 32) | (uint64_t)(0xffffffffu - row);
    }
    kl += __popcll(bal);
  }
}

// ---- device-resident query preparation (padded query-token matrix) ------------------------------
// The host path (LexIndex::search_dev) builds the per-query term slots, idf and key offsets on the
// host from its df mirror.  For a batch whose query tokens are already on the device (the hybrid
// pipeline) that would mean a device -> host copy and a synchronisation in the middle of a step;
// these kernels do the same on the device from the inverted index's offsets.
//
// lex_qstats_kernel: out[0] = live rows, out[1] = summed document length (this index), out[2 +
//   q Lq + i] = live document frequency of query q's i-th token (0 past its length / unknown): the
//   vector a row-sharded corpus all-reduces into corpus-wide statistics.
__global__ void lex_qstats_kernel(const int32_t* __restrict__ tok, const int32_t* __restrict__ qlen,
                                  int B, int Lq, const int64_t* __restrict__ off, int64_t T,
                                  int64_t n_live, int64_t sum_dl, int64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    out[0] = n_live;
    out[1] = sum_dl;
  }
  if (i >= (int64_t)B * Lq) return;
  const int q = (int)(i / Lq), p = (int)(i % Lq);
  const int32_t t = tok[i];
  out[2 + i] = (p < qlen[q] && t >= 0 && t < T) ? off[t + 1] - off[t] : 0;
}

// lex_qcap_kernel: caps[q] = min(sum of the postings of query q's distinct terms, rows) -- the
// candidate keys lex_qprep_kernel will reserve for it -- for a whole batch (one thread per query),
// so a batch whose worst case does not fit one query group is grouped by its actual caps.
__global__ void lex_qcap_kernel(const int32_t* __restrict__ tok, const int32_t* __restrict__ qlen,
                                int B, int Lq, const int64_t* __restrict__ off, int64_t T,
                                int64_t rows, int64_t* __restrict__ caps) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= B) return;
  const int32_t* tq = tok + (int64_t)q * Lq;
  const int L = min(max(qlen[q], 0), Lq);
  int64_t cap = 0;
  for (int i = 0; i < L; ++i) {
    const int32_t t = tq[i];
    if (t < 0 || t >= T) continue;
    bool first = true;
    for (int j = 0; j < i && first; ++j) first = tq[j] != t;
    if (first) cap += off[t + 1] - off[t];
  }
  caps[q] = cap < rows ? cap : rows;
}

// lex_qprep_kernel: one workgroup, thread q = query q of the group (G <= 1024).  Slot q Lq + i is
// the query's i-th token if that is its FIRST occurrence of a term with postings here (start, len,
// idf, multiplicity = occurrences in the query), else empty (len 0): the host path's slots in the
// same order.  idf uses the corpus-wide df / N when gst is given (gst[0], gst[1], gst[2 + df_base +
// q Lq + i] as written by lex_qstats_kernel for the whole batch and summed over the shards; df_base
// = the group's first query x Lq), else this index's.  koff = exclusive
// scan of cap = min(sum of len, rows); kcnt = 0; *avgdl_out = sum_dl / N as the host computes it.
__device__ __forceinline__ float lex_idf_dev(int64_t df, int64_t n_live) {
  const double N = (double)n_live, d = (double)df;
  return (float)log(1.0 + (N - d + 0.5) / (d + 0.5));
}

__global__ __launch_bounds__(1024) void lex_qprep_kernel(
    const int32_t* __restrict__ tok, const int32_t* __restrict__ qlen, int G, int Lq,
    const int64_t* __restrict__ off, int64_t T, int64_t rows, int64_t n_live, int64_t sum_dl,
    const int64_t* __restrict__ gst, int64_t df_base, LexTerm* __restrict__ slots,
    int* __restrict__ slot_off,
    int64_t* __restrict__ koff, int* __restrict__ kcnt, float* __restrict__ avgdl_out) {
  __shared__ int64_t s_wave[16];
  const int q = threadIdx.x, lane = q & 63, wave = q >> 6;
  const int64_t N = gst ? gst[0] : n_live;
  const int64_t sdl = gst ? gst[1] : sum_dl;
  int64_t cap = 0;
  if (q < G) {
    const int32_t* tq = tok + (int64_t)q * Lq;
    const int L = min(max(qlen[q], 0), Lq);
    for (int i = 0; i < Lq; ++i) {
      LexTerm e = {0, 0, 0.f, 0, 0};
      const int32_t t = tq[i];
      if (i < L && t >= 0 && t < T) {
        const int64_t st = off[t], len = off[t + 1] - st;
        bool first = len > 0;
        for (int j = 0; j < i && first; ++j) first = tq[j] != t;
        if (first) {
          int mult = 0;
          for (int j = i; j < L; ++j) mult += tq[j] == t ? 1 : 0;
          const int64_t df = gst ? gst[2 + df_base + (int64_t)q * Lq + i] : len;
          e = {st, (int32_t)len, lex_idf_dev(df, N), mult, 0};
          cap += len;
        }
      }
      slots[(int64_t)q * Lq + i] = e;
    }
    cap = cap < rows ? cap : rows;
    kcnt[q] = 0;
    slot_off[q] = q * Lq;
  }
  // exclusive scan of cap over the group (waves of 64, then the wave totals)
  int64_t incl = cap;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  int64_t base = 0;
  for (int w = 0; w < wave; ++w) base += s_wave[w];
  if (q < G) koff[q] = base + incl - cap;
  if (q == G - 1) {
    koff[G] = base + incl;
    slot_off[G] = G * Lq;
  }
  if (q == 0) *avgdl_out = N > 0 ? (float)((double)sdl / (double)N) : 1.f;
}

// ---- L2 -----------------------------------------------------------------------------------------
// Two passes over the query's candidate keys instead of up to eight radix passes over HBM:
//   pass 1: LDS histogram of a monotone 12-bit log-linear bin of every touched score;
//   wave 0: the highest bin T with count(bin >= T) >= k (suffix scan over the 4096 bins);
//   pass 2: keys with bin >= T are collected into LDS, then the exact block top-k runs on them.
// If more than LSEL_CAP keys share the top bins (ties), the exact radix select runs over the
// keys in HBM instead.
constexpr int LSEL_BINS = 4096;
constexpr int LSEL_CAP = 8192;

__device__ __forceinline__ int score_bin(uint32_t s) {
  const int e = 31 - __clz(s);  // s >= 1
  if (e < 7) return (int)s;     // 1 .. 127 exact
  return ((e - 6) << 7) | (int)((s >> (e - 7)) & 127u);  // <= 25 << 7 | 127 < 4096
}

struct LexSelSmem {
  int hist[LSEL_BINS];
  uint64_t keys[LSEL_CAP];
  SelShared sh;
  int thr, n_ge, nkeys;
};

__global__ __launch_bounds__(SEL_THREADS, 1) void lex_select_kernel(
    const uint64_t* __restrict__ keys, const int* __restrict__ kcnt,
    const int64_t* __restrict__ koff, int k, float* __restrict__ out_score,
    int64_t* __restrict__ out_rows, int64_t row_offset, uint32_t* __restrict__ out_fixed) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  LexSelSmem& S = *reinterpret_cast<LexSelSmem*>(smem_raw);
  const int q = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const uint64_t* kl = keys + koff[q];
  const int n = kcnt[q];
  for (int i = tid; i < LSEL_BINS; i += blockDim.x) S.hist[i] = 0;
  if (tid == 0) S.nkeys = 0;
  __syncthreads();
  for (int i = tid; i < n; i += blockDim.x) atomicAdd(&S.hist[score_bin((uint32_t)(kl[i] >> 32))], 1);
  __syncthreads();
  if (tid < 64) {
    // lane l owns bins [64 l, 64 l + 64); suffix counts from the top bin down
    int c = 0;
    for (int j = 0; j < 64; ++j) c += S.hist[64 * lane + j];
    int suf = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_down(suf, o, 64);
      if (lane + o < 64) suf += v;
    }
    const int kk = n < k ? n : k;
    const uint64_t bal = __ballot(suf >= kk && kk > 0);
    if (tid == 0) {
      S.thr = 0;
      S.n_ge = n;
    }
    if (bal) {
      const int L = 63 - __clzll(bal);
      if (lane == L) {
        int above = suf - c;  // keys in bins of higher lanes
        int t = 64 * lane;
        for (int j = 63; j >= 0; --j) {
          above += S.hist[64 * lane + j];
          if (above >= kk) {
            t = 64 * lane + j;
            break;
          }
        }
        S.thr = t;
        S.n_ge = above;
      }
    }
  }
  __syncthreads();
  const int thr = S.thr;
  int m;
  if (S.n_ge <= LSEL_CAP) {
    for (int i = tid; i < n; i += blockDim.x) {
      const uint64_t key = kl[i];
      if (score_bin((uint32_t)(key >> 32)) >= thr) S.keys[atomicAdd(&S.nkeys, 1)] = key;
    }
    __syncthreads();
    m = block_topk([&](int i) { return S.keys[i]; }, S.nkeys, k, S.sh);
  } else {
    m = block_topk([&](int i) { return kl[i]; }, n, k, S.sh);
  }
  for (int i = tid; i < k; i += blockDim.x) {
    const bool ok = i < m;
    const uint64_t kk = ok ? S.sh.sel[i] : 0ull;
    out_score[(int64_t)q * k + i] = ok ? (float)(uint32_t)(kk >> 32) / LEX_SCALE : -INFINITY;
    out_rows[(int64_t)q * k + i] = ok ? (int64_t)(0xffffffffu - (uint32_t)kk) + row_offset : -1;
    // the exact 2^-16 fixed-point score (fp32 rounds it once it passes 2^24, a score of 256):
    // what a sharded index merges on to keep one index's order
    if (out_fixed) out_fixed[(int64_t)q * k + i] = ok ? (uint32_t)(kk >> 32) : 0u;
  }
}

// ---- F1 -----------------------------------------------------------------------------------------
constexpr int RRF_THREADS = 256;
constexpr int RRF_MAX = 2 * SR_MAX_TOPK;

__global__ __launch_bounds__(RRF_THREADS) void rrf_fuse_kernel(
    const int64_t* __restrict__ rows_a, int ka, const int64_t* __restrict__ rows_b, int kb,
    int rank_const, double min_score, int k_out, double* __restrict__ out_score,
    int64_t* __restrict__ out_rows) {
  __shared__ int64_t row[RRF_MAX];
  __shared__ double score[RRF_MAX];
  __shared__ int match[SR_MAX_TOPK];   // b item j: index in a, or -1
  __shared__ int newpos[SR_MAX_TOPK];  // b item j (unmatched): its item index
  __shared__ int na_s, nb_s, n_s;
  const int q = blockIdx.x, tid = threadIdx.x;
  const int64_t* ra = rows_a + (int64_t)q * ka;
  const int64_t* rb = rows_b + (int64_t)q * kb;
  if (tid == 0) {
    int na = 0, nb = 0;
    while (na < ka && ra[na] >= 0) ++na;  // lists are -1 padded after their valid prefix
    while (nb < kb && rb[nb] >= 0) ++nb;
    na_s = na;
    nb_s = nb;
  }
  __syncthreads();
  const int na = na_s, nb = nb_s;
  for (int i = tid; i < na; i += RRF_THREADS) {
    row[i] = ra[i];
    score[i] = 0.0 + 1.0 / (double)(i + rank_const);
  }
  for (int j = tid; j < nb; j += RRF_THREADS) {
    const int64_t r = rb[j];
    int m = -1;
    for (int i = 0; i < na; ++i)
      if (ra[i] == r) {
        m = i;
        break;
      }
    match[j] = m;
  }
  __syncthreads();
  if (tid == 0) {
    // new rows of list b keep b's order after a's rows (dict insertion order)
    int n = na;
    for (int j = 0; j < nb; ++j) newpos[j] = match[j] < 0 ? n++ : -1;
    n_s = n;
  }
  __syncthreads();
  for (int j = tid; j < nb; j += RRF_THREADS) {
    const double add = 1.0 / (double)(j + rank_const);
    if (match[j] >= 0) {
      score[match[j]] = score[match[j]] + add;  // a row appears at most once per list
    } else {
      row[newpos[j]] = rb[j];
      score[newpos[j]] = 0.0 + add;
    }
  }
  __syncthreads();
  const int n = n_s;
  // rank = items strictly before this one in (score desc, insertion asc) order
  for (int i = tid; i < n; i += RRF_THREADS) {
    const double s = score[i];
    int rank = 0;
    for (int j = 0; j < n; ++j) rank += (score[j] > s || (score[j] == s && j < i)) ? 1 : 0;
    if (rank < k_out) {
      const bool keep = s >= min_score;
      out_score[(int64_t)q * k_out + rank] = keep ? s : -INFINITY;
      out_rows[(int64_t)q * k_out + rank] = keep ? row[i] : -1;
    }
  }
  for (int i = n + tid; i < k_out; i += RRF_THREADS) {
    out_score[(int64_t)q * k_out + i] = -INFINITY;
    out_rows[(int64_t)q * k_out + i] = -1;
  }
}

void launch_rrf_fuse(const int64_t* rows_a, int ka, const int64_t* rows_b, int kb, int B,
                     int rank_const, double min_score, int k_out, double* out_score,
                     int64_t* out_rows, hipStream_t s) {
  SR_CHECK(ka >= 0 && ka <= SR_MAX_TOPK && kb >= 0 && kb <= SR_MAX_TOPK, "rrf: list length > 1024");
  SR_CHECK(k_out >= 1 && k_out <= RRF_MAX, "rrf: k_out must be in [1, 2048]");
  SR_CHECK(rank_const >= 1, "rrf: rank_const must be >= 1");
  if (B <= 0) return;
  ProfScope prof("rrf_fuse", s, 0.0, (double)B * (ka + kb) * 8.0);
  hipLaunchKernelGGL(rrf_fuse_kernel, dim3(B), dim3(RRF_THREADS), 0, s, rows_a, ka, rows_b, kb,
                     rank_const, min_score, k_out, out_score, out_rows);
  SR_LAUNCH_CHECK();
}

// ================================================================================================
// LexIndex
LexIndex::LexIndex(int device, float k1, float b) : device_(device), k1_(k1), b_(b) {
  SR_CHECK(k1 >= 0.f && b >= 0.f && b <= 1.f, "lex: need k1 >= 0 and 0 <= b <= 1");
  DeviceGuard g(device_);
  SR_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  SR_HIP(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  SR_HIP(hipEventRecord(done_, stream_));
}

LexIndex::~LexIndex() {
  DeviceGuard g(device_);
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    (void)hipStreamDestroy(stream_);
  }
  if (done_) (void)hipEventDestroy(done_);
}

static void grow_copy(DevBuf& buf, size_t used_bytes, size_t need_bytes, hipStream_t s) {
  if (need_bytes <= buf.bytes) return;
  size_t cap = std::max<size_t>(need_bytes, std::max<size_t>(buf.bytes * 2, 1 << 16));
  DevBuf nb;
  nb.reserve(cap);
  if (used_bytes) SR_HIP(hipMemcpyAsync(nb.p, buf.p, used_bytes, hipMemcpyDeviceToDevice, s));
  SR_HIP(hipStreamSynchronize(s));
  std::swap(buf.p, nb.p);
  std::swap(buf.bytes, nb.bytes);
}

void LexIndex::add(const int64_t* off, const int32_t* terms, const int32_t* tf, const int32_t* dl,
                   int64_t n, int64_t* first_row) {
  SR_CHECK(n >= 0, "lex.add: negative count");
  if (first_row) *first_row = rows_;
  if (n == 0) return;
  SR_CHECK(off && dl && off[0] == 0, "lex.add: off[0] must be 0");
  const int64_t P = off[n];
  SR_CHECK(P >= 0 && (P == 0 || (terms && tf)), "lex.add: null term arrays");
  SR_CHECK(rows_ + n <= (int64_t)0x7fffffff, "lex.add: more than 2^31 rows");
  std::vector<uint64_t> val((size_t)P);
  for (int64_t i = 0; i < n; ++i) {
    SR_CHECK(off[i + 1] >= off[i], "lex.add: off must be non-decreasing");
    SR_CHECK(dl[i] >= 0, "lex.add: negative document length");
    for (int64_t p = off[i]; p < off[i + 1]; ++p) {
      SR_CHECK(terms[p] >= 0 && terms[p] < kLexMaxVocab, "lex.add: term id out of range [0, 2^26)");
      SR_CHECK(tf[p] >= 1, "lex.add: term frequency must be >= 1");
      val[(size_t)p] = ((uint64_t)(rows_ + i) << 32) | (uint32_t)tf[p];
      vocab_ = std::max<int64_t>(vocab_, (int64_t)terms[p] + 1);
    }
  }
  DeviceGuard g(device_);
  begin(stream_);
  grow_copy(fterm_, (size_t)P_ * 4, (size_t)(P_ + P) * 4, stream_);
  grow_copy(fval_, (size_t)P_ * 8, (size_t)(P_ + P) * 8, stream_);
  grow_copy(dlen_, (size_t)rows_ * 4, (size_t)(rows_ + n) * 4, stream_);
  grow_copy(live_, (size_t)rows_, (size_t)(rows_ + n), stream_);
  if (P) {
    SR_HIP(hipMemcpyAsync(fterm_.as<int32_t>() + P_, terms, (size_t)P * 4, hipMemcpyHostToDevice, stream_));
    SR_HIP(hipMemcpyAsync(fval_.as<uint64_t>() + P_, val.data(), (size_t)P * 8, hipMemcpyHostToDevice, stream_));
  }
  SR_HIP(hipMemcpyAsync(dlen_.as<int32_t>() + rows_, dl, (size_t)n * 4, hipMemcpyHostToDevice, stream_));
  SR_HIP(hipMemsetAsync(live_.as<uint8_t>() + rows_, 1, (size_t)n, stream_));
  SR_HIP(hipStreamSynchronize(stream_));
  end(stream_);
  for (int64_t i = 0; i < n; ++i) {
    dl_host_.push_back(dl[i]);
    live_host_.push_back(1);
    sum_dl_ += dl[i];
  }
  rows_ += n;
  live_n_ += n;
  P_ += P;
  dirty_ = true;
  ++version_;
}

void LexIndex::remove(const int64_t* rows, int64_t n) {
  for (int64_t i = 0; i < n; ++i)
    SR_CHECK(rows[i] >= 0 && rows[i] < rows_, "lex.remove: row out of range");
  for (int64_t i = 0; i < n; ++i) {
    const int64_t r = rows[i];
    if (!live_host_[(size_t)r]) continue;
    live_host_[(size_t)r] = 0;
    --live_n_;
    sum_dl_ -= dl_host_[(size_t)r];
  }
  DeviceGuard g(device_);
  begin(stream_);
  if (rows_) SR_HIP(hipMemcpyAsync(live_.p, live_host_.data(), (size_t)rows_, hipMemcpyHostToDevice, stream_));
  SR_HIP(hipStreamSynchronize(stream_));
  end(stream_);
  dirty_ = true;
  ++version_;
}

void LexIndex::rebuild(hipStream_t s) {
  if (!dirty_) return;
  const int64_t T = vocab_;
  df_host_.assign((size_t)T, 0);
  nnz_ = 0;
  off_.reserve((size_t)(T + 1) * 8);
  if (P_ == 0 || T == 0) {
    max_df_ = 0;
    off_host_.assign((size_t)T + 1, 0);
    SR_HIP(hipMemsetAsync(off_.p, 0, (size_t)(T + 1) * 8, s));
    SR_HIP(hipStreamSynchronize(s));
    dirty_ = false;
    return;
  }
  SR_CHECK(P_ <= (int64_t)0x7fffffff, "lex: more than 2^31 postings per index");
  const int P = (int)P_;
  int end_bit = 1;
  while (end_bit < 32 && ((uint64_t)1 << end_bit) <= (uint64_t)T) ++end_bit;  // keys 0..T
  DevBuf keys_in, keys_out, tmp;
  keys_in.reserve((size_t)P * 4);
  keys_out.reserve((size_t)P * 4);
  post_.reserve((size_t)P * 8);
  {
    ProfScope prof("lex_rebuild_keys", s, 0.0, (double)P * 16.0);
    hipLaunchKernelGGL(lex_keys_kernel, dim3((unsigned)ceil_div(P, 256)), dim3(256), 0, s,
                       fterm_.as<int32_t>(), fval_.as<uint64_t>(), live_.as<uint8_t>(), (int64_t)P,
                       (uint32_t)T, keys_in.as<uint32_t>());
    SR_LAUNCH_CHECK();
  }
  size_t tb_sort = 0;
  SR_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, keys_in.as<uint32_t>(),
                                            keys_out.as<uint32_t>(), fval_.as<uint64_t>(),
                                            post_.as<uint64_t>(), P, 0, end_bit, s));
  tmp.reserve(tb_sort);
  {
    ProfScope prof("lex_rebuild_sort", s, 0.0, (double)P * 24.0);
    SR_HIP(hipcub::DeviceRadixSort::SortPairs(tmp.p, tb_sort, keys_in.as<uint32_t>(),
                                              keys_out.as<uint32_t>(), fval_.as<uint64_t>(),
                                              post_.as<uint64_t>(), P, 0, end_bit, s));
  }
  hipLaunchKernelGGL(lex_offsets_kernel, dim3((unsigned)ceil_div(T + 1, 256)), dim3(256), 0, s,
                     keys_out.as<uint32_t>(), (int64_t)P, T, off_.as<int64_t>());
  SR_LAUNCH_CHECK();
  off_host_.resize((size_t)T + 1);
  SR_HIP(hipMemcpyAsync(off_host_.data(), off_.p, (size_t)(T + 1) * 8, hipMemcpyDeviceToHost, s));
  SR_HIP(hipStreamSynchronize(s));
  nnz_ = off_host_[(size_t)T];
  max_df_ = 0;
  for (int64_t t = 0; t < T; ++t) {
    df_host_[(size_t)t] = (int32_t)(off_host_[(size_t)t + 1] - off_host_[(size_t)t]);
    max_df_ = std::max<int64_t>(max_df_, df_host_[(size_t)t]);
  }
  dirty_ = false;
}

const uint8_t* LexIndex::eligibility(const uint8_t* allow, int64_t mask_key, hipStream_t s) {
  if (!allow) return nullptr;  // postings of dead rows are gone after the rebuild
  if (mask_key == 0 || mask_key != mask_key_ || mask_version_ != version_) {
    std::vector<uint8_t> m((size_t)std::max<int64_t>(rows_, 1));
    for (int64_t r = 0; r < rows_; ++r) m[(size_t)r] = (live_host_[(size_t)r] && allow[r]) ? 1 : 0;
    mask_.reserve(m.size());
    SR_HIP(hipMemcpyAsync(mask_.p, m.data(), (size_t)rows_, hipMemcpyHostToDevice, s));
    SR_HIP(hipStreamSynchronize(s));
    mask_key_ = mask_key;
    mask_version_ = version_;
  }
  return mask_.as<uint8_t>();
}

float LexIndex::idf(int64_t df, int64_t n_live) {
  // Lucene's BM25 idf (always positive), in double then rounded to fp32 once.
  const double N = (double)n_live, d = (double)df;
  return (float)std::log(1.0 + (N - d + 0.5) / (d + 0.5));
}

float LexIndex::avgdl(int64_t sum_dl, int64_t n_live) {
  return n_live > 0 ? (float)((double)sum_dl / (double)n_live) : 1.f;
}

void LexIndex::totals(int64_t* n_live, int64_t* sum_dl) const {
  if (n_live) *n_live = live_n_;
  if (sum_dl) *sum_dl = sum_dl_;
}

void LexIndex::df(const int32_t* terms, int n, int64_t* out) {
  DeviceGuard g(device_);
  begin(stream_);
  rebuild(stream_);
  end(stream_);
  for (int i = 0; i < n; ++i) {
    const int32_t t = terms[i];
    out[i] = (t >= 0 && t < vocab_) ? df_host_[(size_t)t] : 0;
  }
}

void LexIndex::search_dev(const int64_t* qoff, const int32_t* qterms, int B, int k,
                          const uint8_t* allow, int64_t mask_key, float* out_score,
                          int64_t* out_rows, hipStream_t s, const sr_lex_global* glob,
                          int64_t row_offset, uint32_t* out_fixed) {
  SR_CHECK(B >= 0, "lex.search: negative batch");
  SR_CHECK(k >= 1 && k <= SR_MAX_TOPK, "lex.search: top_k must be in [1, 1024]");
  if (B == 0) return;
  SR_CHECK(qoff && qoff[0] == 0, "lex.search: qoff[0] must be 0");
  DeviceGuard g(device_);
  begin(s);
  rebuild(s);
  const uint8_t* elig = eligibility(allow, mask_key, s);
  // per query: distinct known terms with multiplicity, and the touched-list capacity
  struct QT {
    int32_t term, mult;
  };
  std::vector<std::vector<QT>> qt((size_t)B);
  std::vector<int64_t> cap((size_t)B, 0);
  for (int b = 0; b < B; ++b) {
    SR_CHECK(qoff[b + 1] >= qoff[b], "lex.search: qoff must be non-decreasing");
    std::vector<QT>& v = qt[(size_t)b];
    for (int64_t p = qoff[b]; p < qoff[b + 1]; ++p) {
      const int32_t t = qterms[p];
      if (t < 0 || t >= vocab_ || df_host_[(size_t)t] == 0) continue;
      bool seen = false;
      for (auto& e : v)
        if (e.term == t) {
          ++e.mult;
          seen = true;
        }
      if (!seen) {
        v.push_back({t, 1});
        cap[(size_t)b] += df_host_[(size_t)t];
      }
    }
    cap[(size_t)b] = std::min<int64_t>(cap[(size_t)b], rows_);
  }
  // statistics: this index's live rows, or the caller's corpus-wide ones (row-sharded corpus:
  // every shard then scores with the same N, avgdl and df, so merged results equal one index's)
  int64_t N_live = live_n_, sum_dl = sum_dl_;
  std::vector<std::pair<int32_t, int64_t>> gdf;
  if (glob) {
    SR_CHECK(glob->n_live >= 0 && glob->sum_dl >= 0 && (glob->n_terms == 0 || (glob->terms && glob->df)),
             "lex.search: invalid global statistics");
    N_live = glob->n_live;
    sum_dl = glob->sum_dl;
    gdf.reserve((size_t)glob->n_terms);
    for (int i = 0; i < glob->n_terms; ++i) gdf.push_back({glob->terms[i], glob->df[i]});
    std::sort(gdf.begin(), gdf.end());
  }
  auto term_df = [&](int32_t t) -> int64_t {
    if (!glob) return df_host_[(size_t)t];
    auto it = std::lower_bound(gdf.begin(), gdf.end(), std::make_pair(t, (int64_t)INT64_MIN));
    SR_CHECK(it != gdf.end() && it->first == t, "lex.search: query term missing from the global df table");
    return it->second;
  };
  // query blocks: candidate keys within LEX_KEY_BUDGET; grid (queries, row blocks), so the
  // workgroups in flight belong to many queries
  const int64_t rows = std::max<int64_t>(rows_, 1);
  const int NB = (int)ceil_div(rows, LEX_RB);
  SR_CHECK(NB <= 65535, "lex.search: more than 2^30 rows per index");
  const float adl = avgdl(sum_dl, N_live);
  static bool attr_set = false;
  if (!attr_set) {
    SR_HIP(hipFuncSetAttribute((const void*)lex_score_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, LEX_RB * 4));
    SR_HIP(hipFuncSetAttribute((const void*)lex_select_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(LexSelSmem)));
    attr_set = true;
  }
  for (int b0 = 0; b0 < B;) {
    int qb = 0;
    int64_t nkeys = 0;
    while (b0 + qb < B && qb < 65535 && (qb == 0 || nkeys + cap[(size_t)(b0 + qb)] <= LEX_KEY_BUDGET))
      nkeys += cap[(size_t)(b0 + qb++)];
    std::vector<int64_t> koff((size_t)qb + 1, 0);
    std::vector<int> slot_off((size_t)qb + 1, 0);
    std::vector<LexTerm> slots;
    int64_t scored = 0;
    for (int i = 0; i < qb; ++i) {
      koff[(size_t)i + 1] = koff[(size_t)i] + cap[(size_t)(b0 + i)];
      for (const QT& e : qt[(size_t)(b0 + i)]) {
        const int64_t len = df_host_[(size_t)e.term];
        slots.push_back({off_host_[(size_t)e.term], (int32_t)len, idf(term_df(e.term), N_live), e.mult, 0});
        scored += len;
      }
      slot_off[(size_t)i + 1] = (int)slots.size();
    }
    const int nslots = (int)slots.size();
    const size_t b_sl = std::max<size_t>(slots.size(), 1) * sizeof(LexTerm);
    const size_t b_so = (size_t)(qb + 1) * 4, b_ko = (size_t)(qb + 1) * 8, b_cnt = (size_t)qb * 4;
    const size_t b_bnd = (size_t)std::max(nslots, 1) * (NB + 1) * 4;
    const size_t b_keys = (size_t)std::max<int64_t>(koff[(size_t)qb], 1) * 8;
    size_t o = 0;
    auto carve = [&](size_t bytes) {
      const size_t at = o;
      o += (size_t)round_up((int64_t)bytes, 256);
      return at;
    };
    const size_t o_sl = carve(b_sl), o_so = carve(b_so), o_ko = carve(b_ko), o_cnt = carve(b_cnt),
                 o_bnd = carve(b_bnd), o_keys = carve(b_keys), o_avg = carve(4);
    ws_.reserve(o);
    char* w = ws_.as<char>();
    LexTerm* d_sl = reinterpret_cast<LexTerm*>(w + o_sl);
    int* d_so = reinterpret_cast<int*>(w + o_so);
    int64_t* d_ko = reinterpret_cast<int64_t*>(w + o_ko);
    int* d_cnt = reinterpret_cast<int*>(w + o_cnt);
    int32_t* d_bnd = reinterpret_cast<int32_t*>(w + o_bnd);
    uint64_t* d_keys = reinterpret_cast<uint64_t*>(w + o_keys);
    float* d_avg = reinterpret_cast<float*>(w + o_avg);
    uint32_t adl_bits;
    std::memcpy(&adl_bits, &adl, 4);
    SR_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_avg), (int)adl_bits, 1, s));
    if (nslots) SR_HIP(hipMemcpyAsync(d_sl, slots.data(), slots.size() * sizeof(LexTerm), hipMemcpyHostToDevice, s));
    SR_HIP(hipMemcpyAsync(d_so, slot_off.data(), b_so, hipMemcpyHostToDevice, s));
    SR_HIP(hipMemcpyAsync(d_ko, koff.data(), b_ko, hipMemcpyHostToDevice, s));
    SR_HIP(hipMemsetAsync(d_cnt, 0, b_cnt, s));
    if (nslots) {
      const int64_t nb = (int64_t)nslots * (NB + 1);
      hipLaunchKernelGGL(lex_bounds_kernel, dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, s, d_sl,
                         nslots, NB, post_.as<uint64_t>(), d_bnd);
      SR_LAUNCH_CHECK();
      ProfScope prof("lex_score", s, 0.0, (double)scored * 12.0);
      hipLaunchKernelGGL(lex_score_kernel, dim3((unsigned)qb, (unsigned)NB), dim3(LEX_THREADS),
                         LEX_RB * 4, s, d_sl, d_so, d_bnd, NB, post_.as<uint64_t>(),
                         dlen_.as<int32_t>(), elig, rows_, d_avg, k1_, b_, d_cnt, d_ko, d_keys);
      SR_LAUNCH_CHECK();
    }
    {
      ProfScope prof("lex_select", s, 0.0, (double)koff[(size_t)qb] * 8.0);
      hipLaunchKernelGGL(lex_select_kernel, dim3(qb), dim3(SEL_THREADS), sizeof(LexSelSmem), s,
                         d_keys, d_cnt, d_ko, k, out_score + (int64_t)b0 * k,
                         out_rows + (int64_t)b0 * k, row_offset,
                         out_fixed ? out_fixed + (int64_t)b0 * k : nullptr);
      SR_LAUNCH_CHECK();
    }
    // the host vectors above back async copies: finish the block before they go away
    SR_HIP(hipStreamSynchronize(s));
    b0 += qb;
  }
  end(s);
}

void LexIndex::query_stats_dev(const int32_t* tok, const int32_t* qlen, int B, int Lq,
                               int64_t* out, hipStream_t s) {
  SR_CHECK(B >= 0 && Lq >= 0, "lex.query_stats: negative shape");
  DeviceGuard g(device_);
  begin(s);
  rebuild(s);
  off_.reserve(8);
  const int64_t n = (int64_t)B * Lq;
  hipLaunchKernelGGL(lex_qstats_kernel, dim3((unsigned)std::max<int64_t>(1, ceil_div(n, 256))), dim3(256),
                     0, s, tok, qlen, B, Lq, off_.as<int64_t>(), vocab_, live_n_, sum_dl_, out);
  SR_LAUNCH_CHECK();
  end(s);
}

void LexIndex::search_tok_dev(const int32_t* tok, const int32_t* qlen, int B, int Lq, int k,
                              const int64_t* gstats, float* out_score, int64_t* out_rows,
                              hipStream_t s, int64_t row_offset) {
  SR_CHECK(B >= 0 && Lq >= 0, "lex.search_tok: negative shape");
  SR_CHECK(k >= 1 && k <= SR_MAX_TOPK, "lex.search: top_k must be in [1, 1024]");
  if (B == 0) return;
  DeviceGuard g(device_);
  begin(s);
  rebuild(s);
  off_.reserve(8);
  const int64_t rows = std::max<int64_t>(rows_, 1);
  const int NB = (int)ceil_div(rows, LEX_RB);
  SR_CHECK(NB <= 65535, "lex.search: more than 2^30 rows per index");
  static bool attr_set = false;
  if (!attr_set) {
    SR_HIP(hipFuncSetAttribute((const void*)lex_score_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, LEX_RB * 4));
    SR_HIP(hipFuncSetAttribute((const void*)lex_select_kernel,
                               hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(LexSelSmem)));
    attr_set = true;
  }
  // keys per query <= min(Lq * max df, rows), known on the host without looking at the queries:
  // query groups of G <= 1024 sized so the group's keys stay within LEX_KEY_BUDGET.  A batch that
  // fits one such group runs without a host round trip.  Otherwise (a stopword-like term makes the
  // worst case the whole index: ~42 queries per group at 6.25M rows, a 2 GiB key workspace and
  // bounds / score launches over padded slots) the actual per-query caps are computed on the
  // device (lex_qcap_kernel), read back once, and the batch is grouped by them, as search_dev does.
  const int64_t per_q = std::max<int64_t>(1, std::min<int64_t>((int64_t)Lq * max_df_, rows_));
  const int G_worst = (int)std::max<int64_t>(1, std::min<int64_t>({1024, (int64_t)B, LEX_KEY_BUDGET / per_q}));
  std::vector<std::pair<int, int>> groups;  // (first query, queries)
  int64_t keys_alloc = (int64_t)G_worst * per_q;
  int G_alloc = G_worst;
  if (B <= G_worst) {
    groups.push_back({0, B});
  } else {
    caps_.reserve((size_t)B * 8);
    hipLaunchKernelGGL(lex_qcap_kernel, dim3((unsigned)ceil_div(B, 256)), dim3(256), 0, s, tok, qlen, B, Lq,
                       off_.as<int64_t>(), vocab_, rows_, caps_.as<int64_t>());
    SR_LAUNCH_CHECK();
    std::vector<int64_t> cap((size_t)B);
    SR_HIP(hipMemcpyAsync(cap.data(), caps_.p, (size_t)B * 8, hipMemcpyDeviceToHost, s));
    SR_HIP(hipStreamSynchronize(s));
    keys_alloc = 1;
    G_alloc = 1;
    for (int b0 = 0; b0 < B;) {
      int qb = 0;
      int64_t nkeys = 0;
      while (b0 + qb < B && qb < 1024 && (qb == 0 || nkeys + cap[(size_t)(b0 + qb)] <= LEX_KEY_BUDGET))
        nkeys += cap[(size_t)(b0 + qb++)];
      groups.push_back({b0, qb});
      keys_alloc = std::max<int64_t>(keys_alloc, nkeys);
      G_alloc = std::max(G_alloc, qb);
      b0 += qb;
    }
  }
  const int64_t nslots = (int64_t)G_alloc * Lq;
  size_t o = 0;
  auto carve = [&](size_t bytes) {
    const size_t at = o;
    o += (size_t)round_up((int64_t)std::max<size_t>(bytes, 1), 256);
    return at;
  };
  const size_t o_sl = carve((size_t)nslots * sizeof(LexTerm)), o_so = carve((size_t)(G_alloc + 1) * 4),
               o_ko = carve((size_t)(G_alloc + 1) * 8), o_cnt = carve((size_t)G_alloc * 4),
               o_bnd = carve((size_t)nslots * (NB + 1) * 4), o_keys = carve((size_t)keys_alloc * 8),
               o_avg = carve(4);
  ws_.reserve(o);
  char* w = ws_.as<char>();
  LexTerm* d_sl = reinterpret_cast<LexTerm*>(w + o_sl);
  int* d_so = reinterpret_cast<int*>(w + o_so);
  int64_t* d_ko = reinterpret_cast<int64_t*>(w + o_ko);
  int* d_cnt = reinterpret_cast<int*>(w + o_cnt);
  int32_t* d_bnd = reinterpret_cast<int32_t*>(w + o_bnd);
  uint64_t* d_keys = reinterpret_cast<uint64_t*>(w + o_keys);
  float* d_avg = reinterpret_cast<float*>(w + o_avg);
  for (const auto& [b0, qb] : groups) {
    hipLaunchKernelGGL(lex_qprep_kernel, dim3(1), dim3(1024), 0, s, tok + (int64_t)b0 * Lq, qlen + b0,
                       qb, Lq, off_.as<int64_t>(), vocab_, rows_, live_n_, sum_dl_, gstats,
                       (int64_t)b0 * Lq, d_sl, d_so, d_ko, d_cnt, d_avg);
    SR_LAUNCH_CHECK();
    const int64_t ns = (int64_t)qb * Lq;
    if (ns) {
      const int64_t nb = ns * (NB + 1);
      hipLaunchKernelGGL(lex_bounds_kernel, dim3((unsigned)ceil_div(nb, 256)), dim3(256), 0, s, d_sl,
                         (int)ns, NB, post_.as<uint64_t>(), d_bnd);
      SR_LAUNCH_CHECK();
      ProfScope prof("lex_score", s, 0.0, 0.0);
      hipLaunchKernelGGL(lex_score_kernel, dim3((unsigned)qb, (unsigned)NB), dim3(LEX_THREADS),
                         LEX_RB * 4, s, d_sl, d_so, d_bnd, NB, post_.as<uint64_t>(),
                         dlen_.as<int32_t>(), (const uint8_t*)nullptr, rows_, d_avg, k1_, b_, d_cnt,
                         d_ko, d_keys);
      SR_LAUNCH_CHECK();
    }
    {
      ProfScope prof("lex_select", s, 0.0, 0.0);
      hipLaunchKernelGGL(lex_select_kernel, dim3(qb), dim3(SEL_THREADS), sizeof(LexSelSmem), s,
                         d_keys, d_cnt, d_ko, k, out_score + (int64_t)b0 * k,
                         out_rows + (int64_t)b0 * k, row_offset, (uint32_t*)nullptr);
      SR_LAUNCH_CHECK();
    }
  }
  end(s);
}

void LexIndex::search_host(const int64_t* qoff, const int32_t* qterms, int B, int k,
                           const uint8_t* allow, int64_t mask_key, float* out_score,
                           int64_t* out_rows, const sr_lex_global* glob, uint32_t* out_fixed) {
  if (B == 0) return;
  SR_CHECK(out_score && out_rows, "lex.search: null output");
  DeviceGuard g(device_);
  const size_t ob = (size_t)B * k;
  const size_t o_rows = (size_t)round_up((int64_t)ob * 4, 16), o_fix = o_rows + ob * 8;
  out_.reserve(o_fix + (out_fixed ? ob * 4 : 0));
  float* ds = out_.as<float>();
  int64_t* dr = reinterpret_cast<int64_t*>(out_.as<char>() + o_rows);
  uint32_t* dfx = out_fixed ? reinterpret_cast<uint32_t*>(out_.as<char>() + o_fix) : nullptr;
  search_dev(qoff, qterms, B, k, allow, mask_key, ds, dr, stream_, glob, 0, dfx);
  SR_HIP(hipMemcpyAsync(out_score, ds, ob * 4, hipMemcpyDeviceToHost, stream_));
  SR_HIP(hipMemcpyAsync(out_rows, dr, ob * 8, hipMemcpyDeviceToHost, stream_));
  if (out_fixed) SR_HIP(hipMemcpyAsync(out_fixed, dfx, ob * 4, hipMemcpyDeviceToHost, stream_));
  SR_HIP(hipStreamSynchronize(stream_));
}

void LexIndex::stats(int64_t* rows, int64_t* live, int64_t* postings, int64_t* vocab,
                     double* avgdl_out) {
  if (rows) *rows = rows_;
  if (live) *live = live_n_;
  if (postings) *postings = P_;
  if (vocab) *vocab = vocab_;
  if (avgdl_out) *avgdl_out = live_n_ > 0 ? (double)sum_dl_ / (double)live_n_ : 0.0;
}

// Download the forward index (row order) to the host.
void LexIndex::forward(std::vector<int32_t>& fterm, std::vector<uint64_t>& fval) {
  fterm.resize((size_t)P_);
  fval.resize((size_t)P_);
  if (P_) {
    SR_HIP(hipMemcpyAsync(fterm.data(), fterm_.p, (size_t)P_ * 4, hipMemcpyDeviceToHost, stream_));
    SR_HIP(hipMemcpyAsync(fval.data(), fval_.p, (size_t)P_ * 8, hipMemcpyDeviceToHost, stream_));
  }
  SR_HIP(hipStreamSynchronize(stream_));
}

// Snapshot (little endian): "SRMILEX1", float k1, float b, int64 rows, int64 P,
// rows x int32 dl, rows x u8 live, P x int32 term, P x u64 (row << 32 | tf).
void LexIndex::save(const char* path) {
  DeviceGuard g(device_);
  begin(stream_);
  std::vector<int32_t> ft;
  std::vector<uint64_t> fv;
  forward(ft, fv);
  end(stream_);
  std::string tmp = std::string(path) + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw Error(SR_ERR_IO, std::string("lex.save: cannot open ") + path);
  bool ok = std::fwrite("SRMILEX1", 1, 8, f) == 8;
  ok = ok && std::fwrite(&k1_, 4, 1, f) == 1 && std::fwrite(&b_, 4, 1, f) == 1;
  ok = ok && std::fwrite(&rows_, 8, 1, f) == 1 && std::fwrite(&P_, 8, 1, f) == 1;
  ok = ok && (rows_ == 0 || std::fwrite(dl_host_.data(), 4, (size_t)rows_, f) == (size_t)rows_);
  ok = ok && (rows_ == 0 || std::fwrite(live_host_.data(), 1, (size_t)rows_, f) == (size_t)rows_);
  ok = ok && (P_ == 0 || std::fwrite(ft.data(), 4, (size_t)P_, f) == (size_t)P_);
  ok = ok && (P_ == 0 || std::fwrite(fv.data(), 8, (size_t)P_, f) == (size_t)P_);
  ok = (std::fclose(f) == 0) && ok;
  ok = ok && fsync_path(tmp);
  if (!ok || std::rename(tmp.c_str(), path) != 0)
    throw Error(SR_ERR_IO, std::string("lex.save: write failed for ") + path);
}

LexIndex* LexIndex::load(const char* path, int device) {
  FILE* f = std::fopen(path, "rb");
  if (!f) throw Error(SR_ERR_IO, std::string("lex.load: cannot open ") + path);
  char magic[8];
  float k1 = 0.f, b = 0.f;
  int64_t rows = -1, P = -1;
  bool ok = std::fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "SRMILEX1", 8) == 0;
  ok = ok && std::fread(&k1, 4, 1, f) == 1 && std::fread(&b, 4, 1, f) == 1;
  ok = ok && std::fread(&rows, 8, 1, f) == 1 && std::fread(&P, 8, 1, f) == 1 && rows >= 0 && P >= 0 &&
       rows < (int64_t(1) << 31) && P < (int64_t(1) << 40) && std::isfinite(k1) && std::isfinite(b);
  // the exact size the header implies, before anything is allocated
  if (ok) {
    const long here = std::ftell(f);
    ok = std::fseek(f, 0, SEEK_END) == 0 && std::ftell(f) == (long)(32 + rows * 5 + P * 12) &&
         std::fseek(f, here, SEEK_SET) == 0;
  }
  std::vector<int32_t> dl, ft;
  std::vector<uint8_t> live;
  std::vector<uint64_t> fv;
  if (ok) {
    dl.resize((size_t)rows);
    live.resize((size_t)rows);
    ft.resize((size_t)P);
    fv.resize((size_t)P);
    ok = (rows == 0 || std::fread(dl.data(), 4, (size_t)rows, f) == (size_t)rows) &&
         (rows == 0 || std::fread(live.data(), 1, (size_t)rows, f) == (size_t)rows) &&
         (P == 0 || std::fread(ft.data(), 4, (size_t)P, f) == (size_t)P) &&
         (P == 0 || std::fread(fv.data(), 8, (size_t)P, f) == (size_t)P);
  }
  std::fclose(f);
  if (!ok) throw Error(SR_ERR_IO, std::string("lex.load: not a valid lexical snapshot: ") + path);
  // contents the kernels index by: document lengths >= 0, terms in [0, kLexMaxVocab) (a term id
  // sizes the device offset table: a corrupt one near 2^31 asked for ~16 GiB), postings
  // in row order with rows < n_rows and tf >= 1 (a corrupt posting would address past the device
  // arrays)
  for (int64_t r = 0; r < rows && ok; ++r) ok = dl[(size_t)r] >= 0;
  int64_t prev = 0;
  for (int64_t i = 0; i < P && ok; ++i) {
    const int64_t row = (int64_t)(fv[(size_t)i] >> 32);
    const uint32_t tf = (uint32_t)(fv[(size_t)i] & 0xffffffffu);
    ok = ft[(size_t)i] >= 0 && ft[(size_t)i] < kLexMaxVocab && row < rows && row >= prev && tf >= 1 &&
         tf < (1u << 31);
    prev = row;
  }
  if (!ok) throw Error(SR_ERR_IO, std::string("lex.load: corrupt postings in ") + path);
  LexIndex* x = new LexIndex(device, k1, b);
  try {
    x->load_rows(dl, live, ft, fv);
  } catch (...) {
    delete x;
    throw;
  }
  return x;
}

// Replace the contents with a row-ordered forward index (load / compact).
void LexIndex::load_rows(const std::vector<int32_t>& dl, const std::vector<uint8_t>& live,
                         const std::vector<int32_t>& ft, const std::vector<uint64_t>& fv) {
  const int64_t rows = (int64_t)dl.size(), P = (int64_t)ft.size();
  DeviceGuard g(device_);
  begin(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  fterm_.release();
  fval_.release();
  dlen_.release();
  live_.release();
  fterm_.reserve((size_t)std::max<int64_t>(P, 1) * 4);
  fval_.reserve((size_t)std::max<int64_t>(P, 1) * 8);
  dlen_.reserve((size_t)std::max<int64_t>(rows, 1) * 4);
  live_.reserve((size_t)std::max<int64_t>(rows, 1));
  if (P) {
    SR_HIP(hipMemcpyAsync(fterm_.p, ft.data(), (size_t)P * 4, hipMemcpyHostToDevice, stream_));
    SR_HIP(hipMemcpyAsync(fval_.p, fv.data(), (size_t)P * 8, hipMemcpyHostToDevice, stream_));
  }
  if (rows) {
    SR_HIP(hipMemcpyAsync(dlen_.p, dl.data(), (size_t)rows * 4, hipMemcpyHostToDevice, stream_));
    SR_HIP(hipMemcpyAsync(live_.p, live.data(), (size_t)rows, hipMemcpyHostToDevice, stream_));
  }
  SR_HIP(hipStreamSynchronize(stream_));
  end(stream_);
  rows_ = rows;
  P_ = P;
  dl_host_ = dl;
  live_host_ = live;
  live_n_ = 0;
  sum_dl_ = 0;
  vocab_ = 0;
  for (int64_t r = 0; r < rows; ++r)
    if (live[(size_t)r]) {
      ++live_n_;
      sum_dl_ += dl[(size_t)r];
    }
  for (int32_t t : ft) vocab_ = std::max<int64_t>(vocab_, (int64_t)t + 1);
  dirty_ = true;
  ++version_;
}

void LexIndex::compact(int64_t* old_to_new) {
  DeviceGuard g(device_);
  begin(stream_);
  std::vector<int32_t> ft;
  std::vector<uint64_t> fv;
  forward(ft, fv);
  end(stream_);
  std::vector<int64_t> remap((size_t)rows_, -1);
  int64_t n = 0;
  for (int64_t r = 0; r < rows_; ++r)
    if (live_host_[(size_t)r]) remap[(size_t)r] = n++;
  if (old_to_new)
    for (int64_t r = 0; r < rows_; ++r) old_to_new[r] = remap[(size_t)r];
  std::vector<int32_t> dl((size_t)n), ft2;
  std::vector<uint8_t> live((size_t)n, 1);
  std::vector<uint64_t> fv2;
  for (int64_t r = 0; r < rows_; ++r)
    if (remap[(size_t)r] >= 0) dl[(size_t)remap[(size_t)r]] = dl_host_[(size_t)r];
  for (int64_t p = 0; p < P_; ++p) {
    const int64_t r = (int64_t)(fv[(size_t)p] >> 32), nr = remap[(size_t)r];
    if (nr < 0) continue;
    ft2.push_back(ft[(size_t)p]);
    fv2.push_back(((uint64_t)nr << 32) | (fv[(size_t)p] & 0xffffffffull));
  }
  load_rows(dl, live, ft2, fv2);
}

}  // namespace sr
