// K1 / K2: exact cosine top-k over the in-HBM corpus (replaces SeekDB HNSW cosine search,
// super_rag/vectorstore/seekdb_connector.py:98-115), plus the multi-shard merge, the cross-encoder
// pair packer and the rerank ordering.
//
// K1 cosine_scan: sims = C_tile . Q^T on MFMA (v_mfma_f32_16x16x32_f16, fp32 accumulate) for a
// 256-row corpus tile against up to 256 queries per workgroup (8 waves, 32 rows each).  The
// corpus streams once from HBM through a double-buffered LDS-DMA (global_load_lds_dwordx4) ring;
// the query block is L2-resident and restaged per k-step.  The score matrix is never written:
// the epilogue keeps only (query, row) pairs whose similarity is >= the query's running k-th
// best (tau), appending 64-bit keys (ordered(sim) << 32 | ~row) to a per-query candidate list.
// The very first chunk of rows runs in DENSE mode (every key written, no atomics) to seed tau.
//
// K2 select: one workgroup per query loads its candidate keys into LDS, finds the k-th largest
// key by an MSB radix select (8-bit digits, per-wave LDS histograms, wave-parallel suffix scan)
// and bitonic-sorts the k winners.  Keys are unique (row in the low word), so the k-th key is
// exact and ties in similarity resolve by ascending row id, as the oracle does.
#include <cstdlib>

#include "sr_common.h"
#include "sr_kernels.h"
#include "sr_topk.h"

namespace sr {

namespace {

constexpr int SROWS = 256;    // corpus rows per scan workgroup
constexpr int SBK = 64;       // k per stage (fp16 elements)
constexpr int STHREADS = 512; // 8 waves

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ void glds_rows(const half_t* __restrict__ g, int64_t ld, int64_t row0,
                                          int64_t row_last, int k0, half_t* lds_piece, int prow0,
                                          int lane) {
  // One 1 KiB wave-instruction: 8 rows (prow0 .. prow0+7 of the LDS image) x 64 fp16.
  const int r = prow0 + (lane >> 3);
  const int c = swz_chunk(r, lane & 7);
  int64_t gr = row0 + r;
  gr = gr < row_last ? gr : row_last;
  __builtin_amdgcn_global_load_lds((const void*)(g + gr * ld + k0 + c * 8), SR_LDS(lds_piece), 16,
                                   0, 0);
}

__device__ __forceinline__ half8 lds_frag(const half_t* tile, int row, int chunk) {
  return *reinterpret_cast<const half8*>(tile + row * SBK + swz_chunk(row, chunk) * 8);
}

typedef int i8v __attribute__((ext_vector_type(8)));
typedef int i4v __attribute__((ext_vector_type(4)));
// fp8 fragment of a 128-byte K-step row (128 e4m3 elements): the lane's chunks c and c + 4 as one
// 32-byte operand of the block-scaled MFMA (the pairing k_gemm.hip's read_frag8 uses; A and B
// share the slot -> k map, so the products pair up exactly)
__device__ __forceinline__ i8v lds_frag8(const half_t* tile, int row, int chunk) {
  const i4v lo = __builtin_bit_cast(i4v, lds_frag(tile, row, chunk));
  const i4v hi = __builtin_bit_cast(i4v, lds_frag(tile, row, chunk + 4));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// F8: the rows and queries are OCP e4m3 of 256 x (unit vectors; ldc counts 2-byte units, so a
// K-step still moves 128-byte rows, now 128 elements); E8M0 block scales 2^-8 on both operands
// undo the staging factor inside v_mfma_scale_f32_16x16x128_f8f6f4: sims are plain cosines.
template <int QT, bool DENSE, bool F8 = false>
__global__ __launch_bounds__(STHREADS, 1) void cosine_scan_kernel(
    const half_t* __restrict__ corpus, int64_t ldc, const uint8_t* __restrict__ live, int64_t r0,
    int64_t r1, const half_t* __restrict__ Q, int B, const float* __restrict__ tau,
    uint64_t* __restrict__ cand, int* __restrict__ cnt, int cap) {
  constexpr int QROWS = 16 * QT;
  constexpr int STAGE = (SROWS + QROWS) * SBK;  // halfs per stage
  __shared__ __attribute__((aligned(16))) half_t lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t row0 = r0 + (int64_t)blockIdx.x * SROWS;
  const int64_t row_last = r1 - 1;
  const int nk = (int)(ldc / SBK);

  float4v acc[2][QT];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int q = 0; q < QT; ++q) acc[a][q] = float4v{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int kt, int buf) {
    half_t* C = lds + buf * STAGE;
    half_t* Qs = C + SROWS * SBK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int prow = wave * 32 + i * 8;
      glds_rows(corpus, ldc, row0, row_last, kt * SBK, C + prow * SBK, prow, lane);
    }
    for (int i = wave; i < 2 * QT; i += 8)
      glds_rows(Q, ldc, 0, QROWS - 1, kt * SBK, Qs + i * 8 * SBK, i * 8, lane);
  };

  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, cur ^ 1);
    const half_t* C = lds + cur * STAGE;
    const half_t* Qs = C + SROWS * SBK;
    if constexpr (F8) {
      const int c0 = lane >> 4;
      i8v a[2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) a[rt] = lds_frag8(C, wave * 32 + rt * 16 + (lane & 15), c0);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const i8v b = lds_frag8(Qs, qt * 16 + (lane & 15), c0);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          acc[rt][qt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[rt], b, acc[rt][qt], 0, 0,
                                                                           0, 119, 0, 119);
      }
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int chunk = (lane >> 4) + 4 * s;
      half8 a[2];
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) a[rt] = lds_frag(C, wave * 32 + rt * 16 + (lane & 15), chunk);
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
        const half8 b = lds_frag(Qs, qt * 16 + (lane & 15), chunk);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
          acc[rt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[rt], b, acc[rt][qt], 0, 0, 0);
      }
    }
    }
    __syncthreads();
  }

  // Epilogue: lane owns sim(row = row0 + 32w + 16rt + 4(lane>>4) + r, query = 16qt + (lane&15)).
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int q = qt * 16 + (lane & 15);
    if (q >= B) continue;
    const float t = DENSE ? -INFINITY : tau[q];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = row0 + wave * 32 + rt * 16 + 4 * (lane >> 4) + r;
        if (row > row_last) continue;
        const bool alive = live == nullptr || live[row] != 0;
        const float sim = acc[rt][qt][r];
        if constexpr (DENSE) {
          cand[(int64_t)q * cap + (row - r0)] = alive ? make_key(sim, (uint32_t)row) : 0ull;
        } else {
          if (alive && sim >= t) {
            const int pos = atomicAdd(&cnt[q], 1);
            if (pos < cap) cand[(int64_t)q * cap + pos] = make_key(sim, (uint32_t)row);
          }
        }
      }
  }
}

// ------------------------------------------------------------------------------------------------
// K1s cosine_stream (threshold chunks, 65..256 queries): the query block lives in LDS for the whole
// launch and the corpus streams from HBM straight into the MFMA A-operand registers, so the main
// loop has no LDS-DMA staging and no barrier.
//   * a workgroup holds 64 queries (64 x ld fp16 in LDS, 16-byte chunks XOR-swizzled by the query's
//     low 4 bits: the B-fragment reads are conflict-free); B > 64 takes G = ceil(B / 64) workgroups
//     on ONE XCD (a "team": blocks b, b + 8, ... share an XCD) walking the same tiles, so a corpus
//     tile comes from HBM once and the team's other members read it from that XCD's L2
//   * a tile = 512 rows; each of the 8 waves owns 64 of them (4 blocks of 16 rows in the A
//     fragment layout: lane (c, g) holds row c, dims 32 j + 8 g .. + 8 of slice j) and keeps D
//     slices (D x 4 buffer_load_dwordx4) in flight, refilled as each slice is consumed, across
//     tile boundaries; rows past the chunk read as zero (buffer bounds) and are masked
//   * epilogue per wave and tile: v_max3 fast rejection per query column (no memory traffic), hits
//     append to per-query LDS lists (LDS atomics: nothing waits on the streaming loads); the lists
//     are flushed to the candidate lists once per launch with one global atomic per query.  An LDS
//     list that fills up spills keys to the global list directly (per-key atomics).
// Same key set and counts as cosine_scan's threshold mode (cnt[q] = keys appended, > cap means the
// list overflowed and the search re-runs in safe mode).
constexpr int KS_QB = 64;     // queries per workgroup
constexpr int KS_RB = 4;      // 16-row blocks per wave
constexpr int KS_TROWS = 8 * KS_RB * 16;  // rows per tile (512)

template <int NS>
struct KsGeom {
  static constexpr int LD = NS * 32;                       // halfs per row
  static constexpr int QHALFS = KS_QB * LD;
  static constexpr int KSLOT_FIT = (163840 - QHALFS * 2 - 2 * KS_QB * 4) / (KS_QB * 8);
  static constexpr int KSLOT = KSLOT_FIT > 128 ? 128 : (KSLOT_FIT & ~1);
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NS, int D>
__global__ __launch_bounds__(512, 1) void cosine_stream_kernel(
    const half_t* __restrict__ corpus, int64_t r0, int64_t r1, const half_t* __restrict__ Q, int B,
    const float* __restrict__ tau, uint64_t* __restrict__ cand, int* __restrict__ cnt, int cap,
    int G) {
  using Geo = KsGeom<NS>;
  constexpr int LD = Geo::LD, KSLOT = Geo::KSLOT;
  static_assert(NS % D == 0, "the load ring must divide the slices of a row");
  __shared__ __attribute__((aligned(16))) half_t qlds[Geo::QHALFS];
  __shared__ __attribute__((aligned(16))) uint64_t klds[KS_QB * KSLOT];
  __shared__ int kcnt[KS_QB], kbase[KS_QB];

  const int xcd = blockIdx.x & 7, jb = blockIdx.x >> 3;
  const int T = (int)(gridDim.x >> 3) / G;  // teams per XCD
  if (jb >= T * G) return;                  // (whole workgroup: no barrier is skipped by a part)
  const int team = xcd * T + jb / G, qg = jb % G, NT = 8 * T;
  const int64_t n = r1 - r0;
  const int64_t ntiles = (n + KS_TROWS - 1) / KS_TROWS;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int c = lane & 15, g = lane >> 4;

  // query block -> LDS (chunk ch of query q at ch ^ (q & 15)); rows >= B are never keys (tau inf)
  for (int i = tid; i < KS_QB * NS * 4; i += 512) {
    const int q = i / (NS * 4), ch = i - q * (NS * 4);
    const half8 v = *reinterpret_cast<const half8*>(Q + (int64_t)(qg * KS_QB + q) * LD + ch * 8);
    *reinterpret_cast<half8*>(qlds + q * LD + ((ch ^ (q & 15)) * 8)) = v;
  }
  if (tid < KS_QB) kcnt[tid] = 0;
  float t[4];
#pragma unroll
  for (int qb = 0; qb < 4; ++qb) {
    const int q = qg * KS_QB + 16 * qb + c;
    t[qb] = q < B ? tau[q] : INFINITY;
  }
  __syncthreads();

  // B fragment of (query block qb, slice j): query 16 qb + c, chunk 4 j + g, stored at
  // (4 j + g) ^ c = 16 (j >> 2) + (4 (j & 3) ^ (g ^ c)): four lane offsets cover every slice
  int qoff[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) qoff[m] = c * LD + ((4 * m) ^ (g ^ c)) * 8;
  const uint32_t voff = (uint32_t)((c * LD + 8 * g) * 2);  // lane's row / dims in a 16-row block

  auto tile_rsrc = [&](int64_t tl) {
    const int64_t row0 = tl * KS_TROWS + wave * 64;  // chunk-relative
    const int64_t left = n - row0;
    const int64_t bytes = left <= 0 ? 0 : (left >= 64 ? 64 : left) * (int64_t)LD * 2;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(corpus + (r0 + row0) * LD), (short)0,
                                             (int)bytes, 0x00020000);
  };
  auto load = [&](__amdgpu_buffer_rsrc_t rs, int rb, int j) {
    return __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(
                                         rs, voff + 64 * j, rb * 16 * LD * 2, 0));
  };

  int64_t tile = team;
  half8 buf[D][KS_RB];
  auto bfrag = [&](int j, int qb) {
    return *reinterpret_cast<const half8*>(qlds + qb * 16 * LD + (j >> 2) * 128 + qoff[j & 3]);
  };
  half8 bc[4];  // B fragments of the slice being multiplied (slice 0 of every tile: the same)
  if (tile < ntiles) {
    const auto rs = tile_rsrc(tile);
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int rb = 0; rb < KS_RB; ++rb) buf[d][rb] = load(rs, rb, d);
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) bc[qb] = bfrag(0, qb);
  }
  while (tile < ntiles) {
    const int64_t next = tile + NT;
    // (past the last tile: a zero-byte resource, so the ring's refills read nothing)
    const auto rs = tile_rsrc(tile), rn = tile_rsrc(next);
    float4v acc[KS_RB][4];
#pragma unroll
    for (int rb = 0; rb < KS_RB; ++rb)
#pragma unroll
      for (int qb = 0; qb < 4; ++qb) acc[rb][qb] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int s = j % D;
      // next slice's B fragments (LDS), then this slice's 16 MFMAs with the refill of its ring slot
      // (slice j + D of this tile or the next) spread among them
      half8 bn[4];
      const int jn = j + 1 < NS ? j + 1 : 0;
#pragma unroll
      for (int qb = 0; qb < 4; ++qb) bn[qb] = bfrag(jn, qb);
#pragma unroll
      for (int qb = 0; qb < 4; ++qb)
#pragma unroll
        for (int rb = 0; rb < KS_RB; ++rb)
          acc[rb][qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(buf[s][rb], bc[qb], acc[rb][qb], 0, 0, 0);
#pragma unroll
      for (int rb = 0; rb < KS_RB; ++rb)
        buf[s][rb] = j + D < NS ? load(rs, rb, j + D) : load(rn, rb, j + D - NS);
      // schedule: 4 x {MFMA, DS read}, 4 x {2 MFMA, VMEM read}, 4 MFMA
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int qb = 0; qb < 4; ++qb) bc[qb] = bn[qb];
    }
    // epilogue: acc[rb][qb][r] = sim(row tile*512 + 64 wave + 16 rb + 4 g + r, query 16 qb + c)
    const int64_t rw = tile * KS_TROWS + wave * 64;  // chunk-relative first row of the wave
    const int valid = (int)(n - rw < 64 ? n - rw : 64);  // rows of the wave in the chunk (may be <= 0)
    bool hit = false;
#pragma unroll
    for (int qb = 0; qb < 4; ++qb) {
      float mx = -INFINITY;
#pragma unroll
      for (int rb = 0; rb < KS_RB; ++rb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          mx = fmaxf(mx, (16 * rb + 4 * g + r < valid) ? acc[rb][qb][r] : -INFINITY);
      hit |= mx >= t[qb];
    }
    if (__builtin_amdgcn_ballot_w64(hit) != 0) {
#pragma unroll
      for (int qb = 0; qb < 4; ++qb)
#pragma unroll
        for (int rb = 0; rb < KS_RB; ++rb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int rr = 16 * rb + 4 * g + r;
            const float sim = acc[rb][qb][r];
            if (rr < valid && sim >= t[qb]) {
              const int ql = 16 * qb + c;
              const uint64_t key = make_key(sim, (uint32_t)(r0 + rw + rr));
              const int rank = atomicAdd(&kcnt[ql], 1);  // LDS atomic
              if (rank < KSLOT) {
                klds[ql * KSLOT + rank] = key;
              } else {  // the query's LDS list is full: straight to the global list
                const int q = qg * KS_QB + ql;
                const int pos = atomicAdd(&cnt[q], 1);
                if (pos < cap) cand[(int64_t)q * cap + pos] = key;
              }
            }
          }
    }
    tile = next;
  }
  // flush the LDS lists: one reservation per query, then the keys
  __syncthreads();
  if (tid < KS_QB) {
    const int q = qg * KS_QB + tid;
    const int m = min(kcnt[tid], KSLOT);
    kcnt[tid] = m;
    kbase[tid] = (m > 0 && q < B) ? atomicAdd(&cnt[q], m) : 0;
  }
  __syncthreads();
  for (int i = tid; i < KS_QB * KSLOT; i += 512) {
    const int ql = i / KSLOT, e = i - ql * KSLOT;
    if (e < kcnt[ql]) {
      const int pos = kbase[ql] + e;
      if (pos < cap) cand[(int64_t)(qg * KS_QB + ql) * cap + pos] = klds[i];
    }
  }
}

struct SelectSmem {
  uint64_t keys[SEL_CAP];
  SelShared sh;
};

__global__ __launch_bounds__(SEL_THREADS, 1) void topk_select_kernel(
    uint64_t* __restrict__ cand, int* __restrict__ cnt, int cap, float* __restrict__ tau, int k,
    int* __restrict__ overflow, int final_pass, float* __restrict__ out_sim,
    int64_t* __restrict__ out_rows, int64_t row_offset, const uint8_t* __restrict__ live) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  SelectSmem& S = *reinterpret_cast<SelectSmem*>(smem_raw);
  const int q = blockIdx.x, tid = threadIdx.x;
  const int n_raw = cnt[q];
  if (n_raw > cap && tid == 0) atomicOr(overflow, 1);
  const int n_in = min(n_raw, cap);
  uint64_t* list = cand + (int64_t)q * cap;
  // Load non-zero keys (zero = dead row in a dense chunk) of live rows into LDS (the GEMM scan's
  // threshold epilogue does not read the live flags: tombstoned rows are dropped here).
  if (tid == 0) S.sh.nsel = 0;
  __syncthreads();
  for (int i = tid; i < n_in; i += blockDim.x) {
    const uint64_t key = list[i];
    if (key != 0ull && (live == nullptr || live[key_row(key)] != 0)) {
      const int p = atomicAdd(&S.sh.nsel, 1);
      S.keys[p] = key;
    }
  }
  __syncthreads();
  const int n = S.sh.nsel;
  __syncthreads();
  const int m = block_topk([&](int i) { return S.keys[i]; }, n, k, S.sh);
  for (int i = tid; i < m; i += blockDim.x) list[i] = S.sh.sel[i];
  if (tid == 0) {
    cnt[q] = m;
    tau[q] = (m == k) ? key_sim(S.sh.sel[k - 1]) : -INFINITY;
  }
  if (final_pass) {
    for (int i = tid; i < k; i += blockDim.x) {
      const bool ok = i < m;
      out_sim[(int64_t)q * k + i] = ok ? key_sim(S.sh.sel[i]) : -INFINITY;
      out_rows[(int64_t)q * k + i] = ok ? (int64_t)key_row(S.sh.sel[i]) + row_offset : -1;
    }
  }
}

__global__ __launch_bounds__(SEL_THREADS, 1) void topk_merge_kernel(
    const float* __restrict__ sims, const int64_t* __restrict__ rows, int P, int B, int k,
    int k_out, float* __restrict__ out_sim, int64_t* __restrict__ out_rows) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  SelectSmem& S = *reinterpret_cast<SelectSmem*>(smem_raw);
  const int q = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) S.sh.nsel = 0;
  __syncthreads();
  for (int i = tid; i < P * k; i += blockDim.x) {
    const int p = i / k, j = i - p * k;
    const int64_t off = ((int64_t)p * B + q) * k + j;
    const int64_t r = rows[off];
    if (r >= 0) {
      const int pos = atomicAdd(&S.sh.nsel, 1);
      S.keys[pos] = make_key(sims[off], (uint32_t)r);
    }
  }
  __syncthreads();
  const int n = S.sh.nsel;
  __syncthreads();
  const int m = block_topk([&](int i) { return S.keys[i]; }, n, k_out, S.sh);
  for (int i = tid; i < k_out; i += blockDim.x) {
    const bool ok = i < m;
    out_sim[(int64_t)q * k_out + i] = ok ? key_sim(S.sh.sel[i]) : -INFINITY;
    out_rows[(int64_t)q * k_out + i] = ok ? (int64_t)key_row(S.sh.sel[i]) : -1;
  }
}

__global__ void fill_int_kernel(int* __restrict__ p, int n, int v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}
__global__ void fill_float_kernel(float* __restrict__ p, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// ------------------------------------------------------------------------------------------------
// Cross-encoder pair packing (HF fast-tokenizer pair layout, LongestFirst truncation).
__global__ __launch_bounds__(256) void build_pairs_kernel(
    const int32_t* __restrict__ q_tok, const int32_t* __restrict__ q_len, int lq_max,
    const int32_t* __restrict__ p_tok, const int32_t* __restrict__ p_len, int lp_max,
    const int64_t* __restrict__ cand_rows, int B, int K, int S, int style, int bos, int eos,
    int pad, int32_t* __restrict__ out_ids, int32_t* __restrict__ out_mask,
    int32_t* __restrict__ out_type) {
  const int lane = threadIdx.x & 63;
  const int64_t pair = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pair >= (int64_t)B * K) return;
  const int b = (int)(pair / K);
  const int64_t row = cand_rows[pair];
  int lq = min(max(q_len[b], 0), lq_max);
  int lp = row >= 0 ? min(max(p_len[row], 0), lp_max) : 0;
  const int nspec = style == 0 ? 4 : 3;
  const int budget = max(S - nspec, 0);
  // LongestFirst truncation as Hugging Face fast tokenizers do it (tokenizers truncation.rs):
  // the shorter side stays whole if it fits in half the budget, else both get half and the longer
  // side (the passage on ties) gets the odd token.
  if (lq + lp > budget) {
    const bool swap = lq > lp;
    int n1 = swap ? lp : lq;
    int n2 = n1 > budget ? n1 : max(n1, budget - n1);
    if (n1 + n2 > budget) {
      n1 = budget / 2;
      n2 = n1 + budget % 2;
    }
    const int tq = swap ? n2 : n1, tp = swap ? n1 : n2;
    lq = min(lq, tq);
    lp = min(lp, tp);
  }
  const int32_t* qt = q_tok + (int64_t)b * lq_max;
  const int32_t* pt = row >= 0 ? p_tok + row * lp_max : nullptr;
  // Segment boundaries.
  const int q_start = 1;
  const int q_end = q_start + lq;                 // first separator
  const int p_start = q_end + (style == 0 ? 2 : 1);
  const int p_end = p_start + lp;                 // final separator
  const int total = p_end + 1;
  int32_t* oi = out_ids + pair * S;
  int32_t* om = out_mask + pair * S;
  int32_t* ot = out_type ? out_type + pair * S : nullptr;
  for (int s = lane; s < S; s += 64) {
    int id;
    if (s == 0) id = bos;
    else if (s < q_end) id = qt[s - q_start];
    else if (s < p_start) id = eos;
    else if (s < p_end) id = pt[s - p_start];
    else if (s == p_end) id = eos;
    else id = pad;
    oi[s] = id;
    om[s] = s < total ? 1 : 0;
    if (ot) ot[s] = (style == 1 && s >= p_start && s < total) ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void rerank_select_kernel(const float* __restrict__ logits,
                                                            int K, int k_out,
                                                            int32_t* __restrict__ out_index) {
  __shared__ uint64_t v[SR_MAX_TOPK];
  const int b = blockIdx.x;
  int np2 = 1;
  while (np2 < K) np2 <<= 1;
  for (int i = threadIdx.x; i < np2; i += blockDim.x)
    v[i] = i < K ? make_key(logits[(int64_t)b * K + i], (uint32_t)i) : 0ull;
  __syncthreads();
  bitonic_sort_desc(v, np2);
  for (int i = threadIdx.x; i < k_out; i += blockDim.x)
    out_index[(int64_t)b * k_out + i] = i < K ? (int32_t)key_row(v[i]) : -1;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// Host launchers

template <int QT, bool F8 = false>
static void scan_qt(bool dense, dim3 grid, hipStream_t s, const half_t* corpus, int64_t ldc,
                    const uint8_t* live, int64_t r0, int64_t r1, const half_t* Q, int B,
                    const float* tau, uint64_t* cand, int* cnt, int cap) {
  if (dense)
    hipLaunchKernelGGL((cosine_scan_kernel<QT, true, F8>), grid, dim3(STHREADS), 0, s, corpus, ldc,
                       live, r0, r1, Q, B, tau, cand, cnt, cap);
  else
    hipLaunchKernelGGL((cosine_scan_kernel<QT, false, F8>), grid, dim3(STHREADS), 0, s, corpus, ldc,
                       live, r0, r1, Q, B, tau, cand, cnt, cap);
}

int scan_query_tiles(int B) {
  if (B <= 16) return 1;
  if (B <= 32) return 2;
  if (B <= 64) return 4;
  if (B <= 128) return 8;
  return 16;
}

static bool g_scan_legacy = diag_getenv("SR_SCAN_LEGACY") != nullptr;  // (diagnostic build only)

// SR_SCAN_STREAM (read per launch: parity tests switch it): 0 (default) = threshold chunks of 65..256
// queries on the GEMM main loop (launch_cosine_scan_gemm), 1 = on cosine_stream, 2 = cosine_stream for
// every threshold chunk (also B <= 64).  Measured (10M x 768, B = 256, k = 100): cosine_stream
// 8.4 ms vs 4.4 ms for the GEMM scan: the team members do not stay close enough for the XCD's L2 to
// serve 3 of the 4 reads of a tile (8 teams x 786 KB in flight per XCD > 4 MB), so the corpus
// streams ~4x from the Infinity Cache / HBM.
static int scan_stream_mode() {
  const char* e = std::getenv("SR_SCAN_STREAM");
  return e ? (int)std::strtol(e, nullptr, 10) : 0;
}

template <int NS, int D>
static void stream_ns(dim3 grid, hipStream_t s, const half_t* corpus, int64_t r0, int64_t r1,
                      const half_t* Q, int B, const float* tau, uint64_t* cand, int* cnt, int cap,
                      int G) {
  hipLaunchKernelGGL((cosine_stream_kernel<NS, D>), grid, dim3(512), 0, s, corpus, r0, r1, Q, B, tau,
                     cand, cnt, cap, G);
}

// K1s for a threshold chunk; false when the row width has no instantiation (then the caller's
// other kernels run).  Q holds >= 64 * ceil(B / 64) rows of ldc halfs (the store's query buffer is
// 256 rows per block).
static bool launch_cosine_stream(const half_t* corpus, int64_t ldc, int64_t r0, int64_t r1,
                                 const half_t* Q, int B, const float* tau, uint64_t* cand, int* cnt,
                                 int cap, hipStream_t s) {
  if (ldc != 384 && ldc != 512 && ldc != 768 && ldc != 1024) return false;
  const int64_t n = r1 - r0;
  const int G = (B + KS_QB - 1) / KS_QB;
  const int64_t ntiles = ceil_div(n, KS_TROWS);
  const int per_xcd = (int)std::min<int64_t>(32, G * ceil_div(ntiles, 8));
  const dim3 grid((unsigned)(8 * per_xcd));
  ProfScope prof("cosine_scan", s, 2.0 * (double)n * ldc * B, (double)n * ldc * 2.0 + (double)B * ldc * 2.0);
  switch (ldc) {
    case 384: stream_ns<12, 4>(grid, s, corpus, r0, r1, Q, B, tau, cand, cnt, cap, G); break;
    case 512: stream_ns<16, 4>(grid, s, corpus, r0, r1, Q, B, tau, cand, cnt, cap, G); break;
    case 768: stream_ns<24, 4>(grid, s, corpus, r0, r1, Q, B, tau, cand, cnt, cap, G); break;
    default: stream_ns<32, 4>(grid, s, corpus, r0, r1, Q, B, tau, cand, cnt, cap, G); break;
  }
  SR_LAUNCH_CHECK();
  return true;
}

void launch_cosine_scan(bool dense, const half_t* corpus, int64_t ldc, const uint8_t* live,
                        int64_t r0, int64_t r1, const half_t* Q, int B, const float* tau,
                        uint64_t* cand, int* cnt, int cap, hipStream_t s) {
  SR_CHECK(B > 0 && B <= 256, "cosine_scan: 1..256 queries per launch");
  SR_CHECK(ldc % SBK == 0, "cosine_scan: padded dim must be a multiple of 64");
  if (r1 <= r0) return;
  SR_CHECK(!dense || r1 - r0 <= cap, "cosine_scan: dense chunk larger than the candidate list");
  if (!dense && !g_scan_legacy) {
    const int mode = scan_stream_mode();
    if ((mode == 1 && B > 64) || mode == 2)
      if (launch_cosine_stream(corpus, ldc, r0, r1, Q, B, tau, cand, cnt, cap, s)) return;
  }
  const int qt = scan_query_tiles(B);
  if (!dense && qt == 16 && ldc >= 2 * SBK && r1 - r0 >= 8 * SROWS && !g_scan_legacy) {
    // large query blocks: the pipelined 256 x 256 GEMM main loop with the threshold epilogue
    launch_cosine_scan_gemm(corpus, ldc, live, r0, r1, Q, B, tau, cand, cnt, cap, s);
    return;
  }
  const dim3 grid((unsigned)ceil_div(r1 - r0, SROWS));
  const double rows = (double)(r1 - r0);
  ProfScope prof(dense ? "cosine_scan_dense" : "cosine_scan", s, 2.0 * rows * ldc * B,
                 rows * ldc * 2.0 + (double)B * ldc * 2.0 + (dense ? rows * B * 8.0 : 0.0));
  switch (qt) {
    case 1: scan_qt<1>(dense, grid, s, corpus, ldc, live, r0, r1, Q, B, tau, cand, cnt, cap); break;
    case 2: scan_qt<2>(dense, grid, s, corpus, ldc, live, r0, r1, Q, B, tau, cand, cnt, cap); break;
    case 4: scan_qt<4>(dense, grid, s, corpus, ldc, live, r0, r1, Q, B, tau, cand, cnt, cap); break;
    case 8: scan_qt<8>(dense, grid, s, corpus, ldc, live, r0, r1, Q, B, tau, cand, cnt, cap); break;
    default: scan_qt<16>(dense, grid, s, corpus, ldc, live, r0, r1, Q, B, tau, cand, cnt, cap); break;
  }
  SR_LAUNCH_CHECK();
}

// fp8 K1 for up to 64 queries: the small-block kernel above on e4m3 rows (the 256 x 256 GEMM
// main loop, launch_cosine_scan_gemm8, computes 256 query columns whatever B is: at B = 32 seven
// eighths of its MFMA work were padding).  ld8 = row bytes (multiple of 128); same contract as
// launch_cosine_scan (dense: every row's key at position row - r0, no atomics).
void launch_cosine_scan8(bool dense, const uint8_t* corpus8, int64_t ld8, const uint8_t* live,
                         int64_t r0, int64_t r1, const uint8_t* Q8, int B, const float* tau,
                         uint64_t* cand, int* cnt, int cap, hipStream_t s) {
  SR_CHECK(B > 0 && B <= 64, "cosine_scan8: 1..64 queries per launch");
  SR_CHECK(ld8 % 128 == 0, "cosine_scan8: row bytes must be a multiple of 128");
  if (r1 <= r0) return;
  SR_CHECK(!dense || r1 - r0 <= cap, "cosine_scan8: dense chunk larger than the candidate list");
  const dim3 grid((unsigned)ceil_div(r1 - r0, SROWS));
  const double rows = (double)(r1 - r0);
  ProfScope prof(dense ? "cosine_scan8_dense" : "cosine_scan8", s, 2.0 * rows * ld8 * B,
                 rows * ld8 + (double)B * ld8 + (dense ? rows * B * 8.0 : 0.0));
  const half_t* C = reinterpret_cast<const half_t*>(corpus8);
  const half_t* Q = reinterpret_cast<const half_t*>(Q8);
  const int64_t ld = ld8 / 2;  // staging in 2-byte units: 64 per 128-byte K-step
  switch (scan_query_tiles(B)) {
    case 1: scan_qt<1, true>(dense, grid, s, C, ld, live, r0, r1, Q, B, tau, cand, cnt, cap); break;
    case 2: scan_qt<2, true>(dense, grid, s, C, ld, live, r0, r1, Q, B, tau, cand, cnt, cap); break;
    default: scan_qt<4, true>(dense, grid, s, C, ld, live, r0, r1, Q, B, tau, cand, cnt, cap); break;
  }
  SR_LAUNCH_CHECK();
}

static bool g_select_attr_set = false;

static void ensure_select_attrs() {
  if (g_select_attr_set) return;
  SR_HIP(hipFuncSetAttribute((const void*)topk_select_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(SelectSmem)));
  SR_HIP(hipFuncSetAttribute((const void*)topk_merge_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, sizeof(SelectSmem)));
  g_select_attr_set = true;
}

int select_capacity() { return SEL_CAP; }

void launch_topk_select(uint64_t* cand, int* cnt, int cap, float* tau, int B, int k,
                        int* overflow, bool final_pass, float* out_sim, int64_t* out_rows,
                        int64_t row_offset, hipStream_t s, const uint8_t* live) {
  SR_CHECK(k >= 1 && k <= SR_MAX_TOPK, "topk: k must be in [1, 1024]");
  SR_CHECK(cap <= SEL_CAP, "topk: candidate capacity too large");
  ensure_select_attrs();
  ProfScope prof("topk_select", s, 0.0, (double)B * cap * 8.0);
  hipLaunchKernelGGL(topk_select_kernel, dim3(B), dim3(SEL_THREADS), sizeof(SelectSmem), s, cand,
                     cnt, cap, tau, k, overflow, final_pass ? 1 : 0, out_sim, out_rows, row_offset,
                     live);
  SR_LAUNCH_CHECK();
}

void launch_topk_merge(const float* sims, const int64_t* rows, int P, int B, int k, int k_out,
                       float* out_sim, int64_t* out_rows, hipStream_t s) {
  SR_CHECK(k_out >= 1 && k_out <= SR_MAX_TOPK, "merge: k_out must be in [1, 1024]");
  SR_CHECK((int64_t)P * k <= SEL_CAP, "merge: P * k must be <= 16384");
  if (B <= 0) return;
  ensure_select_attrs();
  ProfScope prof("topk_merge", s, 0.0, (double)P * B * k * 12.0);
  hipLaunchKernelGGL(topk_merge_kernel, dim3(B), dim3(SEL_THREADS), sizeof(SelectSmem), s, sims,
                     rows, P, B, k, k_out, out_sim, out_rows);
  SR_LAUNCH_CHECK();
}

void launch_fill_int(int* p, int n, int v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fill_int_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, p, n, v);
  SR_LAUNCH_CHECK();
}
void launch_fill_float(float* p, int n, float v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(fill_float_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, p, n, v);
  SR_LAUNCH_CHECK();
}

void launch_build_pairs(const int32_t* q_tok, const int32_t* q_len, int lq_max,
                        const int32_t* p_tok, const int32_t* p_len, int lp_max,
                        const int64_t* cand_rows, int B, int K, int S, int style, int bos, int eos,
                        int pad, int32_t* out_ids, int32_t* out_mask, int32_t* out_type,
                        hipStream_t s) {
  SR_CHECK(style == 0 || style == 1, "build_pairs: style must be 0 (RoBERTa) or 1 (BERT)");
  SR_CHECK(S >= 4, "build_pairs: sequence too short");
  const int64_t pairs = (int64_t)B * K;
  if (pairs <= 0) return;
  hipLaunchKernelGGL(build_pairs_kernel, dim3((unsigned)ceil_div(pairs, 4)), dim3(256), 0, s,
                     q_tok, q_len, lq_max, p_tok, p_len, lp_max, cand_rows, B, K, S, style, bos,
                     eos, pad, out_ids, out_mask, out_type);
  SR_LAUNCH_CHECK();
}

void launch_rerank_select(const float* logits, int B, int K, int k_out, int32_t* out_index,
                          hipStream_t s) {
  SR_CHECK(K >= 1 && K <= SR_MAX_TOPK && k_out >= 1 && k_out <= K,
           "rerank_select: need 1 <= k_out <= K <= 1024");
  if (B <= 0) return;
  hipLaunchKernelGGL(rerank_select_kernel, dim3(B), dim3(256), 0, s, logits, K, k_out, out_index);
  SR_LAUNCH_CHECK();
}

}  // namespace sr
