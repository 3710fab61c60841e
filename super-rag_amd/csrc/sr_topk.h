// Block-wide exact top-k (MSB radix select + bitonic sort of the winners), shared by K2 (cosine
// candidates, k_search.hip) and the BM25 selection (k_lex.hip).
#pragma once

#include "sr_common.h"

namespace sr {

// ------------------------------------------------------------------------------------------------
// Block-wide top-k over keys in LDS.
constexpr int SEL_THREADS = 512;
constexpr int SEL_CAP = 16384;  // keys per query held in LDS (128 KiB)

__device__ __forceinline__ void bitonic_sort_desc(uint64_t* v, int n /*pow2*/) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < (n >> 1); i += blockDim.x) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const uint64_t a = v[lo], b = v[hi];
        if ((a < b) == desc) {
          v[lo] = b;
          v[hi] = a;
        }
      }
      __syncthreads();
    }
  }
}

struct SelShared {
  int hist[SEL_THREADS / 64][256];
  int tot[256];
  uint64_t sel[SR_MAX_TOPK];
  int nsel;
  int digit;
  int above;
};

// keys(i), i in [0, n): all non-zero, unique (LDS array or a gather from global memory; the
// radix passes re-read them).  On return sh.sel[0..m) holds the m = min(n, k) largest keys sorted
// descending; returns m.
template <class KeyAt>
__device__ int block_topk(KeyAt keys, int n, int k, SelShared& sh) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int shift_final = 0;
  uint64_t prefix = 0;
  if (n > k) {
    int kk = k;
    for (int shift = 56; shift >= 0; shift -= 8) {
      const uint64_t mask_hi = shift == 56 ? 0ull : (~0ull << (shift + 8));
      for (int i = tid; i < (SEL_THREADS / 64) * 256; i += blockDim.x) (&sh.hist[0][0])[i] = 0;
      __syncthreads();
      for (int i = tid; i < n; i += blockDim.x) {
        const uint64_t key = keys(i);
        if ((key & mask_hi) == prefix) atomicAdd(&sh.hist[wave][(key >> shift) & 255], 1);
      }
      __syncthreads();
      if (tid < 256) {
        int t = 0;
#pragma unroll
        for (int w = 0; w < SEL_THREADS / 64; ++w) t += sh.hist[w][tid];
        sh.tot[tid] = t;
      }
      __syncthreads();
      if (wave == 0) {
        // lane l owns digits 4l .. 4l+3; suffix sums from the top digit down.
        int c[4], t = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          c[j] = sh.tot[4 * lane + j];
          t += c[j];
        }
        int suf = t;  // inclusive suffix sum over lanes >= lane
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int v = __shfl_down(suf, o, 64);
          if (lane + o < 64) suf += v;
        }
        const uint64_t bal = __ballot(suf >= kk);
        const int L = 63 - __clzll(bal);
        if (lane == L) {
          int above = suf - t;  // keys in lanes > L
          int dsel = 4 * lane;
          for (int j = 3; j >= 0; --j) {
            if (above + c[j] >= kk) {
              dsel = 4 * lane + j;
              break;
            }
            above += c[j];
          }
          sh.digit = dsel;
          sh.above = above;
        }
      }
      __syncthreads();
      const int d = sh.digit;
      kk -= sh.above;
      prefix |= (uint64_t)d << shift;
      shift_final = shift;
      const int td = sh.tot[d];
      __syncthreads();
      if (td == kk) break;  // every key with this prefix is in the top-k
    }
  }
  if (tid == 0) sh.nsel = 0;
  __syncthreads();
  for (int i = tid; i < n; i += blockDim.x) {
    const uint64_t key = keys(i);
    if (n <= k || (key >> shift_final) >= (prefix >> shift_final)) {
      const int p = atomicAdd(&sh.nsel, 1);
      if (p < SR_MAX_TOPK) sh.sel[p] = key;
    }
  }
  __syncthreads();
  const int m = min(sh.nsel, k);
  int np2 = 1;
  while (np2 < sh.nsel) np2 <<= 1;
  np2 = min(np2, SR_MAX_TOPK);
  for (int i = sh.nsel + tid; i < np2; i += blockDim.x) sh.sel[i] = 0ull;
  __syncthreads();
  bitonic_sort_desc(sh.sel, np2);
  return m;
}

}  // namespace sr
