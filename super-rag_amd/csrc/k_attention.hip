// K5: fused multi-head self-attention for the BERT / XLM-R encoder (padding mask, online softmax).
//
//   ctx[b, s, h*DH + :] = softmax( Q_h K_h^T / sqrt(DH) + mask ) V_h
//
// Input is the fused QKV projection (M x 3d fp16, token m = b*S + s; Q at column h*DH, K at
// d + h*DH, V at 2d + h*DH).  One workgroup = up to 4 waves = 16 query rows per wave of one
// (sequence, head); key/value tiles of 64 keys are staged in LDS and shared by the waves.
//
// Scores are computed transposed (S^T = K Q^T, A = K rows from LDS, B = Q fragment kept in
// registers), so a lane holds 16 scores of ONE query: the row max / row sum need one in-lane
// reduction plus two cross-lane xor-shuffles.  The same lane layout is the B operand of the
// P.V product (O^T = V^T P^T) with a permuted k order (keys 32c+4g+j and 32c+16+4g+j for lane
// group g), so P never leaves the registers; V is stored transposed in LDS to match.
// Accumulation and softmax statistics are fp32; P is rounded to fp16 for the MFMA.
#include <algorithm>
#include <cstdlib>

#include "sr_common.h"
#include "sr_kernels.h"

namespace sr {

namespace {

// 2^x on the hardware v_exp_f32 alone: the library exp2f wraps it in a denormal-result range
// reduction (compare, select, add, ldexp: 6 instructions per score) that softmax does not need (a
// weight below 2^-126 of the row maximum adds nothing to the fp32 sums; -inf still gives 0)
__device__ __forceinline__ float exp2_fast(float x) { return __builtin_amdgcn_exp2f(x); }


constexpr int KT = 64;  // keys per tile

template <int DH>
__global__ __launch_bounds__(256) void attention_kernel(const half_t* __restrict__ qkv,
                                                        const int32_t* __restrict__ mask,
                                                        half_t* __restrict__ ctx, int S, int Sq,
                                                        int d, float scale_log2) {
  constexpr int KS = DH + 8;    // K tile row stride (halfs), padded against bank conflicts
  constexpr int VS = KT + 8;    // V^T row stride (halfs)
  constexpr int NSUB = DH / 32; // k-substeps of the QK^T MFMA
  constexpr int NDT = DH / 16;  // 16-wide d tiles of the output
  __shared__ __attribute__((aligned(16))) half_t Ks[KT * KS];
  __shared__ __attribute__((aligned(16))) half_t Vt[DH * VS];
  __shared__ float kbias[KT];

  const int nw = blockDim.x >> 6;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int h = blockIdx.y, b = blockIdx.z;
  const int q0 = blockIdx.x * (16 * nw) + 16 * wave;
  const int64_t ld = 3 * (int64_t)d;
  const half_t* base = qkv + (int64_t)b * S * ld;
  const int32_t* mrow = mask + (int64_t)b * S;

  // Q fragment (B operand): lane holds Q[q0 + (lane&15)][8*(lane>>4) + 32*s + j].
  half8 qf[NSUB];
  {
    int qr = q0 + (lane & 15);
    qr = qr < S ? qr : S - 1;
#pragma unroll
    for (int s = 0; s < NSUB; ++s)
      qf[s] = *reinterpret_cast<const half8*>(base + (int64_t)qr * ld + h * DH + 8 * (lane >> 4) + 32 * s);
  }

  float m_run = -INFINITY, l_run = 0.f;
  float4v o[NDT];
#pragma unroll
  for (int t = 0; t < NDT; ++t) o[t] = float4v{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < S; k0 += KT) {
    // ---- stage K (row-major) and V^T (transposed) for keys k0 .. k0+63 ----
    constexpr int CPR = DH / 8;  // 16-byte chunks per row
    for (int c = tid; c < KT * CPR; c += blockDim.x) {
      const int r = c & (KT - 1), ch = c / KT;  // consecutive lanes -> consecutive keys
      int key = k0 + r;
      key = key < S ? key : S - 1;
      const half_t* rowp = base + (int64_t)key * ld + h * DH + ch * 8;
      const half8 kv = *reinterpret_cast<const half8*>(rowp + d);
      const half8 vv = *reinterpret_cast<const half8*>(rowp + 2 * d);
      *reinterpret_cast<half8*>(&Ks[r * KS + ch * 8]) = kv;
#pragma unroll
      for (int j = 0; j < 8; ++j) Vt[(ch * 8 + j) * VS + r] = vv[j];
    }
    for (int r = tid; r < KT; r += blockDim.x) {
      const int key = k0 + r;
      kbias[r] = (key < S && mrow[key] != 0) ? 0.f : -INFINITY;
    }
    __syncthreads();

    // ---- S^T tiles: lane holds score(query lane&15, key 16*kt + 4*(lane>>4) + r) ----
    float p[4][4];
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      float4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NSUB; ++s) {
        const half8 kf =
            *reinterpret_cast<const half8*>(&Ks[(16 * kt + (lane & 15)) * KS + 8 * (lane >> 4) + 32 * s]);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf, qf[s], acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[r] * scale_log2 + kbias[16 * kt + 4 * (lane >> 4) + r];
        p[kt][r] = v;
        tmax = fmaxf(tmax, v);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2_fast(m_run - m_use);
    m_run = m_new;
    l_run *= alpha;
#pragma unroll
    for (int t = 0; t < NDT; ++t) o[t] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = exp2_fast(p[kt][r] - m_use);
        p[kt][r] = e;
        l_run += e;
      }

    // ---- O^T += V^T P^T over two 32-key chunks (permuted k order, see header) ----
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      half8 pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (half_t)p[2 * c][j];
        pb[4 + j] = (half_t)p[2 * c + 1][j];
      }
#pragma unroll
      for (int t = 0; t < NDT; ++t) {
        const half_t* vrow = &Vt[(16 * t + (lane & 15)) * VS + 32 * c + 4 * (lane >> 4)];
        const half4 lo = *reinterpret_cast<const half4*>(vrow);
        const half4 hi = *reinterpret_cast<const half4*>(vrow + 16);
        half8 va = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb, o[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }

  l_run += __shfl_xor(l_run, 16, 64);
  l_run += __shfl_xor(l_run, 32, 64);
  const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
  const int q = q0 + (lane & 15);
  if (q < Sq) {
    half_t* out = ctx + ((int64_t)b * Sq + q) * d + h * DH;
#pragma unroll
    for (int t = 0; t < NDT; ++t) {
      const float4v v = o[t] * inv;
      half4 hv = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
      *reinterpret_cast<half4*>(out + 16 * t + 4 * (lane >> 4)) = hv;
    }
  }
}

// ---- K5b: one workgroup per (sequence, head, 128-query block), d_h = 64 -----------------------
// The whole K and V of the head (S_pad = round_up(S, 32) rows of 128 B) are staged ONCE into LDS by
// LDS-DMA (global_load_lds_dwordx4: 8 rows per wave-instruction) and shared by the 4 waves; each
// wave owns 32 query rows (two 16-row tiles), so every K / V fragment read from LDS feeds two
// MFMAs.  Scores are S^T = K Q^T (a lane holds one query's scores: in-lane max / sum plus two
// xor-shuffles); P stays in registers as the B operand of O^T = V^T P^T, whose A operand (V^T) is
// read straight from the row-major V image with ds_read_b64_tr_b16 (no transposing LDS writes).
// LDS images (16-byte chunk c of row r):
//   K: c ^ ((r >> 1) & 7)        -- conflict-free ds_read_b128 of 16 consecutive rows
//   V: c ^ (((r >> 1) & 3) << 1) -- each 32-lane half of a transposed read touches 8 consecutive
//                                   rows x one 32-byte column pair: 8 distinct 32-byte bank slots
// Keys are processed in blocks of 128 with an online softmax (exact for any S <= 512).  Output
// tiles t = 2p, 2p+1 are merged with v_permlane16_swap so each lane stores 8 consecutive dims
// (16 B) of its query row.
constexpr int A2_QB = 128;  // query rows per workgroup

__device__ __forceinline__ int a2_kswz(int r, int c) { return c ^ ((r >> 1) & 7); }

// max / sum over the 4 lanes that share lane & 15 (one query's scores): v_permlane16_swap and
// v_permlane32_swap exchange 16-lane rows in VALU, where __shfl_xor is an LDS round trip; with
// a == b each result pair holds {own, partner}, so the pair's max / sum is the butterfly step (sums
// are commutative: bit-identical to the shuffle form)
__device__ __forceinline__ float rows4_max(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float rows4_sum(float x) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ int a2_vswz(int r, int c) { return c ^ (((r >> 1) & 3) << 1); }

// A operand of the row-sum MFMA: D = ones(16 x 32) . P^T puts the sum of a query's 32 fp16
// probabilities in all 16 rows of its column, so the softmax denominator costs one MFMA per
// 32-key chunk instead of a VALU add per score (and it sums exactly the fp16 weights P.V uses)
__device__ __forceinline__ half8 a2_ones() {
  const half_t one = (half_t)1.0f;
  return half8{one, one, one, one, one, one, one, one};
}

__device__ __forceinline__ half4 tr_read_b64(const half_t* p) {
  typedef short short4_t __attribute__((ext_vector_type(4)));
  short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) short4_t*)(p));
  return __builtin_bit_cast(half4, v);
}

// The transposed V reads of one 32-key chunk (4 d-tiles x lo / hi rows) as ONE inline-asm block that
// ends with its own lgkmcnt(0): the compiler cannot see them as LDS accesses, so it does not wait
// for every in-flight LDS-DMA piece before them (it does before the builtin), and no use of the
// results can be scheduled before the data has arrived (STREAM).
__device__ __forceinline__ void tr_read_chunk_asm(const uint32_t (&addr)[8], uint2 (&v)[8]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\tds_read_b64_tr_b16 %1, %9\n\t"
      "ds_read_b64_tr_b16 %2, %10\n\tds_read_b64_tr_b16 %3, %11\n\t"
      "ds_read_b64_tr_b16 %4, %12\n\tds_read_b64_tr_b16 %5, %13\n\t"
      "ds_read_b64_tr_b16 %6, %14\n\tds_read_b64_tr_b16 %7, %15\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
        "=&v"(v[7])
      : "v"(addr[0]), "v"(addr[1]), "v"(addr[2]), "v"(addr[3]), "v"(addr[4]), "v"(addr[5]),
        "v"(addr[6]), "v"(addr[7])
      : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const half_t* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// ---- one 128-key block for a wave's two 16-query tiles, software-pipelined (STREAM / K5d) ----
// scores S^T = K Q^T of both tiles (16 K fragments, 32 MFMAs)
__device__ __forceinline__ void a2_blk_scores(const half_t* Ks, int k0, const half8 (&qf)[2][2], int lane,
                                              float4v (&sc)[2][8]) {
  constexpr int DH = 64;
  const int g = lane >> 4;
  half8 kf[8][2];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    const int kr = k0 + 16 * kt + (lane & 15);
    kf[kt][0] = *reinterpret_cast<const half8*>(Ks + kr * DH + a2_kswz(kr, g) * 8);
    kf[kt][1] = *reinterpret_cast<const half8*>(Ks + kr * DH + a2_kswz(kr, g + 4) * 8);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      float4v a = {0.f, 0.f, 0.f, 0.f};
      a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kt][0], qf[u][0], a, 0, 0, 0);
      sc[u][kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kt][1], qf[u][1], a, 0, 0, 0);
    }
}

// V^T fragments of the block's four 32-key chunks (key order 32c + 4g + j, then 32c + 16 + 4g + j),
// each chunk one asm block ending in its own lgkmcnt(0) (tr_read_chunk_asm: no compiler vmcnt(0)
// for the LDS-DMA pieces still in flight)
__device__ __forceinline__ void a2_blk_vfrags(const half_t* Vs, int k0, int lane, half8 (&va)[4][4]) {
  constexpr int DH = 64;
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    uint32_t addr[8];
    uint2 vv[8];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = k0 + 32 * c + 16 * hh + 4 * g + q;
        addr[2 * t + hh] = lds_addr(Vs + r * DH + a2_vswz(r, 2 * t + (pp >> 1)) * 8 + 4 * (pp & 1));
      }
    tr_read_chunk_asm(addr, vv);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const half4 lo = __builtin_bit_cast(half4, vv[2 * t]), hi = __builtin_bit_cast(half4, vv[2 * t + 1]);
      va[c][t] = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  }
}

// online softmax of the block (running max, rescale) and O^T += V^T P^T, lsum += ones . P^T
__device__ __forceinline__ void a2_blk_softmax_pv(float4v (&sc)[2][8], const half8 (&va)[4][4],
                                                  const float* kbias, int k0, int lane, float scale_log2,
                                                  float (&m_run)[2], float4v (&o)[2][4],
                                                  float4v (&lsum)[2]) {
  const int g = lane >> 4;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    float tmax = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = sc[u][kt][r] * scale_log2 + kbias[k0 + 16 * kt + 4 * g + r];
        sc[u][kt][r] = v;
        tmax = fmaxf(tmax, v);
      }
    const float tm = rows4_max(tmax);
    const float m_new = fmaxf(m_run[u], tm);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2_fast(m_run[u] - m_use);
    m_run[u] = m_new;
    lsum[u] *= alpha;
#pragma unroll
    for (int t = 0; t < 4; ++t) o[u][t] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[u][kt][r] = exp2_fast(sc[u][kt][r] - m_use);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      half8 pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (half_t)sc[u][2 * c][j];
        pb[4 + j] = (half_t)sc[u][2 * c + 1][j];
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
        o[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[c][t], pb, o[u][t], 0, 0, 0);
      lsum[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2_ones(), pb, lsum[u], 0, 0, 0);
    }
  }
}

// SPLIT (S_pad == 128, all four waves active): the Q fragments and the key mask are requested
// first, then K (LDS-DMA), then V into registers; the score / softmax phase starts once Q and K
// have landed (vmcnt(4): each wave's four V loads may still be in flight) and V is written to its
// LDS image (same swizzle) only before the first P.V MFMA, so V's HBM latency overlaps QK^T +
// softmax.  (V by LDS-DMA would make the compiler wait vmcnt(0) before every ds_read of K.)  amdgpu_waves_per_eu(3): 168
// VGPRs, three workgroups per CU (two query tiles per wave stay interleaved for MFMA ILP).
// NW waves per workgroup (32 query rows each): 4, or 8 for S_pad > 256, where the whole-head K/V
// image (up to 130 KiB at S_pad = 512) allows one workgroup per CU and is then shared by 256
// queries: half the re-staging and two waves per SIMD (S = 512: 3.25 -> 2.04 ms per 1024 x 12
// heads; 16 waves at 128 VGPRs spill and ran 2.73 ms).  SPLIT implies NW == 4.
// STREAM (NW == 8, S_pad == 512, every wave active): K/V pieces are issued in key-block order and
// each 128-key block is awaited only before it is used (counted vmcnt + barrier), so blocks 1..3
// land while block 0.. are being processed; Q and the mask word are loaded right after block 0
// and waited for with it (no plain load is outstanding afterwards, so the counted waits stay exact).
template <bool SPLIT, int NW, bool STREAM = false>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(NW == 8 ? 2 : 3, NW == 8 ? 2 : 3)))
void attention64_kernel(
    const half_t* __restrict__ qkv, const int32_t* __restrict__ mask, half_t* __restrict__ ctx,
    int S, int Sq, int d, float scale_log2) {
  constexpr int DH = 64;
  extern __shared__ __attribute__((aligned(16))) char a2_smem[];
  static_assert(!STREAM || (NW == 8 && !SPLIT), "STREAM runs the 8-wave non-split form");
  const int S_pad = SPLIT ? 128 : STREAM ? 512 : (S + 31) & ~31;
  half_t* Ks = reinterpret_cast<half_t*>(a2_smem);
  half_t* Vs = Ks + S_pad * DH;
  float* kbias = reinterpret_cast<float*>(Vs + S_pad * DH);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = blockIdx.y, b = blockIdx.z;
  const int64_t ld = 3 * (int64_t)d;
  const half_t* base = qkv + (int64_t)b * S * ld + h * DH;

  static_assert(!SPLIT || NW == 4, "SPLIT stages with four waves");
  const int qw = blockIdx.x * (32 * NW) + wave * 32;  // first query row of this wave
  const bool active = qw < Sq;
  half8 qf[2][2];
  half8 vreg[4];  // SPLIT: this wave's V pieces (written to the LDS image after the softmax)
  if constexpr (SPLIT) {
    // Q rows (this workgroup's 128), the key mask words and K by LDS-DMA, then V into registers:
    // no register result is needed before the V loads issue, so one counted wait (vmcnt(4) = all
    // but this wave's 4 V loads) publishes Q, mask and K.
    half_t* Qs = reinterpret_cast<half_t*>(kbias + S_pad);  // 128 rows x 128 B, K's swizzle
    int32_t* ms = reinterpret_cast<int32_t*>(kbias);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int piece = wave + 4 * i;
      const int r = piece * 8 + (lane >> 3);
      const int rq = blockIdx.x * A2_QB + r;
      __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)(rq < S ? rq : S - 1) * ld +
                                                     a2_kswz(r, lane & 7) * 8),
                                       SR_LDS(Qs + piece * 8 * DH), 16, 0, 0);
    }
    if (wave < 2) {
      const int r = wave * 64 + lane;
      __builtin_amdgcn_global_load_lds((const void*)(mask + (int64_t)b * S + (r < S ? r : S - 1)),
                                       SR_LDS(ms + wave * 64), 4, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int piece = wave + 4 * i;
      const int r = piece * 8 + (lane >> 3);
      __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)(r < S ? r : S - 1) * ld + d +
                                                     a2_kswz(r, lane & 7) * 8),
                                       SR_LDS(Ks + piece * 8 * DH), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (wave + 4 * i) * 8 + (lane >> 3);
      vreg[i] = *reinterpret_cast<const half8*>(base + (int64_t)(r < S ? r : S - 1) * ld + 2 * d +
                                                a2_vswz(r, lane & 7) * 8);
    }
    SR_WAITCNT(4, 0);
    __builtin_amdgcn_s_barrier();
    // mask words -> additive key bias in place (keys >= S masked), then the Q fragments
    if (wave < 2) {
      const int r = wave * 64 + lane;
      const int32_t m = ms[r];
      kbias[r] = (r < S && m != 0) ? 0.f : -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = wave * 32 + 16 * u + (lane & 15);
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        qf[u][s2] = *reinterpret_cast<const half8*>(Qs + r * DH + a2_kswz(r, (lane >> 4) + 4 * s2) * 8);
    }
    SR_WAITCNT(4, 0);
    __builtin_amdgcn_s_barrier();
  } else if constexpr (STREAM) {
    auto stage_blk = [&](int blk) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int piece = blk * 16 + wave + 8 * i;
        const int r = piece * 8 + (lane >> 3);
        __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)(r < S ? r : S - 1) * ld + d +
                                                       a2_kswz(r, lane & 7) * 8),
                                         SR_LDS(Ks + piece * 8 * DH), 16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int piece = blk * 16 + wave + 8 * i;
        const int r = piece * 8 + (lane >> 3);
        __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)(r < S ? r : S - 1) * ld + 2 * d +
                                                       a2_vswz(r, lane & 7) * 8),
                                         SR_LDS(Vs + piece * 8 * DH), 16, 0, 0);
      }
    };
    stage_blk(0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int qr = qw + 16 * u + (lane & 15);
      qr = qr < S ? qr : S - 1;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        qf[u][s2] = *reinterpret_cast<const half8*>(base + (int64_t)qr * ld + 8 * (lane >> 4) + 32 * s2);
    }
    const int32_t mk = mask[(int64_t)b * S + (tid < S ? tid : S - 1)];
    SR_WAITCNT(0, 15);  // block 0, Q and the mask word
    stage_blk(1);
    stage_blk(2);
    stage_blk(3);
    kbias[tid] = (tid < S && mk != 0) ? 0.f : -INFINITY;  // 512 threads = S_pad keys
    SR_WAITCNT(12, 0);
    __builtin_amdgcn_s_barrier();
  } else {
    // ---- Q fragments (B operand of S^T): lane holds Q[q][8 (lane>>4) + 32 s .. +7] ----
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int qr = qw + 16 * u + (lane & 15);
      qr = qr < S ? qr : S - 1;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        qf[u][s2] = *reinterpret_cast<const half8*>(base + (int64_t)qr * ld + 8 * (lane >> 4) + 32 * s2);
    }
    // ---- stage K and V (rows >= S replicate row S-1; their keys are masked) ----
    for (int piece = wave; piece < S_pad / 8; piece += NW) {
      const int r = piece * 8 + (lane >> 3);
      const int rr = r < S ? r : S - 1;
      const half_t* rowp = base + (int64_t)rr * ld;
      __builtin_amdgcn_global_load_lds((const void*)(rowp + d + a2_kswz(r, lane & 7) * 8),
                                       SR_LDS(Ks + piece * 8 * DH), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(rowp + 2 * d + a2_vswz(r, lane & 7) * 8),
                                       SR_LDS(Vs + piece * 8 * DH), 16, 0, 0);
    }
    for (int r = tid; r < S_pad; r += 64 * NW)
      kbias[r] = (r < S && mask[(int64_t)b * S + r] != 0) ? 0.f : -INFINITY;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (!SPLIT && !STREAM && !active) return;  // no barrier follows

  const int g = lane >> 4;
  float m_run[2] = {-INFINITY, -INFINITY};
  // o: O^T tiles; lsum: the softmax denominators, accumulated by one extra MFMA per 32-key chunk
  // with an all-ones A operand (every element of lsum[u] = the row sum of the fp16 P it multiplies)
  float4v o[2][4], lsum[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    lsum[u] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) o[u][t] = float4v{0.f, 0.f, 0.f, 0.f};
  }

  for (int k0 = 0; k0 < S_pad; k0 += 128) {
    if constexpr (STREAM) {  // key block k0 / 128 (this wave's later blocks may still be in flight)
      if (k0 > 0) {
        if (k0 == 128) SR_WAITCNT(8, 15);
        else if (k0 == 256) SR_WAITCNT(4, 15);
        else SR_WAITCNT(0, 15);
        __builtin_amdgcn_s_barrier();
      }
      // software-pipelined per 16-query tile u (as K5c): both tiles' score MFMAs and the block's
      // V^T fragments are issued first, then tile 0's softmax runs while tile 1's scores finish and
      // tile 1's softmax beside tile 0's P.V.  Per-value operation order is the generic path's.
      float4v sc[2][8];
      a2_blk_scores(Ks, k0, qf, lane, sc);
      half8 va[4][4];
      a2_blk_vfrags(Vs, k0, lane, va);
      a2_blk_softmax_pv(sc, va, kbias, k0, lane, scale_log2, m_run, o, lsum);
      continue;
    }
    const int nkt = (S_pad - k0) >= 128 ? 8 : (S_pad - k0) / 16;  // 16-key tiles in this block
    float p[2][8][4];
    float tmax[2] = {-INFINITY, -INFINITY};
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      if (kt < nkt) {
        const int kr = k0 + 16 * kt + (lane & 15);
        const half8 k0f = *reinterpret_cast<const half8*>(Ks + kr * DH + a2_kswz(kr, g) * 8);
        const half8 k1f = *reinterpret_cast<const half8*>(Ks + kr * DH + a2_kswz(kr, g + 4) * 8);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float4v acc = {0.f, 0.f, 0.f, 0.f};
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(k0f, qf[u][0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(k1f, qf[u][1], acc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = acc[r] * scale_log2 + kbias[k0 + 16 * kt + 4 * g + r];
            p[u][kt][r] = v;
            tmax[u] = fmaxf(tmax[u], v);
          }
        }
      } else {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int r = 0; r < 4; ++r) p[u][kt][r] = -INFINITY;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const float tm = rows4_max(tmax[u]);
      const float m_new = fmaxf(m_run[u], tm);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = exp2_fast(m_run[u] - m_use);
      m_run[u] = m_new;
      lsum[u] *= alpha;
#pragma unroll
      for (int t = 0; t < 4; ++t) o[u][t] *= alpha;
#pragma unroll
      for (int kt = 0; kt < 8; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) p[u][kt][r] = exp2_fast(p[u][kt][r] - m_use);
    }
    // ---- O^T += V^T P^T over 32-key chunks (key order of the B operand: 32c + 4g + j, then
    //      32c + 16 + 4g + j; the transposed V reads use the same order) ----
    if constexpr (SPLIT) {  // one key block: V lands in LDS here, once
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<half8*>(Vs + (wave + 4 * i) * 8 * DH + lane * 8) = vreg[i];
      SR_WAITCNT(0, 0);
      __builtin_amdgcn_s_barrier();
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (2 * c < nkt) {
        half8 pb[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            pb[u][j] = (half_t)p[u][2 * c][j];
            pb[u][4 + j] = (half_t)p[u][2 * c + 1][j];
          }
        // lane 4q+p of group g: V row k0 + 32c + 16hh + 4g + q, dims 16t + 4p .. +3
        const int q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
        for (int u = 0; u < 2; ++u)
          lsum[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2_ones(), pb[u], lsum[u], 0, 0, 0);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          half4 lo, hi;
          {
            const int r = k0 + 32 * c + 4 * g + q;
            const int ch = a2_vswz(r, 2 * t + (pp >> 1));
            lo = tr_read_b64(Vs + r * DH + ch * 8 + 4 * (pp & 1));
          }
          {
            const int r = k0 + 32 * c + 16 + 4 * g + q;
            const int ch = a2_vswz(r, 2 * t + (pp >> 1));
            hi = tr_read_b64(Vs + r * DH + ch * 8 + 4 * (pp & 1));
          }
          const half8 va = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
          for (int u = 0; u < 2; ++u)
            o[u][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb[u], o[u][t], 0, 0, 0);
        }
      }
    }
  }

  // ---- normalise and store: permlane16_swap merges d-tiles (2p, 2p+1) -> 8 dims per lane ----
  const int odd = g & 1;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const float l = lsum[u][0];
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int q = qw + 16 * u + (lane & 15);
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      half8 hv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(o[u][2 * pp][r]),
                                                         __float_as_uint(o[u][2 * pp + 1][r]), false, false);
        hv[r] = (half_t)(__uint_as_float(sw[0]) * inv);
        hv[4 + r] = (half_t)(__uint_as_float(sw[1]) * inv);
      }
      if (q < Sq)
        *reinterpret_cast<half8*>(ctx + ((int64_t)b * Sq + q) * d + h * DH + 32 * pp + 16 * odd + 4 * (g & 2)) = hv;
    }
  }
}


// ---- K5d: persistent S_pad = 512 attention (d_h = 64, every query; the long-pair reranker) -------
// One 8-wave workgroup per CU walks its XCD's contiguous range of (sequence, head) tiles.  The
// head's whole K / V (4 key blocks of 128 rows, K5b's swizzles) stays in LDS for BOTH 256-query
// passes (A: queries 0..255, B: 256..511), so K and V leave HBM once per (sequence, head) instead
// of once per 256 queries (K5b STREAM).  During pass B each key block, once every wave is past
// it, is refilled by LDS-DMA with the next tile's, and the next pass's Q fragments are loaded right
// after the last block's score MFMAs, so the next tile's loads run under this tile's pass B.  The
// block body is STREAM's (a2_blk_*): per-value operation order, and so the results, are K5b's.
// Waits (per wave, VMEM ops retire in order; stores count): tile prologue vmcnt(12) = block 0,
// Q, mask (blocks 1..3 in flight); pass A block b: vmcnt(8 / 4 / 0) for blocks 1 / 2 / 3; pass B
// block 0: vmcnt(4) = its Q (pass A's 4 ctx stores may be in flight); next tile: vmcnt(8) =
// blocks 0..2, Q and mask (younger: pass B's 4 ctx stores and block 3).  A barrier before every
// block (measured: refilling blocks 0 / 1 together and 2 / 3 after the pass with four barriers
// per tile ran 1.57 instead of 1.39 ms per 1024 x 12-head launch).
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void attention512_kernel(const half_t* __restrict__ qkv, const int32_t* __restrict__ mask,
                         half_t* __restrict__ ctx, int B, int S, int Sq, int d, int heads,
                         float scale_log2) {
  constexpr int DH = 64, SP = 512;
  __shared__ __attribute__((aligned(16))) half_t lds[2 * SP * DH + 2 * SP];  // K, V images, key bias
  half_t* const Ks = lds;
  half_t* const Vs = lds + SP * DH;
  float* const kbias = reinterpret_cast<float*>(lds + 2 * SP * DH);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int ntiles = B * heads;
  int t, t_end;
  const int t_step = gridDim.x >> 3;
  {
    const int xcd = blockIdx.x & 7, q = ntiles >> 3, rem = ntiles & 7;
    const int lo = xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
    t_end = lo + q + (xcd < rem ? 1 : 0);
    t = lo + (blockIdx.x >> 3);
    if (t >= t_end || t_step <= 0) return;
  }
  const int64_t ld = 3 * (int64_t)d;
  auto stage_blk = [&](const half_t* base, int blk) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int piece = blk * 16 + wave + 8 * i;
      const int r = piece * 8 + (lane >> 3);
      __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)(r < S ? r : S - 1) * ld + d +
                                                     a2_kswz(r, lane & 7) * 8),
                                       SR_LDS(Ks + piece * 8 * DH), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int piece = blk * 16 + wave + 8 * i;
      const int r = piece * 8 + (lane >> 3);
      __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)(r < S ? r : S - 1) * ld + 2 * d +
                                                     a2_vswz(r, lane & 7) * 8),
                                       SR_LDS(Vs + piece * 8 * DH), 16, 0, 0);
    }
  };
  half8 qf[2][2];
  auto load_q = [&](const half_t* base, int q0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int qr = q0 + wave * 32 + 16 * u + (lane & 15);
      qr = qr < S ? qr : S - 1;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
        qf[u][s2] = *reinterpret_cast<const half8*>(base + (int64_t)qr * ld + 8 * (lane >> 4) + 32 * s2);
    }
  };
  int b = t / heads, h = t % heads;
  const half_t* base = qkv + (int64_t)b * S * ld + h * DH;
  stage_blk(base, 0);
  load_q(base, 0);
  int32_t mk = mask[(int64_t)b * S + (tid < S ? tid : S - 1)];
  stage_blk(base, 1);
  stage_blk(base, 2);
  stage_blk(base, 3);
  SR_WAITCNT(12, 15);
  kbias[tid] = (tid < S && mk != 0) ? 0.f : -INFINITY;  // 512 threads = SP keys

  for (;;) {
    const int t_next = t + t_step;
    const bool more = t_next < t_end;
    const int b_n = more ? t_next / heads : b, h_n = more ? t_next % heads : h;
    const half_t* base_n = qkv + (int64_t)b_n * S * ld + h_n * DH;
    for (int pass = 0; pass < 2; ++pass) {
      float m_run[2] = {-INFINITY, -INFINITY};
      float4v o[2][4], lsum[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        lsum[u] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) o[u][tt] = float4v{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll 1
      for (int blk = 0; blk < 4; ++blk) {
        if (pass == 0) {
          if (blk == 1) SR_WAITCNT(8, 15);
          else if (blk == 2) SR_WAITCNT(4, 15);
          else if (blk == 3) SR_WAITCNT(0, 15);
        } else if (blk == 0) {
          SR_WAITCNT(4, 15);
        }
        __builtin_amdgcn_s_barrier();
        // pass B: every wave is past block blk - 1 -> the next tile's block blk - 1 goes there
        if (pass == 1 && blk > 0 && more) stage_blk(base_n, blk - 1);
        const int k0 = blk * 128;
        float4v sc[2][8];
        a2_blk_scores(Ks, k0, qf, lane, sc);
        if (blk == 3) {  // qf is free: the next pass's Q fragments (and the next tile's mask word)
          if (pass == 0) {
            load_q(base, 256);
          } else if (more) {
            load_q(base_n, 0);
            mk = mask[(int64_t)b_n * S + (tid < S ? tid : S - 1)];
          }
        }
        half8 va[4][4];
        a2_blk_vfrags(Vs, k0, lane, va);
        a2_blk_softmax_pv(sc, va, kbias, k0, lane, scale_log2, m_run, o, lsum);
      }
      // normalise and store this pass's 256 queries (permlane16_swap: 8 consecutive dims per lane)
      const int odd = g & 1;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float l = lsum[u][0];
        const float inv = l > 0.f ? 1.f / l : 0.f;
        const int q = pass * 256 + wave * 32 + 16 * u + (lane & 15);
#pragma unroll
        for (int p2 = 0; p2 < 2; ++p2) {
          half8 hv;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(o[u][2 * p2][r]),
                                                             __float_as_uint(o[u][2 * p2 + 1][r]), false, false);
            hv[r] = (half_t)(__uint_as_float(sw[0]) * inv);
            hv[4 + r] = (half_t)(__uint_as_float(sw[1]) * inv);
          }
          if (q < Sq)
            *reinterpret_cast<half8*>(ctx + ((int64_t)b * Sq + q) * d + h * DH + 32 * p2 + 16 * odd + 4 * (g & 2)) = hv;
        }
      }
    }
    if (!more) break;
    __builtin_amdgcn_s_barrier();  // every wave is past block 3 and done with the key bias
    stage_blk(base_n, 3);
    SR_WAITCNT(8, 15);
    kbias[tid] = (tid < S && mk != 0) ? 0.f : -INFINITY;
    t = t_next;
    b = b_n;
    h = h_n;
    base = base_n;
  }
}

// ---- K5c: fused QKV projection + attention (S == 128, d_h == 64; the cross-encoder layers) ------
// One workgroup per (256-token panel = two sequences, head h): the 256 x 192 tile
// [Q_h | K_h | V_h] = epi(X . W_h^T) over K = d runs K4's pipelined main loop (LDS-DMA double
// buffer, XOR-swizzled 128-B rows, four MFMA phases per K-step, the K-step-parity wave group issuing
// the staging burst); its epilogue (bias, or the LayerNorm fold rstd (acc - mu c) + b') writes the
// fp16 Q, K, V of the panel into LDS images laid out as K5b's (K / Q: kswz, V: vswz) instead of
// HBM, and the same 8 waves then run K5b's attention on them (waves 4s .. 4s+3: sequence s,
// 32 queries each).  The QKV activation never touches HBM: per token 4.6 KB of writes and reads
// disappear.  Numerics equal the unfused pair bit for bit (same MFMA order per accumulator, same
// epilogue FMAs, same fp16 rounding, same attention code order).
// The next tile's epilogue constants (bias / column sums of its head, row statistics and key mask
// of its panel) are staged into LDS with its K-step 0 (K5c 1,021-1,025 -> 1,028 TF/s;
// profiles/r05_k5c_cstl/).  (Staging the next tile's K-step 1 mid-attention into the dead Q / K
// images instead of after it: +0.3 % K5c alone, but 24 B of spills beside the constants; not kept.)
constexpr int QA_BM = 256;              // tokens per panel
constexpr int QA_BN = 192;              // Q_h, K_h, V_h rows of W
constexpr int QA_STAGE = (QA_BM + QA_BN) * 64;  // halfs per K-step buffer (56 KiB)

__device__ __forceinline__ half8 qa_frag(const half_t* t, int row, int chunk) {
  return *reinterpret_cast<const half8*>(t + row * 64 + a2_kswz(row, chunk) * 8);
}

// 12-MFMA phase: R fragment reads spread among the first MFMAs
#define SR_QA_INTERLEAVE(R)                                                \
  do {                                                                     \
    _Pragma("unroll") for (int _r = 0; _r < (R); ++_r) {                   \
      __builtin_amdgcn_sched_group_barrier(0x008, (R) >= 8 ? 1 : 2, 0);    \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                   \
    }                                                                      \
    __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);                    \
    __builtin_amdgcn_sched_barrier(0);                                     \
  } while (0)

// DIAG (timing experiments only, wrong results): 1 = no K-loop (epilogue + attention on zero
// accumulators), 2 = no attention (the K-loop and the LDS epilogue only).
// CTX8: ctx is written as OCP e4m3 bytes (fp8 mode 5: the O-projection's operand on the
// block-scaled fp8 MFMA), 8 B per lane store instead of 16 -- same store count, so the vmcnt
// bookkeeping below is unchanged.
template <bool LNF, int DIAG = 0, bool CTX8 = false>
__global__ __launch_bounds__(512, 1) void qkv_attn_kernel(
    const half_t* __restrict__ X, int64_t lda, const half_t* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ colsum, const float* __restrict__ mr,
    const int32_t* __restrict__ mask, half_t* __restrict__ ctx, int M, int d, int heads,
    float scale_log2, int hg, uint64_t* __restrict__ stamps) {
  constexpr int DH = 64;
  // DIAG 3 (diagnostic library): per-wave s_memtime phase sums of every tile -- the K-loop, the
  // epilogue into the LDS images, the attention, the tile transition -- stored once at the end
  // (stamps: uint64 [grid x 8 waves x 8] = [tiles, K-loop, epilogue, attention, transition, 0..])
  constexpr bool STAMP = DIAG == 3;
  uint32_t st_t0 = 0, st_sum[5] = {0, 0, 0, 0, 0};
  auto stamp = [&](int phase) __attribute__((always_inline)) {
    if constexpr (STAMP) {
      const uint32_t t1 = (uint32_t)__builtin_amdgcn_s_memtime();
      st_sum[phase] = __builtin_amdgcn_readfirstlane(st_sum[phase] + (t1 - st_t0));
      st_t0 = t1;
    }
  };
  (void)stamps;
  constexpr int IMG = 3 * QA_BM * DH;  // Q, K, V images (96 KiB)
  // LDS: the images, then one K-step buffer (PB) past them; odd K-steps use PA = the first 56 KiB
  // of the image area (dead during the K-loop).  So the next tile's K-step 0 (PB) is staged while
  // this tile's attention reads the images, and its K-step 1 (PA) right after.
  // CSTL: past PB, the tile's epilogue constants (floats): [3 x 64 bias][3 x 64 column sums]
  // [256 x (mu, rstd)][256 key mask (int)] = 4.5 KiB
  constexpr int QA_CSTH = 2304;
  __shared__ __attribute__((aligned(16))) half_t lds[IMG + QA_STAGE + QA_CSTH];
  __shared__ float kbias[QA_BM];
  half_t* const PA = lds;
  half_t* const PB = lds + IMG;
  float* const qcst = reinterpret_cast<float*>(lds + IMG + QA_STAGE);
  (void)qcst;
  // persistent walkers: tile t = (panel, head), head fastest; every XCD walks a contiguous range
  // of tiles so the 12 heads of a panel share its X rows in that XCD's L2 (W stays L2-resident)
  const int panels = (M + QA_BM - 1) / QA_BM, nwg = panels * heads;
  int t, t_end;
  const int t_step = gridDim.x >> 3;
  {
    const int xcd = blockIdx.x & 7, q = nwg >> 3, rem = nwg & 7;
    const int lo = xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
    t_end = lo + q + (xcd < rem ? 1 : 0);
    t = lo + (blockIdx.x >> 3);
    if (t >= t_end || t_step <= 0) return;
  }
  // tile t -> (head group, panel, head in the group), head fastest: the heads are walked in groups
  // of hg (hg = heads: every head of a panel in turn), so an XCD's ~32 concurrent tiles need the W
  // slices of hg heads and ~32 / hg X panels at a time
  const int pg = panels * hg;
  auto tile_h = [&](int tt) __attribute__((always_inline)) { return (tt / pg) * hg + (tt % pg) % hg; };
  auto tile_m = [&](int tt) __attribute__((always_inline)) { return ((tt % pg) / hg) * QA_BM; };
  int h = tile_h(t), m0 = tile_m(t);
  const int K = d, nk = K / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave >> 2, wm = wave & 3, grp = wave >> 2, w4 = wave & 3;
  const int arow = wn * 96 + (lane & 15), brow = wm * 64 + (lane & 15), c0 = lane >> 4;
  (void)w4;

  // staging: the 4 waves of group (kt & 1) issue K-step kt: 6 W pieces (8 rows of one of the
  // Q / K / V segments) + 8 X pieces each
  uint32_t vbw[2], vbx[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int ch = (lane & 7) ^ ((lane >> 4) + 4 * par);
    vbw[par] = (uint32_t)(((int64_t)(lane >> 3) * K + ch * 8) * 2);
    vbx[par] = (uint32_t)(((int64_t)(lane >> 3) * lda + ch * 8) * 2);
  }
  auto stage = [&](int kt, half_t* s, int mm, int hh) __attribute__((always_inline)) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto rw = panel_rsrc(W, (int64_t)3 * d * K * 2);
    const auto rx = panel_rsrc(X + (int64_t)mm * lda, (int64_t)(M - mm < QA_BM ? M - mm : QA_BM) * lda * 2);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int p = w4 * 6 + i;  // rows 8p .. 8p+7 of the tile: segment p >> 3 (Q, K, V)
      const int grow = (p >> 3) * d + hh * DH + 8 * (p & 7);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, SR_LDS(s + p * 8 * 64), 16, vbw[i & 1],
                                               grow * K * 2 + kt * 128, 0, 0);
    }
    int sx = w4 * 8 * 16 * (int)lda + kt * 128;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      asm volatile("" : "+s"(sx));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, SR_LDS(s + (QA_BN + (w4 * 8 + i) * 8) * 64), 16,
                                               vbx[i & 1], sx, 0, 0);
      sx += 16 * (int)lda;
    }
#endif
  };

  // CSTL: group 0's waves stage a tile's constants beside its K-step 0 (older than their ctx
  // stores, so the transition's wait covers them): wave 0 the bias of the head's Q / K / V rows
  // (3 x 256 B), wave 1 their column sums, wave 2 the panel's row statistics (2 x 1 KiB), wave 3 its
  // key mask (1 KiB); rows past M read as zero (masked keys, never stored)
  auto stage_cst = [&](int mm, int hh) __attribute__((always_inline)) {
#if defined(__HIP_DEVICE_COMPILE__)
    {
      const uint32_t l4 = (uint32_t)lane * 4u, l16 = l4 * 4u;
      const int nrow = __builtin_amdgcn_readfirstlane(max(0, min(QA_BM, M - mm)));
      if (w4 < 2) {
        const float* src = w4 == 0 ? bias : colsum;
        if (w4 == 0 || LNF) {
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            const auto r = panel_rsrc(reinterpret_cast<const half_t*>(src + (int64_t)q * d + hh * DH), 256);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, SR_LDS(qcst + 192 * w4 + 64 * q), 4, l4, 0, 0, 0);
          }
        }
      } else if (w4 == 2) {
        if (LNF) {
          const auto r = panel_rsrc(reinterpret_cast<const half_t*>(mr + (int64_t)mm * 2), (int64_t)nrow * 8);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r, SR_LDS(qcst + 384), 16, l16, 0, 0, 0);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(r, SR_LDS(qcst + 640), 16, l16, 1024, 0, 0);
        }
      } else {
        const auto r = panel_rsrc(reinterpret_cast<const half_t*>(mask + mm), (int64_t)nrow * 4);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, SR_LDS(qcst + 896), 16, l16, 0, 0, 0);
      }
    }
#endif
  };

  float4v acc[6][4];
  half8 aX[3], aY[3], bX[4], bY[4];

  // first tile: group 0 stages K-step 0 (PB) and waits for it, group 1 K-step 1 (PA)
  if (grp == 0) {
    stage(0, PB, m0, h);
    stage_cst(m0, h);
    SR_WAITCNT(0, 15);
  } else if (nk > 1) {
    stage(1, PA, m0, h);
  }
  __builtin_amdgcn_s_barrier();
  if constexpr (STAMP) st_t0 = (uint32_t)__builtin_amdgcn_s_memtime();

  for (;;) {
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 3; ++i) aY[i] = qa_frag(PB, arow + 16 * i, c0);
#pragma unroll
    for (int j = 0; j < 4; ++j) bX[j] = qa_frag(PB + QA_BN * 64, brow + 16 * j, c0);

    for (int kt = 0; kt < (DIAG == 1 ? 0 : nk); ++kt) {
      half_t* cur = (kt & 1) ? PA : PB;
      const half_t* nxt = (kt & 1) ? PB : PA;
      const half_t* Bc = cur + QA_BN * 64;
      // p0: A[0..2] x B (k 0..31); reads A[3..5] (k 0..31)
#pragma unroll
      for (int i = 0; i < 3; ++i) aX[i] = qa_frag(cur, arow + 16 * (3 + i), c0);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aY[i], bX[j], acc[i][j], 0, 0, 0);
      SR_QA_INTERLEAVE(3);
      // p1: A[3..5] x B (k 0..31); reads A[0..2], B (k 32..63)
#pragma unroll
      for (int i = 0; i < 3; ++i) aY[i] = qa_frag(cur, arow + 16 * i, c0 + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) bY[j] = qa_frag(Bc, brow + 16 * j, c0 + 4);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[3 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aX[i], bX[j], acc[3 + i][j], 0, 0, 0);
      SR_QA_INTERLEAVE(7);
      // p2: A[0..2] x B' (k 32..63); reads A[3..5] (k 32..63)
#pragma unroll
      for (int i = 0; i < 3; ++i) aX[i] = qa_frag(cur, arow + 16 * (3 + i), c0 + 4);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aY[i], bY[j], acc[i][j], 0, 0, 0);
      SR_QA_INTERLEAVE(3);
      SR_WAITCNT(0, 0);  // K-step kt+1 landed (all waves); buffer kt & 1 is no longer read
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nk && grp == (kt & 1)) stage(kt + 2, cur, m0, h);
      // p3: A[3..5] x B' (k 32..63); reads K-step kt+1's p0 operands
      const bool rn = kt + 1 < nk;
      if (rn) {
#pragma unroll
        for (int i = 0; i < 3; ++i) aY[i] = qa_frag(nxt, arow + 16 * i, c0);
#pragma unroll
        for (int j = 0; j < 4; ++j) bX[j] = qa_frag(nxt + QA_BN * 64, brow + 16 * j, c0);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[3 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aX[i], bY[j], acc[3 + i][j], 0, 0, 0);
      if (rn) {
        SR_QA_INTERLEAVE(7);
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    stamp(1);  // the K-loop
    // ---- epilogue -> LDS images (PA / PB are dead: every wave passed the last barrier after its
    // final LDS reads, and no staging is in flight) ----
    half_t* Qi = lds;
    half_t* Ki = lds + QA_BM * DH;
    half_t* Vi = lds + 2 * QA_BM * DH;
    // the key mask of the panel: loaded here, written to LDS after the image writes (its global
    // load latency then overlaps the constant loads instead of preceding them)
    // (every thread loads -- threads past QA_BM repeat a row -- so no branch merges the value
    // and the load stays in flight until its use)
    const int m_mk = m0 + (tid & (QA_BM - 1));
    const int mkv = reinterpret_cast<const int*>(qcst + 896)[tid & (QA_BM - 1)];
    // column-group outer: the bias / column sums of a group are loaded once (not once per row
    // group), and its LDS image address is one per lane -- the swizzles depend on the row only
    // through (row >> 1) & 7, which a row group's 16 j does not change -- with the row groups at
    // immediate offsets
    const int g = lane >> 4;
    float2 mrj[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ml = wm * 64 + 16 * j + (lane & 15);
      mrj[j] = LNF ? reinterpret_cast<const float2*>(qcst + 384)[ml] : make_float2(0.f, 1.f);
    }
    const int ml0 = wm * 64 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int n = wn * 96 + 16 * i + 4 * g;   // tile row: segment n >> 6, head dim n & 63
      const int seg = n >> 6, dim = n & 63;
      const float4v b = *reinterpret_cast<const float4v*>(qcst + seg * 64 + dim);
      float4v c = {0.f, 0.f, 0.f, 0.f};
      if constexpr (LNF)
        c = *reinterpret_cast<const float4v*>(qcst + 192 + seg * 64 + dim);
      half_t* img = seg == 0 ? Qi : seg == 1 ? Ki : Vi;
      const int chunk = seg == 2 ? a2_vswz(ml0, dim >> 3) : a2_kswz(ml0, dim >> 3);
      half_t* const wp = img + ml0 * DH + chunk * 8 + (dim & 7);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        half4 y;
        if constexpr (LNF) {
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = (half_t)fmaf(mrj[j].y, fmaf(-mrj[j].x, c[r], acc[i][j][r]), b[r]);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) y[r] = (half_t)(acc[i][j][r] + b[r]);
        }
        *reinterpret_cast<half4*>(wp + j * 16 * DH) = y;
      }
    }
    if (tid < QA_BM) kbias[tid] = (m_mk < M && mkv != 0) ? 0.f : -INFINITY;
    __syncthreads();
    stamp(2);  // the epilogue
    const int t_next = t + t_step;
    const bool more = t_next < t_end;
    const int h_n = tile_h(t_next), m0_n = tile_m(t_next);
    if (more && grp == 0) {  // the next tile's K-step 0 (and constants) land during attention
      stage(0, PB, m0_n, h_n);
      stage_cst(m0_n, h_n);
    }

    // ---- attention: waves 4s .. 4s+3 own sequence s of the panel, 32 queries each ----
    const int sq = wave >> 2, qw = (wave & 3) * 32;
    // (a panel may hold one sequence; DIAG 2 skips the attention)
    const bool attend = DIAG != 2 && m0 + QA_BM / 2 * (sq + 1) <= M;
    // the scores S^T = K Q^T of the wave's two 16-query tiles (Q, K fragments from the images)
    float4v sc[2][8];
    if (attend) {
      const half_t* Qs = Qi + sq * 128 * DH;
      const half_t* Ks = Ki + sq * 128 * DH;
      half8 qf[2][2], kf[8][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int r = qw + 16 * u + (lane & 15);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2)
          qf[u][s2] = *reinterpret_cast<const half8*>(Qs + r * DH + a2_kswz(r, g + 4 * s2) * 8);
      }
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) {
        const int kr = 16 * kt + (lane & 15);
        kf[kt][0] = *reinterpret_cast<const half8*>(Ks + kr * DH + a2_kswz(kr, g) * 8);
        kf[kt][1] = *reinterpret_cast<const half8*>(Ks + kr * DH + a2_kswz(kr, g + 4) * 8);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int kt = 0; kt < 8; ++kt) {
          float4v a = {0.f, 0.f, 0.f, 0.f};
          a = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kt][0], qf[u][0], a, 0, 0, 0);
          sc[u][kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(kf[kt][1], qf[u][1], a, 0, 0, 0);
        }
    }
    if (attend) {
      const half_t* Vs = Vi + sq * 128 * DH;
      const float* kb = kbias + sq * 128;
      float4v o[2][4], lsum[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        lsum[u] = float4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) o[u][tt] = float4v{0.f, 0.f, 0.f, 0.f};
      }
      {
        // software-pipelined per 16-query tile u: tile 0's P.V while tile 1's softmax issues (two
        // waves per SIMD in the same phase have no partner work to overlap otherwise).  Per-value
        // operation order is K5b's.
        // V^T fragments of the four 32-key chunks (key order 32c + 4g + j, then 32c + 16 + 4g + j)
        const int q4 = (lane >> 2) & 3, pp = lane & 3;
        half8 va[4][4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            const int r0 = 32 * c + 4 * g + q4, r1 = r0 + 16;
            const half4 lo = tr_read_b64(Vs + r0 * DH + a2_vswz(r0, 2 * tt + (pp >> 1)) * 8 + 4 * (pp & 1));
            const half4 hi = tr_read_b64(Vs + r1 * DH + a2_vswz(r1, 2 * tt + (pp >> 1)) * 8 + 4 * (pp & 1));
            va[c][tt] = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float tmax = -INFINITY;
#pragma unroll
          for (int kt = 0; kt < 8; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = sc[u][kt][r] * scale_log2 + kb[16 * kt + 4 * g + r];
              sc[u][kt][r] = v;
              tmax = fmaxf(tmax, v);
            }
          const float tm = rows4_max(tmax);
          const float m_use = (tm == -INFINITY) ? 0.f : tm;  // (one key block: no rescaling)
#pragma unroll
          for (int kt = 0; kt < 8; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) sc[u][kt][r] = exp2_fast(sc[u][kt][r] - m_use);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            half8 pb;
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              pb[jj] = (half_t)sc[u][2 * c][jj];
              pb[4 + jj] = (half_t)sc[u][2 * c + 1][jj];
            }
#pragma unroll
            for (int tt = 0; tt < 4; ++tt)
              o[u][tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va[c][tt], pb, o[u][tt], 0, 0, 0);
            lsum[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2_ones(), pb, lsum[u], 0, 0, 0);
          }
        }
      }
      // normalise and store (permlane16_swap: 8 consecutive dims per lane)
      const int odd = g & 1;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const float l = lsum[u][0];
        const float inv = l > 0.f ? 1.f / l : 0.f;
        const int q = m0 + sq * 128 + qw + 16 * u + (lane & 15);
#pragma unroll
        for (int p2 = 0; p2 < 2; ++p2) {
          float cv[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(o[u][2 * p2][r]),
                                                             __float_as_uint(o[u][2 * p2 + 1][r]), false, false);
            cv[r] = __uint_as_float(sw[0]) * inv;
            cv[4 + r] = __uint_as_float(sw[1]) * inv;
          }
          const int64_t co = (int64_t)q * d + h * DH + 32 * p2 + 16 * odd + 4 * (g & 2);
          if constexpr (CTX8) {
            const uint2 b8{e4m3x4(cv[0], cv[1], cv[2], cv[3]), e4m3x4(cv[4], cv[5], cv[6], cv[7])};
            *reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(ctx) + co) = b8;
          } else {
            half8 hv;
#pragma unroll
            for (int r = 0; r < 8; ++r) hv[r] = (half_t)cv[r];
            *reinterpret_cast<half8*>(ctx + co) = hv;
          }
        }
      }
    }  // attend
    stamp(3);  // the attention
    if constexpr (STAMP) st_sum[0] = __builtin_amdgcn_readfirstlane(st_sum[0] + 1);
    if (!more) break;
    // every wave is done with the images: the next tile's K-step 1 goes into PA; K-step 0 (group 0,
    // older than this wave's 4 ctx stores) must have landed before the barrier
    __syncthreads();
    if (grp == 1 && nk > 1) stage(1, PA, m0_n, h_n);
    if (grp == 0) {
      if (attend)
        SR_WAITCNT(4, 15);
      else
        SR_WAITCNT(0, 15);
    }
    __builtin_amdgcn_s_barrier();
    stamp(4);  // the transition
    t = t_next;
    h = h_n;
    m0 = m0_n;
  }
  if constexpr (STAMP) {
    if (lane == 0 && stamps) {
      uint64_t* o = stamps + ((int64_t)blockIdx.x * 8 + wave) * 8;
#pragma unroll
      for (int i = 0; i < 5; ++i) o[i] = st_sum[i];
    }
  }
}
}  // namespace

static int g_attn_variant = -1;  // test hook: -1 auto, 0 = K5 (64-key tiles), 1 = K5b (4 waves), 2 = K5b with 8 waves, 3 = auto with K5b STREAM instead of K5d
void attention_force_variant(int v) { g_attn_variant = v; }

void launch_attention(const half_t* qkv, const int32_t* mask, half_t* ctx, int B, int S, int Sq,
                      int d, int heads, hipStream_t stream) {
  const int dh = d / heads;
  SR_CHECK(dh * heads == d && (dh == 64 || dh == 32), "attention: head dim must be 32 or 64");
  if (B <= 0 || S <= 0) return;
  SR_CHECK(Sq >= 1 && Sq <= S, "attention: query rows must be in [1, S]");
  const double flops = 4.0 * B * heads * (double)Sq * S * dh;
  const double bytes = 2.0 * B * (double)S * 3.0 * d + 2.0 * B * (double)Sq * d;
  ProfScope prof("attention", stream, flops, bytes);
  const float scale_log2 = 1.4426950408889634f / sqrtf((float)dh);
  const bool use_b = dh == 64 && S <= 512 && g_attn_variant != 0;
  if (use_b) {
    const int S_pad = (S + 31) & ~31;
    const bool split = S_pad == 128 && Sq > 96;  // K5b SPLIT: one key block, all waves active
    // long sequences: 8 waves (256 queries) per workgroup share one K/V image (auto: S_pad > 256)
    const int nw = (g_attn_variant == 2 || ((g_attn_variant < 0 || g_attn_variant == 3) && S_pad > 256)) ? 8 : 4;
    // SPLIT also stages the workgroup's 128 Q rows (a third S_pad x 64 image)
    const size_t shmem = (size_t)(split && nw == 4 ? 3 : 2) * S_pad * 64 * sizeof(half_t) +
                         (size_t)S_pad * sizeof(float);
    dim3 grid((unsigned)ceil_div(Sq, 32 * nw), heads, B), block(64 * nw);
    if (split && nw == 4)
      hipLaunchKernelGGL((attention64_kernel<true, 4>), grid, block, shmem, stream, qkv, mask, ctx, S,
                         Sq, d, scale_log2);
    else if (nw == 8 && S_pad == 512 && Sq > 480 && g_attn_variant == 3)  // K5b STREAM (A/B)
      hipLaunchKernelGGL((attention64_kernel<false, 8, true>), grid, block, shmem, stream, qkv, mask, ctx,
                         S, Sq, d, scale_log2);
    else if (nw == 8 && S_pad == 512 && Sq > 480 && g_attn_variant != 2) {  // every query: K5d
      const int64_t tiles = (int64_t)B * heads;
      const int walkers = 8 * (int)std::min<int64_t>(32, (tiles + 7) / 8);
      hipLaunchKernelGGL(attention512_kernel, dim3(walkers), dim3(512), 0, stream, qkv, mask, ctx, B, S,
                         Sq, d, heads, scale_log2);
    }
    else if (nw == 8)
      hipLaunchKernelGGL((attention64_kernel<false, 8>), grid, block, shmem, stream, qkv, mask, ctx, S,
                         Sq, d, scale_log2);
    else
      hipLaunchKernelGGL((attention64_kernel<false, 4>), grid, block, shmem, stream, qkv, mask, ctx, S,
                         Sq, d, scale_log2);
  } else {
    const int nw = (int)std::min<int64_t>(4, ceil_div(Sq, 16));
    dim3 grid((unsigned)ceil_div(Sq, 16 * nw), heads, B), block(64 * nw);
    if (dh == 64)
      hipLaunchKernelGGL(attention_kernel<64>, grid, block, 0, stream, qkv, mask, ctx, S, Sq, d,
                         scale_log2);
    else
      hipLaunchKernelGGL(attention_kernel<32>, grid, block, 0, stream, qkv, mask, ctx, S, Sq, d,
                         scale_log2);
  }
  SR_LAUNCH_CHECK();
}


bool qkv_attention_supported(int S, int d, int heads) {
  return S == 128 && heads > 0 && d == heads * 64 && d % 64 == 0;
}

void launch_qkv_attention(int epi, const half_t* X, int64_t lda, const half_t* W, const float* bias,
                          const LnFold* lf, const int32_t* mask, half_t* ctx, int B, int S, int d,
                          int heads, hipStream_t stream, uint8_t* ctx8, uint64_t* stamps) {
  SR_CHECK(qkv_attention_supported(S, d, heads), "qkv_attention: needs S == 128 and d_h == 64");
  SR_CHECK(epi == EPI_BIAS_F16 || (epi == EPI_LNF_F16 && lf && lf->mr && lf->colsum && lf->stat_ld == 1),
           "qkv_attention: epilogue EPI_BIAS_F16 or EPI_LNF_F16 (row statistics + column sums)");
  SR_CHECK(lda >= d && lda % 8 == 0, "qkv_attention: lda must be >= d and a multiple of 8");
  if (B <= 0) return;
  const int64_t M = (int64_t)B * S;
  SR_CHECK(M < (1ll << 31) / 3, "qkv_attention: too many tokens");
  const double flops = 2.0 * M * 3.0 * d * d + 4.0 * B * heads * (double)S * S * 64;
  const double bytes = 2.0 * M * d + (ctx8 ? 1.0 : 2.0) * M * d + 2.0 * 3 * d * (double)d + 4.0 * M;
  ProfScope prof("qkv_attention", stream, flops, bytes);
  const float scale_log2 = 1.4426950408889634f / 8.0f;
  const int64_t tiles = ceil_div(M, 256) * heads;
  SR_CHECK(tiles < (1ll << 31), "qkv_attention: too many tiles");
  // persistent: 8 XCD groups x G walkers, one 8-wave workgroup per CU (153 KiB of LDS)
  const dim3 grid((unsigned)(8 * std::min<int64_t>(32, ceil_div(tiles, 8)))), block(512);
  // head groups of the tile walk (hg | heads): the walk takes every panel with heads [0, hg), then
  // every panel with [hg, 2 hg), ...  An XCD's ~32 concurrent tiles then need ~32 / hg X panels
  // (256 x d fp16) and hg W slices (192 x d fp16) in its 4 MiB L2: the divisor of heads that
  // minimises 32 * 256 / hg + 192 hg (hg = 6 of 12 heads: 1,011 -> 1,033 TF/s and +0.9 % end to
  // end against hg = heads; hg = 4 -5 %, profiles/r05_k5c_hgroup/)
  int hg = heads;
  for (int v = 1; v <= heads; ++v)
    if (heads % v == 0 && 8192.0 / v + 192.0 * v <= 8192.0 / hg + 192.0 * hg) hg = v;
#if SR_WITH_DIAG
  if (const char* e = diag_getenv("SR_QA_HGROUP")) {
    const int v = std::atoi(e);
    if (v > 0 && heads % v == 0) hg = v;
  }
#endif
#if SR_WITH_DIAG
  static const int diag = [] {
    const char* e = diag_getenv("SR_QA_DIAG");
    return e ? std::atoi(e) : 0;
  }();
  SR_CHECK(!stamps || epi == EPI_LNF_F16, "qkv_attention: stamps with the LN-folded epilogue");
  if (stamps)
    hipLaunchKernelGGL((qkv_attn_kernel<true, 3>), grid, block, 0, stream, X, lda, W, bias, lf->colsum,
                       lf->mr, mask, ctx, (int)M, d, heads, scale_log2, hg, stamps);
  else if (epi == EPI_LNF_F16 && diag == 1)
    hipLaunchKernelGGL((qkv_attn_kernel<true, 1>), grid, block, 0, stream, X, lda, W, bias, lf->colsum,
                       lf->mr, mask, ctx, (int)M, d, heads, scale_log2, hg, stamps);
  else if (epi == EPI_LNF_F16 && diag == 2)
    hipLaunchKernelGGL((qkv_attn_kernel<true, 2>), grid, block, 0, stream, X, lda, W, bias, lf->colsum,
                       lf->mr, mask, ctx, (int)M, d, heads, scale_log2, hg, stamps);
  else
#endif
#if SR_WITH_DIAG
  if (ctx8) {  // fp8 mode 5 (diagnostic library): e4m3 ctx for the O-projection on the fp8 MFMA
    half_t* c8 = reinterpret_cast<half_t*>(ctx8);
    if (epi == EPI_LNF_F16)
      hipLaunchKernelGGL((qkv_attn_kernel<true, 0, true>), grid, block, 0, stream, X, lda, W, bias,
                         lf->colsum, lf->mr, mask, c8, (int)M, d, heads, scale_log2, hg, stamps);
    else
      hipLaunchKernelGGL((qkv_attn_kernel<false, 0, true>), grid, block, 0, stream, X, lda, W, bias,
                         nullptr, nullptr, mask, c8, (int)M, d, heads, scale_log2, hg, stamps);
  } else
#else
  SR_CHECK(!ctx8 && !stamps, "qkv_attention: the e4m3 ctx output (fp8 mode 5) and the stamps are in the "
                             "diagnostic library only");
#endif
  if (epi == EPI_LNF_F16)
    hipLaunchKernelGGL(qkv_attn_kernel<true>, grid, block, 0, stream, X, lda, W, bias, lf->colsum,
                       lf->mr, mask, ctx, (int)M, d, heads, scale_log2, hg, stamps);
  else
    hipLaunchKernelGGL(qkv_attn_kernel<false>, grid, block, 0, stream, X, lda, W, bias, nullptr,
                       nullptr, mask, ctx, (int)M, d, heads, scale_log2, hg, stamps);
  SR_LAUNCH_CHECK();
}

}  // namespace sr
