// K3 / K6 / K7 / K8 and small helpers of the encoder: position ids, embedding gather + LayerNorm,
// LayerNorm, pooling + L2 normalisation, classification logits, row normalisation.
// All are HBM-bound row kernels: one wave per row, 16-byte vector accesses, fp32 statistics with
// wave shuffles (two-pass mean / variance held in registers).
#include <algorithm>
#include <cstdlib>

#include "sr_common.h"
#include "sr_kernels.h"

namespace sr {

namespace {

constexpr int MAXV = 8;  // float4 per lane per row: d <= 2048

// Position ids.  BERT (offset 0): pos = s.  XLM-R (offset = padding_idx): HF
// create_position_ids_from_input_ids: pos = (ids != pad) ? padding_idx + cumsum(ids != pad) : pad.
__global__ void positions_kernel(const int32_t* __restrict__ ids, int32_t* __restrict__ pos, int S,
                                 int offset) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int32_t* row = ids + (int64_t)b * S;
  int32_t* out = pos + (int64_t)b * S;
  if (offset == 0) {
    for (int s = lane; s < S; s += 64) out[s] = s;
    return;
  }
  int running = 0;
  for (int s0 = 0; s0 < S; s0 += 64) {
    const int s = s0 + lane;
    const bool keep = s < S && row[s] != offset;
    const uint64_t bal = __ballot(keep);
    const int before = __popcll(bal & ((1ull << lane) - 1));
    if (s < S) out[s] = keep ? offset + running + before + 1 : offset;
    running += __popcll(bal);
  }
}

template <int NV>
__device__ __forceinline__ void ln_store(float4v (&x)[NV], int n4, const float* __restrict__ gamma,
                                         const float* __restrict__ beta, float eps, int d,
                                         half_t* __restrict__ h16, float* __restrict__ h32,
                                         int lane) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (lane + 64 * i < n4) s += x[i][0] + x[i][1] + x[i][2] + x[i][3];
  const float mean = wave_sum(s) / d;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (lane + 64 * i < n4) {
      const float4v t = x[i] - mean;
      v += t[0] * t[0] + t[1] * t[1] + t[2] * t[2] + t[3] * t[3];
    }
  const float rstd = rsqrtf(wave_sum(v) / d + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < n4) {
      const float4v g = reinterpret_cast<const float4v*>(gamma)[c];
      const float4v bb = reinterpret_cast<const float4v*>(beta)[c];
      const float4v y = (x[i] - mean) * rstd * g + bb;
      if (h32) reinterpret_cast<float4v*>(h32)[c] = y;
      half4 hy = {(half_t)y[0], (half_t)y[1], (half_t)y[2], (half_t)y[3]};
      reinterpret_cast<half4*>(h16)[c] = hy;
    }
  }
}

// NV float4 per lane per row (d <= 256 NV): sized to the model so the unrolled gathers do not hold
// MAXV x 3 vectors in registers (186 VGPRs = 2 waves per SIMD at MAXV for d = 768; the gather is
// latency-bound and wants occupancy)
template <int NV>
__global__ __launch_bounds__(256) void embed_ln_kernel(
    const int32_t* __restrict__ ids, const int32_t* __restrict__ pos,
    const int32_t* __restrict__ types, const half_t* __restrict__ wemb,
    const half_t* __restrict__ pemb, const half_t* __restrict__ temb,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, int M, int d,
    int vocab, int max_pos, int type_vocab, half_t* __restrict__ h16, float* __restrict__ h32) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  int id = ids[m];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  int p = pos[m];
  p = p < 0 ? 0 : (p >= max_pos ? max_pos - 1 : p);
  int t = types ? types[m] : 0;
  t = t < 0 ? 0 : (t >= type_vocab ? type_vocab - 1 : t);
  const int n4 = d >> 2;
  float4v x[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < n4) {
      const half4 a = reinterpret_cast<const half4*>(wemb + (int64_t)id * d)[c];
      const half4 bp = reinterpret_cast<const half4*>(pemb + (int64_t)p * d)[c];
      const half4 ct = reinterpret_cast<const half4*>(temb + (int64_t)t * d)[c];
#pragma unroll
      for (int j = 0; j < 4; ++j) x[i][j] = (float)a[j] + (float)bp[j] + (float)ct[j];
    }
  }
  ln_store<NV>(x, n4, gamma, beta, eps, d, h16 + m * d, h32 ? h32 + m * d : nullptr, lane);
}

// y (fp32 or fp16, the GEMM epilogue's bias + residual sum) -> LayerNorm -> h16 (+ h32).
// Each lane loads its whole share of the row before the reductions, so the kernel may run in
// place (y aliasing h16).
template <bool YF16, int NV>
__global__ __launch_bounds__(256) void layernorm_kernel(const void* y, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps,
                                                        int M, int d, half_t* h16,
                                                        float* __restrict__ h32) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const int n4 = d >> 2;
  float4v x[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < n4) {
      if constexpr (YF16) {
        const half4 hv = reinterpret_cast<const half4*>(reinterpret_cast<const half_t*>(y) + m * d)[c];
        x[i] = float4v{(float)hv[0], (float)hv[1], (float)hv[2], (float)hv[3]};
      } else {
        x[i] = reinterpret_cast<const float4v*>(reinterpret_cast<const float*>(y) + m * d)[c];
      }
    }
  }
  ln_store<NV>(x, n4, gamma, beta, eps, d, h16 + m * d, h32 ? h32 + m * d : nullptr, lane);
}

__device__ __forceinline__ float4v load4(const void* base, int64_t idx4, bool f16) {
  if (f16) {
    const half4 h = reinterpret_cast<const half4*>(base)[idx4];
    return float4v{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
  }
  return reinterpret_cast<const float4v*>(base)[idx4];
}

// Pool (CLS row or attention-mask mean) of the final hidden states (fp32, or fp16 for an fp16
// residual stream), then L2-normalise.
__global__ __launch_bounds__(64) void pool_l2_kernel(const void* __restrict__ h, int h_f16,
                                                     const int32_t* __restrict__ mask, int S,
                                                     int d, int pool, void* __restrict__ out,
                                                     int out_dtype, int ld_out) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int n4 = d >> 2;
  float4v x[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) x[i] = float4v{0.f, 0.f, 0.f, 0.f};
  const int64_t seq4 = (int64_t)b * S * n4;  // float4 index of the sequence's first row
  if (pool == SR_POOL_CLS) {
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (lane + 64 * i < n4) x[i] = load4(h, seq4 + lane + 64 * i, h_f16);
  } else {
    float cnt = 0.f;
    for (int s = 0; s < S; ++s) {
      if (mask[(int64_t)b * S + s] == 0) continue;
      cnt += 1.f;
#pragma unroll
      for (int i = 0; i < MAXV; ++i)
        if (lane + 64 * i < n4) x[i] += load4(h, seq4 + (int64_t)s * n4 + lane + 64 * i, h_f16);
    }
    const float inv = cnt > 0.f ? 1.f / cnt : 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) x[i] *= inv;
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i)
    if (lane + 64 * i < n4) ss += x[i][0] * x[i][0] + x[i][1] * x[i][1] + x[i][2] * x[i][2] + x[i][3] * x[i][3];
  const float nrm = sqrtf(wave_sum(ss));
  const float inv = nrm > 0.f ? 1.f / nrm : 0.f;  // zero-norm guard (graphiti helpers.py:100-103)
  if (out_dtype == SR_DTYPE_F32) {
    float* o = reinterpret_cast<float*>(out) + (int64_t)b * ld_out;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (lane + 64 * i < n4) reinterpret_cast<float4v*>(o)[lane + 64 * i] = x[i] * inv;
  } else {
    half_t* o = reinterpret_cast<half_t*>(out) + (int64_t)b * ld_out;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
      if (lane + 64 * i < n4) {
        const float4v v = x[i] * inv;
        half4 hv = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
        reinterpret_cast<half4*>(o)[lane + 64 * i] = hv;
      }
    for (int c = d + lane; c < ld_out; c += 64) o[c] = (half_t)0.f;
  }
}

// logits[p][j] = dot(t[p], w[j]) + bias[j]   (RoBERTa classification head out_proj).
__global__ __launch_bounds__(256) void cls_logits_kernel(const float* __restrict__ t,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ bias, int P,
                                                         int d, int labels,
                                                         float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const int n4 = d >> 2;
  for (int j = 0; j < labels; ++j) {
    float s = 0.f;
    for (int c = lane; c < n4; c += 64) {
      const float4v a = reinterpret_cast<const float4v*>(t + p * d)[c];
      const float4v bw = reinterpret_cast<const float4v*>(w + (int64_t)j * d)[c];
      s += a[0] * bw[0] + a[1] * bw[1] + a[2] * bw[2] + a[3] * bw[3];
    }
    s = wave_sum(s);
    if (lane == 0) out[p * labels + j] = s + bias[j];
  }
}

// out[r][:dim] = fp16(x[r] / ||x[r]||), out[r][dim:ld] = 0.  Zero rows stay zero.
__global__ __launch_bounds__(256) void normalize_rows_kernel(const void* __restrict__ x, int dtype,
                                                             int64_t n, int dim,
                                                             half_t* __restrict__ out, int ld) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  float ss = 0.f;
  if (dtype == SR_DTYPE_F32) {
    const float* row = reinterpret_cast<const float*>(x) + r * dim;
    for (int c = lane; c < dim; c += 64) ss += row[c] * row[c];
    const float nrm = sqrtf(wave_sum(ss));
    const float inv = nrm > 0.f ? 1.f / nrm : 0.f;
    for (int c = lane; c < ld; c += 64) out[r * ld + c] = (half_t)(c < dim ? row[c] * inv : 0.f);
  } else {
    const half_t* row = reinterpret_cast<const half_t*>(x) + r * dim;
    for (int c = lane; c < dim; c += 64) ss += (float)row[c] * (float)row[c];
    const float nrm = sqrtf(wave_sum(ss));
    const float inv = nrm > 0.f ? 1.f / nrm : 0.f;
    for (int c = lane; c < ld; c += 64) out[r * ld + c] = (half_t)(c < dim ? (float)row[c] * inv : 0.f);
  }
}

__global__ void convert_f32_f16_kernel(const float* __restrict__ in, half_t* __restrict__ out,
                                       int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (half_t)in[i];
}

// LayerNorm folding of a projection weight (one workgroup per output row n):
//   w16[n][k] = fp16(W[n][k] * gamma[k]);  colsum[n] = sum_k float(w16[n][k]);
//   bias_out[n] = sum_k W[n][k] * beta[k] + bias[n]      (fp32 master weights)
__global__ __launch_bounds__(256) void fold_ln_weight_kernel(const float* __restrict__ w32,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta,
                                                             const float* __restrict__ bias, int K,
                                                             half_t* __restrict__ w16,
                                                             float* __restrict__ colsum,
                                                             float* __restrict__ bias_out) {
  __shared__ float red[2][4];
  const int n = blockIdx.x, tid = threadIdx.x;
  float cs = 0.f, bs = 0.f;
  for (int k = tid; k < K; k += 256) {
    const float w = w32[(int64_t)n * K + k];
    const half_t h = (half_t)(w * gamma[k]);
    w16[(int64_t)n * K + k] = h;
    cs += (float)h;
    bs = fmaf(w, beta[k], bs);
  }
  cs = wave_sum(cs);
  bs = wave_sum(bs);
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = cs;
    red[1][tid >> 6] = bs;
  }
  __syncthreads();
  if (tid == 0) {
    colsum[n] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    bias_out[n] = red[1][0] + red[1][1] + red[1][2] + red[1][3] + bias[n];
  }
}

// (mu, rstd) per row from Chan partials (n = 128 each): mu = sum S_i / n,
// M2 = sum M2_i + 128 sum (S_i / 128 - mu)^2, rstd = 1 / sqrt(M2 / n + eps).  One thread per row.
__global__ __launch_bounds__(256) void ln_stats_finalize_kernel(const float* __restrict__ stat,
                                                                int nparts, float eps, int M,
                                                                float* __restrict__ mr) {
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  const float* p = stat + m * nparts * 2;
  float sum[16], m2s = 0.f, s = 0.f;
  for (int i = 0; i < nparts; ++i) {
    const float2 v = reinterpret_cast<const float2*>(p)[i];
    sum[i & 15] = v.x;
    s += v.x;
    m2s += v.y;
  }
  const float ntot = 128.f * (float)nparts;
  const float mu = s / ntot;
  for (int i = 0; i < nparts; ++i) {
    const float dm = sum[i & 15] * (1.f / 128.f) - mu;
    m2s += 128.f * dm * dm;
  }
  float2 o;
  o.x = mu;
  o.y = 1.f / sqrtf(m2s / ntot + eps);
  reinterpret_cast<float2*>(mr)[m] = o;
}

// h16 = LayerNorm(u) with (mu, rstd) from mr (one wave per row).
template <int NV>
__global__ __launch_bounds__(256) void ln_apply_kernel(const half_t* __restrict__ u, int64_t ldu,
                                                       const float* __restrict__ mr,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, int M, int d,
                                                       half_t* __restrict__ h16) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const float mu = mr[2 * m], rstd = mr[2 * m + 1];
  const int n4 = d >> 2;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = lane + 64 * i;
    if (c < n4) {
      const half4 hv = reinterpret_cast<const half4*>(u + m * ldu)[c];
      const float4v g = reinterpret_cast<const float4v*>(gamma)[c];
      const float4v bb = reinterpret_cast<const float4v*>(beta)[c];
      half4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (half_t)fmaf(((float)hv[j] - mu) * rstd, g[j], bb[j]);
      reinterpret_cast<half4*>(h16 + m * d)[c] = o;
    }
  }
}

// e4m3 copy of the LayerNorm-NORMALISED residual rows x = (u - mu) rstd (fp8 mode 4's QKV operand:
// the un-normalised u quantised directly loses its centred part to the common offset).  One wave
// per row, 4 columns per lane and step; saturates at +-448 like e4m3x4.
__global__ __launch_bounds__(256) void quantize_norm_fp8_kernel(const half_t* __restrict__ u, int64_t ldu,
                                                                const float* __restrict__ mr, int M, int d,
                                                                uint8_t* __restrict__ x8) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const float mu = mr[2 * m], rstd = mr[2 * m + 1];
  for (int c = lane; c < (d >> 2); c += 64) {
    const half4 hv = reinterpret_cast<const half4*>(u + m * ldu)[c];
    reinterpret_cast<uint32_t*>(x8 + m * d)[c] =
        e4m3x4(((float)hv[0] - mu) * rstd, ((float)hv[1] - mu) * rstd, ((float)hv[2] - mu) * rstd,
               ((float)hv[3] - mu) * rstd);
  }
}

__global__ void scale_f16_kernel(const half_t* in, float scale, half_t* out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = (half_t)((float)in[i] * scale);
}

__global__ void vec_add_kernel(const float* a, const float* b, float* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

}  // namespace

void launch_positions(const int32_t* ids, int32_t* pos, int B, int S, int offset, hipStream_t s) {
  if (B <= 0) return;
  hipLaunchKernelGGL(positions_kernel, dim3(B), dim3(64), 0, s, ids, pos, S, offset);
  SR_LAUNCH_CHECK();
}

void launch_embed_ln(const int32_t* ids, const int32_t* pos, const int32_t* types,
                     const half_t* wemb, const half_t* pemb, const half_t* temb,
                     const float* gamma, const float* beta, float eps, int M, int d, int vocab,
                     int max_pos, int type_vocab, half_t* h16, float* h32, hipStream_t s) {
  SR_CHECK(d % 4 == 0 && d <= 64 * 4 * MAXV, "embed_ln: hidden must be a multiple of 4, <= 2048");
  if (M <= 0) return;
  // HBM bytes: the gathered word rows (fp16) and ids / positions / types in, h16 out (+ h32 for
  // fp32-residual models); the position / type tables are cache-resident
  ProfScope prof("embed_ln", s, 0.0, (double)M * d * (2 + 2 + (h32 ? 4 : 0)) + 12.0 * M);
  const int nv = (int)ceil_div(d / 4, 64);
#define SR_EMB(NV)                                                                                   \
  hipLaunchKernelGGL((embed_ln_kernel<NV>), dim3((unsigned)ceil_div(M, 4)), dim3(256), 0, s, ids, pos, \
                     types, wemb, pemb, temb, gamma, beta, eps, M, d, vocab, max_pos, type_vocab,     \
                     h16, h32)
  if (nv <= 2) SR_EMB(2); else if (nv <= 3) SR_EMB(3); else if (nv <= 4) SR_EMB(4); else SR_EMB(MAXV);
#undef SR_EMB
  SR_LAUNCH_CHECK();
}

void launch_layernorm(const void* y, bool y_f16, const float* gamma, const float* beta, float eps,
                      int M, int d, half_t* h16, float* h32, hipStream_t s) {
  SR_CHECK(d % 4 == 0 && d <= 64 * 4 * MAXV, "layernorm: hidden must be a multiple of 4, <= 2048");
  if (M <= 0) return;
  ProfScope prof("layernorm", s, 0.0, (double)M * d * ((y_f16 ? 2 : 4) + 2 + (h32 ? 4 : 0)));
  const dim3 grid((unsigned)ceil_div(M, 4)), block(256);
  const int nv = (int)ceil_div(d / 4, 64);
#define SR_LN(YF, NV)                                                                            \
  hipLaunchKernelGGL((layernorm_kernel<YF, NV>), grid, block, 0, s, y, gamma, beta, eps, M, d, \
                     h16, h32)
  if (y_f16) {
    if (nv <= 3) SR_LN(true, 3); else if (nv <= 4) SR_LN(true, 4); else SR_LN(true, MAXV);
  } else {
    if (nv <= 3) SR_LN(false, 3); else if (nv <= 4) SR_LN(false, 4); else SR_LN(false, MAXV);
  }
#undef SR_LN
  SR_LAUNCH_CHECK();
}

void launch_pool_l2(const void* h, bool h_f16, const int32_t* mask, int B, int S, int d, int pool,
                    void* out, int out_dtype, int ld_out, hipStream_t s) {
  SR_CHECK(d % 4 == 0 && d <= 64 * 4 * MAXV, "pool: hidden must be a multiple of 4, <= 2048");
  if (B <= 0) return;
  ProfScope prof("pool_l2", s, 0.0, (double)B * d * 4.0 * (pool == SR_POOL_CLS ? 1 : S));
  hipLaunchKernelGGL(pool_l2_kernel, dim3(B), dim3(64), 0, s, h, h_f16 ? 1 : 0, mask, S, d, pool, out,
                     out_dtype, ld_out);
  SR_LAUNCH_CHECK();
}

void launch_cls_logits(const float* t, const float* w, const float* bias, int P, int d,
                       int labels, float* out, hipStream_t s) {
  if (P <= 0) return;
  hipLaunchKernelGGL(cls_logits_kernel, dim3((unsigned)ceil_div(P, 4)), dim3(256), 0, s, t, w,
                     bias, P, d, labels, out);
  SR_LAUNCH_CHECK();
}

void launch_normalize_rows(const void* x, int dtype, int64_t n, int dim, half_t* out, int ld,
                           hipStream_t s) {
  if (n <= 0) return;
  ProfScope prof("normalize_rows", s, 0.0, (double)n * (dim * (dtype == SR_DTYPE_F32 ? 4 : 2) + ld * 2));
  hipLaunchKernelGGL(normalize_rows_kernel, dim3((unsigned)ceil_div(n, 4)), dim3(256), 0, s, x,
                     dtype, n, dim, out, ld);
  SR_LAUNCH_CHECK();
}

void launch_convert_f32_f16(const float* in, half_t* out, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(convert_f32_f16_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                     in, out, n);
  SR_LAUNCH_CHECK();
}

}  // namespace sr

namespace sr {

void launch_fold_ln_weight(const float* w32, const float* gamma, const float* beta,
                           const float* bias, int N, int K, half_t* w16, float* colsum,
                           float* bias_out, hipStream_t s) {
  if (N <= 0) return;
  hipLaunchKernelGGL(fold_ln_weight_kernel, dim3(N), dim3(256), 0, s, w32, gamma, beta, bias, K,
                     w16, colsum, bias_out);
  SR_LAUNCH_CHECK();
}

void launch_ln_stats_finalize(const float* stat, int nparts, float eps, int M, float* mr,
                              hipStream_t s) {
  SR_CHECK(nparts >= 1 && nparts <= 16, "ln_stats_finalize: 1..16 partials per row");
  if (M <= 0) return;
  ProfScope prof("ln_stats_finalize", s, 0.0, (double)M * (nparts * 8.0 + 8.0));
  hipLaunchKernelGGL(ln_stats_finalize_kernel, dim3((unsigned)ceil_div(M, 256)), dim3(256), 0, s,
                     stat, nparts, eps, M, mr);
  SR_LAUNCH_CHECK();
}

void launch_ln_apply(const half_t* u, int64_t ldu, const float* mr, const float* gamma,
                     const float* beta, int M, int d, half_t* h16, hipStream_t s) {
  SR_CHECK(d % 4 == 0 && d <= 64 * 4 * MAXV, "ln_apply: hidden must be a multiple of 4, <= 2048");
  if (M <= 0) return;
  ProfScope prof("ln_apply", s, 0.0, (double)M * d * 4.0);
  hipLaunchKernelGGL(ln_apply_kernel<MAXV>, dim3((unsigned)ceil_div(M, 4)), dim3(256), 0, s, u, ldu,
                     mr, gamma, beta, M, d, h16);
  SR_LAUNCH_CHECK();
}

void launch_quantize_norm_fp8(const half_t* u, int64_t ldu, const float* mr, int M, int d, uint8_t* x8,
                              hipStream_t s) {
  SR_CHECK(d % 4 == 0, "quantize_norm_fp8: hidden must be a multiple of 4");
  if (M <= 0) return;
  ProfScope prof("quantize_norm_fp8", s, 0.0, (double)M * d * 3.0);
  hipLaunchKernelGGL(quantize_norm_fp8_kernel, dim3((unsigned)ceil_div(M, 4)), dim3(256), 0, s, u, ldu,
                     mr, M, d, x8);
  SR_LAUNCH_CHECK();
}

void launch_scale_f16(const half_t* in, float scale, half_t* out, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scale_f16_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, in, scale,
                     out, n);
  SR_LAUNCH_CHECK();
}

// Diagnostic HBM copy (measured-peak yardstick for bench.py): one 16-byte element per lane, one
// pass (no grid-stride loop), the plain "float4 copy" form.
__global__ __launch_bounds__(256) void copy16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                     int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

void launch_copy16(const void* src, void* dst, int64_t bytes, hipStream_t s) {
  SR_CHECK(bytes % 16 == 0, "copy16: bytes must be a multiple of 16");
  if (bytes <= 0) return;
  const int64_t n = bytes / 16;
  SR_CHECK(ceil_div(n, 256) < (1ll << 31), "copy16: too large");
  hipLaunchKernelGGL(copy16_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                     reinterpret_cast<const uint4*>(src), reinterpret_cast<uint4*>(dst), n);
  SR_LAUNCH_CHECK();
}

// ---- K/V-free CLS-only last layer of an LN-folded cross-encoder (encoder.cpp) ---------------------
// With LN folded, K_j = rstd_j (W'_k u_j - mu_j c_k) + d_k and V_j likewise, so for the CLS query q
//   score_h(j) = q_h . K_{j,h} = rstd_j (w_h . u_j - mu_j sum(w_h)) + const_h,   w_h = W'_{k,h}^T q_h
//   ctx_h      = sum_j p_j V_{j,h} = W'_{v,h} z'_h + d_{v,h},   z'_h = sum_j p_j rstd_j (u_j - mu_j)
// (const_h cancels in the softmax; sum_j p_j = 1).  w for all heads is ONE GEMM against a
// block-diagonal [H*D x D] weight, ctx ONE GEMM against a block-diagonal [D x H*D] weight; this
// kernel does the rest per sequence: scores on MFMA (A = u rows straight from HBM, B = w_h from
// LDS), the masked softmax, and z' on VALU (a second, L2 / Infinity-Cache-served read of u).
// U is never projected to K and V: at the bge-reranker-base shape that is 2 x D x D x S FLOP and
// 4 x D x S bytes of K / V per sequence the last layer no longer spends.
template <int D, int HH>
__global__ __launch_bounds__(512) void cls_attn_fold_kernel(const half_t* __restrict__ w,
                                                            const half_t* __restrict__ U,
                                                            const float* __restrict__ mr,
                                                            const int32_t* __restrict__ mask, int S,
                                                            int H, float scale, half_t* __restrict__ z) {
  constexpr int NCH = D / 8;  // 16-byte chunks per row
  __shared__ __attribute__((aligned(16))) half_t wl[16 * D];
  __shared__ __attribute__((aligned(16))) float sc[16 * 512];
  __shared__ float2 mrl[512];
  __shared__ float alpha[16], sig[16];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  const half_t* wb = w + (int64_t)b * H * D;
  const half_t* Ub = U + (int64_t)b * S * D;
  // w_h rows (h >= H: zero), chunk ch of row r at ch ^ (r & 15) (conflict-free B-fragment reads)
  for (int i = tid; i < 16 * NCH; i += 512) {
    const int r = i / NCH, ch = i - r * NCH;
    half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (r < H) v = *reinterpret_cast<const half8*>(wb + (int64_t)r * D + ch * 8);
    *reinterpret_cast<half8*>(wl + r * D + ((ch & ~15) | ((ch ^ r) & 15)) * 8) = v;
  }
  for (int j = tid; j < S; j += 512) {
    const float2 m = *reinterpret_cast<const float2*>(mr + ((int64_t)b * S + j) * 2);
    mrl[j] = mask[(int64_t)b * S + j] ? m : make_float2(0.f, 0.f);
  }
  // alpha_h = sum_i w_h[i] (the fp16 w the scores use)
  for (int h = wave; h < H; h += 8) {
    float a = 0.f;
    for (int i = lane; i < D; i += 64) a += (float)wb[(int64_t)h * D + i];
    a = wave_sum(a);
    if (lane == 0) alpha[h] = a;
  }
  __syncthreads();
  // scores: token block tb (16 tokens) per wave; lane (c, g): A = token 16 tb + c, dims 32 k + 8 g
  for (int tb = wave; tb * 16 < S; tb += 8) {
    const half_t* ur = Ub + (int64_t)(16 * tb + c) * D + 8 * g;
    half8 a[D / 32];
#pragma unroll
    for (int k = 0; k < D / 32; ++k) a[k] = *reinterpret_cast<const half8*>(ur + 32 * k);
    float4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < D / 32; ++k) {
      const int ch = 4 * k + g;
      const half8 bf = *reinterpret_cast<const half8*>(wl + c * D + ((ch & ~15) | ((ch ^ c) & 15)) * 8);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[k], bf, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // acc[r] = w_c . u_j, j = 16 tb + 4 g + r
      const int j = 16 * tb + 4 * g + r;
      const float2 m = mrl[j];
      const bool live = mask[(int64_t)b * S + j] != 0;
      if (c < H) sc[c * S + j] = live ? m.y * (acc[r] - m.x * alpha[c]) * scale : -INFINITY;
    }
  }
  __syncthreads();
  // softmax per head; p'_j = p_j rstd_j (masked tokens: rstd 0), sig_h = sum_j p'_j mu_j
  for (int h = wave; h < H; h += 8) {
    float mx = -INFINITY;
    for (int j = lane; j < S; j += 64) mx = fmaxf(mx, sc[h * S + j]);
    mx = wave_max(mx);
    float l = 0.f;
    for (int j = lane; j < S; j += 64) l += __expf(sc[h * S + j] - mx);
    l = wave_sum(l);
    const float inv = 1.f / l;
    float sg = 0.f;
    for (int j = lane; j < S; j += 64) {
      const float2 m = mrl[j];
      const float pj = __expf(sc[h * S + j] - mx) * inv * m.y;
      sc[h * S + j] = pj;
      sg = fmaf(pj, m.x, sg);
    }
    sg = wave_sum(sg);
    if (lane == 0) sig[h] = sg;
  }
  __syncthreads();
  // z'_h[i] = sum_j p'_j u_j[i] - sig_h: thread t owns dims 2t, 2t + 1
  if (tid < D / 2) {
    float zx[HH], zy[HH];
#pragma unroll
    for (int h = 0; h < HH; ++h) zx[h] = zy[h] = 0.f;
    const half_t* up = Ub + 2 * tid;
    // 16 tokens per step, the next step's 16 loads in flight while this step's FMAs run (the loop
    // is latency-bound on the second read of u otherwise)
    half2_t un[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) un[e] = *reinterpret_cast<const half2_t*>(up + (int64_t)e * D);
    for (int j = 0; j < S; j += 16) {
      half2_t u[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) u[e] = un[e];
      if (j + 16 < S) {
#pragma unroll
        for (int e = 0; e < 16; ++e) un[e] = *reinterpret_cast<const half2_t*>(up + (int64_t)(j + 16 + e) * D);
      }
#pragma unroll
      for (int h = 0; h < HH; ++h) {
        if (h >= H) break;
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          const float4v p = *reinterpret_cast<const float4v*>(sc + h * S + j + 4 * e4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            zx[h] = fmaf(p[e], (float)u[4 * e4 + e][0], zx[h]);
            zy[h] = fmaf(p[e], (float)u[4 * e4 + e][1], zy[h]);
          }
        }
      }
    }
    // z' as an fp16 pair hi + lo (row [hi(H*D) | lo(H*D)]; the ctx GEMM's weight repeats): z' is
    // rounded once per head, not once per token as V was, so it keeps ~22 bits instead of 11
    half_t* zb = z + (int64_t)b * 2 * H * D + 2 * tid;
#pragma unroll
    for (int h = 0; h < HH; ++h) {
      if (h >= H) break;
      const float vx = zx[h] - sig[h], vy = zy[h] - sig[h];
      half2_t hi, lo;
      hi[0] = (half_t)vx;
      hi[1] = (half_t)vy;
      lo[0] = (half_t)(vx - (float)hi[0]);
      lo[1] = (half_t)(vy - (float)hi[1]);
      *reinterpret_cast<half2_t*>(zb + (int64_t)h * D) = hi;
      *reinterpret_cast<half2_t*>(zb + (int64_t)(H + h) * D) = lo;
    }
  }
}

// Single-read form (S <= 128): the score phase keeps each wave's 16 token rows of u in registers
// (its MFMA A fragments, 16 tokens x D); after the softmax the rows go through LDS 32 tokens at a
// time ([token][D + 16] halfs: the 8 rows of a half-wave's transposed read start 32 bytes apart,
// one bank slot each) and z'[16 heads x D] = p' . u runs on MFMA (A = p' as an fp16 hi + lo pair,
// so z' keeps fp32-like precision; B = 8 tokens of one dim per lane by two ds_read_b64_tr_b16, token
// order 4g + j then 16 + 4g + j, which p' follows).  u is read from HBM once (the two-pass form reads
// it twice and accumulates z' on VALU with 4-byte loads); z' leaves through LDS as 16-byte stores.
__device__ __forceinline__ half4 cf_tr_read_b64(const half_t* p) {
  typedef short short4_t __attribute__((ext_vector_type(4)));
  const short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) short4_t*)(p));
  return __builtin_bit_cast(half4, v);
}
constexpr int CF_T = 32;  // tokens per LDS round
// persistent: one workgroup per CU (175 / 239 VGPRs) walks sequences b, b + grid, ...; a wave
// loads its rows of the NEXT sequence as soon as its own round has put this sequence's rows into
// LDS, so the HBM reads overlap the remaining rounds, the z' store and the next sequence's prologue
template <int D, int HH>
__global__ __launch_bounds__(512) void cls_attn_fold1_kernel(const half_t* __restrict__ w,
                                                             const half_t* __restrict__ U,
                                                             const float* __restrict__ mr,
                                                             const int32_t* __restrict__ mask, int B,
                                                             int S, int H, float scale,
                                                             half_t* __restrict__ z) {
  constexpr int NCH = D / 8, KD = D / 32, LDU = D + 16;
  constexpr int NT = D / 16 / 8;  // z' column tiles (16 dims) per wave
  // D = 1024 (128 VGPRs of rows + 32 of z') loads its rows at the top of each sequence instead:
  // the early prefetch spills there
  constexpr bool PF = D <= 768;
  static_assert(CF_T * LDU >= 2 * 16 * D, "the stage area holds z' (hi, lo) on the way out");
  __shared__ __attribute__((aligned(16))) half_t wl[16 * D];
  __shared__ __attribute__((aligned(16))) half_t ust[CF_T * LDU];
  __shared__ __attribute__((aligned(16))) float sc[16 * 128];
  __shared__ float2 mrl[128];
  __shared__ float alpha[16], sig[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int c = lane & 15, g = lane >> 4;
  // this wave's token rows (tb = wave) of sequence bb, all loads in flight before any wait
  const bool has = 16 * wave < S;
  half8 a[KD];
  auto load_rows = [&](int bb) __attribute__((always_inline)) {
    if (has) {
      const half_t* ur = U + ((int64_t)bb * S + 16 * wave + c) * D + 8 * g;
#pragma unroll
      for (int k = 0; k < KD; ++k) a[k] = *reinterpret_cast<const half8*>(ur + 32 * k);
    } else {
#pragma unroll
      for (int k = 0; k < KD; ++k) a[k] = half8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  int b = blockIdx.x;
  if (b >= B) return;
  if (PF) load_rows(b);
  const int rounds = (S + CF_T - 1) / CF_T;
  for (; b < B; b += gridDim.x) {
    const int nb = b + (int)gridDim.x;
    if (!PF) load_rows(b);
    const half_t* wb = w + (int64_t)b * H * D;
    for (int i = tid; i < 16 * NCH; i += 512) {
      const int r = i / NCH, ch = i - r * NCH;
      half8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (r < H) v = *reinterpret_cast<const half8*>(wb + (int64_t)r * D + ch * 8);
      *reinterpret_cast<half8*>(wl + r * D + ((ch & ~15) | ((ch ^ r) & 15)) * 8) = v;
    }
    for (int j = tid; j < S; j += 512) {
      const float2 m = *reinterpret_cast<const float2*>(mr + ((int64_t)b * S + j) * 2);
      mrl[j] = mask[(int64_t)b * S + j] ? m : make_float2(0.f, 0.f);
    }
    for (int i = tid; i < 16 * 128; i += 512) sc[i] = 0.f;  // heads >= H, tokens >= S: p' = 0
    for (int h = wave; h < H; h += 8) {
      float s = 0.f;
      for (int i = lane; i < D; i += 64) s += (float)wb[(int64_t)h * D + i];
      s = wave_sum(s);
      if (lane == 0) alpha[h] = s;
    }
    __syncthreads();
    if (has) {
      float4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KD; ++k) {
        const int ch = 4 * k + g;
        const half8 bf = *reinterpret_cast<const half8*>(wl + c * D + ((ch & ~15) | ((ch ^ c) & 15)) * 8);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[k], bf, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // acc[r] = w_c . u_j, j = 16 wave + 4 g + r
        const int j = 16 * wave + 4 * g + r;
        const float2 m = mrl[j];
        const bool live = mask[(int64_t)b * S + j] != 0;
        if (c < H) sc[c * 128 + j] = live ? m.y * (acc[r] - m.x * alpha[c]) * scale : -INFINITY;
      }
    }
    __syncthreads();
    // softmax per head; p'_j = p_j rstd_j (masked tokens: rstd 0), sig_h = sum_j p'_j mu_j
    for (int h = wave; h < H; h += 8) {
      float mx = -INFINITY;
      for (int j = lane; j < S; j += 64) mx = fmaxf(mx, sc[h * 128 + j]);
      mx = wave_max(mx);
      float l = 0.f;
      for (int j = lane; j < S; j += 64) l += __expf(sc[h * 128 + j] - mx);
      l = wave_sum(l);
      const float inv = 1.f / l;
      float sg = 0.f;
      for (int j = lane; j < S; j += 64) {
        const float2 m = mrl[j];
        const float pj = __expf(sc[h * 128 + j] - mx) * inv * m.y;
        sc[h * 128 + j] = pj;
        sg = fmaf(pj, m.x, sg);
      }
      sg = wave_sum(sg);
      if (lane == 0) sig[h] = sg;
    }
    // z' on MFMA, 32 tokens per round: waves 2r, 2r + 1 put their rows into the stage area, then
    // start loading their rows of the next sequence
    float4v zacc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) zacc[t] = float4v{0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < rounds; ++r) {
      __syncthreads();  // the softmax is done (r = 0) / every wave is past round r - 1's reads
      const bool mine = (wave >> 1) == r;
      if (mine) {
        half_t* dst = ust + (16 * (wave & 1) + c) * LDU + 8 * g;
#pragma unroll
        for (int k = 0; k < KD; ++k) *reinterpret_cast<half8*>(dst + 32 * k) = a[k];
      }
      __syncthreads();
      if (PF && mine && nb < B) load_rows(nb);
      // A = p' (row: head c, k: tokens 32 r + 4 g + j, then 32 r + 16 + 4 g + j) as fp16 hi + lo
      half8 ph, pl;
      {
        const float4v p0 = *reinterpret_cast<const float4v*>(sc + c * 128 + CF_T * r + 4 * g);
        const float4v p1 = *reinterpret_cast<const float4v*>(sc + c * 128 + CF_T * r + 16 + 4 * g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ph[e] = (half_t)p0[e];
          pl[e] = (half_t)(p0[e] - (float)ph[e]);
          ph[4 + e] = (half_t)p1[e];
          pl[4 + e] = (half_t)(p1[e] - (float)ph[4 + e]);
        }
      }
      // B = u tokens (as ph) x dims 16 (wave NT + t) ..: lane 4q + pp of group g addresses token
      // 4 g + q (16 + 4 g + q), dims + 4 pp .. + 3; the transposed read hands lane c its dim's 4 tokens
      const int q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const half_t* col = ust + 16 * (wave * NT + t) + 4 * pp;
        const half4 lo = cf_tr_read_b64(col + (4 * g + q) * LDU);
        const half4 hi = cf_tr_read_b64(col + (16 + 4 * g + q) * LDU);
        const half8 bu = half8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        zacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, bu, zacc[t], 0, 0, 0);
        zacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pl, bu, zacc[t], 0, 0, 0);
      }
    }
    // waves without a round of their own (S <= 96: no rows, or rounds < 4) load the next rows here
    if (PF && (wave >> 1) >= rounds && nb < B) load_rows(nb);
    __syncthreads();  // the stage area becomes z' (hi rows 0 .. H-1, lo rows H .. 2H-1)
    half_t* zo = ust;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = 16 * (wave * NT + t) + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // zacc[t][q] = z'[head 4 g + q][dim n]
        const int h = 4 * g + q;
        if (h < H) {
          const float v = zacc[t][q] - sig[h];
          const half_t hi = (half_t)v;
          zo[h * D + n] = hi;
          zo[(H + h) * D + n] = (half_t)(v - (float)hi);
        }
      }
    }
    __syncthreads();
    half_t* zb = z + (int64_t)b * 2 * H * D;
    for (int i = tid; i < 2 * H * NCH; i += 512)
      *reinterpret_cast<half8*>(zb + 8 * i) = *reinterpret_cast<const half8*>(zo + 8 * i);
    __syncthreads();  // every wave is done with zo, wl, sc, mrl before the next sequence's prologue
  }
}

// Block-diagonal weights of the K/V-free last layer from the folded QKV weight W' [3D x D]:
//   wk_bd [H*D x D]: row h*D + i, column k = W'_k[k][i] for k in head h, else 0
//   wv_bd [D x 2*H*D]: row n, column c*H*D + h*D + i (c = 0, 1: the z' hi / lo halves)
//                      = W'_v[n][i] for h = head of n, else 0
__global__ void kv_blockdiag_kernel(const half_t* __restrict__ wqkv_f, int D, int H,
                                    half_t* __restrict__ wk_bd, half_t* __restrict__ wv_bd) {
  const int dh = D / H;
  const int64_t r = blockIdx.x;  // 0 .. H*D-1 (wk_bd rows), then D rows of wv_bd
  if (r < (int64_t)H * D) {
    const int h = (int)(r / D), i = (int)(r % D);
    for (int k = threadIdx.x; k < D; k += blockDim.x)
      wk_bd[r * D + k] = (k / dh == h) ? wqkv_f[(int64_t)(D + k) * D + i] : (half_t)0.f;
  } else {
    const int n = (int)(r - (int64_t)H * D), h = n / dh;
    const int64_t HD = (int64_t)H * D;
    for (int64_t col = threadIdx.x; col < 2 * HD; col += blockDim.x) {
      const int64_t cm = col % HD;
      wv_bd[(int64_t)n * 2 * HD + col] = (cm / D == h) ? wqkv_f[(int64_t)(2 * D + n) * D + cm % D]
                                                      : (half_t)0.f;
    }
  }
}

bool cls_attn_fold_supported(int S, int D, int H) {
  return (D == 768 || D == 1024) && H >= 1 && H <= 16 && D % H == 0 && D / H == 64 && S % 16 == 0 &&
         S >= 16 && S <= 512;
}

void launch_kv_blockdiag(const half_t* wqkv_f, int D, int H, half_t* wk_bd, half_t* wv_bd,
                         hipStream_t s) {
  hipLaunchKernelGGL(kv_blockdiag_kernel, dim3((unsigned)((int64_t)H * D + D)), dim3(256), 0, s,
                     wqkv_f, D, H, wk_bd, wv_bd);
  SR_LAUNCH_CHECK();
}

void launch_cls_attn_fold(const half_t* w, const half_t* U, const float* mr, const int32_t* mask,
                          int B, int S, int D, int H, half_t* z, hipStream_t s) {
  SR_CHECK(cls_attn_fold_supported(S, D, H), "cls_attn_fold: unsupported shape");
  if (B <= 0) return;
  ProfScope prof("cls_attn_fold", s, 4.0 * B * (double)S * D * H,
                 2.0 * 2.0 * B * (double)S * D + 2.0 * 2.0 * B * (double)H * D);
  const float scale = 0.125f;  // 1 / sqrt(64)
  // the single-read form for S <= 128 (SR_CLS_FOLD_1READ=0: the two-pass form; read per launch)
  const char* e1 = std::getenv("SR_CLS_FOLD_1READ");
  if (S <= 128 && !(e1 && e1[0] == '0')) {
    const unsigned grid = (unsigned)std::min(B, 256);  // one workgroup per CU (registers), persistent
    if (D == 768)
      hipLaunchKernelGGL((cls_attn_fold1_kernel<768, 12>), dim3(grid), dim3(512), 0, s, w, U, mr, mask, B,
                         S, H, scale, z);
    else
      hipLaunchKernelGGL((cls_attn_fold1_kernel<1024, 16>), dim3(grid), dim3(512), 0, s, w, U, mr, mask, B,
                         S, H, scale, z);
    SR_LAUNCH_CHECK();
    return;
  }
  if (D == 768)
    hipLaunchKernelGGL((cls_attn_fold_kernel<768, 12>), dim3((unsigned)B), dim3(512), 0, s, w, U, mr,
                       mask, S, H, scale, z);
  else
    hipLaunchKernelGGL((cls_attn_fold_kernel<1024, 16>), dim3((unsigned)B), dim3(512), 0, s, w, U, mr,
                       mask, S, H, scale, z);
  SR_LAUNCH_CHECK();
}

void launch_vec_add(const float* a, const float* b, float* out, int n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(vec_add_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, a, b, out, n);
  SR_LAUNCH_CHECK();
}

}  // namespace sr
