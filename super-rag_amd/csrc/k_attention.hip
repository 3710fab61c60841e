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
#include "sr_common.h"
#include "sr_kernels.h"

namespace sr {

namespace {

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
    const float alpha = exp2f(m_run - m_use);
    m_run = m_new;
    l_run *= alpha;
#pragma unroll
    for (int t = 0; t < NDT; ++t) o[t] *= alpha;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float e = exp2f(p[kt][r] - m_use);
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

}  // namespace

void launch_attention(const half_t* qkv, const int32_t* mask, half_t* ctx, int B, int S, int Sq,
                      int d, int heads, hipStream_t stream) {
  const int dh = d / heads;
  SR_CHECK(dh * heads == d && (dh == 64 || dh == 32), "attention: head dim must be 32 or 64");
  if (B <= 0 || S <= 0) return;
  SR_CHECK(Sq >= 1 && Sq <= S, "attention: query rows must be in [1, S]");
  const int nw = (int)std::min<int64_t>(4, ceil_div(Sq, 16));
  dim3 grid((unsigned)ceil_div(Sq, 16 * nw), heads, B), block(64 * nw);
  const double flops = 4.0 * B * heads * (double)Sq * S * dh;
  const double bytes = 2.0 * B * (double)S * 3.0 * d + 2.0 * B * (double)Sq * d;
  ProfScope prof("attention", stream, flops, bytes);
  const float scale_log2 = 1.4426950408889634f / sqrtf((float)dh);
  if (dh == 64)
    hipLaunchKernelGGL(attention_kernel<64>, grid, block, 0, stream, qkv, mask, ctx, S, Sq, d,
                       scale_log2);
  else
    hipLaunchKernelGGL(attention_kernel<32>, grid, block, 0, stream, qkv, mask, ctx, S, Sq, d,
                       scale_log2);
  SR_LAUNCH_CHECK();
}

}  // namespace sr
