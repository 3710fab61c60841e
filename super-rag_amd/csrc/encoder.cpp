// Transformer encoder runtime (BERT / XLM-R): replaces the remote embedding server reached through
// litellm.embedding() (super_rag/llm/embed/embedding_service.py:168-175) and the remote
// cross-encoder reached through litellm.arerank() (super_rag/llm/rerank/rerank_service.py:95-104).
//
// Per layer (post-LN BERT block), all on one HIP stream:
//   qkv  = GEMM(h16, Wqkv) + bqkv                 fp16  [M, 3d]     (K4, bias epilogue)
//   ctx  = MHA(qkv, mask)                         fp16  [M, d]      (K5)
//   y32  = GEMM(ctx, Wo) + bo + h32               fp32  [M, d]      (K4, residual epilogue)
//   h    = LayerNorm(y32)                         fp16 + fp32       (K6)
//   f    = GELU(GEMM(h16, W1) + b1)               fp16  [M, F]      (K4, GELU epilogue)
//   y32  = GEMM(f, W2) + b2 + h32                 fp32              (K4, residual epilogue)
//   h    = LayerNorm(y32)                         fp16 + fp32       (K6)
// The residual stream is fp32 by default (fp16 residuals cost ~2x the embedding error,
// DESIGN.md); cross-encoders may run it in fp16 (config.residual_fp16).  With CLS pooling or a
// classification head the last layer is computed for the CLS rows only.
// Embedding mode pools (CLS / masked mean) and L2-normalises (K7); cross-encoder mode applies the
// RoBERTa classification head: tanh(GEMM(h16[CLS rows], Wc) + bc) (fp32) . Wout + bout (K4 + K8).
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "sr_kernels.h"
#include "sr_runtime.h"

namespace sr {

Encoder::Encoder(const sr_encoder_config& cfg, int device) : cfg_(cfg), device_(device) {
  const int d = cfg.hidden;
  SR_CHECK(cfg.vocab_size > 0 && d > 0 && cfg.layers > 0 && cfg.heads > 0 &&
               cfg.intermediate > 0 && cfg.max_position > 0 && cfg.type_vocab > 0,
           "encoder: config fields must be positive");
  SR_CHECK(d % cfg.heads == 0 && (d / cfg.heads == 64 || d / cfg.heads == 32),
           "encoder: head dim must be 32 or 64");
  SR_CHECK(d % 128 == 0 && cfg.intermediate % 128 == 0,
           "encoder: hidden and intermediate must be multiples of 128");
  SR_CHECK(d <= 2048, "encoder: hidden must be <= 2048");
  SR_CHECK(cfg.classifier == 0 || (cfg.classifier == 1 && cfg.num_labels >= 1),
           "encoder: classifier must be 0 or 1 (with num_labels >= 1)");
  max_tokens_ = cfg.max_tokens > 0 ? cfg.max_tokens : 262144;
  DeviceGuard g(device_);
  SR_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  SR_HIP(hipEventCreateWithFlags(&done_, hipEventDisableTiming));

  const int64_t D = d, F = cfg.intermediate;
  {
    // split weights for the DEEP fp32-residual embedders only: measured against the fp32 oracle
    // (tools/embed_split_error.py), the 24-layer bge-m3 needs them (1.07e-3 max relative error
    // without, 5.3e-4 with; bar 1e-3), the 12-layer bge-base does not (6.1e-4 without, 4.1e-4
    // with) and embeds 1.5x faster without (B = 256: 4.28 -> 2.86 ms).  SR_WEIGHT_SPLIT = 0 / 1
    // forces the choice.
    const char* e = std::getenv("SR_WEIGHT_SPLIT");
    const bool deep = cfg.layers > 12;
    split_ = !cfg.residual_fp16 && (e && e[0] ? e[0] != '0' : deep);
  }
  const int64_t sk = split_ ? D : 0, skf = split_ ? F : 0;
  register_target("embeddings.word_embeddings.weight", wemb_, (int64_t)cfg.vocab_size * D, true);
  register_target("embeddings.position_embeddings.weight", pemb_, (int64_t)cfg.max_position * D, true);
  register_target("embeddings.token_type_embeddings.weight", temb_, (int64_t)cfg.type_vocab * D, true);
  register_target("embeddings.LayerNorm.weight", embg_, D, false);
  register_target("embeddings.LayerNorm.bias", embb_, D, false);
  layers_.resize(cfg.layers);
  for (int l = 0; l < cfg.layers; ++l) {
    Layer& L = layers_[l];
    const std::string p = "encoder.layer." + std::to_string(l) + ".";
    register_target(p + "attention.self.query.weight", L.wqkv, D * D, true, 0, 3 * D * D, sk);
    register_target(p + "attention.self.key.weight", L.wqkv, D * D, true, D * D, 3 * D * D, sk);
    register_target(p + "attention.self.value.weight", L.wqkv, D * D, true, 2 * D * D, 3 * D * D, sk);
    register_target(p + "attention.self.query.bias", L.bqkv, D, false, 0, 3 * D);
    register_target(p + "attention.self.key.bias", L.bqkv, D, false, D, 3 * D);
    register_target(p + "attention.self.value.bias", L.bqkv, D, false, 2 * D, 3 * D);
    register_target(p + "attention.output.dense.weight", L.wo, D * D, true, 0, -1, sk);
    register_target(p + "attention.output.dense.bias", L.bo, D, false);
    register_target(p + "attention.output.LayerNorm.weight", L.ln1g, D, false);
    register_target(p + "attention.output.LayerNorm.bias", L.ln1b, D, false);
    register_target(p + "intermediate.dense.weight", L.w1, F * D, true, 0, -1, sk);
    register_target(p + "intermediate.dense.bias", L.b1, F, false);
    register_target(p + "output.dense.weight", L.w2, D * F, true, 0, -1, skf);
    register_target(p + "output.dense.bias", L.b2, D, false);
    register_target(p + "output.LayerNorm.weight", L.ln2g, D, false);
    register_target(p + "output.LayerNorm.bias", L.ln2b, D, false);
  }
  // fp32 masters of the weights that LayerNorm folding rescales (fp16 residual stream only)
  if (cfg.residual_fp16) {
    for (int l = 0; l < cfg.layers; ++l) {
      Layer& L = layers_[l];
      const std::string p = "encoder.layer." + std::to_string(l) + ".";
      L.wqkv32.reserve((size_t)3 * D * D * sizeof(float));
      L.w132.reserve((size_t)F * D * sizeof(float));
      targets_[p + "attention.self.query.weight"].master = L.wqkv32.as<float>();
      targets_[p + "attention.self.key.weight"].master = L.wqkv32.as<float>() + D * D;
      targets_[p + "attention.self.value.weight"].master = L.wqkv32.as<float>() + 2 * D * D;
      targets_[p + "intermediate.dense.weight"].master = L.w132.as<float>();
    }
  }
  if (cfg.classifier == 1) {
    register_target("classifier.dense.weight", wc_, D * D, true);
    register_target("classifier.dense.bias", bc_, D, false);
    register_target("classifier.out_proj.weight", wout_, (int64_t)cfg.num_labels * D, false);
    register_target("classifier.out_proj.bias", bout_, cfg.num_labels, false);
  }
}

Encoder::~Encoder() {
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

void Encoder::register_target(const std::string& name, DevBuf& buf, int64_t numel, bool f16,
                              int64_t offset_elems, int64_t total_elems, int64_t split_k) {
  const int64_t total = total_elems < 0 ? numel : total_elems;
  const size_t esz = f16 ? sizeof(half_t) : sizeof(float);
  const int64_t rep = split_k > 0 ? 2 : 1;  // split: hi and lo halves of every row
  if (buf.p == nullptr) {
    buf.reserve((size_t)total * rep * esz);
    SR_HIP(hipMemset(buf.p, 0, (size_t)total * rep * esz));
  }
  Target t{reinterpret_cast<char*>(buf.p) + offset_elems * rep * esz, numel, f16};
  t.split_k = split_k;
  targets_[name] = t;
  is_set_[name] = false;
}

void Encoder::set_weight(const std::string& name, const float* data, int64_t numel) {
  auto it = targets_.find(name);
  SR_CHECK(it != targets_.end(), "encoder: unknown weight '" + name + "'");
  const Target& t = it->second;
  SR_CHECK(numel == t.numel, "encoder: weight '" + name + "' has " + std::to_string(numel) +
                                 " elements, expected " + std::to_string(t.numel));
  SR_CHECK(data != nullptr, "encoder: null weight data");
  DeviceGuard g(device_);
  begin(stream_);
  SR_HIP(hipStreamSynchronize(stream_));
  if (t.f16 && t.split_k > 0) {  // row r -> [fp16(w) | fp16(w - fp16(w))], 2 split_k halfs
    const int64_t K = t.split_k;
    SR_CHECK(numel % K == 0, "encoder: split weight '" + name + "' is not whole rows");
    std::vector<half_t> h((size_t)numel * 2);
    for (int64_t r = 0; r < numel / K; ++r)
      for (int64_t j = 0; j < K; ++j) {
        const float v = data[r * K + j];
        const half_t hi = (half_t)v;
        h[(size_t)(r * 2 * K + j)] = hi;
        h[(size_t)(r * 2 * K + K + j)] = (half_t)(v - (float)hi);
      }
    SR_HIP(hipMemcpy(t.ptr, h.data(), h.size() * sizeof(half_t), hipMemcpyHostToDevice));
  } else if (t.f16) {
    std::vector<half_t> h((size_t)numel);
    for (int64_t i = 0; i < numel; ++i) h[i] = (half_t)data[i];
    SR_HIP(hipMemcpy(t.ptr, h.data(), (size_t)numel * sizeof(half_t), hipMemcpyHostToDevice));
  } else {
    SR_HIP(hipMemcpy(t.ptr, data, (size_t)numel * sizeof(float), hipMemcpyHostToDevice));
  }
  if (t.master)
    SR_HIP(hipMemcpy(t.master, data, (size_t)numel * sizeof(float), hipMemcpyHostToDevice));
  is_set_[name] = true;
  fold_ready_ = false;
}

// LayerNorm folding: with an fp16 residual stream the two LayerNorms of a block are
// never materialised.  The GEMM that produces a residual sum u also writes per-row Chan partial
// statistics; the next GEMM consumes u itself with LN(u) = (u - mu) rstd gamma + beta folded in:
//   LN(u) . W^T + b = rstd (u . (W diag gamma)^T - mu c) + (W beta + b),  c[n] = sum_k W'[n][k],
// and the residual epilogues rebuild LN(u) element-wise.  SR_LN_FOLD=0 disables it (A/B tests).
bool Encoder::fold_enabled() const {
  if (!cfg_.residual_fp16) return false;
  if (cfg_.hidden % 256 != 0 || cfg_.intermediate % 256 != 0) return false;
  const char* e = std::getenv("SR_LN_FOLD");
  return !(e && e[0] == '0');
}

// K5c (fused QKV projection + attention) for the folded layers at S == 128; SR_FUSED_QKV_ATTN=0
// keeps the QKV GEMM + K5b pair (bit-identical results; A/B tests).  Same-box bench: 461.2 vs
// 454.3 q/s (profiles/r02_fused_qkv_attention/).
static bool fused_qkv_attention_enabled() {
  const char* e = std::getenv("SR_FUSED_QKV_ATTN");
  return !(e && e[0] == '0');
}

// K/V-free CLS-only last layer of the folded cross-encoders (cls_attn_fold, k_encoder_misc.hip):
// no K / V projection of the S tokens; SR_KVFREE_CLS=0 keeps the K, V GEMM + CLS attention (A/B).
static bool kvfree_cls_enabled() {
  const char* e = std::getenv("SR_KVFREE_CLS");
  return !(e && e[0] == '0');
}

void Encoder::set_fp8(int mode) {
  // Product modes: 0 (fp16), 1 (FFN2 fp8), 3 (FFN1 + FFN2 fp8; rank like the fp32 oracle on the
  // discriminative fidelity sets) and the opt-in speed / fidelity trade 2 (also the QKV of layers
  // >= 1 in fp8 on the e4m3 residual copy: std / err 2.0).  Measured and rejected (the
  // diagnostic library keeps them for the record): 4 (QKV in fp8 on normalised e4m3 rows: 2.0) and
  // 5 (mode 3 + the O-projection of the fused layers on e4m3 ctx written by K5c: 6.4).
  SR_CHECK((mode >= 0 && mode <= 3) || (SR_WITH_DIAG && mode >= 4 && mode <= 5),
           "encoder: fp8 mode must be 0 .. 3 (modes 4 / 5 were rejected: diagnostic library only)");
  if (mode) {
    SR_CHECK(fold_enabled(), "encoder: fp8 modes need the LN-folded fp16-residual path");
    SR_CHECK(cfg_.intermediate % 128 == 0 && cfg_.intermediate >= 256 &&
                 (mode < 2 || (cfg_.hidden % 128 == 0 && cfg_.hidden >= 256)),
             "encoder: fp8 GEMMs need K % 128 == 0, K >= 256");
  }
  if (mode != fp8_) {
    fp8_ = mode;
    fold_ready_ = false;  // re-derive the folded weights (and their e4m3 copies)
  }
}

void Encoder::prepare_fold(hipStream_t s) {
  if (fold_ready_) return;
  const int64_t D = cfg_.hidden, F = cfg_.intermediate;
  for (size_t l = 0; l < layers_.size(); ++l) {
    Layer& L = layers_[l];
    L.w1_f.reserve((size_t)F * D * sizeof(half_t));
    L.c1.reserve((size_t)F * sizeof(float));
    L.d1.reserve((size_t)F * sizeof(float));
    launch_fold_ln_weight(L.w132.as<float>(), L.ln1g.as<float>(), L.ln1b.as<float>(),
                          L.b1.as<float>(), (int)F, (int)D, L.w1_f.as<half_t>(), L.c1.as<float>(),
                          L.d1.as<float>(), s);
    L.w2h.reserve((size_t)D * F * sizeof(half_t));  // 0.5 W2: FFN1 stores 2 GELU (exact scale)
    launch_scale_f16(L.w2.as<half_t>(), 0.5f, L.w2h.as<half_t>(), D * F, s);
    if (fp8_ >= 1) {
      L.w2_8.reserve((size_t)D * F);
      L.w2e.reserve((size_t)D);
      launch_quantize_rows_fp8(L.w2h.as<half_t>(), (int)D, (int)F, L.w2_8.as<uint8_t>(),
                               L.w2e.as<uint8_t>(), s);
    }
    if (fp8_ >= 2) {
      L.w1_8.reserve((size_t)F * D);
      L.w1e.reserve((size_t)F);
      L.c1_8.reserve((size_t)F * sizeof(float));
      launch_quantize_rows_fp8(L.w1_f.as<half_t>(), (int)F, (int)D, L.w1_8.as<uint8_t>(),
                               L.w1e.as<uint8_t>(), s);
      launch_colsum_fp8(L.w1_8.as<uint8_t>(), L.w1e.as<uint8_t>(), (int)F, (int)D,
                        L.c1_8.as<float>(), s);
    }
    if (fp8_ == 5) {
      L.wo_8.reserve((size_t)D * D);
      L.woe.reserve((size_t)D);
      launch_quantize_rows_fp8(L.wo.as<half_t>(), (int)D, (int)D, L.wo_8.as<uint8_t>(),
                               L.woe.as<uint8_t>(), s);
    }
    L.b2_f.reserve((size_t)D * sizeof(float));  // FFN2 bias + beta of LN1 (rebuilt residual)
    launch_vec_add(L.b2.as<float>(), L.ln1b.as<float>(), L.b2_f.as<float>(), (int)D, s);
    if (l == 0) continue;  // layer 0 reads the (normalised) embedding LayerNorm output
    const Layer& P = layers_[l - 1];
    const bool kvfree_prep = l + 1 == layers_.size() && kvfree_cls_enabled() &&
                             cls_attn_fold_supported(128, (int)D, cfg_.heads);
    L.bo_f.reserve((size_t)D * sizeof(float));  // O-proj bias + beta of the previous LN2
    launch_vec_add(L.bo.as<float>(), P.ln2b.as<float>(), L.bo_f.as<float>(), (int)D, s);
    L.wqkv_f.reserve((size_t)3 * D * D * sizeof(half_t));
    L.cqkv.reserve((size_t)3 * D * sizeof(float));
    L.dqkv.reserve((size_t)3 * D * sizeof(float));
    launch_fold_ln_weight(L.wqkv32.as<float>(), P.ln2g.as<float>(), P.ln2b.as<float>(),
                          L.bqkv.as<float>(), (int)(3 * D), (int)D, L.wqkv_f.as<half_t>(),
                          L.cqkv.as<float>(), L.dqkv.as<float>(), s);
    if (kvfree_prep) {
      const int64_t HD = (int64_t)cfg_.heads * D;
      L.wk_bd.reserve((size_t)HD * D * sizeof(half_t));
      L.wv_bd.reserve((size_t)D * 2 * HD * sizeof(half_t));
      L.zb.reserve((size_t)HD * sizeof(float));
      SR_HIP(hipMemsetAsync(L.zb.p, 0, (size_t)HD * sizeof(float), s));
      launch_kv_blockdiag(L.wqkv_f.as<half_t>(), (int)D, cfg_.heads, L.wk_bd.as<half_t>(),
                          L.wv_bd.as<half_t>(), s);
    }
    if (fp8_ == 2 || fp8_ == 4) {
      L.wqkv8.reserve((size_t)3 * D * D);
      L.wqkve.reserve((size_t)3 * D);
      L.cqkv8.reserve((size_t)3 * D * sizeof(float));
      launch_quantize_rows_fp8(L.wqkv_f.as<half_t>(), (int)(3 * D), (int)D, L.wqkv8.as<uint8_t>(),
                               L.wqkve.as<uint8_t>(), s);
      launch_colsum_fp8(L.wqkv8.as<uint8_t>(), L.wqkve.as<uint8_t>(), (int)(3 * D), (int)D,
                        L.cqkv8.as<float>(), s);
    }
  }
  if (fp8_ == 4) {  // (mu, rstd) = (0, 1) for every row: mode 4's QKV reads normalised rows
    unit_mr_.reserve(2 * sizeof(float));
    const float one[2] = {0.f, 1.f};
    SR_HIP(hipMemcpyAsync(unit_mr_.p, one, sizeof(one), hipMemcpyHostToDevice, s));
    SR_HIP(hipStreamSynchronize(s));
  }
  fold_ready_ = true;
}

std::string Encoder::missing() const {
  for (const auto& kv : is_set_)
    if (!kv.second) return kv.first;
  return std::string();
}

void Encoder::ensure_ws(int64_t tokens, int B) {
  if (tokens <= ws_tokens_) return;
  SR_HIP(hipEventSynchronize(done_));  // the previous call may still use the old workspace
  const int64_t d = cfg_.hidden, F = cfg_.intermediate;
  ids_.reserve((size_t)tokens * sizeof(int32_t));
  mask_.reserve((size_t)tokens * sizeof(int32_t));
  types_.reserve((size_t)tokens * sizeof(int32_t));
  pos_.reserve((size_t)tokens * sizeof(int32_t));
  h16_.reserve((size_t)tokens * d * sizeof(half_t));
  h32_.reserve((size_t)tokens * d * sizeof(float));
  qkv_.reserve((size_t)tokens * 3 * d * sizeof(half_t));
  ctx_.reserve((size_t)tokens * d * sizeof(half_t));
  y32_.reserve((size_t)tokens * d * sizeof(float));
  ffn_.reserve((size_t)tokens * F * sizeof(half_t));
  u8_.reserve((size_t)tokens * d);
  // split-K partial tiles of the short-M GEMMs (launch_gemm: LnFold.chunk_ws), a fixed 64 MiB
  if (!fold_enabled()) chunk_ws_.reserve(kChunkWsBytes);
  if (cfg_.residual_fp16) {
    statA_.reserve((size_t)tokens * (d / 128 + 1) * 2 * sizeof(float));
    statB_.reserve((size_t)tokens * (d / 128 + 1) * 2 * sizeof(float));
    mrA_.reserve((size_t)tokens * 2 * sizeof(float));
    mrB_.reserve((size_t)tokens * 2 * sizeof(float));
  }
  (void)B;
  ws_tokens_ = tokens;
}

void Encoder::forward_dev(const int32_t* ids, const int32_t* mask, const int32_t* types, int B,
                          int S, int mode, int pool, void* out, int out_dtype, int ld_out,
                          hipStream_t s) {
  SR_CHECK(B >= 0 && S >= 1, "encoder: bad batch shape");
  SR_CHECK(S <= cfg_.max_position - std::max(cfg_.position_offset, 0) - (cfg_.position_offset > 0 ? 1 : 0),
           "encoder: sequence longer than the position table");
  SR_CHECK(mode == 0 || cfg_.classifier == 1, "encoder: model has no classification head");
  SR_CHECK(pool == SR_POOL_CLS || pool == SR_POOL_MEAN, "encoder: pool must be CLS or MEAN");
  SR_CHECK(out_dtype == SR_DTYPE_F32 || out_dtype == SR_DTYPE_F16, "encoder: bad output dtype");
  SR_CHECK(mode == 1 || ld_out >= cfg_.hidden, "encoder: ld_out must be >= hidden");
  const std::string miss = missing();
  if (!miss.empty()) throw Error(SR_ERR_STATE, "encoder: weight not set: " + miss);
  if (B == 0) return;
  DeviceGuard g(device_);
  // s == nullptr is the HIP null stream (torch's default stream): use it as-is.
  begin(s);
  const int d = cfg_.hidden, F = cfg_.intermediate, H = cfg_.heads;
  const int64_t seqs_per_chunk = std::max<int64_t>(1, max_tokens_ / S);
  const int64_t chunk_tokens = std::min<int64_t>((int64_t)B, seqs_per_chunk) * S;
  ensure_ws(chunk_tokens, B);
  if (mode == 1 && clst_.bytes < (size_t)std::min<int64_t>(B, seqs_per_chunk) * d * sizeof(float))
    SR_HIP(hipEventSynchronize(done_));
  if (mode == 1) clst_.reserve((size_t)std::min<int64_t>(B, seqs_per_chunk) * d * sizeof(float));
  half_t* h16 = h16_.as<half_t>();
  float* h32 = h32_.as<float>();
  half_t* qkv = qkv_.as<half_t>();
  half_t* ctx = ctx_.as<half_t>();
  void* y = y32_.p;  // bias + residual sum: fp32, or fp16 with an fp16 residual stream
  half_t* ffn = ffn_.as<half_t>();
  int32_t* pos = pos_.as<int32_t>();
  const bool res16 = cfg_.residual_fp16 != 0;
  const void* hres = res16 ? (const void*)h16 : (const void*)h32;  // residual operand
  float* h32w = res16 ? nullptr : h32;
  const int epi_res = res16 ? EPI_BIAS_RES_F16 : EPI_BIAS_RES_F32;
  // Only the first token's final state is consumed (CLS pooling / classification head): the last
  // layer runs attention for query row 0 only and its O-projection, LayerNorms and FFN on the
  // B CLS rows (exact: every other row of the last layer is dead).
  const bool cls_only = (mode == 1) || (pool == SR_POOL_CLS);

  const bool fold = fold_enabled();
  if (fold) prepare_fold(s);
  const int nparts = d / 128;

  for (int64_t b0 = 0; b0 < B; b0 += seqs_per_chunk) {
    const int nb = (int)std::min<int64_t>(seqs_per_chunk, B - b0);
    const int M = nb * S;
    const int32_t* cids = ids + b0 * S;
    const int32_t* cmask = mask + b0 * S;
    const int32_t* ctypes = types ? types + b0 * S : nullptr;
    launch_positions(cids, pos, nb, S, cfg_.position_offset, s);
    launch_embed_ln(cids, pos, ctypes, wemb_.as<half_t>(), pemb_.as<half_t>(), temb_.as<half_t>(),
                    embg_.as<float>(), embb_.as<float>(), cfg_.ln_eps, M, d, cfg_.vocab_size,
                    cfg_.max_position, cfg_.type_vocab, h16, h32w, s);
    if (fold) {
      // u (un-normalised residual sums) lives in h16 (in place); compact last-layer rows in y32_.
      // sA / mrA: statistics of u after the O-projection, sB / mrB: after FFN2.
      half_t* U = h16;
      half_t* Uc = reinterpret_cast<half_t*>(y);
      float* sA = statA_.as<float>();
      float* sB = statB_.as<float>();
      float* mA = mrA_.as<float>();
      float* mB = mrB_.as<float>();
      uint8_t* u8 = u8_.as<uint8_t>();
      // K5c: QKV projection + attention in one kernel (the QKV activation stays in LDS)
      // fp8 modes: 2 and 3 run FFN1 (and FFN2) on e4m3 copies of the residual sums, mode 2 also the
      // QKV projection of layers >= 1 (then unfused); mode 3 keeps QKV + attention in fp16 (K5c)
      // mode 4 = mode 3 + the QKV projection of layers >= 1 in fp8 on an e4m3 copy of the
      // NORMALISED rows (u - mu) rstd (its own pass after the row statistics; unfused)
      const bool ffn1_8 = fp8_ >= 2, qkv_8 = fp8_ == 2 || fp8_ == 4, qkv_norm8 = fp8_ == 4;
      const bool fuse_qa = fused_qkv_attention_enabled() && !qkv_8 && qkv_attention_supported(S, d, H);
      // mode 5: the fused layers' ctx as e4m3 (in the FFN buffer, dead until this layer's FFN1)
      // and their O-projection on the fp8 MFMA
      const bool o8 = fp8_ == 5 && fuse_qa;
      uint8_t* ctx8 = reinterpret_cast<uint8_t*>(ffn);
      // (qkv_8: mode 2 keeps the e4m3 QKV path in every layer)
      const bool kvfree = cls_only && !qkv_8 && kvfree_cls_enabled() && layers_.size() > 1 &&
                          cls_attn_fold_supported(S, d, H) && layers_.back().wk_bd.p != nullptr;
      for (size_t l = 0; l < layers_.size(); ++l) {
        const Layer& L = layers_[l];
        const bool last = cls_only && l + 1 == layers_.size();
        const Layer* P = l > 0 ? &layers_[l - 1] : nullptr;
        if (fuse_qa && !last) {
          LnFold lq;
          lq.mr = mB;
          lq.colsum = L.cqkv.as<float>();
          if (l == 0)
            launch_qkv_attention(EPI_BIAS_F16, U, d, L.wqkv.as<half_t>(), L.bqkv.as<float>(), nullptr,
                                 cmask, ctx, nb, S, d, H, s, o8 ? ctx8 : nullptr);
          else
            launch_qkv_attention(EPI_LNF_F16, U, d, L.wqkv_f.as<half_t>(), L.dqkv.as<float>(), &lq,
                                 cmask, ctx, nb, S, d, H, s, o8 ? ctx8 : nullptr);
        } else if (l == 0) {
          launch_gemm(EPI_BIAS_F16, U, d, L.wqkv.as<half_t>(), L.bqkv.as<float>(), nullptr, 0, qkv,
                      3 * d, M, 3 * d, d, s);
        } else if (qkv_8) {  // A = e4m3 copy of u (mode 2: by the previous FFN2) or of the
                             // normalised rows (mode 4: quantize_norm_fp8, (mu, rstd) = (0, 1))
          LnFold lq;
          lq.mr = qkv_norm8 ? unit_mr_.as<float>() : mB;
          lq.stat_ld = qkv_norm8 ? 0 : 1;
          lq.colsum = L.cqkv8.as<float>();
          lq.wexp = L.wqkve.as<uint8_t>();
          launch_gemm_f8w(EPI_LNF_F16, u8, d, L.wqkv8.as<uint8_t>(), L.dqkv.as<float>(), nullptr, 0,
                          qkv, 3 * d, M, 3 * d, d, s, &lq);
        } else if (last && kvfree) {
          // K/V-free CLS-only last layer: q of the CLS rows, w_h = W'_{k,h}^T q_h (one GEMM on the
          // block-diagonal weight), scores / softmax / z' per sequence (as an fp16 hi + lo pair),
          // ctx = W'_v z' + d_v (one GEMM, K = 2 H d)
          LnFold lc;  // A = row b*S of each sequence (stride S*d), its statistics at row b*S
          lc.mr = mB;
          lc.stat_ld = S;
          lc.colsum = L.cqkv.as<float>();
          const int64_t HD = (int64_t)H * d;
          half_t* qc = ffn;
          half_t* wq = ffn + (int64_t)nb * d;
          half_t* zq = wq + (int64_t)nb * HD;
          launch_gemm(EPI_LNF_F16, U, (int64_t)S * d, L.wqkv_f.as<half_t>(), L.dqkv.as<float>(), nullptr,
                      0, qc, d, nb, d, d, s, &lc);
          launch_gemm(EPI_BIAS_F16, qc, d, L.wk_bd.as<half_t>(), L.zb.as<float>(), nullptr, 0, wq, HD, nb,
                      (int)HD, d, s);
          launch_cls_attn_fold(wq, U, mB, cmask, nb, S, d, H, zq, s);
          launch_gemm(EPI_BIAS_F16, zq, 2 * HD, L.wv_bd.as<half_t>(), L.dqkv.as<float>() + 2 * d, nullptr,
                      0, ctx, d, nb, d, (int)(2 * HD), s);
        } else if (last && d % 256 == 0) {  // CLS-only last layer: K, V for all rows, Q for CLS rows
          LnFold lq;
          lq.mr = mB;
          lq.colsum = L.cqkv.as<float>() + d;
          launch_gemm(EPI_LNF_F16, U, d, L.wqkv_f.as<half_t>() + (int64_t)d * d, L.dqkv.as<float>() + d,
                      nullptr, 0, qkv + d, 3 * d, M, 2 * d, d, s, &lq);
          LnFold lc;  // A = row b*S of each sequence (stride S*d), its statistics at row b*S
          lc.mr = mB;
          lc.stat_ld = S;
          lc.colsum = L.cqkv.as<float>();
          launch_gemm(EPI_LNF_F16, U, (int64_t)S * d, L.wqkv_f.as<half_t>(), L.dqkv.as<float>(), nullptr,
                      0, qkv, (int64_t)S * 3 * d, nb, d, d, s, &lc);
        } else {  // A = u of the previous block, its LN2 folded into W'
          LnFold lq;
          lq.mr = mB;
          lq.colsum = L.cqkv.as<float>();
          launch_gemm(EPI_LNF_F16, U, d, L.wqkv_f.as<half_t>(), L.dqkv.as<float>(), nullptr, 0, qkv,
                      3 * d, M, 3 * d, d, s, &lq);
        }
        const int Mr = last ? nb : M;
        if (!(fuse_qa && !last) && !(last && kvfree))
          launch_attention(qkv, cmask, ctx, nb, S, last ? 1 : S, d, H, s);
        // O-projection + residual LN2(l-1)(u) -> u1 (in place, or compact rows) + partials sA
        half_t* Uo = last ? Uc : U;
        LnFold lo;
        lo.mr = mB;
        lo.stat_ld = last ? S : 1;
        lo.gamma = P ? P->ln2g.as<float>() : nullptr;
        lo.stat_out = sA;
        lo.y8 = ffn1_8 ? u8 : nullptr;  // e4m3 copy of u1 for the fp8 FFN1
        const int eo = ffn1_8 ? (l == 0 ? EPI_RES16_STATS_Y8 : EPI_LNR16_STATS_Y8)
                                 : (l == 0 ? EPI_RES16_STATS : EPI_LNR16_STATS);
        if (o8 && !last) {  // e4m3 ctx (K5c) x e4m3 W_o rows on the block-scaled fp8 MFMA
          lo.wexp = L.woe.as<uint8_t>();
          launch_gemm_f8w(eo, ctx8, d, L.wo_8.as<uint8_t>(), (l == 0 ? L.bo : L.bo_f).as<float>(), U,
                          d, Uo, d, Mr, d, d, s, &lo);
        } else {
          launch_gemm(eo, ctx, d, L.wo.as<half_t>(),
                      (l == 0 ? L.bo : L.bo_f).as<float>(), U, last ? (int64_t)S * d : d, Uo, d, Mr,
                      d, d, s, &lo);
        }
        launch_ln_stats_finalize(sA, nparts, cfg_.ln_eps, Mr, mA, s);
        // FFN1 on LN1(u1) folded; FFN2 + residual LN1(u1) -> u2 (in place) + partials sB
        LnFold l1;
        l1.mr = mA;
        l1.colsum = L.c1.as<float>();
        if (ffn1_8) {
          l1.colsum = L.c1_8.as<float>();
          l1.wexp = L.w1e.as<uint8_t>();
          launch_gemm_f8w(EPI_LNF_GELU_F8, u8, d, L.w1_8.as<uint8_t>(), L.d1.as<float>(), nullptr, 0,
                          ffn, F, Mr, F, d, s, &l1);
        } else {
          launch_gemm(fp8_ ? EPI_LNF_GELU_F8 : EPI_LNF_GELU_F16, Uo, d, L.w1_f.as<half_t>(),
                      L.d1.as<float>(), nullptr, 0, ffn, F, Mr, F, d, s, &l1);
        }
        LnFold l2;
        l2.mr = mA;
        l2.gamma = L.ln1g.as<float>();
        l2.stat_out = sB;
        l2.wexp = L.w2e.as<uint8_t>();
        l2.y8 = (qkv_8 && !qkv_norm8 && !last) ? u8 : nullptr;  // e4m3 copy of u2 for the next fp8 QKV
        if (fp8_)  // ffn holds e4m3 bytes (F per row)
          launch_gemm_f8w(l2.y8 ? EPI_LNR16_STATS_Y8 : EPI_LNR16_STATS, reinterpret_cast<const uint8_t*>(ffn), F,
                          L.w2_8.as<uint8_t>(), L.b2_f.as<float>(), Uo, d, Uo, d, Mr, d, F, s, &l2);
        else
          launch_gemm(EPI_LNR16_STATS, ffn, F, L.w2h.as<half_t>(), L.b2_f.as<float>(), Uo, d, Uo,
                      d, Mr, d, F, s, &l2);
        launch_ln_stats_finalize(sB, nparts, cfg_.ln_eps, Mr, mB, s);
        if (qkv_norm8 && l + 1 < layers_.size()) launch_quantize_norm_fp8(Uo, d, mB, Mr, d, u8, s);
      }
      // final LayerNorm (LN2 of the last block) of the rows that are consumed -> h16
      const Layer& Lz = layers_.back();
      launch_ln_apply(cls_only ? Uc : U, d, mB, Lz.ln2g.as<float>(), Lz.ln2b.as<float>(),
                      cls_only ? nb : M, d, h16, s);
    }
    // split weights: W = [hi | lo] (N x 2K), the GEMM's K is 2K over the repeated activation
    const int kr = split_ ? 2 : 1;
    auto lin = [&](int epi, const half_t* X, int64_t lda, const half_t* W, const float* b,
                   const void* R, int64_t ldr, void* Y, int64_t ldy, int Mm, int Nn, int Kx) {
      LnFold lx;
      lx.x_k = split_ ? Kx : 0;
      lx.chunk_ws = chunk_ws_.as<float>();
      lx.chunk_ws_bytes = (int64_t)chunk_ws_.bytes;
      launch_gemm(epi, X, lda, W, b, R, ldr, Y, ldy, Mm, Nn, kr * Kx, s, &lx);
    };
    for (size_t l = 0; l < (fold ? 0 : layers_.size()); ++l) {
      const Layer& L = layers_[l];
      const bool last = cls_only && l + 1 == layers_.size();
      lin(EPI_BIAS_F16, h16, d, L.wqkv.as<half_t>(), L.bqkv.as<float>(), nullptr, 0, qkv, 3 * d, M,
          3 * d, d);
      // rows of the rest of the block: all M tokens, or the nb CLS rows (compact) in the last layer
      const int Mr = last ? nb : M;
      launch_attention(qkv, cmask, ctx, nb, S, last ? 1 : S, d, H, s);
      lin(epi_res, ctx, d, L.wo.as<half_t>(), L.bo.as<float>(), hres, last ? (int64_t)S * d : d, y,
          d, Mr, d, d);
      launch_layernorm(y, res16, L.ln1g.as<float>(), L.ln1b.as<float>(), cfg_.ln_eps, Mr, d, h16,
                       h32w, s);
      lin(EPI_BIAS_GELU_F16, h16, d, L.w1.as<half_t>(), L.b1.as<float>(), nullptr, 0, ffn, F, Mr, F,
          d);
      lin(epi_res, ffn, F, L.w2.as<half_t>(), L.b2.as<float>(), hres, d, y, d, Mr, d, F);
      launch_layernorm(y, res16, L.ln2g.as<float>(), L.ln2b.as<float>(), cfg_.ln_eps, Mr, d, h16,
                       h32w, s);
    }
    // final states: row b*S of each sequence, or row b (compact) after a CLS-only last layer
    const int Sf = cls_only ? 1 : S;
    if (mode == 0) {
      const size_t esz = out_dtype == SR_DTYPE_F32 ? sizeof(float) : sizeof(half_t);
      launch_pool_l2(res16 ? (const void*)h16 : (const void*)h32, res16, cmask, nb, Sf, d, pool,
                     reinterpret_cast<char*>(out) + (size_t)b0 * ld_out * esz, out_dtype, ld_out, s);
    } else {
      float* t = clst_.as<float>();
      launch_gemm(EPI_BIAS_TANH_F32, h16, (int64_t)Sf * d, wc_.as<half_t>(), bc_.as<float>(),
                  nullptr, 0, t, d, nb, d, d, s);
      launch_cls_logits(t, wout_.as<float>(), bout_.as<float>(), nb, d, cfg_.num_labels,
                        reinterpret_cast<float*>(out) + b0 * cfg_.num_labels, s);
    }
  }
  end(s);
}

void Encoder::forward_host(const int32_t* ids, const int32_t* mask, const int32_t* types, int B,
                           int S, int mode, int pool, float* out) {
  SR_CHECK(B >= 0 && S >= 1 && (B == 0 || (ids && mask && out)), "encoder: null buffer");
  if (B == 0) return;
  DeviceGuard g(device_);
  const int64_t n = (int64_t)B * S;
  const int64_t out_elems = (int64_t)B * (mode == 0 ? cfg_.hidden : cfg_.num_labels);
  const size_t in_bytes = (size_t)n * sizeof(int32_t) * (types ? 3 : 2);
  hostio_.reserve(in_bytes + (size_t)out_elems * sizeof(float));
  int32_t* dids = hostio_.as<int32_t>();
  int32_t* dmask = dids + n;
  int32_t* dtypes = types ? dmask + n : nullptr;
  float* dout = reinterpret_cast<float*>(hostio_.as<char>() + in_bytes);
  SR_HIP(hipMemcpyAsync(dids, ids, n * sizeof(int32_t), hipMemcpyHostToDevice, stream_));
  SR_HIP(hipMemcpyAsync(dmask, mask, n * sizeof(int32_t), hipMemcpyHostToDevice, stream_));
  if (types) SR_HIP(hipMemcpyAsync(dtypes, types, n * sizeof(int32_t), hipMemcpyHostToDevice, stream_));
  forward_dev(dids, dmask, dtypes, B, S, mode, pool, dout, SR_DTYPE_F32, cfg_.hidden, stream_);
  SR_HIP(hipMemcpyAsync(out, dout, (size_t)out_elems * sizeof(float), hipMemcpyDeviceToHost, stream_));
  SR_HIP(hipStreamSynchronize(stream_));
}

}  // namespace sr
