"""GPU: K5c, the fused QKV projection + attention of the LN-folded encoder layers at S == 128
(k_attention.hip qkv_attn_kernel), against the unfused QKV GEMM + K5b pair (SR_FUSED_QKV_ATTN=0)
bit for bit, and against the fp32 oracle within the fp16-residual band of test_gpu_encoder.py.

Cases: one sequence (a 256-token panel holding one sequence), odd and even sequence counts, ragged
key masks, layer 0 (bias epilogue) and the LayerNorm-folded layers, CLS-only last layer (unfused)
and a mean-pooled embedder whose last layer is fused too, the bge-reranker-base shape, and a
chunked forward (several workspace chunks)."""
import numpy as np
import pytest

from oracle import encoder_ref as R

pytestmark = pytest.mark.gpu


def _cfg(s):
    return R.RefConfig(s.vocab_size, s.hidden, s.layers, s.heads, s.intermediate, s.max_position,
                       s.type_vocab, s.ln_eps, s.position_offset, s.classifier, s.num_labels)


def _batch(spec, B, S, seed):
    rng = np.random.default_rng(seed)
    ids = rng.integers(5, spec.vocab_size, (B, S)).astype(np.int32)
    lens = rng.integers(max(1, S // 3), S + 1, B)
    lens[0] = S
    mask = (np.arange(S)[None] < lens[:, None]).astype(np.int32)
    ids[:, 0] = spec.bos_id
    return np.where(mask == 1, ids, spec.pad_id).astype(np.int32), mask


def _affine_ln(w):
    # non-trivial LayerNorm parameters so the folded epilogues are exercised
    for k in list(w):
        if k.endswith("LayerNorm.weight"):
            w[k] = (1.0 + 0.3 * np.random.default_rng(len(k)).standard_normal(w[k].shape)).astype(np.float32)
        elif k.endswith("LayerNorm.bias"):
            w[k] = (0.2 * np.random.default_rng(len(k) + 1).standard_normal(w[k].shape)).astype(np.float32)
    return w


def _both(monkeypatch, fn):
    monkeypatch.setenv("SR_FUSED_QKV_ATTN", "0")
    ref = fn()
    monkeypatch.setenv("SR_FUSED_QKV_ATTN", "1")
    return fn(), ref


@pytest.mark.parametrize("B", [1, 3, 34, 201])  # 201: 404 tiles, walkers take several
def test_fused_cross_encoder_bit_exact(B, monkeypatch):
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    spec = ModelSpec("t", "xlmr", 1000, 256, 3, 4, 512, 200, 1, 1e-5, 1, classifier=1, bos_id=0,
                     eos_id=2, pad_id=1, residual_fp16=True)
    w = _affine_ln(random_weights(spec, seed=5, style="test"))
    w["classifier.out_proj.weight"] *= 50.0
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, B, 128, seed=B)
    got, unfused = _both(monkeypatch, lambda: enc.cross_score(ids, mask))
    np.testing.assert_array_equal(got, unfused)
    ref = R.cross_logits(_cfg(spec), w, ids, mask)
    assert np.abs(got - ref).max() <= 4e-3 * (1.0 + np.abs(ref).max())


def test_fused_embedder_every_layer_bit_exact(monkeypatch):
    # mean pooling: the last layer is a full layer, so every layer runs the fused kernel
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    spec = ModelSpec("t", "bert", 1000, 256, 2, 4, 512, 200, 2, 1e-12, 0, residual_fp16=True)
    w = _affine_ln(random_weights(spec, seed=6, style="test"))
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 5, 128, seed=7)
    got, unfused = _both(monkeypatch, lambda: enc.embed(ids, mask, pool="mean"))
    np.testing.assert_array_equal(got, unfused)
    ref = R.embed(_cfg(spec), w, ids, mask, pool="mean")
    assert (np.linalg.norm(got - ref, axis=1) <= 4e-3).all()


def test_fused_bge_reranker_shape_chunked(monkeypatch):
    # bge-reranker-base (12 layers, d 768, 12 heads) at S = 128 over several workspace chunks
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    spec = MODELS["bge-reranker-base"]
    w = random_weights(spec, seed=22, style="test")
    w["classifier.out_proj.weight"] *= 50.0
    enc = Encoder(spec, weights=w, max_tokens=128 * 5)
    ids, mask = _batch(spec, 13, 128, seed=3)
    got, unfused = _both(monkeypatch, lambda: enc.cross_score(ids, mask))
    np.testing.assert_array_equal(got, unfused)
    ref = R.cross_logits(_cfg(spec), w, ids, mask)
    assert np.abs(got - ref).max() <= 1e-2 * (1.0 + np.abs(ref).max())


def test_fused_full_chunk_bit_exact(monkeypatch):
    # the bench's chunk: 12,800 pairs x 128 tokens in one launch per layer (76,800 tiles, 300 per
    # persistent walker): fused == unfused bit for bit
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    spec = MODELS["bge-reranker-base"]
    enc = Encoder(spec, weights=random_weights(spec, seed=23, style="hf"), max_tokens=1_638_400)
    ids, mask = _batch(spec, 12_800, 128, seed=4)
    got, unfused = _both(monkeypatch, lambda: enc.cross_score(ids, mask))
    np.testing.assert_array_equal(got, unfused)
    enc.close()
