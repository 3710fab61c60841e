"""GPU parity: encoder kernels (K3 embed+LN, K4 MFMA GEMM, K5 attention, K6 LN, K7 pool+L2,
K8 classification head) and the pair packer / rerank ordering vs the fp32 CPU oracle.

Tolerances (north_star: "embeddings within 1e-3 rel"):
  * sentence embeddings: ||e_gpu - e_ref||_2 / ||e_ref||_2 <= 1e-3 at the bge-base shape
    (fp16 GEMM operands, fp32 accumulation and fp32 residual stream);
  * cross-encoder logits: |l_gpu - l_ref| <= 2e-3 * (1 + |l_ref|), and the per-query top-k
    candidate sets agree modulo candidates whose reference logits lie within that band.
"""
import numpy as np
import pytest

from oracle import encoder_ref as R
from oracle.cosine_topk import same_topk_modulo_ties

pytestmark = pytest.mark.gpu


def _ref_cfg(spec):
    return R.RefConfig(spec.vocab_size, spec.hidden, spec.layers, spec.heads, spec.intermediate,
                       spec.max_position, spec.type_vocab, spec.ln_eps, spec.position_offset,
                       spec.classifier, spec.num_labels)


def _tiny(arch="bert", d=128, L=2, H=2, F=256, classifier=0, V=1000, P=80, res16=False):
    from super_rag_amd.encoder import ModelSpec
    if arch == "bert":
        return ModelSpec("tiny-bert", "bert", V, d, L, H, F, P, 2, 1e-12, 0, classifier=classifier,
                         residual_fp16=res16)
    return ModelSpec("tiny-xlmr", "xlmr", V, d, L, H, F, P, 1, 1e-5, 1, classifier=classifier,
                     bos_id=0, eos_id=2, pad_id=1, residual_fp16=res16)


def _batch(spec, B, S, seed, ragged=True):
    rng = np.random.default_rng(seed)
    ids = rng.integers(5, spec.vocab_size, (B, S)).astype(np.int32)
    lens = rng.integers(max(1, S // 3), S + 1, B) if ragged else np.full(B, S)
    mask = (np.arange(S)[None] < lens[:, None]).astype(np.int32)
    ids[:, 0] = spec.bos_id
    ids = np.where(mask == 1, ids, spec.pad_id).astype(np.int32)
    return ids, mask


def _rel(a, b):
    return np.linalg.norm(a - b, axis=-1) / np.linalg.norm(b, axis=-1)


@pytest.mark.parametrize("arch,H,pool", [("bert", 2, "cls"), ("bert", 4, "mean"),
                                         ("xlmr", 2, "cls")])
@pytest.mark.parametrize("S", [1, 17, 64, 77])
def test_tiny_embed(arch, H, pool, S):
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny(arch, H=H)
    w = random_weights(spec, seed=3, style="test")
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 13, S, seed=S)
    tt = (np.arange(S)[None] >= S // 2).astype(np.int32).repeat(13, 0) if arch == "bert" else None
    got = enc.embed(ids, mask, tt, pool=pool)
    ref = R.embed(_ref_cfg(spec), w, ids, mask, tt, pool=pool)
    assert _rel(got, ref).max() <= 2e-3
    np.testing.assert_allclose(np.linalg.norm(got, axis=1), 1.0, atol=1e-5)


def test_bge_base_shape_embedding_tolerance():
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    spec = MODELS["bge-base-en"]
    w = random_weights(spec, seed=7, style="test")
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 8, 32, seed=1)
    got = enc.embed(ids, mask)
    ref = R.embed(_ref_cfg(spec), w, ids, mask)
    err = _rel(got, ref)
    assert err.max() <= 1e-3, err


def test_bge_base_embedding_independent_of_batch_split_k():
    # Short M runs the embedder's GEMMs split over K chunks (k_gemm.hip KCHUNK: partial tiles +
    # gemm_chunk_reduce_kernel), long M unsplit with the same chunked sums: a query's embedding is
    # bit-identical alone, in a small batch (some GEMMs split, some not) and in a large one (none
    # split: M = 300 x 32 rows gives >= 450 tiles per GEMM).
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    spec = MODELS["bge-base-en"]
    w = random_weights(spec, seed=7, style="test")
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 300, 32, seed=4)
    full = enc.embed(ids, mask)
    for b in (1, 3, 8, 21, 32):
        np.testing.assert_array_equal(enc.embed(ids[:b], mask[:b]), full[:b])
    ref = R.embed(_ref_cfg(spec), w, ids[:3], mask[:3])
    assert _rel(full[:3], ref).max() <= 1e-3


@pytest.mark.parametrize("res16", [False, True])
@pytest.mark.parametrize("S", [16, 64, 130])
def test_tiny_cross_encoder(S, res16):
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("xlmr", classifier=1, P=200, res16=res16)
    w = random_weights(spec, seed=4, style="test")
    w["classifier.out_proj.weight"] *= 50.0  # spread the logits
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 37, S, seed=S)
    got = enc.cross_score(ids, mask)[:, 0]
    ref = R.cross_logits(_ref_cfg(spec), w, ids, mask)[:, 0]
    tol = (4e-3 if res16 else 2e-3) * (1.0 + np.abs(ref).max())
    assert np.abs(got - ref).max() <= tol
    # ranking contract: top-10 of the 37 candidates agree modulo near-ties
    top_g = np.argsort(-got, kind="stable")[:10][None]
    top_r = np.argsort(-ref, kind="stable")[:10][None]
    assert same_topk_modulo_ties(top_g, got[top_g], top_r, ref[top_r], 2 * tol)


def test_chunked_forward_matches_single_launch():
    # max_tokens forces several workspace chunks; results must not depend on the chunking
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("bert")
    w = random_weights(spec, seed=5, style="test")
    a = Encoder(spec, weights=w)
    b = Encoder(spec, weights=w, max_tokens=100)
    ids, mask = _batch(spec, 20, 24, seed=2)
    np.testing.assert_array_equal(a.embed(ids, mask), b.embed(ids, mask))


def test_device_pair_packing_and_rerank_select():
    import torch
    from super_rag_amd.encoder import build_pairs_dev, rerank_select_dev
    rng = np.random.default_rng(0)
    for spec in (_tiny("xlmr"), _tiny("bert")):
        B, K, S, lq, lp, Np = 5, 7, 24, 12, 30, 50
        q_tok = rng.integers(10, 900, (B, lq)).astype(np.int32)
        q_len = rng.integers(0, lq + 1, B).astype(np.int32)
        p_tok = rng.integers(10, 900, (Np, lp)).astype(np.int32)
        p_len = rng.integers(0, lp + 1, Np).astype(np.int32)
        rows = rng.integers(-1, Np, (B, K)).astype(np.int64)
        t = lambda a: torch.from_numpy(a).cuda()
        ids, mask, typ = build_pairs_dev(t(q_tok), t(q_len), t(p_tok), t(p_len), t(rows), S, spec,
                                         with_types=True)
        e_ids, e_mask, e_typ = R.pack_pairs(q_tok, q_len, p_tok, p_len, rows, S, spec.pair_style,
                                            spec.bos_id, spec.eos_id, spec.pad_id)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(ids.cpu().numpy(), e_ids)
        np.testing.assert_array_equal(mask.cpu().numpy(), e_mask)
        np.testing.assert_array_equal(typ.cpu().numpy(), e_typ)
    logits = rng.standard_normal((9, 100)).astype(np.float32)
    logits[0, 10:20] = 1.5  # exact ties -> candidate order
    idx = rerank_select_dev(torch.from_numpy(logits).cuda(), 10).cpu().numpy()
    for b in range(9):
        exp = sorted(range(100), key=lambda j: (-logits[b, j], j))[:10]
        assert idx[b].tolist() == exp


@pytest.mark.parametrize("tile", ["small", "big"])
@pytest.mark.parametrize("pool", ["cls", "mean"])
def test_gemm_tiles_and_cls_only_last_layer(tile, pool, monkeypatch):
    # d=256 / F=512 so the 256x256 MFMA tile is legal; SR_GEMM_TILE forces the tile choice.
    # pool="cls" runs the CLS-only last layer, pool="mean" the full one: both must match.
    from super_rag_amd.encoder import Encoder, random_weights
    monkeypatch.setenv("SR_GEMM_TILE", tile)
    spec = _tiny("bert", d=256, H=4, F=512, L=3)
    w = random_weights(spec, seed=8, style="test")
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 40, 50, seed=9)   # M = 2000 rows: ragged last tiles
    got = enc.embed(ids, mask, pool=pool)
    ref = R.embed(_ref_cfg(spec), w, ids, mask, pool=pool)
    assert _rel(got, ref).max() <= 2e-3


def test_bge_reranker_shape_fp16_residual_ranking():
    # bge-reranker-base shape (XLM-R base, fp16 residual stream as shipped): logits within band,
    # candidate top-10 identical modulo near-ties.
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    spec = MODELS["bge-reranker-base"]
    w = random_weights(spec, seed=21, style="test")
    w["classifier.out_proj.weight"] *= 50.0
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 48, 64, seed=4, ragged=True)
    got = enc.cross_score(ids, mask)[:, 0]
    ref = R.cross_logits(_ref_cfg(spec), w, ids, mask)[:, 0]
    tol = 1e-2 * (1.0 + np.abs(ref).max())
    assert np.abs(got - ref).max() <= tol
    top_g = np.argsort(-got, kind="stable")[:10][None]
    top_r = np.argsort(-ref, kind="stable")[:10][None]
    assert same_topk_modulo_ties(top_g, got[top_g], top_r, ref[top_r], 2 * tol)


@pytest.mark.parametrize("fold", ["1", "0"])
@pytest.mark.parametrize("S", [16, 50, 130])
def test_ln_folded_cross_encoder(fold, S, monkeypatch):
    # fp16 residual stream with d % 256 == 0: the LayerNorms are folded into the GEMMs (per-row
    # Chan statistics from the residual epilogues, gamma folded into W, LN rebuilt in the residual
    # epilogue); SR_LN_FOLD=0 is the materialised-LayerNorm path.  Both match the fp32 oracle.
    from super_rag_amd.encoder import Encoder, random_weights
    monkeypatch.setenv("SR_LN_FOLD", fold)
    spec = _tiny("xlmr", d=256, H=4, F=512, L=3, classifier=1, P=200, res16=True)
    w = random_weights(spec, seed=31, style="test")
    for k in list(w):  # non-trivial LayerNorm affine parameters exercise the folding
        if k.endswith("LayerNorm.weight"):
            w[k] = (1.0 + 0.3 * np.random.default_rng(len(k)).standard_normal(w[k].shape)).astype(np.float32)
        elif k.endswith("LayerNorm.bias"):
            w[k] = (0.2 * np.random.default_rng(len(k) + 1).standard_normal(w[k].shape)).astype(np.float32)
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 33, S, seed=S)
    got = enc.cross_score(ids, mask)
    ref = R.cross_logits(_ref_cfg(spec), w, ids, mask)
    tol = 4e-3 * (1.0 + np.abs(ref).max())
    assert np.abs(got - ref).max() <= tol


@pytest.mark.parametrize("pool", ["cls", "mean"])
def test_ln_folded_embedder(pool):
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("bert", d=256, H=4, F=512, L=2, res16=True)
    w = random_weights(spec, seed=41, style="test")
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 24, 40, seed=5)
    got = enc.embed(ids, mask, pool=pool)
    ref = R.embed(_ref_cfg(spec), w, ids, mask, pool=pool)
    assert _rel(got, ref).max() <= 4e-3


@pytest.mark.parametrize("S", [700, 2048])
def test_bge_m3_widths_long_sequences(S):
    # bge-m3 / bge-reranker-v2-m3 widths (XLM-R large: d 1024, 16 heads, FFN 4096; 2 of the 24
    # layers) at sequence lengths past 512 (max_position 8194): the 64-key-tile attention path,
    # the 256x256 GEMM tiles at d = 1024; CLS embedding and classification logit vs the oracle.
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    emb = ModelSpec("m3-2l", "xlmr", 250002, 1024, 2, 16, 4096, 8194, 1, 1e-5, 1, bos_id=0,
                    eos_id=2, pad_id=1, max_length=8192)
    w = random_weights(emb, seed=51, style="test")
    enc = Encoder(emb, weights=w)
    ids, mask = _batch(emb, 3, S, seed=S)
    got = enc.embed(ids, mask, pool="cls")
    ref = R.embed(_ref_cfg(emb), w, ids, mask, pool="cls")
    assert _rel(got, ref).max() <= 2e-3
    rr = ModelSpec("m3r-2l", "xlmr", 250002, 1024, 2, 16, 4096, 8194, 1, 1e-5, 1, classifier=1,
                   bos_id=0, eos_id=2, pad_id=1, max_length=8192, residual_fp16=True)
    wr = random_weights(rr, seed=52, style="test")
    lg = Encoder(rr, weights=wr).cross_score(ids, mask)
    lg_ref = R.cross_logits(_ref_cfg(rr), wr, ids, mask)
    assert np.abs(lg - lg_ref).max() <= 1e-2 * (1.0 + np.abs(lg_ref).max())


@pytest.mark.parametrize("S", [16, 130])
def test_fp8_ffn_cross_encoder(S):
    # fp8 FFN mode: FFN1 stores e4m3(2 GELU), FFN2 runs the block-scaled fp8 MFMA on an e4m3 copy
    # of W2 / 2 with per-row power-of-two scales.  Against the oracle restating exactly that
    # quantisation (oracle/encoder_ref.py fp8_ffn) the band is the fp16 path's; against the plain
    # fp32 model the logits move by the fp8 rounding.
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("xlmr", d=256, H=4, F=512, L=3, classifier=1, P=200, res16=True)
    w = random_weights(spec, seed=32, style="test")
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 33, S, seed=S + 1)
    got16 = enc.cross_score(ids, mask)
    enc.set_fp8_ffn(True)
    got8 = enc.cross_score(ids, mask)
    ref8 = R.cross_logits(_ref_cfg(spec), w, ids, mask, fp8_ffn=True)
    ref = R.cross_logits(_ref_cfg(spec), w, ids, mask)
    scale = 1.0 + np.abs(ref).max()
    assert not np.array_equal(got8, got16)
    assert np.abs(got8 - ref8).max() <= 8e-3 * scale
    assert np.abs(got8 - ref).max() <= 5e-2 * scale
    enc.set_fp8_ffn(False)
    np.testing.assert_array_equal(enc.cross_score(ids, mask), got16)


@pytest.mark.parametrize("S", [16, 130])
def test_fp8_mode2_cross_encoder(S):
    # fp8 mode 2: FFN1 and the QKV of layers >= 1 also run the block-scaled fp8 MFMA, on e4m3
    # copies of the pre-LN residual sums (written by the Wo / FFN2 epilogues) against e4m3 row
    # copies of the LN-folded weights.  Against the oracle restating that quantisation
    # (oracle/encoder_ref.py _fold8) the band is the fp8 FFN test's; against fp32 the fp8 rounding.
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("xlmr", d=256, H=4, F=512, L=3, classifier=1, P=200, res16=True)
    w = random_weights(spec, seed=34, style="test")
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 33, S, seed=S + 3)
    got1 = (enc.set_fp8(1), enc.cross_score(ids, mask))[1]
    enc.set_fp8(2)
    got2 = enc.cross_score(ids, mask)
    ref2 = R.cross_logits(_ref_cfg(spec), w, ids, mask, fp8=2)
    ref = R.cross_logits(_ref_cfg(spec), w, ids, mask)
    scale = 1.0 + np.abs(ref).max()
    assert not np.array_equal(got2, got1)
    assert np.abs(got2 - ref2).max() <= 8e-3 * scale
    assert np.abs(got2 - ref).max() <= 5e-2 * scale
    enc.set_fp8(1)
    np.testing.assert_array_equal(enc.cross_score(ids, mask), got1)


@pytest.mark.parametrize("S", [16, 128, 130])
def test_fp8_mode3_cross_encoder(S):
    # fp8 mode 3: FFN1 and FFN2 on the block-scaled fp8 MFMA as in mode 2, the QKV projection and
    # attention in fp16 (the fused K5c kernel where supported, S = 128 here): against the oracle
    # restating that quantisation (fp8=3) the band is mode 2's
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("xlmr", d=256, H=4, F=512, L=3, classifier=1, P=200, res16=True)
    w = random_weights(spec, seed=37, style="test")
    enc = Encoder(spec, weights=w)
    ids, mask = _batch(spec, 33, S, seed=S + 5)
    enc.set_fp8(3)
    got3 = enc.cross_score(ids, mask)
    ref3 = R.cross_logits(_ref_cfg(spec), w, ids, mask, fp8=3)
    ref2 = R.cross_logits(_ref_cfg(spec), w, ids, mask, fp8=2)
    ref = R.cross_logits(_ref_cfg(spec), w, ids, mask)
    scale = 1.0 + np.abs(ref).max()
    assert np.abs(got3 - ref3).max() <= 8e-3 * scale
    assert np.abs(got3 - ref).max() <= 5e-2 * scale
    assert not np.array_equal(ref3, ref2)
    enc.set_fp8(0)


def test_fp8_mode2_persistent_tiles():
    # 143k tokens: the persistent fp8 QKV / FFN1 / FFN2 kernels and the _Y8 epilogues
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("xlmr", d=256, H=4, F=512, L=2, classifier=1, P=200, res16=True)
    w = random_weights(spec, seed=35, style="test")
    enc = Encoder(spec, weights=w, max_tokens=1 << 18)
    enc.set_fp8(2)
    ids, mask = _batch(spec, 1100, 130, seed=8, ragged=False)
    got = enc.cross_score(ids, mask)
    ref = R.cross_logits(_ref_cfg(spec), w, ids, mask, fp8=2)
    assert np.abs(got - ref).max() <= 8e-3 * (1.0 + np.abs(ref).max())


def test_fp8_mode_rejects_unfolded_encoder():
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("bert", d=256, H=4, F=512, L=2)
    enc = Encoder(spec, weights=random_weights(spec, seed=36, style="test"))
    with pytest.raises(RuntimeError):
        enc.set_fp8(2)
    with pytest.raises(RuntimeError):
        enc.set_fp8(3)


def test_fp8_ffn_persistent_tiles():
    # enough rows (143k tokens) for the persistent fp8 FFN2 / e4m3-output FFN1 kernels
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("xlmr", d=256, H=4, F=512, L=2, classifier=1, P=200, res16=True)
    w = random_weights(spec, seed=33, style="test")
    enc = Encoder(spec, weights=w, max_tokens=1 << 18)
    enc.set_fp8_ffn(True)
    ids, mask = _batch(spec, 1100, 130, seed=7, ragged=False)
    got8 = enc.cross_score(ids, mask)
    ref8 = R.cross_logits(_ref_cfg(spec), w, ids, mask, fp8_ffn=True)
    assert np.abs(got8 - ref8).max() <= 8e-3 * (1.0 + np.abs(ref8).max())


@pytest.mark.parametrize("S,L,d,H,nb", [(16, 2, 768, 12, 40), (64, 3, 768, 12, 40), (128, 2, 768, 12, 40),
                                        (512, 2, 768, 12, 12), (64, 2, 1024, 16, 40),
                                        (128, 2, 768, 12, 600), (96, 2, 1024, 16, 300)])
def test_kvfree_cls_last_layer(S, L, d, H, nb, monkeypatch):
    # K/V-free CLS-only last layer (cls_attn_fold): with LN folded the CLS query's scores are
    # rstd_j (w_h . u_j - mu_j sum w_h) with w_h = W'_{k,h}^T q_h and its context W'_v z' + d_v, so
    # no token is projected to K / V.  Ragged masks, non-trivial LayerNorm affine parameters, the
    # bge-reranker-base / -v2-m3 head geometries (d 768 / 1024, heads of 64): against the fp32 oracle
    # within the fp16 residual band, and against the K, V GEMM + CLS attention path (SR_KVFREE_CLS=0).
    from super_rag_amd.encoder import Encoder, random_weights
    spec = _tiny("xlmr", d=d, H=H, F=4 * d, L=L, classifier=1, P=max(200, S + 8), res16=True)
    w = random_weights(spec, seed=41 + S, style="test")
    rng = np.random.default_rng(S)
    for k in list(w):
        if k.endswith("LayerNorm.weight"):
            w[k] = (1.0 + 0.3 * rng.standard_normal(w[k].shape)).astype(np.float32)
        elif k.endswith("LayerNorm.bias"):
            w[k] = (0.2 * rng.standard_normal(w[k].shape)).astype(np.float32)
    w["classifier.out_proj.weight"] *= 20.0
    enc = Encoder(spec, weights=w)
    # nb > 256: the single-read kernel's persistent workgroups take several sequences each
    ids, mask = _batch(spec, nb, S, seed=7 + S, ragged=True)
    got = enc.cross_score(ids, mask)[:, 0]
    # S <= 128 takes the single-read kernel (u once from HBM, z' on MFMA); the two-pass form too
    monkeypatch.setenv("SR_CLS_FOLD_1READ", "0")
    two = enc.cross_score(ids, mask)[:, 0]
    monkeypatch.delenv("SR_CLS_FOLD_1READ")
    monkeypatch.setenv("SR_KVFREE_CLS", "0")
    kv = enc.cross_score(ids, mask)[:, 0]
    ref = R.cross_logits(_ref_cfg(spec), w, ids, mask)[:, 0]
    tol = 1e-2 * (1.0 + np.abs(ref).max())
    assert np.abs(got - ref).max() <= tol
    assert np.abs(two - ref).max() <= tol
    assert np.abs(kv - ref).max() <= tol
    # single-read vs two-pass: z' in fp32 either way (MFMA with p' as fp16 hi + lo vs VALU)
    assert np.abs(got - two).max() <= 2e-3 * (1.0 + np.abs(ref).max())
    # the two paths differ only by where fp16 rounding happens (K / V vs w / z')
    assert np.abs(got - kv).max() <= tol
    assert not np.array_equal(got, kv)
