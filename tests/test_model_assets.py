"""CPU: model assets for the product path — no silent synthetic fallback.

A deployment points SUPER_RAG_AMD_WEIGHTS at Hugging Face model directories.  Missing weights or
tokenizer files must raise (and surface as EmbeddingError from the collection factory, as the
reference's base_embedding.py:114-121 / :203-215 do for any creation failure); seeded random weights
and the hashing tokenizer need the explicit SUPER_RAG_AMD_SYNTHETIC opt-in.  A model directory's
config.json / tokenizer.json / 1_Pooling define the ModelSpec of models outside MODELS.
"""
import numpy as np
import pytest

from model_dirs import WORDS, write_model_dir


@pytest.fixture
def product_env(monkeypatch, tmp_path):
    monkeypatch.delenv("SUPER_RAG_AMD_SYNTHETIC", raising=False)
    monkeypatch.setenv("SUPER_RAG_AMD_WEIGHTS", str(tmp_path))
    return tmp_path


def test_missing_checkpoint_and_tokenizer_raise(product_env, monkeypatch):
    from super_rag_amd.encoder import MODELS, ModelAssetsError, model_weights
    from super_rag_amd.tokenizer import Tokenizer
    spec = MODELS["bge-base-en"]
    with pytest.raises(ModelAssetsError, match="bge-base-en/model.safetensors"):
        model_weights(spec)
    with pytest.raises(ModelAssetsError, match="bge-base-en/tokenizer.json"):
        Tokenizer(spec)
    monkeypatch.delenv("SUPER_RAG_AMD_WEIGHTS")
    with pytest.raises(ModelAssetsError, match="SUPER_RAG_AMD_SYNTHETIC"):
        model_weights(spec)
    with pytest.raises(ModelAssetsError, match="SUPER_RAG_AMD_SYNTHETIC"):
        Tokenizer(spec)
    # the explicit opt-in (tests / benchmarks only)
    monkeypatch.setenv("SUPER_RAG_AMD_SYNTHETIC", "1")
    w = model_weights(MODELS["bge-small-en"])
    assert w["embeddings.word_embeddings.weight"].shape == (30522, 384)
    assert Tokenizer(spec).synthetic


def test_explicit_root_wins_over_the_synthetic_opt_in(product_env, monkeypatch):
    from super_rag_amd.encoder import MODELS, ModelAssetsError, model_weights
    monkeypatch.setenv("SUPER_RAG_AMD_SYNTHETIC", "1")
    with pytest.raises(ModelAssetsError):
        model_weights(MODELS["bge-base-en"])   # root set, file missing: misconfiguration


def test_factory_maps_missing_assets_to_embedding_error(product_env):
    from super_rag_amd.embed import get_collection_embedding_service_sync
    from super_rag_amd.errors import EmbeddingError
    from super_rag_amd.nodeflow_pack import LocalCollection
    with pytest.raises(EmbeddingError, match="Failed to create embedding model"):
        get_collection_embedding_service_sync(LocalCollection("c", {"embedding": {"model": "BAAI/bge-m3"}}))
    with pytest.raises(EmbeddingError):
        get_collection_embedding_service_sync(LocalCollection("c", {"embedding": {"model": "nope-7b"}}))


def test_model_directory_defines_spec_weights_and_tokenizer(product_env):
    from super_rag_amd.encoder import model_weights, resolve_spec
    from super_rag_amd.tokenizer import Tokenizer
    write_model_dir(str(product_env), "tiny-embed", "bert", pool="mean", seed=3)
    write_model_dir(str(product_env), "tiny-rerank", "xlmr", classifier=True, seed=4)
    e = resolve_spec("local/tiny-embed")
    assert (e.arch, e.hidden, e.layers, e.pool, e.bos_id, e.eos_id, e.pad_id) == \
        ("bert", 128, 2, "mean", 2, 3, 0)
    r = resolve_spec("tiny-rerank")
    assert (r.arch, r.classifier, r.num_labels, r.position_offset, r.bos_id, r.eos_id, r.pad_id,
            r.max_length, r.residual_fp16) == ("xlmr", 1, 1, 1, 0, 2, 1, 128, True)
    w = model_weights(e)
    assert "encoder.layer.1.output.dense.weight" in w and "pooler.dense.weight" not in w
    assert model_weights(r)["classifier.out_proj.weight"].shape == (1, 128)
    # the real vocabulary: [CLS] ... [SEP] from WordPiece, <s> ... </s></s> ... </s> pairs
    te, tr = Tokenizer(e), Tokenizer(r)
    assert not te.synthetic and not tr.synthetic
    ids, mask = te.encode_batch(["Vector search", "the banana"])
    v = {w: i + 4 for i, w in enumerate(WORDS)}
    assert ids[0].tolist() == [2, v["vector"], v["search"], 3]
    assert mask.tolist() == [[1, 1, 1, 1], [1, 1, 1, 1]]
    pid, pm, _ = tr.encode_pairs("apple", ["banana split", ""])
    assert pid[0, 0] == 0 and pid[0].tolist().count(2) == 3 and pm[1].sum() == 5


def test_tokenizer_pairs_match_the_hf_post_processor(product_env):
    """Our packing of (query, passage) equals tokenizers' own pair encoding with longest_first
    truncation (the behaviour of the cross-encoder tokenizer call)."""
    from tokenizers import Tokenizer as HF

    from super_rag_amd.encoder import resolve_spec
    from super_rag_amd.tokenizer import Tokenizer
    d = write_model_dir(str(product_env), "tiny-rerank", "xlmr", classifier=True, max_pos=34)
    spec = resolve_spec("tiny-rerank")
    ours = Tokenizer(spec)
    hf = HF.from_file(d + "/tokenizer.json")
    hf.enable_truncation(spec.max_length, strategy="longest_first")
    rng = np.random.default_rng(0)
    for _ in range(25):
        q = " ".join(rng.choice(WORDS, rng.integers(1, 12)))
        p = " ".join(rng.choice(WORDS, rng.integers(1, 40)))
        ids, mask, _ = ours.encode_pairs(q, [p])
        assert ids[0][mask[0] == 1].tolist() == hf.encode(q, p).ids


def test_hf_directory_names_keep_case_and_version_suffix(product_env):
    """"BAAI/bge-base-en-v1.5" and "Local/Tiny-Embed-v1.5": spec, checkpoint and tokenizer all come
    from the directory named as the model is named (the spec key is lowercased and
    suffix-stripped, the directory is not)."""
    from super_rag_amd.encoder import MODELS, find_checkpoint, model_weights, resolve_spec
    from super_rag_amd.tokenizer import Tokenizer
    d = write_model_dir(str(product_env), "Tiny-Embed-v1.5", "bert", seed=5)
    e = resolve_spec("Local/Tiny-Embed-v1.5")
    assert e.name == "tiny-embed" and e.source_dir == d and e.hidden == 128
    assert find_checkpoint(e) == d + "/model.safetensors"
    assert "encoder.layer.1.output.dense.weight" in model_weights(e)
    assert not Tokenizer(e).synthetic
    # a built-in shape whose Hugging Face directory carries the version suffix
    import os
    import shutil
    hf_dir = os.path.join(str(product_env), "bge-base-en-v1.5")
    os.makedirs(hf_dir)
    shutil.copy(d + "/tokenizer.json", hf_dir)
    b = resolve_spec("BAAI/bge-base-en-v1.5")
    assert b == MODELS["bge-base-en"] and b.source_dir == hf_dir
    assert Tokenizer(b)._hf is not None
    from super_rag_amd.encoder import ModelAssetsError
    with pytest.raises(ModelAssetsError, match="bge-base-en-v1.5/model.safetensors"):
        find_checkpoint(b)
