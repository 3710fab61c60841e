"""CPU: pinning the oracle (oracle/*) before it is trusted as the GPU parity checker.

* encoder_ref is checked against Hugging Face transformers (BertModel, XLMRobertaModel,
  XLMRobertaForSequenceClassification) on identical seeded weights — the public implementations
  of the remote models the reference calls (BAAI/bge-*, BAAI/bge-reranker-*);
* pack_pairs is checked against a tokenizers/transformers fast tokenizer with the BERT and
  RoBERTa pair post-processors and 'longest_first' truncation;
* cosine_topk is checked against an independent brute-force sort (ties, zero rows, tombstones),
  plus the committed regression vectors tests/golden/oracle_vectors.npz.
"""
import os

import numpy as np
import pytest
import torch

from oracle import encoder_ref as R
from oracle.cosine_topk import (cosine_topk, quantize_like_store, recall_at_k,
                                same_topk_modulo_ties)

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _weights(cfg, seed):
    from super_rag_amd.encoder import ModelSpec, random_weights
    arch = "xlmr" if cfg.position_offset else "bert"
    spec = ModelSpec("t", arch, cfg.vocab_size, cfg.hidden, cfg.layers, cfg.heads, cfg.intermediate,
                     cfg.max_position, cfg.type_vocab, cfg.ln_eps, cfg.position_offset,
                     classifier=cfg.classifier, num_labels=cfg.num_labels)
    return random_weights(spec, seed, "test")


def _load(model, w, prefix):
    sd = {prefix + k: torch.from_numpy(v) for k, v in w.items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all("pooler" in m or "position_ids" in m for m in missing), missing


def test_encoder_ref_matches_transformers_bert():
    from transformers import BertConfig, BertModel
    cfg = R.RefConfig(500, 64, 2, 2, 128, 40, 2, 1e-12)
    w = _weights(cfg, 1)
    hf = BertModel(BertConfig(vocab_size=500, hidden_size=64, num_hidden_layers=2,
                              num_attention_heads=2, intermediate_size=128,
                              max_position_embeddings=40, type_vocab_size=2,
                              layer_norm_eps=1e-12, hidden_act="gelu",
                              attn_implementation="eager"), add_pooling_layer=False).eval()
    _load(hf, w, "")
    rng = np.random.default_rng(0)
    ids = rng.integers(3, 500, (3, 11))
    mask = np.ones_like(ids)
    mask[1, 7:] = 0
    tt = np.zeros_like(ids)
    tt[:, 5:] = 1
    ref = R.encode_hidden(cfg, w, ids, mask, tt).numpy()
    with torch.no_grad():
        got = hf(input_ids=torch.from_numpy(ids), attention_mask=torch.from_numpy(mask),
                 token_type_ids=torch.from_numpy(tt)).last_hidden_state.numpy()
    np.testing.assert_allclose(ref[mask == 1], got[mask == 1], atol=2e-5)


def test_encoder_ref_matches_transformers_xlmr_classifier():
    from transformers import XLMRobertaConfig, XLMRobertaForSequenceClassification
    cfg = R.RefConfig(500, 64, 2, 2, 128, 40, 1, 1e-5, position_offset=1, classifier=1)
    w = _weights(cfg, 2)
    hf = XLMRobertaForSequenceClassification(XLMRobertaConfig(
        vocab_size=500, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
        intermediate_size=128, max_position_embeddings=40, type_vocab_size=1, layer_norm_eps=1e-5,
        pad_token_id=1, num_labels=1, attn_implementation="eager")).eval()
    sd = {("classifier." + k[len("classifier."):] if k.startswith("classifier.") else "roberta." + k): v
          for k, v in w.items()}
    _load(hf, sd, "")
    rng = np.random.default_rng(1)
    ids = rng.integers(3, 500, (4, 9))
    ids[:, 0] = 0
    mask = np.ones_like(ids)
    ids[2, 6:] = 1   # padding (XLM-R positions skip pads)
    mask[2, 6:] = 0
    ref = R.cross_logits(cfg, w, ids, mask)
    with torch.no_grad():
        got = hf(input_ids=torch.from_numpy(ids), attention_mask=torch.from_numpy(mask)).logits.numpy()
    np.testing.assert_allclose(ref, got, atol=2e-5)


def _fast_tokenizer(style):
    from tokenizers import Tokenizer, models, pre_tokenizers, processors
    from transformers import PreTrainedTokenizerFast
    vocab = {w: i for i, w in enumerate(["[PAD]", "[CLS]", "[SEP]", "<s>", "</s>", "<pad>"]
                                        + [f"w{i}" for i in range(60)])}
    tk = Tokenizer(models.WordLevel(vocab, unk_token="[PAD]"))
    tk.pre_tokenizer = pre_tokenizers.Whitespace()
    if style == 1:
        tk.post_processor = processors.TemplateProcessing(
            single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
            special_tokens=[("[CLS]", 1), ("[SEP]", 2)])
        return PreTrainedTokenizerFast(tokenizer_object=tk, pad_token="[PAD]"), vocab, 1, 2, 0
    tk.post_processor = processors.RobertaProcessing(("</s>", 4), ("<s>", 3))
    return PreTrainedTokenizerFast(tokenizer_object=tk, pad_token="<pad>"), vocab, 3, 4, 5


@pytest.mark.parametrize("style", [0, 1])
def test_pack_pairs_matches_hf_pair_tokenisation(style):
    tok, vocab, bos, eos, pad = _fast_tokenizer(style)
    rng = np.random.default_rng(style)
    S = 16
    for trial in range(40):
        lq, lp = rng.integers(0, 14, 2)
        q = [f"w{i}" for i in rng.integers(0, 60, lq)]
        p = [f"w{i}" for i in rng.integers(0, 60, lp)]
        # an empty passage is sent as " " (rerank_service.py:61): a pair with no passage tokens
        enc = tok(" ".join(q) or " ", " ".join(p) or " ", truncation="longest_first", max_length=S,
                  padding="max_length", return_token_type_ids=True)
        q_tok = np.array([[vocab[w] for w in q] + [0] * (14 - lq)], np.int32)
        p_tok = np.array([[vocab[w] for w in p] + [0] * (14 - lp)], np.int32)
        ids, msk, typ = R.pack_pairs(q_tok, [lq], p_tok, [lp], np.array([[0]]), S, style, bos, eos, pad)
        assert ids[0].tolist() == enc["input_ids"], (q, p)
        assert msk[0].tolist() == enc["attention_mask"]
        if style == 1:
            assert typ[0].tolist() == enc["token_type_ids"]


def _brute(corpus, q, k, live=None):
    out = []
    for qq in q:
        qn = qq / np.linalg.norm(qq)
        items = []
        for r, x in enumerate(corpus):
            if live is not None and not live[r]:
                continue
            n = np.linalg.norm(x)
            s = float(qn @ x) / n if n > 0 else 0.0
            items.append((1.0 - s, r))
        items.sort()
        out.append(items[:k])
    return out


def test_cosine_topk_matches_bruteforce_with_ties_zeros_and_tombstones():
    rng = np.random.default_rng(3)
    c = rng.standard_normal((300, 6))
    c[10] = 0.0                    # zero row -> similarity 0
    c[20] = c[21] = c[22] = c[5]   # exact ties: ascending row order
    live = np.ones(300, bool)
    live[::7] = False
    q = rng.standard_normal((5, 6))
    q[0] = c[5]
    d, r = cosine_topk(c, q, 12, live=live, chunk=64)
    for b, items in enumerate(_brute(c, q, 12, live)):
        assert r[b].tolist() == [x[1] for x in items]
        np.testing.assert_allclose(d[b], [x[0] for x in items], atol=1e-12)
    assert r[0][:3].tolist() == [5, 20, 22]     # exact ties by row; row 21 is tombstoned
    d2, r2 = cosine_topk(c[:3], q, 5)
    assert (r2[:, 3:] == -1).all() and np.isinf(d2[:, 3:]).all()


def test_helpers():
    a = np.array([[1, 2, 3]])
    assert recall_at_k(a, np.array([[3, 4, 1]])) == pytest.approx(2 / 3)
    sims = np.array([[0.9, 0.5, 0.5]])
    assert same_topk_modulo_ties(np.array([[1, 2, 4]]), sims, np.array([[1, 2, 3]]), sims, 1e-6)
    assert not same_topk_modulo_ties(np.array([[1, 2, 4]]), np.array([[0.9, 0.5, 0.4]]),
                                     np.array([[1, 2, 3]]), np.array([[0.9, 0.5, 0.45]]), 1e-6)
    x = quantize_like_store(np.array([[3.0, 4.0], [0.0, 0.0]]))
    assert x.dtype == np.float16
    assert x[0].tolist() == np.array([0.6, 0.8], np.float16).tolist() and x[1].tolist() == [0, 0]


def test_oracle_regression_vectors():
    # tests/golden/gen_oracle_vectors.py writes these with the oracle; they pin future edits of it
    z = np.load(os.path.join(GOLDEN, "oracle_vectors.npz"))
    d, r = cosine_topk(z["corpus"], z["queries"], int(z["k"]))
    assert np.array_equal(r, z["rows"]) and np.allclose(d, z["dist"], atol=1e-12)
    cfg = R.RefConfig(*[int(v) if float(v).is_integer() else float(v) for v in z["cfg"]])
    w = {k[2:]: z[k] for k in z.files if k.startswith("w.")}
    e = R.embed(cfg, w, z["ids"], z["mask"])
    np.testing.assert_allclose(e, z["emb"], atol=1e-5)
