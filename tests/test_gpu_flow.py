"""GPU: the reference's search flow end to end on the HIP path, with real model assets.

Built as CollectionService.execute_search_flow builds it (super_rag/service/collection_service.py:
255-346) through super_rag_amd.flow: the pack's vector_search -> merge -> rerank runners
(nodeflow/runners/vector_search.py:52-135, merge.py:40-65, rerank.py:59-202), the collection's
embedder from the real, unpatched get_collection_embedding_service_sync (llm/embed/
base_embedding.py:122-215) and the reranker from the registry — both loaded from Hugging Face model
directories written offline (config.json + model.safetensors + tokenizer.json, tests/model_dirs.py),
no synthetic opt-in.  Ingest goes through VectorIndexer.create_index (index/
vector_and_full_text_index.py:29-129).  Every stage is checked against the oracle run on the token
ids the model's own `tokenizers` pipeline produces (post-processor specials, longest_first pairs).
"""
import asyncio
import os
from types import SimpleNamespace

import numpy as np
import pytest

from model_dirs import WORDS, ref_config, write_model_dir
from oracle import encoder_ref as R
from oracle.cosine_topk import cosine_topk, same_topk_modulo_ties

pytestmark = pytest.mark.gpu


def _texts(n, seed, lo=4, hi=30):
    rng = np.random.default_rng(seed)
    return [" ".join(rng.choice(WORDS, rng.integers(lo, hi))) for _ in range(n)]


def _hf_batch(tok, texts):
    enc = [tok.encode(t).ids for t in texts]
    S = max(len(e) for e in enc)
    ids = np.zeros((len(enc), S), np.int64)
    mask = np.zeros((len(enc), S), np.int64)
    for i, e in enumerate(enc):
        ids[i, :len(e)] = e
        mask[i, :len(e)] = 1
    return ids, mask


@pytest.fixture
def deployment(tmp_path, monkeypatch):
    from super_rag_amd import registry
    from super_rag_amd import vectorstore as V
    write_model_dir(str(tmp_path), "tiny-embed", "bert", hidden=128, layers=2, heads=2, inter=256,
                    max_pos=130, seed=5)
    write_model_dir(str(tmp_path), "tiny-rerank", "xlmr", classifier=True, hidden=128, layers=2,
                    heads=2, inter=256, max_pos=130, seed=6, head_scale=50.0)
    monkeypatch.setenv("SUPER_RAG_AMD_WEIGHTS", str(tmp_path))
    monkeypatch.delenv("SUPER_RAG_AMD_SYNTHETIC", raising=False)
    registry.clear()
    V._collections.clear()
    yield tmp_path
    registry.clear()
    V._collections.clear()


def test_search_flow_matches_the_oracle(deployment):
    from tokenizers import Tokenizer as HF

    from super_rag_amd import nodeflow_pack as P
    from super_rag_amd.embed import get_collection_embedding_service_sync
    from super_rag_amd.encoder import load_safetensors, resolve_spec
    from super_rag_amd.flow import execute_search_flow
    from super_rag_amd.index import VectorIndexer
    from super_rag_amd.vectorstore import VectorStoreConnectorAdaptor

    P.register()
    col = P.LocalCollection("colA", {"embedding": {"model": "BAAI/tiny-embed",
                                                   "model_service_provider": "local",
                                                   "custom_llm_provider": "mi355x"}})
    P.register_collection(col)
    svc, dim = get_collection_embedding_service_sync(col)          # real factory, real assets
    assert dim == 128 and not svc.tokenizer.synthetic
    con = VectorStoreConnectorAdaptor("mi355x", {"collection": P.collection_name_for("colA")}).connector
    con.create_collection(vector_size=dim)
    texts = _texts(80, 1)
    parts = [SimpleNamespace(content=t, metadata={"name": f"doc{i}.md"}) for i, t in enumerate(texts)]
    ids = VectorIndexer(con, svc).create_index(parts)["context_ids"]
    assert len(ids) == 80

    query = "vector search over the river and the mountain"
    items, node = asyncio.run(execute_search_flow(
        query, "colA", "u1", vector_topk=10, rerank_config=("tiny-rerank", "local", "mi355x")))
    assert node == "rerank" and [it.rank for it in items] == list(range(1, 11))
    assert all(it.recall_type == "vector_search" for it in items)
    assert {it.source for it in items} <= {f"doc{i}.md" for i in range(80)}

    # ---- oracle: embeddings of the chunks and the query from the model's own tokenizer ----------
    d = str(deployment)
    espec, rspec = resolve_spec("tiny-embed"), resolve_spec("tiny-rerank")
    we = load_safetensors(os.path.join(d, "tiny-embed", "model.safetensors"))
    wr = load_safetensors(os.path.join(d, "tiny-rerank", "model.safetensors"))
    etok = HF.from_file(os.path.join(d, "tiny-embed", "tokenizer.json"))
    corpus = R.embed(ref_config(espec), we, *_hf_batch(etok, texts))
    qv = R.embed(ref_config(espec), we, *_hf_batch(etok, [query]))
    dist, rows = cosine_topk(corpus, qv, 10)
    got_rows = np.array([[texts.index(it.content) for it in items]])
    got_dist = {texts.index(it.content): it.score for it in items}
    # the candidate set is the oracle's top-10 (modulo near-ties of the fp16 store)
    assert same_topk_modulo_ties(got_rows, 1.0 - np.array([[got_dist[r] for r in got_rows[0]]]),
                                 rows, 1.0 - dist, 2e-3)
    all_d, all_r = cosine_topk(corpus, qv, 80)
    ref_d = dict(zip(all_r[0].tolist(), all_d[0].tolist()))
    for r, s in got_dist.items():     # score = cosine distance (seekdb_connector.py:143)
        assert abs(s - ref_d[r]) < 2e-3

    # ---- oracle: rerank order = logits of (query, passage) pairs, longest_first truncation ----
    rtok = HF.from_file(os.path.join(d, "tiny-rerank", "tokenizer.json"))
    rtok.enable_truncation(rspec.max_length, strategy="longest_first")
    pair_ids, pair_mask = [], []
    for it in items:
        e = rtok.encode(query, it.content).ids
        pair_ids.append(e)
    S = max(len(e) for e in pair_ids)
    pi = np.full((len(items), S), rspec.pad_id, np.int64)
    pm = np.zeros((len(items), S), np.int64)
    for i, e in enumerate(pair_ids):
        pi[i, :len(e)], pm[i, :len(e)] = e, 1
    lg = R.cross_logits(ref_config(rspec), wr, pi, pm)[:, 0]
    tol = 2e-3 * (1 + np.abs(lg).max())
    assert np.all(lg[:-1] >= lg[1:] - tol), lg       # items come out in oracle-logit order
    # rerank reorders only: the vector-search distances are kept
    assert sorted(got_dist.values()) == sorted(it.score for it in items)


def test_search_flow_fallbacks_and_degrade(deployment):
    from super_rag_amd import nodeflow_pack as P
    from super_rag_amd.embed import get_collection_embedding_service_sync
    from super_rag_amd.flow import execute_search_flow
    from super_rag_amd.index import VectorIndexer
    from super_rag_amd.vectorstore import VectorStoreConnectorAdaptor
    P.register()
    col = P.LocalCollection("colB", {"embedding": {"model": "tiny-embed"}})
    P.register_collection(col)
    svc, dim = get_collection_embedding_service_sync(col)
    con = VectorStoreConnectorAdaptor("mi355x", {"collection": "colB"}).connector
    texts = _texts(30, 2)
    VectorIndexer(con, svc).create_index([SimpleNamespace(content=t, metadata={}) for t in texts])
    # rerank off: the reference's fallback order, score (= distance) descending (rerank.py:193)
    items, _ = asyncio.run(execute_search_flow("apple banana", "colB", "u", vector_topk=6, rerank=False))
    assert len(items) == 6
    assert [it.score for it in items] == sorted((it.score for it in items), reverse=True)
    # no default rerank model configured: same fallback
    items2, _ = asyncio.run(execute_search_flow("apple banana", "colB", "u", vector_topk=6))
    assert [it.content for it in items2] == [it.content for it in items]
    # an unknown reranker (no model directory): the service fails, the node falls back
    items3, _ = asyncio.run(execute_search_flow("apple banana", "colB", "u", vector_topk=6,
                                                rerank_config=("no-such-reranker", "p", "c")))
    assert [it.content for it in items3] == [it.content for it in items]
    # a collection whose embedding model has no assets: vector_search degrades to []
    P.register_collection(P.LocalCollection("colC", {"embedding": {"model": "BAAI/bge-m3"}}))
    items4, _ = asyncio.run(execute_search_flow("apple", "colC", "u", vector_topk=6))
    assert items4 == []
