"""CPU: the drop-in boundary replayed against fixtures captured from the REAL reference code
(tests/golden/gen_boundary_fixtures.py -> boundary_fixtures.json).  GPU objects are replaced by
the doubles in tests/doubles.py so only the host-side semantics are compared: text cleaning,
order, error types, reorder-only rerank, connector conversion, merge and fallback order, and the
vector_search runner's tagging / degrade-to-[] behaviour."""
import asyncio
import json
import os

import numpy as np
import pytest

from doubles import HashEncoder, NumpyStore, RelevanceEncoder, TextTokenizer, hash_vec

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "boundary_fixtures.json")))


def _docs(rows):
    from super_rag_amd.models import DocumentWithScore
    return [DocumentWithScore(**r) for r in rows]


def _dump(docs):
    return [{"text": d.text, "score": d.score, "metadata": d.metadata} for d in docs]


@pytest.fixture
def numpy_store():
    from super_rag_amd import vectorstore
    vectorstore.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    vectorstore._collections.clear()
    yield
    vectorstore._collections.clear()
    vectorstore.set_store_backend(vectorstore._native_store, vectorstore._native_load)


def _embedder(max_chunks=3, device_batch=256):
    from super_rag_amd.embed import EmbeddingService
    tok = TextTokenizer()
    return EmbeddingService("openai", "BAAI/bge-m3", "http://x", "k", max_chunks,
                            encoder=HashEncoder(tok, FX["dim"]), tokenizer=tok,
                            device_batch=device_batch), tok


@pytest.mark.parametrize("device_batch", [1, 2, 256])
def test_embed_documents_matches_reference(device_batch):
    f = FX["embed_documents"]
    svc, tok = _embedder(f["max_chunks"], device_batch)
    out = svc.embed_documents(f["input"])
    np.testing.assert_allclose(np.asarray(out), np.asarray(f["output"]), atol=1e-6)
    # the cleaned texts are exactly what the reference sent to the remote embedder
    assert sorted(tok.seen) == sorted(t for b in f["batches_sent"] for t in b)
    q = FX["embed_query"]
    np.testing.assert_allclose(svc.embed_query(q["input"]), q["output"], atol=1e-6)


def test_embed_errors_match_reference():
    svc, _ = _embedder()
    errs = {}
    for key, fn in {"empty_list": lambda: svc.embed_documents([]),
                    "all_empty": lambda: svc.embed_documents(["", "  "]),
                    "blank_query": lambda: svc.embed_query("   ")}.items():
        with pytest.raises(Exception) as ei:
            fn()
        errs[key] = type(ei.value).__name__
    assert errs == FX["embed_errors"]


def _reranker():
    from super_rag_amd.rerank import RerankService
    tok = TextTokenizer()
    return RerankService("jina_ai", "BAAI/bge-reranker-v2-m3", "http://x", "k",
                         encoder=RelevanceEncoder(tok), tokenizer=tok), tok


def test_rerank_reorders_only_like_reference():
    f = FX["rerank"]
    svc, tok = _reranker()
    out = asyncio.run(svc.async_rerank(f["query"], _docs(f["docs"])))
    assert _dump(out) == f["output"]           # permutation with the ORIGINAL scores
    assert [p for _, p in tok.pairs] == f["documents_sent"]   # " " placeholder for empty docs
    assert svc.max_documents == 1000


def test_rerank_errors_match_reference():
    from super_rag_amd.models import DocumentWithScore
    svc, _ = _reranker()
    f = FX["rerank_errors"]
    cases = {"empty_query": lambda: svc.async_rerank(" ", _docs(FX["rerank"]["docs"])),
             "all_invalid": lambda: svc.async_rerank("q", [DocumentWithScore(text="")]),
             "too_many": lambda: svc.async_rerank("q", [DocumentWithScore(text="x")] * 1001)}
    for key, fn in cases.items():
        with pytest.raises(Exception) as ei:
            asyncio.run(fn())
        assert type(ei.value).__name__ == f[key], key
    assert asyncio.run(svc.async_rerank("q", [])) == f["empty_docs_result"]


def test_connector_matches_seekdb_conversion(numpy_store):
    from super_rag_amd.models import QueryWithEmbedding, TextNode
    from super_rag_amd.vectorstore import VectorStoreConnectorAdaptor
    f = FX["connector"]
    con = VectorStoreConnectorAdaptor("mi355x", {"collection": "c1"}).connector
    assert con.store is con and con.collection_name == "c1"
    con.create_collection(vector_size=FX["dim"])
    nodes = [TextNode(text=t, metadata=m, embedding=e)
             for t, m, e in zip(f["corpus"], f["metadatas"], f["embeddings"])]
    ids = con.store.add(nodes)
    assert all(len(i) == 36 and i[14] == "4" for i in ids) == f["ids_are_uuid4"]
    q = QueryWithEmbedding(**f["query"])
    res = con.search(q, collection_name="c1", query_vector=q.embedding, with_vectors=True, limit=4,
                     consistency="majority", search_params={"hnsw_ef": 128, "exact": False},
                     score_threshold=0.9, filter={"chat_id": "x"})
    assert res.query == f["result_query"]
    got = _dump(res.results)
    assert [g["text"] for g in got] == [r["text"] for r in f["results"]]
    assert [g["metadata"] for g in got] == [r["metadata"] for r in f["results"]]
    np.testing.assert_allclose([g["score"] for g in got], [r["score"] for r in f["results"]], atol=1e-9)
    assert sorted(res.results[0].model_dump().keys()) == f["result_fields"]   # no id field
    with pytest.raises(ValueError, match="ids is required"):
        con.delete()
    con.delete(ids=ids[:2])
    got2 = _dump(con.search(q).results)
    assert [g["text"] for g in got2] == [r["text"] for r in f["after_delete_first_two"]]
    # returned metadata is a copy: tagging it must not alter the stored row
    res.results[0].metadata["recall_type"] = "vector_search"
    assert "recall_type" not in _dump(con.search(q).results)[0]["metadata"]


def test_connector_snapshot_and_compaction(numpy_store, tmp_path):
    from super_rag_amd import vectorstore
    from super_rag_amd.models import QueryWithEmbedding, TextNode
    ctx = {"collection": "snap", "snapshot_dir": str(tmp_path)}
    con = vectorstore.MI355XVectorStoreConnector(ctx)
    texts = [f"doc {i}" for i in range(10)]
    ids = con.add([TextNode(text=t, metadata={"i": i}, embedding=hash_vec(t)) for i, t in enumerate(texts)])
    con.delete(ids=ids[:6])                      # > 50% tombstones -> compaction
    q = QueryWithEmbedding(query="doc 7", top_k=10, embedding=hash_vec("doc 7"))
    before = _dump(con.search(q).results)
    assert {d["text"] for d in before} == set(texts[6:])
    vectorstore._collections.clear()             # "restart": reload from the snapshot
    con2 = vectorstore.MI355XVectorStoreConnector(ctx)
    assert _dump(con2.search(q).results) == before
    con2.delete(ids=[ids[7]])
    assert "doc 7" not in {d["text"] for d in _dump(con2.search(q).results)}
    con2.delete_collection()
    assert not os.listdir(tmp_path)


def test_merge_and_rerank_fallback_match_reference():
    from super_rag_amd.nodeflow_pack import (MergeInput, MergeNodeRunner, RerankInput,
                                             RerankNodeRunner, SystemInput)
    f = FX["merge"]
    out, _ = asyncio.run(MergeNodeRunner().run(
        MergeInput(vector_search_docs=_docs(f["vector"]), graph_search_docs=_docs(f["graph"])),
        SystemInput(query="q", user="u")))
    assert _dump(out.docs) == f["output"]
    g = FX["rerank_fallback"]
    a, _ = asyncio.run(RerankNodeRunner().run(RerankInput(use_rerank_service=False, docs=_docs(g["input"])),
                                              SystemInput(query="q", user="u")))
    b, _ = asyncio.run(RerankNodeRunner().run(RerankInput(docs=_docs(g["input"]), model=None),
                                              SystemInput(query="q", user="u")))
    assert _dump(a.docs) == g["disabled"] and _dump(b.docs) == g["unconfigured"]


def test_vector_search_runner_end_to_end(numpy_store, monkeypatch):
    from super_rag_amd import embed as embed_mod
    from super_rag_amd import nodeflow_pack as P
    from super_rag_amd.models import TextNode
    from super_rag_amd.vectorstore import MI355XVectorStoreConnector
    svc, _ = _embedder()
    monkeypatch.setattr(embed_mod, "get_collection_embedding_service_sync", lambda c: (svc, 8))
    P.register()
    assert {"vector_search", "rerank", "merge"} <= set(P.NODE_RUNNER_REGISTRY)
    P.register_collection(P.LocalCollection("col1", {"embedding": {"model": "bge-m3"}}))
    texts = ["alpha", "beta", "gamma", "delta"]
    con = MI355XVectorStoreConnector({"collection": "col1"})
    con.add([TextNode(text=t, metadata={"k": i}, embedding=svc.embed_query(t)) for i, t in enumerate(texts)])
    runner = P.NODE_RUNNER_REGISTRY["vector_search"]["runner"]
    out, so = asyncio.run(runner.run(P.VectorSearchInput(top_k=2, collection_ids=["col1"]),
                                     P.SystemInput(query="gamma", user="u")))
    assert so == {} and len(out.docs) == 2
    assert out.docs[0].text == "gamma" and out.docs[0].score == pytest.approx(0.0, abs=1e-6)
    assert all(d.metadata["recall_type"] == "vector_search" for d in out.docs)
    # unknown collection / failing embedder degrade to [] like the reference
    out2, _ = asyncio.run(runner.run(P.VectorSearchInput(collection_ids=["nope"]),
                                     P.SystemInput(query="x", user="u")))
    assert out2.docs == []
    monkeypatch.setattr(embed_mod, "get_collection_embedding_service_sync",
                        lambda c: (_ for _ in ()).throw(RuntimeError("boom")))
    out3, _ = asyncio.run(runner.run(P.VectorSearchInput(collection_ids=["col1"]),
                                     P.SystemInput(query="x", user="u")))
    assert out3.docs == []


def test_rerank_runner_uses_service_then_falls_back(monkeypatch):
    from super_rag_amd import nodeflow_pack as P
    from super_rag_amd import rerank as rerank_mod
    svc, _ = _reranker()
    monkeypatch.setattr(rerank_mod.RerankService, "__init__",
                        lambda self, *a, **k: self.__dict__.update(svc.__dict__))
    f = FX["rerank"]
    ui = P.RerankInput(model="bge-reranker-v2-m3", model_service_provider="local",
                       custom_llm_provider="mi355x", docs=_docs(f["docs"]))
    out, _ = asyncio.run(P.RerankNodeRunner().run(ui, P.SystemInput(query=f["query"], user="u")))
    assert _dump(out.docs) == f["output"]
    ui_bad = P.RerankInput(model="x", model_service_provider="p", custom_llm_provider="c",
                           docs=_docs(FX["rerank_fallback"]["input"]))
    monkeypatch.setattr(rerank_mod.RerankService, "async_rerank",
                        lambda self, q, d: (_ for _ in ()).throw(RuntimeError("device lost")))
    out2, _ = asyncio.run(P.RerankNodeRunner().run(ui_bad, P.SystemInput(query="q", user="u")))
    assert _dump(out2.docs) == FX["rerank_fallback"]["disabled"]


def test_index_write_path(numpy_store):
    from types import SimpleNamespace
    from super_rag_amd.index import VectorIndexer, chunk_text
    from super_rag_amd.vectorstore import MI355XVectorStoreConnector
    part = SimpleNamespace(content="body", metadata={"titles": ["A", "B"], "name": "f.md",
                                                     "labels": [{"key": "k", "value": "v"}, {"key": "", "value": "x"}]})
    assert chunk_text(part) == "> Hierarchy: A > B\n> Labels: k=v\n\nbody"   # embedding_utils.py:55-80
    svc, tok = _embedder()
    con = MI355XVectorStoreConnector({"collection": "idx"})
    ix = VectorIndexer(con, svc)
    r = ix.create_index([part, SimpleNamespace(content="", metadata={})])
    assert len(r["context_ids"]) == 1 and tok.seen[-1] == chunk_text(part).replace("\n", " ")
    r2 = ix.update_index(r["context_ids"], [part, SimpleNamespace(content="two", metadata={})])
    assert len(r2["context_ids"]) == 2
    assert not set(r["context_ids"]) & set(r2["context_ids"])
    ix.delete_index(r2["context_ids"])
