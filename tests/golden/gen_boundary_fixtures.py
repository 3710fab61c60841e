"""Capture boundary fixtures from the REAL reference code (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_boundary_fixtures.py

Imports the reference's own modules from /root/reference with stubbed third-party / infra modules
(SURVEY.md Appendix A): litellm (remote embed / rerank), pyseekdb (remote HNSW store), config,
DB access.  The stubs are deterministic backends (a hash embedding, a length-based relevance, an
exact cosine "SeekDB"), so the recorded behaviour is the reference's own host-side logic:
text cleaning and batching, order restoration, error types, rerank reorder-only semantics,
connector conversion (score = distance, ids dropped), merge dedupe, rerank fallback order and the
vector_search runner's tagging.  Output: tests/golden/boundary_fixtures.json (data only).
The fixture file is what travels; /root/reference never does.
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import os
import sys
import types

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "boundary_fixtures.json")
DIM = 8


def hash_vec(text: str):
    h = hashlib.sha256(text.encode("utf-8")).digest()
    return [round((b - 128) / 128.0, 6) for b in h[:DIM]]


def relevance(query: str, text: str) -> float:
    # deterministic stand-in for the remote cross-encoder: shared characters, then shorter first
    return len(set(query) & set(text)) - 0.001 * len(text)


class Recorder:
    embed_calls = []
    rerank_calls = []
    query_calls = []


def install_stubs():
    sys.path.insert(0, REF)
    litellm = types.ModuleType("litellm")

    def embedding(**kw):
        Recorder.embed_calls.append({k: v for k, v in kw.items() if k != "api_key"})
        return {"data": [{"embedding": hash_vec(t)} for t in kw["input"]]}

    async def arerank(**kw):
        Recorder.rerank_calls.append({k: v for k, v in kw.items() if k != "api_key"})
        scored = sorted(range(len(kw["documents"])),
                        key=lambda i: (-relevance(kw["query"], kw["documents"][i]), i))
        return {"results": [{"index": i, "relevance_score": relevance(kw["query"], kw["documents"][i])}
                            for i in scored]}

    litellm.embedding = embedding
    litellm.arerank = arerank
    litellm.BaseModel = object
    sys.modules["litellm"] = litellm

    import numpy as np

    class Coll:
        def __init__(self):
            self.rows = {}

        def add(self, ids, embeddings=None, metadatas=None, documents=None):
            for i, e, m, d in zip(ids, embeddings, metadatas, documents):
                self.rows[i] = (np.asarray(e, float), m, d)

        def delete(self, ids):
            for i in ids:
                self.rows.pop(i, None)

        def query(self, query_embeddings, query_texts, n_results):
            Recorder.query_calls.append({"query_texts": query_texts, "n_results": n_results,
                                         "dim": len(query_embeddings)})
            q = np.asarray(query_embeddings, float)
            q = q / np.linalg.norm(q)
            items = []
            for rid, (e, m, d) in self.rows.items():
                items.append((1.0 - float(q @ (e / np.linalg.norm(e))), rid, m, d))
            items.sort(key=lambda t: (t[0], t[1]))
            items = items[:n_results]
            return {"ids": [[t[1] for t in items]], "distances": [[t[0] for t in items]],
                    "documents": [[t[3] for t in items]], "metadatas": [[t[2] for t in items]]}

    class Client:
        colls = {}

        def __init__(self, **kw):
            pass

        def create_collection(self, name, configuration=None, embedding_function=None):
            Client.colls[name] = Coll()

        def get_or_create_collection(self, name):
            return Client.colls.setdefault(name, Coll())

        def delete_collection(self, name):
            Client.colls.pop(name, None)

    class EF:
        def __class_getitem__(cls, item):
            return cls

    pyseekdb = types.ModuleType("pyseekdb")
    pyseekdb.Client = Client
    pyseekdb.HNSWConfiguration = lambda **kw: kw
    pyseekdb.EmbeddingFunction = EF
    sys.modules["pyseekdb"] = pyseekdb

    def pkg(name, path=None):
        m = types.ModuleType(name)
        m.__path__ = [path] if path else []
        sys.modules[name] = m
        return m

    pkg("super_rag", os.path.join(REF, "super_rag"))
    for sub in ("llm", "llm/embed", "llm/rerank", "nodeflow/runners"):
        pkg("super_rag." + sub.replace("/", "."), os.path.join(REF, "super_rag", sub))
    cfg = types.ModuleType("super_rag.config")
    cfg.settings = types.SimpleNamespace(vector_db_type="seekdb", vector_db_context="{}",
                                         embedding_max_chunks_in_batch=10, chunk_size=400,
                                         chunk_overlap_size=20)
    sys.modules["super_rag.config"] = cfg
    pkg("super_rag.db")
    dbm = types.ModuleType("super_rag.db.models")
    dbm.Collection = object
    dbm.APIType = types.SimpleNamespace(EMBEDDING=types.SimpleNamespace(value="embedding"))
    sys.modules["super_rag.db.models"] = dbm
    ops = types.ModuleType("super_rag.db.ops")

    class AsyncOps:
        collections = {}

        async def query_collection(self, user, cid):
            return AsyncOps.collections.get(cid)

        async def query_provider_api_key(self, *a):
            return "key"

        async def query_llm_provider_by_name(self, name):
            return types.SimpleNamespace(base_url="http://stub")

    class SyncOps:
        def query_provider_api_key(self, *a):
            return "key"

        def query_llm_provider_by_name(self, name):
            return types.SimpleNamespace(base_url="http://stub")

        def query_llm_provider_model(self, *a):
            return None

    ops.async_db_ops = AsyncOps()
    ops.db_ops = SyncOps()
    sys.modules["super_rag.db.ops"] = ops
    hist = types.ModuleType("super_rag.utils.history")
    hist.BaseChatMessageHistory = object
    sys.modules["super_rag.utils.history"] = hist
    su = types.ModuleType("super_rag.schema.utils")

    def parseCollectionConfig(c):
        d = json.loads(c) if isinstance(c, str) else c
        e = d["embedding"]
        return types.SimpleNamespace(embedding=types.SimpleNamespace(
            model_service_provider=e.get("model_service_provider"), model=e.get("model"),
            custom_llm_provider=e.get("custom_llm_provider")))

    su.parseCollectionConfig = parseCollectionConfig
    pkg("super_rag.schema")
    sys.modules["super_rag.schema.utils"] = su
    return AsyncOps


def dump_docs(docs):
    return [{"text": d.text, "score": d.score, "metadata": d.metadata} for d in docs]


def err_name(fn):
    try:
        fn()
    except Exception as e:  # noqa: BLE001
        return type(e).__name__
    return None


def main():
    AsyncOps = install_stubs()
    from super_rag.llm.embed.embedding_service import EmbeddingService
    from super_rag.llm.rerank.rerank_service import RerankService
    from super_rag.models import DocumentWithScore, QueryWithEmbedding, TextNode
    from super_rag.nodeflow.base.models import SystemInput
    from super_rag.nodeflow.runners.merge import MergeInput, MergeNodeRunner
    from super_rag.nodeflow.runners.rerank import RerankInput, RerankNodeRunner
    from super_rag.vectorstore.seekdb_connector import SeekDBVectorStoreConnector

    fx = {"dim": DIM}
    # ---- embedder: cleaning, batching, order ----
    svc = EmbeddingService("openai", "BAAI/bge-m3", "http://stub", "k", 3)
    texts = ["a\nb", "", "ccc", "dd\n\ndd", "  ", "e"]
    Recorder.embed_calls.clear()
    out = svc.embed_documents(texts)
    fx["embed_documents"] = {
        "max_chunks": 3, "input": texts, "output": out,
        "batches_sent": sorted([c["input"] for c in Recorder.embed_calls]),
        "call_kwargs": sorted(set(k for c in Recorder.embed_calls for k in c)),
    }
    fx["embed_query"] = {"input": "hello\nworld", "output": svc.embed_query("hello\nworld")}
    fx["embed_errors"] = {
        "empty_list": err_name(lambda: svc.embed_documents([])),
        "all_empty": err_name(lambda: svc.embed_documents(["", "  "])),
        "blank_query": err_name(lambda: svc.embed_query("   ")),
    }

    # ---- reranker: reorder-only, placeholders, limits ----
    rr = RerankService("jina_ai", "BAAI/bge-reranker-v2-m3", "http://stub", "k")
    docs = [DocumentWithScore(text=t, score=s, metadata={"i": i})
            for i, (t, s) in enumerate([("apple pie", 0.3), ("", 0.1), ("banana split", 0.2),
                                        ("cherry", 0.4), ("apple", 0.25)])]
    Recorder.rerank_calls.clear()
    got = asyncio.run(rr.async_rerank("apple tart", docs))
    fx["rerank"] = {"query": "apple tart",
                    "docs": dump_docs(docs),
                    "documents_sent": Recorder.rerank_calls[0]["documents"],
                    "return_documents": Recorder.rerank_calls[0]["return_documents"],
                    "output": dump_docs(got)}

    def arun(coro_fn):
        return lambda: asyncio.run(coro_fn())

    fx["rerank_errors"] = {
        "empty_query": err_name(arun(lambda: rr.async_rerank(" ", docs))),
        "all_invalid": err_name(arun(lambda: rr.async_rerank("q", [DocumentWithScore(text="")]))),
        "too_many": err_name(arun(lambda: rr.async_rerank(
            "q", [DocumentWithScore(text="x")] * 1001))),
        "empty_docs_result": asyncio.run(rr.async_rerank("q", [])),
    }

    # ---- SeekDB connector: add -> search conversion ----
    con = SeekDBVectorStoreConnector({"collection": "c1"})
    con.create_collection(vector_size=DIM)
    corpus = ["alpha", "beta", "gamma", "delta", "epsilon", "zeta", "eta"]
    nodes = [TextNode(text=t, metadata={"n": i, "source": f"s{i}"}, embedding=hash_vec(t))
             for i, t in enumerate(corpus)]
    ids = con.store.add(nodes)
    q = QueryWithEmbedding(query="alphabet", top_k=4, embedding=hash_vec("alphabet"))
    Recorder.query_calls.clear()
    res = con.search(q, collection_name="c1", query_vector=q.embedding, with_vectors=True, limit=4,
                     consistency="majority", search_params={"hnsw_ef": 128, "exact": False},
                     score_threshold=0.9, filter={"chat_id": "x"})
    fx["connector"] = {
        "corpus": corpus, "metadatas": [n.metadata for n in nodes],
        "embeddings": [n.embedding for n in nodes],
        "ids_are_uuid4": all(len(i) == 36 and i[14] == "4" for i in ids),
        "query": {"query": q.query, "top_k": q.top_k, "embedding": q.embedding},
        "query_call": Recorder.query_calls[0],
        "result_query": res.query,
        "results": dump_docs(res.results),
        "result_fields": sorted(res.results[0].model_dump().keys()),
        "delete_without_ids": err_name(lambda: con.delete()),
    }
    con.delete(ids=ids[:2])
    res2 = con.search(q)
    fx["connector"]["after_delete_first_two"] = dump_docs(res2.results)

    # ---- merge + rerank fallback ----
    a = [DocumentWithScore(text="x", score=0.2, metadata={"recall_type": "vector_search"}),
         DocumentWithScore(text="y", score=0.5, metadata={"recall_type": "vector_search"})]
    g = [DocumentWithScore(text="g", score=None, metadata={"recall_type": "graph_search"}),
         DocumentWithScore(text="x", score=0.9, metadata={"recall_type": "graph_search"})]
    merged, _ = asyncio.run(MergeNodeRunner().run(
        MergeInput(vector_search_docs=a, graph_search_docs=g), SystemInput(query="q", user="u")))
    fx["merge"] = {"vector": dump_docs(a), "graph": dump_docs(g), "output": dump_docs(merged.docs)}
    fb_in = [DocumentWithScore(text="p", score=0.1, metadata={"recall_type": "vector_search"}),
             DocumentWithScore(text="g", score=0.0, metadata={"recall_type": "graph_search"}),
             DocumentWithScore(text="r", score=0.7, metadata={"recall_type": "vector_search"}),
             DocumentWithScore(text="s", score=None, metadata={})]
    fb, _ = asyncio.run(RerankNodeRunner().run(RerankInput(use_rerank_service=False, docs=fb_in),
                                               SystemInput(query="q", user="u")))
    fb2, _ = asyncio.run(RerankNodeRunner().run(RerankInput(docs=fb_in, model=None),
                                                SystemInput(query="q", user="u")))
    fx["rerank_fallback"] = {"input": dump_docs(fb_in), "disabled": dump_docs(fb.docs),
                             "unconfigured": dump_docs(fb2.docs)}

    with open(OUT, "w", encoding="utf-8") as f:
        json.dump(fx, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
