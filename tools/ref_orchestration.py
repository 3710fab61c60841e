"""Per-query Python orchestration overhead of the REAL reference search flow (build container only;
BASELINE.md section 3 stage iv).

    PYTHONDONTWRITEBYTECODE=1 python tools/ref_orchestration.py [--queries 300] [--topk 100]

Imports the reference's NodeflowEngine and runners from /root/reference with the stub backends of
tests/golden/gen_boundary_fixtures.py, made constant-time: litellm.embedding returns a precomputed
768-d vector, SeekDB's collection.query a precomputed list of top-k hits, litellm.arerank a
precomputed order.  The flow is built exactly as CollectionService.execute_search_flow builds it
(super_rag/service/collection_service.py:255-346: vector_search -> merge -> rerank) and executed
with engine.execute_nodeflow; the wall time per query is then the reference's own host-side cost
around the three remote calls (object construction, the factory's DB lookups, connector
conversion, merge dedupe, reorder).  Writes profiles/r02_reference_orchestration.json; bench.py
reports it beside the CPU baseline (the GPU box has no /root/reference).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "r02_reference_orchestration.json")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=300)
    ap.add_argument("--topk", type=int, default=100)
    ap.add_argument("--dim", type=int, default=768)
    a = ap.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import gen_boundary_fixtures as G
    AsyncOps = G.install_stubs()
    import litellm
    import pyseekdb

    vec = [((i * 37) % 101 - 50) / 50.0 for i in range(a.dim)]
    hits = {"ids": [[f"id{i}" for i in range(a.topk)]],
            "distances": [[0.1 + i * 1e-3 for i in range(a.topk)]],
            "documents": [[f"passage {i} " * 20 for i in range(a.topk)]],
            "metadatas": [[{"source": f"doc{i}.md", "name": f"doc{i}.md"} for i in range(a.topk)]]}
    order = {"results": [{"index": i, "relevance_score": 1.0 - i * 1e-3}
                         for i in reversed(range(a.topk))]}
    calls = {"embed": 0, "query": 0, "rerank": 0}

    def embedding(**kw):
        calls["embed"] += 1
        return {"data": [{"embedding": vec} for _ in kw["input"]]}

    async def arerank(**kw):
        calls["rerank"] += 1
        return order

    litellm.embedding = embedding
    litellm.arerank = arerank

    class Coll:
        def query(self, query_embeddings, query_texts, n_results):
            calls["query"] += 1
            return hits

    class Client:
        def __init__(self, **kw):
            pass

        def get_or_create_collection(self, name):
            return Coll()

    pyseekdb.Client = Client

    from super_rag.nodeflow.base.models import Edge, NodeflowInstance, NodeInstance
    from super_rag.nodeflow.engine import NodeflowEngine
    import super_rag.nodeflow.runners.merge  # noqa: F401  (registers the runners)
    import super_rag.nodeflow.runners.rerank  # noqa: F401
    import super_rag.nodeflow.runners.vector_search  # noqa: F401
    import types
    col = types.SimpleNamespace(id="col1", user="u", config=json.dumps(
        {"embedding": {"model_service_provider": "p", "model": "BAAI/bge-m3",
                       "custom_llm_provider": "openai"}}))
    AsyncOps.collections["col1"] = col

    def flow(query):
        # collection_service.py:255-346 with vector_search on, graph_search off, rerank on
        nodes = {"vector_search": NodeInstance(id="vector_search", type="vector_search", input_values={
                     "query": query, "top_k": a.topk, "similarity_threshold": 0.2,
                     "collection_ids": ["col1"]}),
                 "merge": NodeInstance(id="merge", type="merge", input_values={
                     "merge_strategy": "union", "deduplicate": True,
                     "vector_search_docs": "{{ nodes.vector_search.output.docs }}"}),
                 "rerank": NodeInstance(id="rerank", type="rerank", input_values={
                     "use_rerank_service": True, "model": "BAAI/bge-reranker-v2-m3",
                     "model_service_provider": "p", "custom_llm_provider": "jina_ai",
                     "docs": "{{ nodes.merge.output.docs }}"})}
        edges = [Edge(source="vector_search", target="merge"), Edge(source="merge", target="rerank")]
        return NodeflowInstance(name="search", title="Search", nodes=nodes, edges=edges)

    async def run_all(n):
        engine = NodeflowEngine()
        out = None
        for i in range(n):
            out, _ = await engine.execute_nodeflow(flow(f"query number {i}"), {"query": f"query number {i}",
                                                                                "user": "u"})
        return out

    import logging
    logging.disable(logging.CRITICAL)       # the reference logs every payload (seekdb_connector.py:108)
    res = asyncio.run(run_all(5))           # warm-up (imports, caches, dimension probe)
    docs = res["rerank"].docs
    assert len(docs) == a.topk, len(docs)
    before = dict(calls)
    t0 = time.perf_counter()
    asyncio.run(run_all(a.queries))
    dt = (time.perf_counter() - t0) / a.queries
    per_q = {k: (calls[k] - before[k]) / a.queries for k in calls}
    rec = {"metric": "reference search-flow orchestration overhead, seconds per query",
           "value": round(dt, 6), "queries": a.queries, "top_k": a.topk, "dim": a.dim,
           "remote_calls_per_query": per_q,
           "method": ("real NodeflowEngine + vector_search/merge/rerank runners "
                      "(collection_service.py:255-346) with constant-time stub backends; logging off"),
           "host": {"python": platform.python_version(), "cpu": platform.processor() or platform.machine(),
                    "threads": 1},
           "note": "measured in the build container (the GPU box has no /root/reference)"}
    with open(OUT, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
