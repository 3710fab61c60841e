"""CPU oracle for the embed -> retrieve -> rerank hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / the timed CPU baseline.  The product path
(``super-rag_amd/super_rag_amd``) never imports it and fails loudly when the HIP library is missing.

What it restates (citations are into the reference at /root/reference):

* ``cosine_topk``  — SeekDB's cosine collection search as the reference configures and consumes it:
  ``HNSWConfiguration(dimension, distance="cosine")`` (super_rag/vectorstore/seekdb_connector.py:56-66),
  ``collection.query(query_embeddings, n_results=top_k)`` (:98-115) and ``score = distance``
  (:117-155).  Exact (not HNSW-approximate) fp64 cosine distance 1 - cos, ties broken by row id;
  zero-norm guard as graphiti's ``normalize_l2`` (graphiti_core/helpers.py:100-103).
* ``encoder_ref`` — the BERT / XLM-R encoders the reference reaches over HTTP
  (llm/embed/embedding_service.py:168-175 -> BAAI/bge-*; llm/rerank/rerank_service.py:95-104 ->
  BAAI/bge-reranker-*).  The models themselves are third-party (public architectures, not in the
  reference); the restatement is pinned against ``transformers`` BertModel / XLMRobertaModel /
  XLMRobertaForSequenceClassification on identical seeded weights (tests/test_oracle.py).
* ``boundary`` — the reference's host-side text handling: newline/empty cleaning of
  ``EmbeddingService.embed_documents`` (embedding_service.py:57-65), rerank input substitution and
  reorder-by-index (rerank_service.py:56-74), merge dedupe (nodeflow/runners/merge.py:56-64) and the
  rerank fallback order (nodeflow/runners/rerank.py:173-202).  Pinned by the boundary fixtures in
  tests/golden/boundary_fixtures.json, captured from the real reference code (tests/golden/
  gen_boundary_fixtures.py).

Parity status: the *arithmetic* of the reference lives in remote services and in the un-vendored
pylibseekdb (pyseekdb 1.0.0b8), so no reference test or fixture pins embedding values, cosine scores
or rerank scores: for those the oracle is "parity unpinned" against the reference itself and is
instead pinned to transformers (encoders) and to an independent brute-force sort (search).
"""
