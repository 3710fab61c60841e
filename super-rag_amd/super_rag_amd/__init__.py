"""super_rag_amd — MI355X-native embed -> retrieve -> rerank hot path for super-rag.

Drop-in replacements for the reference's plugin surfaces:
  * vectorstore.MI355XVectorStoreConnector   (SeekDBVectorStoreConnector, vectorstore/seekdb_connector.py)
  * embed.EmbeddingService                   (llm/embed/embedding_service.py)
  * rerank.RerankService                     (llm/rerank/rerank_service.py)
  * nodeflow_pack.register()                 (nodeflow `vector_search` / `rerank` node runners)
backed by the HIP library in lib/libsrmi.so (include/super_rag_mi355x.h).
"""
__version__ = "0.1.0"
