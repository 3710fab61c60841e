"""ContextManager (super_rag/context/context.py:7-111) on the ``"mi355x"`` vector store."""
from __future__ import annotations

from typing import Any, List, Optional

from .models import QueryWithEmbedding
from .vectorstore import VectorStoreConnectorAdaptor


class ContextManager:
    def __init__(self, collection_name, embedding_model, vectordb_type, vectordb_ctx):
        self.collection_name = collection_name
        self.embedding_model = embedding_model
        self.vectordb_type = vectordb_type
        self.adaptor = VectorStoreConnectorAdaptor(vectordb_type, vectordb_ctx)

    def query(self, query, score_threshold=0.5, topk=3, vector=None, index_types=None, chat_id=None):
        if vector is None:
            vector = self.embedding_model.embed_query(query)
        query_embedding, kw = self._search_args(query, score_threshold, topk, vector, index_types, chat_id)
        return self.adaptor.connector.search(query_embedding, **kw).results

    async def aquery(self, query, score_threshold=0.5, topk=3, vector=None, index_types=None,
                     chat_id=None):
        """query for a coroutine (the connector's asearch: a coalesced search holds no thread)."""
        if vector is None:
            vector = await self.embedding_model.aembed_query(query)
        query_embedding, kw = self._search_args(query, score_threshold, topk, vector, index_types, chat_id)
        conn = self.adaptor.connector
        if hasattr(conn, "asearch"):
            return (await conn.asearch(query_embedding, **kw)).results
        import asyncio
        return (await asyncio.to_thread(conn.search, query_embedding, **kw)).results

    async def aquery_text(self, query, score_threshold=0.5, topk=3, index_types=None, chat_id=None):
        """aquery without a precomputed vector, when the connector can embed and search the
        query in one coalesced step (MI355XVectorStoreConnector.asearch_text); otherwise aquery.
        Same results."""
        conn = self.adaptor.connector
        if not (hasattr(conn, "asearch_text") and conn.can_fuse_embed(self.embedding_model)):
            return await self.aquery(query, score_threshold=score_threshold, topk=topk,
                                     index_types=index_types, chat_id=chat_id)
        filter_condition = self._create_combined_filter(index_types, chat_id)
        return (await conn.asearch_text(query, self.embedding_model, topk,
                                        score_threshold=score_threshold, filter=filter_condition)).results

    def _search_args(self, query, score_threshold, topk, vector, index_types, chat_id):
        filter_condition = self._create_combined_filter(index_types, chat_id)
        query_embedding = QueryWithEmbedding(query=query, top_k=topk, embedding=vector)
        # Same kwargs as context.py:37-47; the store ignores all but top_k, as SeekDB's did.
        return query_embedding, dict(
            collection_name=self.collection_name,
            query_vector=query_embedding.embedding,
            with_vectors=True,
            limit=query_embedding.top_k,
            consistency="majority",
            search_params={"hnsw_ef": 128, "exact": False},
            score_threshold=score_threshold,
            filter=filter_condition,
        )

    def _create_combined_filter(self, index_types: Optional[List[str]] = None,
                                chat_id: Optional[str] = None) -> Optional[Any]:
        if not index_types and not chat_id:
            return None
        clauses = []
        if index_types:
            clauses.append({"or": [{"indexer": {"$in": index_types}},
                                   {"indexer": {"$exists": False}}]})
        if chat_id:
            clauses.append({"chat_id": chat_id})
        return clauses[0] if len(clauses) == 1 else {"and": clauses}
