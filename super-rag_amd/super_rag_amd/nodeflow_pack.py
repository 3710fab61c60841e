"""Nodeflow pack: ``vector_search`` / ``rerank`` (and ``merge``) node runners on the MI355X path.

Registered through the reference's external-pack mechanism: entry point group
``super_rag.nodeflow.packs`` (nodeflow/registry.py:19, :44-60; pyproject ``[project.entry-points]``
in INTEGRATION.md), loaded at app startup (app.py:29).  Registration is a dict write into
NODE_RUNNER_REGISTRY (nodeflow/base/models.py:122-144), so the pack overrides the builtin runners
with identical input/output models.

Runner behaviour mirrors the reference:
  * vector_search (nodeflow/runners/vector_search.py:24-135): first collection id -> collection ->
    embedding service -> ContextManager(vector store) -> embed_query -> query(top_k) -> tag
    metadata.recall_type = "vector_search"; every exception degrades to [].
  * rerank (nodeflow/runners/rerank.py:21-202): service rerank when configured, else / on any
    error the fallback order (graph results first, then score descending).
  * merge (nodeflow/runners/merge.py:12-65): union of the five lists, dedupe by exact text.
  * fulltext_search: the reference declares the node type (schema/view_models.py:276-283,
    FulltextSearchParams{topk, keywords} at :1043-1047) and the merge slot fulltext_search_docs
    (merge.py:18-20) but registers no runner; this one answers it with the device BM25 index
    (lexical.py; collections indexed with VECTOR_DB_CONTEXT {"fulltext": true}), tagging
    metadata.recall_type = "fulltext_search" and degrading every error to [] like vector_search.
Outside a super_rag deployment a minimal local registry with the same decorator and SystemInput
is used, so the pack can be exercised standalone (tests/test_boundary.py).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
from typing import Any, Dict, List, Optional, Tuple

from pydantic import BaseModel, Field, model_validator

from .errors import EmbeddingError, InvalidConfigurationError, ProviderNotFoundError, RerankError
from .models import DocumentWithScore

logger = logging.getLogger(__name__)

# ---- host registry, or a local one with the same surface ------------------------------------------
try:  # pragma: no cover - inside a super_rag deployment
    from super_rag.nodeflow.base.models import (  # type: ignore
        NODE_RUNNER_REGISTRY,
        BaseNodeRunner,
        SystemInput,
        register_node_runner,
    )
    HOST_NODEFLOW = True
except Exception:  # noqa: BLE001
    HOST_NODEFLOW = False
    NODE_RUNNER_REGISTRY: Dict[str, Dict[str, Any]] = {}

    class BaseNodeRunner:
        async def run(self, ui: Any, si: Any) -> Tuple[Any, Dict[str, Any]]:
            raise NotImplementedError

    def register_node_runner(node_type: str, input_model, output_model):
        def decorator(cls):
            NODE_RUNNER_REGISTRY[node_type] = {"runner": cls(), "input_model": input_model,
                                               "output_model": output_model}
            return cls
        return decorator

    class SystemInput:
        def __init__(self, query: str, user: str, history=None, message_id=None, **kwargs):
            self.query = query
            self.user = user
            self.history = history
            self.message_id = message_id
            for k, v in kwargs.items():
                setattr(self, k, v)


# ---- node I/O models (identical fields / defaults to the reference) ---------------------------------
class VectorSearchInput(BaseModel):
    top_k: int = Field(5, description="Number of top results to return")
    similarity_threshold: float = Field(0.2, description="Similarity threshold for vector search")
    collection_ids: Optional[List[str]] = Field(default_factory=list, description="Collection IDs")
    chat_id: Optional[str] = Field(None, description="Chat ID to filter chat documents")


class VectorSearchOutput(BaseModel):
    docs: List[DocumentWithScore]


class FulltextSearchInput(BaseModel):
    top_k: int = Field(5, description="Number of top results to return")
    keywords: Optional[List[str]] = Field(None, description="Custom keywords to use for fulltext search")
    collection_ids: Optional[List[str]] = Field(default_factory=list, description="Collection IDs")
    chat_id: Optional[str] = Field(None, description="Chat ID to filter chat documents")


class FulltextSearchOutput(BaseModel):
    docs: List[DocumentWithScore]


class RerankInput(BaseModel):
    use_rerank_service: bool = Field(default=True)
    model: Optional[str] = Field(default=None)
    model_service_provider: Optional[str] = Field(default=None)
    custom_llm_provider: Optional[str] = Field(default=None)
    docs: List[DocumentWithScore]
    value: Optional[Any] = Field(default=None, exclude=True)

    @model_validator(mode="before")
    @classmethod
    def value_to_docs(cls, data: Any) -> Any:
        if not isinstance(data, dict):
            return data
        if "docs" in data and data["docs"] is not None:
            return data
        val = data.get("value")
        if val is None:
            return data
        if hasattr(val, "docs"):
            data = {**data, "docs": val.docs}
        elif isinstance(val, list):
            data = {**data, "docs": val}
        return data


class RerankOutput(BaseModel):
    docs: List[DocumentWithScore]


class MergeInput(BaseModel):
    merge_strategy: str = Field("union")
    deduplicate: bool = Field(True)
    vector_search_docs: Optional[List[DocumentWithScore]] = Field(default_factory=list)
    fulltext_search_docs: Optional[List[DocumentWithScore]] = Field(default_factory=list)
    graph_search_docs: Optional[List[DocumentWithScore]] = Field(default_factory=list)
    summary_search_docs: Optional[List[DocumentWithScore]] = Field(default_factory=list)
    vision_search_docs: Optional[List[DocumentWithScore]] = Field(default_factory=list)


class MergeOutput(BaseModel):
    docs: List[DocumentWithScore]


# ---- collection resolution ------------------------------------------------------------------------
class LocalCollection:
    """Standalone stand-in for the DB row (id, config JSON with embedding.model)."""

    def __init__(self, id: str, config: dict, user: str = ""):
        self.id = id
        self.config = json.dumps(config)
        self.user = user


class VectorSearchRepository:
    """Collection lookup: the host DB (async_db_ops.query_collection) when available, else a
    local catalog populated by ``register_collection``."""

    catalog: Dict[str, LocalCollection] = {}

    async def get_collection(self, user, collection_id: str):
        if HOST_NODEFLOW:  # pragma: no cover
            from super_rag.db.ops import async_db_ops  # type: ignore
            return await async_db_ops.query_collection(user, collection_id)
        return self.catalog.get(collection_id)


def register_collection(collection: LocalCollection) -> None:
    VectorSearchRepository.catalog[collection.id] = collection


def collection_name_for(collection_id: str) -> str:
    if HOST_NODEFLOW:  # pragma: no cover
        from super_rag.utils.utils import generate_vector_db_collection_name  # type: ignore
        return generate_vector_db_collection_name(collection_id)
    return str(collection_id)  # utils/utils.py:14-15


def vector_db_context() -> dict:
    raw = os.environ.get("SUPER_RAG_AMD_VECTOR_DB_CONTEXT")
    if raw:
        return json.loads(raw)
    if HOST_NODEFLOW:  # pragma: no cover
        from super_rag.config import settings  # type: ignore
        return json.loads(settings.vector_db_context)
    return {}


# ---- runners ---------------------------------------------------------------------------------------
class VectorSearchService:
    def __init__(self, repository: VectorSearchRepository):
        self.repository = repository

    async def execute_vector_search(self, user, query: str, top_k: int, similarity_threshold: float,
                                    collection_ids: List[str], chat_id: Optional[str] = None):
        from .context import ContextManager
        from .embed import get_collection_embedding_service_sync
        from .vectorstore import VECTOR_DB_TYPE

        collection = None
        if collection_ids:
            collection = await self.repository.get_collection(user, collection_ids[0])
        if not collection:
            return []
        try:
            name = collection_name_for(collection.id)
            embedding_model, _ = get_collection_embedding_service_sync(collection)
            ctx = vector_db_context()
            ctx["collection"] = name
            cm = ContextManager(name, embedding_model, VECTOR_DB_TYPE, ctx)

            # The reference runs these synchronously on the event loop (vector_search.py:76-86);
            # here the query is embedded and searched as one coalesced device step
            # (ContextManager.aquery_text: concurrent requests share one embed batch and one
            # search batch) awaited without holding a thread, so the loop stays free and
            # concurrent requests batch.  Same calls, same results.
            results = await cm.aquery_text(query, score_threshold=similarity_threshold, topk=top_k,
                                           index_types=["vector"], chat_id=chat_id)
            for item in results:
                if item.metadata is None:
                    item.metadata = {}
                item.metadata["recall_type"] = "vector_search"
            return results
        except ProviderNotFoundError as e:
            logger.warning("Vector search skipped for collection %s: %s", collection.id, e)
            return []
        except EmbeddingError as e:
            logger.warning("Vector search skipped for collection %s: %s", collection.id, e)
            return []
        except Exception as e:  # noqa: BLE001 - the reference degrades every error to []
            logger.error("Vector search failed for collection %s: %s", collection.id, e)
            return []


class VectorSearchNodeRunner(BaseNodeRunner):
    def __init__(self):
        self.repository = VectorSearchRepository()
        self.service = VectorSearchService(self.repository)

    async def run(self, ui: VectorSearchInput, si) -> Tuple[VectorSearchOutput, dict]:
        chat_id = ui.chat_id or getattr(si, "chat_id", None)
        collection_ids = ui.collection_ids or getattr(si, "collection_ids", [])
        docs = await self.service.execute_vector_search(
            user=si.user, query=si.query, top_k=ui.top_k,
            similarity_threshold=ui.similarity_threshold, collection_ids=collection_ids,
            chat_id=chat_id)
        return VectorSearchOutput(docs=docs), {}


class FulltextSearchNodeRunner(BaseNodeRunner):
    def __init__(self):
        self.repository = VectorSearchRepository()

    async def run(self, ui: FulltextSearchInput, si) -> Tuple[FulltextSearchOutput, dict]:
        from .vectorstore import MI355XVectorStoreConnector
        collection_ids = ui.collection_ids or getattr(si, "collection_ids", [])
        chat_id = ui.chat_id or getattr(si, "chat_id", None)
        collection = None
        if collection_ids:
            collection = await self.repository.get_collection(si.user, collection_ids[0])
        if not collection:
            return FulltextSearchOutput(docs=[]), {}
        try:
            ctx = vector_db_context()
            ctx["collection"] = collection_name_for(collection.id)
            conn = MI355XVectorStoreConnector(ctx)
            # the chat filter of the vector path (context/context.py:74-111; applied with
            # ctx["honor_filter"]); the rows are the vector rows, so no indexer clause
            flt = {"chat_id": chat_id} if chat_id else None
            docs = await asyncio.to_thread(conn.fulltext_search, si.query, ui.top_k, ui.keywords,
                                           filter=flt)
            for item in docs:
                if item.metadata is None:
                    item.metadata = {}
                item.metadata["recall_type"] = "fulltext_search"
            return FulltextSearchOutput(docs=docs), {}
        except Exception as e:  # noqa: BLE001 - degrade to [] like vector_search
            logger.error("Fulltext search failed for collection %s: %s", collection.id, e)
            return FulltextSearchOutput(docs=[]), {}


class RerankNodeRunner(BaseNodeRunner):
    async def run(self, ui: RerankInput, si) -> Tuple[RerankOutput, dict]:
        docs = ui.docs
        if not docs:
            return RerankOutput(docs=[]), {}
        if not ui.use_rerank_service:
            return RerankOutput(docs=self._apply_fallback_strategy(docs)), {}
        try:
            if not self._is_rerank_config_valid(ui):
                return RerankOutput(docs=self._apply_fallback_strategy(docs)), {}
            return RerankOutput(docs=await self._perform_actual_rerank(ui, si)), {}
        except (InvalidConfigurationError, ProviderNotFoundError, RerankError) as e:
            logger.warning("Rerank service failed, using fallback strategy: %s", e)
        except Exception as e:  # noqa: BLE001
            logger.error("Unexpected error during rerank, using fallback strategy: %s", e)
        return RerankOutput(docs=self._apply_fallback_strategy(docs)), {}

    def _is_rerank_config_valid(self, ui: RerankInput) -> bool:
        return bool(ui.model and ui.model.strip() and ui.model_service_provider
                    and ui.model_service_provider.strip() and ui.custom_llm_provider
                    and ui.custom_llm_provider.strip())

    async def _perform_actual_rerank(self, ui: RerankInput, si) -> List[DocumentWithScore]:
        from .rerank import RerankService
        svc = RerankService(rerank_provider=ui.custom_llm_provider, rerank_model=ui.model,
                            rerank_service_url="", rerank_service_api_key="")
        svc.validate_configuration()
        return await svc.async_rerank(si.query, ui.docs)

    def _apply_fallback_strategy(self, docs: List[DocumentWithScore]) -> List[DocumentWithScore]:
        graph, other = [], []
        for doc in docs:
            (graph if (doc.metadata or {}).get("recall_type", "") == "graph_search" else other).append(doc)
        other.sort(key=lambda x: x.score if x.score is not None else 0.0, reverse=True)
        return graph + other


class MergeNodeRunner(BaseNodeRunner):
    async def run(self, ui: MergeInput, si) -> Tuple[MergeOutput, dict]:
        if ui.merge_strategy not in ["union"]:
            raise ValueError(f"Unknown merge strategy: {ui.merge_strategy}")
        all_docs = ((ui.vector_search_docs or []) + (ui.fulltext_search_docs or [])
                    + (ui.graph_search_docs or []) + (ui.summary_search_docs or [])
                    + (ui.vision_search_docs or []))
        if not ui.deduplicate:
            return MergeOutput(docs=all_docs), {}
        seen, out = set(), []
        for d in all_docs:
            if d.text not in seen:
                seen.add(d.text)
                out.append(d)
        return MergeOutput(docs=out), {}


def register(include_merge: bool = False) -> None:
    """Entry point of the ``super_rag.nodeflow.packs`` group: (re-)register the runners."""
    register_node_runner("vector_search", input_model=VectorSearchInput,
                         output_model=VectorSearchOutput)(VectorSearchNodeRunner)
    register_node_runner("rerank", input_model=RerankInput, output_model=RerankOutput)(RerankNodeRunner)
    register_node_runner("fulltext_search", input_model=FulltextSearchInput,
                         output_model=FulltextSearchOutput)(FulltextSearchNodeRunner)
    if include_merge or not HOST_NODEFLOW:
        register_node_runner("merge", input_model=MergeInput, output_model=MergeOutput)(MergeNodeRunner)
