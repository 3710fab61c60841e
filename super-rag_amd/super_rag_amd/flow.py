"""The search flow of POST /collections/{id}/searches on the pack's runners.

Mirrors CollectionService.execute_search_flow (super_rag/service/collection_service.py:229-366):
the same node inputs — vector_search {query, top_k, similarity_threshold, collection_ids[, chat_id]}
-> merge {merge_strategy "union", deduplicate, vector_search_docs} -> rerank
{use_rerank_service = model is not None, model, model_service_provider, custom_llm_provider, docs}
— executed in the flow's dependency order with the runners this pack registers
(nodeflow_pack.py), and the rerank output mapped to SearchResultItem{rank, score, content,
source, recall_type, metadata} (:352-364).  Inside a super_rag deployment the host's own
NodeflowEngine runs the same runners (the pack overrides the builtins); this driver is the
standalone form used by the tests and the HTTP seam.  Graph search (graphiti) is out of scope.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

from pydantic import BaseModel

from .nodeflow_pack import (NODE_RUNNER_REGISTRY, MergeInput, RerankInput, SystemInput,
                            VectorSearchInput, register)


class SearchResultItem(BaseModel):
    """schema/view_models.py SearchResultItem fields used by the search route."""
    rank: int
    score: Optional[float] = None
    content: Optional[str] = None
    source: Optional[str] = None
    recall_type: Optional[str] = None
    metadata: Optional[Dict[str, Any]] = None


async def execute_search_flow(query: str, collection_id: str, search_user_id: str, *,
                              vector_topk: Optional[int] = 5, vector_similarity: float = 0.2,
                              rerank: bool = True,
                              rerank_config: Tuple[Optional[str], Optional[str], Optional[str]] =
                              (None, None, None),
                              chat_id: Optional[str] = None) -> Tuple[List[SearchResultItem], str]:
    """(items, rerank node id) — collection_service.py:229-366 without the graph_search branch.
    ``vector_topk=None`` drops the vector_search node (data.vector_search unset); ``rerank_config``
    is the (model, model_service_provider, custom_llm_provider) the reference reads from
    default_model_service.get_default_rerank_config."""
    if "vector_search" not in NODE_RUNNER_REGISTRY:
        register()
    si = SystemInput(query=query, user=search_user_id)
    if chat_id:
        si.chat_id = chat_id
    merge_values: Dict[str, Any] = {"merge_strategy": "union", "deduplicate": True}
    if vector_topk is not None:
        vs_values: Dict[str, Any] = {"top_k": vector_topk, "similarity_threshold": vector_similarity,
                                     "collection_ids": [collection_id]}
        if chat_id:
            vs_values["chat_id"] = chat_id
        vs = NODE_RUNNER_REGISTRY["vector_search"]["runner"]
        vs_out, _ = await vs.run(VectorSearchInput(**vs_values), si)
        merge_values["vector_search_docs"] = vs_out.docs
    merged, _ = await NODE_RUNNER_REGISTRY["merge"]["runner"].run(MergeInput(**merge_values), si)
    if rerank:
        model, msp, provider = rerank_config
        use_service = model is not None
    else:
        model, msp, provider, use_service = None, None, None, False
    rr, _ = await NODE_RUNNER_REGISTRY["rerank"]["runner"].run(
        RerankInput(use_rerank_service=use_service, model=model, model_service_provider=msp,
                    custom_llm_provider=provider, docs=merged.docs), si)
    # (typed values from the runners: constructed without re-validation, 100 per request)
    items = [SearchResultItem.model_construct(rank=i + 1, score=d.score, content=d.text,
                                              source=(d.metadata or {}).get("source", ""),
                                              recall_type=(d.metadata or {}).get("recall_type", ""),
                                              metadata=d.metadata)
             for i, d in enumerate(rr.docs)]
    return items, "rerank"
