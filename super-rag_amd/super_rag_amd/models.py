"""Wire types of the hot path (super_rag/models/models.py:222-321).

When the host application (super_rag) is importable its own classes are used, so the
DocumentWithScore objects this package returns validate inside the reference's node models
(VectorSearchOutput, RerankInput, ...).  Standalone, identical definitions are provided.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

try:  # pragma: no cover - exercised only inside a super_rag deployment
    from super_rag.models import (  # type: ignore
        DocumentWithScore,
        Query,
        QueryResult,
        QueryWithEmbedding,
        TextNode,
    )
    HOST_MODELS = True
except Exception:  # noqa: BLE001 - any import failure means "standalone"
    from pydantic import BaseModel

    HOST_MODELS = False

    class TextNode:
        """Text node (models.py:222-256): text, metadata, embedding."""

        def __init__(self, text: str, metadata: Optional[Dict[str, Any]] = None,
                     embedding: Optional[list] = None):
            self.text = text
            self.metadata = metadata or {}
            self.embedding = embedding

        def to_dict(self) -> Dict[str, Any]:
            return {"text": self.text, "metadata": self.metadata, "embedding": self.embedding}

        @classmethod
        def from_dict(cls, data: Dict[str, Any]) -> "TextNode":
            return cls(text=data.get("text", ""), metadata=data.get("metadata", {}),
                       embedding=data.get("embedding"))

    class DocumentWithScore(BaseModel):
        """models.py:263-266 — no id field: ids never leave the connector."""
        text: Optional[str] = None
        score: Optional[float] = None
        metadata: Optional[dict] = None

    class Query(BaseModel):
        query: str
        top_k: Optional[int] = 3

    class QueryWithEmbedding(Query):
        embedding: List[float]

    class QueryResult(BaseModel):
        query: str
        results: List[DocumentWithScore]

__all__ = ["TextNode", "DocumentWithScore", "Query", "QueryWithEmbedding", "QueryResult",
           "HOST_MODELS"]
