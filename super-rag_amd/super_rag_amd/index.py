"""Write path: chunk text -> embed on the GPU -> add to the in-HBM store.

Mirrors create_embeddings_and_store (super_rag/llm/embed/embedding_utils.py:13-95): the same
"> Hierarchy: ..." / "> Labels: ..." prefixes are prepended to the chunk text that gets embedded,
``metadata["source"] = metadata["name"]`` is set, and the uuid strings returned by the store are
the ``context_ids`` the indexer keeps (index/vector_and_full_text_index.py:29-225).  Chunking
uses the host application's ``rechunk`` when super_rag is importable; standalone, each part is
one chunk (parts are expected pre-chunked).
"""
from __future__ import annotations

import logging
from typing import List

from .models import TextNode

logger = logging.getLogger(__name__)


def chunk_text(part) -> str:
    """Text that gets embedded for one chunk (embedding_utils.py:55-80)."""
    meta = getattr(part, "metadata", None) or {}
    paddings = []
    if "titles" in meta:
        paddings.append("> Hierarchy: " + " > ".join(meta["titles"]))
    if "labels" in meta:
        labels = ["%s=%s" % (it["key"], it["value"]) for it in meta.get("labels", [{}])
                  if it.get("key", None) and it.get("value", None)]
        if labels:
            paddings.append("> Labels: " + " ".join(labels))
    prefix = "\n".join(paddings)
    return f"{prefix}\n\n{part.content}" if prefix else part.content


def build_nodes(chunked_parts) -> List[TextNode]:
    nodes = []
    for part in chunked_parts:
        if not part.content:
            continue
        metadata = dict(getattr(part, "metadata", None) or {})
        metadata["source"] = metadata.get("name", "")
        nodes.append(TextNode(text=chunk_text(part), metadata=metadata))
    return nodes


def create_embeddings_and_store(parts, vector_store_adaptor, embedding_model, chunk_size: int = 1500,
                                chunk_overlap: int = 200, tokenizer=None) -> List[str]:
    if not parts:
        return []
    try:  # pragma: no cover - host chunker when available
        from super_rag.chunk.chunking import rechunk  # type: ignore
        from super_rag.utils.tokenizer import get_default_tokenizer  # type: ignore
        chunked = rechunk(parts, chunk_size, chunk_overlap, tokenizer or get_default_tokenizer())
    except Exception:  # noqa: BLE001
        chunked = parts
    nodes = build_nodes(chunked)
    if not nodes:
        return []
    vectors = embedding_model.embed_documents([n.text for n in nodes])
    for n, v in zip(nodes, vectors):
        n.embedding = v
    logger.info("processed document with %d parts and %d chunks", len(parts), len(nodes))
    return vector_store_adaptor.connector.store.add(nodes)


class VectorIndexer:
    """create / update / delete of one document's vector index (vector_and_full_text_index.py)."""

    def __init__(self, connector, embedding_service):
        self.connector = connector
        self.embedding = embedding_service

    def create_index(self, parts) -> dict:
        class _Adaptor:
            connector = self.connector
        ids = create_embeddings_and_store(parts, _Adaptor, self.embedding)
        return {"context_ids": ids}

    def update_index(self, old_context_ids: List[str], parts) -> dict:
        if old_context_ids:
            self.connector.delete(ids=old_context_ids)
        return self.create_index(parts)

    def delete_index(self, context_ids: List[str]) -> None:
        if context_ids:
            self.connector.delete(ids=context_ids)
