"""Drop-in EmbeddingService (super_rag/llm/embed/embedding_service.py:22-194) on the MI355X encoder.

Same constructor, same methods, same validation and text cleaning, same error types.  Instead of
fanning batches of ``max_chunks`` texts out to 8 HTTP threads (:72-99), texts are tokenised on
the host and embedded in-process on the GPU in device batches (length-sorted to limit padding,
order restored), CLS-pooled and L2-normalised like the BGE models the reference calls.
"""
from __future__ import annotations

import asyncio
import json
import logging
from typing import List, Optional, Sequence

import numpy as np

from ._native import device_gate
from .errors import (BatchProcessingError, EmbeddingError, EmptyTextError,
                     InvalidConfigurationError)

logger = logging.getLogger(__name__)


class EmbeddingService:
    def __init__(self, embedding_provider: str, embedding_model: str, embedding_service_url: str,
                 embedding_service_api_key: str, embedding_max_chunks_in_batch: int,
                 multimodal: bool = False, caching: bool = True, *, encoder=None, tokenizer=None,
                 device: Optional[int] = None, device_batch: int = 256, coalesce: bool = True):
        self.embedding_provider = embedding_provider
        self.model = embedding_model
        self.api_base = embedding_service_url          # accepted for signature parity; unused
        self.api_key = embedding_service_api_key       # accepted for signature parity; unused
        self.max_chunks = embedding_max_chunks_in_batch
        self.max_workers = 8
        self.multimodal = multimodal
        self.caching = caching
        self.device_batch = max(1, int(device_batch))
        self.coalesce = bool(coalesce)
        if encoder is None:
            from .registry import get_model
            encoder, tokenizer = get_model(embedding_model, device)
        self.encoder = encoder
        self.tokenizer = tokenizer

    @property
    def dimension(self) -> int:
        return int(self.encoder.spec.hidden)

    @staticmethod
    def _embed_with(encoder, tokenizer, device_batch: int, texts: Sequence[str]) -> np.ndarray:
        order = sorted(range(len(texts)), key=lambda i: len(texts[i]))
        out = np.empty((len(texts), int(encoder.spec.hidden)), dtype=np.float32)
        for s in range(0, len(order), device_batch):
            idx = order[s:s + device_batch]
            try:
                ids, mask = tokenizer.encode_batch([texts[i] for i in idx])
                with device_gate(getattr(encoder, "device", 0), "embed"):
                    out[idx] = encoder.embed(ids, mask)
            except Exception as e:  # noqa: BLE001 - a failed device batch, as in :94-99
                raise BatchProcessingError(batch_size=len(idx), reason=f"device batch failed: {e}") from e
        return out

    def _embed_clean(self, texts: Sequence[str]) -> np.ndarray:
        return self._embed_with(self.encoder, self.tokenizer, self.device_batch, texts)

    def embed_documents(self, contents: List[str]) -> List[List[float]]:
        if not contents:
            raise EmptyTextError(0)
        empty = [i for i, t in enumerate(contents) if not t or not t.strip()]
        if empty:
            logger.warning("Found %d empty content at indices: %s", len(empty), empty)
            if len(empty) == len(contents):
                raise EmptyTextError(len(empty))
        try:
            clean = [t.replace("\n", " ") if t and t.strip() else " " for t in contents]
            return self._embed_clean(clean).tolist()
        except (EmptyTextError, BatchProcessingError, EmbeddingError):
            raise
        except Exception as e:  # noqa: BLE001
            raise EmbeddingError(f"Embedding API error: {e}",
                                 {"provider": self.embedding_provider, "model": self.model}) from e

    async def aembed_documents(self, contents: List[str]) -> List[List[float]]:
        return await asyncio.to_thread(self.embed_documents, contents)

    def embed_query(self, content: str) -> List[float]:
        if not content or not content.strip():
            raise EmptyTextError(1)
        if not self.coalesce:
            return self.embed_documents([content])[0]
        # concurrent single-query calls (one per search request, embedding_service.py:114) are
        # coalesced into one device batch per encoder (coalesce.py); results are per query
        try:
            return self._query_coalescer()(content.replace("\n", " ")).tolist()
        except BatchProcessingError:
            raise
        except Exception as e:  # noqa: BLE001
            raise EmbeddingError(f"Embedding API error: {e}",
                                 {"provider": self.embedding_provider, "model": self.model}) from e

    def _query_coalescer(self):
        coal = getattr(self.encoder, "_query_coalescer", None)
        if coal is None:
            from .coalesce import Coalescer
            enc, tok, dev_b = self.encoder, self.tokenizer, self.device_batch

            def run(texts):
                return list(EmbeddingService._embed_with(enc, tok, dev_b, texts))
            coal = Coalescer(run, max_batch=self.device_batch)
            setattr(self.encoder, "_query_coalescer", coal)
        return coal

    async def aembed_query(self, content: str) -> List[float]:
        """embed_query for a coroutine: the coalesced query awaits its batch without holding a
        worker thread (coalesce.Coalescer.acall); same result and errors."""
        if not self.coalesce:
            return await asyncio.to_thread(self.embed_query, content)
        if not content or not content.strip():
            raise EmptyTextError(1)
        try:
            return (await self._query_coalescer().acall(content.replace("\n", " "))).tolist()
        except BatchProcessingError:
            raise
        except Exception as e:  # noqa: BLE001
            raise EmbeddingError(f"Embedding API error: {e}",
                                 {"provider": self.embedding_provider, "model": self.model}) from e

    def is_multimodal(self) -> bool:
        return self.multimodal


def _collection_config(collection) -> dict:
    cfg = getattr(collection, "config", collection)
    if isinstance(cfg, str):
        cfg = json.loads(cfg)
    if hasattr(cfg, "model_dump"):
        cfg = cfg.model_dump()
    if not isinstance(cfg, dict):
        raise TypeError(f"unsupported collection config {type(cfg)}")
    return cfg


def get_collection_embedding_service_sync(collection, device: Optional[int] = None):
    """(EmbeddingService, dim) for a collection — llm/embed/base_embedding.py:122-215.

    The collection config's ``embedding.model`` selects the resident encoder; provider and key
    lookups are unnecessary for the in-process model.  The dimension comes from the model shape
    (no "dimension_probe" embed, base_embedding.py:56)."""
    try:
        cfg = _collection_config(collection)
    except Exception as e:  # noqa: BLE001
        raise InvalidConfigurationError("collection.config", getattr(collection, "config", None),
                                        f"Invalid collection configuration: {e}") from e
    emb = cfg.get("embedding") or {}
    model = emb.get("model")
    if not model:
        raise InvalidConfigurationError("embedding.model", model, "Model name cannot be empty")
    provider = emb.get("custom_llm_provider") or "mi355x"
    try:
        svc = EmbeddingService(provider, model, "", "", emb.get("max_chunks", 10), device=device)
    except EmbeddingError:
        raise
    except Exception as e:  # noqa: BLE001 - unknown model, missing checkpoint / tokenizer, device
        # base_embedding.py:114-121: every creation failure surfaces as EmbeddingError
        logger.error("Failed to create embedding model %s/%s: %s", provider, model, e)
        raise EmbeddingError(f"Failed to create embedding model: {e}",
                             {"provider": provider, "model": model}) from e
    return svc, svc.dimension
