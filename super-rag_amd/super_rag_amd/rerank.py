"""Drop-in RerankService (super_rag/llm/rerank/rerank_service.py:21-232) on the MI355X
cross-encoder.

Same constructor / ``max_documents`` / ``async_rerank`` / ``validate_configuration`` and error
types.  ``_rank_texts`` scores the (query, passage) pairs in-process (XLM-R cross-encoder +
classification head) instead of ``litellm.arerank`` and returns the indices ordered by relevance
(logit desc, index asc), so ``async_rerank`` reorders the documents and keeps their original
scores exactly as the reference does (:74).
"""
from __future__ import annotations

import asyncio
import os
import logging
from typing import List, Optional

import numpy as np

from ._native import device_gate
from .errors import InvalidConfigurationError, InvalidDocumentError, RerankError, TooManyDocumentsError

logger = logging.getLogger(__name__)

# A coroutine tokenises its pairs on the event loop when at most this many of its passages miss
# the tokenizer's cache (the warm case: ~0.2 ms), in a worker thread otherwise (a cold request's
# HF encode of ~100 passages of up to 512 tokens would stall every other request on the loop).
OFFLOOP_TOKENIZE_MISSES = 8


class RerankService:
    def __init__(self, rerank_provider: str, rerank_model: str, rerank_service_url: str,
                 rerank_service_api_key: str, caching: bool = True, *, encoder=None,
                 tokenizer=None, device: Optional[int] = None, device_batch: int = 4096,
                 coalesce: bool = True):
        self.rerank_provider = rerank_provider
        self.model = rerank_model
        self.api_base = rerank_service_url      # accepted for signature parity; unused
        self.api_key = rerank_service_api_key   # accepted for signature parity; unused
        self.caching = caching
        self.max_documents = 1000
        self.device_batch = max(1, int(device_batch))
        self.coalesce = bool(coalesce)
        if encoder is None:
            from .registry import get_model
            encoder, tokenizer = get_model(rerank_model, device)
        self.encoder = encoder
        self.tokenizer = tokenizer

    def score(self, query: str, texts: List[str]) -> np.ndarray:
        """Raw cross-encoder logits, one per text.  Concurrent calls (one per search request)
        are coalesced into shared device batches per cross-encoder (coalesce.py).  The batch
        leader packs every caller's pairs: packing in the callers, concurrently, measured slower
        (GIL contention; 210.7 vs 228.1 q/s, profiles/r03_dropin/)."""
        if not self.coalesce:
            return self._score_many(self.encoder, self.tokenizer, self.device_batch, [(query, texts)])[0]
        return self._pair_coalescer()((query, list(texts)))

    def _pair_coalescer(self):
        coal = getattr(self.encoder, "_pair_coalescer", None)
        if coal is None:
            from .coalesce import Coalescer
            enc, tok, dev_b = self.encoder, self.tokenizer, self.device_batch
            coal = Coalescer(lambda items: RerankService._score_many(enc, tok, dev_b, items),
                             max_batch=max(1, dev_b // 100))
            setattr(self.encoder, "_pair_coalescer", coal)
        return coal

    @staticmethod
    def _score_many(encoder, tokenizer, device_batch: int, items) -> List[np.ndarray]:
        """[(query, texts)] -> per item logits."""
        return RerankService._score_encoded(
            encoder, device_batch, [tokenizer.encode_pairs(q, t) for q, t in items])

    @staticmethod
    def _score_encoded(encoder, device_batch: int, enc) -> List[np.ndarray]:
        """[(ids, mask, type_ids)] of encode_pairs -> per item logits; the pairs of all items
        share device batches (padded to a common width; the padding is masked, so logits do not
        depend on the batch composition)."""
        with_types = encoder.spec.pair_style == 1
        n = [e[0].shape[0] for e in enc]
        S = max(e[0].shape[1] for e in enc)
        # bucketed width: up to 128 tokens -> 128 (the fused QKV + attention kernel and the K/V-free
        # last layer take S = 128 / S % 16 == 0), longer -> a multiple of 16 within max_length
        cap = max(S, int(getattr(encoder.spec, "max_length", S)))
        S = min(128 if S <= 128 else -(-S // 16) * 16, cap)
        ids = np.full((sum(n), S), encoder.spec.pad_id, dtype=np.int32)
        mask = np.zeros((sum(n), S), dtype=np.int32)
        tt = np.zeros((sum(n), S), dtype=np.int32)
        o = 0
        for (ei, em, et), k in zip(enc, n):
            w = ei.shape[1]
            ids[o:o + k, :w] = ei
            mask[o:o + k, :w] = em
            tt[o:o + k, :w] = et
            o += k
        out = np.empty(ids.shape[0], dtype=np.float32)
        with device_gate(getattr(encoder, "device", 0), "rerank"):
            for s in range(0, ids.shape[0], device_batch):
                sl = slice(s, s + device_batch)
                out[sl] = encoder.cross_score(ids[sl], mask[sl], tt[sl] if with_types else None)[:, 0]
        res, o = [], 0
        for k in n:
            res.append(out[o:o + k])
            o += k
        return res

    async def async_rerank(self, query: str, results: list) -> list:
        try:
            if not query or not query.strip():
                raise InvalidDocumentError("Query cannot be empty")
            if not results:
                logger.info("No documents to rerank, returning empty list")
                return []
            if len(results) > self.max_documents:
                raise TooManyDocumentsError(document_count=len(results),
                                            max_documents=self.max_documents, model_name=self.model)
            texts, invalid = [], []
            for i, doc in enumerate(results):
                if not doc or not hasattr(doc, "text") or not doc.text or not doc.text.strip():
                    invalid.append(i)
                    texts.append(" ")
                else:
                    texts.append(doc.text)
            if invalid:
                logger.warning("Found %d invalid documents at indices: %s", len(invalid), invalid)
                if len(invalid) == len(results):
                    raise InvalidDocumentError("All documents are empty or invalid",
                                               document_count=len(results))
            order = await self._rank_texts(query, texts)
            return [results[i] for i in order if 0 <= i < len(results)]
        except (InvalidDocumentError, TooManyDocumentsError, RerankError):
            raise
        except Exception as e:  # noqa: BLE001
            raise RerankError(f"Rerank API error: {e}",
                              {"provider": self.rerank_provider, "model": self.model}) from e

    def _encoded_coalescer(self):
        """Coalescer of already tokenised pairs (the coroutine path): each request tokenises its
        own pairs on the event loop while the device runs the previous batch, and the batch
        leader only packs and scores.  (Tokenised by the leader, ~30 requests' pairs took ~55 ms
        per ~66 ms device batch with the device idle meanwhile, profiles/r05_dropin/.)"""
        coal = getattr(self.encoder, "_encoded_pair_coalescer", None)
        if coal is None:
            from .coalesce import Coalescer
            enc, dev_b = self.encoder, self.device_batch
            coal = Coalescer(lambda items: RerankService._score_encoded(enc, dev_b, items),
                             max_batch=max(1, dev_b // 100),
                             min_fill=int(os.environ.get("SUPER_RAG_AMD_RERANK_MIN_FILL", "1")),
                             max_wait_s=float(os.environ.get("SUPER_RAG_AMD_RERANK_MAX_WAIT_MS", "0")) * 1e-3)
            setattr(self.encoder, "_encoded_pair_coalescer", coal)
        return coal

    async def _rank_texts(self, query: str, texts: List[str]) -> List[int]:
        try:
            if self.coalesce:  # awaits its shared batch without holding a thread (coalesce.acall)
                texts = list(texts)
                misses = getattr(self.tokenizer, "cache_misses", None)
                cold = (misses(texts) if misses is not None else len(texts)) > OFFLOOP_TOKENIZE_MISSES
                if cold:
                    encoded = await asyncio.to_thread(self.tokenizer.encode_pairs, query, texts)
                else:
                    encoded = self.tokenizer.encode_pairs(query, texts)
                logits = await self._encoded_coalescer().acall(encoded)
            else:
                logits = await asyncio.to_thread(self.score, query, texts)
        except Exception as e:  # noqa: BLE001
            raise RerankError(f"Internal rerank operation failed: {e}",
                              {"provider": self.rerank_provider, "model": self.model,
                               "document_count": len(texts)}) from e
        return sorted(range(len(texts)), key=lambda i: (-float(logits[i]), i))

    def validate_configuration(self) -> None:
        # provider / model as in rerank_service.py:219-232; key and base URL are not needed
        # by the in-process model.
        if not self.rerank_provider:
            raise InvalidConfigurationError("rerank_provider", self.rerank_provider,
                                            "Provider cannot be empty")
        if not self.model:
            raise InvalidConfigurationError("model", self.model, "Model name cannot be empty")
