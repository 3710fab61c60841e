"""Batched, device-resident search pipeline: query embed -> exact top-K -> cross-encoder rerank.

This is the throughput path behind the reference's per-request flow
(service/collection_service.py:229-366: vector_search -> merge -> rerank): B queries are processed
per call, every intermediate stays in HBM, and the only host round trip is the store's overflow
flag check.  With torch.distributed initialised (one process per GPU, backend "nccl" = RCCL over
xGMI) the corpus is row-sharded: each rank embeds its own B queries, the query embeddings are
all-gathered (C1), every rank scans its shard for all world*B queries, the per-shard top-K lists
are exchanged with one all_to_all (C2: each rank receives the lists of ITS queries) and merged by
K2, and each rank reranks its own B queries.  Passage tokens for the cross-encoder are replicated
per GPU (N x Lp int32, 3.8 GB at 10M x 94) so the pair packer never crosses ranks.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from .encoder import Encoder, build_pairs_dev, rerank_select_dev
from .store import NativeStore, topk_merge_dev


@dataclass
class PipelineResult:
    rows: torch.Tensor         # [B, k_final] int64 global row ids (reranked order)
    logits: torch.Tensor       # [B, k_final] fp32 cross-encoder logits
    cand_rows: torch.Tensor    # [B, K] int64 search candidates (distance order)
    cand_sims: torch.Tensor    # [B, K] fp32 cosine similarity (distance = 1 - sim)


class SearchPipeline:
    def __init__(self, embedder: Encoder, reranker: Encoder, store: NativeStore,
                 passage_tok: torch.Tensor, passage_len: torch.Tensor, k_candidates: int = 100,
                 k_final: int = 10, pair_len: int = 128, shard_offset: int = 0, group=None,
                 merge_fn=topk_merge_dev):
        self.embedder = embedder
        self.reranker = reranker
        self.store = store
        self.p_tok = passage_tok
        self.p_len = passage_len
        self.K = int(k_candidates)
        self.k = int(k_final)
        self.S = int(pair_len)
        self.offset = int(shard_offset)
        self.group = group
        self.merge_fn = merge_fn
        import torch.distributed as dist
        self.world = dist.get_world_size(group) if (group is not None or
                                                     (dist.is_available() and dist.is_initialized())) else 1

    def embed(self, q_ids: torch.Tensor, q_mask: torch.Tensor) -> torch.Tensor:
        return self.embedder.embed_dev(q_ids, q_mask, fp16=True)

    def retrieve(self, q_emb: torch.Tensor):
        """[B, d] fp16 unit queries of this rank -> merged global top-K (sims, rows) [B, K]."""
        B = q_emb.shape[0]
        if self.world == 1:
            return self.store.search_dev(q_emb, self.K, row_offset=self.offset)
        import torch.distributed as dist
        # RCCL moves device tensors; the gloo backend (CPU tests, rehearsals of several ranks on
        # one GPU) stages the same exchange through host memory
        host = dist.get_backend(self.group) == "gloo" and q_emb.is_cuda
        dev = q_emb.device
        qx = q_emb.contiguous().cpu() if host else q_emb.contiguous()
        allq = torch.empty((self.world * B, q_emb.shape[1]), dtype=q_emb.dtype, device=qx.device)
        dist.all_gather_into_tensor(allq, qx, group=self.group)
        sims, rows = self.store.search_dev(allq.to(dev) if host else allq, self.K,
                                           row_offset=self.offset)
        if host:
            sims, rows = sims.cpu(), rows.cpu()
        rs = torch.empty_like(sims)
        rr = torch.empty_like(rows)
        dist.all_to_all_single(rs, sims, group=self.group)
        dist.all_to_all_single(rr, rows, group=self.group)
        if host:
            rs, rr = rs.to(dev), rr.to(dev)
        return self.merge_fn(rs.view(self.world, B, self.K), rr.view(self.world, B, self.K),
                             self.K, device=q_emb.device.index or 0)

    def rerank(self, q_tok: torch.Tensor, q_len: torch.Tensor, cand_rows: torch.Tensor):
        B = cand_rows.shape[0]
        ids, mask, types = build_pairs_dev(q_tok, q_len, self.p_tok, self.p_len, cand_rows, self.S,
                                           self.reranker.spec,
                                           with_types=self.reranker.spec.pair_style == 1)
        logits = self.reranker.cross_score_dev(ids, mask, types)[:, 0].view(B, self.K)
        logits = logits.masked_fill(cand_rows < 0, float("-inf"))
        idx = rerank_select_dev(logits, self.k).long()
        return cand_rows.gather(1, idx), logits.gather(1, idx)

    def run(self, q_ids, q_mask, q_tok, q_len) -> PipelineResult:
        q = self.embed(q_ids, q_mask)
        sims, rows = self.retrieve(q)
        final_rows, final_logits = self.rerank(q_tok, q_len, rows)
        return PipelineResult(final_rows, final_logits, rows, sims)
