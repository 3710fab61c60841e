"""Batched, device-resident search pipeline: query embed -> exact top-K -> cross-encoder rerank.

This is the throughput path behind the reference's per-request flow
(service/collection_service.py:229-366: vector_search -> merge -> rerank): B queries are processed
per call, every intermediate stays in HBM, and the only host round trip is the store's overflow
flag check.  With torch.distributed initialised (one process per GPU, backend "nccl" = RCCL over
xGMI) the corpus is row-sharded: each rank embeds its own B queries, the query embeddings are
all-gathered (C1), every rank scans its shard for all world*B queries, the per-shard top-K lists
are exchanged with one all_to_all (C2: each rank receives the lists of ITS queries) and merged by
K2, and each rank reranks its own B queries.  Passage tokens for the cross-encoder are either
replicated per GPU (N x Lp int32: 3.8 GB at 10M x 94, 18.8 GB at 50M) or, with
``shard_passages=True``, held per shard like the rows (passage_tok = the shard's rows) and the
candidates' tokens fetched from their owning ranks per batch (C3: all_gather of the candidate ids,
one all_to_all of the owned token rows, world * B * K * Lp * 4 bytes per rank: 77 MB at 8 ranks).

Hybrid mode (``lexical=`` a NativeLexIndex over the shard's rows, BASELINE config 5): the rerank
candidates are the rrf fusion (graphiti rrf, search_utils.py:1762-1778) of the dense top-k_each and
the BM25 top-k_each of the query tokens.  Sharded, every shard scores BM25 with the corpus-wide N,
avgdl and document frequencies (all-reduced per batch), both per-shard lists go through the same
all_to_all + K2 merge, so the fused candidates equal a single index's.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from .encoder import Encoder, build_pairs_dev, rerank_select_dev
from .store import NativeStore, topk_merge_dev


@dataclass
class PipelineResult:
    rows: torch.Tensor         # [B, k_final] int64 global row ids (reranked order)
    logits: torch.Tensor       # [B, k_final] fp32 cross-encoder logits
    cand_rows: torch.Tensor    # [B, K] int64 search candidates (distance order)
    cand_sims: torch.Tensor    # [B, K] fp32 cosine similarity (distance = 1 - sim); rrf score
                               # of the fused candidates in hybrid mode


class StageClock:
    """Per-stage time of SearchPipeline.run (bench.py's stage_ms): marks at the stage boundaries,
    each interval charged to the stage named by the mark that ends it -- embed, search (K1 / BM25
    / K2 merge / rrf), exchange (C1 all_gather of the queries, C2 all_to_all of the per-shard lists,
    the BM25 statistics all_reduce, C3 passage fetch) and rerank (pair packing, cross-encoder, top-k
    select).  On device tensors a mark is a HIP event recorded on the current stream (the stream
    every library kernel of the pipeline is launched on; an RCCL collective is ordered into it by
    torch, so the event after a collective marks its completion); on host tensors (the gloo CPU
    path) a perf_counter stamp.  Events are read back once, in read().
    The exchange marks name their collective ("exchange.c1" ...): read() also returns each one's
    share as exchange_c1 (query all_gather), exchange_c2 (all_to_all of the per-shard lists),
    exchange_bm25_allreduce (hybrid: the corpus statistics) and exchange_c3 (passage fetch), whose
    sum is exchange."""

    STAGES = ("embed", "search", "exchange", "rerank")
    EXCHANGES = ("c1", "c2", "bm25_allreduce", "c3")

    def __init__(self):
        self.marks = []          # (stage, event or float) in issue order; None stage = start
        self.steps = 0

    def mark(self, stage, like=None):
        dev = like is not None and like.is_cuda
        if dev:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.marks.append((stage, e))
        else:
            self.marks.append((stage, time.perf_counter()))

    def start(self, like=None):
        self.steps += 1
        self.mark(None, like)

    def read(self) -> dict:
        """{stage: ms per step} over the marks so far (synchronises recorded events)."""
        tot = {s: 0.0 for s in self.STAGES}
        tot.update({"exchange_" + x: 0.0 for x in self.EXCHANGES})
        prev = None
        for stage, m in self.marks:
            if stage is not None and prev is not None:
                if isinstance(m, float) and isinstance(prev, float):
                    dt = (m - prev) * 1e3
                elif not isinstance(m, float) and not isinstance(prev, float):
                    m.synchronize()
                    dt = prev.elapsed_time(m)
                else:  # (a host stamp next to an event: not comparable, not charged)
                    dt = 0.0
                main, _, sub = stage.partition(".")
                tot[main] += dt
                if sub:
                    tot["exchange_" + sub] += dt
            prev = m
        n = max(1, self.steps)
        return {s: round(v / n, 4) for s, v in tot.items()}


class SearchPipeline:
    def __init__(self, embedder: Encoder, reranker: Encoder, store: NativeStore,
                 passage_tok: torch.Tensor, passage_len: torch.Tensor, k_candidates: int = 100,
                 k_final: int = 10, pair_len: int = 128, shard_offset: int = 0, group=None,
                 merge_fn=topk_merge_dev, lexical=None, k_each: int | None = None,
                 rank_const: int = 1, force_exchange: bool = False, shard_passages: bool = False):
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
        self.lexical = lexical
        self.k_each = int(k_each or self.K)
        self.rank_const = int(rank_const)
        import torch.distributed as dist
        self.world = dist.get_world_size(group) if (group is not None or
                                                     (dist.is_available() and dist.is_initialized())) else 1
        # force_exchange: run the collectives even in a world of one (the RCCL calls of the
        # sharded path exercised on a one-GPU box)
        self.exchange = self.world > 1 or bool(force_exchange)
        # passage_tok / passage_len hold only rows [shard_offset, shard_offset + len) (C3 fetch)
        self.shard_passages = bool(shard_passages) and self.exchange
        self.clock: StageClock | None = None   # set a StageClock to time the stages of run()

    def _mark(self, stage, like):
        if self.clock is not None:
            self.clock.mark(stage, like)

    def embed(self, q_ids: torch.Tensor, q_mask: torch.Tensor) -> torch.Tensor:
        return self.embedder.embed_dev(q_ids, q_mask, fp16=True)

    def retrieve(self, q_emb: torch.Tensor):
        """[B, d] fp16 unit queries of this rank -> merged global top-K (sims, rows) [B, K]."""
        B = q_emb.shape[0]
        if not self.exchange:
            return self.store.search_dev(q_emb, self.K, row_offset=self.offset)
        import torch.distributed as dist
        # RCCL moves device tensors; the gloo backend (CPU tests, rehearsals of several ranks on
        # one GPU) stages the same exchange through host memory
        host = dist.get_backend(self.group) == "gloo" and q_emb.is_cuda
        dev = q_emb.device
        qx = q_emb.contiguous().cpu() if host else q_emb.contiguous()
        allq = torch.empty((self.world * B, q_emb.shape[1]), dtype=q_emb.dtype, device=qx.device)
        dist.all_gather_into_tensor(allq, qx, group=self.group)
        allq = allq.to(dev) if host else allq
        self._mark("exchange.c1", allq)
        sims, rows = self.store.search_dev(allq, self.K, row_offset=self.offset)
        self._mark("search", sims)
        return self._exchange(sims, rows, B, self.K, host, dev)

    def _exchange(self, sims, rows, B, k, host, dev):
        import torch.distributed as dist
        if host:
            sims, rows = sims.cpu(), rows.cpu()
        rs = torch.empty_like(sims)
        rr = torch.empty_like(rows)
        dist.all_to_all_single(rs, sims, group=self.group)
        dist.all_to_all_single(rr, rows, group=self.group)
        if host:
            rs, rr = rs.to(dev), rr.to(dev)
        self._mark("exchange.c2", rs)
        out = self.merge_fn(rs.view(self.world, B, k), rr.view(self.world, B, k), k,
                            device=dev.index or 0)
        self._mark("search", out[0])
        return out

    def retrieve_hybrid(self, q_emb: torch.Tensor, q_tok: torch.Tensor, q_len: torch.Tensor):
        """Dense top-k_each + BM25 top-k_each (query tokens) fused by rrf -> (rrf score, rows)
        [B, K] of this rank's queries.  Everything stays on the device: the query tokens go to the
        lexical kernels as a padded [B, Lq] matrix (sr_lex_search_tok_dev), and sharded, the
        corpus-wide N, summed length and per-(query, position) df are one device vector
        (sr_lex_query_stats_dev) summed by one all_reduce (RCCL) before scoring."""
        from .lexical import rrf_fuse_dev
        B = q_emb.shape[0]
        dev = q_emb.device
        ke = self.k_each
        toks, lens = q_tok.to(torch.int32).contiguous(), q_len.to(torch.int32).contiguous()
        gst = None
        if not self.exchange:
            allq = q_emb
        else:
            import torch.distributed as dist
            host = dist.get_backend(self.group) == "gloo" and q_emb.is_cuda

            def gather(x):
                x = x.contiguous().cpu() if host else x.contiguous()
                out = torch.empty((self.world * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype,
                                  device=x.device)
                dist.all_gather_into_tensor(out, x, group=self.group)
                return out.to(dev) if host else out
            allq, toks, lens = gather(q_emb), gather(toks), gather(lens)
            self._mark("exchange.c1", allq)
            gst = self.lexical.query_stats_dev(toks, lens)
            self._mark("search", gst)
            if host:
                g = gst.cpu()
                dist.all_reduce(g, group=self.group)
                gst = g.to(dev)
            else:
                dist.all_reduce(gst, group=self.group)
            self._mark("exchange.bm25_allreduce", gst)
        sims, rows = self.store.search_dev(allq, ke, row_offset=self.offset)
        lsc, lrows = self.lexical.search_tok_dev(toks, lens, ke, gstats=gst, row_offset=self.offset)
        self._mark("search", lsc)
        if self.exchange:
            import torch.distributed as dist
            host = dist.get_backend(self.group) == "gloo" and q_emb.is_cuda
            sims, rows = self._exchange(sims, rows, B, ke, host, dev)
            lsc, lrows = self._exchange(lsc, lrows, B, ke, host, dev)
        score, fused = rrf_fuse_dev(rows, lrows, self.K, self.rank_const)
        self._mark("search", score)
        return score.float(), fused

    def passages(self, cand_rows: torch.Tensor):
        """(token table, lengths, [B, K] indices into them) for this rank's candidates (global
        rows, -1 = none).  Replicated: the full table and the rows themselves.  Sharded (C3): the
        candidate ids of every rank are all-gathered, each rank copies the token rows it owns
        (zeros elsewhere) into the slots of the asking rank, one all_to_all returns every rank its
        candidates' rows from all owners, and the sum over sources (exactly one owner per row)
        is the compact [B * K, Lp] table of this rank's candidates."""
        if not self.shard_passages:
            return self.p_tok, self.p_len, cand_rows
        import torch.distributed as dist
        B, K = cand_rows.shape
        dev = cand_rows.device
        host = dist.get_backend(self.group) == "gloo" and cand_rows.is_cuda
        rx = cand_rows.contiguous().cpu() if host else cand_rows.contiguous()
        allr = torch.empty((self.world * B, K), dtype=rx.dtype, device=rx.device)
        dist.all_gather_into_tensor(allr, rx, group=self.group)
        allr = allr.to(self.p_tok.device)
        loc = allr - self.offset
        own = (allr >= 0) & (loc >= 0) & (loc < self.p_tok.shape[0])
        li = torch.where(own, loc, torch.zeros_like(loc))
        tok = self.p_tok[li] * own.unsqueeze(-1).to(self.p_tok.dtype)   # [world*B, K, Lp]
        ln = self.p_len[li] * own.to(self.p_len.dtype)                   # [world*B, K]
        if host:
            tok, ln = tok.cpu(), ln.cpu()
        rt, rl = torch.empty_like(tok), torch.empty_like(ln)
        dist.all_to_all_single(rt, tok, group=self.group)
        dist.all_to_all_single(rl, ln, group=self.group)
        Lp = tok.shape[-1]
        tq = rt.view(self.world, B * K, Lp).sum(0, dtype=self.p_tok.dtype).to(dev)
        lq = rl.view(self.world, B * K).sum(0, dtype=self.p_len.dtype).to(dev)
        idx = torch.arange(B * K, device=dev, dtype=cand_rows.dtype).view(B, K)
        idx = torch.where(cand_rows >= 0, idx, torch.full_like(idx, -1))
        self._mark("exchange.c3", idx)
        return tq, lq, idx

    def rerank(self, q_tok: torch.Tensor, q_len: torch.Tensor, cand_rows: torch.Tensor):
        B = cand_rows.shape[0]
        p_tok, p_len, prow = self.passages(cand_rows)
        ids, mask, types = build_pairs_dev(q_tok, q_len, p_tok, p_len, prow, self.S,
                                           self.reranker.spec,
                                           with_types=self.reranker.spec.pair_style == 1)
        logits = self.reranker.cross_score_dev(ids, mask, types)[:, 0].view(B, self.K)
        logits = logits.masked_fill(cand_rows < 0, float("-inf"))
        idx = rerank_select_dev(logits, self.k).long()
        out = cand_rows.gather(1, idx), logits.gather(1, idx)
        self._mark("rerank", out[1])
        return out

    def run(self, q_ids, q_mask, q_tok, q_len) -> PipelineResult:
        if self.clock is not None:
            self.clock.start(q_ids)
        q = self.embed(q_ids, q_mask)
        self._mark("embed", q)
        if self.lexical is not None:
            sims, rows = self.retrieve_hybrid(q, q_tok, q_len)
        else:
            sims, rows = self.retrieve(q)
        self._mark("search", rows)
        final_rows, final_logits = self.rerank(q_tok, q_len, rows)
        return PipelineResult(final_rows, final_logits, rows, sims)
