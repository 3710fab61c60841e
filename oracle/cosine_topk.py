"""Exact cosine top-k (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Restates the SeekDB cosine collection as the reference uses it:
  * super_rag/vectorstore/seekdb_connector.py:56-66   HNSWConfiguration(distance="cosine")
  * super_rag/vectorstore/seekdb_connector.py:98-115  collection.query(query_embeddings, n_results=top_k)
  * super_rag/vectorstore/seekdb_connector.py:117-155 DocumentWithScore(score=distance), ascending
Distance is 1 - cos(q, x) computed in fp64; results ordered by (distance asc, row asc) — the HNSW
ordering of SeekDB is approximate and unpinned, the exact order is the contract here.
Zero vectors get similarity 0 (graphiti_core/helpers.py:100-103 normalize_l2 guard).
"""
from __future__ import annotations

import numpy as np


def normalize_rows(x: np.ndarray) -> np.ndarray:
    """L2-normalise rows in fp64; zero rows stay zero."""
    x = np.asarray(x, dtype=np.float64)
    n = np.linalg.norm(x, axis=-1, keepdims=True)
    return np.divide(x, n, out=np.zeros_like(x), where=n > 0)


def quantize_like_store(x: np.ndarray) -> np.ndarray:
    """What the MI355X store keeps: fp32 row normalisation, then rounding to fp16."""
    x32 = np.asarray(x, dtype=np.float32)
    n = np.sqrt((x32.astype(np.float32) ** 2).sum(axis=-1, keepdims=True, dtype=np.float32))
    inv = np.divide(np.float32(1.0), n, out=np.zeros_like(n), where=n > 0)
    return (x32 * inv).astype(np.float16)


def cosine_topk(corpus: np.ndarray, queries: np.ndarray, k: int, live: np.ndarray | None = None,
                normalize: bool = True, chunk: int = 65536):
    """Return (dist[B,k] fp64, rows[B,k] int64), rows sorted by (dist asc, row asc).

    Missing entries (k > live rows) are dist=+inf, row=-1, as the C-ABI reports them.
    ``normalize=False`` uses the rows as given (e.g. fp16 rows read back from the store).
    """
    q = np.asarray(queries, dtype=np.float64)
    if normalize:
        q = normalize_rows(q)
    B = q.shape[0]
    n = corpus.shape[0]
    best_s = np.full((B, 0), -np.inf)
    best_r = np.zeros((B, 0), dtype=np.int64)
    for r0 in range(0, n, chunk):
        c = np.asarray(corpus[r0:r0 + chunk], dtype=np.float64)
        if normalize:
            c = normalize_rows(c)
        s = q @ c.T
        if live is not None:
            s[:, ~np.asarray(live[r0:r0 + chunk], dtype=bool)] = -np.inf
        rows = np.broadcast_to(np.arange(r0, r0 + c.shape[0], dtype=np.int64), s.shape)
        best_s = np.concatenate([best_s, s], axis=1)
        best_r = np.concatenate([best_r, rows], axis=1)
        # keep the k best by (sim desc, row asc): lexsort keys, last is primary
        order = np.lexsort((best_r, -best_s), axis=1)[:, :k]
        best_s = np.take_along_axis(best_s, order, axis=1)
        best_r = np.take_along_axis(best_r, order, axis=1)
    dist = np.full((B, k), np.inf)
    rows_out = np.full((B, k), -1, dtype=np.int64)
    m = best_s.shape[1]
    valid = np.isfinite(best_s)
    dist[:, :m] = np.where(valid, 1.0 - best_s, np.inf)
    rows_out[:, :m] = np.where(valid, best_r, -1)
    return dist, rows_out


def recall_at_k(found: np.ndarray, truth: np.ndarray) -> float:
    """Mean |found ∩ truth| / |truth| over queries (rows < 0 ignored)."""
    tot, hit = 0, 0
    for f, t in zip(found, truth):
        ts = {int(x) for x in t if x >= 0}
        fs = {int(x) for x in f if x >= 0}
        tot += len(ts)
        hit += len(ts & fs)
    return hit / max(tot, 1)


def same_topk_modulo_ties(rows_a, sims_a, rows_ref, sims_ref, eps: float) -> bool:
    """Identical id sets, except that ids whose reference similarity lies within eps of the k-th
    reference similarity may be exchanged (fp ties)."""
    for ra, sa, rr, sr in zip(rows_a, sims_a, rows_ref, sims_ref):
        ra = [int(x) for x in ra if x >= 0]
        rr_l = [int(x) for x in rr if x >= 0]
        if len(ra) != len(rr_l):
            return False
        if set(ra) == set(rr_l):
            continue
        kth = float(np.min(np.asarray(sr)[: len(rr_l)]))
        ref = {int(r): float(s) for r, s in zip(rr, sr) if r >= 0}
        got = {int(r): float(s) for r, s in zip(ra, sa)}
        for r in set(rr_l) ^ set(ra):
            s = ref.get(r, got.get(r))
            if s is None or abs(s - kth) > eps:
                return False
    return True
