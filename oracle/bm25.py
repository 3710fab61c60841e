"""BM25 top-k and reciprocal-rank fusion (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

BM25 — parity unpinned against the reference: the reference has no lexical scorer (its
``fulltext_search`` node type, schema/view_models.py:276-283, and the merge slot
``fulltext_search_docs``, nodeflow/runners/merge.py:18-20, have no backend).  This restates the
library's own documented definition (DESIGN.md "Hybrid retrieval", k_lex.hip header) in numpy
float32, one rounded operation at a time, so the device result must match it bit for bit:
  idf(t)  = fp32(ln(1 + (N - df + 0.5) / (df + 0.5)))       (fp64, libm log; N, df over live rows)
  avgdl   = fp32(sum(dl live) / N)
  w       = idf * ((tf * (k1 + 1)) / (tf + k1 * ((1 - b) + b * (dl / avgdl))))   (fp32)
  q       = max(1, rint(w * 2^16)) * multiplicity of the term in the query      (integer)
  score   = fp32(sum q) / 2^16, top-k by (score desc, row asc).
A brute-force pure-Python fp64 restatement (``bm25_scores_loop``) cross-checks the vectorised one.

rrf — restates graphiti ``rrf`` (super_rag/graphiti/graphiti_core/search/search_utils.py:1762-1778):
scores[uuid] += 1 / (i + rank_const) over each list in order; sort by score descending, stably (ties
keep first-appearance order); keep scores >= min_score.  Pinned by tests/golden/rrf_fixtures.json,
captured from the real reference function (tests/golden/gen_rrf_fixtures.py).
"""
from __future__ import annotations

import math
from collections import Counter, defaultdict

import numpy as np

SCALE = 65536


def _consts(k1, b):
    k1 = np.float32(k1)
    b = np.float32(b)
    return k1, b, np.float32(1.0) - b, k1 + np.float32(1.0)


def idf32(n_live: int, df: int) -> np.float32:
    return np.float32(math.log(1.0 + (n_live - df + 0.5) / (df + 0.5)))


def avgdl32(dl, live) -> np.float32:
    n = int(np.count_nonzero(live))
    if n == 0:
        return np.float32(1.0)
    return np.float32(float(int(np.asarray(dl, dtype=np.int64)[np.asarray(live, bool)].sum())) / n)


class LexCorpus:
    """Inverted index of the oracle, built with numpy from the C-ABI's document arrays
    (off int64[n+1], terms int32, tf int32, dl int32: distinct terms per document)."""

    def __init__(self, off, terms, tf, dl, live=None):
        self.off = np.asarray(off, dtype=np.int64)
        self.n = len(self.off) - 1
        self.terms = np.asarray(terms, dtype=np.int64)[: self.off[-1]]
        self.tf = np.asarray(tf, dtype=np.int64)[: self.off[-1]]
        self.dl = np.asarray(dl, dtype=np.int64)
        self.live = np.ones(self.n, bool) if live is None else np.asarray(live, bool).copy()
        self.row = np.repeat(np.arange(self.n, dtype=np.int64), np.diff(self.off))
        self._index()

    def _index(self):
        keep = self.live[self.row]
        t, r, f = self.terms[keep], self.row[keep], self.tf[keep]
        order = np.argsort(t, kind="stable")
        self.p_term, self.p_row, self.p_tf = t[order], r[order], f[order]
        self.vocab = int(self.terms.max()) + 1 if self.terms.size else 0
        self.df = np.bincount(self.p_term, minlength=self.vocab)
        self.start = np.concatenate([[0], np.cumsum(self.df)])

    def remove(self, rows):
        self.live[np.asarray(rows, dtype=np.int64)] = False
        self._index()

    def docs(self):
        """Per row the list of (term, tf) (for the scalar restatement)."""
        return [list(zip(self.terms[self.off[i]:self.off[i + 1]].tolist(),
                         self.tf[self.off[i]:self.off[i + 1]].tolist())) for i in range(self.n)]


def bm25_fixed_scores(corpus: LexCorpus, query, k1=1.2, b=0.75, allow=None, stats=None):
    """Fixed-point score (int64) of every row for one query (list of term ids, repeats count);
    0 = no match.  stats = (n_live, sum_dl, df: term -> int) of a whole row-sharded corpus (every
    shard scores its rows with the corpus-wide N, avgdl and df), or None for this corpus's own."""
    k1, b, omb, k1p1 = _consts(k1, b)
    if stats is None:
        n_live = int(corpus.live.sum())
        adl = avgdl32(corpus.dl, corpus.live)
        df_of = lambda t: int(corpus.df[t])
    else:
        n_live, sum_dl, df_of = int(stats[0]), int(stats[1]), stats[2]
        adl = np.float32(float(sum_dl) / n_live) if n_live > 0 else np.float32(1.0)
    acc = np.zeros(corpus.n, dtype=np.int64)
    elig = corpus.live if allow is None else corpus.live & np.asarray(allow, dtype=bool)
    for t, mult in Counter(int(x) for x in query).items():
        if t < 0 or t >= corpus.vocab or corpus.df[t] == 0:
            continue
        s0, s1 = corpus.start[t], corpus.start[t + 1]
        rows, tf = corpus.p_row[s0:s1], corpus.p_tf[s0:s1].astype(np.float32)
        keep = elig[rows]
        rows, tf = rows[keep], tf[keep]
        d = corpus.dl[rows].astype(np.float32)
        idf = idf32(n_live, df_of(t))
        t1 = d / adl
        norm = k1 * (omb + b * t1)
        w = idf * ((tf * k1p1) / (tf + norm))
        q = np.maximum(np.float32(1.0), np.rint(w * np.float32(SCALE))).astype(np.int64)
        acc[rows] += q * mult
    assert acc.max(initial=0) < 2 ** 32, "fixed-point accumulator overflow"
    return acc


def bm25_scores_loop(docs, dl, live, query, k1=1.2, b=0.75):
    """Scalar pure-Python restatement (small cases): float64 BM25 per row, for a tolerance check of
    the fixed-point vectorised path."""
    n_live = sum(1 for x in live if x)
    adl = sum(d for d, x in zip(dl, live) if x) / max(n_live, 1)
    df = Counter(t for r, terms in enumerate(docs) if live[r] for t, _ in terms)
    out = [0.0] * len(docs)
    for t, mult in Counter(query).items():
        if df.get(t, 0) == 0:
            continue
        idf = math.log(1.0 + (n_live - df[t] + 0.5) / (df[t] + 0.5))
        for r, terms in enumerate(docs):
            if not live[r]:
                continue
            for tt, tf in terms:
                if tt == t:
                    out[r] += mult * idf * tf * (k1 + 1) / (tf + k1 * (1 - b + b * dl[r] / adl))
    return out


def bm25_topk(corpus: LexCorpus, queries, k, k1=1.2, b=0.75, allow=None, stats=None):
    """-> (score [B,k] fp32 desc, rows [B,k] int64); -inf / -1 past the matching rows.  stats: as
    bm25_fixed_scores (a list of per-query stats, or one for every query)."""
    B = len(queries)
    scores = np.full((B, k), -np.inf, dtype=np.float32)
    rows = np.full((B, k), -1, dtype=np.int64)
    for i, q in enumerate(queries):
        st = stats[i] if isinstance(stats, list) else stats
        acc = bm25_fixed_scores(corpus, q, k1, b, allow, st)
        hit = np.nonzero(acc)[0]
        order = hit[np.lexsort((hit, -acc[hit]))][:k]
        m = len(order)
        rows[i, :m] = order
        scores[i, :m] = acc[order].astype(np.float32) / np.float32(SCALE)
    return scores, rows


def rrf(results, rank_const=1, min_score=0.0):
    """graphiti rrf over lists of hashable ids -> (ids, scores)."""
    scores = defaultdict(float)
    for result in results:
        for i, u in enumerate(result):
            scores[u] += 1 / (i + rank_const)
    items = sorted(scores.items(), key=lambda kv: kv[1], reverse=True)
    return ([u for u, s in items if s >= min_score], [s for u, s in items if s >= min_score])


def rrf_rows(rows_a, rows_b, k, rank_const=1, min_score=0.0):
    """rrf of per-query row lists (-1 padded) -> (score [B,k] fp64, rows [B,k]); -inf / -1 pad."""
    B = len(rows_a)
    scores = np.full((B, k), -np.inf, dtype=np.float64)
    rows = np.full((B, k), -1, dtype=np.int64)
    for i in range(B):
        a = [int(r) for r in rows_a[i] if r >= 0]
        bb = [int(r) for r in rows_b[i] if r >= 0]
        ids, sc = rrf([a, bb], rank_const, min_score)
        m = min(k, len(ids))
        rows[i, :m] = ids[:m]
        scores[i, :m] = sc[:m]
    return scores, rows
