"""Lexical (BM25) retrieval and dense + lexical hybrid fusion: host side of sr_lex_* /
sr_rrf_fuse / sr_hybrid_search (include/super_rag_mi355x.h).

The reference declares the pieces but ships no backend: a ``fulltext_search`` node type and
``FulltextSearchParams{topk, keywords}`` (schema/view_models.py:276-283, :1043-1047), a
``fulltext_search_docs`` merge slot (nodeflow/runners/merge.py:18-20) and a
``enable_vector_and_fulltext`` collection flag.  Here:

  * ``analyze(text)``: lower-case, Unicode ``\\w+`` tokens (no stemming, no stop words);
  * ``Vocab``: term -> int32 id per collection (persisted with the collection snapshot);
  * ``NativeLexIndex``: the device BM25 index (k_lex.hip): Okapi BM25, k1 = 1.2, b = 0.75, Lucene's
    idf ln(1 + (N - df + 0.5) / (df + 0.5)) over live rows, scores in 2^-16 fixed point;
  * ``rrf_fuse`` / ``hybrid_search``: reciprocal-rank fusion as graphiti's ``rrf``
    (graphiti_core/search/search_utils.py:1762-1778), on the device.
There is no CPU fallback: every entry point needs the HIP library and a GPU.
"""
from __future__ import annotations

import ctypes
import re
from collections import Counter
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _native as N

_TOKEN = re.compile(r"\w+", re.UNICODE)
K1 = 1.2
B = 0.75


def analyze(text: Optional[str]) -> List[str]:
    """Text -> lexical tokens (lower-cased Unicode word characters)."""
    return _TOKEN.findall(text.lower()) if text else []


class Vocab:
    """Term string <-> dense int32 id."""

    def __init__(self, terms: Iterable[str] = ()):
        self.terms: List[str] = []
        self.ids: Dict[str, int] = {}
        for t in terms:
            self.ids.setdefault(t, len(self.terms))
            if len(self.ids) > len(self.terms):
                self.terms.append(t)

    def __len__(self) -> int:
        return len(self.terms)

    def doc_ids(self, tokens: Sequence[str]) -> List[int]:
        """Ids of a document's tokens, adding new terms."""
        out = []
        for t in tokens:
            i = self.ids.get(t)
            if i is None:
                i = self.ids[t] = len(self.terms)
                self.terms.append(t)
            out.append(i)
        return out

    def query_ids(self, tokens: Sequence[str]) -> List[int]:
        """Ids of a query's tokens; unknown terms are dropped (they match no row)."""
        return [self.ids[t] for t in tokens if t in self.ids]


def doc_arrays(docs: Sequence[Sequence[int]]):
    """Token-id lists -> (off int64[n+1], terms int32, tf int32, dl int32): each document's distinct
    terms in first-occurrence order with their counts; dl = token count."""
    off = np.zeros(len(docs) + 1, dtype=np.int64)
    terms: List[int] = []
    tfs: List[int] = []
    dl = np.empty(len(docs), dtype=np.int32)
    for i, d in enumerate(docs):
        c = Counter(d)
        terms.extend(c.keys())
        tfs.extend(c.values())
        off[i + 1] = len(terms)
        dl[i] = len(d)
    return off, np.asarray(terms, dtype=np.int32), np.asarray(tfs, dtype=np.int32), dl


def query_arrays(queries: Sequence[Sequence[int]]):
    qoff = np.zeros(len(queries) + 1, dtype=np.int64)
    flat: List[int] = []
    for i, q in enumerate(queries):
        flat.extend(int(t) for t in q)
        qoff[i + 1] = len(flat)
    qterms = np.asarray(flat if flat else [0], dtype=np.int32)
    return qoff, qterms


class LexGlobalC(ctypes.Structure):
    """sr_lex_global: corpus-wide statistics of a row-sharded lexical corpus."""
    _fields_ = [("n_live", ctypes.c_int64), ("sum_dl", ctypes.c_int64), ("terms", ctypes.c_void_p),
                ("df", ctypes.c_void_p), ("n_terms", ctypes.c_int)]


def _mask(allow, n_rows: int):
    a = np.ascontiguousarray(np.asarray(allow, dtype=np.uint8))
    if a.shape != (n_rows,):
        raise ValueError(f"allow mask must have {n_rows} entries, got {a.shape}")
    return a if n_rows else np.zeros(1, dtype=np.uint8)


class NativeLexIndex:
    """BM25 index over the rows of a store, resident in HBM of one device."""

    def __init__(self, device: int = 0, k1: float = K1, b: float = B, _handle=None):
        self._h = None
        if _handle is None:
            N.require_gpu()
            h = ctypes.c_void_p()
            N.call("sr_lex_create", int(device), float(k1), float(b), ctypes.byref(h))
            _handle = h
        self._h = _handle
        self.device = int(device)

    @classmethod
    def load(cls, path: str, device: int = 0) -> "NativeLexIndex":
        N.require_gpu()
        h = ctypes.c_void_p()
        N.call("sr_lex_load", path.encode(), int(device), ctypes.byref(h))
        return cls(device, _handle=h)

    def close(self) -> None:
        if self._h:
            N.load().sr_lex_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, docs: Sequence[Sequence[int]]) -> int:
        """Append documents (token-id lists); returns the first row id."""
        if not len(docs):
            return self.stats()["rows"]
        return self.add_arrays(*doc_arrays(docs))

    def add_arrays(self, off, terms, tf, dl) -> int:
        """Bulk append of pre-tokenised documents in the C-ABI layout (doc_arrays output:
        off int64[n+1], distinct terms int32 with counts tf int32, lengths dl int32)."""
        off = np.ascontiguousarray(off, dtype=np.int64)
        terms = np.ascontiguousarray(terms, dtype=np.int32)
        tf = np.ascontiguousarray(tf, dtype=np.int32)
        dl = np.ascontiguousarray(dl, dtype=np.int32)
        n = len(off) - 1
        if terms.size == 0:
            terms, tf = np.zeros(1, np.int32), np.ones(1, np.int32)
        first = ctypes.c_int64(0)
        N.call("sr_lex_add", self._h, N.ptr(off), N.ptr(terms), N.ptr(tf), N.ptr(dl), n,
               ctypes.byref(first))
        return int(first.value)

    def remove(self, rows) -> None:
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        N.call("sr_lex_remove", self._h, N.ptr(r), r.shape[0])

    def compact(self) -> np.ndarray:
        n = self.stats()["rows"]
        m = np.empty(max(n, 1), dtype=np.int64)
        N.call("sr_lex_compact", self._h, N.ptr(m))
        return m[:n]

    def save(self, path: str) -> None:
        N.call("sr_lex_save", self._h, path.encode())

    def stats(self) -> dict:
        v = [ctypes.c_int64(0) for _ in range(4)]
        a = ctypes.c_double(0.0)
        N.call("sr_lex_stats", self._h, *[ctypes.byref(x) for x in v], ctypes.byref(a))
        return {"rows": v[0].value, "live": v[1].value, "postings": v[2].value,
                "vocab": v[3].value, "avgdl": a.value}

    def search(self, queries: Sequence[Sequence[int]], k: int, allow=None, mask_key: int = 0,
               global_stats=None, fixed: bool = False):
        """BM25 top-k per query (token-id lists) -> (score [B,k] fp32 desc, rows [B,k] int64).
        global_stats: (n_live, sum_dl, terms, df) of a whole row-sharded corpus (ShardedLex).
        fixed: also return the exact 2^-16 fixed-point scores [B,k] uint32 (sr_lex_search_global_
        fixed; the fp32 scores round above 256), the key a sharded merge orders by."""
        Bq = len(queries)
        scores = np.empty((Bq, k), dtype=np.float32)
        rows = np.empty((Bq, k), dtype=np.int64)
        fx = np.zeros((Bq, k), dtype=np.uint32) if fixed else None
        if Bq == 0:
            return (scores, rows, fx) if fixed else (scores, rows)
        qoff, qterms = query_arrays(queries)
        a = None if allow is None else _mask(allow, self.stats()["rows"])
        g = None
        if global_stats is not None:
            n_live, sum_dl, gt, gdf = global_stats
            gt = np.ascontiguousarray(gt, dtype=np.int32)
            gdf = np.ascontiguousarray(gdf, dtype=np.int64)
            g = LexGlobalC(int(n_live), int(sum_dl), gt.ctypes.data, gdf.ctypes.data, int(gt.size))
        if fixed:
            N.call("sr_lex_search_global_fixed", self._h, N.ptr(qoff), N.ptr(qterms), Bq, int(k),
                   None if a is None else N.ptr(a), int(mask_key),
                   None if g is None else ctypes.byref(g), N.ptr(scores), N.ptr(rows), N.ptr(fx))
            return scores, rows, fx
        if g is None:
            N.call("sr_lex_search", self._h, N.ptr(qoff), N.ptr(qterms), Bq, int(k),
                   None if a is None else N.ptr(a), int(mask_key), N.ptr(scores), N.ptr(rows))
        else:
            N.call("sr_lex_search_global", self._h, N.ptr(qoff), N.ptr(qterms), Bq, int(k),
                   None if a is None else N.ptr(a), int(mask_key), ctypes.byref(g), N.ptr(scores),
                   N.ptr(rows))
        return scores, rows

    def totals(self):
        """(live rows, summed document length) of this index."""
        n, d = ctypes.c_int64(0), ctypes.c_int64(0)
        N.call("sr_lex_totals", self._h, ctypes.byref(n), ctypes.byref(d))
        return int(n.value), int(d.value)

    def df(self, terms) -> np.ndarray:
        """Live document frequency of each term id (0 for unknown terms)."""
        t = np.ascontiguousarray(np.asarray(terms, dtype=np.int32))
        out = np.zeros(t.shape[0], dtype=np.int64)
        if t.size:
            N.call("sr_lex_df", self._h, N.ptr(t), t.shape[0], N.ptr(out))
        return out

    def search_dev(self, qoff, qterms, k: int, global_stats=None, row_offset: int = 0,
                   out_score=None, out_rows=None, stream=None):
        """Device outputs: (score [B,k] fp32, rows [B,k] int64 + row_offset) torch tensors.
        qoff / qterms: host arrays (query_arrays); global_stats: (n_live, sum_dl, terms, df) of the
        whole row-sharded corpus, or None for this index's own statistics."""
        import torch
        qoff = np.ascontiguousarray(qoff, dtype=np.int64)
        qterms = np.ascontiguousarray(qterms, dtype=np.int32)
        Bq = len(qoff) - 1
        dev = torch.device("cuda", self.device)
        if out_score is None:
            out_score = torch.empty((Bq, k), dtype=torch.float32, device=dev)
        if out_rows is None:
            out_rows = torch.empty((Bq, k), dtype=torch.int64, device=dev)
        g = None
        if global_stats is not None:
            n_live, sum_dl, gt, gdf = global_stats
            gt = np.ascontiguousarray(gt, dtype=np.int32)
            gdf = np.ascontiguousarray(gdf, dtype=np.int64)
            g = LexGlobalC(int(n_live), int(sum_dl), gt.ctypes.data, gdf.ctypes.data, int(gt.size))
        N.call("sr_lex_search_dev", self._h, N.ptr(qoff), N.ptr(qterms), Bq, int(k),
               None if g is None else ctypes.byref(g), N.ptr(out_score), N.ptr(out_rows),
               int(row_offset), N.stream_handle(stream))
        return out_score, out_rows

    def query_stats_dev(self, tok, qlen, stream=None):
        """Device-resident queries (torch int32 tok [B, Lq], qlen [B] on this device) -> int64 device
        vector [live rows, summed length, df of every (query, position)]: the statistics a
        row-sharded corpus all-reduces before search_tok_dev (no host synchronisation)."""
        import torch
        tok, qlen = _dev_i32(tok), _dev_i32(qlen)
        B, Lq = tok.shape
        out = torch.empty(2 + B * Lq, dtype=torch.int64, device=tok.device)
        N.call("sr_lex_query_stats_dev", self._h, N.ptr(tok), N.ptr(qlen), B, Lq, N.ptr(out),
               N.stream_handle(stream))
        return out

    def search_tok_dev(self, tok, qlen, k: int, gstats=None, row_offset: int = 0, stream=None):
        """BM25 top-k of device-resident queries (query i = tok[i, :qlen[i]], term ids) -> device
        (score [B, k] fp32, rows [B, k] int64 + row_offset); gstats: the all-reduced
        query_stats_dev vector of a row-sharded corpus, or None for this index's own statistics.
        Identical results to search_dev on the same queries, without a host copy of the queries;
        asynchronous unless the batch exceeds one worst-case query group (B x Lq x max df keys
        over the 2 GiB budget, or B > 1024): then the device-computed per-query caps are read back
        once (one synchronisation of `stream`) to size the groups."""
        import torch
        tok, qlen = _dev_i32(tok), _dev_i32(qlen)
        B, Lq = tok.shape
        score = torch.empty((B, k), dtype=torch.float32, device=tok.device)
        rows = torch.empty((B, k), dtype=torch.int64, device=tok.device)
        if gstats is not None:
            gstats = gstats.contiguous()
            assert gstats.dtype == torch.int64 and gstats.numel() == 2 + B * Lq and gstats.is_cuda
        N.call("sr_lex_search_tok_dev", self._h, N.ptr(tok), N.ptr(qlen), B, Lq, int(k),
               None if gstats is None else N.ptr(gstats), N.ptr(score), N.ptr(rows),
               int(row_offset), N.stream_handle(stream))
        return score, rows

    def hybrid(self, store, queries, query_terms, k: int, k_each: Optional[int] = None,
               rank_const: int = 1, min_score: float = float("-inf"), allow=None, mask_key: int = 0):
        """hybrid_search over (store, this index)."""
        return hybrid_search(store, self, queries, query_terms, k, k_each, rank_const, min_score,
                             allow, mask_key)


class ShardedLex:
    """BM25 index of a row-sharded collection (store.ShardedStore, ctx "devices"): one lexical shard
    per store shard, on the same device and holding the same rows (the store's routing tables), so
    a fulltext / hybrid collection can span GPUs.  Every shard scores with the corpus-wide N,
    summed length and df of the query terms (sr_lex_search_global; the totals and df are summed on
    the host, as the connector's queries are host arrays), each shard's top-k is mapped to global
    rows and the lists merge on (exact 2^-16 fixed-point score desc, global row asc) -- one
    index's order, so results equal a single-device collection's for every score (the shards'
    fp32 scores round above 256; sr_lex_search_global_fixed returns the exact ones).  Global rows are
    the store's: ``add`` must follow the store's add of the same rows (the connector's order)."""

    MAGIC = "SRMILEXSHARDS1"

    def __init__(self, store, factory=None, _shards=None, _tables=None):
        self.store = store
        self.devices = list(store.devices)
        factory = factory or (lambda dev: NativeLexIndex(dev))
        self.shards = _shards if _shards is not None else [factory(d) for d in self.devices]
        self.tables = _tables if _tables is not None else [np.zeros(0, np.int64) for _ in self.devices]

    def _n(self) -> int:
        return sum(len(t) for t in self.tables)

    def add(self, docs) -> int:
        """Documents of global rows [first, first + n) (first = rows so far), each to the shard
        the store put its row on."""
        first = self._n()
        n = len(docs)
        g = np.arange(first, first + n, dtype=np.int64)
        if n and (g[-1] >= len(self.store.shard_of)):
            raise RuntimeError("lexical rows ahead of the store")
        for s, sh in enumerate(self.shards):
            sel = np.nonzero(self.store.shard_of[g] == s)[0] if n else np.zeros(0, np.int64)
            if not sel.size:
                continue
            loc = self.store.local_of[g[sel]]
            got = sh.add([docs[i] for i in sel.tolist()])
            if int(got) != int(loc[0]) or not np.array_equal(loc, np.arange(loc[0], loc[0] + len(loc))):
                raise RuntimeError("lexical shard rows out of step with the store shard")
            self.tables[s] = np.concatenate([self.tables[s], g[sel]])
        return first

    def _route(self, rows):
        r = np.asarray(rows, dtype=np.int64)
        owner = np.full(self._n(), -1, np.int64)
        local = np.full(self._n(), -1, np.int64)
        for s, t in enumerate(self.tables):
            owner[t] = s
            local[t] = np.arange(len(t))
        return r, owner, local

    def remove(self, rows) -> None:
        r, owner, local = self._route(rows)
        for s, sh in enumerate(self.shards):
            sel = r[owner[r] == s]
            if sel.size:
                sh.remove(local[sel])

    def compact(self) -> np.ndarray:
        n = self._n()
        alive = np.zeros(n, bool)
        for s, sh in enumerate(self.shards):
            m = np.asarray(sh.compact())
            keep = m >= 0
            alive[self.tables[s][keep]] = True
            self.tables[s] = self.tables[s][keep]
        remap = np.full(n, -1, np.int64)
        remap[alive] = np.arange(int(alive.sum()))
        self.tables = [remap[t] for t in self.tables]
        return remap

    def stats(self) -> dict:
        out = {"rows": 0, "live": 0}
        for sh in self.shards:
            st = sh.stats()
            out["rows"] += st["rows"]
            out["live"] += st["live"]
        return out

    def totals(self):
        n = d = 0
        for sh in self.shards:
            a, b = sh.totals()
            n, d = n + a, d + b
        return n, d

    def global_stats(self, queries):
        terms = np.unique(np.asarray([int(t) for q in queries for t in q], dtype=np.int64)).astype(np.int32)
        n_live, sum_dl = self.totals()
        df = np.zeros(terms.size, np.int64)
        for sh in self.shards:
            df += np.asarray(sh.df(terms), np.int64)
        return n_live, sum_dl, terms, df

    def search(self, queries, k: int, allow=None, mask_key: int = 0):
        Bq = len(queries)
        st = self.global_stats(queries)
        scores, rows = [], []
        for s, sh in enumerate(self.shards):
            a = None if allow is None else np.asarray(allow, dtype=np.uint8)[self.tables[s]]
            # a shard's device mask cache is keyed per shard (0 = never cached)
            mk = (int(mask_key) << 6) | s if (a is not None and mask_key) else 0
            # merged on the exact fixed-point scores (fp32 rounds them above 256, where a merge
            # on fp32 would order two distinct scores by row): one index's order for every score
            sc, r, fx = sh.search(queries, k, allow=a, mask_key=mk, global_stats=st, fixed=True)
            t = self.tables[s]
            g = np.where(r >= 0, t[np.clip(r, 0, None)] if len(t) else -1, -1)
            scores.append(np.where(g >= 0, np.asarray(fx, np.int64), -1))
            rows.append(g)
        S, R = np.concatenate(scores, 1), np.concatenate(rows, 1)
        out_s = np.full((Bq, k), -np.inf, np.float32)
        out_r = np.full((Bq, k), -1, np.int64)
        for b in range(Bq):
            big = np.where(R[b] >= 0, R[b], np.iinfo(np.int64).max)
            o = np.lexsort((big, -S[b]))[:k]
            ok = R[b][o] >= 0
            out_s[b, : ok.sum()] = S[b][o][ok].astype(np.float32) / np.float32(65536.0)
            out_r[b, : ok.sum()] = R[b][o][ok]
        return out_s, out_r

    def hybrid(self, store, queries, query_terms, k: int, k_each: Optional[int] = None,
               rank_const: int = 1, min_score: float = float("-inf"), allow=None, mask_key: int = 0):
        """Dense top-k_each over the sharded store and BM25 top-k_each over these shards, fused by
        rrf (sr_hybrid_search's three steps on a sharded collection)."""
        k_each = int(k_each or k)
        _, dense = store.search(queries, k_each, allow=allow, mask_key=mask_key)
        _, lex = self.search(query_terms, k_each, allow=allow, mask_key=mask_key)
        return _rrf_rows(dense, lex, k, rank_const, min_score, self.devices[0])

    def save(self, path: str) -> None:
        import json
        import os
        for i, sh in enumerate(self.shards):
            sh.save(f"{path}.s{i}")
        np.savez(f"{path}.rows.tmp.npz", **{f"s{i}": t for i, t in enumerate(self.tables)})
        os.replace(f"{path}.rows.tmp.npz", f"{path}.rows.npz")
        with open(path + ".tmp", "w") as f:
            json.dump({"magic": self.MAGIC, "shards": len(self.shards)}, f)
        os.replace(path + ".tmp", path)

    @classmethod
    def is_manifest(cls, path: str) -> bool:
        with open(path, "rb") as f:
            return cls.MAGIC.encode() in f.read(64)

    @classmethod
    def load(cls, path: str, store, loader=None) -> "ShardedLex":
        import json
        with open(path) as f:
            man = json.load(f)
        if man.get("magic") != cls.MAGIC or int(man["shards"]) != len(store.devices):
            raise IOError(f"{path}: a {man.get('shards')}-shard lexical index cannot load on "
                          f"devices {store.devices}")
        loader = loader or (lambda p, dev: NativeLexIndex.load(p, dev))
        shards = [loader(f"{path}.s{i}", d) for i, d in enumerate(store.devices)]
        with np.load(f"{path}.rows.npz") as z:
            tables = [z[f"s{i}"].astype(np.int64) for i in range(len(store.devices))]
        return cls(store, _shards=shards, _tables=tables)


def _rrf_rows(rows_a, rows_b, k, rank_const, min_score, device):
    """rrf of two host row lists on the device (rrf_fuse), or through the test seam."""
    return _rrf_impl[0](rows_a, rows_b, k, rank_const, min_score, device)


def _dev_i32(t):
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise TypeError("device-resident lexical queries must be CUDA tensors")
    return t.to(torch.int32).contiguous()


def rrf_fuse(rows_a, rows_b, k: int, rank_const: int = 1, min_score: float = 0.0,
             device: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Device rrf of two ranked row lists per query ([B, ka], [B, kb], -1 padded)."""
    N.require_gpu()
    a = np.ascontiguousarray(np.asarray(rows_a, dtype=np.int64))
    b = np.ascontiguousarray(np.asarray(rows_b, dtype=np.int64))
    Bq = a.shape[0]
    assert b.shape[0] == Bq
    scores = np.empty((Bq, k), dtype=np.float64)
    rows = np.empty((Bq, k), dtype=np.int64)
    N.call("sr_rrf_fuse", N.ptr(a), a.shape[1], N.ptr(b), b.shape[1], Bq, int(rank_const),
           float(min_score), int(k), N.ptr(scores), N.ptr(rows), int(device))
    return scores, rows


def rrf_fuse_dev(rows_a, rows_b, k: int, rank_const: int = 1, min_score: float = float("-inf"),
                 stream=None):
    """rrf of two ranked row lists per query on the device (torch int64 [B, ka], [B, kb], -1
    padded) -> (score [B, k] fp64, rows [B, k] int64) device tensors."""
    import torch
    a, b = rows_a.contiguous(), rows_b.contiguous()
    Bq = a.shape[0]
    scores = torch.empty((Bq, k), dtype=torch.float64, device=a.device)
    rows = torch.empty((Bq, k), dtype=torch.int64, device=a.device)
    N.call("sr_rrf_fuse_dev", N.ptr(a), a.shape[1], N.ptr(b), b.shape[1], Bq, int(rank_const),
           float(min_score), int(k), N.ptr(scores), N.ptr(rows), a.device.index or 0,
           N.stream_handle(stream))
    return scores, rows


def hybrid_search(store, lex: NativeLexIndex, queries, query_terms: Sequence[Sequence[int]], k: int,
                  k_each: Optional[int] = None, rank_const: int = 1,
                  min_score: float = float("-inf"), allow=None, mask_key: int = 0):
    """Dense top-k_each (cosine, store) and BM25 top-k_each (lex) fused by rrf on the device ->
    (rrf score [B,k] fp64 desc, rows [B,k] int64)."""
    q = np.ascontiguousarray(np.asarray(queries, dtype=np.float32))
    if q.ndim == 1:
        q = q[None]
    Bq = q.shape[0]
    assert len(query_terms) == Bq
    k_each = int(k_each or k)
    scores = np.empty((Bq, k), dtype=np.float64)
    rows = np.empty((Bq, k), dtype=np.int64)
    if Bq == 0:
        return scores, rows
    qoff, qterms = query_arrays(query_terms)
    a = None if allow is None else _mask(allow, store.count()[0])
    N.call("sr_hybrid_search", store._h, lex._h, N.ptr(q), N.ptr(qoff), N.ptr(qterms), Bq, int(k),
           k_each, int(rank_const), float(min_score), None if a is None else N.ptr(a),
           int(mask_key), N.ptr(scores), N.ptr(rows))
    return scores, rows


_rrf_impl = [lambda a, b, k, rc, ms, dev: rrf_fuse(a, b, k, rc, ms, dev)]


def set_rrf_backend(fn) -> None:
    """Test seam: replace the host-list rrf used by ShardedLex.hybrid (CPU doubles)."""
    _rrf_impl[0] = fn or (lambda a, b, k, rc, ms, dev: rrf_fuse(a, b, k, rc, ms, dev))
