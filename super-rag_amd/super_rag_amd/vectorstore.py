"""Drop-in vector-store connector: the SeekDB collection replaced by the in-HBM cosine store.

Mirrors SeekDBVectorStoreConnector (super_rag/vectorstore/seekdb_connector.py:31-155):
  * ``__init__(ctx, **kw)`` with ``ctx["collection"]``; ``.store`` is the connector itself
    (embedding_utils.py:95 calls ``connector.store.add``); ``.collection_name``;
  * ``create_collection(vector_size=...)``  (HNSW cosine -> exact cosine, :56-66)
  * ``add(nodes) -> uuid4 string ids``        (:68-85)
  * ``delete(ids=[...])`` / ValueError("ids is required") (:90-96), ``delete_collection()``
  * ``search(QueryWithEmbedding, **kw) -> QueryResult`` with ``score = cosine distance``
    ascending and no ids in the documents (:98-155); the extra kwargs the reference passes
    (limit, score_threshold, filter, search_params, ...) are accepted and ignored, as there.
Opt-in lexical retrieval (ctx ``fulltext``): every added node's text is also indexed for BM25 on
the device (lexical.py, k_lex.hip); ``fulltext_search(text, top_k, keywords)`` backs the
reference's ``fulltext_search`` node type, and ctx ``hybrid`` makes ``search`` fuse the dense and
the BM25 rankings by reciprocal rank on the device (score = rrf score, descending).  Both work on
collections sharded over several devices (ctx ``devices``: lexical.ShardedLex, corpus-wide BM25
statistics), with the same results as one device.
Collections are process-wide (like a server): every connector object for the same collection
name sees the same rows.  Row ids <-> uuid strings, texts and metadata live on the host; vectors
live in HBM.  With ``ctx["snapshot_dir"]`` a collection is reloaded at construction and
re-snapshotted after every add/delete (checkpoint/resume; SeekDB persisted server-side).
"""
from __future__ import annotations

import asyncio

import copy
import json
from collections import OrderedDict
import logging
import os
import threading
import uuid
from typing import Any, Callable, Dict, List, Optional

import numpy as np

from ._native import devices_gate
from .models import DocumentWithScore, QueryResult

logger = logging.getLogger(__name__)

VECTOR_DB_TYPE = "mi355x"
MASK_CACHE_SIZE = 8      # filter masks kept per collection (n_rows bytes each)


def _native_store(dim: int, device: int):
    from .store import NativeStore
    return NativeStore(dim, device=device)


def _native_load(path: str, device: int):
    from .store import NativeStore
    return NativeStore.load(path, device=device)


def _native_lex(device: int):
    from .lexical import NativeLexIndex
    return NativeLexIndex(device)


def _native_lex_load(path: str, device: int):
    from .lexical import NativeLexIndex
    return NativeLexIndex.load(path, device)


_store_factory: Callable = _native_store
_store_loader: Callable = _native_load
_lex_factory: Callable = _native_lex
_lex_loader: Callable = _native_lex_load


def set_store_backend(factory: Callable, loader: Callable | None = None) -> None:
    """Test seam: replace how per-collection stores are created / loaded."""
    global _store_factory, _store_loader
    _store_factory = factory
    _store_loader = loader or _native_load


def set_lex_backend(factory: Callable, loader: Callable | None = None) -> None:
    """Test seam: replace how per-collection lexical indexes are created / loaded."""
    global _lex_factory, _lex_loader
    _lex_factory = factory
    _lex_loader = loader or _native_lex_load


def _make_store(dim: int, device: int, devices: Optional[List[int]]):
    """One store on `device`, or a ShardedStore over ctx["devices"] (one shard per entry)."""
    if devices and len(devices) > 1:
        from .store import ShardedStore
        return ShardedStore(dim, devices, factory=lambda d, dev: _store_factory(d, dev))
    return _store_factory(dim, devices[0] if devices else device)


def _load_store(path: str, device: int, devices: Optional[List[int]]):
    from .store import ShardedStore
    if ShardedStore.is_manifest(path):
        return ShardedStore.load(path, devices or [device], loader=_store_loader)
    if devices and len(devices) > 1:
        raise IOError(f"{path}: a single-device collection cannot load on devices {devices}")
    return _store_loader(path, devices[0] if devices else device)



def _json_copy(v):
    """Deep copy of JSON-like metadata (dict / list / scalars), ~10x cheaper than copy.deepcopy:
    every returned document owns its metadata, as SeekDB's JSON-decoded results did."""
    if isinstance(v, dict):
        return {k: _json_copy(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_json_copy(x) for x in v]
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    return copy.deepcopy(v)


# DocumentWithScore without re-validation for the connector's own, already typed values (text str,
# score float, metadata dict): 100 per request on the per-request path
_make_doc = getattr(DocumentWithScore, "model_construct", DocumentWithScore)

class _Collection:
    def __init__(self, name: str, dim: int, device: int, store=None,
                 devices: Optional[List[int]] = None):
        self.name = name
        self.dim = dim
        self.device = device
        self.devices = devices
        self.store = store if store is not None else _make_store(dim, device, devices)
        self.ids: List[Optional[str]] = []       # row -> uuid (None once deleted)
        self.row_of: Dict[str, int] = {}
        self.texts: List[Optional[str]] = []
        self.metadatas: List[Optional[dict]] = []
        self.lock = threading.RLock()
        self.coalescer = None   # created on first coalesced search (coalesce.py)
        self.text_coalescers: Dict[int, Any] = {}  # encoder id -> fused embed + search batches
        self.version = 0        # bumped on every add / delete / compaction
        # filter -> (version, mask_key, allow mask): a small LRU (each mask is n_rows bytes)
        self.masks: "OrderedDict[str, tuple]" = OrderedDict()
        self.lex = None         # BM25 index over the same rows (ctx "fulltext"), lexical.py
        self.vocab = None
        self.journal = None     # persist.Journal with ctx["snapshot_dir"]

    def ensure_lex(self) -> None:
        """Create the lexical index, back-filling the rows added before it existed.  A collection
        sharded over several devices gets a ShardedLex over the same shards."""
        if self.lex is not None:
            return
        from .lexical import ShardedLex, Vocab, analyze
        vocab = Vocab()
        if hasattr(self.store, "shard_of"):
            lex = ShardedLex(self.store, factory=lambda dev: _lex_factory(dev))
        else:
            lex = _lex_factory(self.device)
        if self.ids:
            lex.add([vocab.doc_ids(analyze(t)) if t is not None else [] for t in self.texts])
            dead = [r for r, u in enumerate(self.ids) if u is None]
            if dead:
                lex.remove(np.asarray(dead, dtype=np.int64))
        self.lex, self.vocab = lex, vocab

    # -- checkpoint / resume (persist.py) ----------------------------------------------------------
    def persist_add(self, first_row: int, vecs, ids, texts, metadatas) -> None:
        if self.journal is None:
            return
        if self.journal.gen is None:
            self.journal.checkpoint(self)          # first base of a new collection
        else:
            self.journal.append_add(first_row, vecs, ids, texts, metadatas)

    def persist_delete(self, rows, compacted: bool) -> None:
        if self.journal is None:
            return
        if compacted or self.journal.gen is None:
            self.journal.checkpoint(self)          # rows were renumbered: new base
        else:
            self.journal.append_delete(rows)

    def maybe_checkpoint(self, ratio: float) -> None:
        j = self.journal
        if j is not None and j.gen is not None and \
                j.journal_bytes() > ratio * j.base_bytes() + (64 << 20):
            j.checkpoint(self)

    def _replay(self, rec: dict) -> None:
        if rec["op"] == "add":
            vecs = self.journal.vectors(rec, self.dim)
            rows = self.store.add(vecs)
            if int(rows[0]) != int(rec["row"]) or len(rows) != len(rec["ids"]):
                raise IOError(f"{self.journal.log_path}: add replays at row {int(rows[0])}, "
                              f"journaled at {rec['row']}")
            if self.lex is not None:
                from .lexical import analyze
                self.lex.add([self.vocab.doc_ids(analyze(t)) for t in rec["texts"]])
            for u, t, m in zip(rec["ids"], rec["texts"], rec["metadatas"]):
                self.row_of[u] = len(self.ids)
                self.ids.append(u)
                self.texts.append(t)
                self.metadatas.append(m)
        elif rec["op"] == "del":
            rows = np.asarray(rec["rows"], dtype=np.int64)
            self.store.remove(rows)
            if self.lex is not None:
                self.lex.remove(rows)
            for r in rows.tolist():
                self.row_of.pop(self.ids[r], None)
                self.ids[r] = self.texts[r] = self.metadatas[r] = None
        else:
            raise IOError(f"{self.journal.log_path}: unknown journal op {rec['op']!r}")

    @classmethod
    def restore(cls, name: str, directory: str, device: int,
                devices: Optional[List[int]] = None) -> Optional["_Collection"]:
        from .persist import Journal
        j = Journal(directory, name)
        meta = j.read_meta()
        if meta is None:
            return None
        gen = meta.get("gen")            # None: the round-1 layout (<name>.srmi, no journal)
        store = _load_store(j.store_path(gen), device, devices)
        n_rows, _ = store.count()
        if n_rows != meta.get("n_rows", len(meta["ids"])) or n_rows != len(meta["ids"]):
            raise IOError(f"snapshot of {name} is inconsistent: {n_rows} stored rows, metadata "
                          f"for {len(meta['ids'])} (generation {gen})")
        c = cls(name, int(meta["dim"]), device, store=store, devices=devices)
        c.ids = meta["ids"]
        c.texts = meta["texts"]
        c.metadatas = meta["metadatas"]
        c.row_of = {u: i for i, u in enumerate(c.ids) if u is not None}
        if "lex_vocab" in meta and os.path.exists(j.lex_path(gen)):
            from .lexical import ShardedLex, Vocab
            if ShardedLex.is_manifest(j.lex_path(gen)):
                if not hasattr(store, "shard_of"):
                    raise IOError(f"{j.lex_path(gen)}: a sharded lexical index for a single-device store")
                c.lex = ShardedLex.load(j.lex_path(gen), store, loader=lambda p, d: _lex_loader(p, d))
            else:
                c.lex = _lex_loader(j.lex_path(gen), device)
            c.vocab = Vocab(meta["lex_vocab"])
        j.gen = gen
        c.journal = j
        for rec in j.records(gen):
            c._replay(rec)
        if gen is None:
            j.checkpoint(c)              # migrate to the journaled layout
        return c


_registry_lock = threading.Lock()
_collections: Dict[str, _Collection] = {}
_mask_serial = 0   # device-mask cache keys (sr_store_search_masked)


def _get(name: str) -> Optional[_Collection]:
    with _registry_lock:
        return _collections.get(name)


class MI355XVectorStoreConnector:
    def __init__(self, ctx: Dict[str, Any], **kwargs: Any):
        self.ctx = ctx
        self.collection_name = ctx["collection"]
        self.vector_size = ctx.get("vector_size", 1024)
        self.distance = ctx.get("distance", "cosine")
        if self.distance != "cosine":
            raise ValueError(f"unsupported distance '{self.distance}' (only cosine)")
        self.device = int(ctx.get("device", os.environ.get("SUPER_RAG_AMD_DEVICE", 0)))
        # ctx "devices": shard the collection's rows over several GPUs (store.ShardedStore)
        devs = ctx.get("devices")
        self.devices = [int(d) for d in devs] if devs else None
        self.snapshot_dir = ctx.get("snapshot_dir")
        self.coalesce = bool(ctx.get("coalesce", True))
        self.max_batch = int(ctx.get("max_batch", 256))
        # opt-in: apply the score_threshold / filter kwargs the reference passes and SeekDB's
        # connector ignores (seekdb_connector.py:99-100).  Off by default = reference behaviour.
        self.honor_score_threshold = bool(ctx.get("honor_score_threshold", False))
        self.honor_filter = bool(ctx.get("honor_filter", False))
        self.compact_ratio = float(ctx.get("compact_ratio", 0.5))
        # opt-in lexical retrieval: BM25 index of the node texts; hybrid = rrf-fused search
        self.hybrid = bool(ctx.get("hybrid", False))
        self.fulltext = bool(ctx.get("fulltext", False)) or self.hybrid
        self.hybrid_k_each = ctx.get("hybrid_k_each")
        self.rrf_rank_const = int(ctx.get("rrf_rank_const", 1))
        self.scan_dtype = str(ctx.get("scan_dtype", "fp16"))   # "fp8": e4m3 scan + fp16 re-score
        self.checkpoint_ratio = float(ctx.get("checkpoint_ratio", 1.0))
        self.store = self
        if self.snapshot_dir and _get(self.collection_name) is None:
            c = _Collection.restore(self.collection_name, self.snapshot_dir, self.device,
                                    self.devices)
            if c is not None:
                with _registry_lock:
                    _collections.setdefault(self.collection_name, c)
        c = _get(self.collection_name)
        if c is not None:
            self._apply_scan_dtype(c)

    def _apply_scan_dtype(self, c: _Collection) -> None:
        if getattr(c, "scan_dtype", "fp16") != self.scan_dtype and hasattr(c.store, "set_scan_dtype"):
            with c.lock:
                c.store.set_scan_dtype(self.scan_dtype)
                c.scan_dtype = self.scan_dtype

    # -- collection lifecycle ---------------------------------------------------------------------
    def _get_or_create(self, dim: int) -> _Collection:
        with _registry_lock:
            c = _collections.get(self.collection_name)
            if c is None:
                c = _Collection(self.collection_name, int(dim), self.device,
                                devices=self.devices)
                if self.snapshot_dir:
                    from .persist import Journal
                    c.journal = Journal(self.snapshot_dir, self.collection_name)
                _collections[self.collection_name] = c
        self._apply_scan_dtype(c)
        return c

    def create_collection(self, **kwargs: Any):
        vector_size = int(kwargs.get("vector_size") or self.vector_size)
        c = self._get_or_create(vector_size)
        if c.dim != vector_size:
            raise ValueError(f"collection {self.collection_name} exists with dimension {c.dim}, "
                             f"not {vector_size}")

    def delete_collection(self):
        with _registry_lock:
            c = _collections.pop(self.collection_name, None)
        if c is not None and hasattr(c.store, "close"):
            c.store.close()
        if self.snapshot_dir:
            from .persist import Journal
            Journal(self.snapshot_dir, self.collection_name).remove_all()

    # -- mutation ---------------------------------------------------------------------------------
    def add(self, nodes) -> List[str]:
        if not nodes:
            return []
        vecs = np.asarray([n.embedding for n in nodes], dtype=np.float32)
        if vecs.ndim != 2:
            raise ValueError("every node needs an embedding of the same dimension")
        c = self._get_or_create(vecs.shape[1])
        if vecs.shape[1] != c.dim:
            raise ValueError(f"embedding dimension {vecs.shape[1]} != collection dimension {c.dim}")
        ids = [str(uuid.uuid4()) for _ in nodes]
        with c.lock:
            if self.fulltext:
                c.ensure_lex()
            rows = c.store.add(vecs)
            if c.lex is not None:
                from .lexical import analyze
                first = c.lex.add([c.vocab.doc_ids(analyze(n.text)) for n in nodes])
                assert first == int(rows[0]), "lexical index out of step with the store"
            first = len(c.ids)
            for u, r, n in zip(ids, rows, nodes):
                assert int(r) == len(c.ids)
                c.ids.append(u)
                c.row_of[u] = int(r)
                c.texts.append(n.text)
                c.metadatas.append(copy.deepcopy(n.metadata) if n.metadata is not None else None)
            c.version += 1
            c.persist_add(first, vecs, ids, c.texts[first:], c.metadatas[first:])
            c.maybe_checkpoint(self.checkpoint_ratio)
        logger.debug("Added %d documents to collection %s", len(ids), self.collection_name)
        return ids

    def delete(self, **delete_kwargs: Any):
        ids = delete_kwargs.get("ids")
        if not ids:
            raise ValueError("ids is required")
        c = _get(self.collection_name)
        if c is None:
            return
        with c.lock:
            rows = [c.row_of.pop(u) for u in ids if u in c.row_of]
            if rows:
                c.store.remove(np.asarray(rows, dtype=np.int64))
                if c.lex is not None:
                    c.lex.remove(np.asarray(rows, dtype=np.int64))
                for r in rows:
                    c.ids[r] = None
                    c.texts[r] = None
                    c.metadatas[r] = None
                n_rows, n_live = c.store.count()
                compacted = bool(n_rows and n_live < (1.0 - self.compact_ratio) * n_rows)
                if compacted:
                    self._compact(c)
                c.version += 1
                c.persist_delete(rows, compacted)
                c.maybe_checkpoint(self.checkpoint_ratio)

    def _compact(self, c: _Collection) -> None:
        remap = c.store.compact()
        if c.lex is not None:
            lremap = c.lex.compact()
            assert np.array_equal(np.asarray(lremap), np.asarray(remap)), "lexical remap differs"
        keep = [i for i, r in enumerate(remap) if r >= 0]
        c.ids = [c.ids[i] for i in keep]
        c.texts = [c.texts[i] for i in keep]
        c.metadatas = [c.metadatas[i] for i in keep]
        c.row_of = {u: i for i, u in enumerate(c.ids)}

    # -- query ------------------------------------------------------------------------------------
    def search(self, query, **kwargs):
        c = _get(self.collection_name)
        if c is None or query.top_k is None or query.top_k <= 0:
            return QueryResult(query=query.query, results=[])
        q = np.asarray(query.embedding, dtype=np.float32)
        flt = kwargs.get("filter") if self.honor_filter else None
        thr = kwargs.get("score_threshold") if self.honor_score_threshold else None
        if self.hybrid:
            # rrf of the dense and the BM25 rankings on the device; score = rrf score (desc)
            return QueryResult(query=query.query,
                               results=self._hybrid(c, q, query.query or "", int(query.top_k), flt))
        if self.coalesce:
            # concurrent single-query searches share one device batch (coalesce.py)
            results = self._coalescer(c)((q, int(query.top_k), flt))
        else:
            results = self._search_batch(c, [(q, int(query.top_k), flt)])[0]
        return QueryResult(query=query.query, results=self._threshold(results, thr))

    async def asearch(self, query, **kwargs):
        """search for a coroutine: a coalesced dense search awaits its device batch without
        holding a worker thread (coalesce.Coalescer.acall); hybrid / uncoalesced searches run
        search in a worker thread.  Same results."""
        c = _get(self.collection_name)
        if c is None or query.top_k is None or query.top_k <= 0 or self.hybrid or not self.coalesce:
            return await asyncio.to_thread(self.search, query, **kwargs)
        q = np.asarray(query.embedding, dtype=np.float32)
        flt = kwargs.get("filter") if self.honor_filter else None
        thr = kwargs.get("score_threshold") if self.honor_score_threshold else None
        results = await self._coalescer(c).acall((q, int(query.top_k), flt))
        return QueryResult(query=query.query, results=self._threshold(results, thr))

    def can_fuse_embed(self, embedding_model) -> bool:
        """Whether asearch_text applies: a coalescing dense connector and this package's
        coalescing EmbeddingService (its encoder and tokenizer in this process)."""
        # (SUPER_RAG_AMD_FUSE_EMBED_SEARCH=0: the two coalesced steps, for A/B measurements)
        if os.environ.get("SUPER_RAG_AMD_FUSE_EMBED_SEARCH", "1") == "0":
            return False
        return (self.coalesce and not self.hybrid and bool(getattr(embedding_model, "coalesce", False))
                and getattr(embedding_model, "encoder", None) is not None
                and getattr(embedding_model, "tokenizer", None) is not None
                and hasattr(type(embedding_model), "_embed_with"))

    async def asearch_text(self, text: str, embedding_model, top_k: int, **kwargs):
        """embed_query + search of one request as ONE coalesced step: concurrent requests' query
        texts are embedded in one device batch and searched in one device batch, back to back,
        by the same leader (instead of an embed batch and then a separate search batch, whose
        coalescers each saw about half the requests in flight).  Same embedding bits (the encoder's
        outputs do not depend on the batch: k_gemm.hip KCHUNK), same search, same errors
        (EmptyTextError before anything runs, BatchProcessingError for a failed device batch)."""
        from .errors import EmptyTextError
        if not text or not text.strip():
            raise EmptyTextError(1)
        c = _get(self.collection_name)
        if c is None or top_k is None or top_k <= 0:
            await embedding_model.aembed_query(text)
            return QueryResult(query=text, results=[])
        flt = kwargs.get("filter") if self.honor_filter else None
        thr = kwargs.get("score_threshold") if self.honor_score_threshold else None
        item = (text.replace("\n", " "), int(top_k), flt)
        results = await self._text_coalescer(c, embedding_model).acall(item)
        return QueryResult(query=text, results=self._threshold(results, thr))

    def _text_coalescer(self, c, em):
        key = id(em.encoder)
        co = c.text_coalescers.get(key)
        if co is None:
            with c.lock:
                co = c.text_coalescers.get(key)
                if co is None:
                    from .coalesce import Coalescer
                    enc, tok, dev_b = em.encoder, em.tokenizer, em.device_batch
                    embed_with = type(em)._embed_with

                    def run(items, c=c):
                        vecs = embed_with(enc, tok, dev_b, [t for t, _, _ in items])
                        return self._search_batch(c, [(vecs[i], k, flt) for i, (_, k, flt) in enumerate(items)])
                    co = Coalescer(run, max_batch=min(self.max_batch, dev_b))
                    c.text_coalescers[key] = co
        return co

    def _coalescer(self, c):
        if c.coalescer is None:
            with c.lock:
                if c.coalescer is None:
                    from .coalesce import Coalescer
                    c.coalescer = Coalescer(lambda items, c=c: self._search_batch(c, items),
                                            max_batch=self.max_batch)
        return c.coalescer

    @staticmethod
    def _threshold(results, thr):
        if thr is None:
            return results
        # similarity = 1 - distance >= threshold (results are distance-ascending: a prefix)
        return [d for d in results if 1.0 - d.score >= float(thr)]

    @staticmethod
    def _allow_mask(c: _Collection, flt):
        """(mask_key, allow[n_rows]) for a filter, cached per collection version."""
        from .filters import canonical, matches
        key = canonical(flt)
        hit = c.masks.get(key)
        if hit is not None and hit[0] == c.version:
            c.masks.move_to_end(key)
            return hit[1], hit[2]
        allow = np.fromiter((u is not None and matches(flt, md)
                             for u, md in zip(c.ids, c.metadatas)), dtype=np.uint8, count=len(c.ids))
        global _mask_serial
        with _registry_lock:
            _mask_serial += 1
            mkey = _mask_serial
        c.masks[key] = (c.version, mkey, allow)
        c.masks.move_to_end(key)
        for k in [k for k, v in c.masks.items() if v[0] != c.version]:
            del c.masks[k]                      # stale: the rows changed since
        while len(c.masks) > MASK_CACHE_SIZE:
            c.masks.popitem(last=False)
        return mkey, allow

    @staticmethod
    def _search_batch(c: _Collection, items) -> List[List[DocumentWithScore]]:
        """[(query vector, top_k, filter)] -> per query [DocumentWithScore] (distance asc, no
        ids).  Queries with the same filter share one device search."""
        out: List[List[DocumentWithScore]] = [[] for _ in items]
        groups: Dict[str, list] = {}
        for i, (_, _, flt) in enumerate(items):
            groups.setdefault("" if flt is None else json.dumps(flt, sort_keys=True, default=str),
                              []).append(i)
        with c.lock:
            for key, idx in groups.items():
                Q = np.stack([np.asarray(items[i][0], dtype=np.float32).reshape(-1) for i in idx])
                kmax = max(items[i][1] for i in idx)
                if key == "":
                    with devices_gate(_store_devices(c.store), "search"):
                        dist, rows = c.store.search(Q, kmax)
                else:
                    mkey, allow = MI355XVectorStoreConnector._allow_mask(c, items[idx[0]][2])
                    with devices_gate(_store_devices(c.store), "search"):
                        dist, rows = c.store.search(Q, kmax, allow=allow, mask_key=mkey)
                for j, i in enumerate(idx):
                    k = items[i][1]
                    out[i] = [_make_doc(text=c.texts[r], score=float(d),
                                        metadata=_json_copy(c.metadatas[r]))
                              for d, r in zip(dist[j, :k].tolist(), rows[j, :k].tolist()) if r >= 0]
        return out

    def _hybrid(self, c: _Collection, q, text: str, k: int, flt) -> List[DocumentWithScore]:
        from .lexical import analyze
        with c.lock:
            c.ensure_lex()
            terms = c.vocab.query_ids(analyze(text))
            k_each = int(self.hybrid_k_each or max(k, 4 * k))
            k_each = min(k_each, 1024)
            k = min(k, 2 * k_each)
            allow, mkey = None, 0
            if flt is not None:
                mkey, allow = self._allow_mask(c, flt)
            with devices_gate(_store_devices(c.store), "search"):
                scores, rows = c.lex.hybrid(c.store, q.reshape(1, -1), [terms], k, k_each,
                                            self.rrf_rank_const, allow=allow, mask_key=mkey)
            return [_make_doc(text=c.texts[r], score=float(s), metadata=_json_copy(c.metadatas[r]))
                    for s, r in zip(scores[0].tolist(), rows[0].tolist()) if r >= 0]

    def fulltext_search(self, query_text: str, top_k: int, keywords: Optional[List[str]] = None,
                        **kwargs: Any) -> List[DocumentWithScore]:
        """BM25 top-k over the collection's texts (the reference's ``fulltext_search`` node,
        FulltextSearchParams{topk, keywords}); score = BM25 score, descending.  ``keywords``, when
        given, replace the query text's terms.  kwargs ``filter`` is honoured with
        ctx["honor_filter"], as in search()."""
        c = _get(self.collection_name)
        if c is None or top_k is None or top_k <= 0:
            return []
        from .lexical import analyze
        text = " ".join(keywords) if keywords else (query_text or "")
        flt = kwargs.get("filter") if self.honor_filter else None
        with c.lock:
            c.ensure_lex()
            terms = c.vocab.query_ids(analyze(text))
            if not terms:
                return []
            allow, mkey = None, 0
            if flt is not None:
                mkey, allow = self._allow_mask(c, flt)
            with devices_gate(_store_devices(c.store), "search"):
                scores, rows = c.lex.search([terms], min(int(top_k), 1024), allow=allow,
                                            mask_key=mkey)
            return [_make_doc(text=c.texts[r], score=float(s), metadata=_json_copy(c.metadatas[r]))
                    for s, r in zip(scores[0].tolist(), rows[0].tolist()) if r >= 0]

    def get_vectors(self, ids: List[str]) -> np.ndarray:
        """Stored (normalised, fp16-rounded) vectors for uuids (with_vectors=True support)."""
        c = _get(self.collection_name)
        if c is None:
            raise KeyError(self.collection_name)
        with c.lock:
            return c.store.get(np.asarray([c.row_of[u] for u in ids], dtype=np.int64))


def _store_devices(store) -> List[int]:
    """The devices a collection's store computes on: every shard's for a ShardedStore (its
    searches run on all of them), else the store's one device."""
    devs = getattr(store, "devices", None)
    return list(devs) if devs else [int(getattr(store, "device", 0))]


class VectorStoreConnectorAdaptor:
    """vectorstore/connector.py:4-15 with the ``"mi355x"`` arm."""

    def __init__(self, vector_store_type, ctx: Dict[str, Any], **kwargs: Any) -> None:
        self.ctx = ctx
        self.vector_store_type = vector_store_type
        if vector_store_type == VECTOR_DB_TYPE:
            self.connector = MI355XVectorStoreConnector(ctx, **kwargs)
        else:
            raise ValueError("unsupported vector store type:", vector_store_type)
