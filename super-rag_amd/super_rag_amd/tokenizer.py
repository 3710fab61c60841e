"""Host-side tokenisation for the in-process encoders.

The reference never tokenises: text goes to remote servers (embedding_service.py:168-175,
rerank_service.py:95-104).  In-process we need token ids: the model's Hugging Face ``tokenizer.json``
(``$SUPER_RAG_AMD_WEIGHTS/<model>/tokenizer.json`` or an explicit path) through the
``tokenizers`` library.  A missing vocabulary is an error; the deterministic hashing tokenizer of
the same id range (synthetic: embeddings only self-consistent, not BGE-compatible) needs the
explicit opt-in ``SUPER_RAG_AMD_SYNTHETIC=1`` (tests, benchmarks) or ``synthetic=True``.
"""
from __future__ import annotations

import logging
import os
import re
import threading
from collections import OrderedDict
from typing import List, Sequence, Tuple

import numpy as np

_WORD = re.compile(r"[぀-ヿ㐀-䶿一-鿿가-힯]|\w+|[^\w\s]",
                   re.UNICODE)
_PUNCT = re.compile(r"[^\w\s]")
_FIRST_ID = 1000  # ids below are reserved for specials / control tokens


def _words_of(text: str) -> List[str]:
    """_WORD.findall(text); for ASCII text without punctuation that is str.split() (every
    whitespace-separated chunk is one \\w+ word), several times faster."""
    if text.isascii() and _PUNCT.search(text) is None:
        return text.split()
    return _WORD.findall(text)
logger = logging.getLogger(__name__)


def _fnv1a(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def longest_first(a: int, b: int, budget: int):
    """Pair lengths kept by Hugging Face fast tokenizers' LongestFirst truncation
    (tokenizers utils/truncation.rs), the tokenizer bge rerankers load."""
    budget = max(budget, 0)
    if a + b <= budget:
        return a, b
    swap = a > b
    n1, n2 = (b, a) if swap else (a, b)
    n2 = n1 if n1 > budget else max(n1, budget - n1)
    if n1 + n2 > budget:
        n1 = budget // 2
        n2 = n1 + budget % 2
    if swap:
        n1, n2 = n2, n1
    return min(a, n1), min(b, n2)


def longest_first_arrays(a: int, b: np.ndarray, budget: int):
    """longest_first for one query length a against an array of passage lengths b."""
    budget = max(budget, 0)
    b = np.asarray(b, dtype=np.int64)
    a_arr = np.full_like(b, a)
    fits = a_arr + b <= budget
    swap = a_arr > b
    n1 = np.where(swap, b, a_arr)
    n2 = np.where(n1 > budget, n1, np.maximum(n1, budget - n1))
    over = n1 + n2 > budget
    n1 = np.where(over, budget // 2, n1)
    n2 = np.where(over, budget // 2 + budget % 2, n2)
    na = np.where(swap, n2, n1)
    nb = np.where(swap, n1, n2)
    na = np.where(fits, a_arr, np.minimum(a_arr, na))
    nb = np.where(fits, b, np.minimum(b, nb))
    return na, nb


class Tokenizer:
    def __init__(self, spec, path: str | None = None, synthetic: bool | None = None,
                 cache_mb: float | None = None):
        from .encoder import ModelAssetsError, synthetic_allowed
        self.spec = spec
        self.max_length = spec.max_length
        self._hf = None
        if path is None and not synthetic:
            d = spec.asset_dir
            if d is not None:
                path = os.path.join(d, "tokenizer.json")
        if path:
            if not os.path.exists(path):
                raise ModelAssetsError(f"tokenizer for {spec.name} not found: {path}")
            from tokenizers import Tokenizer as HFTokenizer
            self._hf = HFTokenizer.from_file(path)
        elif synthetic or (synthetic is None and synthetic_allowed()):
            logger.warning("%s: hashing tokenizer (synthetic opt-in), not the model vocabulary",
                           spec.name)
        else:
            raise ModelAssetsError(
                f"no tokenizer for {spec.name}: set SUPER_RAG_AMD_WEIGHTS to a directory holding "
                f"{spec.name}/tokenizer.json (or pass path=); the hashing tokenizer needs the "
                f"explicit opt-in SUPER_RAG_AMD_SYNTHETIC=1")
        self.synthetic = self._hf is None
        # caches: a search request re-scores passages the collection already holds, so the
        # content ids of recently seen texts are kept -- ONE int32 array per text in an LRU
        # (a hit moves the text to the young end) bounded by bytes (4 per token + the text's
        # length), SUPER_RAG_AMD_TOKEN_CACHE_MB (default 64 MiB per tokenizer) -- and the hashing
        # tokenizer memoises its word ids
        self._cache: "OrderedDict[str, np.ndarray]" = OrderedDict()
        self._cache_bytes = 0
        # one lock around every read-modify of the LRU: the tokenizer is shared between the
        # worker threads of aembed_documents, the coalescer leaders and uncoalesced rerank calls
        # (get + move_to_end / pop + popitem are separate steps; another thread's eviction in
        # between raised KeyError and drifted the byte count).  The HF encode stays outside it.
        self._cache_lock = threading.Lock()
        self._cache_cap_bytes = int(float(os.environ.get("SUPER_RAG_AMD_TOKEN_CACHE_MB", "64")) * (1 << 20)) \
            if cache_mb is None else int(cache_mb * (1 << 20))
        self._words: dict = {}

    # -- content tokens (no specials) -------------------------------------------------------------
    def _lookup_many(self, texts: Sequence[str]) -> List:
        with self._cache_lock:
            out = []
            for t in texts:
                a = self._cache.get(t)
                if a is not None:
                    self._cache.move_to_end(t)
                out.append(a)
            return out

    def cache_misses(self, texts: Sequence[str]) -> int:
        """How many of texts are not in the content-id cache (the LRU order is not touched)."""
        with self._cache_lock:
            return sum(1 for t in texts if t not in self._cache)

    def content_ids(self, text: str) -> List[int]:
        return self._content_arrays_many([text])[0].tolist()

    def content_ids_many(self, texts: Sequence[str]) -> List[List[int]]:
        """content_ids of many texts; the misses of an HF tokenizer go through one encode_batch
        (the Rust tokenizer, parallel) instead of one call each."""
        return [a.tolist() for a in self._content_arrays_many(texts)]

    def _content_arrays_many(self, texts: Sequence[str]) -> List[np.ndarray]:
        """Content ids of many texts as int32 arrays (the cached form; do not modify them)."""
        out: List = self._lookup_many(texts)
        miss = [i for i, o in enumerate(out) if o is None]
        if not miss:
            return out
        if self._hf is not None and len(miss) > 1:
            enc = self._hf.encode_batch([texts[i] for i in miss], add_special_tokens=False)
            ids = [e.ids for e in enc]
        elif self._hf is not None:
            ids = [self._hf.encode(texts[miss[0]], add_special_tokens=False).ids]
        else:
            # memoised words through one C-level map per text; only new words take _word_id
            # (the drop-in tokenises ~100 passages per request under the interpreter lock: 13.9 ->
            # 7-8 ms per 100 passages; one process at 64 callers 280.1 -> 289.1 q/s, profiles/r06_tok/)
            d, wid = self._words, self._word_id
            ids = []
            for i in miss:
                ws = _words_of(texts[i])
                got = list(map(d.get, ws))
                j = -1
                while None in got:  # (new words: rare once the memo is warm)
                    j = got.index(None, j + 1)
                    got[j] = wid(ws[j])
                ids.append(got)
        with self._cache_lock:
            for i, c in zip(miss, ids):
                a = np.asarray(c, dtype=np.int32)
                out[i] = a
                self._remember(texts[i], a)
        return out

    def _word_id(self, w: str) -> int:
        i = self._words.get(w)
        if i is None:
            i = _FIRST_ID + _fnv1a(w.lower()) % (self.spec.vocab_size - _FIRST_ID)
            if len(self._words) < (1 << 20):
                self._words[w] = i
        return i

    def _remember(self, text: str, ids: np.ndarray) -> None:
        # (caller holds _cache_lock)
        cost = 4 * int(ids.size) + len(text) + 64
        if cost > self._cache_cap_bytes:
            return
        old = self._cache.pop(text, None)
        if old is not None:
            self._cache_bytes -= 4 * int(old.size) + len(text) + 64
        while self._cache and self._cache_bytes + cost > self._cache_cap_bytes:
            k, v = self._cache.popitem(last=False)            # least recently used first
            self._cache_bytes -= 4 * int(v.size) + len(k) + 64
        self._cache[text] = ids
        self._cache_bytes += cost

    def content_batch(self, texts: Sequence[str], max_len: int) -> Tuple[np.ndarray, np.ndarray]:
        """[N, max_len] int32 content tokens (truncated, zero padded) and [N] lengths."""
        out = np.zeros((len(texts), max_len), dtype=np.int32)
        lens = np.zeros(len(texts), dtype=np.int32)
        for i, a in enumerate(self._content_arrays_many(texts)):
            ids = a[:max_len]
            out[i, : ids.size] = ids
            lens[i] = ids.size
        return out, lens

    # -- single sequences: [CLS] text [SEP] / <s> text </s> ---------------------------------------
    def encode_batch(self, texts: Sequence[str], max_length: int | None = None):
        """(ids, mask) int32 [B, S], padded to the longest sequence (dynamic padding)."""
        L = min(max_length or self.max_length, self.max_length)
        seqs = []
        for c in self.content_ids_many(texts):
            seqs.append([self.spec.bos_id] + c[: L - 2] + [self.spec.eos_id])
        S = max(len(s) for s in seqs)
        ids = np.full((len(seqs), S), self.spec.pad_id, dtype=np.int32)
        mask = np.zeros((len(seqs), S), dtype=np.int32)
        for i, s in enumerate(seqs):
            ids[i, : len(s)] = s
            mask[i, : len(s)] = 1
        return ids, mask

    # -- (query, passage) pairs for cross-encoders ------------------------------------------------
    def encode_pairs(self, query: str, passages: Sequence[str], max_length: int | None = None):
        """(ids, mask, type_ids) [P, S] with the model's pair layout and 'longest_first'
        truncation (the behaviour of tokenizer(pairs, truncation=True) used by bge rerankers);
        an empty passage is a pair with no passage tokens, like the " " placeholder of
        rerank_service.py:61.  Array form (no per-pair Python lists): the per-request rerank
        path packs ~100 pairs per query under the GIL, the list form cost ~29 us per pair
        (profiles/r03_dropin/); identical output to encode_pairs_ref."""
        L = min(max_length or self.max_length, self.max_length)
        q = np.asarray(self.content_ids(query), dtype=np.int32)
        plist = self._content_arrays_many(passages)
        P = len(plist)
        style = self.spec.pair_style
        nspec = 4 if style == 0 else 3
        nsep = 2 if style == 0 else 1
        bos, eos, pad = self.spec.bos_id, self.spec.eos_id, self.spec.pad_id
        lp = np.fromiter((len(b) for b in plist), dtype=np.int64, count=P)
        na, nb = longest_first_arrays(len(q), lp, L - nspec)
        total = na + nb + nspec
        S = int(total.max()) if P else nspec
        cols = np.arange(S)[None, :]
        ids = np.full((P, S), pad, dtype=np.int32)
        ids[:, 0] = bos
        w = min(len(q), S - 1)
        if w > 0:  # the query slab; its tail past na is overwritten by separators / passage below
            ids[:, 1:1 + w] = q[None, :w]
        rows = np.arange(P)
        for k in range(nsep):
            ids[rows, 1 + na + k] = eos
        # passage tokens: pair i's first nb_i content ids at columns 1 + na_i + nsep ...
        if nb.sum():
            starts = np.zeros(P + 1, dtype=np.int64)
            np.cumsum(lp, out=starts[1:])
            flat = np.concatenate(plist)
            r = np.repeat(rows, nb)
            within = np.arange(int(nb.sum())) - np.repeat(np.cumsum(nb) - nb, nb)
            ids[r, np.repeat(1 + na + nsep, nb) + within] = flat[np.repeat(starts[:-1], nb) + within]
        ids[rows, total - 1] = eos
        mask = (cols < total[:, None]).astype(np.int32)
        ids[mask == 0] = pad
        if style == 0:
            tt = np.zeros((P, S), dtype=np.int32)
        else:
            tt = ((cols >= (na + 2)[:, None]) & (mask == 1)).astype(np.int32)
        return ids, mask, tt

    def encode_pairs_ref(self, query: str, passages: Sequence[str], max_length: int | None = None):
        """The list form of encode_pairs (test reference)."""
        L = min(max_length or self.max_length, self.max_length)
        q = self.content_ids(query)
        style = self.spec.pair_style
        nspec = 4 if style == 0 else 3
        bos, eos = self.spec.bos_id, self.spec.eos_id
        seqs, types = [], []
        for b in self.content_ids_many(passages):
            a = q
            na, nb = longest_first(len(a), len(b), L - nspec)
            a, b = a[:na], b[:nb]
            if style == 0:
                s = [bos] + a + [eos, eos] + b + [eos]
                t = [0] * len(s)
            else:
                s = [bos] + a + [eos] + b + [eos]
                t = [0] * (len(a) + 2) + [1] * (len(b) + 1)
            seqs.append(s)
            types.append(t)
        S = max(len(s) for s in seqs)
        ids = np.full((len(seqs), S), self.spec.pad_id, dtype=np.int32)
        mask = np.zeros((len(seqs), S), dtype=np.int32)
        tt = np.zeros((len(seqs), S), dtype=np.int32)
        for i, (s, t) in enumerate(zip(seqs, types)):
            ids[i, : len(s)] = s
            mask[i, : len(s)] = 1
            tt[i, : len(t)] = t
        return ids, mask, tt
