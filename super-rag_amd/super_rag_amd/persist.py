"""Checkpoint / resume of a collection: base snapshot + append-only journal.

SeekDB persisted vectors server-side; the reference's ingest adds one document's chunks per call
(llm/embed/embedding_utils.py:95) and deletes by context_ids (index/vector_and_full_text_index.py:
110-129, :185-210).  Rewriting a 10M-row snapshot on every such call would move > 15 GB per add, so
mutations are journaled and only compaction / journal growth writes a new base:

    <name>.json           commit point: {"gen", "dim", "n_rows", ids, texts, metadatas, lex vocab}
    <name>.g<gen>.srmi    the store's rows at generation gen (sr_store_save: tmp + rename)
    <name>.g<gen>.srlex   the lexical index at gen (when the collection has one)
    <name>.log            JSON lines {"g": gen, "op": "add" | "del", ...}, one per mutation
    <name>.vlog           the added fp32 vectors, raw, addressed by byte offset from the log

A checkpoint writes the gen+1 base files, then replaces <name>.json (atomic rename: the commit),
then resets the journal and removes the gen files.  Restore loads the base named by the json,
checks its row count, and replays the journal lines of that generation in order; a torn last line
(crash mid-append) is cut off the log before anything is appended after it (otherwise the next
record would be glued onto the fragment and the whole line lost on the restore after that), and
lines of older generations are ignored.  Replaying an add re-inserts the
same fp32 vectors through the same normalisation, so the restored rows are bit-identical.
Journal bytes per add are proportional to the rows added (vectors 4·dim B per row + their text
and metadata), independent of the collection size.
"""
from __future__ import annotations

import json
import os
import re
from typing import List, Optional

import numpy as np


def _fsync_write(f, data) -> None:
    f.write(data)
    f.flush()
    os.fsync(f.fileno())


class Journal:
    def __init__(self, directory: str, name: str):
        self.dir = directory
        self.name = name
        self.base = os.path.join(directory, name)
        self.gen: Optional[int] = None          # generation of the committed base

    # -- paths --------------------------------------------------------------------------------------
    @property
    def meta_path(self) -> str:
        return self.base + ".json"

    def store_path(self, gen: Optional[int]) -> str:
        return self.base + (".srmi" if gen is None else f".g{gen}.srmi")

    def lex_path(self, gen: Optional[int]) -> str:
        return self.base + (".srlex" if gen is None else f".g{gen}.srlex")

    @property
    def log_path(self) -> str:
        return self.base + ".log"

    @property
    def vlog_path(self) -> str:
        return self.base + ".vlog"

    def journal_bytes(self) -> int:
        return sum(os.path.getsize(p) for p in (self.log_path, self.vlog_path) if os.path.exists(p))

    def base_bytes(self) -> int:
        """Bytes of the committed base: the store file plus, for a sharded collection, its shard
        stores and row tables (<name>.g<gen>.srmi is then only the manifest), plus the lexical
        index, so the checkpoint ratio compares the journal with the real snapshot size."""
        if self.gen is None or not os.path.isdir(self.dir):
            return 0
        pat = self._pattern(re.escape(f".g{self.gen}"))
        return sum(os.path.getsize(os.path.join(self.dir, fn)) for fn in os.listdir(self.dir)
                   if pat.fullmatch(fn) and not fn.endswith(".tmp"))

    def _sync_generation(self, gen: int) -> None:
        """fsync every file of base generation `gen` and the directory, before the commit names it."""
        pat = self._pattern(re.escape(f".g{gen}"))
        for fn in os.listdir(self.dir):
            if pat.fullmatch(fn) and not fn.endswith(".tmp"):
                fd = os.open(os.path.join(self.dir, fn), os.O_RDONLY)
                try:
                    os.fsync(fd)
                finally:
                    os.close(fd)
        self._sync_dir()

    def _sync_dir(self) -> None:
        fd = os.open(self.dir, os.O_RDONLY)
        try:
            os.fsync(fd)
        finally:
            os.close(fd)

    # -- checkpoint -----------------------------------------------------------------------------------
    def checkpoint(self, c) -> None:
        """Write the full state of collection `c` as generation gen+1 and reset the journal."""
        os.makedirs(self.dir, exist_ok=True)
        gen = (self.gen or 0) + 1
        c.store.save(self.store_path(gen))
        n_rows, _ = c.store.count()
        meta = {"gen": gen, "dim": c.dim, "n_rows": int(n_rows), "ids": c.ids, "texts": c.texts,
                "metadatas": c.metadatas}
        if c.lex is not None:
            c.lex.save(self.lex_path(gen))
            meta["lex_vocab"] = c.vocab.terms
        self._sync_generation(gen)                            # base bytes durable before the commit
        tmp = self.meta_path + ".tmp"
        with open(tmp, "w", encoding="utf-8") as f:
            _fsync_write(f, json.dumps(meta))
        os.replace(tmp, self.meta_path)                       # commit
        self._sync_dir()
        old = self.gen
        self.gen = gen
        for p in (self.log_path, self.vlog_path):
            if os.path.exists(p):
                os.remove(p)
        self._remove_generation(old)

    def _pattern(self, gen_re: str) -> "re.Pattern":
        n = re.escape(self.name)
        return re.compile(n + gen_re + r"\.(srmi|srlex)(\.s\d+|\.rows(\.tmp)?\.npz)?(\.tmp)?")

    def _remove_generation(self, gen: Optional[int]) -> None:
        """Files of one base generation (store, shard stores and tables, lexical index)."""
        pat = self._pattern("" if gen is None else re.escape(f".g{gen}"))
        for fn in os.listdir(self.dir):
            if pat.fullmatch(fn):
                os.remove(os.path.join(self.dir, fn))

    # -- journal --------------------------------------------------------------------------------------
    def _append(self, rec: dict) -> None:
        with open(self.log_path, "a", encoding="utf-8") as f:
            _fsync_write(f, json.dumps(rec) + "\n")

    def append_add(self, first_row: int, vecs: np.ndarray, ids: List[str], texts: List[str],
                   metadatas: List[Optional[dict]]) -> None:
        v = np.ascontiguousarray(np.asarray(vecs, dtype=np.float32))
        with open(self.vlog_path, "ab") as f:
            off = f.tell()
            _fsync_write(f, v.tobytes())
        self._append({"g": self.gen, "op": "add", "row": int(first_row), "n": int(v.shape[0]),
                      "off": off, "ids": ids, "texts": texts, "metadatas": metadatas})

    def append_delete(self, rows) -> None:
        self._append({"g": self.gen, "op": "del", "rows": [int(r) for r in rows]})

    # -- restore --------------------------------------------------------------------------------------
    def read_meta(self) -> Optional[dict]:
        if not os.path.exists(self.meta_path):
            return None
        with open(self.meta_path, encoding="utf-8") as f:
            return json.load(f)

    def records(self, gen) -> List[dict]:
        """Journal lines of generation `gen`, in order.  A torn last line (a crash mid-append:
        never acknowledged) is dropped AND truncated away, so the next _append starts on a fresh
        line instead of extending the fragment into a line no later restore could parse."""
        if not os.path.exists(self.log_path):
            return []
        out = []
        good = 0                                   # byte offset just past the last complete line
        with open(self.log_path, "rb") as f:
            for line in f:
                if not line.endswith(b"\n"):
                    break
                good += len(line)
                rec = json.loads(line.decode("utf-8"))
                if rec.get("g") == gen:
                    out.append(rec)
        if good != os.path.getsize(self.log_path):
            os.truncate(self.log_path, good)
            fd = os.open(self.log_path, os.O_RDONLY)
            try:
                os.fsync(fd)
            finally:
                os.close(fd)
        return out

    def vectors(self, rec: dict, dim: int) -> np.ndarray:
        n = int(rec["n"])
        with open(self.vlog_path, "rb") as f:
            f.seek(int(rec["off"]))
            buf = f.read(n * dim * 4)
        if len(buf) != n * dim * 4:
            raise IOError(f"{self.vlog_path}: truncated vectors for the add at row {rec['row']}")
        return np.frombuffer(buf, dtype=np.float32).reshape(n, dim)

    def remove_all(self) -> None:
        """Delete every file of this collection (and only this collection's)."""
        if not os.path.isdir(self.dir):
            return
        base = self._pattern(r"(\.g\d+)?")
        own = re.compile(re.escape(self.name) + r"\.(json|json\.tmp|log|vlog)")
        for fn in os.listdir(self.dir):
            if base.fullmatch(fn) or own.fullmatch(fn):
                os.remove(os.path.join(self.dir, fn))
