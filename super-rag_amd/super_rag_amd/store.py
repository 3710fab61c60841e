"""Python handle of the in-HBM cosine store (sr_store_* in include/super_rag_mi355x.h)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N


class NativeStore:
    """Exact cosine top-k over L2-normalised fp16 rows resident in HBM of one device.

    Row ids are int64 positions (append order); the vector-store connector maps them to the
    uuid strings the reference hands out (seekdb_connector.py:68-85).
    """

    def __init__(self, dim: int, device: int = 0, capacity: int = 1024, _handle=None):
        self._h = None
        if _handle is None:
            N.require_gpu()
            h = ctypes.c_void_p()
            N.call("sr_store_create", int(dim), int(device), int(capacity), ctypes.byref(h))
            _handle = h
        self._h = _handle
        self.device = int(device)
        d = ctypes.c_int32(0)
        N.call("sr_store_dim", self._h, ctypes.byref(d))
        self.dim = int(d.value)

    @classmethod
    def load(cls, path: str, device: int = 0) -> "NativeStore":
        N.require_gpu()
        h = ctypes.c_void_p()
        N.call("sr_store_load", path.encode(), int(device), ctypes.byref(h))
        return cls(0, device, _handle=h)

    def close(self) -> None:
        if self._h:
            N.load().sr_store_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- mutation ---------------------------------------------------------------------------------
    def add(self, vecs) -> np.ndarray:
        v = np.ascontiguousarray(np.asarray(vecs, dtype=np.float32))
        if v.ndim != 2 or v.shape[1] != self.dim:
            raise ValueError(f"expected (n, {self.dim}) vectors, got {v.shape}")
        rows = np.empty(v.shape[0], dtype=np.int64)
        N.call("sr_store_add", self._h, N.ptr(v), v.shape[0], N.ptr(rows))
        return rows

    def add_dev(self, vecs, stream=None) -> int:
        """Append rows from a device tensor (fp32/fp16, [n, dim]); returns the first row id."""
        import torch
        assert vecs.is_cuda and vecs.is_contiguous() and vecs.shape[1] == self.dim
        dt = N.SR_DTYPE_F16 if vecs.dtype == torch.float16 else N.SR_DTYPE_F32
        if vecs.dtype not in (torch.float16, torch.float32):
            raise TypeError("add_dev: fp16 or fp32 rows")
        first = ctypes.c_int64(0)
        N.call("sr_store_add_dev", self._h, N.ptr(vecs), dt, vecs.shape[0], ctypes.byref(first),
               N.stream_handle(stream))
        return int(first.value)

    def remove(self, rows) -> None:
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        N.call("sr_store_remove", self._h, N.ptr(r), r.shape[0])

    def compact(self) -> np.ndarray:
        n, _ = self.count()
        m = np.empty(max(n, 1), dtype=np.int64)
        N.call("sr_store_compact", self._h, N.ptr(m))
        return m[:n]

    def set_scan_dtype(self, dtype: str) -> None:
        """"fp16" (default) or "fp8": scan an OCP e4m3 copy of the rows with the block-scaled fp8
        MFMA and re-score the candidates exactly on the fp16 rows (sr_store_set_scan_dtype)."""
        code = {"fp16": N.SR_DTYPE_F16, "fp8": N.SR_DTYPE_FP8_E4M3}[dtype]
        N.call("sr_store_set_scan_dtype", self._h, code)

    def save(self, path: str) -> None:
        N.call("sr_store_save", self._h, path.encode())

    # -- queries ----------------------------------------------------------------------------------
    def count(self):
        n, live = ctypes.c_int64(0), ctypes.c_int64(0)
        N.call("sr_store_count", self._h, ctypes.byref(n), ctypes.byref(live))
        return int(n.value), int(live.value)

    def get(self, rows) -> np.ndarray:
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        out = np.empty((r.shape[0], self.dim), dtype=np.float32)
        N.call("sr_store_get", self._h, N.ptr(r), r.shape[0], N.ptr(out))
        return out

    def search(self, queries, k: int, allow=None, mask_key: int = 0):
        """Host path: returns (dist [B,k] fp32, rows [B,k] int64); dist = 1 - cos, ascending.
        ``allow`` (bool/uint8 [n_rows]) restricts the candidates to the allowed rows (the mask is
        cached on the device while ``mask_key`` != 0 and the store is unchanged)."""
        q = np.ascontiguousarray(np.asarray(queries, dtype=np.float32))
        if q.ndim == 1:
            q = q[None]
        if q.shape[1] != self.dim:
            raise ValueError(f"query dim {q.shape[1]} != store dim {self.dim}")
        B = q.shape[0]
        dist = np.empty((B, k), dtype=np.float32)
        rows = np.empty((B, k), dtype=np.int64)
        if allow is None:
            N.call("sr_store_search", self._h, N.ptr(q), B, int(k), N.ptr(dist), N.ptr(rows))
        else:
            n, _ = self.count()
            a = np.ascontiguousarray(np.asarray(allow, dtype=np.uint8))
            if a.shape != (n,):
                raise ValueError(f"allow mask must have {n} entries, got {a.shape}")
            if n == 0:
                a = np.zeros(1, dtype=np.uint8)
            N.call("sr_store_search_masked", self._h, N.ptr(q), B, int(k), N.ptr(a), int(mask_key),
                   N.ptr(dist), N.ptr(rows))
        return dist, rows

    def search_sim(self, queries, k: int, allow=None, mask_key: int = 0):
        """search() returning (sim [B,k] fp32 descending, -inf when missing; rows [B,k]): the
        exact similarities, for merging several stores' lists (ShardedStore)."""
        q = np.ascontiguousarray(np.asarray(queries, dtype=np.float32))
        if q.ndim == 1:
            q = q[None]
        if q.shape[1] != self.dim:
            raise ValueError(f"query dim {q.shape[1]} != store dim {self.dim}")
        B = q.shape[0]
        sim = np.empty((B, k), dtype=np.float32)
        rows = np.empty((B, k), dtype=np.int64)
        a = None
        if allow is not None:
            n, _ = self.count()
            a = np.ascontiguousarray(np.asarray(allow, dtype=np.uint8))
            if a.shape != (n,):
                raise ValueError(f"allow mask must have {n} entries, got {a.shape}")
            if n == 0:
                a = np.zeros(1, dtype=np.uint8)
        N.call("sr_store_search_sim", self._h, N.ptr(q), B, int(k), N.ptr(a) if a is not None else None,
               int(mask_key) if a is not None else 0, N.ptr(sim), N.ptr(rows))
        return np.where(rows >= 0, sim, -np.inf).astype(np.float32), rows

    def search_dev(self, q, k: int, out_sim=None, out_rows=None, row_offset: int = 0, stream=None):
        """Device path: q [B, >=dim] fp16/fp32 device tensor (only the first `dim` columns are
        read when q is exactly [B, dim]; a padded fp16 [B, ld] query must be sliced by the caller).
        Returns (sim [B,k] fp32, rows [B,k] int64) device tensors."""
        import torch
        assert q.is_cuda and q.is_contiguous() and q.shape[1] == self.dim
        B = q.shape[0]
        dt = N.SR_DTYPE_F16 if q.dtype == torch.float16 else N.SR_DTYPE_F32
        if out_sim is None:
            out_sim = torch.empty((B, k), dtype=torch.float32, device=q.device)
        if out_rows is None:
            out_rows = torch.empty((B, k), dtype=torch.int64, device=q.device)
        N.call("sr_store_search_dev", self._h, N.ptr(q), dt, B, int(k), N.ptr(out_sim),
               N.ptr(out_rows), int(row_offset), N.stream_handle(stream))
        return out_sim, out_rows


def topk_merge_dev(sims, rows, k_out: int, device: int = 0, stream=None):
    """Merge [P, B, k] per-shard lists (device tensors) into [B, k_out] (sim desc, row asc)."""
    import torch
    P, B, k = sims.shape
    out_sim = torch.empty((B, k_out), dtype=torch.float32, device=sims.device)
    out_rows = torch.empty((B, k_out), dtype=torch.int64, device=sims.device)
    N.call("sr_topk_merge_dev", N.ptr(sims.contiguous()), N.ptr(rows.contiguous()), P, B, k,
           int(k_out), N.ptr(out_sim), N.ptr(out_rows), int(device), N.stream_handle(stream))
    return out_sim, out_rows


class NativeStoreSet:
    """One collection row-sharded over several devices behind ONE native handle
    (sr_store_set_*, SURVEY §8(b)'s sr_store_create(dim, dtype, devices, n_dev)): the library keeps
    one in-HBM store per listed device, hands out global row ids in insertion order, searches the
    shards concurrently and merges by (distance asc, row asc) — results equal one NativeStore's.
    Host-buffer interface (add / remove / get / count / search with an optional allow mask);
    snapshots, compaction and the device-buffer paths stay with ShardedStore / NativeStore."""

    def __init__(self, dim: int, devices, dtype: str = "fp16"):
        N.require_gpu()
        devs = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
        if devs.size == 0:
            raise ValueError("NativeStoreSet needs at least one device")
        code = {"fp16": N.SR_DTYPE_F16, "fp8": N.SR_DTYPE_FP8_E4M3}[dtype]
        self._h = None
        h = ctypes.c_void_p()
        N.call("sr_store_set_create", int(dim), code, N.ptr(devs), int(devs.size), ctypes.byref(h))
        self._h = h
        self.dim = int(dim)
        self.devices = [int(d) for d in devs]

    def close(self) -> None:
        if self._h:
            N.load().sr_store_set_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add(self, vecs) -> np.ndarray:
        v = np.ascontiguousarray(np.asarray(vecs, dtype=np.float32))
        if v.ndim != 2 or v.shape[1] != self.dim:
            raise ValueError(f"expected (n, {self.dim}) vectors, got {v.shape}")
        rows = np.empty(v.shape[0], dtype=np.int64)
        N.call("sr_store_set_add", self._h, N.ptr(v), int(v.shape[0]), N.ptr(rows))
        return rows

    def remove(self, rows) -> None:
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        N.call("sr_store_set_remove", self._h, N.ptr(r), int(r.size))

    def count(self):
        n, live, sh = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
        N.call("sr_store_set_count", self._h, ctypes.byref(n), ctypes.byref(live), ctypes.byref(sh))
        return int(n.value), int(live.value)

    def get(self, rows) -> np.ndarray:
        r = np.ascontiguousarray(np.asarray(rows, dtype=np.int64))
        out = np.empty((r.size, self.dim), dtype=np.float32)
        N.call("sr_store_set_get", self._h, N.ptr(r), int(r.size), N.ptr(out))
        return out

    def set_scan_dtype(self, dtype: str) -> None:
        N.call("sr_store_set_set_scan_dtype", self._h,
               {"fp16": N.SR_DTYPE_F16, "fp8": N.SR_DTYPE_FP8_E4M3}[dtype])

    def search(self, queries, k: int, allow=None, mask_key: int = 0):
        q = np.ascontiguousarray(np.asarray(queries, dtype=np.float32))
        if q.ndim == 1:
            q = q[None]
        if q.shape[1] != self.dim:
            raise ValueError(f"query dim {q.shape[1]} != store dim {self.dim}")
        B = q.shape[0]
        dist = np.empty((B, k), dtype=np.float32)
        rows = np.empty((B, k), dtype=np.int64)
        a = None
        if allow is not None:
            n, _ = self.count()
            a = np.ascontiguousarray(np.asarray(allow, dtype=np.uint8))
            if a.shape != (n,):
                raise ValueError(f"allow mask must have {n} entries, got {a.shape}")
        N.call("sr_store_set_search", self._h, N.ptr(q), B, int(k),
               N.ptr(a) if a is not None else None, int(mask_key) if a is not None else 0,
               N.ptr(dist), N.ptr(rows))
        return dist, rows


class ShardedStore:
    """One collection row-sharded over several stores / devices (VECTOR_DB_CONTEXT "devices").

    Same host interface as NativeStore.  Global row ids are the insertion order across all shards
    (exactly the ids one NativeStore would hand out), so results equal a single store's: each add
    batch goes to the shard with the fewest rows (ties: lowest index), a per-shard table maps its
    local rows to global rows.  search() without a filter runs K1 + K2 on every device (each on
    its current stream, so the devices scan concurrently), maps local rows to global rows on the
    device, moves the (B, k) lists to the first device and merges them there with K2 topk_merge
    (sr_topk_merge_dev: similarity desc, global row asc).  Filtered searches run each shard's
    masked search and merge the short lists on the host with the same order.

    ``factory(dim, device)`` builds one shard (NativeStore; test doubles on CPU).
    """

    MAGIC = "SRMISHARDS1"

    def __init__(self, dim: int, devices, factory=None, _shards=None, _tables=None):
        self.dim = int(dim)
        self.devices = [int(d) for d in devices]
        if not self.devices:
            raise ValueError("ShardedStore needs at least one device")
        factory = factory or (lambda d, dev: NativeStore(d, device=dev))
        self.shards = _shards if _shards is not None else [factory(self.dim, d) for d in self.devices]
        self.tables = _tables if _tables is not None else [np.zeros(0, np.int64) for _ in self.devices]
        self._rebuild_index()
        self._dev_tables = None      # per-shard global-row tables on the devices (lazy)

    def _rebuild_index(self) -> None:
        n = sum(len(t) for t in self.tables)
        self.shard_of = np.full(n, -1, np.int32)
        self.local_of = np.full(n, -1, np.int64)
        for s, t in enumerate(self.tables):
            self.shard_of[t] = s
            self.local_of[t] = np.arange(len(t))

    # -- mutation -----------------------------------------------------------------------------------
    def add(self, vecs) -> np.ndarray:
        v = np.ascontiguousarray(np.asarray(vecs, dtype=np.float32))
        if v.ndim != 2 or v.shape[1] != self.dim:
            raise ValueError(f"expected (n, {self.dim}) vectors, got {v.shape}")
        s = int(np.argmin([len(t) for t in self.tables]))
        first = len(self.shard_of)
        local = self.shards[s].add(v)
        if len(local) and int(local[0]) != len(self.tables[s]):
            raise RuntimeError("shard row numbering out of step")
        rows = np.arange(first, first + v.shape[0], dtype=np.int64)
        self.tables[s] = np.concatenate([self.tables[s], rows])
        self.shard_of = np.concatenate([self.shard_of, np.full(len(rows), s, np.int32)])
        self.local_of = np.concatenate([self.local_of, np.asarray(local, np.int64)])
        self._dev_tables = None
        return rows

    def remove(self, rows) -> None:
        r = np.asarray(rows, dtype=np.int64)
        for s in range(len(self.shards)):
            sel = r[self.shard_of[r] == s]
            if sel.size:
                self.shards[s].remove(self.local_of[sel])

    def compact(self) -> np.ndarray:
        n = len(self.shard_of)
        alive = np.zeros(n, bool)
        for s, sh in enumerate(self.shards):
            m = np.asarray(sh.compact())
            keep = m >= 0
            alive[self.tables[s][keep]] = True
            self.tables[s] = self.tables[s][keep]           # new local order = old order
        remap = np.full(n, -1, np.int64)
        remap[alive] = np.arange(int(alive.sum()))
        self.tables = [remap[t] for t in self.tables]
        self._rebuild_index()
        self._dev_tables = None
        return remap

    def set_scan_dtype(self, dtype: str) -> None:
        for sh in self.shards:
            sh.set_scan_dtype(dtype)

    def close(self) -> None:
        for sh in self.shards:
            if hasattr(sh, "close"):
                sh.close()

    # -- queries ------------------------------------------------------------------------------------
    def count(self):
        n = live = 0
        for sh in self.shards:
            a, b = sh.count()
            n, live = n + a, live + b
        return n, live

    def get(self, rows) -> np.ndarray:
        r = np.asarray(rows, dtype=np.int64)
        out = np.empty((r.shape[0], self.dim), dtype=np.float32)
        for s in range(len(self.shards)):
            sel = np.nonzero(self.shard_of[r] == s)[0]
            if sel.size:
                out[sel] = self.shards[s].get(self.local_of[r[sel]])
        return out

    def search(self, queries, k: int, allow=None, mask_key: int = 0):
        q = np.ascontiguousarray(np.asarray(queries, dtype=np.float32))
        if q.ndim == 1:
            q = q[None]
        if q.shape[1] != self.dim:
            raise ValueError(f"query dim {q.shape[1]} != store dim {self.dim}")
        if allow is None and all(hasattr(sh, "search_dev") for sh in self.shards):
            return self._search_device(q, int(k))
        return self._search_host(q, int(k), allow, mask_key)

    def _search_host(self, q, k, allow, mask_key):
        B = q.shape[0]
        dists, rows = [], []
        # native shards hand back their exact similarities: the merge then orders by similarity as
        # one store does (1 - sim in fp32 can merge two neighbouring similarities into one distance)
        exact = all(hasattr(sh, "search_sim") for sh in self.shards)
        for s, sh in enumerate(self.shards):
            a = None if allow is None else np.asarray(allow, dtype=np.uint8)[self.tables[s]]
            if exact:
                sim, r = sh.search_sim(q, k, allow=a, mask_key=mask_key)
                d = -sim.astype(np.float64)    # merge key; converted back to 1 - sim below
            else:
                d, r = sh.search(q, k, allow=a, mask_key=mask_key) if a is not None else sh.search(q, k)
            d = np.asarray(d)          # the shards' own precision (fp32 from the device)
            g = np.where(r >= 0, self.tables[s][np.clip(r, 0, None)] if len(self.tables[s]) else -1, -1)
            dists.append(np.where(g >= 0, d, np.inf))
            rows.append(g)
        D, R = np.concatenate(dists, 1), np.concatenate(rows, 1)
        out_d = np.full((B, k), np.inf, D.dtype)
        out_r = np.full((B, k), -1, np.int64)
        for b in range(B):
            big = np.where(R[b] >= 0, R[b], np.iinfo(np.int64).max)
            o = np.lexsort((big, D[b]))[:k]
            out_d[b], out_r[b] = D[b][o], np.where(np.isfinite(D[b][o]), R[b][o], -1)
        if exact:  # -sim -> 1 - sim in fp32, as the single store reports it
            ok = out_r >= 0
            out_d = np.where(ok, (np.float32(1.0) - (-out_d).astype(np.float32)), np.inf).astype(np.float32)
        return out_d, out_r

    def _search_device(self, q, k):
        import torch
        dev0 = torch.device("cuda", self.devices[0])
        if self._dev_tables is None:
            self._dev_tables = [torch.as_tensor(t, device=torch.device("cuda", d))
                                for t, d in zip(self.tables, self.devices)]
        qh = torch.from_numpy(q)
        sims, rows = [], []
        for sh, d, tab in zip(self.shards, self.devices, self._dev_tables):
            dev = torch.device("cuda", d)
            with torch.cuda.device(dev):
                qd = qh.to(dev, non_blocking=False)
                sim, loc = sh.search_dev(qd, k, stream=torch.cuda.current_stream(dev))
                ok = loc >= 0
                glob = torch.where(ok, tab[loc.clamp_min(0)] if tab.numel() else loc, loc)
                sims.append(torch.where(ok, sim, torch.full_like(sim, float("-inf"))).to(dev0))
                rows.append(glob.to(dev0))
        with torch.cuda.device(dev0):
            s, r = topk_merge_dev(torch.stack(sims), torch.stack(rows), k, device=self.devices[0],
                                  stream=torch.cuda.current_stream(dev0))
            s, r = s.cpu().numpy(), r.cpu().numpy()
        dist = np.where(r >= 0, np.float32(1.0) - s, np.float32(np.inf)).astype(np.float32)
        return dist, np.where(r >= 0, r, -1)

    # -- persistence --------------------------------------------------------------------------------
    def save(self, path: str) -> None:
        """<path>: manifest; <path>.s<i>: shard i (store snapshot); <path>.rows.npz: tables."""
        import json
        import os
        for i, sh in enumerate(self.shards):
            sh.save(f"{path}.s{i}")
        np.savez(f"{path}.rows.tmp.npz", **{f"s{i}": t for i, t in enumerate(self.tables)})
        os.replace(f"{path}.rows.tmp.npz", f"{path}.rows.npz")
        with open(path + ".tmp", "w") as f:
            json.dump({"magic": self.MAGIC, "dim": self.dim, "shards": len(self.shards)}, f)
        os.replace(path + ".tmp", path)

    @classmethod
    def is_manifest(cls, path: str) -> bool:
        with open(path, "rb") as f:
            head = f.read(64)
        return cls.MAGIC.encode() in head

    @classmethod
    def load(cls, path: str, devices, loader=None) -> "ShardedStore":
        import json
        with open(path) as f:
            man = json.load(f)
        devices = list(devices)
        if man.get("magic") != cls.MAGIC or len(devices) != int(man["shards"]):
            raise IOError(f"{path}: a {man.get('shards')}-shard collection cannot load on "
                          f"devices {devices}")
        loader = loader or (lambda p, dev: NativeStore.load(p, device=dev))
        shards = [loader(f"{path}.s{i}", d) for i, d in enumerate(devices)]
        with np.load(f"{path}.rows.npz") as z:
            tables = [z[f"s{i}"].astype(np.int64) for i in range(len(devices))]
        return cls(int(man["dim"]), devices, _shards=shards, _tables=tables)
