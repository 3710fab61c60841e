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
