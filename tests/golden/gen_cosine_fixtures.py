"""Capture cosine-similarity fixtures from the REAL reference functions (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_cosine_fixtures.py

The reference's search arithmetic runs in the un-vendored pylibseekdb (HNSW, distance="cosine",
super_rag/vectorstore/seekdb_connector.py:56-66); the only cosine code the reference itself holds is
graphiti's ``calculate_cosine_similarity`` (super_rag/graphiti/graphiti_core/search/search_utils.py:
56-67: dot / (|a| |b|), 0 when either norm is 0) and ``normalize_l2`` (graphiti_core/helpers.py:
100-103: x / |x|, zero vectors unchanged).  This script imports both from /root/reference (missing
third-party modules stubbed, as gen_rrf_fixtures.py does), evaluates them on seeded cases and writes
inputs + outputs to tests/golden/cosine_fixtures.npz (data only; /root/reference never travels).

Cases, for dims 64 / 384 / 768 / 1024 (8 queries each):
  random      Gaussian rows
  clustered   rows = 16 centres + small noise (near ties), queries near the centres
  ties_zeros  exact duplicate rows (equal cosines: order by row), zero rows, one zero query
  scaled      rows scaled by 2^e, e in [-10, 10] (cosine is scale free)
  sparse      rows with 1-8 non-zeros (large fp16 elements)
All vector entries are small integers times 1/16 (exactly representable in fp16 / fp32) times a
per-row power of two, stored as int8 + exponent so the fixture stays small; the cosines are the
reference's fp64 results, bit-exact.
"""
from __future__ import annotations

import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_rrf_fixtures import REF, _AnyAttr  # noqa: E402  (same stub recipe)

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cosine_fixtures.npz")
DIMS = {64: 256, 384: 128, 768: 128, 1024: 64}   # dim -> corpus rows per case
NQ = 8


def _import(module: str, attr: str):
    for _ in range(200):
        try:
            return getattr(importlib.import_module(module), attr)
        except ModuleNotFoundError as e:
            name = e.name
            if not name or name.startswith("super_rag"):
                raise
            for k in [m for m in sys.modules if m.startswith("super_rag")]:
                del sys.modules[k]
            parts = name.split(".")
            for i in range(1, len(parts) + 1):
                sys.modules.setdefault(".".join(parts[:i]), _AnyAttr(".".join(parts[:i])))
    raise RuntimeError(f"could not import {module}.{attr}")


def _q16(x, rng_scale=16.0):
    """Round to multiples of 1/16, clipped to int8 range: (int8 codes)."""
    return np.clip(np.rint(x * rng_scale), -127, 127).astype(np.int8)


def make_case(family: str, dim: int, n: int, rng: np.random.Generator):
    """(corpus codes int8 [n, dim], corpus exp int8 [n], query codes [NQ, dim], query exp [NQ])."""
    cexp = np.zeros(n, np.int8)
    qexp = np.zeros(NQ, np.int8)
    if family == "random":
        c = _q16(rng.standard_normal((n, dim)) * 2.0)
        q = _q16(rng.standard_normal((NQ, dim)) * 2.0)
    elif family == "clustered":
        cent = rng.standard_normal((16, dim)) * 2.0
        c = _q16(cent[np.arange(n) % 16] + 0.15 * rng.standard_normal((n, dim)))
        q = _q16(cent[rng.integers(0, 16, NQ)] + 0.3 * rng.standard_normal((NQ, dim)))
    elif family == "ties_zeros":
        c = _q16(rng.standard_normal((n, dim)) * 2.0)
        for dst, src in ((3, 1), (7, 1), (12, 1), (20, 5), (21, 5), (n - 1, 5)):
            c[dst] = c[src]
        c[[2, 9, n // 2]] = 0
        q = _q16(rng.standard_normal((NQ, dim)) * 2.0)
        q[0] = c[1]               # duplicates 1, 3, 7, 12 tie exactly at cos = 1
        q[1] = c[5]
        q[NQ - 1] = 0             # zero query: every cosine is 0
    elif family == "scaled":
        c = _q16(rng.standard_normal((n, dim)) * 2.0)
        q = _q16(rng.standard_normal((NQ, dim)) * 2.0)
        cexp = rng.integers(-10, 11, n).astype(np.int8)
        qexp = rng.integers(-10, 11, NQ).astype(np.int8)
        c[5] = c[4]               # same direction, different scale: equal cosines
        cexp[4], cexp[5] = -7, 9
    elif family == "sparse":
        c = np.zeros((n, dim), np.int8)
        for r in range(n):
            nz = rng.choice(dim, rng.integers(1, 9), replace=False)
            c[r, nz] = rng.integers(-127, 128, nz.size)
        q = np.zeros((NQ, dim), np.int8)
        for r in range(NQ):
            nz = rng.choice(dim, rng.integers(1, 9), replace=False)
            q[r, nz] = rng.integers(-127, 128, nz.size)
        q[0] = c[0]
        c[rng.integers(0, n)] = c[0]
    else:
        raise ValueError(family)
    return c, cexp, q, qexp


def values(codes, exp):
    """fp64 vectors: codes / 16 * 2^exp (exact in fp16 and fp32)."""
    return codes.astype(np.float64) / 16.0 * np.exp2(exp.astype(np.float64))[:, None]


FAMILIES = ("random", "clustered", "ties_zeros", "scaled", "sparse")


def main():
    sys.path.insert(0, REF)
    cos = _import("super_rag.graphiti.graphiti_core.search.search_utils", "calculate_cosine_similarity")
    norm = _import("super_rag.graphiti.graphiti_core.helpers", "normalize_l2")
    rng = np.random.default_rng(20261016)
    out = {}
    names = []
    for dim, n in DIMS.items():
        for fam in FAMILIES:
            name = f"{fam}_{dim}"
            c, ce, q, qe = make_case(fam, dim, n, rng)
            C, Q = values(c, ce), values(q, qe)
            sims = np.array([[float(cos(list(qq), list(cc))) for cc in C] for qq in Q], np.float64)
            out[name + ".c"], out[name + ".ce"], out[name + ".q"], out[name + ".qe"] = c, ce, q, qe
            out[name + ".cos"] = sims
            names.append(name)
    # normalize_l2 on a few vectors of each dim, zero vectors included
    for dim in DIMS:
        v = _q16(rng.standard_normal((6, dim)) * 2.0)
        v[2] = 0
        e = rng.integers(-10, 11, 6).astype(np.int8)
        V = values(v, e)
        out[f"norm_{dim}.v"], out[f"norm_{dim}.e"] = v, e
        out[f"norm_{dim}.out"] = np.stack([np.asarray(norm(list(x)), np.float64) for x in V])
    out["cases"] = np.array(names)
    out["source"] = np.array("super_rag/graphiti/graphiti_core/search/search_utils.py:56-67 "
                             "(calculate_cosine_similarity); graphiti_core/helpers.py:100-103 "
                             "(normalize_l2)")
    np.savez_compressed(OUT, **out)
    print(f"wrote {len(names)} cosine cases ({sum(o.size for k, o in out.items() if k.endswith('.cos'))}"
          f" reference cosines) to {OUT}")


if __name__ == "__main__":
    main()
