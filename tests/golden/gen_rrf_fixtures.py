"""Capture reciprocal-rank-fusion fixtures from the REAL reference function (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_rrf_fixtures.py

The hybrid dense + BM25 path fuses its two ranked lists the way the reference's only fusion
precedent does: graphiti ``rrf`` (super_rag/graphiti/graphiti_core/search/search_utils.py:1762-1778).
This script imports that module from /root/reference with every third-party module the import
chain reports missing stubbed by an empty module (graphiti pulls dotenv, neo4j, openai, ... at import time; rrf itself is pure
Python), runs rrf on seeded ranked lists (overlapping, disjoint, equal-score ties, min_score cuts)
and writes inputs + outputs to tests/golden/rrf_fixtures.json (data only; /root/reference never
travels).
"""
from __future__ import annotations

import json
import os
import random
import sys
import types

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "rrf_fixtures.json")


def _dummy(name):
    class _Meta(type):
        def __getattr__(cls, n):
            if n.startswith("__"):
                raise AttributeError(n)
            return _dummy(n)

        def __or__(cls, other):
            return cls

        __ror__ = __or__

        def __getitem__(cls, item):
            return cls

    class _Dummy(metaclass=_Meta):
        def __init__(self, *a, **k):
            pass

        def __call__(self, *a, **k):
            return a[0] if len(a) == 1 and callable(a[0]) and not k else _Dummy()

        def __getattr__(self, n):
            return _Dummy()

        @classmethod
        def __get_pydantic_core_schema__(cls, source, handler):
            from pydantic_core import core_schema
            return core_schema.any_schema()

    _Dummy.__name__ = name
    return _Dummy


class _AnyAttr(types.ModuleType):
    """Stub module: every attribute is a permissive dummy class (usable as a base, decorator,
    type annotation, ...)."""
    __path__: list = []

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        d = _dummy(name)
        setattr(self, name, d)
        return d


def _import_rrf():
    """Import rrf, stubbing each third-party module the import chain reports missing."""
    import importlib
    for _ in range(200):
        try:
            return importlib.import_module("super_rag.graphiti.graphiti_core.search.search_utils").rrf
        except ModuleNotFoundError as e:
            name = e.name
            if not name or name.startswith("super_rag"):
                raise
            for k in [m for m in sys.modules if m.startswith("super_rag")]:
                del sys.modules[k]
            parts = name.split(".")
            for i in range(1, len(parts) + 1):
                sys.modules.setdefault(".".join(parts[:i]), _AnyAttr(".".join(parts[:i])))
    raise RuntimeError("could not import rrf")


def main():
    sys.path.insert(0, REF)
    rrf = _import_rrf()

    rng = random.Random(7)
    cases = []
    # hand-made: overlap, reorder, ties in score (a only-dense item at rank i and a lexical-only
    # item at rank i score the same)
    hand = [
        ([["a", "b", "c"], ["c", "d", "a"]], 1, 0.0),
        ([["a", "b"], ["c", "d"]], 1, 0.0),
        ([["x"], []], 1, 0.0),
        ([[], []], 1, 0.0),
        ([["a", "b", "c", "d"], ["d", "c", "b", "a"]], 1, 0.0),
        ([["a", "b", "c"], ["b", "e", "f"]], 60, 0.0),
        ([["a", "b", "c"], ["b", "e", "f"]], 1, 0.4),
    ]
    for lists, rc, ms in hand:
        cases.append({"lists": lists, "rank_const": rc, "min_score": ms})
    for t in range(40):
        n_universe = rng.randint(1, 60)
        ka, kb = rng.randint(0, 30), rng.randint(0, 30)
        uni = [f"r{i}" for i in range(n_universe)]
        a = rng.sample(uni, min(ka, n_universe))
        b = rng.sample(uni, min(kb, n_universe))
        rc = rng.choice([1, 1, 2, 60])
        ms = rng.choice([0.0, 0.0, 0.05, 0.5])
        cases.append({"lists": [a, b], "rank_const": rc, "min_score": ms})
    for c in cases:
        ids, scores = rrf(c["lists"], rank_const=c["rank_const"], min_score=c["min_score"])
        c["ids"] = ids
        c["scores"] = [float(s).hex() for s in scores]   # exact doubles
    with open(OUT, "w") as f:
        json.dump({"source": "super_rag/graphiti/graphiti_core/search/search_utils.py:1762-1778 (rrf)",
                   "cases": cases}, f, indent=0)
    print(f"wrote {len(cases)} cases to {OUT}")


if __name__ == "__main__":
    main()
