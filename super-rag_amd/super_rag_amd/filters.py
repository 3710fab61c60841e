"""Metadata filter evaluation for the vector store's opt-in filtered search.

The reference builds SeekDB-style filter dicts in ContextManager._create_combined_filter
(context/context.py:74-111), e.g.
    {"and": [{"or": [{"indexer": {"$in": ["vector"]}}, {"indexer": {"$exists": False}}]},
             {"chat_id": "c1"}]}
and passes them to the connector, which ignores them (seekdb_connector.py:99-100).  With
``ctx["honor_filter"]`` the MI355X connector applies them: rows whose metadata does not match are
excluded from the device search (sr_store_search_masked), so a query still gets its k best
matching rows.  Supported: and / or / not (with or without "$"), field equality and the operators
$eq $ne $in $nin $exists $gt $gte $lt $lte $contains; a list of clauses is a conjunction.
"""
from __future__ import annotations

import json
from typing import Any, Mapping

_MISSING = object()


def canonical(flt: Any) -> str:
    """Stable cache key of a filter."""
    return json.dumps(flt, sort_keys=True, default=str)


def _field(cond: Any, val: Any) -> bool:
    present = val is not _MISSING
    if not isinstance(cond, Mapping):
        return present and val == cond
    for op, arg in cond.items():
        if op == "$eq":
            ok = present and val == arg
        elif op == "$ne":
            ok = not (present and val == arg)
        elif op == "$in":
            ok = present and val in arg
        elif op == "$nin":
            ok = not (present and val in arg)
        elif op == "$exists":
            ok = present == bool(arg)
        elif op in ("$gt", "$gte", "$lt", "$lte"):
            try:
                ok = present and {"$gt": val > arg, "$gte": val >= arg,
                                  "$lt": val < arg, "$lte": val <= arg}[op]
            except TypeError:
                ok = False
        elif op == "$contains":
            try:
                ok = present and arg in val
            except TypeError:
                ok = False
        else:
            raise ValueError(f"unsupported filter operator {op!r}")
        if not ok:
            return False
    return True


def matches(flt: Any, metadata: Mapping | None) -> bool:
    """Does a row's metadata satisfy the filter?  ``None`` matches everything."""
    if flt is None:
        return True
    md = metadata or {}
    if isinstance(flt, (list, tuple)):
        return all(matches(c, md) for c in flt)
    if not isinstance(flt, Mapping):
        raise ValueError(f"unsupported filter {flt!r}")
    for key, cond in flt.items():
        if key in ("and", "$and"):
            ok = all(matches(c, md) for c in cond)
        elif key in ("or", "$or"):
            ok = any(matches(c, md) for c in cond)
        elif key in ("not", "$not"):
            ok = not matches(cond, md)
        else:
            ok = _field(cond, md.get(key, _MISSING))
        if not ok:
            return False
    return True
