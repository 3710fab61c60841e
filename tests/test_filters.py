"""CPU: opt-in score_threshold / metadata filtering of the connector.  The
reference passes both to SeekDB's connector, which ignores them (seekdb_connector.py:99-100,
context/context.py:37-47); off by default here too, on with ctx["honor_*"]: a filtered query gets
the k best MATCHING rows (the mask is applied inside the device search, not after top-k)."""
import numpy as np
import pytest

from doubles import NumpyStore


def test_filter_language():
    from super_rag_amd.filters import matches
    from super_rag_amd.context import ContextManager
    cm = ContextManager.__new__(ContextManager)
    f = cm._create_combined_filter(["vector"], "c1")   # exactly what context.py:74-111 builds
    assert matches(f, {"indexer": "vector", "chat_id": "c1"})
    assert matches(f, {"chat_id": "c1"})                       # indexer $exists False
    assert not matches(f, {"indexer": "graph", "chat_id": "c1"})
    assert not matches(f, {"indexer": "vector", "chat_id": "c2"})
    assert not matches(f, None)
    assert matches(None, {"x": 1})
    assert matches({"$and": [{"n": {"$gte": 2, "$lt": 5}}, {"t": {"$nin": ["a"]}}]}, {"n": 3, "t": "b"})
    assert not matches({"n": {"$gt": 3}}, {"n": "x"})          # incomparable -> no match
    assert matches({"$not": {"k": 1}}, {"k": 2}) and matches({"tags": {"$contains": "z"}}, {"tags": ["z"]})
    with pytest.raises(ValueError):
        matches({"k": {"$regex": "."}}, {"k": "a"})


@pytest.fixture
def conn_factory():
    from super_rag_amd import vectorstore as V
    V.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    V._collections.clear()
    yield lambda **kw: V.MI355XVectorStoreConnector({"collection": "flt", **kw})
    V._collections.clear()
    V.set_store_backend(V._native_store, V._native_load)


def _oracle(vecs, metas, alive, q, k, pred):
    qn = q / np.linalg.norm(q)
    d = 1.0 - (vecs / np.linalg.norm(vecs, axis=1, keepdims=True)) @ qn
    idx = [i for i in np.lexsort((np.arange(len(d)), d)) if alive[i] and pred(metas[i])]
    return [(int(i), float(d[i])) for i in idx[:k]]


@pytest.mark.parametrize("coalesce", [True, False])
def test_filtered_search_returns_k_best_matching_rows(conn_factory, coalesce):
    from super_rag_amd.context import ContextManager
    from super_rag_amd.filters import matches
    from super_rag_amd.models import TextNode
    rng = np.random.default_rng(0)
    n = 400
    vecs = rng.standard_normal((n, 12))
    metas = [{"i": i, "chat_id": f"c{i % 3}", **({"indexer": "vector"} if i % 5 else
                                                  ({"indexer": "graph"} if i % 2 else {}))}
             for i in range(n)]
    conn = conn_factory(honor_filter=True, honor_score_threshold=True, coalesce=coalesce)
    ids = conn.store.add([TextNode(text=f"t{i}", metadata=m, embedding=v.tolist())
                          for i, (m, v) in enumerate(zip(metas, vecs))])
    alive = np.ones(n, bool)
    cm = ContextManager("flt", None, "mi355x", {"collection": "flt", "honor_filter": True,
                                                 "honor_score_threshold": True, "coalesce": coalesce})
    f = cm._create_combined_filter(["vector"], "c1")
    for step in range(3):
        q = rng.standard_normal(12)
        hits = cm.query("q", score_threshold=-1.0, topk=9, vector=q.tolist(), index_types=["vector"],
                        chat_id="c1")
        want = _oracle(vecs, metas, alive, q, 9, lambda m: matches(f, m))
        assert [h.metadata["i"] for h in hits] == [i for i, _ in want]
        np.testing.assert_allclose([h.score for h in hits], [d for _, d in want], atol=1e-7)
        # threshold: only similarity >= thr survives (a prefix of the distance order)
        thr = 1.0 - want[4][1]
        hits_t = cm.query("q", score_threshold=thr, topk=9, vector=q.tolist(), index_types=["vector"],
                          chat_id="c1")
        assert [h.metadata["i"] for h in hits_t] == [i for i, _ in want[:5]]
        # deleting matching rows invalidates the cached mask
        gone = [want[0][0], want[1][0]]
        conn.delete(ids=[ids[i] for i in gone])
        alive[gone] = False


def test_filters_are_ignored_by_default_like_the_reference(conn_factory):
    from super_rag_amd.context import ContextManager
    from super_rag_amd.models import TextNode
    conn = conn_factory()
    conn.store.add([TextNode(text=f"t{i}", metadata={"chat_id": "other"},
                             embedding=[1.0, float(i)]) for i in range(5)])
    cm = ContextManager("flt", None, "mi355x", {"collection": "flt"})
    hits = cm.query("q", score_threshold=0.99, topk=3, vector=[1.0, 0.0], chat_id="c1")
    assert len(hits) == 3   # neither the chat_id filter nor the threshold is applied


def test_filter_mask_cache_is_bounded(conn_factory):
    from super_rag_amd import vectorstore as V
    from super_rag_amd.models import QueryWithEmbedding, TextNode
    conn = conn_factory(honor_filter=True, coalesce=False)
    conn.store.add([TextNode(text=f"t{i}", metadata={"chat_id": f"c{i % 20}"},
                             embedding=[1.0, float(i)]) for i in range(40)])
    q = QueryWithEmbedding(query="q", top_k=3, embedding=[1.0, 0.0])
    for c in range(20):                           # 20 distinct filters
        hits = conn.search(q, filter={"chat_id": c and f"c{c}" or "c0"}).results
        assert all(h.metadata["chat_id"] == f"c{c}" for h in hits)
    masks = V._get("flt").masks
    assert len(masks) == V.MASK_CACHE_SIZE
    conn.search(q, filter={"chat_id": "c19"})     # a hit refreshes its entry
    assert next(reversed(masks)).find("c19") >= 0
    conn.store.add([TextNode(text="new", metadata={"chat_id": "c1"}, embedding=[0.0, 1.0])])
    conn.search(q, filter={"chat_id": "c1"})      # version changed: stale masks are dropped
    assert len(masks) == 1
