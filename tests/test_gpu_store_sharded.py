"""GPU: a collection sharded over several stores (ctx "devices") returns exactly one store's results.

Two shards on the box's one GPU exercise the same code as one shard per GPU: per-shard K1 + K2,
local -> global rows on the device, K2 topk_merge (sr_topk_merge_dev) on the first device; filtered
searches through the per-shard masked search and the host merge.  Reference surface:
MI355XVectorStoreConnector.search == SeekDBVectorStoreConnector.search (seekdb_connector.py:98-155),
configured from VECTOR_DB_CONTEXT (config.py:65-67).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(n, dim, seed):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((64, dim)).astype(np.float32)
    return c[np.arange(n) % 64] + 0.5 * rng.standard_normal((n, dim)).astype(np.float32)


def test_sharded_store_equals_single_store():
    from super_rag_amd.store import NativeStore, ShardedStore
    dim = 768
    x = _data(60_000, dim, 1)
    one, sh = NativeStore(dim), ShardedStore(dim, [0, 0])
    for s in range(0, 60_000, 7_000):                    # batches alternate between the shards
        assert one.add(x[s:s + 7000]).tolist() == sh.add(x[s:s + 7000]).tolist()
    dup = np.repeat(x[3:4], 3, 0)
    one.add(dup)
    sh.add(dup)                                          # exact ties in both shards
    q = _data(33, dim, 2)
    q[0] = x[3]
    for k in (1, 10, 100):
        d1, r1 = one.search(q, k)
        d2, r2 = sh.search(q, k)                         # device path + topk_merge_dev
        assert np.array_equal(r1, r2)
        assert np.array_equal(d1, d2)
    dead = np.arange(0, 60_003, 5)
    one.remove(dead)
    sh.remove(dead)
    allow = (np.arange(60_003) % 3 != 0).astype(np.uint8)
    d1, r1 = one.search(q, 50, allow=allow, mask_key=7)
    d2, r2 = sh.search(q, 50, allow=allow, mask_key=7)   # per-shard masked search, host merge
    assert np.array_equal(r1, r2) and np.array_equal(d1, d2)
    # 300 queries x k = 100 through the host merge: neighbours whose fp32 similarities differ by
    # one ulp but share one fp32 distance keep one store's order (merge on the similarities)
    q3 = _data(300, dim, 5)
    d1, r1 = one.search(q3, 100, allow=allow, mask_key=8)
    d2, r2 = sh.search(q3, 100, allow=allow, mask_key=8)
    np.testing.assert_array_equal(d1, d2)
    np.testing.assert_array_equal(r1, r2)
    assert np.array_equal(one.compact(), sh.compact())
    d1, r1 = one.search(q, 100)
    d2, r2 = sh.search(q, 100)
    assert np.array_equal(r1, r2) and np.array_equal(d1, d2)
    np.testing.assert_array_equal(one.get(np.arange(100)), sh.get(np.arange(100)))
    one.close()
    sh.close()


def test_connector_devices_ctx_matches_single_device(tmp_path):
    from super_rag_amd import vectorstore as V
    from super_rag_amd.models import QueryWithEmbedding, TextNode
    V._collections.clear()
    x = _data(5000, 384, 3)
    single = V.MI355XVectorStoreConnector({"collection": "s1", "device": 0})
    multi = V.MI355XVectorStoreConnector({"collection": "s2", "devices": [0, 0],
                                          "snapshot_dir": str(tmp_path)})
    for con in (single, multi):
        ids = []
        for s in range(0, 5000, 600):
            ids += con.add([TextNode(text=f"doc {i}", metadata={"i": i}, embedding=x[i].tolist())
                            for i in range(s, min(5000, s + 600))])
        con.delete(ids=ids[100:160])
    qs = [QueryWithEmbedding(query="q", top_k=k, embedding=v.tolist())
          for k, v in zip((1, 8, 64), _data(3, 384, 4))]
    dump = lambda con: [[(d.text, d.score) for d in con.search(q).results] for q in qs]
    want = dump(single)
    assert dump(multi) == want
    V._collections.clear()
    again = V.MI355XVectorStoreConnector({"collection": "s2", "devices": [0, 0],
                                          "snapshot_dir": str(tmp_path)})
    assert dump(again) == want
    again.delete_collection()
    single.delete_collection()
    V._collections.clear()


@pytest.mark.parametrize("dtype", ["fp16", "fp8"])
def test_native_store_set_equals_single_store(dtype):
    # ONE native handle over three shards (sr_store_set_*, SURVEY 8(b) sr_store_create(dim, dtype,
    # devices, n_dev)); the same device listed three times runs the multi-GPU code on one card:
    # concurrent per-shard K1 + K2 (one host thread per shard), global rows, host merge
    from super_rag_amd.store import NativeStore, NativeStoreSet
    dim = 384
    x = _data(50_000, dim, 3)
    one, st = NativeStore(dim), NativeStoreSet(dim, [0, 0, 0], dtype=dtype)
    if dtype == "fp8":
        one.set_scan_dtype("fp8")
    for s, e in ((0, 9_000), (9_000, 9_001), (9_001, 30_000), (30_000, 41_000), (41_000, 50_000)):
        assert one.add(x[s:e]).tolist() == st.add(x[s:e]).tolist()      # uneven batches
    dup = np.repeat(x[7:8], 4, 0)
    one.add(dup)
    st.add(dup)                                                          # exact ties across shards
    rows_all = np.arange(50_004)
    assert np.array_equal(one.get(rows_all[::97]), st.get(rows_all[::97]))
    q = _data(300, dim, 4)
    q[0] = x[7]
    for k in (1, 10, 100):
        d1, r1 = one.search(q, k)
        d2, r2 = st.search(q, k)
        bad = np.argwhere(r1 != r2)
        if bad.size:
            b0, j0 = bad[0]
            print("k", k, "first mismatch", b0, j0, "rows", r1[b0, j0 - 1:j0 + 2], r2[b0, j0 - 1:j0 + 2],
                  "dist", d1[b0, j0 - 1:j0 + 2], d2[b0, j0 - 1:j0 + 2], "n bad", len(bad),
                  "queries", np.unique(bad[:, 0])[:20])
            s1 = dict(zip(r1[b0].tolist(), d1[b0].tolist()))
            s2 = dict(zip(r2[b0].tolist(), d2[b0].tolist()))
            print("dist of same rows differ:", [(r, s1[r], s2[r]) for r in s1 if r in s2 and s1[r] != s2[r]][:5])
        np.testing.assert_array_equal(d1, d2)
        np.testing.assert_array_equal(r1, r2)
    dead = np.arange(1, 50_004, 7)
    one.remove(dead)
    st.remove(dead)
    assert one.count() == st.count()
    allow = (np.arange(50_004) % 3 != 0).astype(np.uint8)
    for key in (0, 11, 11):                                              # cached mask reused
        d1, r1 = one.search(q[:40], 20, allow=allow, mask_key=key)
        d2, r2 = st.search(q[:40], 20, allow=allow, mask_key=key)
        assert np.array_equal(r1, r2)
        assert np.array_equal(d1, d2)
    # short lists: k beyond the live rows of a tiny set
    tiny = NativeStoreSet(dim, [0, 0], dtype=dtype)
    tiny.add(x[:3])
    d, r = tiny.search(q[:2], 5)
    assert (r[:, 3:] == -1).all() and np.isinf(d[:, 3:]).all()
    assert sorted(r[0, :3].tolist()) == [0, 1, 2]


@pytest.mark.parametrize("mode", ["fulltext", "hybrid"])
def test_sharded_fulltext_hybrid_collection_equals_one_device(mode):
    """ctx "devices" with "fulltext" / "hybrid" on the HIP path: per-shard BM25 (sr_lex_search_global
    with the corpus-wide statistics) merged on (score, row) and rrf-fused with the sharded dense
    list == the single-device collection (sr_lex_search / sr_hybrid_search), with a filter and
    after deletes."""
    from super_rag_amd import vectorstore as V
    from super_rag_amd.lexical import ShardedLex
    from super_rag_amd.models import QueryWithEmbedding, TextNode
    rng = np.random.default_rng(5)
    words = [f"w{i}" for i in range(300)]
    V._collections.clear()
    try:
        base = {mode: True, "honor_filter": True}
        one = V.MI355XVectorStoreConnector({**base, "collection": "lx1"})
        many = V.MI355XVectorStoreConnector({**base, "collection": "lx2", "devices": [0, 0, 0]})
        x = _data(3000, 64, 7)
        ids1, ids2 = [], []
        for s in range(0, 3000, 250):
            nodes = [TextNode(text=" ".join(rng.choice(words, rng.integers(2, 30))),
                              metadata={"i": i, "chat_id": f"c{i % 4}"}, embedding=x[i].tolist())
                     for i in range(s, s + 250)]
            ids1 += one.add(nodes)
            ids2 += many.add(nodes)
        assert isinstance(V._get("lx2").lex, ShardedLex)
        qs = [" ".join(rng.choice(words, rng.integers(1, 6))) for _ in range(12)]
        qv = _data(12, 64, 8)

        def dump(con, flt=None):
            kw = {"filter": flt} if flt else {}
            if mode == "fulltext":
                return [[(d.text, d.score) for d in con.fulltext_search(q, 20, **kw)] for q in qs]
            return [[(d.text, d.score) for d in
                     con.search(QueryWithEmbedding(query=q, top_k=20, embedding=v.tolist()), **kw).results]
                    for q, v in zip(qs, qv)]
        assert dump(one) == dump(many)
        flt = {"chat_id": {"$in": ["c1", "c3"]}}
        assert dump(one, flt) == dump(many, flt)
        dead = rng.choice(3000, 700, replace=False)
        one.delete(ids=[ids1[i] for i in dead])
        many.delete(ids=[ids2[i] for i in dead])
        a, b = dump(one), dump(many)
        assert a == b and sum(len(r) for r in a) > 100
    finally:
        V._collections.clear()
