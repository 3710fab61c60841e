"""CPU: a collection row-sharded over several stores (VECTOR_DB_CONTEXT "devices": [...]).

Global row ids follow insertion order across shards, so a sharded collection must return exactly
what one store returns — same rows, same (distance asc, row asc) order — through adds, deletes,
compaction, filters and a snapshot round trip (the reference's connector is configured from
VECTOR_DB_CONTEXT: super_rag/config.py:65-67, vectorstore/connector.py:4-15).  The shards here are
the NumpyStore doubles (host merge path); tests/test_gpu_store_sharded.py runs the device path.
"""
import numpy as np
import pytest

from doubles import NumpyStore


def _pair(P=3, dim=6):
    from super_rag_amd.store import ShardedStore
    return NumpyStore(dim), ShardedStore(dim, list(range(P)), factory=lambda d, dev: NumpyStore(d))


def test_sharded_equals_single_through_mutations():
    rng = np.random.default_rng(0)
    one, sh = _pair()
    for n in (5, 17, 1, 40, 9, 30):
        x = rng.standard_normal((n, 6)).astype(np.float32)
        assert one.add(x).tolist() == sh.add(x).tolist()
    x = rng.standard_normal((4, 6)).astype(np.float32)
    one.add(np.repeat(x[:1], 4, 0))          # exact ties across shards: order by global row
    sh.add(np.repeat(x[:1], 4, 0))
    assert {int(s) for s in sh.shard_of} == {0, 1, 2}
    q = rng.standard_normal((7, 6)).astype(np.float32)
    q[0] = x[0]
    for k in (1, 5, 30, 200):
        d1, r1 = one.search(q, k)
        d2, r2 = sh.search(q, k)
        assert np.array_equal(r1, r2)
        np.testing.assert_allclose(d1[r1 >= 0], d2[r2 >= 0], atol=1e-12)
    dead = np.arange(0, 100, 3)
    one.remove(dead)
    sh.remove(dead)
    assert one.count() == sh.count()
    allow = (np.arange(106) % 4 != 1).astype(np.uint8)
    for a in (None, allow):
        d1, r1 = one.search(q, 12, allow=a) if a is not None else one.search(q, 12)
        d2, r2 = sh.search(q, 12, allow=a) if a is not None else sh.search(q, 12)
        assert np.array_equal(r1, r2)
    m1, m2 = one.compact(), sh.compact()
    assert np.array_equal(m1, m2)
    assert np.array_equal(one.search(q, 20)[1], sh.search(q, 20)[1])
    np.testing.assert_array_equal(one.get(np.arange(10)), sh.get(np.arange(10)))


def test_connector_with_devices_matches_one_device_and_restores(tmp_path):
    from super_rag_amd import vectorstore as V
    from super_rag_amd.models import QueryWithEmbedding, TextNode
    V.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    V._collections.clear()
    try:
        rng = np.random.default_rng(1)
        vecs = rng.standard_normal((60, 8))
        one = V.MI355XVectorStoreConnector({"collection": "one"})
        many = V.MI355XVectorStoreConnector({"collection": "many", "devices": [0, 0, 0],
                                             "snapshot_dir": str(tmp_path)})
        ids_m = []
        for c in (one, many):
            ids = []
            for s in range(0, 60, 7):
                ids += c.add([TextNode(text=f"t{i}", metadata={"i": i}, embedding=vecs[i].tolist())
                              for i in range(s, min(60, s + 7))])
            c.delete(ids=ids[5:9])
            ids_m.append(ids)
        qs = [QueryWithEmbedding(query="q", top_k=k, embedding=rng.standard_normal(8).tolist())
              for k in (1, 6, 25)]
        dump = lambda con: [[(d.text, d.score) for d in con.search(q).results] for q in qs]
        want = dump(one)
        assert dump(many) == want
        V._collections.clear()                                   # restart: sharded snapshot
        again = V.MI355XVectorStoreConnector({"collection": "many", "devices": [0, 0, 0],
                                              "snapshot_dir": str(tmp_path)})
        assert dump(again) == want
        assert type(V._get("many").store).__name__ == "ShardedStore"
        V._collections.clear()
        with pytest.raises(IOError, match="3-shard"):
            V.MI355XVectorStoreConnector({"collection": "many", "devices": [0, 0],
                                          "snapshot_dir": str(tmp_path)})
        V._collections.clear()
        again = V.MI355XVectorStoreConnector({"collection": "many", "devices": [0, 0, 0],
                                              "snapshot_dir": str(tmp_path)})
        again.delete_collection()
        assert list(tmp_path.iterdir()) == []
    finally:
        V._collections.clear()
        V.set_store_backend(V._native_store, V._native_load)


def _text_nodes(n, seed):
    from super_rag_amd.models import TextNode
    rng = np.random.default_rng(seed)
    words = ["alpha", "beta", "gamma", "delta", "eps", "zeta", "eta", "theta", "iota", "kappa",
             "lambda", "mu", "nu", "xi", "omicron", "pi"]
    out = []
    for i in range(n):
        t = " ".join(rng.choice(words, rng.integers(1, 9)))
        out.append(TextNode(text=f"{t} doc{i % 7}", metadata={"i": i, "chat_id": f"c{i % 3}"},
                            embedding=rng.standard_normal(8).round(4).tolist()))
    return out


@pytest.mark.parametrize("mode", ["fulltext", "hybrid"])
def test_sharded_fulltext_and_hybrid_collections_equal_one_device(mode, tmp_path):
    """ctx "devices" + "fulltext" / "hybrid" (VERDICT r2 item 6): the collection's BM25 index is
    sharded with its rows (lexical.ShardedLex, corpus-wide statistics), and fulltext_search /
    hybrid search / filters / deletes / compaction / restore give what one device gives."""
    from doubles import NumpyLex, NumpyStore
    from oracle.bm25 import rrf_rows
    from super_rag_amd import lexical, vectorstore as V
    from super_rag_amd.models import QueryWithEmbedding
    V.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    V.set_lex_backend(lambda dev: NumpyLex(dev), NumpyLex.load)
    lexical.set_rrf_backend(lambda a, b, k, rc, ms, dev: rrf_rows(a, b, k, rc, ms))
    V._collections.clear()
    try:
        base = {mode: True, "honor_filter": True}
        one = V.MI355XVectorStoreConnector({**base, "collection": "one"})
        many = V.MI355XVectorStoreConnector({**base, "collection": "many", "devices": [0, 1, 2],
                                             "snapshot_dir": str(tmp_path)})
        nodes = _text_nodes(60, 1)
        ids1, ids3 = [], []
        for a in range(0, 60, 7):                        # several add batches: rows spread over shards
            ids1 += one.add(nodes[a:a + 7])
            ids3 += many.add(nodes[a:a + 7])
        c = V._get("many")
        assert isinstance(c.lex, lexical.ShardedLex) and len({int(s) for s in c.store.shard_of}) == 3

        def same(q_text, emb, flt=None):
            kw = {"filter": flt} if flt else {}
            if mode == "fulltext":
                a = [(d.text, d.score) for d in one.fulltext_search(q_text, 9, **kw)]
                b = [(d.text, d.score) for d in many.fulltext_search(q_text, 9, **kw)]
            else:
                q = QueryWithEmbedding(query=q_text, top_k=9, embedding=emb)
                a = [(d.text, d.score) for d in one.search(q, **kw).results]
                b = [(d.text, d.score) for d in many.search(q, **kw).results]
            assert a == b and (len(a) > 0 or q_text == "omega"), (a, b)

        rng = np.random.default_rng(2)
        queries = ["alpha beta", "pi pi zeta", "doc3 kappa", "omega", "eta theta iota mu"]
        for qt in queries:
            same(qt, rng.standard_normal(8).tolist() if qt != "omega" else nodes[5].embedding)
        flt = {"and": [{"chat_id": "c1"}, {"i": {"$gte": 10}}]}
        same("alpha gamma", nodes[3].embedding, flt)
        dead = [3, 4, 5, 17, 30, 31, 32, 33, 50]
        one.delete(ids=[ids1[i] for i in dead])
        many.delete(ids=[ids3[i] for i in dead])
        for qt in queries[:3]:
            same(qt, nodes[7].embedding)
        # compaction (> half of the rows dead) renumbers both indexes consistently
        dead2 = [i for i in range(60) if i % 3 != 0 and i not in dead]
        one.delete(ids=[ids1[i] for i in dead2])
        many.delete(ids=[ids3[i] for i in dead2])
        assert V._get("many").store.count()[0] < 60
        for qt in queries:
            same(qt, nodes[9].embedding)
        # restore from the snapshot: the sharded lexical index comes back with its routing
        V._collections.pop("many")
        many = V.MI355XVectorStoreConnector({**base, "collection": "many", "devices": [0, 1, 2],
                                             "snapshot_dir": str(tmp_path)})
        assert isinstance(V._get("many").lex, lexical.ShardedLex)
        for qt in queries:
            same(qt, nodes[12].embedding)
    finally:
        V._collections.clear()
        V.set_store_backend(V._native_store, V._native_load)
        V.set_lex_backend(V._native_lex, V._native_lex_load)
        lexical.set_rrf_backend(None)


def test_sharded_bm25_merges_on_exact_fixed_point_scores():
    """above a BM25 score of 256 distinct 2^-16 fixed-point scores share one fp32 value;
    the sharded merge orders by the exact fixed-point score (then global row), as one index does,
    not by row among equal fp32 scores."""
    import numpy as np
    from super_rag_amd import lexical

    big = (300 << 16)                       # score 300: fp32 spacing there is 2^-15 > 2^-16
    assert np.float32(big) == np.float32(big + 1)

    class Shard:
        def __init__(self, fx, rows):
            self.fx, self.rows = np.asarray([fx], np.uint32), np.asarray([rows], np.int64)

        def totals(self):
            return 10, 100

        def df(self, terms):
            return np.ones(len(terms), np.int64)

        def search(self, queries, k, allow=None, mask_key=0, global_stats=None, fixed=False):
            assert fixed
            sc = self.fx.astype(np.float32) / np.float32(65536)
            return sc[:, :k], self.rows[:, :k], self.fx[:, :k]

    class Store:
        devices = [0, 1]

    # shard 0 holds global row 0 with the LOWER exact score, shard 1 global row 5 with the higher
    s0, s1 = Shard([big, 7 << 16], [0, 1]), Shard([big + 1, 0], [0, -1])
    lex = lexical.ShardedLex(Store(), _shards=[s0, s1],
                             _tables=[np.asarray([0, 2], np.int64), np.asarray([5], np.int64)])
    sc, rows = lex.search([[3, 4]], 3)
    assert rows[0].tolist() == [5, 0, 2]
    assert sc[0].tolist() == [np.float32(big + 1) / 65536, np.float32(big) / 65536, 7.0]
