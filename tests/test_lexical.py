"""CPU: BM25 / rrf oracle pinned (rrf against fixtures captured from the reference's own function;
BM25 fixed point against a scalar fp64 restatement), the host-side analyzer / vocabulary / array
packing, and the connector's fulltext + hybrid paths over test doubles."""
import json
import os

import numpy as np
import pytest

from doubles import NumpyLex, NumpyStore

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rrf_fixtures.json")


def test_rrf_oracle_matches_reference_fixtures():
    from oracle.bm25 import rrf
    cases = json.load(open(GOLD))["cases"]
    assert len(cases) >= 40
    for c in cases:
        ids, scores = rrf(c["lists"], rank_const=c["rank_const"], min_score=c["min_score"])
        assert ids == c["ids"]
        assert [float(s).hex() for s in scores] == c["scores"]   # bit-exact doubles


def test_rrf_rows_pads_and_cuts():
    from oracle.bm25 import rrf_rows
    s, r = rrf_rows(np.array([[3, 1, -1]]), np.array([[1, 7, 3]]), 5)
    # 1: 1/2 + 1/1, 3: 1/1 + 1/3, 7: 1/2
    assert r.tolist() == [[1, 3, 7, -1, -1]]
    assert s[0, :3].tolist() == [1.5, 1 + 1 / 3, 0.5] and np.isinf(s[0, 3:]).all()


def _corpus(rng, n, vocab, zipf=1.3, max_len=60):
    docs = [list((rng.zipf(zipf, rng.integers(0, max_len)) - 1) % vocab) for _ in range(n)]
    return docs


def test_bm25_fixed_point_matches_scalar_restatement():
    from oracle.bm25 import LexCorpus, bm25_fixed_scores, bm25_scores_loop, bm25_topk
    from super_rag_amd.lexical import doc_arrays
    rng = np.random.default_rng(1)
    docs = _corpus(rng, 250, 150)
    off, t, tf, dl = doc_arrays(docs)
    C = LexCorpus(off, t, tf, dl)
    C.remove([0, 7, 11])
    D = C.docs()
    queries = [list((rng.zipf(1.3, rng.integers(1, 6)) - 1) % 150) for _ in range(12)]
    queries.append([3, 3, 3])          # multiplicity
    queries.append([10 ** 6])          # unknown term
    queries.append([])                 # empty query
    for q in queries:
        ref = np.asarray(bm25_scores_loop(D, dl.tolist(), C.live.tolist(), q))
        fx = bm25_fixed_scores(C, q) / 65536.0
        # each term contributes <= 0.5 ulp of 2^-16 (+ the max(1, .) floor) of fixed-point error
        assert np.abs(fx - ref).max(initial=0) <= len(q) * 2 ** -16 + 1e-9
        assert (fx[~C.live] == 0).all()
    s, r = bm25_topk(C, queries, 7)
    assert (r[-1] == -1).all() and (r[-2] == -1).all()
    for i in range(len(queries)):
        valid = r[i] >= 0
        assert (np.diff(s[i][valid]) <= 0).all()


def test_analyzer_vocab_and_arrays():
    from super_rag_amd.lexical import Vocab, analyze, doc_arrays, query_arrays
    assert analyze("Hello, World! héllo_2 x") == ["hello", "world", "héllo_2", "x"]
    assert analyze(None) == [] and analyze("") == []
    v = Vocab()
    a = v.doc_ids(["b", "a", "b"])
    assert a == [0, 1, 0] and v.query_ids(["a", "zzz", "b"]) == [1, 0]
    assert Vocab(v.terms).ids == v.ids
    off, terms, tf, dl = doc_arrays([[5, 3, 5], [], [2]])
    assert off.tolist() == [0, 2, 2, 3] and terms.tolist() == [5, 3, 2]
    assert tf.tolist() == [2, 1, 1] and dl.tolist() == [3, 0, 1]
    qoff, qt = query_arrays([[1, 1], []])
    assert qoff.tolist() == [0, 2, 2] and qt.tolist() == [1, 1]


@pytest.fixture
def conn_factory():
    from super_rag_amd import vectorstore as V
    V.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    V.set_lex_backend(lambda dev: NumpyLex(dev), NumpyLex.load)
    V._collections.clear()
    yield lambda **kw: V.MI355XVectorStoreConnector({"collection": "lex", **kw})
    V._collections.clear()
    V.set_store_backend(V._native_store, V._native_load)
    V.set_lex_backend(V._native_lex, V._native_lex_load)


WORDS = "alpha beta gamma delta epsilon zeta eta theta iota kappa lambda mu".split()


def _nodes(rng, n, dim=6):
    from super_rag_amd.models import TextNode
    out = []
    for i in range(n):
        words = rng.choice(WORDS, size=rng.integers(1, 12)).tolist()
        out.append(TextNode(text=" ".join(words) + f" doc{i}", metadata={"i": i, "chat": i % 2},
                            embedding=rng.standard_normal(dim).tolist()))
    return out


def test_connector_fulltext_search_is_bm25_over_texts(conn_factory, tmp_path):
    from oracle.bm25 import LexCorpus, bm25_topk
    from super_rag_amd.lexical import Vocab, analyze, doc_arrays
    rng = np.random.default_rng(2)
    conn = conn_factory(fulltext=True, snapshot_dir=str(tmp_path), honor_filter=True)
    nodes = _nodes(rng, 80)
    ids = conn.store.add(nodes[:50])
    ids += conn.store.add(nodes[50:])
    conn.delete(ids=[ids[3], ids[4]])
    voc = Vocab()
    docs = [voc.doc_ids(analyze(n.text)) for n in nodes]
    live = np.ones(80, bool)
    live[[3, 4]] = False
    C = LexCorpus(*doc_arrays(docs), live)
    for text, kw in (("gamma delta", None), ("Alpha alpha mu", None), ("", ["kappa", "zeta"]),
                     ("nothing-known", None)):
        hits = conn.fulltext_search(text, 6, keywords=kw)
        q = voc.query_ids(analyze(" ".join(kw) if kw else text))
        s, r = bm25_topk(C, [q], 6)
        want = [int(x) for x in r[0] if x >= 0]
        assert [h.metadata["i"] for h in hits] == want
        np.testing.assert_array_equal([h.score for h in hits], s[0][: len(want)])
    # metadata filter (honor_filter) restricts the candidates
    hits = conn.fulltext_search("beta", 50, filter={"chat": 1})
    assert hits and all(h.metadata["chat"] == 1 for h in hits)
    # snapshot: a fresh registry reloads the lexical index and vocabulary
    from super_rag_amd import vectorstore as V
    V._collections.clear()
    conn2 = conn_factory(fulltext=True, snapshot_dir=str(tmp_path))
    assert [h.metadata["i"] for h in conn2.fulltext_search("gamma delta", 6)] == \
        [h.metadata["i"] for h in conn.fulltext_search("gamma delta", 6)]


def test_connector_hybrid_search_is_rrf_of_dense_and_bm25(conn_factory):
    from oracle.bm25 import rrf
    from super_rag_amd.models import QueryWithEmbedding
    rng = np.random.default_rng(3)
    conn = conn_factory(hybrid=True, hybrid_k_each=8)
    nodes = _nodes(rng, 60)
    conn.store.add(nodes)
    plain = conn_factory(fulltext=True)
    for _ in range(4):
        qv = rng.standard_normal(6)
        text = " ".join(rng.choice(WORDS, 3))
        res = conn.search(QueryWithEmbedding(query=text, top_k=5, embedding=qv.tolist())).results
        dense = plain.search(QueryWithEmbedding(query=text, top_k=8, embedding=qv.tolist())).results
        lexical = plain.fulltext_search(text, 8)
        ids, scores = rrf([[d.metadata["i"] for d in dense], [d.metadata["i"] for d in lexical]])
        assert [d.metadata["i"] for d in res] == ids[:5]
        assert [d.score for d in res] == scores[:5]


def test_fulltext_backfills_rows_added_before_it_was_enabled(conn_factory):
    rng = np.random.default_rng(4)
    plain = conn_factory()
    nodes = _nodes(rng, 20)
    ids = plain.store.add(nodes)
    plain.delete(ids=[ids[0]])
    ft = conn_factory(fulltext=True)
    hits = ft.fulltext_search("doc0 doc1 doc5", 5)
    assert sorted(h.metadata["i"] for h in hits) == [1, 5]
    ft.store.add(_nodes(rng, 3))    # rows stay in step after the back-fill
    assert ft.fulltext_search("doc2", 3)[0].metadata["i"] == 2


def test_fulltext_search_node_runner(conn_factory, monkeypatch):
    import asyncio
    from super_rag_amd import nodeflow_pack as P
    monkeypatch.setenv("SUPER_RAG_AMD_VECTOR_DB_CONTEXT", json.dumps({"fulltext": True,
                                                                      "honor_filter": True}))
    P.register()
    assert "fulltext_search" in P.NODE_RUNNER_REGISTRY
    P.register_collection(P.LocalCollection("lex", {"embedding": {"model": "bge-m3"}}))
    from super_rag_amd.models import TextNode
    from super_rag_amd.vectorstore import MI355XVectorStoreConnector
    con = MI355XVectorStoreConnector({"collection": "lex", "fulltext": True})
    con.add([TextNode(text=t, metadata={"chat_id": c}, embedding=[1.0, float(i)])
             for i, (t, c) in enumerate([("red apple pie", "a"), ("green apple", "b"),
                                         ("blue sky", "a"), ("apple apple tart", "a")])])
    runner = P.NODE_RUNNER_REGISTRY["fulltext_search"]["runner"]
    out, so = asyncio.run(runner.run(P.FulltextSearchInput(top_k=5, collection_ids=["lex"]),
                                     P.SystemInput(query="apple", user="u")))
    assert so == {} and [d.text for d in out.docs][0] == "apple apple tart"
    assert {d.text for d in out.docs} == {"red apple pie", "green apple", "apple apple tart"}
    assert all(d.metadata["recall_type"] == "fulltext_search" for d in out.docs)
    # keywords replace the query terms; chat_id filters
    out, _ = asyncio.run(runner.run(P.FulltextSearchInput(keywords=["sky"], collection_ids=["lex"]),
                                    P.SystemInput(query="apple", user="u")))
    assert [d.text for d in out.docs] == ["blue sky"]
    out, _ = asyncio.run(runner.run(P.FulltextSearchInput(chat_id="b", collection_ids=["lex"]),
                                    P.SystemInput(query="apple", user="u")))
    assert [d.text for d in out.docs] == ["green apple"]
    out, _ = asyncio.run(runner.run(P.FulltextSearchInput(collection_ids=["missing"]),
                                    P.SystemInput(query="apple", user="u")))
    assert out.docs == []
