"""CPU: request coalescing (super_rag_amd/coalesce.py) — concurrent single-query calls share a
device batch and get exactly the results they would get alone; failures reach every caller of the
failed batch; the connector's search and the embedder's embed_query use it (CPU doubles stand in
for the HIP store / encoder, tests/doubles.py)."""
import threading
import time

import numpy as np
import pytest

from doubles import HashEncoder, NumpyStore, TextTokenizer, hash_vec


def _hammer(fn, args, threads=24):
    out = [None] * len(args)
    errs = []
    start = threading.Barrier(threads)

    def worker(t):
        start.wait()
        for i in range(t, len(args), threads):
            try:
                out[i] = fn(args[i])
            except Exception as e:  # noqa: BLE001
                errs.append(e)
    ts = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
        assert not t.is_alive(), "coalescer deadlocked"
    return out, errs


def test_coalescer_batches_while_busy_and_keeps_per_item_results():
    from super_rag_amd.coalesce import Coalescer
    sizes = []

    def run(items):
        sizes.append(len(items))
        time.sleep(0.01)
        return [x * x for x in items]
    c = Coalescer(run, max_batch=8)
    out, errs = _hammer(c, list(range(96)))
    assert not errs
    assert out == [x * x for x in range(96)]
    assert max(sizes) <= 8 and c.items == 96
    assert c.batches < 96          # concurrent callers were batched
    assert c(7) == 49              # an idle coalescer runs a lone call at once


def test_coalescer_propagates_batch_failures():
    from super_rag_amd.coalesce import Coalescer

    def run(items):
        time.sleep(0.005)
        if any(x % 5 == 0 for x in items):
            raise ValueError("bad batch")
        return [x + 1 for x in items]
    c = Coalescer(run, max_batch=4)
    out, errs = _hammer(c, list(range(1, 41)), threads=8)
    assert errs and all(isinstance(e, ValueError) for e in errs)
    assert all(o is None or o == i + 2 for i, o in enumerate(out))
    assert c(3) == 4               # still serviceable after failures


def test_connector_coalesced_search_equals_one_by_one():
    from super_rag_amd import vectorstore as V
    from super_rag_amd.models import QueryWithEmbedding, TextNode
    V.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    V._collections.clear()
    try:
        rng = np.random.default_rng(0)
        conn = V.MI355XVectorStoreConnector({"collection": "coal", "coalesce": True, "max_batch": 16})
        vecs = rng.standard_normal((500, 16)).astype(np.float32)
        conn.store.add([TextNode(text=f"t{i}", metadata={"i": i}, embedding=v.tolist())
                        for i, v in enumerate(vecs)])
        qs = [QueryWithEmbedding(query=f"q{i}", top_k=1 + i % 9,
                                 embedding=rng.standard_normal(16).tolist()) for i in range(120)]
        solo = V.MI355XVectorStoreConnector({"collection": "coal", "coalesce": False})
        want = [[(d.text, d.score) for d in solo.search(q).results] for q in qs]
        got, errs = _hammer(lambda q: [(d.text, d.score) for d in conn.search(q).results], qs)
        assert not errs
        assert got == want
        c = V._collections["coal"]
        assert c.coalescer.items == len(qs) and c.coalescer.batches < len(qs)
    finally:
        V._collections.clear()
        V.set_store_backend(V._native_store, V._native_load)


def test_embed_query_coalesced_equals_one_by_one():
    from super_rag_amd.embed import EmbeddingService
    tok = TextTokenizer()
    enc = HashEncoder(tok, 8)
    svc = EmbeddingService("openai", "BAAI/bge-m3", "", "", 10, encoder=enc, tokenizer=tok)
    texts = [f"query number {i}\nwith a newline" for i in range(64)]
    got, errs = _hammer(svc.embed_query, texts, threads=16)
    assert not errs
    for t, g in zip(texts, got):
        np.testing.assert_allclose(g, hash_vec(t.replace("\n", " "), 8), atol=1e-6)
    assert enc._query_coalescer.items == 64
    with pytest.raises(Exception):
        svc.embed_query("   ")


def test_rerank_scores_coalesced_equal_one_by_one():
    from doubles import RelevanceEncoder, relevance
    from super_rag_amd.rerank import RerankService
    tok = TextTokenizer()
    enc = RelevanceEncoder(tok)
    svc = RerankService("jina_ai", "BAAI/bge-reranker-v2-m3", "", "", encoder=enc, tokenizer=tok,
                        device_batch=64)
    rng = np.random.default_rng(3)
    items = [(f"query {i}", [f"passage {j} of {i}" * int(rng.integers(1, 4))
                             for j in range(int(rng.integers(1, 30)))]) for i in range(40)]
    got, errs = _hammer(lambda it: svc.score(*it), items, threads=12)
    assert not errs
    for (q, ts), g in zip(items, got):
        np.testing.assert_allclose(g, [relevance(q, t) for t in ts], rtol=1e-6)
    assert enc._pair_coalescer.items == 40
