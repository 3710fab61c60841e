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


def test_rerank_batch_width_is_bucketed_and_padding_is_masked():
    # _score_many pads a device batch to 128 (<= 128 tokens) or a multiple of 16 within the model's
    # max_length, so per-request batches take the S = 128 fused attention and the K/V-free last
    # layer; the padding is masked, so the logits equal the unpadded ones.  The device calls are
    # counted under the "rerank" stage of device_gate.
    from types import SimpleNamespace
    from super_rag_amd._native import gate_busy
    from super_rag_amd.rerank import RerankService

    class Tok:
        def encode_pairs(self, q, texts):
            w = len(q)
            ids = np.arange(len(texts) * w, dtype=np.int32).reshape(len(texts), w) + 3
            mask = np.ones_like(ids)
            mask[:, w - 2:] = np.arange(len(texts))[:, None] % 2  # ragged rows
            return ids, mask, np.zeros_like(ids)

    class Enc:
        spec = SimpleNamespace(pad_id=1, pair_style=0, max_length=512)
        device = 0

        def __init__(self):
            self.widths = []

        def cross_score(self, ids, mask, types=None):
            self.widths.append(ids.shape[1])
            return ((ids * mask).sum(1, dtype=np.int64) % 10007).astype(np.float32)[:, None]

    tok = Tok()
    for w, want in [(7, 128), (100, 128), (128, 128), (130, 144), (505, 512), (512, 512)]:
        enc = Enc()
        before = gate_busy().get(0, {}).get("rerank", (0.0, 0))[1]
        items = [("q" * w, ["a", "b", "c"]), ("q" * max(1, w - 5), ["d"])]
        got = RerankService._score_many(enc, tok, 4096, items)
        assert enc.widths == [want]
        for (q, ts), g in zip(items, got):
            ids, mask, _ = tok.encode_pairs(q, ts)
            np.testing.assert_array_equal(g, ((ids * mask).sum(1, dtype=np.int64) % 10007).astype(np.float32))
        assert gate_busy()[0]["rerank"][1] == before + 1


def test_devices_gate_takes_every_shard_device_in_order():
    """a sharded collection's search holds the gate of EVERY device it computes on
    (ascending order), so it serialises with embed / rerank batches on those devices and its busy
    time is charged to each of them; a single-device store keeps its one gate."""
    import threading
    from super_rag_amd._native import devices_gate, gate_busy, device_gate
    from super_rag_amd.vectorstore import _store_devices

    class Sharded:
        devices = [3, 1, 2]

    class One:
        device = 5

    assert _store_devices(Sharded()) == [3, 1, 2] and _store_devices(One()) == [5]
    before = gate_busy()
    with devices_gate([3, 1, 2, 1], "search"):
        # another thread cannot take device 2's gate while the sharded search holds it
        got = []

        def other():
            with device_gate(2, "embed"):
                got.append(1)
        t = threading.Thread(target=other)
        t.start()
        t.join(0.2)
        assert t.is_alive() and not got
    t.join(2.0)
    assert not t.is_alive() and got == [1]
    after = gate_busy()
    for d in (1, 2, 3):
        assert after[d]["search"][1] == before.get(d, {}).get("search", (0, 0))[1] + 1


def test_coalescer_acall_batches_coroutines_without_threads_and_mixes_with_threads():
    """Coalescer.acall: concurrent coroutines share batches, each gets its own item's result,
    a failing batch raises in every coroutine of it, and thread callers on the same queue still
    get theirs (a coroutine's slot is led by the worker thread, a thread caller's by itself)."""
    import asyncio
    from super_rag_amd.coalesce import Coalescer
    sizes = []
    gate = threading.Event()

    def run(items):
        sizes.append(len(items))
        gate.wait(0.02)
        if any(i == -1 for i in items):
            raise ValueError("bad item")
        return [i * i for i in items]

    c = Coalescer(run, max_batch=16)

    async def many(n):
        return await asyncio.gather(*[c.acall(i) for i in range(n)])

    got = asyncio.run(many(200))
    assert got == [i * i for i in range(200)]
    assert max(sizes) > 1 and sum(sizes) == 200 and c.items == 200

    async def failing():
        return await asyncio.gather(c.acall(3), c.acall(-1), return_exceptions=True)

    res = asyncio.run(failing())
    assert any(isinstance(r, ValueError) for r in res)

    # threads and coroutines on one queue
    out_threads = {}

    def thread_caller(i):
        out_threads[i] = c(i)

    async def mixed():
        ts = [threading.Thread(target=thread_caller, args=(1000 + i,)) for i in range(8)]
        for t in ts:
            t.start()
        vals = await asyncio.gather(*[c.acall(i) for i in range(64)])
        for t in ts:
            t.join(timeout=30)
            assert not t.is_alive()
        return vals

    vals = asyncio.run(mixed())
    assert vals == [i * i for i in range(64)]
    assert out_threads == {1000 + i: (1000 + i) ** 2 for i in range(8)}


def test_async_paths_equal_the_sync_ones():
    """The coroutine paths the flow uses -- EmbeddingService.aembed_query, ContextManager.aquery
    (connector.asearch) and RerankService.async_rerank -- await Coalescer.acall and return what
    the sync calls return, concurrently, with the empty-query error kept."""
    import asyncio
    from super_rag_amd import vectorstore as V
    from super_rag_amd.context import ContextManager
    from super_rag_amd.embed import EmbeddingService
    from super_rag_amd.models import TextNode
    from doubles import RelevanceEncoder
    from super_rag_amd.rerank import RerankService
    V.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    V._collections.clear()
    try:
        tok = TextTokenizer()
        enc = HashEncoder(tok, 16)
        emb = EmbeddingService("openai", "BAAI/bge-m3", "", "", 10, encoder=enc, tokenizer=tok)
        conn = V.MI355XVectorStoreConnector({"collection": "acoal", "coalesce": True, "max_batch": 16})
        rng = np.random.default_rng(1)
        conn.store.add([TextNode(text=f"passage {i} " * int(rng.integers(1, 4)), metadata={"i": i},
                                 embedding=rng.standard_normal(16).tolist()) for i in range(300)])
        cm = ContextManager("acoal", emb, "mi355x", {"collection": "acoal", "coalesce": True,
                                                     "max_batch": 16})
        rer = RerankService("jina_ai", "BAAI/bge-reranker-v2-m3", "", "", encoder=RelevanceEncoder(tok),
                            tokenizer=tok, device_batch=256)
        queries = [f"query {i}" for i in range(48)]

        def sync_one(q):
            docs = cm.query(q, topk=1 + len(q) % 7, index_types=["vector"])
            return [(d.text, d.score) for d in docs]

        want = [sync_one(q) for q in queries]

        async def async_one(q):
            v = await emb.aembed_query(q)
            docs = await cm.aquery(q, topk=1 + len(q) % 7, vector=v, index_types=["vector"])
            ranked = await rer.async_rerank(q, docs)
            return [(d.text, d.score) for d in docs], [d.text for d in ranked]

        async def run_all():
            return await asyncio.gather(*[async_one(q) for q in queries])

        got = asyncio.run(run_all())
        assert [g[0] for g in got] == want
        for q, (docs, ranked) in zip(queries, got):
            assert sorted(ranked) == sorted(t for t, _ in docs)
        assert enc._query_coalescer.items == 2 * len(queries)  # sync + async
        with pytest.raises(Exception):
            asyncio.run(emb.aembed_query("   "))
    finally:
        V._collections.clear()
        V.set_store_backend(V._native_store, V._native_load)


def test_coalescer_fill_wait():
    """min_fill / max_wait_s: a leader that finds fewer than min_fill items waits (up to
    max_wait_s) for more, so items arriving meanwhile share its batch; alone, it runs once the
    wait expires.  Results stay per item."""
    from super_rag_amd.coalesce import Coalescer
    sizes = []

    def run(items):
        sizes.append(len(items))
        return [i * 10 for i in items]

    c = Coalescer(run, max_batch=16, min_fill=4, max_wait_s=2.0)
    out = {}

    def call(i):
        out[i] = c(i)

    ts = [threading.Thread(target=call, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
        time.sleep(0.05)
    for t in ts:
        t.join(10)
    assert out == {i: i * 10 for i in range(4)} and sizes == [4]
    c2 = Coalescer(run, max_batch=16, min_fill=8, max_wait_s=0.1)
    t0 = time.monotonic()
    assert c2(7) == 70
    assert 0.09 <= time.monotonic() - t0 < 2.0 and sizes[-1] == 1


def test_fused_embed_search_equals_embed_then_search():
    """ContextManager.aquery_text (the flow's vector search: one coalesced embed + search step,
    MI355XVectorStoreConnector.asearch_text) returns what aembed_query + aquery return, for
    concurrent requests with mixed top_k, batches them, and keeps the empty-query error; a
    connector that cannot fuse (not coalescing) falls back to the two-step path."""
    import asyncio
    from super_rag_amd import vectorstore as V
    from super_rag_amd.context import ContextManager
    from super_rag_amd.embed import EmbeddingService
    from super_rag_amd.errors import EmptyTextError
    from super_rag_amd.models import TextNode
    V.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    V._collections.clear()
    try:
        tok = TextTokenizer()
        enc = HashEncoder(tok, 16)
        emb = EmbeddingService("openai", "BAAI/bge-m3", "", "", 10, encoder=enc, tokenizer=tok)
        ctx = {"collection": "fused", "coalesce": True, "max_batch": 16}
        conn = V.MI355XVectorStoreConnector(dict(ctx))
        rng = np.random.default_rng(2)
        conn.store.add([TextNode(text=f"passage {i}", metadata={"i": i},
                                 embedding=rng.standard_normal(16).tolist()) for i in range(400)])
        cm = ContextManager("fused", emb, "mi355x", dict(ctx))
        queries = [f"query {i}\nline two" if i % 5 == 0 else f"query {i}" for i in range(60)]

        async def two_step(q):
            v = await emb.aembed_query(q)
            docs = await cm.aquery(q, topk=1 + i_of[q] % 9, vector=v, index_types=["vector"])
            return [(d.text, d.score) for d in docs]

        async def fused(q):
            docs = await cm.aquery_text(q, topk=1 + i_of[q] % 9, index_types=["vector"])
            return [(d.text, d.score) for d in docs]

        i_of = {q: i for i, q in enumerate(queries)}

        async def run_all(fn):
            return await asyncio.gather(*[fn(q) for q in queries])

        want = asyncio.run(run_all(two_step))
        got = asyncio.run(run_all(fused))
        assert got == want
        co = list(V._collections["fused"].text_coalescers.values())
        assert len(co) == 1 and co[0].items == len(queries) and co[0].batches < len(queries)
        with pytest.raises(EmptyTextError):
            asyncio.run(cm.aquery_text("  ", topk=3))
        solo = ContextManager("fused", emb, "mi355x", {"collection": "fused", "coalesce": False})
        assert asyncio.run(solo.aquery_text(queries[3], topk=4, index_types=["vector"])) == \
            asyncio.run(cm.aquery(queries[3], topk=4, index_types=["vector"]))
    finally:
        V._collections.clear()
        V.set_store_backend(V._native_store, V._native_load)


def test_thread_caller_does_not_serve_coroutines_after_its_own_batch():
    """A thread caller that leads a batch hands the coroutines queued behind it to the coalescer's
    own leader thread: it returns after its own batch instead of running theirs."""
    import asyncio
    from super_rag_amd.coalesce import Coalescer
    ran_in = []
    started = threading.Event()

    def run(items):
        ran_in.append((threading.current_thread().name, list(items)))
        if items == ["sync"]:
            started.set()
            time.sleep(0.2)  # the coroutines queue up behind this batch
        return [f"r-{i}" for i in items]

    c = Coalescer(run, max_batch=4)
    out = {}

    def sync_caller():
        out["sync"] = c("sync")
        out["sync_done_batches"] = c.batches

    t = threading.Thread(target=sync_caller, name="sync-caller")
    t.start()
    started.wait(5)

    async def coros():
        return await asyncio.gather(*[c.acall(i) for i in range(10)])

    vals = asyncio.run(coros())
    t.join(10)
    assert not t.is_alive()
    assert out["sync"] == "r-sync" and vals == [f"r-{i}" for i in range(10)]
    # the sync caller ran exactly its own batch
    assert [n for n, items in ran_in if n == "sync-caller"] == ["sync-caller"]


@pytest.mark.timeout(60)
def test_coroutines_are_served_when_the_loop_executor_is_full_or_the_loop_thread_blocks():
    """the coroutines' leader must not need a worker of the caller's event loop.
    (a) the loop's default executor has ONE worker, held by a sync caller blocked on the same
    coalescer (asyncio.to_thread(c, ...)) while coroutines queue; (b) a sync __call__ made on the
    loop thread itself while coroutines of that loop are queued.  Both finish, results per item."""
    import asyncio
    import concurrent.futures as cf
    from super_rag_amd.coalesce import Coalescer
    started = threading.Event()

    def run(items):
        if "slow" in items:
            started.set()
            time.sleep(0.15)
        return [f"r-{i}" for i in items]

    c = Coalescer(run, max_batch=4)

    async def case_a():
        loop = asyncio.get_running_loop()
        loop.set_default_executor(cf.ThreadPoolExecutor(max_workers=1))
        blocked = asyncio.create_task(asyncio.to_thread(c, "slow"))
        while not started.is_set():
            await asyncio.sleep(0.005)
        more_sync = [asyncio.create_task(asyncio.to_thread(c, f"s{i}")) for i in range(3)]
        vals = await asyncio.wait_for(asyncio.gather(*[c.acall(i) for i in range(12)]), 10)
        rest = await asyncio.wait_for(asyncio.gather(blocked, *more_sync), 10)
        return vals, rest

    vals, rest = asyncio.run(case_a())
    assert vals == [f"r-{i}" for i in range(12)]
    assert rest == ["r-slow"] + [f"r-s{i}" for i in range(3)]

    started.clear()

    async def case_b():
        queued = [asyncio.ensure_future(c.acall(i)) for i in range(6)]
        await asyncio.sleep(0)  # the coroutines enqueue; the loop thread then blocks in __call__
        own = c("slow")
        vals = await asyncio.wait_for(asyncio.gather(*queued), 10)
        return own, vals

    own, vals = asyncio.run(case_b())
    assert own == "r-slow" and vals == [f"r-{i}" for i in range(6)]
    assert not c._busy
