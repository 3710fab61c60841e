"""GPU: the drop-in boundary classes driven the way the reference drives them, on the HIP path.

EmbeddingService.embed_documents -> MI355XVectorStoreConnector.add / ContextManager.query ->
RerankService.async_rerank, every stage checked against the CPU oracle on the same token ids and
weights (oracle/encoder_ref.py, oracle/cosine_topk.py).  The connector's reference semantics
(score = cosine distance ascending, no ids in the documents, deletes by uuid, reorder-only rerank)
are asserted on real kernels, not on the CPU doubles of test_boundary.py."""
import asyncio
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from oracle import encoder_ref as R  # noqa: E402
from oracle.cosine_topk import cosine_topk, quantize_like_store  # noqa: E402


def _cfg(s):
    return R.RefConfig(s.vocab_size, s.hidden, s.layers, s.heads, s.intermediate, s.max_position,
                       s.type_vocab, s.ln_eps, s.position_offset, s.classifier, s.num_labels)


def _texts(n, seed):
    rng = np.random.default_rng(seed)
    words = [f"w{i}" for i in range(400)]
    return [" ".join(rng.choice(words, rng.integers(3, 40))) for _ in range(n)]


def test_embed_store_search_rerank_delete_through_the_drop_in_classes():
    from super_rag_amd.context import ContextManager
    from super_rag_amd.embed import EmbeddingService
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    from super_rag_amd.models import TextNode
    from super_rag_amd.rerank import RerankService
    from super_rag_amd.tokenizer import Tokenizer
    from super_rag_amd import vectorstore as V

    es = ModelSpec("t-bert", "bert", 30522, 256, 2, 4, 512, 128, 2, 1e-12, 0)
    rs = ModelSpec("t-xlmr", "xlmr", 30522, 256, 2, 4, 512, 130, 1, 1e-5, 1, classifier=1,
                   bos_id=0, eos_id=2, pad_id=1, max_length=128, residual_fp16=True)
    we, wr = random_weights(es, seed=3, style="test"), random_weights(rs, seed=4, style="test")
    wr["classifier.out_proj.weight"] *= 50.0
    etok, rtok = Tokenizer(es), Tokenizer(rs)
    emb = EmbeddingService("openai", "BAAI/bge-m3", "", "", 10, encoder=Encoder(es, weights=we),
                           tokenizer=etok, device_batch=64)
    rer = RerankService("jina_ai", "BAAI/bge-reranker-v2-m3", "", "", encoder=Encoder(rs, weights=wr),
                        tokenizer=rtok)

    # ingest: embed_documents == oracle on the same ids (per device batch, dynamic padding)
    docs = _texts(300, 1)
    vecs = np.asarray(emb.embed_documents(docs), dtype=np.float32)
    ref = np.concatenate([R.embed(_cfg(es), we, *etok.encode_batch([d])) for d in docs[:40]])
    assert np.linalg.norm(vecs[:40] - ref, axis=1).max() < 2e-3

    V._collections.clear()
    ctx = {"collection": "gpu_boundary", "device": 0}
    conn = V.VectorStoreConnectorAdaptor("mi355x", ctx).connector
    conn.create_collection(vector_size=es.hidden)
    ids = conn.store.add([TextNode(text=t, metadata={"i": i}, embedding=v.tolist())
                          for i, (t, v) in enumerate(zip(docs, vecs))])
    assert len(set(ids)) == len(docs)

    # query through ContextManager with the reference's kwargs: distances ascending, no ids
    cm = ContextManager("gpu_boundary", emb, "mi355x", ctx)
    q = "w7 w12 w300 w45"
    qv = np.asarray(emb.embed_query(q), dtype=np.float32)
    hits = cm.query(q, score_threshold=0.2, topk=8, vector=qv.tolist())
    stored = conn.get_vectors(ids).astype(np.float64)
    d_ref, r_ref = cosine_topk(stored, quantize_like_store(qv[None]), 8, normalize=False)
    assert [h.metadata["i"] for h in hits] == r_ref[0].tolist()
    np.testing.assert_allclose([h.score for h in hits], d_ref[0], atol=2e-3)
    assert all(not hasattr(h, "id") or getattr(h, "id", None) is None for h in hits)
    assert [h.score for h in hits] == sorted(h.score for h in hits)

    # rerank: permutation by oracle logits (desc, index asc), original distance scores kept
    out = asyncio.run(rer.async_rerank(q, hits))
    ids_p, mask_p, _ = rtok.encode_pairs(q, [h.text for h in hits])
    lg = R.cross_logits(_cfg(rs), wr, ids_p, mask_p)[:, 0]
    got_lg = rer.score(q, [h.text for h in hits])
    assert np.abs(got_lg - lg).max() <= 1e-2 * (1 + np.abs(lg).max())
    order = sorted(range(len(hits)), key=lambda i: (-got_lg[i], i))
    assert [o.metadata["i"] for o in out] == [hits[i].metadata["i"] for i in order]
    assert sorted(o.score for o in out) == sorted(h.score for h in hits)

    # delete by uuid: the deleted rows never come back
    top = hits[0].metadata["i"]
    conn.delete(ids=[ids[top]])
    again = cm.query(q, topk=8, vector=qv.tolist())
    assert top not in [h.metadata["i"] for h in again]
    assert [h.metadata["i"] for h in again[:7]] == r_ref[0].tolist()[1:8]
    conn.delete_collection()


def test_concurrent_requests_coalesce_into_device_batches_with_identical_results():
    # 48 concurrent single-query requests (the reference API is one query per request): the
    # embedder's embed_query, the connector's search and the reranker's scoring are coalesced into
    # shared device batches; every result equals the one-by-one result.
    import threading
    from super_rag_amd.embed import EmbeddingService
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    from super_rag_amd.models import QueryWithEmbedding, TextNode
    from super_rag_amd.rerank import RerankService
    from super_rag_amd.tokenizer import Tokenizer
    from super_rag_amd import vectorstore as V

    es = ModelSpec("t-bert", "bert", 30522, 256, 2, 4, 512, 128, 2, 1e-12, 0)
    rs = ModelSpec("t-xlmr", "xlmr", 30522, 256, 2, 4, 512, 130, 1, 1e-5, 1, classifier=1,
                   bos_id=0, eos_id=2, pad_id=1, max_length=128, residual_fp16=True)
    enc = Encoder(es, weights=random_weights(es, seed=5, style="test"))
    renc = Encoder(rs, weights=random_weights(rs, seed=6, style="test"))
    emb = EmbeddingService("openai", "m", "", "", 10, encoder=enc, tokenizer=Tokenizer(es))
    solo_emb = EmbeddingService("openai", "m", "", "", 10, encoder=enc, tokenizer=Tokenizer(es),
                                coalesce=False)
    rer = RerankService("jina_ai", "r", "", "", encoder=renc, tokenizer=Tokenizer(rs))
    solo_rer = RerankService("jina_ai", "r", "", "", encoder=renc, tokenizer=Tokenizer(rs),
                             coalesce=False)
    docs = _texts(2000, 7)
    V._collections.clear()
    conn = V.MI355XVectorStoreConnector({"collection": "gpu_coal", "device": 0})
    solo = V.MI355XVectorStoreConnector({"collection": "gpu_coal", "device": 0, "coalesce": False})
    conn.store.add([TextNode(text=t, metadata={"i": i}, embedding=v)
                    for i, (t, v) in enumerate(zip(docs, emb.embed_documents(docs)))])
    queries = _texts(48, 8)

    def one_by_one(q):
        v = solo_emb.embed_query(q)
        hits = solo.search(QueryWithEmbedding(query=q, top_k=10, embedding=v)).results
        return v, [(h.metadata["i"], h.score) for h in hits], solo_rer.score(q, [h.text for h in hits])

    def coalesced(q):
        v = emb.embed_query(q)
        hits = conn.search(QueryWithEmbedding(query=q, top_k=10, embedding=v)).results
        return v, [(h.metadata["i"], h.score) for h in hits], rer.score(q, [h.text for h in hits])

    want = [one_by_one(q) for q in queries]
    got = [None] * len(queries)
    start = threading.Barrier(16)

    def worker(t):
        start.wait()
        for i in range(t, len(queries), 16):
            got[i] = coalesced(queries[i])
    ts = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    for (v0, h0, l0), (v1, h1, l1) in zip(want, got):
        np.testing.assert_allclose(v1, v0, atol=1e-6)
        assert [i for i, _ in h1] == [i for i, _ in h0]
        np.testing.assert_allclose([s for _, s in h1], [s for _, s in h0], atol=1e-6)
        np.testing.assert_allclose(l1, l0, atol=1e-5)
    assert enc._query_coalescer.batches < len(queries)
    assert V._collections["gpu_coal"].coalescer.items == len(queries)
    conn.delete_collection()


def test_http_seam_on_the_hip_models():
    # the OpenAI /embeddings + Jina /rerank server in front of real HIP encoders returns what the
    # drop-in services return (the wire seam adds no numerics)
    from fastapi.testclient import TestClient
    from super_rag_amd.embed import EmbeddingService
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    from super_rag_amd.rerank import RerankService
    from super_rag_amd.server import create_app
    from super_rag_amd.tokenizer import Tokenizer

    es = ModelSpec("t-bert", "bert", 30522, 256, 2, 4, 512, 128, 2, 1e-12, 0)
    rs = ModelSpec("t-xlmr", "xlmr", 30522, 256, 2, 4, 512, 130, 1, 1e-5, 1, classifier=1,
                   bos_id=0, eos_id=2, pad_id=1, max_length=128, residual_fp16=True)
    emb = EmbeddingService("openai", "e", "", "", 10, encoder=Encoder(es, weights=random_weights(es, 9, "test")),
                           tokenizer=Tokenizer(es))
    rer = RerankService("jina_ai", "r", "", "", encoder=Encoder(rs, weights=random_weights(rs, 10, "test")),
                        tokenizer=Tokenizer(rs))
    client = TestClient(create_app(lambda m: emb, lambda m: rer))
    texts = _texts(20, 11)
    body = client.post("/v1/embeddings", json={"model": "BAAI/bge-m3", "input": texts}).json()
    np.testing.assert_allclose([d["embedding"] for d in body["data"]], emb.embed_documents(texts), atol=1e-6)
    q = "w3 w9 w27"
    res = client.post("/v1/rerank", json={"model": "BAAI/bge-reranker-v2-m3", "query": q,
                                          "documents": texts}).json()["results"]
    lg = rer.score(q, texts)
    assert [r["index"] for r in res] == sorted(range(len(texts)), key=lambda i: (-lg[i], i))


def test_ingest_write_path_long_chunks():
    # VectorIndexer.create/update/delete_index (index/vector_and_full_text_index.py:29-225) with
    # chunk-sized inputs (~400-600 tokens, truncated at the model's 512): GPU embeddings == oracle,
    # the chunks are searchable, updates replace ids, deletes remove them.
    from types import SimpleNamespace
    from super_rag_amd.embed import EmbeddingService
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    from super_rag_amd.index import VectorIndexer, chunk_text
    from super_rag_amd.models import QueryWithEmbedding
    from super_rag_amd.tokenizer import Tokenizer
    from super_rag_amd import vectorstore as V

    es = ModelSpec("t-small", "bert", 30522, 384, 2, 6, 1536, 512, 2, 1e-12, 0)
    w = random_weights(es, seed=12, style="test")
    tok = Tokenizer(es)
    svc = EmbeddingService("openai", "BAAI/bge-small-en", "", "", 10, encoder=Encoder(es, weights=w),
                           tokenizer=tok, device_batch=16)
    rng = np.random.default_rng(13)
    words = [f"t{i}" for i in range(3000)]
    parts = [SimpleNamespace(content=" ".join(rng.choice(words, int(rng.integers(380, 620)))),
                             metadata={"name": f"doc{i}.md", "titles": ["Doc", f"S{i}"]})
             for i in range(40)]
    V._collections.clear()
    conn = V.MI355XVectorStoreConnector({"collection": "gpu_ingest", "device": 0})
    ix = VectorIndexer(conn, svc)
    ids = ix.create_index(parts)["context_ids"]
    assert len(ids) == len(parts)
    texts = [chunk_text(p).replace("\n", " ") for p in parts]
    lens = [len(tok.encode_batch([t])[0][0]) for t in texts]
    assert max(lens) == 512                                  # truncated at max_length
    for i in (int(np.argmax(lens)), int(np.argmin(lens))):
        ref = R.embed(_cfg(es), w, *tok.encode_batch([texts[i]]))[0]
        got = conn.get_vectors([ids[i]])[0]
        assert np.linalg.norm(got - ref) < 4e-3              # fp16-stored row vs fp32 oracle
    qv = svc.embed_query(texts[5])
    hits = conn.search(QueryWithEmbedding(query="q", top_k=3, embedding=qv)).results
    assert hits[0].metadata["source"] == "doc5.md" and hits[0].score < 1e-3
    new_ids = ix.update_index(ids[:10], parts[:10])["context_ids"]
    assert not set(new_ids) & set(ids) and conn.store is conn
    n_rows, n_live = V._collections["gpu_ingest"].store.count()
    assert n_live == len(parts)
    ix.delete_index(new_ids + ids[10:])
    assert V._collections["gpu_ingest"].store.count()[1] == 0
    conn.delete_collection()


def test_native_library_first_then_torch_in_one_process():
    # PyTorch bundles its own HIP runtime: the binding must not let the native library bind a
    # second one that torch then cannot initialise (_native.load imports torch first).
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "from super_rag_amd import _native as N\n"
            "from super_rag_amd.lexical import rrf_fuse\n"
            "import numpy as np\n"
            "N.require_gpu(); rrf_fuse(np.array([[1, 2]]), np.array([[2, 3]]), 3)\n"
            "import torch; torch.cuda.init(); assert torch.cuda.device_count() >= 1\n"
            "print('ok')\n") % (root, os.path.join(root, "super-rag_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110)
    assert out.returncode == 0 and "ok" in out.stdout, out.stderr[-2000:]
