"""CPU: the OpenAI /embeddings + Jina /rerank wire seam (super_rag_amd/server.py) — request and
response shapes of the dialects litellm speaks for the reference (embedding_service.py:168-175,
rerank_service.py:95-104), ordering, top_n, errors.  CPU doubles stand in for the encoders."""
import base64

import numpy as np
import pytest

from doubles import HashEncoder, RelevanceEncoder, TextTokenizer, hash_vec, relevance


@pytest.fixture
def client():
    from fastapi.testclient import TestClient
    from super_rag_amd.embed import EmbeddingService
    from super_rag_amd.rerank import RerankService
    from super_rag_amd.server import create_app

    def emb(model):
        tok = TextTokenizer()
        return EmbeddingService("openai", model, "", "", 10, encoder=HashEncoder(tok, 8), tokenizer=tok)

    def rer(model):
        tok = TextTokenizer()
        return RerankService("jina_ai", model, "", "", encoder=RelevanceEncoder(tok), tokenizer=tok)
    return TestClient(create_app(emb, rer))


def test_openai_embeddings_dialect(client):
    for path in ("/v1/embeddings", "/embeddings"):
        r = client.post(path, json={"model": "BAAI/bge-m3", "input": ["a b\nc", "dd", ""]})
        assert r.status_code == 200
        body = r.json()
        assert body["object"] == "list" and body["model"] == "BAAI/bge-m3"
        assert [d["index"] for d in body["data"]] == [0, 1, 2]
        # same cleaning as the reference: '\n' -> ' ', empty -> ' '
        for d, t in zip(body["data"], ["a b c", "dd", " "]):
            assert d["object"] == "embedding"
            np.testing.assert_allclose(d["embedding"], hash_vec(t, 8), atol=1e-6)
    r = client.post("/v1/embeddings", json={"input": "single", "encoding_format": "base64"})
    v = np.frombuffer(base64.b64decode(r.json()["data"][0]["embedding"]), dtype="<f4")
    np.testing.assert_allclose(v, hash_vec("single", 8), atol=1e-6)
    assert client.post("/v1/embeddings", json={"input": []}).status_code == 400
    assert client.post("/v1/embeddings", json={"input": ["", " "]}).status_code == 400


def test_jina_rerank_dialect(client):
    q = "rerank me"
    docs = ["unrelated", "rerank", {"text": "me too"}, "", "rerank me please"]
    texts = ["unrelated", "rerank", "me too", " ", "rerank me please"]
    want = sorted(range(5), key=lambda i: (-relevance(q, texts[i]), i))
    for path in ("/v1/rerank", "/rerank"):
        r = client.post(path, json={"model": "BAAI/bge-reranker-v2-m3", "query": q,
                                    "documents": docs, "return_documents": False})
        assert r.status_code == 200
        res = r.json()["results"]
        assert [x["index"] for x in res] == want
        assert all("document" not in x for x in res)
        s = [x["relevance_score"] for x in res]
        assert s == sorted(s, reverse=True) and all(0.0 < x < 1.0 for x in s)
    r = client.post("/v1/rerank", json={"query": q, "documents": docs, "top_n": 2,
                                        "return_documents": True})
    res = r.json()["results"]
    assert [x["index"] for x in res] == want[:2]
    assert res[0]["document"]["text"] == texts[want[0]]
    assert client.post("/v1/rerank", json={"query": " ", "documents": ["x"]}).status_code == 400
    assert client.post("/v1/rerank", json={"query": "q", "documents": ["x"] * 1001}).status_code == 400
    assert client.post("/v1/rerank", json={"query": "q", "documents": []}).json()["results"] == []
