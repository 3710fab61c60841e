"""Wire-level seam: an HTTP server speaking the two dialects the reference's
model clients use, backed by the in-process MI355X encoders.

The reference reaches its models through litellm with ``api_base = LLMProvider.base_url``
(embedding_service.py:168-175: ``litellm.embedding(custom_llm_provider="openai", ...)``;
rerank_service.py:95-104: ``litellm.arerank(custom_llm_provider="jina_ai",
return_documents=False, ...)``).  Pointing a provider's ``base_url`` at this server is a zero-code
drop-in for an unmodified reference deployment:

  POST /v1/embeddings, /embeddings   OpenAI: {"model", "input": str | [str], "encoding_format"?}
      -> {"object": "list", "data": [{"object": "embedding", "index", "embedding"}], "model", "usage"}
  POST /v1/rerank, /rerank           Jina: {"model", "query", "documents": [str | {"text"}],
                                     "top_n"?, "return_documents"?}
      -> {"model", "results": [{"index", "relevance_score", "document"?}], "usage"}

Embeddings are the model's pooled, L2-normalised vectors (embed.EmbeddingService); rerank results
are ordered by cross-encoder logit (desc, index asc) with ``relevance_score = sigmoid(logit)`` (the
bge-reranker normalisation; the reference only consumes the order, rerank_service.py:115-135).
Requests run in FastAPI's worker threads, so concurrent requests coalesce into device batches
(coalesce.py).  Errors map to HTTP 400 (validation) / 500 (device) with an OpenAI-style body.
"""
import base64
import math
import threading
from typing import Any, Callable, Dict, List, Optional, Union

import numpy as np
from pydantic import BaseModel


class EmbeddingRequest(BaseModel):
    model: Optional[str] = None
    input: Union[str, List[str]]
    encoding_format: Optional[str] = "float"
    user: Optional[str] = None
    dimensions: Optional[int] = None


class RerankRequest(BaseModel):
    model: Optional[str] = None
    query: str
    documents: List[Union[str, Dict[str, Any]]]
    top_n: Optional[int] = None
    return_documents: Optional[bool] = False


def _services(embedder_factory: Optional[Callable[[str], Any]],
              reranker_factory: Optional[Callable[[str], Any]]):
    lock = threading.Lock()
    emb: Dict[str, Any] = {}
    rer: Dict[str, Any] = {}

    def default_embedder(model: str):
        from .embed import EmbeddingService
        return EmbeddingService("openai", model, "", "", 10)

    def default_reranker(model: str):
        from .rerank import RerankService
        return RerankService("jina_ai", model, "", "")

    ef = embedder_factory or default_embedder
    rf = reranker_factory or default_reranker

    def get(cache, factory, model):
        with lock:
            s = cache.get(model)
            if s is None:
                s = factory(model)
                cache[model] = s
            return s
    return (lambda m: get(emb, ef, m)), (lambda m: get(rer, rf, m))


def create_app(embedder_factory: Optional[Callable[[str], Any]] = None,
               reranker_factory: Optional[Callable[[str], Any]] = None,
               default_embed_model: str = "BAAI/bge-m3",
               default_rerank_model: str = "BAAI/bge-reranker-v2-m3"):
    """FastAPI app.  The factories map a request's model name to an EmbeddingService /
    RerankService (default: the resident registry models of embed.py / rerank.py)."""
    from fastapi import FastAPI
    from fastapi.responses import JSONResponse

    from .errors import EmbeddingError, EmptyTextError, InvalidDocumentError, TooManyDocumentsError

    get_embedder, get_reranker = _services(embedder_factory, reranker_factory)
    app = FastAPI(title="super-rag MI355X model server")

    def error(status: int, message: str, kind: str):
        return JSONResponse(status_code=status,
                            content={"error": {"message": message, "type": kind, "code": status}})

    def embeddings(req: EmbeddingRequest):
        model = req.model or default_embed_model
        texts = [req.input] if isinstance(req.input, str) else list(req.input)
        try:
            svc = get_embedder(model)
            vecs = np.asarray(svc.embed_documents(texts), dtype=np.float32)
        except (EmptyTextError, ValueError, KeyError) as e:
            return error(400, str(e), "invalid_request_error")
        except EmbeddingError as e:
            return error(500, str(e), "server_error")
        if req.dimensions:
            if req.dimensions > vecs.shape[1]:
                return error(400, f"dimensions {req.dimensions} > model dimension {vecs.shape[1]}",
                             "invalid_request_error")
            vecs = vecs[:, : req.dimensions]
            vecs /= np.maximum(np.linalg.norm(vecs, axis=1, keepdims=True), 1e-12)
        data = []
        for i, v in enumerate(vecs):
            emb = (base64.b64encode(v.astype("<f4").tobytes()).decode()
                   if req.encoding_format == "base64" else v.tolist())
            data.append({"object": "embedding", "index": i, "embedding": emb})
        tokens = _count_tokens(svc, texts)
        return {"object": "list", "data": data, "model": model,
                "usage": {"prompt_tokens": tokens, "total_tokens": tokens}}

    def rerank(req: RerankRequest):
        model = req.model or default_rerank_model
        texts = [d if isinstance(d, str) else str(d.get("text", "")) for d in req.documents]
        if not req.query or not req.query.strip():
            return error(400, "Query cannot be empty", "invalid_request_error")
        if not texts:
            return {"model": model, "results": [], "usage": {"total_tokens": 0}}
        try:
            svc = get_reranker(model)
            if len(texts) > svc.max_documents:
                raise TooManyDocumentsError(document_count=len(texts), max_documents=svc.max_documents,
                                            model_name=model)
            logits = np.asarray(svc.score(req.query, [t if t.strip() else " " for t in texts]))
        except (InvalidDocumentError, TooManyDocumentsError, ValueError, KeyError) as e:
            return error(400, str(e), "invalid_request_error")
        except Exception as e:  # noqa: BLE001 - RerankError and device failures
            return error(500, str(e), "server_error")
        order = sorted(range(len(texts)), key=lambda i: (-float(logits[i]), i))
        if req.top_n is not None:
            order = order[: max(0, req.top_n)]
        results = []
        for i in order:
            r = {"index": i, "relevance_score": 1.0 / (1.0 + math.exp(-float(logits[i])))}
            if req.return_documents:
                r["document"] = {"text": texts[i]}
            results.append(r)
        return {"model": model, "results": results,
                "usage": {"total_tokens": _count_pair_tokens(svc, req.query, texts)}}

    for path in ("/v1/embeddings", "/embeddings"):
        app.post(path)(embeddings)
    for path in ("/v1/rerank", "/rerank"):
        app.post(path)(rerank)

    @app.get("/health")
    def health():
        return {"status": "ok"}

    return app


def _count_tokens(svc, texts) -> int:
    tok = getattr(svc, "tokenizer", None)
    if tok is None or not hasattr(tok, "content_ids"):
        return 0
    return int(sum(len(tok.content_ids(t)) + 2 for t in texts))


def _count_pair_tokens(svc, query, texts) -> int:
    tok = getattr(svc, "tokenizer", None)
    if tok is None or not hasattr(tok, "content_ids"):
        return 0
    q = len(tok.content_ids(query))
    return int(sum(q + len(tok.content_ids(t)) + 4 for t in texts))


def main(argv=None) -> None:  # pragma: no cover - process entry point
    import argparse

    import uvicorn
    ap = argparse.ArgumentParser(description="OpenAI /embeddings + Jina /rerank server on MI355X")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8090)
    a = ap.parse_args(argv)
    uvicorn.run(create_app(), host=a.host, port=a.port, workers=1)


if __name__ == "__main__":  # pragma: no cover
    main()
