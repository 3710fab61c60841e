"""Process-wide cache of resident encoders (model name, device) -> (Encoder, Tokenizer).

The reference builds a new EmbeddingService per query and resolves provider / key / base_url with
three synchronous DB lookups (llm/embed/base_embedding.py:122-215) before an HTTP round trip.
Here a model is loaded into HBM once per process and device and shared by every service object.
"""
from __future__ import annotations

import os
import threading

from .encoder import Encoder, ModelSpec, resolve_spec
from .tokenizer import Tokenizer

_lock = threading.Lock()
_models: dict = {}
_next = [0]


def default_device() -> int:
    """SUPER_RAG_AMD_DEVICES="0,1,..." places model replicas on those GPUs, one device per call in
    turn (the reference builds a service object per request, so requests spread over the GPUs);
    else SUPER_RAG_AMD_DEVICE (default 0)."""
    devs = os.environ.get("SUPER_RAG_AMD_DEVICES", "").strip()
    if devs:
        ids = [int(x) for x in devs.split(",") if x.strip()]
        if ids:
            with _lock:
                i = _next[0] % len(ids)
                _next[0] += 1
            return ids[i]
    return int(os.environ.get("SUPER_RAG_AMD_DEVICE", "0"))


def get_model(model: str | ModelSpec, device: int | None = None, seed: int = 0):
    """Return the shared (Encoder, Tokenizer) for a model name such as "BAAI/bge-m3"."""
    spec = model if isinstance(model, ModelSpec) else resolve_spec(model)
    dev = default_device() if device is None else int(device)
    key = (spec.name, spec.asset_dir, dev)
    with _lock:
        hit = _models.get(key)
        if hit is None:
            hit = (Encoder(spec, device=dev, seed=seed), Tokenizer(spec))
            _models[key] = hit
        return hit


def clear() -> None:
    with _lock:
        for enc, _ in _models.values():
            enc.close()
        _models.clear()
