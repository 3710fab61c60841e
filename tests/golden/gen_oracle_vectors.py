"""Regenerate tests/golden/oracle_vectors.npz (small oracle outputs used as regression vectors).

    python tests/golden/gen_oracle_vectors.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

from oracle import encoder_ref as R  # noqa: E402
from oracle.cosine_topk import cosine_topk  # noqa: E402
from super_rag_amd.encoder import ModelSpec, random_weights  # noqa: E402


def main():
    rng = np.random.default_rng(1234)
    corpus = rng.standard_normal((256, 16)).astype(np.float32)
    queries = rng.standard_normal((4, 16)).astype(np.float32)
    k = 10
    dist, rows = cosine_topk(corpus, queries, k)
    spec = ModelSpec("tiny", "bert", 300, 64, 2, 2, 128, 32, 2, 1e-12, 0)
    w = random_weights(spec, 5, "test")
    cfg = R.RefConfig(300, 64, 2, 2, 128, 32, 2, 1e-12, 0, 0, 1)
    ids = rng.integers(5, 300, (3, 12)).astype(np.int32)
    mask = np.ones_like(ids)
    mask[2, 8:] = 0
    emb = R.embed(cfg, w, ids, mask)
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_vectors.npz"),
                        corpus=corpus, queries=queries, k=k, dist=dist, rows=rows, ids=ids, mask=mask,
                        emb=emb, cfg=np.array([300, 64, 2, 2, 128, 32, 2, 1e-12, 0, 0, 1], dtype=np.float64),
                        **{"w." + n: v for n, v in w.items()})


if __name__ == "__main__":
    main()
