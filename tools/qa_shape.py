"""Drive the reranker encoder at S = 128 (PMC / timing harness for K5c, diagnostic):
    python tools/qa_shape.py [--pairs 4096] [--reps 3]   (K5c is the default; SR_FUSED_QKV_ATTN=0: unfused)"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]
os.environ.setdefault("SUPER_RAG_AMD_SYNTHETIC", "1")

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    rs = MODELS["bge-reranker-base"]
    enc = Encoder(rs, weights=random_weights(rs, 1, "hf"), max_tokens=a.pairs * 128)
    rng = np.random.default_rng(0)
    ids = rng.integers(1000, rs.vocab_size, (a.pairs, 128)).astype(np.int32)
    ids[:, 0] = rs.bos_id
    mask = np.ones_like(ids)
    enc.cross_score(ids, mask)
    t0 = time.perf_counter()
    for _ in range(a.reps):
        enc.cross_score(ids, mask)
    print(f"{a.pairs} pairs: {(time.perf_counter() - t0) / a.reps * 1e3:.2f} ms per forward")


if __name__ == "__main__":
    main()
