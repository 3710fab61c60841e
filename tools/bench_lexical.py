"""Lexical (BM25) and hybrid retrieval benchmark on one MI355X (BASELINE config 5:
"hybrid dense+BM25-lexical score fusion"); diagnostic, not the headline bench.py line.

    python tools/bench_lexical.py [--docs 6250000] [--batch 256] [--k 100] [--steps 5]

Synthetic corpus (seeded): document lengths uniform in [mean/2, 3 mean/2] tokens, token ids Zipf(1.2)
over a 1M-term vocabulary (folded), distinct (term, tf) per document; queries: 4-8 ids from the same
Zipf law with the 100 most frequent ids (stop-word-like) excluded.  Dense side of the hybrid: a
docs x 1024 fp16 corpus (config-5 shard width).  Prints one JSON line: BM25 q/s, hybrid q/s, the
lex_score kernel's rate against HBM (algorithmic bytes = 12 per scored posting: the 8-byte posting
+ the 4-byte document length) and the oracle's CPU q/s on a sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from super_rag_amd import _native as N  # noqa: E402
from super_rag_amd.lexical import NativeLexIndex, hybrid_search  # noqa: E402
from super_rag_amd.store import NativeStore  # noqa: E402

BYTES_PER_POSTING = 12
HBM_PEAK_GBS = 8000.0


def gen_docs(n, vocab, mean_len, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(mean_len // 2, mean_len * 3 // 2 + 1, n).astype(np.int64)
    out_off = np.zeros(n + 1, np.int64)
    terms_l, tf_l = [], []
    blk = 1 << 20
    for d0 in range(0, n, blk):                    # bounded host memory per block
        L = lens[d0:d0 + blk]
        t = (rng.zipf(1.2, int(L.sum())) - 1) % vocab
        doc = np.repeat(np.arange(len(L), dtype=np.int64), L)
        key, cnt = np.unique(doc * vocab + t, return_counts=True)
        d = key // vocab
        terms_l.append((key % vocab).astype(np.int32))
        tf_l.append(cnt.astype(np.int32))
        per = np.bincount(d, minlength=len(L))
        out_off[d0 + 1:d0 + len(L) + 1] = out_off[d0] + np.cumsum(per)
    return out_off, np.concatenate(terms_l), np.concatenate(tf_l), lens.astype(np.int32)


def gen_queries(B, vocab, seed):
    rng = np.random.default_rng(seed)
    return [(((rng.zipf(1.2, rng.integers(4, 9)) - 1) % (vocab - 100)) + 100).tolist()
            for _ in range(B)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=2_000_000)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--mean-len", type=int, default=48)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-queries", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.time()
    off, terms, tf, dl = gen_docs(a.docs, a.vocab, a.mean_len, 0)
    print(f"# corpus: {a.docs} docs, {len(terms)} postings ({time.time() - t0:.1f} s)", flush=True)
    lex = NativeLexIndex()
    lex.add_arrays(off, terms, tf, dl)
    qs = gen_queries(a.batch, a.vocab, 2)
    df = np.bincount(terms, minlength=a.vocab)
    scored = int(sum(df[np.unique(q)].sum() for q in qs))

    torch.cuda.synchronize()
    t = time.perf_counter()
    lex.search(qs[:1], a.k)                         # first search: device CSR build (radix sort)
    build_s = time.perf_counter() - t
    print(f"# index build {build_s * 1e3:.1f} ms", flush=True)
    lex.search(qs, a.k)                             # warm-up
    N.profile_enable(True)
    N.profile_read()
    t = time.perf_counter()
    for _ in range(a.steps):
        lex.search(qs, a.k)
    bm25_s = (time.perf_counter() - t) / a.steps
    prof = N.profile_read()
    N.profile_enable(False)
    ls = prof.get("lex_score", {"launches": 0, "total_ms": 0.0})
    sel = prof.get("lex_select", {"launches": 0, "total_ms": 0.0})
    score_ms = ls["total_ms"] / a.steps
    algo = scored * BYTES_PER_POSTING
    gbs = algo / (score_ms * 1e-3) / 1e9 if score_ms else None
    print(f"# bm25: {bm25_s * 1e3:.2f} ms/batch, lex_score {score_ms:.3f} ms, "
          f"lex_select {sel['total_ms'] / a.steps:.3f} ms", flush=True)

    # hybrid: dense corpus of the same rows (random fp16 rows, 1024-d), rrf fusion on the device
    store = NativeStore(a.dim, capacity=a.docs)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    for r in range(0, a.docs, 1 << 20):
        store.add_dev(torch.randn((min(a.docs, r + (1 << 20)) - r, a.dim), generator=g,
                                  device=dev, dtype=torch.float32))
    torch.cuda.synchronize()
    qv = torch.randn((a.batch, a.dim), generator=g, device=dev).cpu().numpy()
    hybrid_search(store, lex, qv, qs, 10, a.k)      # warm-up
    N.profile_enable(True)
    N.profile_read()
    t = time.perf_counter()
    for _ in range(a.steps):
        hybrid_search(store, lex, qv, qs, 10, a.k)
    hyb_s = (time.perf_counter() - t) / a.steps
    hprof = N.profile_read()
    N.profile_enable(False)
    rrf_ms = hprof.get("rrf_fuse", {"total_ms": 0.0})["total_ms"] / a.steps

    # CPU baseline: the oracle (numpy, 1 thread) on a sample of the same queries
    from oracle.bm25 import LexCorpus, bm25_topk
    t = time.perf_counter()
    C = LexCorpus(off, terms, tf, dl)
    cpu_build = time.perf_counter() - t
    t = time.perf_counter()
    bm25_topk(C, qs[:a.cpu_queries], a.k)
    cpu_qs = a.cpu_queries / (time.perf_counter() - t)
    rec = {"metric": "BM25 top-k queries/sec and hybrid (dense top-k + BM25 top-k, rrf) queries/sec",
           "docs": a.docs, "postings": int(len(terms)), "vocab": a.vocab, "batch": a.batch,
           "k": a.k, "steps": a.steps,
           "bm25_qps": round(a.batch / bm25_s, 1), "bm25_ms_per_batch": round(bm25_s * 1e3, 3),
           "hybrid_qps": round(a.batch / hyb_s, 1), "hybrid_ms_per_batch": round(hyb_s * 1e3, 3),
           "index_build_ms": round(build_s * 1e3, 1),
           "rrf_fuse_ms": round(rrf_ms, 4),
           "lex_select_ms": round(sel["total_ms"] / a.steps, 4),
           "roofline": {"kernel": "lex_score", "bound": "hbm", "achieved": round(gbs, 1) if gbs else None,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(gbs / HBM_PEAK_GBS, 4) if gbs else None,
                        "algorithmic_B_per_batch": algo,
                        "postings_scored_per_batch": scored, "kernel_ms": round(score_ms, 4)},
           "cpu_baseline": {"value": round(cpu_qs, 3), "unit": "queries/s", "cores": 1,
                            "kind": "port", "sample": f"oracle/bm25.py bm25_topk, {a.cpu_queries} "
                            f"of the batch's queries, same corpus (index build {cpu_build:.1f} s "
                            "not counted)"}}
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
