"""K1 scan precision benchmark on one MI355X (diagnostic; BASELINE config 5 "fp8 MFMA GEMM path").

    python tools/bench_search_fp8.py [--rows 10000000] [--dim 768] [--batch 256] [--k 100]

Clustered synthetic corpus (bench.py's generator), search-only queries = corpus rows + 0.3 noise.
Times search_dev with the fp16 scan and with the fp8 scan (e4m3 rows, block-scaled MFMA, exact fp16
re-scoring of the top max(2k, k + 32)), reports per-batch time, the scan kernels' HBM rate
(algorithmic bytes: the rows scanned once per query block; fp16 2 B, fp8 1 B per element) and the
fp8 result's recall against the fp16 result.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from super_rag_amd import _native as N  # noqa: E402
from super_rag_amd.store import NativeStore  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    gc = torch.Generator(device="cpu")
    gc.manual_seed(0)
    centers = torch.randn((1024, a.dim), generator=gc).to(dev)
    st = NativeStore(a.dim, capacity=a.rows)
    for c0 in range(0, a.rows, 1 << 20):
        st.add_dev(bench.gen_corpus_chunk(c0, min(a.rows, c0 + (1 << 20)), a.dim, centers, dev))
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    idx = torch.randint(0, a.rows, (a.batch,), generator=g, device=dev)
    q = torch.cat([bench.gen_corpus_chunk(int(i), int(i) + 1, a.dim, centers, dev) for i in idx.tolist()])
    q = q + 0.3 * torch.randn(q.shape, generator=g, device=dev)
    torch.cuda.synchronize()
    out = {"metric": "K1 search ms per batch, fp16 vs fp8 scan", "rows": a.rows, "dim": a.dim,
           "batch": a.batch, "k": a.k}
    res = {}
    for mode in ("fp16", "fp8"):
        t = time.perf_counter()
        st.set_scan_dtype(mode)
        torch.cuda.synchronize()
        if mode == "fp8":
            out["fp8_quantize_ms"] = round((time.perf_counter() - t) * 1e3, 1)
        st.search_dev(q, a.k)
        torch.cuda.synchronize()
        N.profile_enable(True)
        N.profile_read()
        t = time.perf_counter()
        for _ in range(a.steps):
            s, r = st.search_dev(q, a.k)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / a.steps * 1e3
        prof = N.profile_read()
        N.profile_enable(False)
        kern = "cosine_scan8" if mode == "fp8" else "cosine_scan"
        kms = prof.get(kern, {"total_ms": 0.0})["total_ms"] / a.steps
        ebytes = 1 if mode == "fp8" else 2
        ld = -(-a.dim // 128) * 128 if mode == "fp8" else -(-a.dim // 64) * 64
        algo = a.rows * ld * ebytes * -(-a.batch // 256)
        out[mode] = {"ms_per_batch": round(ms, 3), "qps": round(a.batch / ms * 1e3, 1),
                     "scan_kernel_ms": round(kms, 3),
                     "scan_GBps": round(algo / (kms * 1e-3) / 1e9, 1) if kms else None,
                     "scan_frac_of_8TBps": round(algo / (kms * 1e-3) / 8e12, 4) if kms else None,
                     "kernels_ms": {k2: round(v["total_ms"] / a.steps, 3) for k2, v in prof.items()}}
        res[mode] = (s.cpu(), r.cpu())
    r16, r8 = res["fp16"][1], res["fp8"][1]
    for kk in sorted({10, a.k}):
        hit = sum(len(set(r16[b, :kk].tolist()) & set(r8[b, :kk].tolist())) for b in range(a.batch))
        out[f"fp8_recall@{kk}_vs_fp16"] = round(hit / (a.batch * kk), 5)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
