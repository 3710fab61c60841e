"""GEMM microbenchmark + parity (diagnostic; not part of the product).

    python tools/gemm_bench.py [--variants 1,2] [--M 524288] [--reps 10]

For every variant: parity of each epilogue against a torch fp32 reference on a ragged M, then the
encoder shapes of the reranker / embedder timed with HIP events (interleaved rounds, median).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import torch  # noqa: E402

from super_rag_amd import _native as N  # noqa: E402


RES_LD0 = False  # --res-ld0: every output row reads residual row 0 (L2-resident), a diagnostic


def gemm(variant, epi, X, W, b, R, Y):
    if variant < 0:  # torch / hipBLASLt GEMM without epilogue, as a yardstick
        torch.matmul(X, W.T, out=Y) if Y.dtype == X.dtype else torch.matmul(X, W.T)
        return
    M, K = X.shape
    Nn = W.shape[0]
    N.call_diag("sr_diag_gemm", variant, epi, X.data_ptr(), X.stride(0), W.data_ptr(), b.data_ptr(),
           R.data_ptr() if R is not None else None, 0 if R is None or RES_LD0 else R.stride(0),
           Y.data_ptr(), Y.stride(0), M, Nn, K, 0, torch.cuda.current_stream().cuda_stream)


def reference(epi, X, W, b, R):
    y = X.float() @ W.float().T + b
    if epi == 1:
        y = torch.nn.functional.gelu(y)
    elif epi in (2, 4):
        y = y + R.float()
    elif epi == 3:
        y = torch.tanh(y)
    return y


def out_dtype(epi):
    return torch.float32 if epi in (2, 3) else torch.float16


def parity(variant, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    ok = True
    for (M, Nn, K) in ((1000, 512, 768), (4096, 768, 3072), (300, 256, 128)):
        X = (torch.randn(M, K, device=dev, generator=g) * 0.5).half()
        W = (torch.randn(Nn, K, device=dev, generator=g) * 0.02).half()
        b = torch.randn(Nn, device=dev, generator=g) * 0.1
        for epi in range(5):
            R = None
            if epi == 2:
                R = torch.randn(M, Nn, device=dev, generator=g)
            elif epi == 4:
                R = torch.randn(M, Nn, device=dev, generator=g).half()
            Y = torch.empty(M, Nn, device=dev, dtype=out_dtype(epi))
            gemm(variant, epi, X, W, b, R, Y)
            ref = reference(epi, X, W, b, R)
            err = (Y.float() - ref).abs().max().item()
            tol = 2e-3 * max(1.0, ref.abs().max().item())
            if not err <= tol:
                ok = False
            print(f"  parity v{variant} epi{epi} {M}x{Nn}x{K}: max|err| {err:.2e} (tol {tol:.1e})"
                  f"{'' if err <= tol else '  FAIL'}")
    return ok


def parity_big(variant, dev):
    """Multi-tile persistent shapes (every walker hands over several tiles), epilogues 0/1/4."""
    g = torch.Generator(device=dev).manual_seed(5)
    ok = True
    for (M, Nn, K) in ((70000, 768, 768), (40000, 2304, 768), (20000, 768, 3072)):
        X = (torch.randn(M, K, device=dev, generator=g) * 0.5).half()
        W = (torch.randn(Nn, K, device=dev, generator=g) * 0.02).half()
        b = torch.randn(Nn, device=dev, generator=g) * 0.1
        for epi in (0, 1, 4):
            R = torch.randn(M, Nn, device=dev, generator=g).half() if epi == 4 else None
            Y = torch.full((M, Nn), float("nan"), device=dev, dtype=torch.float16)
            gemm(variant, epi, X, W, b, R, Y)
            ref = reference(epi, X, W, b, R)
            err = (Y.float() - ref).abs().max().item()
            tol = 2e-3 * max(1.0, ref.abs().max().item())
            ok = ok and err <= tol
            print(f"  parity-big v{variant} epi{epi} {M}x{Nn}x{K}: max|err| {err:.2e} (tol {tol:.1e})"
                  f"{'' if err <= tol else '  FAIL'}")
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--M", type=int, default=524288)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--res-ld0", action="store_true", help="residual row stride 0 (timing only)")
    ap.add_argument("--no-parity", action="store_true")
    a = ap.parse_args()
    global RES_LD0
    dev = torch.device("cuda", 0)
    variants = [int(v) for v in a.variants.split(",")]
    all_ok = a.no_parity or all(parity(v, dev) for v in variants if v >= 0 and v not in (6, 7, 9, 10, 11))
    all_ok = all_ok and (a.no_parity or all(parity_big(v, dev) for v in variants if v in (4, 5)))
    RES_LD0 = a.res_ld0
    M = a.M
    shapes = [("qkv", 2304, 768, 0), ("ffn1_gelu", 3072, 768, 1), ("ffn2_res16", 768, 3072, 4),
              ("oproj_res16", 768, 768, 4), ("ffn2_res32", 768, 3072, 2)]
    bufs = {}
    g = torch.Generator(device=dev).manual_seed(1)
    for name, Nn, K, epi in shapes:
        X = (torch.randn(M, K, device=dev, generator=g) * 0.5).half()
        W = (torch.randn(Nn, K, device=dev, generator=g) * 0.02).half()
        b = torch.randn(Nn, device=dev, generator=g) * 0.1
        R = (torch.randn(M, Nn, device=dev, generator=g).half() if epi == 4 else
             torch.randn(M, Nn, device=dev, generator=g) if epi == 2 else None)
        Y = torch.empty(M, Nn, device=dev, dtype=out_dtype(epi))
        bufs[name] = (epi, X, W, b, R, Y, 2.0 * M * Nn * K)
    res = {(v, n): [] for v in variants for n in bufs}
    for _ in range(a.rounds):
        for v in variants:
            for name, (epi, X, W, b, R, Y, fl) in bufs.items():
                gemm(v, epi, X, W, b, R, Y)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    gemm(v, epi, X, W, b, R, Y)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / a.reps
                res[(v, name)].append(fl / ms / 1e9)
    for (v, name), tf in sorted(res.items()):
        tf.sort()
        print(f"v{v} {name:12s} M={M}: median {tf[len(tf) // 2]:7.1f} TF/s  (min {tf[0]:.1f}, max {tf[-1]:.1f})")
    print("PARITY", "OK" if all_ok else "FAIL")


if __name__ == "__main__":
    main()
