"""FFN1 (LayerNorm-folded GEMM + 2 GELU epilogue) microbenchmark and parity (diagnostic).

    python tools/ffn1_bench.py [--M 524288] [--reps 10] [--rounds 3] [--f8]

Times the product kernel (diag 0) against the main loop alone (2), the epilogue math without its
stores (5) and the stores without the math (6) at the reranker's FFN1 shape (N 3072, K 768), after
a parity check of diag 0 against a torch fp32 reference on sampled rows.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import torch  # noqa: E402

from super_rag_amd import _native as N  # noqa: E402


def e4m3(t):
    return t.float().clamp(-448, 448).to(torch.float8_e4m3fn)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=524288)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--f8", action="store_true")
    ap.add_argument("--diags", default="0,2,5,6")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, Nn, K = a.M, a.N, a.K
    u = torch.randn(M, K, device=dev, generator=g) * 0.7 + 0.05   # un-normalised residual rows
    W = (torch.randn(Nn, K, device=dev, generator=g) * 0.04)      # LN-folded weight W diag(gamma)
    bias = torch.randn(Nn, device=dev, generator=g) * 0.1
    mu = u.mean(1)
    rstd = torch.rsqrt(u.var(1, unbiased=False) + 1e-5)
    mr = torch.stack([mu, rstd], 1).contiguous()
    stream = torch.cuda.current_stream().cuda_stream
    if a.f8:
        X = e4m3(u).view(torch.uint8).contiguous()
        amax = W.abs().amax(1).clamp_min(1e-30)
        e = torch.floor(torch.log2(448.0 / amax)).to(torch.int32)
        W8 = e4m3(W * torch.exp2(e.float())[:, None]).view(torch.uint8).contiguous()
        wexp = (127 - e).to(torch.uint8).contiguous()
        Wd = W8.view(torch.float8_e4m3fn).float() * torch.exp2(-e.float())[:, None]
        Xd = X.view(torch.float8_e4m3fn).float()
        Wop, wexp_p, lda, ldy = W8, wexp.data_ptr(), K, Nn
        Y = torch.empty(M, Nn, device=dev, dtype=torch.uint8)
    else:
        X = u.half()
        Wd = W.half().float()
        Xd = X.float()
        Wop, wexp_p, lda, ldy = W.half().contiguous(), None, K, Nn
        Y = torch.empty(M, Nn, device=dev, dtype=torch.float16)
    colsum = Wd.sum(1).contiguous()

    def run(diag):
        N.call_diag("sr_diag_ffn1", diag, 1 if a.f8 else 0, X.data_ptr(), lda, Wop.data_ptr(), wexp_p,
               bias.data_ptr(), colsum.data_ptr(), mr.data_ptr(), Y.data_ptr(), ldy, M, Nn, K, 0, stream)

    run(0)
    torch.cuda.synchronize()
    rows = torch.randint(0, M, (512,), device=dev, generator=g)
    pre = mr[rows, 1:2] * (Xd[rows] @ Wd.T - mr[rows, 0:1] * colsum[None]) + bias[None]
    ref = 2.0 * torch.nn.functional.gelu(pre)
    got = Y[rows].view(torch.float8_e4m3fn).float() if a.f8 else Y[rows].float()
    err = (got - ref).abs()
    rel = (err / ref.abs().clamp_min(1.0)).max().item()
    tol = 0.07 if a.f8 else 2e-3
    print(f"parity diag0 {'f8' if a.f8 else 'f16'} M={M}: max|err| {err.max().item():.3e}, max rel {rel:.3e} "
          f"(tol {tol}) {'OK' if rel <= tol else 'FAIL'}", flush=True)
    fl = 2.0 * M * Nn * K
    diags = [int(d) for d in a.diags.split(",")]
    res = {d: [] for d in diags}
    for _ in range(a.rounds):
        for d in diags:
            run(d)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run(d)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            res[d].append((fl / ms / 1e9, ms))
    names = {0: "product", 2: "main loop only", 5: "math, no stores", 6: "stores, no math",
             7: "stores to tile 0", 8: "one storer (OST)"}
    for d in diags:
        v = sorted(res[d])
        tf, ms = v[len(v) // 2]
        print(f"diag {d} {names[d]:16s} {'f8' if a.f8 else 'f16'}: {tf:7.1f} TF/s  {ms:.3f} ms "
              f"(min {v[0][0]:.1f}, max {v[-1][0]:.1f})", flush=True)
    if rel > tol:
        sys.exit(1)


if __name__ == "__main__":
    main()
