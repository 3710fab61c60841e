"""One GEMM shape / variant / epilogue launched repeatedly (for rocprofv3 PMC passes; diagnostic).

    python tools/gemm_shape.py --variant 5 --epi 1 --N 3072 --K 768 [--M 524288] [--reps 20]
Variants as sr_diag_gemm: 5 persistent pipelined (shipped), 9 = no epilogue, 10 = epilogue math
only, 11 = stores only (timing diagnostics, wrong results).  Prints the mean TF/s (HIP events).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import torch  # noqa: E402

from super_rag_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", type=int, default=5)
    ap.add_argument("--epi", type=int, default=1)
    ap.add_argument("--M", type=int, default=524288)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    X = (torch.randn(a.M, a.K, device=dev, generator=g) * 0.5).half()
    W = (torch.randn(a.N, a.K, device=dev, generator=g) * 0.02).half()
    b = torch.randn(a.N, device=dev, generator=g) * 0.1
    R = None
    if a.epi == 2:
        R = torch.randn(a.M, a.N, device=dev, generator=g)
    elif a.epi == 4:
        R = torch.randn(a.M, a.N, device=dev, generator=g).half()
    Y = torch.empty(a.M, a.N, device=dev, dtype=torch.float32 if a.epi in (2, 3) else torch.float16)
    st = torch.cuda.current_stream().cuda_stream

    def run():
        N.call_diag("sr_diag_gemm", a.variant, a.epi, X.data_ptr(), X.stride(0), W.data_ptr(), b.data_ptr(),
               R.data_ptr() if R is not None else None, R.stride(0) if R is not None else 0,
               Y.data_ptr(), Y.stride(0), a.M, a.N, a.K, 0, st)
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(f"v{a.variant} epi{a.epi} {a.M}x{a.N}x{a.K}: {ms:.3f} ms  {2.0 * a.M * a.N * a.K / ms / 1e9:.1f} TF/s",
          flush=True)


if __name__ == "__main__":
    main()
