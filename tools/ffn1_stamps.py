"""In-kernel phase stamps of the persistent fp16 FFN1 GEMM (diagnostic library, sr_diag_ffn1_stamps):
where a tile's cycles go -- K-step 0, K-step 1, the rest of the K-loop, the epilogue, the tile
transition -- with the product epilogue (diag 9), with its math but no global stores (diag 10), and
with the product epilogue but no staging of the next tile in its shadow (diag 11, timing only).

    python tools/ffn1_stamps.py [--M 524288] [--reps 5]

Per phase: mean cycles per tile over all waves (s_memtime ticks = shader cycles), per wave group.
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
    ap.add_argument("--M", type=int, default=524288)
    ap.add_argument("--N", type=int, default=3072)
    ap.add_argument("--K", type=int, default=768)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, Nn, K = a.M, a.N, a.K
    u = torch.randn(M, K, device=dev, generator=g) * 0.7 + 0.05
    W = (torch.randn(Nn, K, device=dev, generator=g) * 0.04).half().contiguous()
    bias = torch.randn(Nn, device=dev, generator=g) * 0.1
    mr = torch.stack([u.mean(1), torch.rsqrt(u.var(1, unbiased=False) + 1e-5)], 1).contiguous()
    X = u.half().contiguous()
    colsum = W.float().sum(1).contiguous()
    Y = torch.empty(M, Nn, device=dev, dtype=torch.float16)
    tiles = (Nn // 256) * ((M + 255) // 256)
    grid = 8 * min(32, (tiles + 7) // 8)
    st = torch.zeros(grid * 8 * 8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    names = ["K-step 0", "K-step 1", "rest of K-loop", "epilogue", "transition"]
    for diag, what in ((9, "product epilogue"), (10, "math, no global stores"),
                       (11, "product epilogue, next tile not staged (wrong results)")):
        acc = None
        for r in range(a.reps + 1):
            st.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            N.call_diag("sr_diag_ffn1_stamps", diag, X.data_ptr(), K, W.data_ptr(), bias.data_ptr(),
                        colsum.data_ptr(), mr.data_ptr(), Y.data_ptr(), Nn, M, Nn, K, st.data_ptr(), 0,
                        stream)
            e1.record()
            torch.cuda.synchronize()
            if r == 0:
                continue  # warmup
            s = st.view(grid, 8, 8).double().cpu()
            acc = s if acc is None else acc + s
            ms = e0.elapsed_time(e1)
        s = acc / a.reps
        tr = s[:, :, 0].clamp_min(1)
        per = s[:, :, 1:6] / tr[..., None]          # cycles per tile transition, per wave
        nk = int(s[0, 0, 6].item())
        tf = 2.0 * M * Nn * K / (ms * 1e-3) / 1e12
        print(f"diag {diag} ({what}): {tf:.1f} TF/s (last rep, stamps on), {nk} K-steps per tile, "
              f"{tr.mean().item():.1f} tiles per wave")
        for grp, sl in (("all", slice(0, 8)), ("group 0", slice(0, 4)), ("group 1", slice(4, 8))):
            m = per[:, sl, :].mean(dim=(0, 1))
            tot = m.sum().item()
            print(f"  {grp:8s} " + "  ".join(f"{n} {v:8.0f}" for n, v in zip(names, m.tolist())) +
                  f"  | tile {tot:8.0f} cycles, K-loop per K-step {(m[0] + m[1] + m[2]).item() / nk:6.0f}")


if __name__ == "__main__":
    main()
