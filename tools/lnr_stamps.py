"""In-kernel phase stamps of the persistent residual + statistics GEMM (EPI_LNR16_STATS: the
cross-encoder's O-projection, K = 768, and FFN2, K = 3072; diagnostic library,
sr_diag_gemm_lnr_stats_stamps): where a tile's cycles go -- K-step 0, K-step 1, the rest of the
K-loop, the half-tile residual epilogue, the tile transition -- beside the unstamped product's
TF/s on the same operands (sr_diag_gemm_lnr_stats).

    python tools/lnr_stamps.py [--M 524288] [--reps 5]

Per phase: mean cycles per tile over all waves (s_memtime ticks = shader cycles), per wave group.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import torch  # noqa: E402

from super_rag_amd import _native as N  # noqa: E402


def run_shape(M, Nn, K, reps, dev, ldr0=False):
    g = torch.Generator(device=dev).manual_seed(K)
    X = (torch.randn(M, K, device=dev, generator=g) * 0.5).half()
    W = (torch.randn(Nn, K, device=dev, generator=g) * 0.02).half()
    b = torch.randn(Nn, device=dev, generator=g) * 0.1
    gamma = 1.0 + torch.randn(Nn, device=dev, generator=g) * 0.2
    R = (torch.randn(M, Nn, device=dev, generator=g) * 0.8 + 0.3).half()
    Rf = R.float()
    mr = torch.stack([Rf.mean(1), torch.rsqrt(Rf.var(1, unbiased=False) + 1e-5)], 1).contiguous()
    del Rf
    Y = torch.empty(M, Nn, device=dev, dtype=torch.float16)
    st = torch.empty(M, Nn // 128, 2, device=dev)
    tiles = (Nn // 256) * ((M + 255) // 256)
    grid = 8 * min(32, (tiles + 7) // 8)
    stamps = torch.zeros(grid * 8 * 8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    fl = 2.0 * M * Nn * K

    def product():
        N.call_diag("sr_diag_gemm_lnr_stats", X.data_ptr(), K, W.data_ptr(), b.data_ptr(), R.data_ptr(), Nn,
                    mr.data_ptr(), gamma.data_ptr(), Y.data_ptr(), Nn, M, Nn, K, st.data_ptr(), 0, stream)

    def stamped():
        # (ldr0: every row reads the residual of row 0 -- L1 / L2 hits, wrong results: timing only)
        N.call_diag("sr_diag_gemm_lnr_stats_stamps", X.data_ptr(), K, W.data_ptr(), b.data_ptr(), R.data_ptr(),
                    0 if ldr0 else Nn, mr.data_ptr(), gamma.data_ptr(), Y.data_ptr(), Nn, M, Nn, K, st.data_ptr(),
                    stamps.data_ptr(), 0, stream)

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        product()
    e0.record()
    for _ in range(reps):
        product()
    e1.record()
    torch.cuda.synchronize()
    tf = fl * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12
    acc = None
    stamped()
    for _ in range(reps):
        stamps.zero_()
        stamped()
        torch.cuda.synchronize()
        s = stamps.view(grid, 8, 8).double().cpu()
        acc = s if acc is None else acc + s
    s = acc / reps
    tr = s[:, :, 0].clamp_min(1)
    per = s[:, :, 1:6] / tr[..., None]
    nk = int(s[0, 0, 6].item())
    names = ["K-step 0", "K-step 1", "rest of K-loop", "epilogue", "transition"]
    print(f"M {M} N {Nn} K {K}{' (residual rows all row 0: timing only)' if ldr0 else ''}: product {tf:.1f} TF/s, {nk} K-steps per tile, "
          f"{tr.mean().item():.1f} tiles per wave", flush=True)
    for grp, sl in (("all", slice(0, 8)), ("group 0", slice(0, 4)), ("group 1", slice(4, 8))):
        m = per[:, sl, :].mean(dim=(0, 1))
        tot = m.sum().item()
        print(f"  {grp:8s} " + "  ".join(f"{n} {v:8.0f}" for n, v in zip(names, m.tolist())) +
              f"  | tile {tot:8.0f} cycles, K-loop per K-step {(m[0] + m[1] + m[2]).item() / nk:6.0f}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=524288)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for K in (768, 3072):
        run_shape(a.M, 768, K, a.reps, dev)
    run_shape(a.M, 768, 768, a.reps, dev, ldr0=True)


if __name__ == "__main__":
    main()
