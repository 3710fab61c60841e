"""In-kernel phase stamps of K5c (fused QKV projection + attention, diagnostic library,
sr_diag_qkv_attention_stamps): where a (panel, head) tile's cycles go -- the K-loop, the epilogue
into the LDS images, the attention, the tile transition -- at the cross-encoder's shape.

    python tools/k5c_stamps.py [--pairs 12800] [--reps 5] [--d 768]

Per phase: mean cycles per tile over all waves (s_memtime ticks), per wave group.
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
    ap.add_argument("--pairs", type=int, default=12800)
    ap.add_argument("--d", type=int, default=768)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    S, d = 128, a.d
    H = d // 64
    M = a.pairs * S
    u = torch.randn(M, d, device=dev, generator=g) * 0.7 + 0.05
    X = u.half().contiguous()
    W = (torch.randn(3 * d, d, device=dev, generator=g) * 0.04).half().contiguous()
    bias = torch.randn(3 * d, device=dev, generator=g) * 0.1
    colsum = W.float().sum(1).contiguous()
    mr = torch.stack([u.mean(1), torch.rsqrt(u.var(1, unbiased=False) + 1e-5)], 1).contiguous()
    del u
    mask = torch.ones(a.pairs, S, dtype=torch.int32, device=dev)
    mask[:, 100:] = (torch.rand(a.pairs, S - 100, device=dev, generator=g) < 0.5).int()
    ctx = torch.empty(M, d, dtype=torch.float16, device=dev)
    tiles = ((M + 255) // 256) * H
    grid = 8 * min(32, (tiles + 7) // 8)
    st = torch.zeros(grid * 8 * 8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    acc = None
    for r in range(a.reps + 1):
        st.zero_()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        N.call_diag("sr_diag_qkv_attention_stamps", X.data_ptr(), d, W.data_ptr(), bias.data_ptr(),
                    colsum.data_ptr(), mr.data_ptr(), mask.data_ptr(), ctx.data_ptr(), a.pairs, S, d, H,
                    st.data_ptr(), 0, stream)
        e1.record()
        torch.cuda.synchronize()
        if r == 0:
            continue
        s = st.view(grid, 8, 8).double().cpu()
        acc = s if acc is None else acc + s
        ms = e0.elapsed_time(e1)
    s = acc / a.reps
    flops = 2.0 * M * 3 * d * d + 4.0 * a.pairs * H * S * S * 64
    print(f"K5c stamps: {flops / ms / 1e9:.1f} TF/s (last rep, stamps on), {tiles} tiles, "
          f"{s[:, :, 0].mean():.1f} tiles per wave")
    names = ["K-loop", "epilogue", "attention", "transition"]
    for label, sl in (("all", slice(0, 8)), ("group 0", slice(0, 4)), ("group 1", slice(4, 8))):
        t = s[:, sl, 0].clamp_min(1)
        per = [float((s[:, sl, 1 + i] / t).mean()) for i in range(4)]
        print(f"  {label:8s} " + "  ".join(f"{n} {v:8.0f}" for n, v in zip(names, per))
              + f"  | tile {sum(per):8.0f} cycles")


if __name__ == "__main__":
    main()
