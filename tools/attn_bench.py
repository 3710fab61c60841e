"""Attention microbenchmark (diagnostic): both K5 kernels at the reranker shape, HIP-event timed.

    python tools/attn_bench.py [--B 4096] [--S 128] [--Sq 128]
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
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--S", type=int, default=128)
    ap.add_argument("--Sq", type=int, default=128)
    ap.add_argument("--heads", type=int, default=12)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    d = 64 * a.heads
    qkv = torch.randn(a.B * a.S, 3 * d, device=dev).half()
    mask = torch.ones(a.B, a.S, device=dev, dtype=torch.int32)
    ctx = torch.empty(a.B * a.Sq, d, device=dev, dtype=torch.float16)
    st = torch.cuda.current_stream().cuda_stream
    byt = 2.0 * a.B * a.S * 3 * d + 2.0 * a.B * a.Sq * d
    fl = 4.0 * a.B * a.heads * a.Sq * a.S * 64
    res = {0: [], 1: [], 2: [], 3: [], -1: []}
    for _ in range(3):
        for v in (0, 1, 2, 3, -1):
            try:
                N.call_diag("sr_diag_attention", v, qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), a.B,
                       a.S, a.Sq, d, a.heads, 0, st)
            except N.NativeError:  # an older library without this variant
                continue
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                N.call_diag("sr_diag_attention", v, qkv.data_ptr(), mask.data_ptr(), ctx.data_ptr(), a.B,
                       a.S, a.Sq, d, a.heads, 0, st)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.reps)
    for v, ms in res.items():
        if not ms:
            continue
        ms.sort()
        m = ms[len(ms) // 2]
        print(f"attention v{v} B={a.B} S={a.S} Sq={a.Sq}: {m:.3f} ms  {byt / m / 1e6:.0f} GB/s  "
              f"{fl / m / 1e9:.0f} TF/s")


if __name__ == "__main__":
    main()
