"""K1 chunk-rate probe (diagnostic): is the slow middle threshold chunk of a 10M-row B = 256 search
a clock (DVFS) transient?  Runs the search 6 times plain, then 6 times each right behind a ~5 ms
fp16 matmul that keeps the matrix pipes busy up to the search's first kernel; run it under
`rocprofv3 --kernel-trace` and read the per-dispatch durations (tools/k1_schedule.py).

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/k1_dvfs_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from super_rag_amd.store import NativeStore  # noqa: E402


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--predummy-gb", type=float, default=0.0,
                    help="allocate (and keep) this many GB before the store (other physical memory)")
    ap.add_argument("--capacity", type=int, default=10_000_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    rows, dim, B, k = 10_000_000, 768, 256, 100
    g = torch.Generator(device="cpu").manual_seed(0)
    centers = torch.randn((1024, dim), generator=g).to(dev)
    dummy = torch.empty(int(a.predummy_gb * 1e9), dtype=torch.uint8, device=dev) if a.predummy_gb else None
    st = NativeStore(dim, capacity=max(rows, a.capacity))
    for c0 in range(0, rows, 1 << 20):
        st.add_dev(bench.gen_corpus_chunk(c0, min(rows, c0 + (1 << 20)), dim, centers, dev))
    gq = torch.Generator(device=dev).manual_seed(3)
    q = torch.randn((B, dim), generator=gq, device=dev)
    a = torch.randn((8192, 8192), device=dev, dtype=torch.float16)
    torch.cuda.synchronize()
    for _ in range(6):
        st.search_dev(q, k)
    torch.cuda.synchronize()
    for _ in range(6):
        for _ in range(3):
            a @ a
        st.search_dev(q, k)
    torch.cuda.synchronize()
    print("done", dummy is not None, flush=True)


if __name__ == "__main__":
    main()
