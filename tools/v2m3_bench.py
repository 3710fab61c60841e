"""bge-reranker-v2-m3 rerank stage alone (bench.py's v2m3 field without its fidelity part), for
same-box A/Bs of library builds / settings: one JSON line per run.

    SUPER_RAG_AMD_LIB=... python tools/v2m3_bench.py [--v2m3-steps 3]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    a = bench.parse()
    torch.cuda.set_device(0)
    out = bench.v2m3_field(a, 0, torch.device("cuda", 0), fidelity=False)
    print(json.dumps({k: v for k, v in out.items() if k.endswith(("_qps", "_ms_per_step", "_roofline"))}),
          flush=True)


if __name__ == "__main__":
    main()
