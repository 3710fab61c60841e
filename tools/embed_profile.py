"""Per-kernel profile of the embed stage alone: the bench's embedder
(bge-base-en, seeded weights, S = 32) on B = 256 resident queries, the library's HIP-event
profile over `reps` forwards, printed as ms per forward by kernel name; plus the same embeddings'
max |e - e_ref| against a variant run when --compare-tile is given (diagnostic).

    python tools/embed_profile.py [--batch 256] [--q-len 32] [--reps 50] [--model bge-base-en]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import torch  # noqa: E402

from super_rag_amd import _native as N  # noqa: E402
from super_rag_amd.encoder import MODELS, Encoder, random_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--q-len", type=int, default=32)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--model", default="bge-base-en")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    es = MODELS[a.model]
    enc = Encoder(es, device=0, weights=random_weights(es, seed=11, style="hf"), max_tokens=a.batch * a.q_len)
    g = torch.Generator(device=dev).manual_seed(3)
    ids = torch.randint(1000, es.vocab_size, (a.batch, a.q_len), generator=g, device=dev, dtype=torch.int32)
    ids[:, 0] = 101
    mask = torch.ones_like(ids)
    for _ in range(5):
        enc.embed_dev(ids, mask)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        enc.embed_dev(ids, mask)
    e1.record()
    torch.cuda.synchronize()
    wall = e0.elapsed_time(e1) / a.reps
    N.profile_enable(True)
    for _ in range(a.reps):
        enc.embed_dev(ids, mask)
    torch.cuda.synchronize()
    N.profile_enable(False)
    prof = N.profile_read()
    rows = sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"])
    out = {"model": a.model, "batch": a.batch, "q_len": a.q_len, "ms_per_embed_wall": round(wall, 3),
           "kernels": {k: {"ms_per_embed": round(v["total_ms"] / a.reps, 4),
                           "launches_per_embed": round(v["launches"] / a.reps, 2),
                           "tflops": round(v["flops"] / 1e12 / (v["total_ms"] * 1e-3), 1) if v["flops"] else None,
                           "gbs": round(v["bytes"] / 1e9 / (v["total_ms"] * 1e-3), 1) if v["bytes"] else None}
                       for k, v in rows}}
    print(json.dumps(out, indent=1))
    enc.close()


if __name__ == "__main__":
    main()
