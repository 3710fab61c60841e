"""Host cost of one synchronous embed call (the drop-in's EmbeddingService path:
Encoder.embed = sr_encoder_forward, host ids in, host embeddings out, synchronised) against the
device time of the same forward (HIP events around back-to-back embed_dev calls), per batch size.

    python tools/embed_host_cost.py [--batches 1 8 20 32] [--reps 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from super_rag_amd import _native as N  # noqa: E402
from super_rag_amd.encoder import MODELS, Encoder, random_weights  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 8, 20, 32])
    ap.add_argument("--q-len", type=int, default=32)
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    es = MODELS["bge-base-en"]
    enc = Encoder(es, device=0, weights=random_weights(es, seed=11, style="hf"))
    dev = torch.device("cuda", 0)
    out = {}
    for B in a.batches:
        rng = np.random.default_rng(B)
        ids = rng.integers(1000, es.vocab_size, (B, a.q_len)).astype(np.int32)
        ids[:, 0] = 101
        mask = np.ones_like(ids)
        for _ in range(5):
            enc.embed(ids, mask)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            enc.embed(ids, mask)
        host_ms = (time.perf_counter() - t0) / a.reps * 1e3
        di, dm = torch.from_numpy(ids).to(dev), torch.from_numpy(mask).to(dev)
        for _ in range(5):
            enc.embed_dev(di, dm)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            enc.embed_dev(di, dm)
        e1.record()
        torch.cuda.synchronize()
        dev_ms = e0.elapsed_time(e1) / a.reps
        # host time to enqueue one forward (no synchronisation): launches only
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        enc.embed_dev(di, dm)
        enq_ms = (time.perf_counter() - t0) * 1e3
        torch.cuda.synchronize()
        N.profile_enable(True)
        enc.embed_dev(di, dm)
        torch.cuda.synchronize()
        N.profile_enable(False)
        launches = sum(v["launches"] for v in N.profile_read().values())
        out[B] = {"sync_call_ms": round(host_ms, 3), "device_ms": round(dev_ms, 3),
                  "enqueue_ms": round(enq_ms, 3), "launches": launches}
        print(B, out[B], flush=True)
    print(json.dumps(out))
    enc.close()


if __name__ == "__main__":
    main()
