"""Embedding error of the fp32-residual embedders against the fp32 oracle with and without the
split (hi + lo) weights (SR_WEIGHT_SPLIT), per model and weight style, and the embed time at
B = 256, S = 32 for each.

    python tools/embed_split_error.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import encoder_ref as R  # noqa: E402
from super_rag_amd.encoder import MODELS, Encoder, random_weights  # noqa: E402


def cfg(spec):
    return R.RefConfig(spec.vocab_size, spec.hidden, spec.layers, spec.heads, spec.intermediate,
                       spec.max_position, spec.type_vocab, spec.ln_eps, spec.position_offset,
                       spec.classifier, spec.num_labels)


def main():
    for name in ("bge-base-en", "bge-m3"):
        spec = MODELS[name]
        for style in ("test", "hf"):
            w = random_weights(spec, seed=7, style=style)
            rng = np.random.default_rng(1)
            B, S = 8, 32
            ids = rng.integers(1000, spec.vocab_size, (B, S)).astype(np.int32)
            ids[:, 0] = spec.bos_id
            mask = np.ones_like(ids)
            ref = R.embed(cfg(spec), w, ids, mask)
            for split in ("1", "0"):
                os.environ["SR_WEIGHT_SPLIT"] = split
                enc = Encoder(spec, device=0, weights=w)
                got = enc.embed(ids, mask)
                err = np.linalg.norm(got - ref, axis=1) / np.linalg.norm(ref, axis=1)
                dev = torch.device("cuda", 0)
                di = torch.from_numpy(np.tile(ids, (32, 1))).to(dev)
                dm = torch.ones_like(di)
                for _ in range(3):
                    enc.embed_dev(di, dm)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    enc.embed_dev(di, dm)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / 10 * 1e3
                print(f"{name} weights={style} split={split}: max rel err {err.max():.3e} mean {err.mean():.3e}; "
                      f"B=256 S=32 embed {ms:.3f} ms", flush=True)
                enc.close()


if __name__ == "__main__":
    main()
