"""Diagnostic: K/V-free CLS last layer vs the K, V GEMM path vs the fp32 oracle on the
bge-reranker-base shape (seeded 'hf' random weights as tests/test_gpu_configs.py config 3)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]
os.environ.setdefault("SUPER_RAG_AMD_SYNTHETIC", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import encoder_ref as R  # noqa: E402
from super_rag_amd.encoder import MODELS, Encoder, random_weights  # noqa: E402


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.set_float32_matmul_precision("highest")
    rs = MODELS["bge-reranker-base"]
    cfg = R.RefConfig(rs.vocab_size, rs.hidden, rs.layers, rs.heads, rs.intermediate, rs.max_position,
                      rs.type_vocab, rs.ln_eps, rs.position_offset, rs.classifier, rs.num_labels)
    for seed in (12, 13):
        wr = random_weights(rs, seed, "hf")
        enc = Encoder(rs, weights=wr, max_tokens=400 * 128)
        rng = np.random.default_rng(seed)
        ids = rng.integers(1000, rs.vocab_size, (400, 128)).astype(np.int32)
        ids[:, 0] = rs.bos_id
        ids[:, 31] = rs.eos_id
        ids[:, 32] = rs.eos_id
        ids[:, -1] = rs.eos_id
        mask = np.ones_like(ids)
        new = enc.cross_score(ids, mask)[:, 0]
        os.environ["SR_KVFREE_CLS"] = "0"
        old = enc.cross_score(ids, mask)[:, 0]
        del os.environ["SR_KVFREE_CLS"]
        wg = {k: torch.as_tensor(v, device="cuda") for k, v in wr.items()}
        ref = R.cross_logits(cfg, wg, ids, mask)[:, 0]
        print(f"seed {seed}: std {ref.std():.3e}  |new-ref| max {np.abs(new - ref).max():.3e} mean "
              f"{np.abs(new - ref).mean():.3e}  |old-ref| max {np.abs(old - ref).max():.3e} mean "
              f"{np.abs(old - ref).mean():.3e}  |new-old| max {np.abs(new - old).max():.3e}", flush=True)
        enc.close()


if __name__ == "__main__":
    main()
