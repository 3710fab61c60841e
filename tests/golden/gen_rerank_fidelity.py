"""Regenerate tests/golden/rerank_fidelity.npz: fp32-oracle logits of the relevance-structured
bge-reranker-base (super_rag_amd/synthetic.py) on 8 queries x 100 candidates at S_pair = 128.

    python tests/golden/gen_rerank_fidelity.py [--model bge-reranker-v2-m3]

--model bge-reranker-v2-m3 writes rerank_fidelity_v2m3.npz: the same construction at the shape of
the reranker the reference actually seeds (BAAI/bge-reranker-v2-m3,
migration/sql/model_configs_init.sql:4148; XLM-R large: 24 layers, 1024-d, 16 heads, FFN 4096).

The rerank contract is order by relevance (rerank_service.py:115-135; the local cross-encoder
scores [query, passage] pairs and sorts descending, graphiti bge_reranker_client.py:28-38).  The
weights and the candidate sets are regenerated from their seeds by the tests and bench.py; the
fixture holds the token ids, a weight checksum (so a drift of the generator is caught) and the
oracle logits (oracle/encoder_ref.py, torch-CPU fp32, the restatement pinned to transformers in
tests/test_oracle.py).
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "super-rag_amd")]

from oracle import encoder_ref as R  # noqa: E402
from super_rag_amd.encoder import MODELS  # noqa: E402
from super_rag_amd.synthetic import (fidelity_setup, weight_checksum)  # noqa: E402


FILES = {"bge-reranker-base": "rerank_fidelity.npz", "bge-reranker-v2-m3": "rerank_fidelity_v2m3.npz"}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bge-reranker-base", choices=sorted(FILES))
    spec = MODELS[ap.parse_args().model]
    w, ids, mask, overlap, meta = fidelity_setup(spec)
    cfg = R.RefConfig(spec.vocab_size, spec.hidden, spec.layers, spec.heads, spec.intermediate,
                      spec.max_position, spec.type_vocab, spec.ln_eps, spec.position_offset,
                      spec.classifier, spec.num_labels)
    t0 = time.time()
    logits = np.concatenate([R.cross_logits(cfg, w, ids[i:i + 100], mask[i:i + 100])[:, 0]
                             for i in range(0, ids.shape[0], 100)]).astype(np.float32)
    print(f"oracle: {ids.shape[0]} pairs in {time.time() - t0:.0f} s; per-query logit std "
          f"{logits.reshape(-1, 100).std(1).round(3).tolist()}")
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), FILES[spec.name]),
                        ids=ids, mask=mask, overlap=overlap, logits=logits,
                        checksum=np.float64(weight_checksum(w)), **{k: np.int64(v) for k, v in meta.items()})


if __name__ == "__main__":
    main()
