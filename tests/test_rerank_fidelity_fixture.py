"""CPU: the ranking-fidelity fixture (tests/golden/rerank_fidelity.npz) is what its generator and
the oracle say it is: same token ids and weight checksum from the seeds, the pair layout of the
oracle's packer (HF XLM-R pair encoding), and the oracle logits of a sample of the pairs.  The set
is discriminative: per query the logit std is ~1 and the logit follows the query-term overlap."""
import os

import numpy as np

FIX = os.path.join(os.path.dirname(__file__), "golden", "rerank_fidelity.npz")


def test_fixture_regenerates_and_matches_the_oracle():
    from model_dirs import ref_config
    from oracle import encoder_ref as R
    from super_rag_amd.encoder import MODELS
    from super_rag_amd.synthetic import FIDELITY, fidelity_setup, weight_checksum
    fx = np.load(FIX)
    spec = MODELS["bge-reranker-base"]
    w, ids, mask, overlap, m = fidelity_setup(spec)
    assert np.array_equal(ids, fx["ids"]) and np.array_equal(mask, fx["mask"])
    assert np.array_equal(overlap, fx["overlap"])
    assert abs(weight_checksum(w) - float(fx["checksum"])) <= 1e-9 * abs(float(fx["checksum"]))
    # the pair layout is the oracle packer's: <s> q </s></s> p </s>
    q = ids[::100, 1:1 + m["q_len"]]
    p = ids[:, 3 + m["q_len"]:-1]
    pid, pm, _ = R.pack_pairs(q, np.full(len(q), m["q_len"]), p, np.full(len(p), m["p_len"]),
                              np.arange(len(p)).reshape(len(q), 100), m["pair_len"], 0,
                              spec.bos_id, spec.eos_id, spec.pad_id)
    assert np.array_equal(pid, ids) and np.array_equal(pm, mask)
    # oracle logits of a sample (12 layers on the CPU)
    sl = np.r_[0:6, 395:400, 794:800]
    lg = R.cross_logits(ref_config(spec), w, ids[sl], mask[sl])[:, 0]
    np.testing.assert_allclose(lg, fx["logits"][sl], atol=2e-5)
    ref = fx["logits"].reshape(-1, 100)
    assert (ref.std(1) > 0.5).all()
    assert all(np.corrcoef(ref[b], overlap[b])[0, 1] > 0.7 for b in range(ref.shape[0]))
    assert FIDELITY["queries"] == ref.shape[0] >= 8


def test_v2m3_fixture_regenerates_and_matches_the_oracle():
    """The full-depth bge-reranker-v2-m3 fixture (24 layers, 1024-d): ids and
    weight checksum from the seeds, oracle logits of a sample of pairs, discriminative spread."""
    from model_dirs import ref_config
    from oracle import encoder_ref as R
    from super_rag_amd.encoder import MODELS
    from super_rag_amd.synthetic import fidelity_setup, weight_checksum
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "rerank_fidelity_v2m3.npz"))
    spec = MODELS["bge-reranker-v2-m3"]
    assert (spec.layers, spec.hidden, spec.heads, spec.intermediate) == (24, 1024, 16, 4096)
    w, ids, mask, overlap, _ = fidelity_setup(spec)
    assert np.array_equal(ids, fx["ids"]) and np.array_equal(mask, fx["mask"])
    assert np.array_equal(overlap, fx["overlap"])
    assert abs(weight_checksum(w) - float(fx["checksum"])) <= 1e-9 * abs(float(fx["checksum"]))
    sl = np.r_[0:2, 399:400, 797:800]
    lg = R.cross_logits(ref_config(spec), w, ids[sl], mask[sl])[:, 0]
    np.testing.assert_allclose(lg, fx["logits"][sl], atol=3e-5)
    ref = fx["logits"].reshape(-1, 100)
    assert (ref.std(1) > 0.5).all()
    assert all(np.corrcoef(ref[b], overlap[b])[0, 1] > 0.7 for b in range(ref.shape[0]))
