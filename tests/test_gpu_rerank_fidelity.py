"""GPU: ranking fidelity of the cross-encoder kernels on a discriminative reranker at the bench
shape.

The rerank contract is an order by relevance (rerank_service.py:115-135; the local cross-encoder
scores [query, passage] pairs and sorts them descending, graphiti bge_reranker_client.py:28-38).
Seeded random weights spread one query's 100 logits by std ~1e-2, so they cannot show that the
fp16 kernels rank like the fp32 oracle.  The relevance-structured bge-reranker-base
(super_rag_amd/synthetic.py: 12 layers, 768-d, XLM-R + classification head; a structured
construction, not a weight scaling) spreads them by std ~1 over candidate sets that share 0..15
of the query's terms.  On 8 queries x 100 pairs at S_pair = 128 against the fp32 oracle
(tests/golden/rerank_fidelity.npz, tests/golden/gen_rerank_fidelity.py):
  fp16 (the default precision)  every query's logit std >= 100 x its max |logit error|, and the
                                top-10 identical to the oracle's modulo ties within a band of
                                1 % of the logit std;
  fp8 mode 3 (config 5's path)  gated like fp16: std / err >= 50 and the
                                top-10 identical modulo the same ties on every query;
  fp8 modes 1 / 2 (opt-in)      top-10 agreement with the oracle reported (and floored);
  the pipeline path             the same set through SearchPipeline.rerank -- the device pair
                                packer, K5c, the K/V-free last layer, rerank_select_dev -- with the
                                candidates scattered over a passage table.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(__file__), "golden", "rerank_fidelity.npz")
RATIO_MIN = 100.0      # logit std / max |logit - oracle| per query
RATIO_MIN_FP8 = 50.0   # fp8 mode 3 (measured >= 91 in round 3)
TIE_BAND = 0.01        # ties: within 1 % of the query's logit std of the oracle's 10th logit


@pytest.fixture(scope="module")
def fidelity():
    import torch
    from super_rag_amd.encoder import MODELS, Encoder
    from super_rag_amd.synthetic import fidelity_setup, weight_checksum
    fx = np.load(FIX)
    spec = MODELS["bge-reranker-base"]
    w, ids, mask, overlap, _ = fidelity_setup(spec)
    assert np.array_equal(ids, fx["ids"]) and np.array_equal(overlap, fx["overlap"])
    assert abs(weight_checksum(w) - float(fx["checksum"])) <= 1e-9 * abs(float(fx["checksum"]))
    enc = Encoder(spec, weights=w, max_tokens=ids.size)
    dids = torch.from_numpy(ids).cuda()
    dmask = torch.from_numpy(mask).cuda()
    yield enc, dids, dmask, fx["logits"].reshape(-1, 100), w, spec
    enc.close()


def _top10_agree(lg, ref, band):
    """Top-10 of lg == top-10 of ref, except rows within `band` of ref's 10th logit may swap."""
    want = np.argsort(-ref, kind="stable")[:10]
    got = np.argsort(-lg, kind="stable")[:10]
    if set(want) == set(got):
        return True
    kth = ref[want[-1]]
    return all(abs(ref[j] - kth) <= band for j in set(want) ^ set(got))


def test_fp16_reranker_ranks_like_the_oracle(fidelity):
    enc, ids, mask, ref, _, _ = fidelity
    enc.set_fp8(0)
    lg = enc.cross_score_dev(ids, mask)[:, 0].float().cpu().numpy().reshape(-1, 100)
    std = ref.std(1)
    err = np.abs(lg - ref).max(1)
    print("fp16 rerank fidelity: logit std per query", std.round(3).tolist())
    print("  max |logit - oracle| per query", err.round(5).tolist(), " std / err min",
          round(float((std / err).min()), 1))
    assert (std >= RATIO_MIN * err).all(), (std / err)
    for b in range(ref.shape[0]):
        assert _top10_agree(lg[b], ref[b], TIE_BAND * std[b]), b
        assert np.argmax(lg[b]) == np.argmax(ref[b]) or \
            abs(ref[b][np.argmax(lg[b])] - ref[b].max()) <= TIE_BAND * std[b]


def test_oracle_on_the_gpu_reproduces_the_fixture(fidelity):
    """The committed CPU fixture equals the same restatement run in fp32 on this GPU (TF32 off)."""
    import torch
    from model_dirs import ref_config
    from oracle import encoder_ref as R
    _, ids, mask, ref, w, spec = fidelity
    old = torch.backends.cuda.matmul.allow_tf32, torch.get_float32_matmul_precision()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.set_float32_matmul_precision("highest")
    try:
        wg = {k: torch.as_tensor(v, device="cuda") for k, v in w.items()}
        g = R.cross_logits(ref_config(spec), wg, ids[:200].cpu().numpy(), mask[:200].cpu().numpy())
    finally:
        torch.backends.cuda.matmul.allow_tf32 = old[0]
        torch.set_float32_matmul_precision(old[1])
    assert np.abs(g[:, 0].reshape(-1, 100) - ref[:2]).max() <= 1e-4


@pytest.mark.parametrize("mode", [3])
def test_fp8_mode3_ranks_like_the_oracle(fidelity, mode):
    """Config 5's fp8 reranker path (mode 3: FFN1 + FFN2 on the block-scaled fp8 MFMA, QKV +
    attention fp16; mode 5: also the O-projection of the K5c layers on e4m3 ctx) gated as the fp16
    path is: a regression to mode 2's figures (overlap 0.85, max error 0.44) fails here."""
    enc, ids, mask, ref, _, _ = fidelity
    enc.set_fp8(mode)
    try:
        lg = enc.cross_score_dev(ids, mask)[:, 0].float().cpu().numpy().reshape(-1, 100)
    finally:
        enc.set_fp8(0)
    std = ref.std(1)
    err = np.abs(lg - ref).max(1)
    print(f"fp8 mode {mode}: max |logit - oracle| per query", err.round(4).tolist(), " std / err min",
          round(float((std / err).min()), 1))
    assert (std >= RATIO_MIN_FP8 * err).all(), (std / err)
    for b in range(ref.shape[0]):
        assert _top10_agree(lg[b], ref[b], TIE_BAND * std[b]), b


def test_pipeline_rerank_path_ranks_like_the_oracle(fidelity):
    """SearchPipeline.rerank on the fidelity set: the 800 candidate passages sit at shuffled rows of
    a 1,000-row passage token table (200 decoy rows), the candidate lists name those rows in a
    shuffled order, and the device path packs the pairs (build_pairs_dev: bit-exact against the
    fixture's pairs), scores them (K5c + the K/V-free CLS-only last layer) and selects the top-10
    (rerank_select_dev).  The final rows equal the oracle's top-10 modulo ties within 1 % of the
    logit std, and the returned logits match the oracle's to the fp16 bound."""
    import torch
    from super_rag_amd.pipeline import SearchPipeline, build_pairs_dev
    from super_rag_amd.synthetic import FIDELITY, relevance_candidates
    enc, ids, _, ref, _, spec = fidelity
    m = FIDELITY
    nq, nc = m["queries"], m["cand"]
    q, p, _ = relevance_candidates(spec, nq, nc, m["q_len"], m["p_len"], seed=m["cand_seed"])
    rng = np.random.default_rng(7)
    n_rows = nq * nc + 200
    row_of = rng.permutation(n_rows)[: nq * nc]          # table row of candidate i = b * nc + j
    table = rng.integers(1000, spec.vocab_size, (n_rows, m["p_len"])).astype(np.int32)
    table[row_of] = p
    order = np.stack([rng.permutation(nc) for _ in range(nq)])   # list position -> candidate j
    cand = np.stack([row_of[b * nc + order[b]] for b in range(nq)]).astype(np.int64)
    dev = torch.device("cuda", 0)
    p_tok = torch.from_numpy(table).to(dev)
    p_len = torch.full((n_rows,), m["p_len"], dtype=torch.int32, device=dev)
    q_tok = torch.from_numpy(q).to(dev)
    q_len = torch.full((nq,), m["q_len"], dtype=torch.int32, device=dev)
    rows_dev = torch.from_numpy(cand).to(dev)
    pids, _, _ = build_pairs_dev(q_tok, q_len, p_tok, p_len, rows_dev, m["pair_len"], spec)
    want_ids = ids.cpu().numpy().reshape(nq, nc, -1)[np.arange(nq)[:, None], order].reshape(nq * nc, -1)
    np.testing.assert_array_equal(pids.cpu().numpy(), want_ids)
    enc.set_fp8(0)
    pipe = SearchPipeline(None, enc, None, p_tok, p_len, k_candidates=nc, k_final=10,
                          pair_len=m["pair_len"])
    rows, logits = pipe.rerank(q_tok, q_len, rows_dev)
    rows, logits = rows.cpu().numpy(), logits.float().cpu().numpy()
    std = ref.std(1)
    for b in range(nq):
        want = np.argsort(-ref[b], kind="stable")[:10]            # candidate indices j
        kth = ref[b][want[-1]]
        got_j = [int(np.nonzero(row_of[b * nc: (b + 1) * nc] == r)[0][0]) for r in rows[b]]
        for j in set(want.tolist()) ^ set(got_j):
            assert abs(ref[b][j] - kth) <= TIE_BAND * std[b], (b, j)
        assert np.all(np.diff(logits[b]) <= 0), b                 # descending
        assert np.abs(logits[b] - ref[b][got_j]).max() * RATIO_MIN <= std[b], b


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_fp8_modes_top10_agreement(fidelity, mode):
    """The product fp8 precision modes (1: FFN2 on e4m3; 2: also FFN1 and QKV; 3: FFN1 + FFN2, QKV
    fp16) against the fp32
    oracle on the same discriminative set: agreement is reported; the floor only catches a broken
    mode (seeded-random weights could not tell these apart at all: 0.55 overlap vs fp16)."""
    enc, ids, mask, ref, _, _ = fidelity
    enc.set_fp8(mode)
    try:
        lg = enc.cross_score_dev(ids, mask)[:, 0].float().cpu().numpy().reshape(-1, 100)
    finally:
        enc.set_fp8(0)
    top = [len(set(np.argsort(-lg[b])[:10]) & set(np.argsort(-ref[b])[:10])) / 10 for b in range(ref.shape[0])]
    top1 = np.mean([np.argmax(lg[b]) == np.argmax(ref[b]) for b in range(ref.shape[0])])
    err = np.abs(lg - ref).max(1)
    print(f"fp8 mode {mode}: top-10 overlap with the oracle {np.mean(top):.3f} (per query {top}), "
          f"top-1 equal {top1:.2f}, max |logit err| {err.max():.4f}, logit std {ref.std(1).mean():.3f}")
    assert np.mean(top) >= 0.8
