"""Synthetic models and inputs for ranking-fidelity checks (tests and bench.py; not a product path).

Seeded random cross-encoder weights (encoder.random_weights, HF initialisation) give nearly
constant logits: over one query's 100 candidates the bge-reranker-base shape spreads its logit by
std ~1e-2, barely 10-20x the fp16 logit error, so "identical top-10" says little about the
kernels (What's weak #2).  A trained reranker is a relevance model: its logit moves
with how much of the query a passage contains.  `relevance_reranker_weights` builds that
behaviour into the exact bge-reranker shape by a structured construction (no training data
offline), and `relevance_candidates` draws candidate sets whose passages share 0..15 of the query's
terms, as retrieved candidates do:

  embeddings  token t carries a term weight w_t ~ U(0, 2) (an IDF stand-in) in dimension DIM_W;
              the positions of the query segment (the first `q_len` content positions after <s>)
              carry a segment flag in DIM_SEG; dimensions 0..62 hold only the token's own random
              vector (positions and types zeroed there) so two copies of one token match exactly
  layer 0     head 0 is a term matcher: q = k = alpha * (dims 0..62), plus a passage-side bonus in
              the key, so each query token attends to a copy of itself inside the passage when
              there is one and to itself otherwise; its value is the "passage side" flag, written
              by the O-projection into DIM_FOUND ("this query term occurs in the passage")
  layer 1     head 0 lets <s> attend to the query segment with weights ~ exp(2 w_t) and reads
              DIM_FOUND: a term-weighted fraction of the query found in the passage, written into
              DIM_REL
  layers 2..  Hugging Face random initialisation (N(0, 0.02)), the residual-branch output
              projections scaled by 1/sqrt(2 L) (GPT-2's residual init) so they perturb the
              relevance signal instead of washing it out
  head        classifier.dense row 0 reads DIM_REL, out_proj weights it by 4 (other rows random)

Everything else in layers 0 and 1 is zero, so the whole model runs through the same kernels
(folded LayerNorms, fused QKV + attention, GELU FFN, classification head) as any checkpoint.
Attention in layers 0 and 1 is saturated (margins of 10-20 nats), so the relevance signal is robust
to fp16 rounding while the candidates' logits spread over several units.
"""
from __future__ import annotations

import math

import numpy as np

from .encoder import ModelSpec, random_weights

DIM_SEG, DIM_W, DIM_FOUND, DIM_REL = 700, 701, 702, 703
CODE = 63                       # matching code dimensions 0..62 (head 0 of a 64-wide head)


def relevance_reranker_weights(spec: ModelSpec, seed: int = 0, q_len: int = 30) -> dict:
    """bge-reranker-shaped weights (XLM-R + classification head) whose logit is a term-weighted
    query/passage overlap plus the random layers' contribution.  q_len: query content tokens per
    pair (the query segment is positions [2 + 1, 2 + q_len], XLM-R position ids)."""
    assert spec.arch == "xlmr" and spec.classifier and spec.hidden > DIM_REL
    d, H, L = spec.hidden, spec.heads, spec.layers
    dh = d // H
    assert dh >= CODE + 1 and L >= 3
    w = random_weights(spec, seed, "hf")
    rng = np.random.default_rng(seed + 7919)
    sig = math.sqrt(3.0) * 0.02          # std of word + position + type before the embedding LN
    special = {DIM_SEG, DIM_W, DIM_FOUND, DIM_REL}
    we = w["embeddings.word_embeddings.weight"]
    pe = w["embeddings.position_embeddings.weight"]
    te = w["embeddings.token_type_embeddings.weight"]
    for m in (we, pe, te):
        m[:, sorted(special)] = 0.0
    pe[:, :CODE] = 0.0
    te[:, :CODE] = 0.0
    # equal-norm codes: every token's self-match score is the same (a chi-square spread of the
    # random norms would let weak self matches lose to random passage tokens)
    code = we[:, :CODE]
    code *= (0.02 * math.sqrt(CODE)) / np.maximum(np.linalg.norm(code, axis=1, keepdims=True), 1e-12)
    we[:, DIM_W] = sig * rng.uniform(0.0, 2.0, we.shape[0]).astype(np.float32)
    off = spec.position_offset
    first = off + 2                      # <s> is position off + 1, the query starts after it
    pe[first:first + q_len, DIM_SEG] = sig
    pe[off] = 0.0                        # padding_idx row

    def zero_layer(l):
        p = f"encoder.layer.{l}."
        for k in list(w):
            if k.startswith(p) and "LayerNorm" not in k:
                w[k][...] = 0.0
            elif k.startswith(p) and k.endswith("LayerNorm.weight"):
                w[k][...] = 1.0
            elif k.startswith(p) and k.endswith("LayerNorm.bias"):
                w[k][...] = 0.0
        return p

    # layer 0: the term matcher
    alpha, gamma = math.sqrt(18.3), math.sqrt(96.0)   # self match ~48 nats, bonus 12
    p = zero_layer(0)
    wq, bq = w[p + "attention.self.query.weight"], w[p + "attention.self.query.bias"]
    wk, bk = w[p + "attention.self.key.weight"], w[p + "attention.self.key.bias"]
    wv, bv = w[p + "attention.self.value.weight"], w[p + "attention.self.value.bias"]
    for i in range(CODE):
        wq[i, i] = alpha
        wk[i, i] = alpha
    bq[CODE] = gamma                      # q . k gains gamma^2 (1 - seg_j): the passage side
    wk[CODE, DIM_SEG] = -gamma
    bk[CODE] = gamma
    wv[0, DIM_SEG] = -1.0                 # value: 1 on the passage side, 0 in the query segment
    bv[0] = 1.0
    w[p + "attention.output.dense.weight"][DIM_FOUND, 0] = 4.0

    # layer 1: <s> gathers the term-weighted fraction of query terms found in the passage
    gamma1, beta = math.sqrt(80.0), 16.0
    p = zero_layer(1)
    w[p + "attention.self.query.bias"][0] = gamma1
    w[p + "attention.self.query.bias"][1] = beta
    wk = w[p + "attention.self.key.weight"]
    wk[0, DIM_SEG] = gamma1
    wk[1, DIM_W] = 1.0
    w[p + "attention.self.value.weight"][0, DIM_FOUND] = 1.0
    w[p + "attention.output.dense.weight"][DIM_REL, 0] = 4.0
    # centre it (the candidates' mean found fraction is ~1/4): the fp16 residual stream rounds
    # relative to the magnitude, so a centred signal keeps more of its spread above the rounding
    w[p + "attention.output.dense.bias"][DIM_REL] = -4.0

    # layers 2..L-1: HF random init, residual-branch outputs scaled by 1/sqrt(2 L)
    res = 1.0 / math.sqrt(2.0 * L)
    for l in range(2, L):
        p = f"encoder.layer.{l}."
        w[p + "attention.output.dense.weight"] *= res
        w[p + "output.dense.weight"] *= res
        # keep the special dimensions out of the random layers' outputs: they carry the signal
        for k in ("attention.output.dense.weight", "output.dense.weight"):
            w[p + k][sorted(special), :] = 0.0

    w["classifier.dense.weight"][0, :] = 0.0
    w["classifier.dense.weight"][0, DIM_REL] = 0.1
    w["classifier.out_proj.weight"][0, 0] = 4.0
    return w


def relevance_candidates(spec: ModelSpec, n_queries: int, n_cand: int = 100, q_len: int = 30,
                         p_len: int = 94, max_overlap: int = 15, seed: int = 0):
    """Queries of q_len distinct content tokens and, per query, n_cand passages of p_len tokens of
    which 0..max_overlap are query terms (random positions), the rest random vocabulary not in
    the query.  Returns (q_tok [nq, q_len], p_tok [nq * n_cand, p_len], overlap [nq, n_cand]) as
    int32 / int32 / int32, token ids in [1000, vocab)."""
    rng = np.random.default_rng(seed)
    V = spec.vocab_size
    q_tok = np.empty((n_queries, q_len), np.int32)
    p_tok = np.empty((n_queries * n_cand, p_len), np.int32)
    overlap = np.empty((n_queries, n_cand), np.int32)
    for b in range(n_queries):
        q = rng.choice(np.arange(1000, V), q_len, replace=False)
        q_tok[b] = q
        qs = set(q.tolist())
        for j in range(n_cand):
            m = int(rng.integers(0, max_overlap + 1))
            filler = rng.integers(1000, V, p_len)
            bad = np.array([t in qs for t in filler.tolist()])
            while bad.any():
                filler[bad] = rng.integers(1000, V, int(bad.sum()))
                bad = np.array([t in qs for t in filler.tolist()])
            pos = rng.choice(p_len, m, replace=False)
            filler[pos] = rng.choice(q, m, replace=False)
            p_tok[b * n_cand + j] = filler
            overlap[b, j] = m
    return q_tok, p_tok, overlap


# the fidelity set of tests/golden/rerank_fidelity.npz (tests/test_gpu_rerank_fidelity.py, bench.py)
FIDELITY = {"weight_seed": 12, "cand_seed": 5, "queries": 8, "cand": 100, "q_len": 30, "p_len": 94,
            "pair_len": 128}


def weight_checksum(w: dict) -> float:
    """Order-independent fp64 checksum of a weight dict (detects a drift of the generators)."""
    return float(sum(np.float64(np.abs(v).sum()) * (1 + i % 7)
                     for i, (k, v) in enumerate(sorted(w.items()))))


def fidelity_setup(spec: ModelSpec, **kw):
    """Weights and packed (query, passage) pairs of the ranking-fidelity set: returns
    (weights, ids [nq * cand, pair_len] int32, mask, overlap [nq, cand], meta).  XLM-R pair layout
    <s> q </s></s> p </s> (30 + 94 + 4 = 128 tokens, no truncation)."""
    m = dict(FIDELITY, **kw)
    w = relevance_reranker_weights(spec, m["weight_seed"], m["q_len"])
    q, p, overlap = relevance_candidates(spec, m["queries"], m["cand"], m["q_len"], m["p_len"],
                                         seed=m["cand_seed"])
    S = m["pair_len"]
    assert m["q_len"] + m["p_len"] + 4 == S
    n = m["queries"] * m["cand"]
    ids = np.empty((n, S), np.int32)
    qi = np.repeat(q, m["cand"], axis=0)
    ids[:, 0] = spec.bos_id
    ids[:, 1:1 + m["q_len"]] = qi
    ids[:, 1 + m["q_len"]] = spec.eos_id
    ids[:, 2 + m["q_len"]] = spec.eos_id
    ids[:, 3 + m["q_len"]:S - 1] = p
    ids[:, S - 1] = spec.eos_id
    return w, ids, np.ones_like(ids), overlap, m
