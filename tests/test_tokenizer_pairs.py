"""Pair packing: the array form of Tokenizer.encode_pairs (per-request rerank path) equals the list
form (encode_pairs_ref) and the HF LongestFirst truncation rule, on random query / passage lengths
around and beyond the budget, both pair styles (XLM-R <s> q </s></s> p </s>, BERT [CLS] q [SEP] p
[SEP] with token types), empty passages."""
import random

import numpy as np

from super_rag_amd.encoder import MODELS
from super_rag_amd.tokenizer import Tokenizer, longest_first, longest_first_arrays


def test_longest_first_arrays_equals_scalar_rule():
    bs = np.arange(0, 160)
    for a in range(0, 60, 3):
        for budget in (0, 1, 2, 3, 10, 61, 124, 125, 508):
            na, nb = longest_first_arrays(a, bs, budget)
            for b in bs:
                assert (na[b], nb[b]) == longest_first(a, int(b), budget)


def test_encode_pairs_array_form_equals_list_form():
    words = [f"w{i}" for i in range(400)]
    rng = random.Random(5)
    for name in ("bge-reranker-base", "bge-base-en"):
        tok = Tokenizer(MODELS[name], synthetic=True)
        for _ in range(120):
            q = " ".join(rng.choice(words) for _ in range(rng.randint(0, 140)))
            ps = [" ".join(rng.choice(words) for _ in range(rng.randint(0, 180)))
                  for _ in range(rng.randint(1, 24))]
            if rng.random() < 0.25:
                ps.append("")
            ml = rng.choice([None, 4, 16, 64, 128, 512])
            got, ref = tok.encode_pairs(q, ps, ml), tok.encode_pairs_ref(q, ps, ml)
            for x, y in zip(got, ref):
                assert x.dtype == y.dtype and x.shape == y.shape
                np.testing.assert_array_equal(x, y)
