"""CPU: the search oracle pinned to the reference's own cosine code.

tests/golden/cosine_fixtures.npz holds the outputs of graphiti's ``calculate_cosine_similarity``
(super_rag/graphiti/graphiti_core/search/search_utils.py:56-67) and ``normalize_l2``
(graphiti_core/helpers.py:100-103), imported from /root/reference by
tests/golden/gen_cosine_fixtures.py, on 20 cases (random, clustered, exact ties + zero rows +
a zero query, power-of-two scaled rows, sparse rows; dims 64/384/768/1024).  oracle/cosine_topk.py
must reproduce those cosines to fp64 rounding and rank rows by (cosine desc, row asc) — the
SeekDB distance order (score = 1 - cos ascending, seekdb_connector.py:117-155).
"""
import os

import numpy as np
import pytest

from oracle.cosine_topk import cosine_topk, normalize_rows

FIX = os.path.join(os.path.dirname(__file__), "golden", "cosine_fixtures.npz")


def load_cases():
    z = np.load(FIX)
    out = []
    for name in z["cases"].tolist():
        val = lambda c, e: c.astype(np.float64) / 16.0 * np.exp2(e.astype(np.float64))[:, None]
        out.append((name, val(z[name + ".c"], z[name + ".ce"]), val(z[name + ".q"], z[name + ".qe"]),
                    z[name + ".cos"]))
    return out


def reference_order(cos):
    """Rows by (cos desc, row asc) per query: the order SeekDB's distance = 1 - cos yields."""
    n = cos.shape[1]
    return np.stack([np.lexsort((np.arange(n), -c)) for c in cos])


CASES = load_cases()


def test_fixture_covers_the_requested_cases():
    names = [c[0] for c in CASES]
    for fam in ("random", "clustered", "ties_zeros", "scaled", "sparse"):
        for dim in (64, 384, 768, 1024):
            assert f"{fam}_{dim}" in names
    assert sum(c[3].size for c in CASES) >= 20_000


@pytest.mark.parametrize("name,C,Q,cos", CASES, ids=[c[0] for c in CASES])
def test_oracle_reproduces_reference_cosines_and_order(name, C, Q, cos):
    n = C.shape[0]
    dist, rows = cosine_topk(C, Q, n, chunk=48)       # several chunks: exercises the running merge
    sims = np.empty_like(cos)
    np.put_along_axis(sims, rows, 1.0 - dist, axis=1)
    np.testing.assert_allclose(sims, cos, rtol=0, atol=4e-15)
    ref = reference_order(cos)
    for b in range(Q.shape[0]):
        if np.array_equal(rows[b], ref[b]):
            continue
        # only fp64 near-ties (|delta cos| < 1e-14) may be ordered differently
        diff = np.nonzero(rows[b] != ref[b])[0]
        assert np.all(np.abs(cos[b, rows[b, diff]] - cos[b, ref[b, diff]]) < 1e-14), (name, b)


def test_exact_ties_and_zero_vectors_follow_the_reference():
    case = {c[0]: c for c in CASES}
    for dim in (64, 384, 768, 1024):
        _, C, Q, cos = case[f"ties_zeros_{dim}"]
        # duplicates of row 1 (rows 3, 7, 12) tie at cos 1 with query 0: ascending row order
        _, rows = cosine_topk(C, Q, 4)
        assert rows[0].tolist() == [1, 3, 7, 12]
        assert np.allclose(cos[0, [1, 3, 7, 12]], 1.0)
        # the zero query: the reference returns 0 for every row -> rows 0..k-1 in order
        _, rows = cosine_topk(C, Q, 5)
        assert np.all(cos[-1] == 0) and rows[-1].tolist() == [0, 1, 2, 3, 4]
        # zero rows have cosine 0 against every query
        assert np.all(cos[:, [2, 9]] == 0)


def test_normalize_rows_matches_reference_normalize_l2():
    z = np.load(FIX)
    for dim in (64, 384, 768, 1024):
        v = z[f"norm_{dim}.v"].astype(np.float64) / 16.0 * np.exp2(z[f"norm_{dim}.e"].astype(np.float64))[:, None]
        np.testing.assert_allclose(normalize_rows(v), z[f"norm_{dim}.out"], rtol=0, atol=1e-16)
        assert np.all(z[f"norm_{dim}.out"][2] == 0)      # zero vector left unchanged
