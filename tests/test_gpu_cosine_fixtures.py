"""GPU parity against the reference's own cosine code (tests/golden/cosine_fixtures.npz).

The fixture's cosines are graphiti's ``calculate_cosine_similarity`` (super_rag/graphiti/
graphiti_core/search/search_utils.py:56-67) evaluated by the reference itself in the build
container (tests/golden/gen_cosine_fixtures.py).  The store (K1 cosine_scan + K2 topk_select)
must return, for every query, the top-k rows of that reference ranking (distance = 1 - cos
ascending, ties by row: seekdb_connector.py:117-155) with distances within 1e-4 of 1 - cos_ref
plus the fp16 rounding the store applies to its normalised rows (measured per pair from the same
fp16 rounding on the host, so the bound is exact rather than a blanket tolerance).
"""
import numpy as np
import pytest

from oracle.cosine_topk import cosine_topk, quantize_like_store, same_topk_modulo_ties
from test_cosine_fixtures import CASES

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,C,Q,cos", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("k", [10, 100])
def test_store_topk_matches_reference_cosines(name, C, Q, cos, k):
    from super_rag_amd.store import NativeStore
    n, dim = C.shape
    k = min(k, n)
    s = NativeStore(dim, device=0)
    s.add(C.astype(np.float32))
    d_gpu, r_gpu = s.search(Q.astype(np.float32), k)
    assert (r_gpu >= 0).all()
    # per-pair rounding budget: cosine of the fp16-rounded unit vectors vs the reference cosine
    qq = quantize_like_store(Q).astype(np.float64)
    cq = quantize_like_store(C).astype(np.float64)
    rnd = np.abs(qq @ cq.T - cos)
    tol = 1e-4 + rnd
    got = 1.0 - d_gpu.astype(np.float64)
    want = np.take_along_axis(cos, r_gpu, axis=1)
    assert np.all(np.abs(got - want) <= np.take_along_axis(tol, r_gpu, axis=1)), name
    # reference top-k (cos desc, row asc) modulo ties within the rounding band
    order = np.stack([np.lexsort((np.arange(n), -c)) for c in cos])[:, :k]
    eps = 1e-4 + float(rnd.max()) * 2
    assert same_topk_modulo_ties(r_gpu, got, order, np.take_along_axis(cos, order, 1), eps), name
    # bit-exact index order against the oracle run on the rows as the store holds them
    d_or, r_or = cosine_topk(s.get(np.arange(n)).astype(np.float64), qq, k, normalize=False)
    assert same_topk_modulo_ties(r_gpu, got, r_or, 1.0 - d_or, 2e-6), name
    s.close()


def test_store_exact_ties_and_zero_query_order():
    from super_rag_amd.store import NativeStore
    case = {c[0]: c for c in CASES}
    for dim in (64, 384, 768, 1024):
        _, C, Q, cos = case[f"ties_zeros_{dim}"]
        s = NativeStore(dim, device=0)
        s.add(C.astype(np.float32))
        d, r = s.search(Q.astype(np.float32), 5)
        assert r[0, :4].tolist() == [1, 3, 7, 12]           # equal cosines: ascending row
        assert r[-1].tolist() == [0, 1, 2, 3, 4]            # zero query: cos 0 everywhere
        np.testing.assert_allclose(d[-1], 1.0, atol=0)
        s.close()
