"""GPU: every BASELINE.json configuration at its own size, on the HIP path.

  config 1  bge-small-en embed of 1k chunks (S = 128) through the ingest path + top-5 through the
            connector (the reference's CPU plumbing configuration, here on the GPU)
  config 2  1M x 768 corpus, 12-layer bge-base-en embed, B = 32, exact top-10
  config 3  the same corpus + 12-layer bge-reranker-base (XLM-R base) at S_pair = 128, top-100 -> 10
  config 4  10M x 768 corpus, B = 256, top-100 -> rerank -> 10 (one GPU holds the whole corpus)
  config 5  24-layer bge-m3 embed at S = 32 and S = 8192; the 6.25M x 1024 per-GPU shard scanned in
            fp8 and fused with BM25 over the passage tokens by rrf

Weights are seeded random with the models' exact shapes ("hf" initialisation, classifier head
unscaled); corpora follow bench.py's clustered distribution.  Checks:
embeddings against the oracle (oracle/encoder_ref.py; the 24-layer / 8192-token cases run the same
torch restatement in fp32 on the GPU, TF32 off), search against the fp64 oracle on the rows the
store holds, rerank logits against the oracle on the GPU's candidates, and at the 10M / 6.25M sizes
the size-independent properties: recall@10 vs exact fp32 >= 0.99, rrf(dense, BM25) identity.
Reference call sites replaced: embedding_service.py:168-175, seekdb_connector.py:98-115,
rerank_service.py:95-104.
"""
import gc
import os

import numpy as np
import pytest

from model_dirs import ref_config
from oracle import encoder_ref as R
from oracle.cosine_topk import cosine_topk, quantize_like_store, recall_at_k, same_topk_modulo_ties

pytestmark = pytest.mark.gpu

# fp16 GEMM operands / fp32 accumulation, fp32 residual (embedders): ||e - e_ref||_2 per embedding
EMB_TOL = 1e-3            # north_star: embeddings within 1e-3
# bge-reranker-base with the fp16 residual stream, unscaled head, S_pair = 128: |logit - ref|.
# Seeded-random logits spread by std 1.3e-2; the fp16 path's error is mean ~1.9e-4 with a max over
# the 400 logits of 6.7e-4 .. 1.02e-3 across builds (tools/diag_kvfree.py, profiles/r03_kvfree/):
# changes of rounding order alone (the FFN1 erf table, the K/V-free last layer) move single logits
# by <= 2.1e-4.  1.5e-3 (~0.11 std) keeps the check 7x tighter than this shape's documented band
# 1e-2 (1 + max|l|) without failing on that spread; ranking fidelity proper is pinned by
# test_gpu_rerank_fidelity.py (discriminative weights, std / err >= 120).
RERANK_TOL = 1.5e-3
# and the MEAN |logit - ref| over the 400 logits (measured 1.9e-4): a
# systematic drift fails here even while every single logit stays under RERANK_TOL
RERANK_MEAN_TOL = 3e-4
# the default K/V-free last layer against the SR_KVFREE_CLS=0 path on the same pairs
KVFREE_TOL = 3e-4
# and the SR_KVFREE_CLS=0 path (K, V GEMM + CLS attention) against the fp32 oracle itself
# (ADVICE r3 / VERDICT r4 item 4b): the alternative last layer is held to the same absolute bar
KV_PATH_TOL = 1e-3


def _free():
    import torch
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _corpus_store(n, dim, seed_centers=0):
    import torch
    from bench import gen_corpus_chunk
    from super_rag_amd.store import NativeStore
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(seed_centers)
    centers = torch.randn((1024, dim), generator=g).to(dev)
    store = NativeStore(dim, device=0, capacity=n)
    for c0 in range(0, n, 1 << 20):
        store.add_dev(gen_corpus_chunk(c0, min(n, c0 + (1 << 20)), dim, centers, dev))
    torch.cuda.synchronize()
    return store, centers


def _queries(spec, B, S, seed):
    import torch
    g = torch.Generator(device="cuda").manual_seed(seed)
    ids = torch.randint(1000, spec.vocab_size, (B, S), generator=g, device="cuda", dtype=torch.int32)
    ids[:, 0] = spec.bos_id
    ids[:, -1] = spec.eos_id
    return ids, torch.ones_like(ids)


def _exact_top(q, centers, n, dim, k):
    """Exact fp32 top-k over the unquantised corpus (torch on the GPU, chunked)."""
    import torch
    from bench import gen_corpus_chunk
    best_s = torch.full((q.shape[0], 0), -2.0, device=q.device)
    best_r = torch.zeros((q.shape[0], 0), dtype=torch.int64, device=q.device)
    for c0 in range(0, n, 1 << 20):
        x = torch.nn.functional.normalize(gen_corpus_chunk(c0, min(n, c0 + (1 << 20)), dim, centers,
                                                           q.device), dim=1)
        best_s = torch.cat([best_s, q @ x.T], 1)
        best_r = torch.cat([best_r, torch.arange(c0, c0 + x.shape[0], device=q.device).expand(q.shape[0], -1)], 1)
        top = best_s.topk(k, dim=1)
        best_s, best_r = top.values, best_r.gather(1, top.indices)
    return best_r.cpu().numpy()


def _gpu_weights(w):
    import torch
    return {k: torch.as_tensor(v, device="cuda") for k, v in w.items()}


@pytest.fixture
def fp32_highest():
    import torch
    old = torch.backends.cuda.matmul.allow_tf32, torch.get_float32_matmul_precision()
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.set_float32_matmul_precision("highest")
    yield
    torch.backends.cuda.matmul.allow_tf32 = old[0]
    torch.set_float32_matmul_precision(old[1])


@pytest.fixture(scope="module")
def corpus_1m():
    store, centers = _corpus_store(1_000_000, 768)
    stored = store.get(np.arange(1_000_000))          # the fp16 rows as the store holds them
    yield store, centers, stored
    store.close()
    _free()


def test_config1_bge_small_ingest_1k_chunks_top5():
    """Config 1: 1,000 chunks of 128 tokens embedded by the 12-layer bge-small-en (d_h = 32: the
    K5 attention) through VectorIndexer.create_index (index/vector_and_full_text_index.py:29-129)
    into the connector, then top-5 through MI355XVectorStoreConnector.search
    (seekdb_connector.py:98-155); embeddings against the oracle on a sample, the top-5 against the
    fp64 oracle over the rows the store holds."""
    from types import SimpleNamespace
    from super_rag_amd import vectorstore as V
    from super_rag_amd.embed import EmbeddingService
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    from super_rag_amd.index import VectorIndexer, chunk_text
    from super_rag_amd.models import QueryWithEmbedding
    from super_rag_amd.tokenizer import Tokenizer
    es = MODELS["bge-small-en"]
    w = random_weights(es, 31, "hf")
    tok = Tokenizer(es)
    svc = EmbeddingService("openai", "BAAI/bge-small-en", "", "", 10, encoder=Encoder(es, weights=w),
                           tokenizer=tok, device_batch=128)
    rng = np.random.default_rng(32)
    words = [f"w{i}" for i in range(5000)]
    parts = [SimpleNamespace(content=" ".join(rng.choice(words, 126)), metadata={"name": f"c{i}.md"})
             for i in range(1000)]
    V._collections.clear()
    conn = V.MI355XVectorStoreConnector({"collection": "config1", "device": 0})
    ids = VectorIndexer(conn, svc).create_index(parts)["context_ids"]
    assert len(ids) == 1000
    stored = conn.get_vectors(ids)
    texts = [chunk_text(p).replace("\n", " ") for p in parts]
    for i in (0, 499, 999):
        t_ids, t_mask = tok.encode_batch([texts[i]])
        ref = R.embed(ref_config(es), w, t_ids, t_mask)[0]
        assert np.linalg.norm(stored[i] - ref) <= 4e-3        # fp16-stored row vs fp32 oracle
    q = stored[rng.choice(1000, 16, replace=False)] + 0.3 * rng.standard_normal((16, es.hidden)).astype(np.float32)
    got = [[h.metadata["source"] for h in conn.search(QueryWithEmbedding(query="q", top_k=5,
                                                                         embedding=v.tolist())).results]
           for v in q]
    d_ref, r_ref = cosine_topk(stored, quantize_like_store(q), 5, normalize=False)
    for b in range(16):
        want = [f"c{r}.md" for r in r_ref[b]]
        assert got[b] == want or sorted(got[b]) == sorted(want)   # order modulo exact ties
    conn.delete_collection()
    V._collections.clear()


def test_config2_bge_base_embed_and_top10_over_1m(corpus_1m):
    import torch
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    store, _, stored = corpus_1m
    es = MODELS["bge-base-en"]
    we = random_weights(es, 11, "hf")
    emb = Encoder(es, weights=we, max_tokens=32 * 32)
    ids, mask = _queries(es, 32, 32, seed=2)
    q = emb.embed_dev(ids, mask, fp16=False)
    e_ref = R.embed(ref_config(es), we, ids.cpu().numpy(), mask.cpu().numpy())
    err = np.linalg.norm(q.cpu().numpy() - e_ref, axis=1)
    print(f"config2 embed: max ||e - e_ref|| {err.max():.2e} over 32 queries")
    assert err.max() <= EMB_TOL
    sims, rows = store.search_dev(q, 10)
    qh = quantize_like_store(q.cpu().numpy()).astype(np.float64)
    d_ref, r_ref = cosine_topk(stored, qh, 10, normalize=False)
    s, r = sims.cpu().numpy(), rows.cpu().numpy()
    assert same_topk_modulo_ties(r, s, r_ref, 1.0 - d_ref, 1e-4)
    np.testing.assert_allclose(1.0 - s, d_ref, atol=1e-4)
    emb.close()
    del q, sims, rows
    _free()


def test_config3_rerank_top100_to_10_over_1m(corpus_1m, fp32_highest):
    import torch
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    from super_rag_amd.pipeline import SearchPipeline
    store, _, stored = corpus_1m
    es, rs = MODELS["bge-base-en"], MODELS["bge-reranker-base"]
    we, wr = random_weights(es, 11, "hf"), random_weights(rs, 12, "hf")
    emb = Encoder(es, weights=we, max_tokens=32 * 32)
    rer = Encoder(rs, weights=wr, max_tokens=32 * 100 * 128)
    g = torch.Generator(device="cuda").manual_seed(5)
    N = 1_000_000
    p_tok = torch.randint(1000, rs.vocab_size, (N, 94), generator=g, device="cuda", dtype=torch.int32)
    p_len = torch.full((N,), 94, dtype=torch.int32, device="cuda")
    ids, mask = _queries(es, 32, 32, seed=3)
    q_tok = torch.randint(1000, rs.vocab_size, (32, 30), generator=g, device="cuda", dtype=torch.int32)
    q_len = torch.full((32,), 30, dtype=torch.int32, device="cuda")
    pipe = SearchPipeline(emb, rer, store, p_tok, p_len, k_candidates=100, k_final=10, pair_len=128)
    res = pipe.run(ids, mask, q_tok, q_len)
    torch.cuda.synchronize()
    cand = res.cand_rows.cpu().numpy()
    # candidates: exact top-100 of the stored rows for the GPU's fp16 queries
    q16 = pipe.embed(ids, mask).float().cpu().numpy()
    d_ref, r_ref = cosine_topk(stored, quantize_like_store(q16).astype(np.float64), 100, normalize=False)
    assert same_topk_modulo_ties(cand, res.cand_sims.cpu().numpy(), r_ref, 1.0 - d_ref, 1e-4)
    # logits of 4 queries x 100 pairs (S = 128) against the fp32 restatement
    nq = 4
    pt, pl = p_tok.cpu().numpy(), p_len.cpu().numpy()
    pids, pmask, _ = R.pack_pairs(q_tok[:nq].cpu().numpy(), q_len[:nq].cpu().numpy(), pt, pl,
                                  cand[:nq], 128, 0, rs.bos_id, rs.eos_id, rs.pad_id)
    lg_ref = R.cross_logits(ref_config(rs), _gpu_weights(wr), pids, pmask)[:, 0].reshape(nq, 100)
    lg = rer.cross_score_dev(*[torch.from_numpy(np.ascontiguousarray(a)).cuda().int()
                               for a in (pids, pmask)])[:, 0].view(nq, 100).cpu().numpy()
    dlog = np.abs(lg - lg_ref).max()
    dmean = np.abs(lg - lg_ref).mean()
    print(f"config3 rerank: max |logit - ref| {dlog:.2e}, mean {dmean:.2e}, logit std "
          f"{lg_ref.std():.2e}, max |logit| {np.abs(lg_ref).max():.2e}")
    assert dlog <= RERANK_TOL
    assert dmean <= RERANK_MEAN_TOL
    # the K/V-free CLS-only last layer against the K, V GEMM + CLS attention path on the same
    # pairs: a rounding-order change only, measured <= 2.1e-4
    os.environ["SR_KVFREE_CLS"] = "0"
    try:
        lg_kv = rer.cross_score_dev(*[torch.from_numpy(np.ascontiguousarray(a)).cuda().int()
                                      for a in (pids, pmask)])[:, 0].view(nq, 100).cpu().numpy()
    finally:
        del os.environ["SR_KVFREE_CLS"]
    dkv = np.abs(lg - lg_kv).max()
    dkv_ref = np.abs(lg_kv - lg_ref).max()
    print(f"config3 rerank: K/V-free vs K/V last layer max |dlogit| {dkv:.2e}, K/V path vs ref "
          f"{dkv_ref:.2e}")
    assert dkv <= KVFREE_TOL
    assert dkv_ref <= KV_PATH_TOL
    final, flog = res.rows.cpu().numpy(), res.logits.cpu().numpy()
    for b in range(nq):
        order = sorted(range(100), key=lambda j: (-lg_ref[b, j], j))[:10]
        assert same_topk_modulo_ties(final[b:b + 1], flog[b:b + 1], cand[b, order][None],
                                     lg_ref[b, order][None], 2 * RERANK_TOL)
    emb.close()
    rer.close()
    del p_tok, res
    _free()


def test_config4_10m_b256_recall_and_full_step():
    import torch
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    from super_rag_amd.pipeline import SearchPipeline
    N = 10_000_000
    store, centers = _corpus_store(N, 768)
    es, rs = MODELS["bge-base-en"], MODELS["bge-reranker-base"]
    emb = Encoder(es, weights=random_weights(es, 11, "hf"), max_tokens=256 * 32)
    rer = Encoder(rs, weights=random_weights(rs, 12, "hf"), max_tokens=1 << 19)
    g = torch.Generator(device="cuda").manual_seed(5)
    p_tok = torch.randint(1000, rs.vocab_size, (N, 94), generator=g, device="cuda", dtype=torch.int32)
    p_len = torch.full((N,), 94, dtype=torch.int32, device="cuda")
    ids, mask = _queries(es, 256, 32, seed=2)
    q_tok = torch.randint(1000, rs.vocab_size, (256, 30), generator=g, device="cuda", dtype=torch.int32)
    q_len = torch.full((256,), 30, dtype=torch.int32, device="cuda")
    pipe = SearchPipeline(emb, rer, store, p_tok, p_len, k_candidates=100, k_final=10, pair_len=128)
    res = pipe.run(ids, mask, q_tok, q_len)
    q = emb.embed_dev(ids[:32], mask[:32], fp16=False)
    truth = _exact_top(q, centers, N, 768, 10)
    rec = recall_at_k(res.cand_rows[:32, :10].cpu().numpy(), truth)
    print(f"config4: recall@10 of the search stage vs exact fp32 {rec:.4f} (32 queries)")
    assert rec >= 0.99
    final, cand = res.rows.cpu().numpy(), res.cand_rows.cpu().numpy()
    assert final.shape == (256, 10) and (final >= 0).all() and (final < N).all()
    for b in range(256):
        assert set(final[b].tolist()) <= set(cand[b].tolist()) and len(set(final[b].tolist())) == 10
    assert np.all(np.diff(res.logits.cpu().numpy(), axis=1) <= 0)      # logit descending
    store.close()
    emb.close()
    rer.close()
    del p_tok, res, pipe
    _free()


def test_config4_reranker_full_chunk_batch_invariance():
    """The bench's reranker chunk: 12,800 pairs x 128 tokens = 1,638,400 tokens in one persistent-GEMM
    launch per layer.  Every stage is row- or sequence-local, so the logits of a 400-pair subset
    computed inside the full chunk equal the subset's own launch bit for bit (a tile-walk or
    hand-over fault at 6,400 tiles would break this); four of them against the oracle."""
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    rs = MODELS["bge-reranker-base"]
    w = random_weights(rs, 12, "hf")
    rer = Encoder(rs, weights=w, max_tokens=1_638_400)
    rng = np.random.default_rng(9)
    B, S = 12_800, 128
    ids = rng.integers(1000, rs.vocab_size, (B, S)).astype(np.int32)
    lens = rng.integers(96, S + 1, B)
    mask = (np.arange(S)[None] < lens[:, None]).astype(np.int32)
    ids[:, 0] = rs.bos_id
    ids = np.where(mask == 1, ids, rs.pad_id).astype(np.int32)
    full = rer.cross_score(ids, mask)[:, 0]
    pick = np.sort(rng.choice(B, 400, replace=False))[::-1].copy()   # reversed order as well
    sub = rer.cross_score(ids[pick], mask[pick])[:, 0]
    np.testing.assert_array_equal(full[pick], sub)
    ref = R.cross_logits(ref_config(rs), w, ids[pick[:4]], mask[pick[:4]])[:, 0]
    assert np.abs(sub[:4] - ref).max() <= RERANK_TOL
    rer.close()
    _free()


@pytest.mark.parametrize("B,S", [(8, 32), (1, 8192)])
def test_config5_bge_m3_24_layers(B, S, fp32_highest):
    import torch
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    spec = MODELS["bge-m3"]
    w = random_weights(spec, 21, "hf")
    enc = Encoder(spec, weights=w, max_tokens=B * S)
    ids, mask = _queries(spec, B, S, seed=S)
    if B > 1:                                   # a ragged batch: padding masked, XLM-R positions
        ids[1, S // 2:] = spec.pad_id
        mask[1, S // 2:] = 0
        ids[1, S // 2 - 1] = spec.eos_id
    e = enc.embed_dev(ids, mask, fp16=False).cpu().numpy()
    e_ref = R.embed(ref_config(spec), _gpu_weights(w), ids.cpu().numpy(), mask.cpu().numpy())
    err = np.linalg.norm(e - e_ref, axis=1)
    print(f"config5 bge-m3 24L B={B} S={S}: max ||e - e_ref|| {err.max():.2e}")
    assert err.max() <= EMB_TOL
    enc.close()
    _free()


def test_config5_fp8_hybrid_shard_6_25m():
    import torch
    from bench import build_lexical
    from oracle.bm25 import rrf_rows
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    from super_rag_amd.lexical import query_arrays
    from super_rag_amd.pipeline import SearchPipeline
    N, dim = 6_250_000, 1024
    store, centers = _corpus_store(N, dim)
    store.set_scan_dtype("fp8")
    es, rs = MODELS["bge-m3"], MODELS["bge-reranker-base"]
    emb = Encoder(es, weights=random_weights(es, 21, "hf"), max_tokens=256 * 32)
    rer = Encoder(rs, weights=random_weights(rs, 12, "hf"), max_tokens=1 << 19)
    g = torch.Generator(device="cuda").manual_seed(5)
    p_tok = torch.randint(1000, rs.vocab_size, (N, 94), generator=g, device="cuda", dtype=torch.int32)
    p_len = torch.full((N,), 94, dtype=torch.int32, device="cuda")
    lex = build_lexical(p_tok, p_len, 0)
    ids, mask = _queries(es, 256, 32, seed=2)
    q_tok = torch.randint(1000, rs.vocab_size, (256, 30), generator=g, device="cuda", dtype=torch.int32)
    q_len = torch.full((256,), 30, dtype=torch.int32, device="cuda")
    pipe = SearchPipeline(emb, rer, store, p_tok, p_len, k_candidates=100, k_final=10, pair_len=128,
                          lexical=lex, k_each=100)
    res = pipe.run(ids, mask, q_tok, q_len)
    q16 = pipe.embed(ids, mask)
    _, dense = store.search_dev(q16, 100)
    qoff, qterms = query_arrays([q_tok[i, :30].cpu().numpy() for i in range(256)])
    _, lexical = lex.search_dev(qoff, qterms, 100)
    so, ro = rrf_rows(dense.cpu().numpy(), lexical.cpu().numpy(), 100, 1)
    np.testing.assert_array_equal(res.cand_rows.cpu().numpy(), ro)      # fused = rrf(dense, BM25)
    np.testing.assert_allclose(res.cand_sims.cpu().numpy(), so.astype(np.float32))
    q = emb.embed_dev(ids[:32], mask[:32], fp16=False)
    truth = _exact_top(q, centers, N, dim, 10)
    rec = recall_at_k(dense[:32, :10].cpu().numpy(), truth)
    print(f"config5: fp8-scan recall@10 vs exact fp32 {rec:.4f} (32 queries, 6.25M x 1024)")
    assert rec >= 0.99
    store.close()
    emb.close()
    rer.close()
    del p_tok, res, pipe, lex
    _free()
