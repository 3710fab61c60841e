"""GPU parity of the whole batched hot path (SearchPipeline: embed -> exact top-K -> pair packing
-> cross-encoder -> top-k) against the oracle composition, stage by stage, on one GPU."""
import numpy as np
import pytest

from oracle import encoder_ref as R
from oracle.cosine_topk import cosine_topk, quantize_like_store, same_topk_modulo_ties

pytestmark = pytest.mark.gpu


def _cfg(s):
    return R.RefConfig(s.vocab_size, s.hidden, s.layers, s.heads, s.intermediate, s.max_position,
                       s.type_vocab, s.ln_eps, s.position_offset, s.classifier, s.num_labels)


@pytest.mark.parametrize("res16", [False, True])
def test_pipeline_stages_match_oracle(res16):
    import torch
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    from super_rag_amd.pipeline import SearchPipeline
    from super_rag_amd.store import NativeStore

    es = ModelSpec("e", "bert", 2000, 128, 2, 2, 256, 64, 2, 1e-12, 0)
    rs = ModelSpec("r", "xlmr", 2000, 128, 2, 2, 256, 80, 1, 1e-5, 1, classifier=1, bos_id=0,
                   eos_id=2, pad_id=1, residual_fp16=res16)
    we, wr = random_weights(es, 1, "test"), random_weights(rs, 2, "test")
    wr["classifier.out_proj.weight"] *= 50.0
    emb, rer = Encoder(es, weights=we), Encoder(rs, weights=wr)
    rng = np.random.default_rng(0)
    N, B, K, k, S, Lq, Lp = 20000, 12, 20, 5, 48, 10, 40
    corpus = rng.standard_normal((N, 128)).astype(np.float32)
    store = NativeStore(128)
    store.add(corpus)
    p_tok = rng.integers(5, 2000, (N, Lp)).astype(np.int32)
    p_len = rng.integers(1, Lp + 1, N).astype(np.int32)
    q_ids = rng.integers(5, 2000, (B, 16)).astype(np.int32)
    q_ids[:, 0] = 101
    q_mask = np.ones_like(q_ids)
    q_tok = rng.integers(5, 2000, (B, Lq)).astype(np.int32)
    q_len = rng.integers(1, Lq + 1, B).astype(np.int32)
    t = lambda a: torch.from_numpy(a).cuda()
    pipe = SearchPipeline(emb, rer, store, t(p_tok), t(p_len), k_candidates=K, k_final=k, pair_len=S)
    res = pipe.run(t(q_ids), t(q_mask), t(q_tok), t(q_len))
    q16 = pipe.embed(t(q_ids), t(q_mask)).float().cpu().numpy()
    torch.cuda.synchronize()

    # stage 1: embeddings vs the fp32 oracle
    e_ref = R.embed(_cfg(es), we, q_ids, q_mask)
    assert (np.linalg.norm(q16 - e_ref, axis=1) <= 2e-3).all()
    # stage 2: candidates = exact top-K of the store rows for the GPU's own (fp16) query vectors
    stored = store.get(np.arange(N))
    d_ref, r_ref = cosine_topk(stored, quantize_like_store(q16), K, normalize=False)
    cand = res.cand_rows.cpu().numpy()
    sims = res.cand_sims.cpu().numpy()
    assert same_topk_modulo_ties(cand, sims, r_ref, 1.0 - d_ref, 1e-4)
    # stage 3+4: pair packing and cross-encoder logits on the GPU's candidates
    ids, mask, _ = R.pack_pairs(q_tok, q_len, p_tok, p_len, cand, S, 0, 0, 2, 1)
    lg_ref = R.cross_logits(_cfg(rs), wr, ids, mask)[:, 0].reshape(B, K)
    tol = (4e-3 if res16 else 2e-3) * (1.0 + np.abs(lg_ref).max())
    final = res.rows.cpu().numpy()
    flog = res.logits.cpu().numpy()
    for b in range(B):
        order = sorted(range(K), key=lambda j: (-lg_ref[b, j], j))[:k]
        exp_rows = cand[b, order]
        assert same_topk_modulo_ties(final[b:b + 1], flog[b:b + 1], exp_rows[None],
                                     lg_ref[b, order][None], 2 * tol)
        got = dict(zip(cand[b].tolist(), range(K)))
        np.testing.assert_allclose(flog[b], lg_ref[b, [got[r] for r in final[b]]], atol=tol)


def test_hybrid_pipeline_candidates_are_rrf_of_dense_and_bm25():
    # hybrid SearchPipeline (config 5): candidates = rrf(dense top-k_each, BM25 top-k_each over the
    # passage tokens with the query tokens); BM25 side against the oracle, bit-exact
    import torch
    from oracle.bm25 import LexCorpus, bm25_topk, rrf_rows
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    from super_rag_amd.lexical import NativeLexIndex, doc_arrays
    from super_rag_amd.pipeline import SearchPipeline
    from super_rag_amd.store import NativeStore
    es = ModelSpec("e", "bert", 2000, 128, 2, 2, 256, 64, 2, 1e-12, 0)
    rs = ModelSpec("r", "xlmr", 600, 128, 2, 2, 256, 80, 1, 1e-5, 1, classifier=1, bos_id=0,
                   eos_id=2, pad_id=1, residual_fp16=True)
    emb, rer = Encoder(es, weights=random_weights(es, 1, "test")), Encoder(rs, weights=random_weights(rs, 2, "test"))
    rng = np.random.default_rng(4)
    N, B, K, ke, k, S = 12000, 16, 40, 30, 5, 48
    corpus = rng.standard_normal((N, 128)).astype(np.float32)
    p_tok = ((rng.zipf(1.3, (N, 40)) - 1) % 590 + 5).astype(np.int32)
    p_len = rng.integers(1, 41, N).astype(np.int32)
    store = NativeStore(128)
    store.add(corpus)
    docs = [p_tok[i, :p_len[i]].tolist() for i in range(N)]
    lex = NativeLexIndex()
    lex.add(docs)
    q_ids = rng.integers(5, 2000, (B, 16)).astype(np.int32)
    q_ids[:, 0] = 101
    q_tok = ((rng.zipf(1.3, (B, 10)) - 1) % 590 + 5).astype(np.int32)
    q_len = rng.integers(1, 11, B).astype(np.int32)
    t = lambda a: torch.from_numpy(a).cuda()
    pipe = SearchPipeline(emb, rer, store, t(p_tok), t(p_len), k_candidates=K, k_final=k,
                          pair_len=S, lexical=lex, k_each=ke)
    res = pipe.run(t(q_ids), t(np.ones_like(q_ids)), t(q_tok), t(q_len))
    q16 = pipe.embed(t(q_ids), t(np.ones_like(q_ids)))
    _, dense = store.search_dev(q16, ke)
    queries = [q_tok[i, :q_len[i]].tolist() for i in range(B)]
    _, lexical = bm25_topk(LexCorpus(*doc_arrays(docs)), queries, ke)
    so, ro = rrf_rows(dense.cpu().numpy(), lexical, K, 1)
    np.testing.assert_array_equal(res.cand_rows.cpu().numpy(), ro)
    np.testing.assert_allclose(res.cand_sims.cpu().numpy(), so.astype(np.float32))
    final = res.rows.cpu().numpy()
    for b in range(B):
        assert set(final[b].tolist()) <= set(ro[b].tolist())


def _sharded_worker(rank, world, port, out_q):
    # one rank of a world-size-2 SearchPipeline sharing the box's GPU (gloo exchange staged through
    # host memory; the same code runs over RCCL, one rank per GPU, in bench.py)
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "super-rag_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        res = _run_pipeline(rank, world)
        res_h = _run_pipeline(rank, world, hybrid=True)
        res_p = _run_pipeline(rank, world, shard_passages=True)
        res_hp = _run_pipeline(rank, world, hybrid=True, shard_passages=True)
        out_q.put((rank, (res, res_h, res_p, res_hp)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _rccl_worker(port, out_q):
    # a world of one over the nccl backend (RCCL) with the exchange forced on: the all_gather /
    # all_to_all / all_reduce calls of the sharded path run on device tensors
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "super-rag_amd")]
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        res = _run_pipeline(0, 1, force_exchange=True)
        res_h = _run_pipeline(0, 1, hybrid=True, force_exchange=True)
        res_p = _run_pipeline(0, 1, force_exchange=True, shard_passages=True)
        out_q.put((res, res_h, res_p))
    finally:
        dist.destroy_process_group()


def test_rccl_exchange_world_one_equals_plain_path():
    import os
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(29500 + os.getpid() % 150, q))
    p.start()
    res, res_h, res_p = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    plain, plain_h = _run_pipeline(0, 1), _run_pipeline(0, 1, hybrid=True)
    for got, want in ((res, plain), (res_h, plain_h), (res_p, plain)):
        for f in ("rows", "cand_rows", "cand_sims", "logits"):
            np.testing.assert_array_equal(got[f], want[f])


def _run_pipeline(rank, world, sharded=True, hybrid=False, force_exchange=False, shard_passages=False):
    # rank's B queries; sharded: over rows [r0, r1) of the corpus (shard_offset r0) inside a
    # world-size process group, else over the whole corpus in a single process
    import torch
    from super_rag_amd.encoder import Encoder, ModelSpec, random_weights
    from super_rag_amd.pipeline import SearchPipeline
    from super_rag_amd.store import NativeStore
    es = ModelSpec("e", "bert", 2000, 128, 2, 2, 256, 64, 2, 1e-12, 0)
    rs = ModelSpec("r", "xlmr", 2000, 128, 2, 2, 256, 80, 1, 1e-5, 1, classifier=1, bos_id=0,
                   eos_id=2, pad_id=1, residual_fp16=True)
    emb = Encoder(es, weights=random_weights(es, 1, "test"))
    rer = Encoder(rs, weights=random_weights(rs, 2, "test"))
    rng = np.random.default_rng(0)
    N, B, K, k, S = 30001, 8, 20, 5, 48
    corpus = rng.standard_normal((N, 128)).astype(np.float32)
    p_tok = rng.integers(5, 2000, (N, 40)).astype(np.int32)
    p_len = rng.integers(1, 41, N).astype(np.int32)
    q_ids = rng.integers(5, 2000, (world * B, 16)).astype(np.int32)
    q_ids[:, 0] = 101
    q_tok = rng.integers(5, 2000, (world * B, 10)).astype(np.int32)
    q_len = rng.integers(1, 11, world * B).astype(np.int32)
    per = (N + world - 1) // world
    r0, r1 = (rank * per, min(N, (rank + 1) * per)) if sharded else (0, N)
    store = NativeStore(128)
    store.add(corpus[r0:r1])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    lex = None
    if hybrid:
        # BM25 over the shard's passage tokens (ids folded onto a small Zipf vocabulary so
        # documents share terms); corpus-wide statistics are all-reduced by the pipeline
        from super_rag_amd.lexical import NativeLexIndex
        lex = NativeLexIndex()
        lex.add([(p_tok[i, :p_len[i]] % 97 + 5).tolist() for i in range(r0, r1)])
        q_tok = q_tok % 97 + 5
    # shard_passages: this rank holds only its shard's passage rows; the C3 fetch brings the
    # candidates' rows from their owners
    pt, pl = (p_tok[r0:r1], p_len[r0:r1]) if shard_passages else (p_tok, p_len)
    pipe = SearchPipeline(emb, rer, store, t(pt), t(pl), k_candidates=K, k_final=k,
                          pair_len=S, shard_offset=r0, lexical=lex, k_each=16 if hybrid else None,
                          force_exchange=force_exchange, shard_passages=shard_passages)
    mine = slice(rank * B, (rank + 1) * B)
    res = pipe.run(t(q_ids[mine]), t(np.ones_like(q_ids[mine])), t(q_tok[mine]), t(q_len[mine]))
    torch.cuda.synchronize()
    return {f: getattr(res, f).cpu().numpy() for f in ("rows", "logits", "cand_rows", "cand_sims")}


def test_two_rank_sharded_pipeline_equals_single_process():
    # world-size-2 rehearsal of the multi-GPU path on one GPU: C1 all-gather of the query
    # embeddings, per-shard top-K with global row offsets, C2 all-to-all, K2 merge, rerank of the
    # rank's own queries == the single-process pipeline over the whole corpus.
    import os
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 200
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_both = dict(q.get(timeout=240) for _ in range(world))
    got = {r: v[0] for r, v in got_both.items()}
    got_h = {r: v[1] for r, v in got_both.items()}
    got_p = {r: v[2] for r, v in got_both.items()}
    got_hp = {r: v[3] for r, v in got_both.items()}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process: every rank's queries over the full corpus
    import torch.distributed as dist
    assert not dist.is_initialized()
    full = {r: _run_pipeline(r, world, sharded=False) for r in range(world)}
    full_h = {r: _run_pipeline(r, world, sharded=False, hybrid=True) for r in range(world)}
    for r in range(world):
        # hybrid: global BM25 statistics make the sharded fused candidates equal one index's
        np.testing.assert_array_equal(got_h[r]["cand_rows"], full_h[r]["cand_rows"])
        np.testing.assert_array_equal(got_h[r]["cand_sims"], full_h[r]["cand_sims"])
        np.testing.assert_array_equal(got_h[r]["rows"], full_h[r]["rows"])
    for r in range(world):
        np.testing.assert_array_equal(got[r]["cand_rows"], full[r]["cand_rows"])
        np.testing.assert_allclose(got[r]["cand_sims"], full[r]["cand_sims"], atol=1e-6)
        np.testing.assert_array_equal(got[r]["rows"], full[r]["rows"])
        np.testing.assert_allclose(got[r]["logits"], full[r]["logits"], atol=1e-5)
        # sharded passage tokens (C3 fetch) == the replicated table, bit for bit (dense and hybrid)
        for f in ("rows", "cand_rows", "cand_sims", "logits"):
            np.testing.assert_array_equal(got_p[r][f], got[r][f])
            np.testing.assert_array_equal(got_hp[r][f], got_h[r][f])


def test_bench_launches_its_own_ranks():
    """`python bench.py --gpus 2` (no torch.distributed.run) starts both ranks itself; gloo lets
    them share the box's one GPU.  The JSON line reports the world the backend formed."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--corpus-rows", "200000", "--batch", "32",
                        "--steps", "1", "--warmup", "1", "--batches", "1", "--no-cpu-baseline",
                        "--rerank-max-tokens", "65536"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 64
    assert "reports world_size 2" in r.stderr
