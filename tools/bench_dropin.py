"""Throughput of the DROP-IN per-request path on one GPU.

The reference serves one query per request: POST /collections/{id}/searches (api/collections.py:
272-279) -> CollectionService.execute_search_flow (service/collection_service.py:229-366):
vector_search -> merge -> rerank.  Here C concurrent closed-loop callers each run that flow through
this package's drop-in pieces exactly as the route would: super_rag_amd.flow.execute_search_flow
with the pack's runners (nodeflow_pack.py), the collection's EmbeddingService (embed_query
coalesced per encoder), ContextManager -> MI355XVectorStoreConnector.search (coalesced per
collection), RerankService.async_rerank (pairs of concurrent requests coalesced per cross-encoder),
12-layer bge-base-en embedder and bge-reranker-base cross-encoder (seeded synthetic weights, the
hashing tokenizer: SUPER_RAG_AMD_SYNTHETIC), vector_topk = 100 candidates reranked at S_pair <= 128.

Reported per concurrency: requests/s, mean coalesced batch per stage (items / device batches of
each Coalescer), the device time per stage (device_gate hold time: fraction of the run, ms per
device batch), p50 / p99 request latency.  The batched SearchPipeline number (bench.py's headline)
is the ceiling this path approaches as batches fill; the reference's own host orchestration costs
5.1 ms per query (profiles/r02_reference_orchestration.json) before any model work.

    python tools/bench_dropin.py [--rows 100000] [--concurrency 64 256] [--seconds 15]

From BULK_ROWS (1M) rows on, the collection is built by the bulk device path (build_collection_bulk:
rows generated on the GPU, texts pooled), so the drop-in path can be measured on config 4's 10M-row
corpus; bench.py hands its own headline store over instead of building a second one.
"""
from __future__ import annotations

import argparse
import asyncio
import concurrent.futures
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "super-rag_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

os.environ.setdefault("SUPER_RAG_AMD_SYNTHETIC", "1")

import numpy as np  # noqa: E402

WORDS = [f"w{i:04d}" for i in range(20000)]
EMBED_MODEL = "bge-base-en"
RERANK_MODEL = "bge-reranker-base"


def build_collection(col_id: str, rows: int, dim: int = 768, words_per_chunk: int = 90, seed: int = 0):
    """A collection of `rows` chunks through the connector's add (texts + clustered vectors)."""
    from super_rag_amd import nodeflow_pack as P
    from super_rag_amd.models import TextNode
    from super_rag_amd.vectorstore import VectorStoreConnectorAdaptor
    P.register()
    P.register_collection(P.LocalCollection(col_id, {"embedding": {"model": EMBED_MODEL}}))
    con = VectorStoreConnectorAdaptor("mi355x", {"collection": P.collection_name_for(col_id)}).connector
    con.create_collection(vector_size=dim)
    rng = np.random.default_rng(seed)
    centers = rng.standard_normal((256, dim)).astype(np.float32)
    step = 20000
    for a in range(0, rows, step):
        n = min(step, rows - a)
        v = centers[(np.arange(a, a + n)) % 256] + 0.5 * rng.standard_normal((n, dim)).astype(np.float32)
        w = rng.integers(0, len(WORDS), (n, words_per_chunk))
        nodes = [TextNode(text=" ".join(WORDS[j] for j in w[i]), metadata={"source": f"d{a + i}.md"},
                          embedding=v[i].tolist()) for i in range(n)]
        con.add(nodes)
    return con


TEXT_POOL = 100000      # distinct chunk texts of a bulk-built collection (row r: pool[r % TEXT_POOL])
BULK_ROWS = 1000000     # from this size on, run() builds the collection by the bulk device path


class PooledRows:
    """Read-only row -> value view for a bulk-built collection: row r holds pool[r % len(pool)]
    (10M rows with 100k distinct chunk texts / metadata records: a 10M-entry list of 500-byte
    strings would not fit the setup time)."""
    __slots__ = ("pool", "n", "fmt")

    def __init__(self, pool, n: int, fmt=None):
        self.pool, self.n, self.fmt = pool, int(n), fmt

    def __len__(self):
        return self.n

    def __getitem__(self, r):
        if isinstance(r, slice):
            return [self[i] for i in range(*r.indices(self.n))]
        r = int(r)
        if r < 0:
            r += self.n
        if not 0 <= r < self.n:
            raise IndexError(r)
        return self.fmt(r) if self.fmt is not None else self.pool[r % len(self.pool)]

    def __iter__(self):
        return (self[i] for i in range(self.n))


def build_collection_bulk(col_id: str, rows: int, dim: int = 768, words_per_chunk: int = 90,
                          seed: int = 0, store=None):
    """build_collection at any size, without the per-node host path: the clustered rows are
    generated on the GPU in 1M-row chunks and appended with NativeStore.add_dev, or an existing
    store is adopted (bench.py hands over the headline's 10M-row corpus, built once); texts and
    metadata are PooledRows over TEXT_POOL chunks.  Search results, the flow and the rerank are the
    connector's own; only ingest differs (not measured here).  Returns the connector."""
    import torch
    from super_rag_amd import nodeflow_pack as P
    from super_rag_amd import vectorstore as V
    P.register()
    P.register_collection(P.LocalCollection(col_id, {"embedding": {"model": EMBED_MODEL}}))
    con = V.VectorStoreConnectorAdaptor("mi355x", {"collection": P.collection_name_for(col_id)}).connector
    con.create_collection(vector_size=dim)
    c = V._collections[con.collection_name]
    if store is not None:
        own = c.store
        c.store = store
        if hasattr(own, "close"):
            own.close()
        rows = int(store.count()[0])
    else:
        dev = torch.device("cuda", c.device)
        g = torch.Generator(device=dev).manual_seed(seed)
        centers = torch.randn(256, dim, generator=g, device=dev)
        step = 1 << 20
        for a in range(0, rows, step):
            n = min(step, rows - a)
            v = centers[torch.arange(a, a + n, device=dev) % 256] + \
                0.5 * torch.randn(n, dim, generator=g, device=dev)
            c.store.add_dev(v.contiguous())
            del v
        torch.cuda.synchronize()
    rng = np.random.default_rng(seed)
    npool = min(TEXT_POOL, rows)
    w = rng.integers(0, len(WORDS), (npool, words_per_chunk))
    with c.lock:
        # (each row's text is distinct, as in a real corpus -- the merge node drops repeated texts
        # and the tokenizer cache would otherwise be warm on a 10M-row corpus: the pooled chunk
        # plus the row's own tag)
        pool = [" ".join(WORDS[j] for j in w[i]) for i in range(npool)]
        c.texts = PooledRows(pool, rows, fmt=lambda r: f"{pool[r % npool]} r{r}")
        c.metadatas = PooledRows([{"source": f"d{i}.md"} for i in range(npool)], rows)
        c.ids = PooledRows(None, rows, fmt=lambda r: f"bulk-{r}")
        c.row_of = {}
        c.version += 1
    return con


def release_collection(col_id: str) -> None:
    """Drop a bulk collection from the registry WITHOUT closing an adopted store (its owner, the
    bench's headline workload, still holds it)."""
    from super_rag_amd import nodeflow_pack as P
    from super_rag_amd import vectorstore as V
    with V._registry_lock:
        V._collections.pop(P.collection_name_for(col_id), None)


def _coalescers():
    """(name, Coalescer) of the embed / search / rerank stages, once they exist."""
    from super_rag_amd import registry
    from super_rag_amd import vectorstore as V
    out = {}
    for (name, _dir, _dev), (enc, _tok) in list(registry._models.items()):
        c = getattr(enc, "_query_coalescer", None)
        if c is not None:
            out["embed"] = c
        c = getattr(enc, "_encoded_pair_coalescer", None) or getattr(enc, "_pair_coalescer", None)
        if c is not None:
            out["rerank"] = c
    for col in list(V._collections.values()):
        if col.coalescer is not None:
            out["search"] = col.coalescer
        for co in list(getattr(col, "text_coalescers", {}).values()):
            out["embed_search"] = co
    return out


async def _closed_loop(n_callers: int, seconds: float, col_id: str, queries, lat: list):
    from super_rag_amd.flow import execute_search_flow
    t_end = time.perf_counter() + seconds
    done = [0]

    async def caller(i):
        j = i
        while time.perf_counter() < t_end:
            q = queries[j % len(queries)]
            j += n_callers
            t0 = time.perf_counter()
            items, _ = await execute_search_flow(q, col_id, "bench", vector_topk=100,
                                                 rerank_config=(RERANK_MODEL, "local", "mi355x"))
            lat.append(time.perf_counter() - t0)
            if len(items) != 100:
                raise RuntimeError(f"expected 100 reranked items, got {len(items)}")
            done[0] += 1
    await asyncio.gather(*[caller(i) for i in range(n_callers)])
    return done[0]


_PROFILES: list = []


def _profiled_worker_init():
    """(--profile) one cProfile.Profile per worker thread, merged at the end."""
    import cProfile
    pr = cProfile.Profile()
    _PROFILES.append(pr)
    pr.enable()


def measure(concurrency: int, seconds: float, col_id: str, queries, profile: bool = False,
            lat_out: str | None = None) -> dict:
    loop = asyncio.new_event_loop()
    # one worker thread per concurrent request for the blocking device calls (asyncio.to_thread):
    # the default executor's min(32, cpus + 4) threads would cap the coalesced batches at 32
    loop.set_default_executor(concurrent.futures.ThreadPoolExecutor(
        max_workers=concurrency + 8, initializer=_profiled_worker_init if profile else None))
    try:
        from super_rag_amd._native import gate_busy
        before = {k: (c.batches, c.items) for k, c in _coalescers().items()}
        busy0 = gate_busy()
        lat: list = []
        t0 = time.perf_counter()
        n = loop.run_until_complete(_closed_loop(concurrency, seconds, col_id, queries, lat))
        dt = time.perf_counter() - t0
        after = {k: (c.batches, c.items) for k, c in _coalescers().items()}
        busy1 = gate_busy()
    finally:
        loop.close()
    stages = {}
    for k, (b, i) in after.items():
        b0, i0 = before.get(k, (0, 0))
        if b > b0:
            stages[k] = {"batches": b - b0, "mean_batch": round((i - i0) / (b - b0), 2)}
    # device time by stage: the device_gate hold times (each stage's calls synchronise), as a
    # fraction of the run and per device batch
    for d, st in busy1.items():
        for k, (sec, holds) in st.items():
            s0, h0 = busy0.get(d, {}).get(k, (0.0, 0))
            if holds > h0:
                e = stages.setdefault(k, {})
                e["device_busy_frac"] = round((sec - s0) / dt, 3)
                e["device_ms_per_batch"] = round((sec - s0) / (holds - h0) * 1e3, 2)
    lat_ms = np.asarray(lat) * 1e3
    if lat_out:
        np.save(lat_out, lat_ms.astype(np.float32))
    return {"concurrency": concurrency, "requests": n, "seconds": round(dt, 2),
            "qps": round(n / dt, 1), "p50_ms": round(float(np.percentile(lat_ms, 50)), 1),
            "p99_ms": round(float(np.percentile(lat_ms, 99)), 1), "coalesced": stages}


def wait_for_go(path: str, timeout_s: float = 1800.0) -> float:
    """Block (no GPU touched) until `path` exists, then return the start time it holds: bench.py
    starts its serving processes before it initialises the GPU itself and releases them once its
    timed region is over (no exec from a process that has initialised the GPU)."""
    t_end = time.time() + timeout_s
    while not os.path.exists(path):
        if time.time() > t_end:
            raise SystemExit(f"bench_dropin: no go file {path} after {timeout_s:.0f} s")
        time.sleep(0.2)
    time.sleep(0.1)
    with open(path) as f:
        return float(json.load(f)["start_at"])


WINDOW_GAP_S = 4.0


def _windows(concurrency, seconds: float, start_at: float):
    """Yield (concurrency, seconds late) at each window's start: with a common start time
    (several serving processes on one GPU) window i starts at start_at + i (seconds +
    WINDOW_GAP_S) in every process, so the processes measure every window together; a process
    whose setup overran the start reports how late its window began."""
    for i, c in enumerate(concurrency):
        t = start_at + i * (seconds + WINDOW_GAP_S) if start_at > 0 else 0.0
        if t > time.time():
            time.sleep(t - time.time())
        yield c, (round(max(0.0, time.time() - t), 2) if start_at > 0 else 0.0)


def run(rows: int = 100000, concurrency=(64, 256), seconds: float = 15.0, warmup: int = 16,
        start_at: float = 0.0, lat_out: str | None = None, store=None) -> dict:
    """store: adopt this NativeStore as the collection's rows (bench.py: the headline's corpus)."""
    col_id = "dropin"
    t = time.time()
    bulk = store is not None or rows >= BULK_ROWS
    if bulk:
        build_collection_bulk(col_id, rows, store=store)
        if store is not None:
            rows = int(store.count()[0])
    else:
        build_collection(col_id, rows)
    setup = time.time() - t
    try:
        rng = np.random.default_rng(7)
        queries = [" ".join(WORDS[j] for j in rng.integers(0, len(WORDS), 24)) for _ in range(4096)]
        # warm up: models resident, kernels compiled, coalescers created
        measure(min(warmup, max(concurrency)), 3.0, col_id, queries)
        out = {"path": ("execute_search_flow (collection_service.py:229-366) -> pack vector_search / "
                        "merge / rerank runners -> EmbeddingService.embed_query + connector.search + "
                        "RerankService.async_rerank, coalesced; 12-layer bge-base-en + bge-reranker-base "
                        "(synthetic weights, hashing tokenizer); vector_topk 100, S_pair <= 128"),
               "rows": rows, "setup_s": round(setup, 1),
               "collection": ("bulk: rows on the device (NativeStore.add_dev or the headline's store), "
                              f"texts: one of {TEXT_POOL} pooled chunks + the row tag, distinct per row") if bulk else "connector add()",
               "runs": [dict(measure(c, seconds, col_id, queries,
                                     lat_out=(f"{lat_out}_c{c}.npy" if lat_out else None)), late_s=late)
                        for c, late in _windows(concurrency, seconds, start_at)],
               "reference_orchestration_ms_per_query": 5.14}
    finally:
        if store is not None:
            release_collection(col_id)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100000)
    ap.add_argument("--concurrency", type=int, nargs="+", default=[64, 256])
    ap.add_argument("--seconds", type=float, default=15.0)
    ap.add_argument("--start-at", type=float, default=0.0,
                    help="wall-clock time (time.time()) to start the measured runs at, after "
                         "setup and warmup: several processes serving from one GPU measure together")
    ap.add_argument("--go-file", default=None,
                    help="wait for this file (written by bench.py) before touching the GPU; it "
                         "holds the common start time of the measured runs")
    ap.add_argument("--lat-out", default=None,
                    help="save each run's request latencies (ms) to <lat-out>_c<C>.npy")
    ap.add_argument("--profile", action="store_true",
                    help="cProfile the event loop and every worker thread of one run at "
                         "--profile-concurrency (host time per request by function), printed after "
                         "the JSON line")
    ap.add_argument("--profile-concurrency", type=int, default=64,
                    help="1: no GIL contention, so the per-function times are the host CPU cost")
    a = ap.parse_args()
    if a.profile:
        import cProfile
        import pstats
        (build_collection_bulk if a.rows >= BULK_ROWS else build_collection)("dropin", a.rows)
        rng = np.random.default_rng(7)
        queries = [" ".join(WORDS[j] for j in rng.integers(0, len(WORDS), 24)) for _ in range(4096)]
        measure(16, 3.0, "dropin", queries)
        main_pr = cProfile.Profile()
        main_pr.enable()
        r = measure(a.profile_concurrency, a.seconds, "dropin", queries, profile=True)
        main_pr.disable()
        print(json.dumps(r), flush=True)
        for pr in _PROFILES:
            pr.disable()
        st = pstats.Stats(main_pr)
        for pr in _PROFILES:
            st.add(pr)
        st.sort_stats("tottime").print_stats(45)
        return
    start_at = wait_for_go(a.go_file) if a.go_file else a.start_at
    print(json.dumps(run(a.rows, a.concurrency, a.seconds, start_at=start_at, lat_out=a.lat_out)),
          flush=True)


if __name__ == "__main__":
    main()
