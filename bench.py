"""Benchmark of the embed -> exact top-K -> cross-encoder rerank hot path on MI355X.

BASELINE.json metric: "queries/sec (embed+ANN top-10+rerank) over 10M x 768-d @1/2/4/8 GPU;
recall@10".  One step = one batch of B synthetic queries per rank through the whole path:
  bge-base-en (768-d, 12L) query embed at S=32  ->  exact cosine top-100 over the 10M x 768 fp16
  corpus (row-sharded over the ranks)  ->  bge-reranker-base (XLM-R base) cross-encoder on the
  100 candidates per query at S_pair=128  ->  top-10.
Weights are seeded random (no checkpoints offline), inputs synthetic.

Launch: python bench.py [--gpus N --steps K --warmup W].  Under torch.distributed.run (WORLD_SIZE
set) every process is one rank on one GPU (RCCL); run directly with --gpus N > 1 the script
starts the N ranks itself through torch.distributed.run before anything touches the GPU, waits for
them and exits with the first non-zero rank status.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "super-rag_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_HBM_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_F16_TFLOPS = 2500.0    # dense fp16/bf16 MFMA spec (no sparsity)
PEAK_F8_TFLOPS = 5000.0     # dense fp8 MFMA spec (no sparsity)
# compute dtype of the line per reranker precision mode (bench --fp8)
FP8_DTYPES = {0: "f16", 1: "f16+fp8ffn", 2: "f16+fp8gemm", 3: "f16+fp8mlp", 5: "f16+fp8mlp+o"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without WORLD_SIZE the script launches them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--corpus-rows", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=256, help="queries per rank per step")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--k-cand", type=int, default=100)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--q-len", type=int, default=32)
    ap.add_argument("--pair-len", type=int, default=128)
    ap.add_argument("--passage-len", type=int, default=94)
    ap.add_argument("--embed-model", default="bge-base-en")
    ap.add_argument("--rerank-model", default="bge-reranker-base")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip recall@10 and the measured peaks (A/B timing runs only)")
    ap.add_argument("--rerank-max-tokens", type=int, default=1638400,
                    help="cross-encoder tokens per chunk (workspace ~15 KB per token; 1,638,400 = "
                         "2 chunks per step: +0.8 %% over 524,288, profiles/r02_ab_chunks.log)")
    ap.add_argument("--cpu-queries", type=int, default=32,
                    help="cpu_baseline: queries embedded (and at most this many reranked) on the host")
    ap.add_argument("--cpu-rerank-budget-s", type=float, default=20.0,
                    help="cpu_baseline: rerank whole queries (100 pairs each) until this many seconds "
                         "of host time are spent (at least one query; the per-query time is the "
                         "mean over the queries done, no extrapolation)")
    ap.add_argument("--cpu-search-rows", type=int, default=0,
                    help="cpu_baseline: corpus rows scanned by the host search (0 = the whole corpus)")
    ap.add_argument("--batches", type=int, default=4, help="distinct resident query batches")
    ap.add_argument("--dropin-seconds", type=float, default=8.0,
                    help="drop_in field: seconds per concurrency (64, 256) of the per-request path "
                         "(0 = skip)")
    ap.add_argument("--dropin-rows", type=int, default=10000000,
                    help="drop_in field: chunks in the connector collection it searches (default: "
                         "config 4's 10M; equal to the headline's corpus, the single-process run "
                         "adopts that store, and the serving processes bulk-build their own)")
    ap.add_argument("--dropin-procs", type=int, default=4,
                    help="drop_in field: also run this many serving processes on the GPU together "
                         "(started before this process touches the GPU, released after the timed "
                         "region; 0 / 1 = skip)")
    ap.add_argument("--dropin-mp-concurrency", default="32,64",
                    help="drop_in field: callers per serving process of the multi-process run, one "
                         "measured window each (all processes together)")
    ap.add_argument("--workload", default="config4", choices=["config4", "config5"],
                    help="config4 (default, the BASELINE metric) or config5: bge-m3 embed, 6.25M x "
                         "1024 rows per GPU scanned in fp8, BM25 over the passage tokens fused by "
                         "rrf (hybrid), rerank")
    ap.add_argument("--fp8-ffn", action="store_true",
                    help="reranker in the opt-in fp8 FFN precision mode (e4m3 FFN activations, "
                         "block-scaled fp8 MFMA for FFN2); reported with dtype f16+fp8ffn")
    ap.add_argument("--fp8", type=int, default=0, choices=(0, 1, 2, 3, 5),
                    help="reranker fp8 precision mode: 1 = --fp8-ffn (FFN2), 2 = also FFN1 and QKV "
                         "on e4m3 residual copies, 3 = FFN1 + FFN2 fp8 with QKV + attention fp16 "
                         "(dtype f16+fp8ffn / f16+fp8gemm / f16+fp8mlp); the rejected mode 5 (3 + "
                         "the O-projection on e4m3 ctx) only with SUPER_RAG_AMD_LIB=<libsrmi_diag.so>")
    ap.add_argument("--replicate-passages", action="store_true",
                    help="N > 1: keep the whole passage token table on every rank (default: each "
                         "rank holds its shard's rows, the candidates' rows are fetched per batch, "
                         "SearchPipeline shard_passages / C3)")
    ap.add_argument("--dist-backend", default=os.environ.get("SR_BENCH_BACKEND", "nccl"),
                    help="nccl (= RCCL, one rank per GPU) or gloo (rehearsal: ranks may share a GPU)")
    ap.add_argument("--config5-steps", type=int, default=5,
                    help="config5 field of the default (config4) line: timed steps of BASELINE "
                         "config 5 on its fp8 path (bge-m3 embed, 6.25M x 1024 rows per GPU "
                         "scanned in fp8, BM25 + rrf on the device, reranker in fp8 mode 3), run "
                         "after the headline with the config-4 objects freed (0 = skip)")
    ap.add_argument("--config5-warmup", type=int, default=2)
    ap.add_argument("--v2m3-steps", type=int, default=3,
                    help="v2m3 field of the default line: timed steps of the rerank stage alone with "
                         "bge-reranker-v2-m3 (the reranker the reference seeds; 24 layers, 1024-d) "
                         "in fp16 and in fp8 mode 3, after the config5 field (0 = skip)")
    a = ap.parse_args()
    if a.workload == "config5":
        as_config5(a)
        a.no_cpu_baseline = True
    return a


def as_config5(a):
    """BASELINE config 5 on one rank's share: bge-m3 (1024-d) embed, the 50M / 8-GPU shard size
    (6.25M rows) per rank scanned in fp8, BM25 over the passage tokens fused by rrf."""
    a.workload = "config5"
    a.embed_model, a.dim = "bge-m3", 1024
    if a.corpus_rows == 10_000_000:  # default: the 50M / 8-GPU shard size per GPU (weak)
        a.corpus_rows = 6_250_000 * int(os.environ.get("WORLD_SIZE", "1"))
    return a


def build_lexical(p_tok, p_len, device):
    """BM25 index of passage-token rows (device [n, L] int32, full length): each row's distinct
    tokens and counts are found on the GPU (sort + run starts), then handed to sr_lex_add."""
    from super_rag_amd.lexical import NativeLexIndex
    lex = NativeLexIndex(device=device)
    n, L = p_tok.shape
    step = 1 << 20
    for c0 in range(0, n, step):
        t, _ = torch.sort(p_tok[c0:c0 + step].long(), dim=1)
        new = torch.ones_like(t, dtype=torch.bool)
        new[:, 1:] = t[:, 1:] != t[:, :-1]
        flat = new.flatten()
        starts = torch.nonzero(flat).flatten()
        ends = torch.cat([starts[1:], torch.tensor([flat.numel()], device=t.device)])
        off = torch.zeros(t.shape[0] + 1, dtype=torch.int64, device=t.device)
        off[1:] = torch.cumsum(new.sum(1), 0)
        lex.add_arrays(off.cpu().numpy(), t.flatten()[flat].int().cpu().numpy(),
                       (ends - starts).int().cpu().numpy(), p_len[c0:c0 + step].cpu().numpy())
    return lex


def gen_corpus_chunk(r0, r1, dim, centers, dev):
    """Rows r0..r1 of the clustered synthetic corpus: x_i = c_{i mod 1024} + 0.5 eps_i, with eps
    drawn per 1M-row block from a generator seeded by the block index (shard-independent)."""
    out = torch.empty((r1 - r0, dim), dtype=torch.float32, device=dev)
    blk = 1 << 20
    r = r0
    while r < r1:
        b = r // blk
        b_end = min(r1, (b + 1) * blk)
        g = torch.Generator(device=dev)
        g.manual_seed(1_000_003 + b)
        eps = torch.randn(((b + 1) * blk - b * blk, dim), generator=g, device=dev)
        lo, hi = r - b * blk, b_end - b * blk
        idx = torch.arange(r, b_end, device=dev) % centers.shape[0]
        out[r - r0:b_end - r0] = centers[idx] + 0.5 * eps[lo:hi]
        r = b_end
    return out


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, script: str | None = None, env=None) -> int:
    """Start n ranks of `script` (default: this file) with torch.distributed.run on 127.0.0.1 and
    wait for them.  Called before any GPU call in this process (the parent never initialises HIP;
    the ranks are child processes, not an exec).  Returns 0 or the first failing rank's status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           script or os.path.abspath(__file__), *argv]
    print(f"[bench] launching {n} ranks: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and (a.gpus or 1) > 1:
        sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
    # the multi-process drop-in run's serving processes start NOW, before this process initialises
    # the GPU (they wait for a go file and touch nothing until then)
    mp = None
    if ("WORLD_SIZE" not in os.environ or os.environ.get("WORLD_SIZE") == "1") and not a.no_extras \
            and a.dropin_seconds > 0 and a.dropin_procs > 1 and a.workload == "config4":
        mp = DropinProcs(a.dropin_procs, a.dropin_rows, a.dropin_seconds,
                         concurrency=[int(c) for c in a.dropin_mp_concurrency.split(",")])
    try:
        run_bench(a, mp)
    finally:
        if mp is not None:
            mp.stop()


class DropinProcs:
    """N serving processes of the drop-in per-request path on this GPU (tools/bench_dropin.py, one
    collection, models and coalescers each), started as child processes before the bench
    initialises the GPU; release() lets them set up and measure together -- one window per
    callers-per-process value C, every process starting window i at the same wall-clock time --
    and collect() sums their throughput and pools their request latencies per window.
    Closed-loop callers obey Little's law: mean latency = callers / throughput, so N x C callers
    at X q/s wait N C / X on average whatever the batching policy (4 x 64 at ~420 q/s: ~610 ms)."""

    # The serving processes' configuration (a deployment of N serving processes sets it in their
    # environment): the rerank coalescer waits up to 30 ms for 24 queued requests when it finds
    # fewer.  With N processes sharing the GPU the wait costs no device time (the others fill it),
    # and larger rerank batches run more efficiently: 4 x 32 at 415.8 -> 428.9-430.2 q/s with
    # lower p50 (DESIGN, profiles/r06_fill/).  One process keeps the default (no wait).
    SERVING_ENV = {"SUPER_RAG_AMD_RERANK_MIN_FILL": "24", "SUPER_RAG_AMD_RERANK_MAX_WAIT_MS": "30"}

    def __init__(self, n, rows, seconds, concurrency=(32, 64), script=None):
        import tempfile
        self.dir = tempfile.mkdtemp(prefix="sr_dropin_")
        self.go = os.path.join(self.dir, "go.json")
        self.conc = list(concurrency)
        self.procs = []
        for i in range(n):
            cmd = [sys.executable, "-u", script or os.path.join(ROOT, "tools", "bench_dropin.py"),
                   "--rows", str(rows), "--concurrency", *map(str, self.conc),
                   "--seconds", str(seconds),
                   "--go-file", self.go, "--lat-out", os.path.join(self.dir, f"lat{i}")]
            out = open(os.path.join(self.dir, f"p{i}.json"), "w")
            err = open(os.path.join(self.dir, f"p{i}.err"), "w")
            env = {**os.environ, **self.SERVING_ENV}
            self.procs.append((subprocess.Popen(cmd, stdout=out, stderr=err, env=env), out, err))

    def release(self, delay_s=90.0):
        with open(self.go + ".tmp", "w") as f:
            json.dump({"start_at": time.time() + delay_s}, f)
        os.replace(self.go + ".tmp", self.go)

    def collect(self, timeout_s=300.0):
        runs, lats = [], []
        t_end = time.time() + timeout_s
        for i, (p, out, err) in enumerate(self.procs):
            try:
                rc = p.wait(timeout=max(1.0, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                rc = "timeout"
            out.close()
            err.close()
            if rc != 0:
                with open(err.name) as f:
                    tail = f.read()[-600:]
                return {"error": f"serving process {i} exited {rc}: {tail}"}
            with open(out.name) as f:
                runs.append(json.loads(f.read().strip().splitlines()[-1])["runs"])
            lats.append([np.load(os.path.join(self.dir, f"lat{i}_c{c}.npy")) for c in self.conc])
        windows = []
        for w, c in enumerate(self.conc):
            rw = [r[w] for r in runs]
            lat = np.concatenate([lt[w] for lt in lats])
            qps = sum(r["qps"] for r in rw)
            windows.append({
                "concurrency_per_proc": c, "callers": c * len(rw), "qps": round(qps, 1),
                "per_proc_qps": [r["qps"] for r in rw],
                "per_proc_late_s": [r.get("late_s", 0.0) for r in rw],
                "p50_ms": round(float(np.percentile(lat, 50)), 1),
                "p99_ms": round(float(np.percentile(lat, 99)), 1),
                "mean_ms": round(float(lat.mean()), 1),
                "littles_law_mean_ms": round(c * len(rw) / qps * 1e3, 1) if qps else None,
                "requests": int(sum(r["requests"] for r in rw)),
                "seconds": max(r["seconds"] for r in rw),
                "rerank_mean_batch": [r["coalesced"].get("rerank", {}).get("mean_batch") for r in rw]})
        return {"procs": len(runs), "windows": windows, "serving_env": dict(self.SERVING_ENV),
                "note": "closed-loop callers: mean latency = callers / q/s (Little's law)"}

    def stop(self):
        for p, out, err in self.procs:
            if p.poll() is None:
                p.kill()
                p.wait()
            out.close()
            err.close()
        import shutil
        shutil.rmtree(self.dir, ignore_errors=True)


def run_bench(a, mp=None):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus is not None and a.gpus != world:
        sys.exit(f"bench: --gpus {a.gpus} but the launcher started {world} rank(s)")
    if a.dist_backend == "gloo":  # rehearsal mode: ranks may share the visible GPUs
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import torch.distributed as dist
    if world > 1:
        if a.dist_backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        ver = torch.cuda.nccl.version() if a.dist_backend != "gloo" else None
        print(f"[bench] rank {rank}/{world}: backend {dist.get_backend()} reports world_size "
              f"{dist.get_world_size()}" + (f", RCCL {ver}" if ver else "") + f", device {dev}",
              file=sys.stderr, flush=True)
        if dist.get_world_size() != world:
            sys.exit(f"bench: backend world_size {dist.get_world_size()} != WORLD_SIZE {world}")

    comm = comm_record(dist, world, a.dist_backend)

    from super_rag_amd import _native as N

    W = setup_workload(a, world, rank, local, dev)
    es, rs, w_embed, w_rerank = W.es, W.rs, W.w_embed, W.w_rerank
    embedder, reranker, store, centers = W.embedder, W.reranker, W.store, W.centers
    p_tok, batches, pipe = W.p_tok, W.batches, W.pipe
    N_total, r0, r1, shard_p, setup_s, step_rows = W.N_total, W.r0, W.r1, W.shard_p, W.setup_s, W.step_rows
    dt, prof = timed_steps(W, a, world, dev, dist)
    queries = world * a.batch * a.steps
    value = queries / dt
    stage_ms = dict(W.stage_ms, note=("HIP events on the launch stream at the stage boundaries "
                                      "of every timed step, ms per step (max over ranks); exchange "
                                      "= C1 query all_gather + C2 list all_to_all + C3 passage "
                                      "fetch (+ the BM25 statistics all_reduce in hybrid mode)"))

    # ---- recall@10 of the search stage vs exact fp32 (outside the timed region) -----------------
    recall = search_recall(W, a, dev) if world == 1 and not a.no_extras else None

    peaks = None
    if rank == 0 and not a.no_extras:
        try:  # (the diagnostic library: reported, never a reason to lose the product's line)
            peaks = measured_peaks(dev)
        except Exception as e:  # noqa: BLE001
            peaks = {"error": f"{type(e).__name__}: {e}"[:300]}

    # ---- search-only at B = 32 (config 2's query block) on this rank's shard: fp16 and fp8 -----
    search32 = None
    if rank == 0 and not a.no_extras and a.workload == "config4":
        search32 = search_b32(store, centers, N_total, r0, r1, a.dim, dev)

    # ---- fp8 precision modes: final top-10 vs the fp16 reranker on the same candidates -----------
    fp8_fidelity = None
    if a.fp8 and world == 1:
        r8 = pipe.run(*batches[0])
        reranker.set_fp8(0)
        r16 = pipe.run(*batches[0])
        reranker.set_fp8(a.fp8)
        f8, f16 = r8.rows.cpu(), r16.rows.cpu()
        overlap = sum(len(set(f8[i].tolist()) & set(f16[i].tolist())) for i in range(f8.shape[0]))
        l16 = r16.logits.float().cpu()
        fp8_fidelity = {"top10_overlap_vs_f16": round(overlap / f8.numel(), 4),
                        "top1_equal_vs_f16": round(float((f8[:, 0] == f16[:, 0]).float().mean()), 4),
                        "final_logit_std_f16": round(float(l16.std()), 5),
                        "queries": int(f8.shape[0])}

    # ---- ranking fidelity on a discriminative reranker (outside the timed region) ---------------
    fidelity = None
    if rank == 0 and not a.no_extras:
        fidelity = rerank_fidelity(rs, local)

    # ---- the drop-in per-request path (not the headline): concurrent callers through the pack's
    # runners, coalesced embed / search / rerank, one query per request (tools/bench_dropin.py) ----
    drop_in = None
    if rank == 0 and world == 1 and not a.no_extras and a.dropin_seconds > 0:
        from tools.bench_dropin import run as dropin_run
        # (the headline's own corpus when the sizes agree: built once, as VERDICT r5 item 4 asks)
        try:
            drop_in = dropin_run(rows=a.dropin_rows, concurrency=(64, 256), seconds=a.dropin_seconds,
                                 store=W.store if a.dropin_rows == N_total and world == 1 else None)
        except Exception as e:  # noqa: BLE001 - the headline line must survive a drop-in failure
            import traceback
            traceback.print_exc()
            drop_in = {"error": f"{type(e).__name__}: {e}"}
        drop_in["pipeline_qps_same_box"] = round(value, 2)
        if mp is not None:
            # N serving processes on this GPU, C callers each (one window per C), measured
            # together (this process idle meanwhile): the per-process host cost (~5 ms of Python
            # per request) spread over N interpreters
            mp.release()
            drop_in["multi_process"] = mp.collect()

    # ---- roofline of the dominant kernel -------------------------------------------------------
    wl = "config5" if a.workload == "config5" and a.fp8 == 3 else None
    roof = add_held_peak(dominant_roofline(prof, wl), peaks)
    step_ms = dt / a.steps * 1e3
    kern = kernel_table(prof, a.steps, top=12)
    search_roof = scan_roofline(prof, wl)

    # ---- CPU baseline: the oracle on a bounded sample (rank 0, N=1) ----------------------------
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a, es, rs, w_embed, w_rerank, centers, batches[0], p_tok, N_total,
                           embedder, dev)

    # ---- BASELINE config 5 on its fp8 path: its own timed steps after the
    # headline, with the config-4 objects freed first --------------------------------------------
    config5 = None
    if a.workload == "config4" and not a.no_extras and a.config5_steps > 0:
        del embedder, reranker, store, p_tok, batches, pipe
        free_workload(W)
        config5 = config5_field(a, world, rank, local, dev, dist,
                                (fidelity or {}).get("fp8_mode3"))
        if config5:
            add_held_peak(config5.get("roofline"), peaks)

    # ---- the reference's seeded reranker (bge-reranker-v2-m3) on the rerank stage alone ---------
    v2m3 = None
    if a.workload == "config4" and not a.no_extras and a.v2m3_steps > 0 and rank == 0:
        v2m3 = v2m3_field(a, local, dev)

    workload = ("config4: bge-base-en embed (S=32) + exact cosine top-100 over "
                f"{N_total} x {a.dim} fp16 corpus (row-sharded) + bge-reranker-base "
                f"rerank of 100 pairs (S={a.pair_len}) -> top-{a.k}")
    metric = "queries/sec (embed+ANN top-10+rerank) over 10M x 768-d; recall@10"
    if a.workload == "config5":
        workload = (f"config5: bge-m3 embed (S={a.q_len}) + fp8 cosine top-{a.k_cand} over "
                    f"{N_total} x {a.dim} rows (row-sharded, fp16 re-scored) + BM25 top-{a.k_cand} "
                    f"over the passage tokens, rrf-fused on the device + {a.rerank_model} rerank of "
                    f"{a.k_cand} pairs (S={a.pair_len}) -> top-{a.k}")
        metric = "queries/sec (config 5: bge-m3 embed + hybrid fp8-dense/BM25 retrieval + rerank)"
    line = {
        "metric": metric,
        "value": round(value, 2), "unit": "queries/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": FP8_DTYPES[a.fp8],
        "data": "synthetic",
        "config": {"workload": workload,
                   "queries_per_rank": a.batch, "global_batch": world * a.batch,
                   "corpus_rows": N_total, "rows_per_rank": r1 - r0, "weights": "seeded random",
                   "parallelism": f"corpus row-shard x{world}, query DP x{world}",
                   "passages": "sharded (C3 fetch)" if shard_p else "replicated",
                   "comm": comm},
        "recall_at_10": recall,
        **({"rerank_fp8_fidelity": fp8_fidelity} if fp8_fidelity else {}),
        "rerank_fidelity": fidelity,
        "drop_in": drop_in,
        "roofline": roof,
        "search_roofline": search_roof,
        "search_b32": search32,
        "measured_peaks": peaks,
        "cpu_baseline": cpu,
        "config5": config5,
        "v2m3": v2m3,
        "kernels": kern,
        "setup_s": round(setup_s, 1),
        "stage_ms": stage_ms,
    }
    # LAST: a compact summary, so a reader of the line's tail (the driver keeps the end of
    # stdout) sees the headline, recall, fidelity verdicts, drop-in latency and the extra fields
    line["summary"] = summary(line)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def summary(line):
    """The line's key results in a few hundred bytes (printed last in the JSON line)."""
    def fid(f):
        if not f:
            return None
        return {m: f"{v['top10_identical_mod_ties']} top-10 identical, std/err {v['min_std_over_err']}"
                for m, v in f.items() if isinstance(v, dict) and "top10_identical_mod_ties" in v}

    def drop(d):
        if not d or "runs" not in d:
            return None
        r64 = next((r for r in d["runs"] if r.get("concurrency") == 64), d["runs"][0])
        out = {"c64_qps": r64.get("qps"), "c64_p50_ms": r64.get("p50_ms"), "c64_p99_ms": r64.get("p99_ms")}
        mp = d.get("multi_process")
        if mp and "windows" in mp:
            out["multi_process"] = {f"{mp['procs']}x{w['concurrency_per_proc']}":
                                    {"qps": w["qps"], "p50_ms": w["p50_ms"], "p99_ms": w["p99_ms"]}
                                    for w in mp["windows"]}
        return out

    c5, v2 = line.get("config5"), line.get("v2m3")
    roof = line.get("roofline") or {}
    return {
        "value": line["value"], "unit": line["unit"], "n_gpus": line["n_gpus"],
        "ms_per_step": line["ms_per_step"], "recall_at_10": line.get("recall_at_10"),
        "stage_ms": {k: v for k, v in (line.get("stage_ms") or {}).items() if k != "note"},
        "dominant_kernel": roof.get("kernel"), "roofline_frac": roof.get("frac"),
        "roofline_frac_of_held_peak": roof.get("frac_of_held_peak"),
        "rerank_fidelity": fid(line.get("rerank_fidelity")),
        "drop_in": drop(line.get("drop_in")),
        "config5": {"value": c5["value"], "ms_per_step": c5["ms_per_step"],
                    "recall_at_10": c5.get("recall_at_10")} if c5 else None,
        "v2m3": {k: v2.get(k) for k in ("fp16_qps", "fp8_mode3_qps", "fidelity")} if v2 else None,
    }


def v2m3_field(a, local, dev, fidelity=True):
    """bge-reranker-v2-m3 -- the reranker the reference seeds (migration/sql/model_configs_init.sql:
    4148; XLM-R large: 24 layers, 1024-d, 16 heads, FFN 4096) -- on the rerank stage alone at the
    bench shape: a.batch queries x a.k_cand candidates (S_pair = a.pair_len) per step, the pairs
    packed on the device from a 1M-row synthetic passage table (SearchPipeline.rerank: pair
    packing, cross-encoder, top-k select), seeded random weights; timed in fp16 and in fp8 mode 3
    (a.v2m3_steps steps each after one warmup), plus its ranking fidelity on the relevance-structured
    24-layer set (tests/golden/rerank_fidelity_v2m3.npz) in both precisions."""
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    from super_rag_amd.pipeline import SearchPipeline
    from super_rag_amd import _native as N
    rs = MODELS["bge-reranker-v2-m3"]
    w = random_weights(rs, seed=13, style="hf")
    rer = Encoder(rs, device=local, weights=w, max_tokens=a.rerank_max_tokens)
    del w
    out = {"model": "bge-reranker-v2-m3 (24 layers, 1024-d; seeded random weights)",
           "workload": (f"rerank stage alone: {a.batch} queries x {a.k_cand} candidates, S_pair="
                        f"{a.pair_len}, -> top-{a.k} (device pair packing + cross-encoder + select)"),
           "steps": a.v2m3_steps, "warmup": 1}
    try:
        g = torch.Generator(device=dev)
        g.manual_seed(17)
        n_p = 1 << 20
        p_tok = torch.randint(1000, rs.vocab_size, (n_p, a.passage_len), generator=g, device=dev,
                              dtype=torch.int32)
        p_len = torch.full((n_p,), a.passage_len, dtype=torch.int32, device=dev)
        lq = a.q_len - 2
        qtok = torch.randint(1000, rs.vocab_size, (a.batch, lq), generator=g, device=dev, dtype=torch.int32)
        qlen = torch.full((a.batch,), lq, dtype=torch.int32, device=dev)
        cand = torch.randint(0, n_p, (a.batch, a.k_cand), generator=g, device=dev, dtype=torch.int64)
        pipe = SearchPipeline(None, rer, None, p_tok, p_len, k_candidates=a.k_cand, k_final=a.k,
                              pair_len=a.pair_len)
        for mode, name in ((0, "fp16"), (3, "fp8_mode3")):
            rer.set_fp8(mode)
            pipe.rerank(qtok, qlen, cand)
            torch.cuda.synchronize()
            N.profile_enable(True)
            t0 = time.perf_counter()
            for _ in range(a.v2m3_steps):
                pipe.rerank(qtok, qlen, cand)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            N.profile_enable(False)
            prof = N.profile_read()
            out[f"{name}_qps"] = round(a.batch * a.v2m3_steps / dt, 2)
            out[f"{name}_ms_per_step"] = round(dt / a.v2m3_steps * 1e3, 2)
            out[f"{name}_roofline"] = {k: v for k, v in dominant_roofline(prof).items()
                                       if k in ("kernel", "achieved", "peak", "unit", "frac")}
        rer.set_fp8(0)
    finally:
        rer.close()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    if not fidelity:
        return out
    fid = rerank_fidelity(rs, local, modes=((0, "fp16"), (3, "fp8_mode3")))
    out["fidelity"] = ({m: f"{v['top10_identical_mod_ties']} top-10 identical, std/err "
                           f"{v['min_std_over_err']}" for m, v in fid.items() if isinstance(v, dict)}
                       if fid else None)
    out["fidelity_detail"] = fid
    return out


def setup_workload(a, world, rank, local, dev):
    """Everything one step needs, resident on this rank's GPU: the embedder and reranker (seeded
    random weights of the named shapes), this rank's corpus rows (and the fp8 scan copy and the
    BM25 index of the passage tokens for config 5), the passage token table, a.batches resident
    query batches and the SearchPipeline over them.  Returns a namespace; free_workload() releases
    the device memory."""
    from types import SimpleNamespace
    from super_rag_amd.encoder import MODELS, Encoder, random_weights
    from super_rag_amd.pipeline import SearchPipeline
    from super_rag_amd.store import NativeStore

    t_setup = time.time()
    es, rs = MODELS[a.embed_model], MODELS[a.rerank_model]
    assert es.hidden == a.dim
    w_embed = random_weights(es, seed=11, style="hf")
    w_rerank = random_weights(rs, seed=12, style="hf")
    embedder = Encoder(es, device=local, weights=w_embed, max_tokens=a.batch * a.q_len)
    reranker = Encoder(rs, device=local, weights=w_rerank, max_tokens=a.rerank_max_tokens)
    if a.fp8_ffn:
        a.fp8 = max(a.fp8, 1)
    if a.fp8:
        reranker.set_fp8(a.fp8)

    # ---- corpus shard (rows [r0, r1) of the global corpus) -------------------------------------
    N_total = a.corpus_rows
    per = (N_total + world - 1) // world
    r0, r1 = rank * per, min(N_total, (rank + 1) * per)
    gc = torch.Generator(device="cpu")
    gc.manual_seed(0)
    centers = torch.randn((1024, a.dim), generator=gc).to(dev)
    store = NativeStore(a.dim, device=local, capacity=r1 - r0)
    step_rows = 1 << 20
    for c0 in range(r0, r1, step_rows):
        chunk = gen_corpus_chunk(c0, min(r1, c0 + step_rows), a.dim, centers, dev)
        store.add_dev(chunk)
        del chunk
    torch.cuda.synchronize()
    if a.workload == "config5":
        store.set_scan_dtype("fp8")   # config 5: the fp8 MFMA scan (exact fp16 re-scoring)
    # passage token table for the cross-encoder (content tokens, no specials), generated whole so
    # every world size sees the same tokens; at N > 1 each rank keeps only its shard's rows
    gp = torch.Generator(device=dev)
    gp.manual_seed(5)
    p_tok = torch.randint(1000, rs.vocab_size, (N_total, a.passage_len), generator=gp, device=dev,
                          dtype=torch.int32)
    p_len = torch.full((N_total,), a.passage_len, dtype=torch.int32, device=dev)

    # ---- resident synthetic query batches ------------------------------------------------------
    gq = torch.Generator(device=dev)
    gq.manual_seed(2 + rank)
    batches = []
    for _ in range(a.batches):
        ids = torch.randint(1000, es.vocab_size, (a.batch, a.q_len), generator=gq, device=dev,
                            dtype=torch.int32)
        ids[:, 0] = es.bos_id
        ids[:, -1] = es.eos_id
        mask = torch.ones_like(ids)
        lq = a.q_len - 2
        qtok = torch.randint(1000, rs.vocab_size, (a.batch, lq), generator=gq, device=dev,
                             dtype=torch.int32)
        qlen = torch.full((a.batch,), lq, dtype=torch.int32, device=dev)
        batches.append((ids, mask, qtok, qlen))
    lexical = build_lexical(p_tok[r0:r1], p_len[r0:r1], local) if a.workload == "config5" else None
    shard_p = world > 1 and not a.replicate_passages
    if shard_p:
        p_tok, p_len = p_tok[r0:r1].clone(), p_len[r0:r1].clone()
        torch.cuda.empty_cache()
    pipe = SearchPipeline(embedder, reranker, store, p_tok, p_len, k_candidates=a.k_cand,
                          k_final=a.k, pair_len=a.pair_len, shard_offset=r0, lexical=lexical,
                          k_each=a.k_cand, shard_passages=shard_p)
    torch.cuda.synchronize()
    return SimpleNamespace(es=es, rs=rs, w_embed=w_embed, w_rerank=w_rerank, embedder=embedder,
                           reranker=reranker, store=store, centers=centers, p_tok=p_tok,
                           p_len=p_len, batches=batches, lexical=lexical, pipe=pipe,
                           N_total=N_total, r0=r0, r1=r1, shard_p=shard_p, step_rows=step_rows,
                           setup_s=time.time() - t_setup)


def search_recall(W, a, dev, nq=32):
    """recall@10 of the search stage (the store's top-k: fp16 K1, or for config 5 the fp8 scan
    re-scored in fp16) for nq queries of batch 0 vs the exact fp32 top-k over the unquantised
    rows (regenerated on the device chunk by chunk)."""
    ids, mask, _, _ = W.batches[0]
    nq = min(nq, a.batch)
    q16 = W.embedder.embed_dev(ids[:nq], mask[:nq], fp16=False)
    _, rows = W.store.search_dev(q16, a.k)
    best_s = torch.full((nq, 0), -2.0, device=dev)
    best_r = torch.zeros((nq, 0), dtype=torch.int64, device=dev)
    for c0 in range(0, W.N_total, W.step_rows):
        x = gen_corpus_chunk(c0, min(W.N_total, c0 + W.step_rows), a.dim, W.centers, dev)
        s = q16 @ torch.nn.functional.normalize(x, dim=1).T
        best_s = torch.cat([best_s, s], 1)
        best_r = torch.cat([best_r, torch.arange(c0, c0 + x.shape[0], device=dev).expand(nq, -1)], 1)
        top = best_s.topk(a.k, dim=1)
        best_s, best_r = top.values, best_r.gather(1, top.indices)
    hit = sum(len(set(rows[i].tolist()) & set(best_r[i].tolist())) for i in range(nq))
    return hit / (nq * a.k)


def dominant_roofline(prof, workload=None):
    """Roofline record of the kernel with the largest total time: ALGORITHMIC flops (or bytes)
    of its launches / their summed HIP-event durations against the spec peak (5 PF/s for the fp8
    GEMMs, 2.5 PF/s f16, 8 TB/s HBM), with the PMC traffic of the committed summary."""
    dom_name, dom = max(prof.items(), key=lambda kv: kv[1]["total_ms"])
    avg_ms = dom["total_ms"] / dom["launches"]
    if dom["flops"] > 0 and not dom_name.startswith("cosine_scan"):
        achieved = dom["flops"] / (dom["total_ms"] * 1e-3) / 1e12
        peak = PEAK_F8_TFLOPS if dom_name.startswith("gemm_f8") else PEAK_F16_TFLOPS
        roof = {"bound": "mfma", "achieved": round(achieved, 1), "peak": peak,
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None}
    else:
        achieved = dom["bytes"] / (dom["total_ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": None}
    roof.update({"kernel": dom_name, "launches": dom["launches"], "avg_ms": round(avg_ms, 4),
                 "per_launch": (f"{dom['flops'] / dom['launches']:.4g} FLOP" if roof["bound"] == "mfma"
                                else f"{dom['bytes'] / dom['launches']:.4g} B"),
                 "algorithmic_B_per_launch": round(dom["bytes"] / dom["launches"])})
    return apply_pmc(roof, dom_name, prof.keys(), workload=workload)


def kernel_table(prof, steps, top=None):
    """Per logical kernel: ms per step, launches, and its rate (TF/s against its flops, or GB/s of
    algorithmic bytes for the memory kernels); fp8 GEMMs also as a fraction of the 5 PF/s peak.
    top: only the `top` kernels by time (the rest summed into "(others)")."""
    out = {}
    items = sorted(prof.items(), key=lambda kv: -kv[1]["total_ms"])
    rest = items[top:] if top else []
    for k, v in items[:top] if top else items:
        rate = (v["flops"] / 1e12 if v["flops"] > 0 else v["bytes"] / 1e9) / (v["total_ms"] * 1e-3)
        e = {"ms_per_step": round(v["total_ms"] / steps, 3), "launches": v["launches"],
             ("tflops" if v["flops"] > 0 else "gbs"): round(rate, 1)}
        if v["flops"] > 0 and (k.startswith("gemm_f8") or k.startswith("cosine_scan8")):
            e["frac_of_fp8_peak"] = round(rate / PEAK_F8_TFLOPS, 4)
        out[k] = e
    if rest:
        out["(others)"] = {"kernels": len(rest),
                           "ms_per_step": round(sum(v["total_ms"] for _, v in rest) / steps, 3)}
    return out


def scan_roofline(prof, workload=None):
    """K1 (cosine_scan*) against HBM: the scans' algorithmic bytes / their time, and the ceiling
    max(bytes / 8 TB/s, flop / MFMA peak) (at B = 256 the scan sits at the ridge)."""
    scan = {k: v for k, v in prof.items() if k.startswith("cosine_scan")}
    if not scan:
        return None
    sb = sum(v["bytes"] for v in scan.values())
    sm = sum(v["total_ms"] for v in scan.values())
    search_roof = {"bound": "hbm", "achieved": round(sb / (sm * 1e-3) / 1e9, 1),
                   "peak": PEAK_HBM_GBS, "unit": "GB/s",
                   "frac": round(sb / (sm * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}
    apply_pmc(search_roof, "cosine_scan8" if "cosine_scan8" in scan else "cosine_scan", prof.keys(),
              workload=workload)
    search_roof.pop("pmc_provenance", None)  # (the same record as roofline's)
    mfma_s = sum(v["flops"] / ((PEAK_F8_TFLOPS if k.startswith("cosine_scan8") else PEAK_F16_TFLOPS) * 1e12)
                 for k, v in scan.items())
    ceil_ms = max(sb / (PEAK_HBM_GBS * 1e9), mfma_s) * 1e3
    search_roof["ceiling"] = {"ms": round(ceil_ms, 3), "achieved_ms": round(sm, 3),
                              "frac": round(ceil_ms / sm, 4),
                              "note": "max(bytes / 8 TB/s, flop / MFMA peak (2.5 PF/s f16, 5 PF/s fp8)) over the timed steps"}
    return search_roof


def config5_field(a, world, rank, local, dev, dist, mode3_fidelity):
    """BASELINE config 5 on its fp8 path, beside the config-4 headline: bge-m3
    embed (24 layers, 1024-d, S = q_len), this rank's 6.25M x 1024 rows of the 50M corpus scanned
    in fp8 (block-scaled MFMA, exact fp16 re-scoring), BM25 top-100 over the passage tokens and
    rrf fusion on the device, bge-reranker-base in fp8 mode 3 (FFN1 + FFN2 on the fp8 MFMA), top-10.
    Its own warmup / timed steps (max over ranks), kernels, roofline (fp8 GEMMs against 5 PF/s),
    recall@10 of the dense stage, and mode 3's ranking fidelity on the discriminative set."""
    a5 = config5_args(a)
    W = setup_workload(a5, world, rank, local, dev)
    try:
        dt, prof = timed_steps(W, a5, world, dev, dist)
        stage_ms5 = W.stage_ms
        recall = search_recall(W, a5, dev) if world == 1 else None
    finally:
        setup_s = W.setup_s
        free_workload(W)
    value = world * a5.batch * a5.steps / dt
    return {
        "metric": "queries/sec (config 5: bge-m3 embed + hybrid fp8-dense/BM25 retrieval + rerank)",
        "value": round(value, 2), "unit": "queries/s", "n_gpus": world, "steps": a5.steps,
        "warmup": a5.warmup, "ms_per_step": round(dt / a5.steps * 1e3, 3),
        "dtype": "f16+fp8mlp",
        "workload": (f"config5: bge-m3 embed (S={a5.q_len}) + fp8 cosine top-{a5.k_cand} over "
                     f"{a5.corpus_rows} x {a5.dim} rows (row-sharded, fp16 re-scored) + BM25 "
                     f"top-{a5.k_cand} over the passage tokens, rrf-fused on the device + "
                     f"{a5.rerank_model} rerank in fp8 mode 3 (FFN1 + FFN2 block-scaled fp8 MFMA, "
                     f"QKV + attention fp16) of {a5.k_cand} pairs (S={a5.pair_len}) -> top-{a5.k}"),
        "corpus_rows": a5.corpus_rows, "rows_per_rank": shard_rows(a5.corpus_rows, world, rank),
        "recall_at_10": recall,
        "rerank_fp8_mode3_fidelity": mode3_fidelity,
        "stage_ms": stage_ms5,
        "roofline": dominant_roofline(prof, "config5"),
        "search_roofline": scan_roofline(prof, "config5"),
        "kernels": kernel_table(prof, a5.steps, top=10),
        "setup_s": round(setup_s, 1),
    }


def config5_args(a):
    """The config-5 field's arguments from the headline's: config 5's models and shard size, the
    reranker in fp8 mode 3, the field's own step counts."""
    import copy
    a5 = as_config5(copy.copy(a))
    if a.corpus_rows != 10_000_000:   # a smaller corpus asked for: scale the config-5 shard alike
        a5.corpus_rows = a.corpus_rows
    a5.fp8, a5.fp8_ffn = 3, False
    a5.steps, a5.warmup = a.config5_steps, a.config5_warmup
    return a5


def shard_rows(n_total, world, rank):
    per = (n_total + world - 1) // world
    return min(n_total, (rank + 1) * per) - rank * per


def free_workload(W):
    """Release a workload's device memory (encoder workspaces, corpus, BM25 index, tokens)."""
    for obj in (W.embedder, W.reranker, W.store, W.lexical):
        if obj is not None:
            obj.close()
    for k in list(vars(W)):
        setattr(W, k, None)
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def timed_steps(W, a, world, dev, dist):
    """a.warmup untimed steps, then EXACTLY a.steps steps bracketed by a barrier and a device
    synchronisation on both sides; the library's HIP-event profile of the timed region; the time
    is the max over ranks.  Returns (seconds, per-kernel profile)."""
    from super_rag_amd import _native as N
    from super_rag_amd.pipeline import StageClock
    for i in range(a.warmup):
        W.pipe.run(*W.batches[i % a.batches])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    W.pipe.clock = StageClock()   # HIP events at the stage boundaries of every timed step
    N.profile_enable(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(a.steps):
        W.pipe.run(*W.batches[i % a.batches])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    N.profile_enable(False)
    prof = N.profile_read()
    W.stage_ms = W.pipe.clock.read()
    W.pipe.clock = None
    if world > 1:
        t = torch.tensor([dt], device=dev if a.dist_backend != "gloo" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        # per-stage ms per step: the max over ranks of each stage (the exchange waits for the
        # slowest rank, so its max is the critical one)
        # (the stages, then the exchange's per-collective keys exchange_c1 / _c2 /
        # _bm25_allreduce / _c3)
        keys = list(W.stage_ms)
        st = torch.tensor([W.stage_ms[k] for k in keys], dtype=torch.float64,
                          device=dev if a.dist_backend != "gloo" else "cpu")
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        W.stage_ms = {k: round(float(v), 4) for k, v in zip(keys, st.tolist())}
    return dt, prof


def comm_record(dist, world, backend):
    """The communicator as the ranks see it (config.comm of the JSON line): the process group's
    backend and world size as torch.distributed reports them (None / 1 without a group at N = 1)
    and the RCCL version torch links (torch.cuda.nccl.version(): RCCL on ROCm)."""
    try:
        ver = torch.cuda.nccl.version()
        rccl = ".".join(str(x) for x in ver) if isinstance(ver, tuple) else str(ver)
    except Exception as e:  # noqa: BLE001 - reported, not fatal
        rccl = f"unavailable ({type(e).__name__})"
    init = dist.is_available() and dist.is_initialized()
    return {"backend": dist.get_backend() if init else None,
            "world_size": dist.get_world_size() if init else 1,
            "launched_world_size": world, "requested_backend": backend if world > 1 else None,
            "rccl_version": rccl}


def search_b32(store, centers, n_total, r0, r1, dim, dev, reps=10):
    """K1 + K2 alone for a block of 32 search-only queries (corpus rows + 0.3 noise, seed 3; SURVEY
    section 8(d)) over this rank's rows: the config-2 query block, HBM-bound.  Reported per scan
    dtype with the scan kernels' algorithmic HBM rate (rows x row bytes per query block) against
    the 8 TB/s spec; the fp8 scan reads e4m3 rows (1 B per element) and re-scores exactly in fp16."""
    from super_rag_amd import _native as N
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    idx = torch.randint(r0, r1, (32,), generator=g, device=dev)
    q = torch.cat([gen_corpus_chunk(int(i), int(i) + 1, dim, centers, dev) for i in idx.tolist()])
    q = q + 0.3 * torch.randn(q.shape, generator=g, device=dev)
    out = {"queries": 32, "k": 10, "rows": r1 - r0, "dim": dim}
    ref_rows = None
    for mode in ("fp16", "fp8"):
        store.set_scan_dtype(mode)
        _, rows = store.search_dev(q, 10)
        torch.cuda.synchronize()
        N.profile_enable(True)
        N.profile_read()
        t0 = time.perf_counter()
        for _ in range(reps):
            store.search_dev(q, 10)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        N.profile_enable(False)
        prof = N.profile_read()
        scan = {k: v for k, v in prof.items() if k.startswith("cosine_scan")}
        sb, sm = sum(v["bytes"] for v in scan.values()), sum(v["total_ms"] for v in scan.values())
        gbs = sb / (sm * 1e-3) / 1e9
        out[mode] = {"ms_per_batch": round(dt * 1e3, 3), "qps": round(32 / dt, 1),
                     "scan_ms": round(sm / reps, 3), "scan_GBps": round(gbs, 1),
                     "frac": round(gbs / PEAK_HBM_GBS, 4)}
        if mode == "fp16":
            ref_rows = rows.cpu()
        else:
            r8 = rows.cpu()
            out["fp8_recall_at_10_vs_fp16"] = round(
                sum(len(set(r8[i].tolist()) & set(ref_rows[i].tolist())) for i in range(32)) / 320, 4)
    store.set_scan_dtype("fp16")
    out["fp8_speedup"] = round(out["fp16"]["ms_per_batch"] / out["fp8"]["ms_per_batch"], 3)
    return out


def rerank_fidelity(rs, device, modes=((0, "fp16"), (1, "fp8_mode1"), (2, "fp8_mode2"),
                                         (3, "fp8_mode3"))):
    """Ranking fidelity of the cross-encoder kernels at the bench shape (12 layers, 768-d, S_pair =
    128; bge-reranker-v2-m3's 24 layers, 1024-d with --rerank-model bge-reranker-v2-m3) on a
    DISCRIMINATIVE reranker: the relevance-structured weights of super_rag_amd/synthetic.py (the
    bench's seeded-random reranker spreads one query's logits by std ~1e-2 only) on 8 queries x
    100 candidates sharing 0..15 query terms, against the fp32 oracle's logits committed in
    tests/golden/rerank_fidelity{,_v2m3}.npz (data; tests/golden/gen_rerank_fidelity.py).  Per precision
    mode: max |logit error|, the smallest per-query (logit std / max error), top-10 identical modulo
    ties within 1 % of the logit std, mean top-10 overlap, top-1 equal."""
    from super_rag_amd.encoder import Encoder
    from super_rag_amd.synthetic import fidelity_setup
    fixture = {"bge-reranker-base": "rerank_fidelity.npz",
               "bge-reranker-v2-m3": "rerank_fidelity_v2m3.npz"}.get(rs.name)
    path = os.path.join(ROOT, "tests", "golden", fixture) if fixture else None
    if path is None or not os.path.exists(path):
        return None
    fx = np.load(path)
    w, ids, mask, _, m = fidelity_setup(rs)
    if not np.array_equal(ids, fx["ids"]):
        return {"error": "fidelity fixture does not match its generator"}
    ref = fx["logits"].reshape(-1, m["cand"])
    std = ref.std(1)
    enc = Encoder(rs, device=device, weights=w, max_tokens=ids.size)
    dids = torch.from_numpy(ids).to(f"cuda:{device}")
    dmask = torch.from_numpy(mask).to(f"cuda:{device}")
    out = {"set": (f"{ref.shape[0]} queries x {m['cand']} pairs, S_pair={m['pair_len']}, "
                   f"{rs.name} shape, relevance-structured weights (super_rag_amd/synthetic.py) vs the "
                   f"fp32 oracle (tests/golden/{fixture})"),
           "logit_std_mean": round(float(std.mean()), 4)}
    try:
        for mode, name in modes:
            enc.set_fp8(mode)
            lg = enc.cross_score_dev(dids, dmask)[:, 0].float().cpu().numpy().reshape(ref.shape)
            err = np.abs(lg - ref).max(1)
            ident = 0
            overlap = []
            for b in range(ref.shape[0]):
                want = np.argsort(-ref[b], kind="stable")[:10]
                got = np.argsort(-lg[b], kind="stable")[:10]
                kth = ref[b][want[-1]]
                ident += int(all(abs(ref[b][j] - kth) <= 0.01 * std[b] for j in set(want) ^ set(got)))
                overlap.append(len(set(want) & set(got)) / 10)
            out[name] = {"max_logit_err": round(float(err.max()), 5),
                         "min_std_over_err": round(float((std / np.maximum(err, 1e-12)).min()), 1),
                         "top10_identical_mod_ties": f"{ident}/{ref.shape[0]}",
                         "top10_overlap": round(float(np.mean(overlap)), 3),
                         "top1_equal": round(float(np.mean([np.argmax(lg[b]) == np.argmax(ref[b])
                                                            for b in range(ref.shape[0])])), 3)}
    finally:
        enc.close()
    return out


def measured_peaks(dev):
    """peaks measured on this box beside the spec values the roofline divides by.
    HBM: STREAM-style copy of a 2 GiB buffer (read + write bytes) by the library's 16-byte copy
    kernel (sr_diag_copy) and by torch; MFMA: the K4 main loop alone
    (sr_diag_gemm variant 9, no epilogue) at the reranker's FFN1 shape, random fp16 operands."""
    import torch
    from super_rag_amd import _native as N
    out = {}
    x = torch.empty(1 << 30, dtype=torch.float16, device=dev).normal_()
    y = torch.empty_like(x)
    st = torch.cuda.current_stream().cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, fn in (("hbm_copy_GBs", lambda: N.call_diag("sr_diag_copy", x.data_ptr(), y.data_ptr(),
                                                     x.numel() * 2, 0, st)),
                     ("hbm_torch_copy_GBs", lambda: y.copy_(x))):
        fn()
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(2.0 * x.numel() * 2 * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e9, 1)
    del x, y
    M, Nn, K = 131072, 3072, 768
    X = torch.randn(M, K, device=dev).half()
    W = torch.randn(Nn, K, device=dev).half() * 0.03
    bias = torch.zeros(Nn, device=dev)
    Y = torch.empty(M, Nn, device=dev, dtype=torch.float16)

    def g():
        N.call_diag("sr_diag_gemm", 9, 0, X.data_ptr(), X.stride(0), W.data_ptr(), bias.data_ptr(), None, 0,
               Y.data_ptr(), Y.stride(0), M, Nn, K, 0, st)
    g()
    e0.record()
    for _ in range(10):
        g()
    e1.record()
    torch.cuda.synchronize()
    out["mfma_f16_gemm_mainloop_TFs"] = round(2.0 * M * Nn * K * 10 / (e0.elapsed_time(e1) * 1e-3) / 1e12, 1)
    del X, W, Y
    out.update(mfma_rate_peaks(dev))
    out["note"] = ("measured on this box after the timed region; roofline.peak stays the spec value "
                   "(HBM 8 TB/s, f16 2.5 PF / fp8 5 PF at 2.4 GHz); mfma_*_peak_TFs_held: the MFMA "
                   "issue-rate microbenchmark (sr_diag_mfma_rate: every CU, 8 waves x 8 independent "
                   "chains, random operands, >= 2 s of launches first) at the clock the chip held "
                   "under it (s_memtime / s_memrealtime)")
    return out


def mfma_rate_peaks(dev, warm_s=2.0, timed=4):
    """The MFMA issue-rate peak on this box: sr_diag_mfma_rate in the
    product's f16 and block-scaled fp8 shapes, back-to-back launches for warm_s seconds (DVFS
    settles), then `timed` launches between HIP events; the clock from the kernel's own
    s_memtime / s_memrealtime stamps (median over workgroups) of the timed launches."""
    import time as _t
    import torch
    from super_rag_amd import _native as N
    out = {}
    blocks = 1024
    sink = torch.empty(blocks * 512, device=dev)
    stamps = torch.zeros(blocks * 2, device=dev, dtype=torch.int64)
    st = torch.cuda.current_stream().cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for f8, K, iters, name in ((0, 32, 500, "f16"), (1, 128, 250, "f8")):
        flop = blocks * 8.0 * iters * 8 * 16 * 16 * K * 2

        def launch():
            N.call_diag("sr_diag_mfma_rate", f8, blocks, iters, sink.data_ptr(), stamps.data_ptr(), 0, st)
        t0 = _t.perf_counter()
        while _t.perf_counter() - t0 < warm_s:
            launch()
            torch.cuda.synchronize()
        e0.record()
        for _ in range(timed):
            launch()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / timed
        s = stamps.view(blocks, 2).double().cpu()
        clk = (s[:, 0] / s[:, 1].clamp(min=1) * 0.1).median().item()   # GHz (realtime: 100 MHz)
        out[f"mfma_{name}_peak_TFs_held"] = round(flop / (ms * 1e-3) / 1e12, 1)
        out[f"mfma_{name}_clock_ghz"] = round(clk, 3)
        out[f"mfma_{name}_frac_of_spec"] = round(flop / (ms * 1e-3) / 1e12 /
                                                 (PEAK_F8_TFLOPS if f8 else PEAK_F16_TFLOPS), 4)
    return out


def add_held_peak(roof, peaks):
    """roofline.frac_of_held_peak: achieved / the MFMA peak measured on this box (the f16 or fp8
    figure by the kernel's operands); roofline.frac stays against the spec peak."""
    if not roof or not peaks or roof.get("bound") != "mfma":
        return roof
    key = "mfma_f8_peak_TFs_held" if str(roof.get("kernel", "")).startswith("gemm_f8") else "mfma_f16_peak_TFs_held"
    if peaks.get(key):
        roof["held_peak"] = peaks[key]
        roof["frac_of_held_peak"] = round(roof["achieved"] / peaks[key], 4)
    return roof


def source_fingerprint(root=ROOT):
    """sha256 over the native sources (super-rag_amd/csrc/*, include/*.h) in name order: names the
    kernel code a PMC summary was collected on (tools/profile_round.sh writes it beside the passes)."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(root, "super-rag_amd", "csrc", "*")) +
                   glob.glob(os.path.join(root, "include", "*.h")))
    for fn in files:
        if os.path.isfile(fn):
            h.update(os.path.relpath(fn, root).encode())
            with open(fn, "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def pmc_file(root=ROOT):
    """(relative path, parsed summary) of the committed PMC summary (profiles/*_pmc_traffic.json,
    tools/pmc_traffic.py) taken on the current native sources (its source fingerprint), else the
    last one by name, or (None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(root, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None, None
    fp = source_fingerprint(root)
    parsed = []
    for path in files:
        try:
            with open(path) as f:
                parsed.append((path, json.load(f)))
        except (OSError, ValueError):
            continue
    if not parsed:
        return None, None
    match = [(p, d) for p, d in parsed if d.get("source_sha256") == fp]
    path, d = (match or parsed)[-1]
    return os.path.relpath(path, root), d


# ProfScope names (the bench's kernel table) that differ from the logical names tools/pmc_traffic.py
# derives from the mangled kernel names (the same kernels)
PMC_ALIASES = {"cls_attn_fold1": "cls_attn_fold", "cosine_scan_dense": "cosine_scan"}


def _pmc_name(k):
    return PMC_ALIASES.get(k, k)


def pmc_kernels(d, workload=None):
    """The per-kernel records of a PMC summary for a workload: config 4 (the default bench) at the
    top level, config 5's fp8 path under workloads.config5 (tools/pmc_traffic.py)."""
    if d is None:
        return {}
    if workload in (None, "config4"):
        return d.get("kernels", {})
    return d.get("workloads", {}).get(workload, {}).get("kernels", {})


def pmc_provenance(run_kernels, root=ROOT, workload=None):
    """Which PMC summary the roofline's `traffic` / `pmc_*` fields come from and whether it
    describes THIS run: the summary's commit and native-source fingerprint (recorded on the box by
    tools/profile_round.sh) against the running tree's, and the kernels timed here against the
    summary's (names normalised through PMC_ALIASES; the summary also holds setup kernels the
    timed region does not launch, which is no difference).  stale = the sources differ, or a kernel
    timed here is missing from the summary (another workload / precision mode, or kernels added
    since): the counters then describe other code, so the roofline reports traffic null and keeps
    the stale numbers beside it."""
    path, d = pmc_file(root)
    if d is None:
        return None
    mine = {_pmc_name(k) for k in run_kernels}
    theirs = {_pmc_name(k) for k in pmc_kernels(d, workload)}
    fp = d.get("source_sha256")
    src_match = None if fp is None else fp == source_fingerprint(root)
    missing = sorted(mine - theirs)
    reasons = []
    if src_match is False:
        reasons.append("native sources differ from the profiled tree")
    if missing:
        reasons.append(f"kernels timed here but absent from the summary: {missing}")
    return {"file": path, "workload": workload or "config4", "commit": d.get("commit"), "source_sha256": fp,
            "source_match": src_match, "kernel_set_match": not missing,
            "stale": bool(reasons), "stale_reasons": reasons}


def pmc_record(kernel, root=ROOT, workload=None):
    """The kernel's record in the newest committed PMC summary (tools/pmc_traffic.py), or None."""
    _, d = pmc_file(root)
    if d is None:
        return None
    ks = {_pmc_name(k): v for k, v in pmc_kernels(d, workload).items()}
    return ks.get(_pmc_name(kernel))


def pmc_traffic(kernel, root=ROOT, workload=None):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes over this same bench command, gfx950 fetch correction applied).
    Counters cannot be read live inside the timed region, so the value is the profiled run's."""
    path, d = pmc_file(root)
    if d is None:
        return None, None
    k = pmc_record(kernel, root, workload)
    if not k:
        return None, None
    where = f"{path}" + (f" [workloads.{workload}]" if workload not in (None, "config4") else "")
    return k["traffic_B"], (f"{where}: fetch {k['fetch_B']} B + write "
                            f"{k['write_B']} B per launch (mean over {k['launches']} launches)")


def apply_pmc(roof, kernel, run_kernels, root=ROOT, workload=None):
    """Fill roof["traffic"] (+ pmc clock / utilisation) from the PMC summary, with its provenance;
    a stale summary's numbers move to roof["stale_pmc"] and traffic stays null."""
    traffic, src = pmc_traffic(kernel, root, workload)
    rec = pmc_record(kernel, root, workload)
    prov = pmc_provenance(run_kernels, root, workload)
    roof["pmc_provenance"] = prov
    fields = {"traffic": traffic, "traffic_source": src}
    if rec and rec.get("clock_ghz") and roof.get("bound") == "mfma":
        # the clock the chip holds under this MFMA load (DVFS) and the matrix-pipe utilisation
        # measured by the PMC pass: frac of the spec peak vs of the peak at the held clock
        fields["pmc_clock_ghz"] = rec["clock_ghz"]
        fields["pmc_mfma_util"] = rec.get("mfma_util")
        fields["peak_at_held_clock"] = round(roof["peak"] * rec["clock_ghz"] / 2.4, 1)
    if rec and rec.get("traffic_B") and roof.get("algorithmic_B_per_launch"):
        # PMC traffic over the algorithmic bytes (> 1: re-reads beyond L2)
        fields["traffic_over_algorithmic"] = round(rec["traffic_B"] / roof["algorithmic_B_per_launch"], 3)
    if prov and prov["stale"]:
        roof["traffic"] = None
        roof["stale_pmc"] = fields
    else:
        roof.update(fields)
    return roof


def cpu_cores() -> int:
    """CPUs this process may use: its affinity set, capped by the cgroup CPU quota (the GPU box
    grants 16 CPUs per GPU: cpu.max = 1600000 100000 while os.cpu_count() shows the machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return n


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            return next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        return "unknown"


def cpu_baseline(a, es, rs, w_embed, w_rerank, centers, batch, p_tok, N_total, embedder, dev):
    """The oracle (oracle/*, the CPU restatement) timed on the host cores,
    stage by stage, with no extrapolation:
      embed   a.cpu_queries queries (S = q_len) through the fp32 torch-CPU encoder;
      search  the full batch of queries (this rank's B) against the whole corpus as a batched
              fp32 torch matmul + topk, streamed in 1M-row chunks (each chunk is generated and
              L2-normalised on the GPU and copied to pinned host memory outside the timed part);
      rerank  whole queries of k_cand (query, passage) pairs at S_pair through the fp32
              cross-encoder, one query's pairs per call, until --cpu-rerank-budget-s is spent.
    End-to-end q/s = 1 / (embed + search + rerank seconds per query)."""
    from oracle import encoder_ref as R
    threads = cpu_cores()
    torch.set_num_threads(threads)
    cfg = lambda s: R.RefConfig(s.vocab_size, s.hidden, s.layers, s.heads, s.intermediate,
                                s.max_position, s.type_vocab, s.ln_eps, s.position_offset,
                                s.classifier, s.num_labels)
    log = lambda m: print(f"[cpu_baseline] {m}", file=sys.stderr, flush=True)
    nq = min(a.cpu_queries, a.batch)
    ids, mask, qtok, qlen = batch
    wt_e = {k: torch.from_numpy(v) for k, v in w_embed.items()}
    wt_r = {k: torch.from_numpy(v) for k, v in w_rerank.items()}
    # ---- (i) embed -----------------------------------------------------------------------------
    ids_h, mask_h = ids[:nq].cpu().numpy(), mask[:nq].cpu().numpy()
    t0 = time.perf_counter()
    R.embed(cfg(es), wt_e, ids_h, mask_h)
    t_embed = time.perf_counter() - t0
    log(f"embed {nq} queries: {t_embed:.2f} s ({threads} threads)")
    # ---- (ii) exact fp32 cosine top-k over the whole corpus, batched ---------------------------
    q = embedder.embed_dev(ids, mask, fp16=False).cpu()      # [B, d] unit queries (inputs)
    rows_total = a.cpu_search_rows or N_total
    step = 1 << 20
    host = torch.empty((step, a.dim), dtype=torch.float32).pin_memory()
    best_s = torch.full((q.shape[0], 0), -2.0)
    best_r = torch.zeros((q.shape[0], 0), dtype=torch.int64)
    t_search = 0.0
    for c0 in range(0, rows_total, step):
        c1 = min(rows_total, c0 + step)
        x = torch.nn.functional.normalize(gen_corpus_chunk(c0, c1, a.dim, centers, dev), dim=1)
        host[: c1 - c0].copy_(x)
        del x
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s = q @ host[: c1 - c0].T
        v, i = s.topk(a.k_cand, dim=1)
        best_s = torch.cat([best_s, v], 1)
        best_r = torch.cat([best_r, i + c0], 1)
        top = best_s.topk(a.k_cand, dim=1)
        best_s, best_r = top.values, best_r.gather(1, top.indices)
        t_search += time.perf_counter() - t0
    del host
    log(f"search {q.shape[0]} queries x {rows_total} rows: {t_search:.2f} s")
    # ---- (iii) cross-encoder rerank of k_cand pairs per query -----------------------------------
    cand = best_r[:nq]
    pt = p_tok[cand.reshape(-1).to(p_tok.device)].view(nq, a.k_cand, -1).cpu().numpy()
    pids, pmask, _ = R.pack_pairs(qtok[:nq].cpu().numpy(), qlen[:nq].cpu().numpy(),
                                  pt.reshape(nq * a.k_cand, -1), np.full(nq * a.k_cand, pt.shape[-1]),
                                  np.arange(nq * a.k_cand).reshape(nq, a.k_cand), a.pair_len, 0,
                                  rs.bos_id, rs.eos_id, rs.pad_id)
    t_rerank = 0.0
    nq_r = 0
    for i in range(nq):
        sl = slice(i * a.k_cand, (i + 1) * a.k_cand)
        t0 = time.perf_counter()
        R.cross_logits(cfg(rs), wt_r, pids[sl], pmask[sl])
        t_rerank += time.perf_counter() - t0
        nq_r += 1
        log(f"rerank {nq_r} queries: {t_rerank:.1f} s")
        if t_rerank >= a.cpu_rerank_budget_s:
            break
    per_q = {"embed": t_embed / nq, "search": t_search / q.shape[0], "rerank": t_rerank / nq_r}
    # (iv) the reference flow's own host-side orchestration per query (NodeflowEngine + runners,
    # constant-time stub backends), measured in the build container by tools/ref_orchestration.py
    orch = None
    orch_path = os.path.join(ROOT, "profiles", "r02_reference_orchestration.json")
    if os.path.exists(orch_path):
        with open(orch_path) as f:
            orch = json.load(f)
        per_q["orchestration"] = float(orch["value"])
    total = sum(per_q.values())
    return {"value": round(1.0 / total, 4), "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": (f"oracle (torch-CPU fp32) on {threads} threads, no extrapolation: embed "
                       f"{nq} queries (S={a.q_len}); exact cosine top-{a.k_cand} of {q.shape[0]} "
                       f"queries over all {rows_total} x {a.dim} rows as a batched fp32 matmul + "
                       f"topk in 1M-row chunks; rerank {nq_r} whole queries x {a.k_cand} pairs "
                       f"(S={a.pair_len}; as many as fit a {a.cpu_rerank_budget_s:.0f} s host-time "
                       f"budget, measured not extrapolated); end to end = 1 / sum of per-query "
                       f"stage times"),
            "cpu_model": cpu_model(), "machine_cpus": os.cpu_count(),
            "stage_s_per_query": {k: round(v, 5) for k, v in per_q.items()},
            "stage_qps": {k: round(1.0 / v, 3) for k, v in per_q.items()},
            "stage_s_total": {"embed": round(t_embed, 3), "search": round(t_search, 3),
                              "rerank": round(t_rerank, 3)},
            "stage_queries": {"embed": nq, "search": int(q.shape[0]), "rerank": nq_r},
            "orchestration_source": (f"{os.path.relpath(orch_path, ROOT)} ({orch['method']}; "
                                     f"{orch['note']})") if orch else None}


if __name__ == "__main__":
    main()
