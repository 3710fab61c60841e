"""CPU tests of bench.py's PMC provenance: the roofline's traffic / pmc fields
name the summary file, its commit and source fingerprint, and go stale -- traffic null, the old
numbers kept beside it -- when the summary's kernel set or native sources differ from this run's."""
import json
import os
import shutil

import pytest

import bench


def _tree(tmp_path, kernels, sha):
    root = tmp_path / "repo"
    for d in ("profiles", "super-rag_amd/csrc", "include"):
        (root / d).mkdir(parents=True)
    (root / "super-rag_amd/csrc/k.hip").write_text("kernel v1\n")
    (root / "include/a.h").write_text("int f(void);\n")
    summary = {"source": "gpurun_out/prof_x", "commit": "abc123", "method": "test",
               "source_sha256": sha,
               "kernels": {k: {"launches": 4, "fetch_B": 100, "write_B": 20, "traffic_B": 120,
                               "clock_ghz": 1.8, "mfma_util": 0.5} for k in kernels}}
    (root / "profiles/r99_pmc_traffic.json").write_text(json.dumps(summary))
    return str(root)


def test_fresh_summary_fills_traffic(tmp_path):
    root = _tree(tmp_path, ["gemm_a", "scan"], None)
    sha = bench.source_fingerprint(root)
    with open(os.path.join(root, "profiles/r99_pmc_traffic.json")) as f:
        d = json.load(f)
    d["source_sha256"] = sha
    with open(os.path.join(root, "profiles/r99_pmc_traffic.json"), "w") as f:
        json.dump(d, f)
    roof = {"bound": "mfma", "peak": 2500.0}
    bench.apply_pmc(roof, "gemm_a", ["gemm_a", "scan"], root)
    assert roof["traffic"] == 120
    assert roof["pmc_provenance"]["stale"] is False
    assert roof["pmc_provenance"]["file"] == os.path.join("profiles", "r99_pmc_traffic.json")
    assert roof["pmc_provenance"]["commit"] == "abc123"
    assert roof["pmc_clock_ghz"] == 1.8 and "stale_pmc" not in roof


def test_kernel_set_difference_marks_stale(tmp_path):
    root = _tree(tmp_path, ["gemm_a", "scan"], None)
    roof = {"bound": "mfma", "peak": 2500.0}
    bench.apply_pmc(roof, "gemm_a", ["gemm_a", "scan", "gemm_new"], root)
    prov = roof["pmc_provenance"]
    assert prov["stale"] and not prov["kernel_set_match"]
    assert "gemm_new" in prov["stale_reasons"][0]
    assert roof["traffic"] is None and roof["stale_pmc"]["traffic"] == 120
    assert "pmc_clock_ghz" not in roof


def test_setup_kernels_and_profscope_aliases_are_no_difference(tmp_path):
    """The summary counts every library kernel of the profiled run (setup kernels such as
    fold_ln_weight included) under the mangled-name logical names; the bench times its ProfScope
    names (cls_attn_fold for cls_attn_fold1_kernel, cosine_scan_dense for the EPI_SCAN kernel)."""
    root = _tree(tmp_path, ["gemm_a", "cosine_scan", "cls_attn_fold1", "fold_ln_weight"], None)
    prov = bench.pmc_provenance(["gemm_a", "cosine_scan_dense", "cls_attn_fold"], root)
    assert prov["kernel_set_match"] and not prov["stale"], prov
    roof = {"bound": "hbm", "peak": 8000.0}
    bench.apply_pmc(roof, "cosine_scan_dense", ["gemm_a", "cosine_scan_dense"], root)
    assert roof["traffic"] == 120


def test_source_change_marks_stale(tmp_path):
    root = _tree(tmp_path, ["gemm_a"], None)
    sha = bench.source_fingerprint(root)
    with open(os.path.join(root, "profiles/r99_pmc_traffic.json")) as f:
        d = json.load(f)
    d["source_sha256"] = sha
    with open(os.path.join(root, "profiles/r99_pmc_traffic.json"), "w") as f:
        json.dump(d, f)
    with open(os.path.join(root, "super-rag_amd/csrc/k.hip"), "a") as f:
        f.write("changed\n")
    prov = bench.pmc_provenance(["gemm_a"], root)
    assert prov["source_match"] is False and prov["stale"]


def test_no_summary(tmp_path):
    root = tmp_path / "empty"
    (root / "profiles").mkdir(parents=True)
    roof = {"bound": "hbm", "peak": 8000.0}
    bench.apply_pmc(roof, "scan", ["scan"], str(root))
    assert roof["traffic"] is None and roof["pmc_provenance"] is None


def test_comm_record_single_process():
    import torch.distributed as dist
    rec = bench.comm_record(dist, 1, "nccl")
    assert rec["world_size"] == 1 and rec["backend"] is None and rec["requested_backend"] is None
    assert "rccl_version" in rec


def test_parse_defaults_and_config5_field_args(monkeypatch):
    """The default command's arguments, and the config-5 field derived from them (VERDICT r3
    item 3): bge-m3 at 1024-d, the 6.25M-row shard per rank, fp8 mode 3, its own step counts."""
    import sys
    monkeypatch.setattr(sys, "argv", ["bench.py"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    a = bench.parse()
    assert a.workload == "config4" and a.embed_model == "bge-base-en" and a.corpus_rows == 10_000_000
    assert a.config5_steps > 0 and a.dropin_procs >= 2 and a.fp8 == 0
    a5 = bench.config5_args(a)
    assert (a5.workload, a5.embed_model, a5.dim, a5.corpus_rows, a5.fp8) == \
        ("config5", "bge-m3", 1024, 6_250_000, 3)
    assert (a5.steps, a5.warmup) == (a.config5_steps, a.config5_warmup)
    assert a.workload == "config4" and a.dim == 768            # the headline's args untouched
    monkeypatch.setattr(sys, "argv", ["bench.py", "--corpus-rows", "200000"])
    assert bench.config5_args(bench.parse()).corpus_rows == 200000
    monkeypatch.setattr(sys, "argv", ["bench.py", "--workload", "config5"])
    c = bench.parse()
    assert c.embed_model == "bge-m3" and c.no_cpu_baseline


def test_dropin_procs_release_and_collect(tmp_path):
    """bench.DropinProcs with a stand-in serving script (no GPU): the children wait for the go
    file, start at its common time, and collect() sums their throughput and pools the latencies
    of all of them for p50 / p99, one window per callers-per-process value, with Little's law's
    mean beside the measured one."""
    script = tmp_path / "fake_dropin.py"
    script.write_text(
        "import argparse, json, os, sys, time\n"
        "import numpy as np\n"
        "sys.path.insert(0, %r)\n"
        "from tools.bench_dropin import wait_for_go\n"
        "ap = argparse.ArgumentParser()\n"
        "for a in ('--rows', '--seconds', '--go-file', '--lat-out'): ap.add_argument(a)\n"
        "ap.add_argument('--concurrency', type=int, nargs='+')\n"
        "a = ap.parse_args()\n"
        "assert a.concurrency == [32, 64]\n"
        "t0 = wait_for_go(a.go_file, timeout_s=60)\n"
        "assert abs(t0 - time.time()) < 30\n"
        "i = int(a.lat_out[-1])\n"
        "runs = []\n"
        "for w, c in enumerate(a.concurrency):\n"
        "    np.save(a.lat_out + '_c%%d.npy' %% c, np.full(100, 10.0 * (i + 1) * (w + 1), np.float32))\n"
        "    runs.append({'qps': 100.0 + i, 'requests': 100, 'seconds': 1.0, 'p50_ms': 1, 'p99_ms': 2,\n"
        "                 'coalesced': {'rerank': {'mean_batch': 4.0}}})\n"
        "print(json.dumps({'runs': runs}))\n" % bench.ROOT)
    mp = bench.DropinProcs(3, 100, 1.0, concurrency=(32, 64), script=str(script))
    try:
        mp.release(delay_s=0.5)
        r = mp.collect(timeout_s=120)
    finally:
        mp.stop()
    assert r["procs"] == 3 and len(r["windows"]) == 2
    w32, w64 = r["windows"]
    assert w32["concurrency_per_proc"] == 32 and w32["callers"] == 96
    assert w32["qps"] == 303.0 and w32["requests"] == 300
    assert w32["p50_ms"] == 20.0 and w32["p99_ms"] == 30.0 and w32["mean_ms"] == 20.0
    assert w64["p50_ms"] == 40.0 and w64["littles_law_mean_ms"] == round(192 / 303.0 * 1e3, 1)
    s = bench.summary({"value": 1, "unit": "q", "n_gpus": 1, "ms_per_step": 1,
                       "drop_in": {"runs": [{"concurrency": 64, "qps": 9, "p50_ms": 1, "p99_ms": 2}],
                                   "multi_process": r}})
    assert s["drop_in"]["multi_process"]["3x32"]["qps"] == 303.0
    assert not os.path.exists(mp.dir)


def test_dropin_windows_start_together():
    """tools/bench_dropin._windows: with a common start time, window i begins at start + i
    (seconds + gap) in every process; without one, immediately."""
    import time
    from tools.bench_dropin import WINDOW_GAP_S, _windows
    t0 = time.time() + 0.3
    seen = []
    for c, late in _windows([16, 32], 0.2, t0):
        seen.append((c, time.time(), late))
    assert [c for c, _, _ in seen] == [16, 32]
    assert seen[0][1] >= t0 and seen[1][1] >= t0 + 0.2 + WINDOW_GAP_S
    assert all(0.0 <= late < 0.2 for _, _, late in seen)
    assert list(_windows([8], 5.0, 0.0)) == [(8, 0.0)]
    # a start time already past: the window begins at once and reports how late it is
    (c, late), = list(_windows([4], 1.0, time.time() - 2.0))
    assert c == 4 and late >= 2.0


def test_config5_workload_section(tmp_path):
    """the config-5 field's roofline reads its own section of the summary
    (workloads.config5: the fp8 path's kernels), never config 4's per-launch means of the same
    kernel names; a summary without the section leaves it stale."""
    root = _tree(tmp_path, ["gemm_a", "qkv_attention"], None)
    sha = bench.source_fingerprint(root)
    path = os.path.join(root, "profiles/r99_pmc_traffic.json")
    with open(path) as f:
        d = json.load(f)
    d["source_sha256"] = sha
    with open(path, "w") as f:
        json.dump(d, f)
    run5 = ["gemm_f8_lnfold_gelu_out8", "qkv_attention", "cosine_scan8"]
    roof = {"bound": "mfma", "peak": 5000.0, "algorithmic_B_per_launch": 500}
    bench.apply_pmc(roof, "gemm_f8_lnfold_gelu_out8", run5, root, workload="config5")
    assert roof["traffic"] is None and roof["pmc_provenance"]["stale"]
    d["workloads"] = {"config5": {"kernels": {k: {"launches": 2, "fetch_B": 700, "write_B": 300,
                                                  "traffic_B": 1000, "clock_ghz": 1.9,
                                                  "mfma_util": 0.6} for k in run5}}}
    with open(path, "w") as f:
        json.dump(d, f)
    roof = {"bound": "mfma", "peak": 5000.0, "algorithmic_B_per_launch": 500}
    bench.apply_pmc(roof, "qkv_attention", run5, root, workload="config5")
    assert roof["traffic"] == 1000 and not roof["pmc_provenance"]["stale"]
    assert roof["pmc_provenance"]["workload"] == "config5"
    assert roof["traffic_over_algorithmic"] == 2.0 and roof["pmc_mfma_util"] == 0.6
    roof4 = {"bound": "mfma", "peak": 2500.0}
    bench.apply_pmc(roof4, "qkv_attention", ["gemm_a", "qkv_attention"], root)
    assert roof4["traffic"] == 120          # config 4 keeps the top-level records


def test_logical_names_of_the_fp8_gemm_kernels():
    """tools/pmc_traffic.logical: the F8IN instantiations (4th template argument true) carry the
    bench's gemm_f8_* names, so config 5's PMC section matches its timed kernels."""
    import sys
    sys.path.insert(0, os.path.join(bench.ROOT, "tools"))
    from pmc_traffic import logical
    k = "_ZN2sr12_GLOBAL__N_116gemm_pipe_kernelILi{}ELb1ELi0ELb{}EEEvPKDF16_lS3_PKfPKvlPvliiiNS_6LnFoldE"
    assert logical(k.format(11, 1)) == "gemm_f8_lnfold_gelu_out8"
    assert logical(k.format(8, 1)) == "gemm_f8_lnres16_stats"
    assert logical(k.format(8, 0)) == "gemm_f16_lnres16_stats"
    assert logical(k.format(6, 0)) == "gemm_f16_lnfold_gelu"
    assert logical("_ZN2sr12_GLOBAL__N_115qkv_attn_kernelILb1ELi0ELb0EEEvPKDF16_") == "qkv_attention"


def test_bulk_dropin_collection_adopts_a_store_and_pools_texts():
    """the drop-in path measured on the headline corpus.  build_collection_bulk
    adopts an existing store (bench.py hands over its 10M-row corpus), serves pooled texts /
    metadata through the connector's own search, and release_collection leaves the adopted store
    open for its owner."""
    import sys
    sys.path.insert(0, os.path.join(bench.ROOT, "tests"))
    import numpy as np
    from doubles import NumpyStore
    from super_rag_amd import vectorstore as V
    from super_rag_amd.models import QueryWithEmbedding
    from tools import bench_dropin as D
    V.set_store_backend(lambda dim, dev: NumpyStore(dim, dev), NumpyStore.load)
    V._collections.clear()
    try:
        rng = np.random.default_rng(3)
        st = NumpyStore(16)
        st.add(rng.standard_normal((5000, 16)).astype(np.float32))
        old_pool = D.TEXT_POOL
        D.TEXT_POOL = 700
        try:
            con = D.build_collection_bulk("bulk-t", 0, dim=16, store=st)
        finally:
            D.TEXT_POOL = old_pool
        c = V._collections[con.collection_name]
        assert c.store is st and len(c.texts) == 5000 and len(c.ids) == 5000
        assert c.texts[4321].startswith(c.texts[4321 % 700].rsplit(" ", 1)[0]) and c.texts[-1] == c.texts[4999]
        assert len(set(c.texts[i] for i in range(0, 5000, 7))) == len(range(0, 5000, 7))  # distinct
        assert c.metadatas[1403] == {"source": "d3.md"} and c.ids[12] == "bulk-12"
        with pytest.raises(IndexError):
            c.texts[5000]
        q = st.get(np.asarray([4321]))[0]
        res = con.search(QueryWithEmbedding(query="x", top_k=3, embedding=list(map(float, q))))
        assert res.results[0].text == c.texts[4321] and res.results[0].score < 1e-4
        D.release_collection("bulk-t")
        assert con.collection_name not in V._collections and st.count()[0] == 5000
    finally:
        V._collections.clear()
        V.set_store_backend(V._native_store, V._native_load)


def test_held_peak_fraction():
    """roofline.frac_of_held_peak = achieved / the MFMA peak measured on the
    box (f16 or fp8 by the kernel); frac stays against the spec peak."""
    peaks = {"mfma_f16_peak_TFs_held": 2000.0, "mfma_f8_peak_TFs_held": 4000.0}
    r = bench.add_held_peak({"bound": "mfma", "achieved": 1000.0, "frac": 0.4,
                             "kernel": "gemm_f16_lnres16_stats"}, peaks)
    assert r["frac_of_held_peak"] == 0.5 and r["held_peak"] == 2000.0 and r["frac"] == 0.4
    r = bench.add_held_peak({"bound": "mfma", "achieved": 1000.0, "kernel": "gemm_f8_x"}, peaks)
    assert r["frac_of_held_peak"] == 0.25
    r = bench.add_held_peak({"bound": "hbm", "achieved": 5000.0, "kernel": "cosine_scan"}, peaks)
    assert "frac_of_held_peak" not in r
