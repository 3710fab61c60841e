"""Per-kernel HBM traffic from rocprofv3 PMC passes (diagnostic tool, runs here on the merged
gpurun_out/ files; not part of the product).

    python tools/pmc_traffic.py gpurun_out/prof_<tag> profiles/<round>_pmc_traffic.json

Reads the FETCH_SIZE pass (fetch/pmc_1/run_counter_collection.csv) and the WRITE_SIZE pass
(write/pmc_1/...), each collected in its own run as MI355X_MICROARCH.md §HBM prescribes, and writes
per logical kernel (the names `sr_profile_*` / bench.py use) the mean bytes per launch:
  fetch_B = FETCH_SIZE (KiB) x 1024 x 2   (gfx950: FETCH_SIZE counts half the bytes of a wide
                                           coalesced streaming read — 128-B requests tallied as 64 B)
  write_B = WRITE_SIZE (KiB) x 1024        (exact for 16-B-per-lane stores)
Both counters come from the L2 memory-side request counters, so Infinity-Cache hits are included.

With a third pass (mfma/pmc_1: SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE) it also reports per kernel
the clock the chip held (GRBM_GUI_ACTIVE is summed over the 8 XCDs: / 8 / duration) and the matrix
pipe utilisation = MFMA busy cycles (16 per v_mfma_f32_16x16x32_f16, 32 per block-scaled
v_mfma_scale_f32_16x16x128_f8f6f4, summed over SIMDs) / (1024 SIMDs x duration x held clock).

The same three passes over config 5's fp8 path (`bench.py --workload config5 --fp8 3`, under
<prof>/c5/ when tools/profile_round.sh collected them) land in out["workloads"]["config5"]: the
config-5 kernels (cosine_scan8, gemm_f8_*, *_y8, lex_*, rescore, rrf_fuse) and the bge-m3 shapes of
the embed GEMMs are another workload's launches, never averaged with config 4's.
"""
import os
import csv
import json
import re
import sys
from collections import defaultdict

EPI_NAMES = {0: "gemm_f16_bias", 1: "gemm_f16_bias_gelu", 2: "gemm_f16_bias_residual",
             3: "gemm_f16_bias_tanh", 4: "gemm_f16_bias_residual16", 5: "gemm_f16_lnfold",
             6: "gemm_f16_lnfold_gelu", 7: "gemm_f16_residual16_stats",
             8: "gemm_f16_lnres16_stats",
             9: "cosine_scan",    # K1 threshold chunks on the GEMM main loop (EPI_SCAN)
             10: "cosine_scan8",  # the fp8 scan (EPI_SCAN8)
             11: "gemm_f16_lnfold_gelu_out8", 12: "gemm_f16_residual16_stats_y8",
             13: "gemm_f16_lnres16_stats_y8"}


def logical(name):
    """Mangled HIP kernel name -> the library's logical kernel name (None for foreign kernels)."""
    if "_ZN2sr" not in name and not name.startswith("sr::"):
        return None
    m = re.search(r"gemm_\w*?kernelILi(\d+)E(\w*)", name)
    if m:
        base = EPI_NAMES.get(int(m.group(1)), f"gemm_epi{m.group(1)}")
        # template <EPI, PERSIST, DIAG, F8IN>: "...ILi<EPI>ELb<P>ELi<D>ELb1E" is the F8IN variant
        if re.match(r"Lb[01]ELi\d+ELb1E", m.group(2)):
            base = base.replace("gemm_f16_", "gemm_f8_")
        return base
    m = re.search(r"\d+([a-z0-9_]+?)_kernel", name) or re.search(r"::(\w+?)_kernel", name)
    base = m.group(1) if m else name
    base = re.sub(r"^sr\d+", "", base)  # kernels in namespace sr itself (not the anonymous one)
    if base.startswith("attention"):
        return "attention"
    if base == "qkv_attn":
        return "qkv_attention"   # K5c's ProfScope name
    return base


def read(path, counter):
    tot = defaultdict(float)
    n = defaultdict(int)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = logical(row["Kernel_Name"])
            if k is None:
                continue
            tot[k] += float(row["Counter_Value"])
            n[k] += 1
    return tot, n


def kernels_of(src):
    """{logical kernel: fetch / write / traffic bytes per launch (+ clock, mfma_util)} of the
    three passes under src (fetch/, write/, mfma/)."""
    f_tot, f_n = read(f"{src}/fetch/pmc_1/run_counter_collection.csv", "FETCH_SIZE")
    w_tot, w_n = read(f"{src}/write/pmc_1/run_counter_collection.csv", "WRITE_SIZE")
    ks = {}
    for k in sorted(set(f_tot) | set(w_tot)):
        fb = f_tot.get(k, 0.0) / max(f_n.get(k, 1), 1) * 1024 * 2
        wb = w_tot.get(k, 0.0) / max(w_n.get(k, 1), 1) * 1024
        ks[k] = {"launches": f_n.get(k, 0), "fetch_B": round(fb), "write_B": round(wb),
                 "traffic_B": round(fb + wb)}
    mf = f"{src}/mfma/pmc_1/run_counter_collection.csv"
    if os.path.exists(mf):
        busy, gui, dur, seen = defaultdict(float), defaultdict(float), defaultdict(float), set()
        with open(mf) as f:
            for row in csv.DictReader(f):
                k = logical(row["Kernel_Name"])
                if k is None:
                    continue
                if row["Counter_Name"] == "SQ_VALU_MFMA_BUSY_CYCLES":
                    busy[k] += float(row["Counter_Value"])
                elif row["Counter_Name"] == "GRBM_GUI_ACTIVE":
                    gui[k] += float(row["Counter_Value"])
                if row["Dispatch_Id"] not in seen:
                    seen.add(row["Dispatch_Id"])
                    dur[k] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9
        for k in dur:
            if dur[k] <= 0 or k not in ks:
                continue
            clk = gui[k] / 8.0 / dur[k]
            ks[k]["clock_ghz"] = round(clk / 1e9, 3)
            ks[k]["mfma_util"] = round(busy[k] / (1024.0 * dur[k] * clk), 4) if clk else None
    return ks


def main():
    src, dst = sys.argv[1], sys.argv[2]
    prov = {}
    if os.path.exists(f"{src}/provenance.json"):  # written on the box by tools/profile_round.sh
        with open(f"{src}/provenance.json") as f:
            prov = json.load(f)
    try:
        import subprocess
        commit = subprocess.run(["git", "rev-parse", "HEAD"], capture_output=True, text=True,
                                check=True).stdout.strip()
        dirty = subprocess.run(["git", "status", "--porcelain", "--", "super-rag_amd/csrc", "include"],
                               capture_output=True, text=True, check=True).stdout.strip()
        commit += "+uncommitted native sources" if dirty else ""
    except Exception:  # noqa: BLE001
        commit = None
    out = {"source": src, "commit": commit, "source_sha256": prov.get("source_sha256"),
           "method": "rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes over "
                     "`bench.py --steps 1 --warmup 1`; FETCH_SIZE x2 (gfx950 correction), "
                     "KiB -> bytes; mean per launch",
           "kernels": kernels_of(src)}
    if os.path.exists(f"{src}/mfma/pmc_1/run_counter_collection.csv"):
        out["method"] += ("; mfma pass: clock = GRBM_GUI_ACTIVE / 8 / duration, mfma_util = "
                          "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration x clock)")
    if os.path.exists(f"{src}/c5/fetch/pmc_1/run_counter_collection.csv"):
        out["workloads"] = {"config5": {
            "command": "bench.py --workload config5 --fp8 3 --steps 1 --warmup 1 --no-cpu-baseline "
                       "--no-extras (the bench line's config5 field: bge-m3 embed, fp8 scan, BM25 + "
                       "rrf, reranker in fp8 mode 3)",
            "kernels": kernels_of(f"{src}/c5")}}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    sections = [("config4", out["kernels"])] + [(w, v["kernels"]) for w, v in out.get("workloads", {}).items()]
    for name, ks in sections:
        print(f"== {name}")
        for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["traffic_B"] * kv[1]["launches"]):
            print(f"{k:32s} launches {v['launches']:5d}  fetch {v['fetch_B'] / 1e6:10.2f} MB  "
                  f"write {v['write_B'] / 1e6:10.2f} MB  per launch  clock {v.get('clock_ghz')} GHz  "
                  f"mfma_util {v.get('mfma_util')}")


if __name__ == "__main__":
    main()
