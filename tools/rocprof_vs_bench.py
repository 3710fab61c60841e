"""Per logical kernel: mean launch duration from the rocprofv3 kernel trace of the bench command vs
the bench's own HIP-event timing of the same command (diagnostic; writes a small text table).

    python tools/rocprof_vs_bench.py gpurun_out/prof_<tag> > profiles/<tag>_rocprof_vs_bench.txt
"""
import csv
import json
import sys
from collections import Counter, defaultdict

from pmc_traffic import logical


def main():
    src = sys.argv[1]
    tot, n = defaultdict(float), Counter()
    with open(f"{src}/trace/run_kernel_trace.csv") as f:
        for r in csv.DictReader(f):
            k = logical(r["Kernel_Name"])
            if k:
                tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
                n[k] += 1
    line = [l for l in open(f"{src}/bench_trace.log") if l.startswith("{")][-1]
    b = json.loads(line)
    print("rocprofv3 --kernel-trace (warmup + timed steps, profiled clock) vs bench.py HIP events "
          "(timed steps), same command")
    print(f"{'kernel':28s} {'rocprof ms':>10s} {'launches':>8s} {'bench ms':>9s} {'launches':>8s} {'ratio':>6s}")
    for k, v in sorted(b["kernels"].items(), key=lambda kv: -kv[1]["ms_per_step"])[:10]:
        bavg = v["ms_per_step"] * b["steps"] / v["launches"]
        r = tot[k] / n[k] if n[k] else float("nan")
        print(f"{k:28s} {r:10.4f} {n[k]:8d} {bavg:9.4f} {v['launches']:8d} {r / bavg:6.3f}")
    split_by_predecessor(f"{src}/trace/run_kernel_trace.csv")


def split_by_predecessor(path, top=6):
    """One logical kernel serves several GEMMs of a layer (the residual + statistics GEMM is both
    the O-projection, after the attention, and FFN2, after FFN1): its launches split by the kernel
    launched before it on the same queue, with the mean duration of each group."""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            k = logical(r["Kernel_Name"])
            if k:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k,
                             r.get("Queue_Id", r.get("Stream_Id", "0"))))
    rows.sort()
    prev, tot, n = {}, defaultdict(float), Counter()
    for t0, t1, k, q in rows:
        key = (k, prev.get(q, "-"))
        tot[key] += (t1 - t0) * 1e-6
        n[key] += 1
        prev[q] = k
    print()
    print("launches split by the kernel before them on the same queue (mean ms, total ms)")
    for key in sorted(tot, key=lambda x: -tot[x])[:top * 2]:
        print(f"{key[0]:28s} after {key[1]:28s} {n[key]:6d} x {tot[key] / n[key]:8.4f} ms = {tot[key]:9.2f} ms")


if __name__ == "__main__":
    main()
