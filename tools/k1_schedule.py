"""Per-chunk K1 timings from a rocprofv3 kernel trace (diagnostic).

    rocprofv3 --kernel-trace -d gpurun_out/k1g8 -o run -- python3 tools/bench_search_fp8.py --steps 3
    python tools/k1_schedule.py gpurun_out/k1g8 [...]

Prints, per trace, the durations of the cosine_scan / cosine_scan8 dispatches in launch order
grouped per search call (a call = the dispatches between two normalize_rows launches), so the
chunk schedule (rows per chunk) can be read next to the per-chunk time."""
import csv
import glob
import json
import os
import sys


def _rows(trace_dir):
    """(name, start, end) of every dispatch: the CSV kernel trace, or the rocpd database
    (rocprofv3's default output format on ROCm 7.2)."""
    f = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if f:
        return [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in csv.DictReader(open(f[0]))]
    import sqlite3
    db = glob.glob(os.path.join(trace_dir, "**", "*.db"), recursive=True)[0]
    return list(sqlite3.connect(db).execute("select name, start, end from kernels"))


def calls(trace_dir):
    """Per search call (dispatches after a normalize_rows): the scan dispatches (the dense first
    chunk, then the threshold chunks on the GEMM main loop) as (kind, microseconds)."""
    out, cur = [], None
    for name, t0, t1 in sorted(_rows(trace_dir), key=lambda r: r[1]):
        us = (t1 - t0) / 1e3
        if "normalize_rows" in name:
            cur = []
            out.append(cur)
        elif cur is not None and ("cosine_scan" in name or "gemm_pipe" in name or "cosine_stream" in name):
            cur.append(("dense" if "cosine_scan" in name else "chunk", round(us, 1)))
    return out


if __name__ == "__main__":
    res = {d: calls(d) for d in sys.argv[1:]}
    print(json.dumps(res, indent=1))
