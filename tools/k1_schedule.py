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


def calls(trace_dir):
    f = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    out, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "normalize_rows" in name:
            cur = []
            out.append(cur)
        elif cur is not None and ("cosine_scan" in name or "topk_select" in name or "rescore" in name):
            short = ("scan8" if "scan8" in name or "f8" in name else "scan") if "scan" in name else \
                    ("select" if "select" in name else "rescore")
            cur.append((short, round(us, 1)))
    return out


if __name__ == "__main__":
    res = {d: calls(d)[-4:] for d in sys.argv[1:]}
    print(json.dumps(res, indent=1))
