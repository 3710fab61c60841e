"""Summary of tools/gpu_dropin_mp.sh: per (processes, callers per process) the total q/s over the
processes sharing one GPU and the POOLED request latency percentiles (every request of every
process), beside Little's law for a closed loop: mean latency = callers in flight / throughput."""
import glob
import json
import os
import re
import sys

import numpy as np

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dropin_mp"
out = {}
for f in sorted(glob.glob(os.path.join(d, "n*_p*.json"))):
    m = re.match(r"n(\d+)(?:_c(\d+))?_p(\d+)\.json", os.path.basename(f))
    n, c, i = int(m.group(1)), int(m.group(2) or 64), int(m.group(3))
    r = json.load(open(f))["runs"][0]
    e = out.setdefault((n, c), {"procs": n, "callers_per_proc": c, "qps": 0.0, "per_proc_qps": [],
                                "rerank_mean_batch": [], "_lat": []})
    e["qps"] = round(e["qps"] + r["qps"], 1)
    e["per_proc_qps"].append(r["qps"])
    e["rerank_mean_batch"].append(r["coalesced"].get("rerank", {}).get("mean_batch"))
    lat = os.path.join(d, f"lat_n{n}_c{c}_p{i}_c{c}.npy")
    if os.path.exists(lat):
        e["_lat"].append(np.load(lat))
res = []
for k in sorted(out):
    e = out.pop(k) if False else out[k]
    lat = np.concatenate(e.pop("_lat")) if e["_lat"] else None
    if lat is not None and lat.size:
        e["p50_ms"] = round(float(np.percentile(lat, 50)), 1)
        e["p99_ms"] = round(float(np.percentile(lat, 99)), 1)
        e["mean_ms"] = round(float(lat.mean()), 1)
    else:
        e.pop("_lat", None)
    e["littles_law_mean_ms"] = round(1e3 * e["procs"] * e["callers_per_proc"] / max(e["qps"], 1e-9), 1)
    res.append(e)
print(json.dumps(res, indent=1))
