"""Summary of tools/gpu_dropin_mp.sh: total q/s over the processes sharing one GPU, per process count."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dropin_mp"
out = {}
for f in sorted(glob.glob(os.path.join(d, "n*_p*.json"))):
    n = int(os.path.basename(f).split("_")[0][1:])
    r = json.load(open(f))["runs"][0]
    e = out.setdefault(n, {"procs": n, "qps": 0.0, "per_proc_qps": [], "p50_ms": [], "p99_ms": [],
                           "rerank_mean_batch": []})
    e["qps"] = round(e["qps"] + r["qps"], 1)
    e["per_proc_qps"].append(r["qps"])
    e["p50_ms"].append(r["p50_ms"])
    e["p99_ms"].append(r["p99_ms"])
    e["rerank_mean_batch"].append(r["coalesced"].get("rerank", {}).get("mean_batch"))
print(json.dumps([out[k] for k in sorted(out)], indent=1))
