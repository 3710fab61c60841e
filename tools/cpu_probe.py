"""Probe the GPU box's host CPU: core counts, model, fp32 GEMM rate at several thread counts."""
import os, time, json, platform
import torch
out = {"cpu_count": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)),
       "omp": os.environ.get("OMP_NUM_THREADS"), "torch_threads": torch.get_num_threads()}
try:
    with open("/proc/cpuinfo") as f:
        out["model"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
except Exception as e:
    out["model"] = str(e)
try:
    with open("/sys/fs/cgroup/cpu.max") as f:
        out["cgroup_cpu_max"] = f.read().strip()
except Exception as e:
    out["cgroup_cpu_max"] = None
a = torch.randn(4096, 768); b = torch.randn(768, 65536)
for t in sorted({8, 16, 32, out["affinity"]}):
    torch.set_num_threads(t)
    a @ b
    t0 = time.perf_counter(); n = 5
    for _ in range(n):
        a @ b
    dt = (time.perf_counter() - t0) / n
    out[f"gemm_tflops_{t}thr"] = round(2 * 4096 * 768 * 65536 / dt / 1e12, 3)
print(json.dumps(out))
