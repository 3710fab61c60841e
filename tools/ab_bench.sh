#!/bin/bash
# Same-box A/B of library builds / settings: tools/ab_bench.sh TAG spec1 spec2 ...
# spec = path/to/lib.so[@VAR=VALUE[,VAR2=VALUE2]]; interleaved, 2 rounds; each run:
# bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras $AB_BENCH_ARGS with SUPER_RAG_AMD_LIB=path.
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
for round in 1 2; do
  for spec in "$@"; do
    lib=${spec%%@*}
    envs=""
    [[ "$spec" == *@* ]] && envs=${spec#*@}
    name=$(basename $lib .so)${envs:+_${envs//[=,]/_}}
    env SUPER_RAG_AMD_LIB=$lib ${envs//,/ } timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 \
      --no-cpu-baseline --no-extras $AB_BENCH_ARGS > $OUT/${name}_r$round.log 2>&1 || exit 1
    python - "$OUT/${name}_r$round.log" "$name" "$round" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["kernels"]
top = " ".join(f"{n}={v.get('tflops', v.get('gbs'))}" for n, v in list(k.items())[:5])
print(f"{sys.argv[2]} r{sys.argv[3]}: {d['value']} q/s  {top}", flush=True)
PY
  done
done
