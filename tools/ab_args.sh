#!/bin/bash
# Same-box A/B of bench.py arguments: tools/ab_args.sh TAG "args1" "args2" ...  (2 interleaved rounds)
TAG=$1; shift
OUT=gpurun_out/abargs_$TAG
mkdir -p $OUT
for round in 1 2; do
  i=0
  for args in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-extras $args \
      > $OUT/a${i}_r$round.log 2>&1 || exit 1
    python - "$OUT/a${i}_r$round.log" "$args" "$round" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = d["kernels"]
top = " ".join(f"{n}={v['ms_per_step']}ms" for n, v in list(k.items())[:6])
print(f"[{sys.argv[2]}] r{sys.argv[3]}: {d['value']} q/s  {top}", flush=True)
PY
  done
done
