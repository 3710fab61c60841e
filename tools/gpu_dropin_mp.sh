#!/bin/bash
# Drop-in per-request path with N serving processes on one GPU (each process: its own models,
# collection and coalescers; C callers each), measured over the same 10 s window, for every
# N in $DROPIN_PROCS (default "1 2 4") and C in $DROPIN_C (default 64).
# Summary: python tools/dropin_mp_summary.py gpurun_out/dropin_mp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && OUT=${DROPIN_OUT:-gpurun_out/dropin_mp} && mkdir -p $OUT
for c_ in ${DROPIN_C:-64}; do
for np_ in ${DROPIN_PROCS:-1 2 4}; do
  t0=$(python3 -c "import time; print(time.time() + ${DROPIN_DELAY:-75})")
  pids=()
  for i in $(seq 0 $((np_ - 1))); do
    timeout -k 10 240 python -u tools/bench_dropin.py --seconds 10 --concurrency $c_ --start-at "$t0" \
      --rows ${DROPIN_ROWS:-100000} \
      --lat-out $OUT/lat_n${np_}_c${c_}_p${i} \
      > $OUT/n${np_}_c${c_}_p${i}.json 2> $OUT/n${np_}_c${c_}_p${i}.err &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait "$p" || exit 1; done
done
done
