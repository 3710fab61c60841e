#!/bin/bash
# Round-4 GPU step: tools/gpu_r04.sh TAG "pytest files" [ab libs...]
#   parity subset first (-x), then same-box A/B of library builds (tools/ab_bench.sh).
TAG=${1:?tag}; TESTS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 240 --timeout-method thread \
    > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
  tail -3 gpurun_out/$TAG/tests.log
fi
if [ $# -gt 0 ]; then
  bash tools/ab_bench.sh $TAG "$@" || exit 1
fi
exit 0
