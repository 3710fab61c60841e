cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/qa_diag
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/qa_diag/base.log 2>&1 || exit 1
SR_QA_DIAG=2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/qa_diag/noattn.log 2>&1 || exit 1
SR_QA_DIAG=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/qa_diag/noloop.log 2>&1 || exit 1
