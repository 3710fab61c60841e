# Round-3 final tree, part 1: the driver's own commands (GPU tests, default bench 20 / 5)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r03f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r03f/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03f/smoke.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03f/bench_20x5.log 2>&1 || exit 1
