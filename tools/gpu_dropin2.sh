cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/dropin7
timeout -k 10 400 python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_flow.py -x -q --timeout 250 --timeout-method thread > gpurun_out/dropin7/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_dropin.py --seconds 10 > gpurun_out/dropin7/dropin.json 2>gpurun_out/dropin7/dropin.err || exit 1
timeout -k 10 300 python -u tools/bench_dropin.py --profile --seconds 8 > gpurun_out/dropin7/profile.log 2>&1 || exit 1
