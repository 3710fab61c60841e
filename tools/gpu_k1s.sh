cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/k1s
timeout -k 10 400 python -u -m pytest tests/test_gpu_store.py -x -v --timeout 200 --timeout-method thread > gpurun_out/k1s/store_tests.log 2>&1 || exit 1
SR_SCAN_STREAM=0 timeout -k 10 200 python -u tools/bench_search_fp8.py --steps 5 > gpurun_out/k1s/search_gemm.json 2>gpurun_out/k1s/search_gemm.err || exit 1
SR_SCAN_STREAM=1 timeout -k 10 200 python -u tools/bench_search_fp8.py --steps 5 > gpurun_out/k1s/search_stream.json 2>gpurun_out/k1s/search_stream.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k1s/trace -o run -- python3 tools/bench_search_fp8.py --steps 3 > gpurun_out/k1s/trace.log 2>&1 || exit 1
python3 tools/k1_schedule.py gpurun_out/k1s/trace > gpurun_out/k1s/chunks.json
SR_SCAN_STREAM=1 timeout -k 10 200 python -u tools/bench_search_fp8.py --rows 131072 --steps 20 > gpurun_out/k1s/search_stream_l3.json 2>&1 || exit 1
SR_SCAN_STREAM=0 timeout -k 10 200 python -u tools/bench_search_fp8.py --rows 131072 --steps 20 > gpurun_out/k1s/search_gemm_l3.json 2>&1 || exit 1
