#!/bin/bash
# Round-6 GPU validation, tag $1, parts $2 (comma list):
#   c3     test_config3 with its printed error figures (-s)
#   tests  the whole -m gpu suite
#   smoke  __graft_entry__.smoke()
#   bench  the driver's default bench (20 / 5)
#   dropin tools/gpu_dropin_mp.sh ($DROPIN_PROCS x $DROPIN_C) + its pooled summary
#   prof   tools/profile_round.sh (rocprofv3 trace + PMC, config 4 and config 5's fp8 path)
TAG=${1:?tag}; PARTS=${2:-tests,smoke,bench}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/$TAG
for P in ${PARTS//,/ }; do
  case $P in
    stats) timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -k "stats" -v -s --timeout 240 --timeout-method thread > gpurun_out/$TAG/stats.log 2>&1 || exit 1 ;;
    embedsm) for B in ${EMB_B:-1 8 32 256}; do
               timeout -k 10 200 python -u tools/embed_profile.py --batch $B --reps 30 > gpurun_out/$TAG/embed_profile_b$B.json 2> gpurun_out/$TAG/embed_profile_b$B.err || exit 1
             done ;;
    enct) timeout -k 10 400 python -u -m pytest tests/test_gpu_encoder.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/enc_tests.log 2>&1 || exit 1 ;;
    embedab) L=$PWD/super-rag_amd/super_rag_amd/lib_ab
         for V in ${VARS:?VARS}; do for B in ${EMB_B:-8 256}; do
           if [ $V = prod ]; then E=""; else E="SUPER_RAG_AMD_LIB=$L/libsrmi_$V.so SUPER_RAG_AMD_DIAG_LIB=$L/libsrmi_diag_$V.so"; fi
           env $E timeout -k 10 200 python -u tools/embed_profile.py --batch $B --reps 30 > gpurun_out/$TAG/embed_${V}_b$B.json 2> gpurun_out/$TAG/embed_${V}_b$B.err || exit 1
         done; done ;;
    dmp) L=$PWD/super-rag_amd/super_rag_amd/lib_ab
         for V in ${VARS:?VARS}; do
           if [ $V = prod ]; then E=""; else E="SUPER_RAG_AMD_LIB=$L/libsrmi_$V.so SUPER_RAG_AMD_DIAG_LIB=$L/libsrmi_diag_$V.so"; fi
           env $E DROPIN_PROCS=4 DROPIN_C=32 DROPIN_ROWS=${DROPIN_ROWS:-10000000} DROPIN_OUT=gpurun_out/$TAG/dmp_$V \
             timeout -k 10 400 bash tools/gpu_dropin_mp.sh || exit 1
         done ;;
    c5ab) L=$PWD/super-rag_amd/super_rag_amd/lib_ab
         for V in ${VARS:?VARS}; do
           if [ $V = prod ]; then E=""; else E="SUPER_RAG_AMD_LIB=$L/libsrmi_$V.so SUPER_RAG_AMD_DIAG_LIB=$L/libsrmi_diag_$V.so"; fi
           env $E timeout -k 10 400 python -u bench.py --workload config5 --fp8 3 --steps 10 --warmup 3 --no-extras > gpurun_out/$TAG/c5ab_$V.log 2>&1 || exit 1
           tail -n 1 gpurun_out/$TAG/c5ab_$V.log >> gpurun_out/$TAG/c5ab_all.jsonl
         done ;;
    restests) timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_rerank_fidelity.py tests/test_gpu_rerank_fidelity_v2m3.py tests/test_gpu_configs.py tests/test_gpu_encoder.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/restests.log 2>&1 || exit 1 ;;
    hostcost) timeout -k 10 200 python -u tools/embed_host_cost.py > gpurun_out/$TAG/embed_host_cost.log 2>&1 || exit 1 ;;
    gilab) for G in ${GILS:-0 0.5}; do
             SUPER_RAG_AMD_GIL_SWITCH_MS=$G timeout -k 10 400 python -u tools/bench_dropin.py --rows 10000000 --concurrency 64 --seconds 10 \
               > gpurun_out/$TAG/d1_gil$G.json 2> gpurun_out/$TAG/d1_gil$G.err || exit 1
             SUPER_RAG_AMD_GIL_SWITCH_MS=$G DROPIN_PROCS=4 DROPIN_C=32 DROPIN_ROWS=10000000 DROPIN_DELAY=100 \
               DROPIN_OUT=gpurun_out/$TAG/dmp_gil$G timeout -k 10 400 bash tools/gpu_dropin_mp.sh || exit 1
           done ;;
    tokab) for T in ${TOKS:-1 0}; do
             SUPER_RAG_AMD_TOK_SLOW=$T timeout -k 10 400 python -u tools/bench_dropin.py --rows 10000000 --concurrency 64 --seconds 10 \
               > gpurun_out/$TAG/d1_tok$T.json 2> gpurun_out/$TAG/d1_tok$T.err || exit 1
             SUPER_RAG_AMD_TOK_SLOW=$T DROPIN_PROCS=4 DROPIN_C=32 DROPIN_ROWS=10000000 DROPIN_DELAY=100 \
               DROPIN_OUT=gpurun_out/$TAG/dmp_tok$T timeout -k 10 400 bash tools/gpu_dropin_mp.sh || exit 1
           done ;;
    fillab) for F in ${FILLS:-1:0 12:10 16:20}; do
             MF=${F%%:*}; MW=${F##*:}
             SUPER_RAG_AMD_RERANK_MIN_FILL=$MF SUPER_RAG_AMD_RERANK_MAX_WAIT_MS=$MW DROPIN_PROCS=4 DROPIN_C=32 DROPIN_ROWS=10000000 \
               DROPIN_DELAY=100 DROPIN_OUT=gpurun_out/$TAG/dmp_fill${MF}_${MW} timeout -k 10 400 bash tools/gpu_dropin_mp.sh || exit 1
           done ;;
    fill1) for F in ${FILLS:-1:0 16:20}; do
             MF=${F%%:*}; MW=${F##*:}
             SUPER_RAG_AMD_RERANK_MIN_FILL=$MF SUPER_RAG_AMD_RERANK_MAX_WAIT_MS=$MW timeout -k 10 400 python -u tools/bench_dropin.py \
               --rows 10000000 --concurrency 64 --seconds 10 > gpurun_out/$TAG/d1_fill${MF}_${MW}.json 2> gpurun_out/$TAG/d1_fill${MF}_${MW}.err || exit 1
           done ;;
    spliterr) timeout -k 10 600 python -u tools/embed_split_error.py > gpurun_out/$TAG/embed_split_error.log 2>&1 || exit 1 ;;
    embedprof) timeout -k 10 200 python -u tools/embed_profile.py > gpurun_out/$TAG/embed_profile.json 2> gpurun_out/$TAG/embed_profile.err || exit 1 ;;
    xstag) for S in ${XSTAG:-0 -4 -8 -11 -16 0}; do
             echo "== stagger $S" >> gpurun_out/$TAG/xstag.log
             SR_GEMM_STAGGER=$S timeout -k 10 200 python -u tools/ffn1_bench.py --M 1638400 --diags 0 --rounds 3 >> gpurun_out/$TAG/xstag.log 2>&1 || exit 1
           done ;;
    f8ab) L=$PWD/super-rag_amd/super_rag_amd
          for r in 1 2; do for D in $L/lib/libsrmi_diag.so $L/lib_ab/libsrmi_diag_${F8AB:-interp}.so; do
            echo "== $(basename $D) r$r" >> gpurun_out/$TAG/f8ab.log
            SUPER_RAG_AMD_DIAG_LIB=$D timeout -k 10 200 python -u tools/ffn1_bench.py --f8 --M 1638400 --diags 0 --rounds 2 >> gpurun_out/$TAG/f8ab.log 2>&1 || exit 1
          done; done ;;
    lnrab) L=$PWD/super-rag_amd/super_rag_amd/lib_ab; V=${VAR:?VAR}
         SUPER_RAG_AMD_DIAG_LIB=$L/libsrmi_diag_$V.so timeout -k 10 300 python -u tools/lnr_stamps.py > gpurun_out/$TAG/lnr_stamps_$V.log 2>&1 || exit 1
         SUPER_RAG_AMD_LIB=$L/libsrmi_$V.so SUPER_RAG_AMD_DIAG_LIB=$L/libsrmi_diag_$V.so timeout -k 10 300 \
           python -u -m pytest tests/test_gpu_gemm.py -k stats -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG/stats_$V.log 2>&1 || exit 1
         SUPER_RAG_AMD_LIB=$L/libsrmi_$V.so SUPER_RAG_AMD_DIAG_LIB=$L/libsrmi_diag_$V.so timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench_20x5_$V.log 2>&1 || exit 1 ;;
    benchab) L=$PWD/super-rag_amd/super_rag_amd/lib_ab
         for V in ${VARS:?VARS}; do
           if [ $V = prod ]; then E=""; else E="SUPER_RAG_AMD_LIB=$L/libsrmi_$V.so SUPER_RAG_AMD_DIAG_LIB=$L/libsrmi_diag_$V.so"; fi
           env $E timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-extras > gpurun_out/$TAG/benchab_$V.log 2>&1 || exit 1
           tail -n 1 gpurun_out/$TAG/benchab_$V.log >> gpurun_out/$TAG/benchab_all.jsonl
         done ;;
    lnrst) timeout -k 10 300 python -u tools/lnr_stamps.py > gpurun_out/$TAG/lnr_stamps.log 2>&1 || exit 1 ;;
    peaks) timeout -k 10 200 python -u -c "import torch, json, bench; print(json.dumps(bench.mfma_rate_peaks(torch.device('cuda', 0))))" > gpurun_out/$TAG/peaks.log 2>&1 || exit 1 ;;
    c3) timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k config3 -x -v -s --timeout 240 --timeout-method thread > gpurun_out/$TAG/c3.log 2>&1 || exit 1 ;;
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/$TAG/gpu_tests.log 2>&1 || exit 1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit 1 ;;
    bench) timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench_20x5.log 2>&1 || exit 1 ;;
    modes) for M in 3; do
             timeout -k 10 300 python -u bench.py --fp8 $M --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/$TAG/bench_fp8m$M.log 2>&1 || exit 1
             timeout -k 10 400 python -u bench.py --workload config5 --fp8 $M --steps 10 --warmup 3 --no-extras > gpurun_out/$TAG/bench_c5_fp8m$M.log 2>&1 || exit 1
           done ;;
    prof) rm -rf gpurun_out/prof_$TAG && bash tools/profile_round.sh $TAG > gpurun_out/$TAG/profile_round.log 2>&1 || exit 1
          python3 tools/pmc_traffic.py gpurun_out/prof_$TAG gpurun_out/$TAG/${TAG}_pmc_traffic.json > gpurun_out/$TAG/pmc_traffic.log 2>&1 || exit 1
          python3 tools/rocprof_vs_bench.py gpurun_out/prof_$TAG > gpurun_out/$TAG/rocprof_vs_bench.txt 2>&1 || exit 1
          (cd tools && python3 -c "import sys; from rocprof_vs_bench import split_by_predecessor as s; s(sys.argv[1])" \
             ../gpurun_out/prof_$TAG/c5/trace/run_kernel_trace.csv) > gpurun_out/$TAG/c5_split.txt 2>&1 || exit 1
          cp gpurun_out/prof_$TAG/trace/run_kernel_stats.csv gpurun_out/$TAG/${TAG}_rocprof_kernel_stats.csv
          cp gpurun_out/prof_$TAG/c5/trace/run_kernel_stats.csv gpurun_out/$TAG/${TAG}_c5_rocprof_kernel_stats.csv 2>/dev/null
          find gpurun_out/prof_$TAG -name "*.csv" -size +1M -delete ;;
    ffn1) timeout -k 10 300 python -u tools/ffn1_bench.py --diags ${FFN1_DIAGS:-0,2} --rounds 3 > gpurun_out/$TAG/ffn1.log 2>&1 || exit 1
          timeout -k 10 300 python -u tools/ffn1_bench.py --M 1638400 --diags ${FFN1_DIAGS:-0,2} --rounds 3 > gpurun_out/$TAG/ffn1_1638k.log 2>&1 || exit 1 ;;
    stamps) timeout -k 10 300 python -u tools/ffn1_stamps.py > gpurun_out/$TAG/ffn1_stamps.log 2>&1 || exit 1 ;;
    k5cst) timeout -k 10 300 python -u tools/k5c_stamps.py > gpurun_out/$TAG/k5c_stamps.log 2>&1 || exit 1 ;;
    v5) SUPER_RAG_AMD_LIB=$PWD/super-rag_amd/super_rag_amd/lib/libsrmi_diag.so timeout -k 10 400 python -u bench.py --workload config5 --fp8 5 --steps 10 --warmup 3 --no-extras > gpurun_out/$TAG/bench_c5_fp8m5_diaglib.log 2>&1 || exit 1 ;;
    ab) L=super-rag_amd/super_rag_amd/lib_ab
        timeout -k 10 900 bash tools/ab_bench.sh $TAG ${AB_LIBS:-$L/libsrmi_base.so $L/libsrmi_cstl.so $L/libsrmi_rpf.so} > gpurun_out/$TAG/ab.log 2>&1 || exit 1 ;;
    dropin) rm -rf gpurun_out/dropin_mp && timeout -k 10 1000 bash tools/gpu_dropin_mp.sh || exit 1
            python3 tools/dropin_mp_summary.py gpurun_out/dropin_mp > gpurun_out/$TAG/dropin_mp.txt 2>&1 || exit 1 ;;
    v2ab) D=$PWD/super-rag_amd/super_rag_amd/lib/libsrmi_diag.so
          for r in 1 2; do for hg in 0 16 4; do
            env SUPER_RAG_AMD_LIB=$D $( [ $hg -gt 0 ] && echo SR_QA_HGROUP=$hg ) timeout -k 10 300 \
              python -u tools/v2m3_bench.py --v2m3-steps 3 > gpurun_out/$TAG/v2m3_hg${hg}_r$r.log 2>&1 || exit 1
            echo "hg=$hg r$r $(tail -1 gpurun_out/$TAG/v2m3_hg${hg}_r$r.log)" >> gpurun_out/$TAG/v2ab.txt
          done; done ;;
    var) L=$PWD/super-rag_amd/super_rag_amd/lib_ab; V=${VAR:?VAR}
         SUPER_RAG_AMD_LIB=$L/libsrmi_$V.so SUPER_RAG_AMD_DIAG_LIB=$L/libsrmi_diag_$V.so timeout -k 10 400 \
           python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_ffn1_epilogue.py tests/test_gpu_encoder.py \
           tests/test_gpu_rerank_fidelity.py tests/test_gpu_rerank_fidelity_v2m3.py tests/test_gpu_configs.py \
           tests/test_gpu_fused_attention.py -x -q \
           --timeout 240 --timeout-method thread > gpurun_out/$TAG/var_tests_$V.log 2>&1 || exit 1
         [ "${VAR_FFN1:-1}" = 1 ] && for r in 1 2; do for D in $PWD/super-rag_amd/super_rag_amd/lib/libsrmi_diag.so $L/libsrmi_diag_$V.so; do
           echo "== $(basename $D) r$r" >> gpurun_out/$TAG/var_ffn1_$V.log
           SUPER_RAG_AMD_DIAG_LIB=$D timeout -k 10 300 python -u tools/ffn1_bench.py --diags 0,2 --rounds 2 $VAR_FFN1_ARGS \
             >> gpurun_out/$TAG/var_ffn1_$V.log 2>&1 || exit 1
         done; done; true ;;
    gloo2) timeout -k 10 600 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-extras \
             --no-cpu-baseline > gpurun_out/$TAG/bench_2rank_gloo.log 2>&1 || exit 1 ;;
    dprof) timeout -k 10 400 python -u tools/bench_dropin.py --profile --profile-concurrency 64 --seconds 10 \
             > gpurun_out/$TAG/dropin_profile_c64.txt 2>&1 || exit 1
           timeout -k 10 400 python -u tools/bench_dropin.py --profile --profile-concurrency 1 --seconds 10 \
             > gpurun_out/$TAG/dropin_profile_c1.txt 2>&1 || exit 1 ;;
    d1) timeout -k 10 400 python -u tools/bench_dropin.py --concurrency 64 256 --seconds 10 \
          > gpurun_out/$TAG/dropin_1proc.json 2> gpurun_out/$TAG/dropin_1proc.err || exit 1 ;;
    ffn1t) timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn1_epilogue.py -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG/ffn1_tests.log 2>&1 || exit 1 ;;
    *) echo "unknown part $P"; exit 2 ;;
  esac
done
exit 0
