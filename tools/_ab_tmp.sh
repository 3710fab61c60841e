set -o pipefail
bash tools/ab_bench.sh lg ab/libsrmi_head.so ab/libsrmi_linegelu.so ab/libsrmi_prio.so
