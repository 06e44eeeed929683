#!/bin/bash
# kernel trace of the fp8-lo prefill (512 rows, 2 iterations):  bash tools/gpu_pf_trace.sh <tag>
set -o pipefail
TAG=${1:-pf}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
rm -rf /tmp/pf8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pf8 -o pf --output-format csv -- python3 tools/prefill_probe.py 512 2 exact8 > $OUT/pf8_trace_$TAG.log 2>&1 || { echo "pf8 trace failed $?"; tail -20 $OUT/pf8_trace_$TAG.log; exit 1; }
find /tmp/pf8 -name '*kernel_stats.csv' -exec cp {} $OUT/pf8_kernel_stats_$TAG.csv \;
cut -d, -f1-8 $OUT/pf8_kernel_stats_$TAG.csv | head -30
