#!/bin/bash
# kernel trace of the layer-API context decoder (32 layers, ragged 512 rows)
set -o pipefail
TAG=${1:-ctxtr}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
rm -rf /tmp/ctr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ctr -o ctr --output-format csv -- /tmp/cdb 32 1 200 150 100 62 > $OUT/ctx_trace_$TAG.log 2>&1 || { echo "trace failed"; tail -20 $OUT/ctx_trace_$TAG.log; exit 1; }
find /tmp/ctr -name '*kernel_stats.csv' -exec cp {} $OUT/ctx_kernel_stats_$TAG.csv \;
cut -d, -f1-5 $OUT/ctx_kernel_stats_$TAG.csv | head -32
