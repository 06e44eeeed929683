#!/bin/bash
# context-decoder session: ctx tests, the ragged timing both ways, then a kernel trace
set -o pipefail
TAG=${1:-ctx2}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
fatal() { case $1 in 0|1) return 1;; *) echo "fatal rc $1 at $2"; return 0;; esac; }
echo "[$(date +%T)] pytest ctx"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ctx_history.py tests/test_gpu_context_ops.py tests/test_cpp_api.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_ctx_$TAG.log 2>&1
rc=$?; grep -E "FAILED|ERROR|rel-L2|passed|failed| us" $OUT/pytest_ctx_$TAG.log | tail -40
fatal $rc pytest_ctx && exit $rc
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/ctx_bench_$TAG.jsonl
for uf in 0 1 0; do
  for lens in "512" "200 150 100 62"; do
    LLMI_CTX_UNFUSED=$uf timeout -k 10 120 /tmp/cdb 32 3 $lens >> $OUT/ctx_bench_$TAG.jsonl; rc=$?
    fatal $rc ctx_bench && exit $rc
  done
done
cat $OUT/ctx_bench_$TAG.jsonl
rm -rf /tmp/ctr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ctr -o ctr --output-format csv -- /tmp/cdb 32 1 200 150 100 62 > $OUT/ctx_trace_$TAG.log 2>&1 || { echo "trace failed"; tail -20 $OUT/ctx_trace_$TAG.log; exit 1; }
find /tmp/ctr -name '*kernel_stats.csv' -exec cp {} $OUT/ctx_kernel_stats_$TAG.csv \;
find /tmp/ctr -name '*kernel_trace.csv' -exec cp {} $OUT/ctx_kernel_trace_$TAG.csv \;
cut -d, -f1-4 $OUT/ctx_kernel_stats_$TAG.csv | head -24
echo "[$(date +%T)] done"
