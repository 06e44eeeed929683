#!/bin/bash
# stream-K session: its tests first, then the context suite, then the ragged context bench
# with and without stream-K (LLMI_SK=0), then a kernel trace
set -o pipefail
TAG=${1:-sk}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] stream-K tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_context_ops.py -k "stream_k" -x -v -s -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_sk_$TAG.log 2>&1
rc=$?; grep -E "PASSED|FAILED|rel-L2|passed|failed|Error" $OUT/pytest_sk_$TAG.log | tail -12
[ $rc -eq 0 ] || { tail -30 $OUT/pytest_sk_$TAG.log; exit $rc; }
echo "[$(date +%T)] context suite"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ctx_history.py tests/test_gpu_context_ops.py tests/test_cpp_api.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_ctx_$TAG.log 2>&1
rc=$?; tail -3 $OUT/pytest_ctx_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_ctx_$TAG.log | head; exit $rc; }
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/ctx_bench_$TAG.jsonl
for sk in 1 0 1 0; do
  for lens in "512" "200 150 100 62"; do
    LLMI_SK=$sk timeout -k 10 120 /tmp/cdb 32 3 $lens | sed "s/^{/{\"sk\": $sk, /" >> $OUT/ctx_bench_$TAG.jsonl || exit 1
  done
done
cat $OUT/ctx_bench_$TAG.jsonl
rm -rf /tmp/ctr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ctr -o ctr --output-format csv -- /tmp/cdb 32 1 200 150 100 62 > $OUT/ctx_trace_$TAG.log 2>&1 || { echo "trace failed"; exit 1; }
find /tmp/ctr -name '*kernel_stats.csv' -exec cp {} $OUT/ctx_kernel_stats_$TAG.csv \;
find /tmp/ctr -name '*kernel_trace.csv' -exec cp {} $OUT/ctx_kernel_trace_$TAG.csv \;
cut -d, -f1-4 $OUT/ctx_kernel_stats_$TAG.csv | head -12
echo "[$(date +%T)] done"
