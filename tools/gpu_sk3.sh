#!/bin/bash
# stream-K with sibling row tiles: tests, then the ragged context bench with stream-K off / on
# gate_up only / on gate_up + q/k/v, then kernel stats for the last
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_context_ops.py -k "stream_k or residual or ffn" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_sk3.log 2>&1
rc=$?; tail -2 $OUT/pytest_sk3.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_sk3.log | head; exit $rc; }
LLMI_SK_LINEAR=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_context_ops.py -k "stream_k or proj" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_sk3b.log 2>&1
rc=$?; tail -2 $OUT/pytest_sk3b.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_sk3b.log | head; exit $rc; }
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/ctx_bench_sk3.jsonl
for pass in 1 2; do
  for v in "0 0" "1 0" "1 1"; do
    set -- $v
    LLMI_SK=$1 LLMI_SK_LINEAR=$2 timeout -k 10 120 /tmp/cdb 32 3 200 150 100 62 | sed "s/^{/{\"sk\": $1, \"sk_linear\": $2, /" >> $OUT/ctx_bench_sk3.jsonl || exit 1
  done
done
cat $OUT/ctx_bench_sk3.jsonl
rm -rf /tmp/ctr
LLMI_SK_LINEAR=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ctr -o ctr --output-format csv -- /tmp/cdb 32 1 200 150 100 62 > $OUT/ctx_trace_sk3.log 2>&1 || exit 1
find /tmp/ctr -name '*kernel_stats.csv' -exec cp {} $OUT/ctx_kernel_stats_sk3.csv \;
grep gemm3 $OUT/ctx_kernel_stats_sk3.csv | cut -d, -f1-4
