#!/bin/bash
# stream-K on gate_up: prefill tests, then prefill timing exact / fp8-lo with and without it,
# then the context decoder bench with and without it
set -o pipefail
TAG=${1:-sk2}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] prefill + context tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_prefill.py tests/test_gpu_context_ops.py tests/test_gpu_ctx_history.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_sk2_$TAG.log 2>&1
rc=$?; tail -3 $OUT/pytest_sk2_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_sk2_$TAG.log | head; exit $rc; }
LLMI_SK_F8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_prefill.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_sk2f8_$TAG.log 2>&1
rc=$?; tail -2 $OUT/pytest_sk2f8_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/pytest_sk2f8_$TAG.log | head; exit $rc; }
: > $OUT/pf_sk_$TAG.jsonl
for pass in 1 2; do
  for v in "1 0" "0 0" "1 1"; do
    set -- $v
    r=$(LLMI_SK=$1 LLMI_SK_F8=$2 timeout -k 10 200 python -u tools/prefill_probe.py 512 5 2> $OUT/pf_sk.err) || { echo "probe failed"; tail -5 $OUT/pf_sk.err; exit 1; }
    echo "{\"sk\": $1, \"sk_f8\": $2, \"r\": $r}" | tee -a $OUT/pf_sk_$TAG.jsonl
  done
done
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/ctx_bench_$TAG.jsonl
for sk in 1 0 1 0; do
  LLMI_SK=$sk timeout -k 10 120 /tmp/cdb 32 3 200 150 100 62 | sed "s/^{/{\"sk\": $sk, /" >> $OUT/ctx_bench_$TAG.jsonl || exit 1
done
cat $OUT/ctx_bench_$TAG.jsonl
echo "[$(date +%T)] done"
