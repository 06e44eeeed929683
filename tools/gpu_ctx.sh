#!/bin/bash
# context-layer session: ctx history tests (fused + unfused), then the 512-row ragged timing both ways
set -o pipefail
TAG=${1:-ctx}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
echo "[$(date +%T)] pytest ctx"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ctx_history.py tests/test_gpu_context_ops.py tests/test_cpp_api.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_ctx_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|rel-L2|passed|failed" $OUT/pytest_ctx_$TAG.log | tail -40
[ $rc -eq 0 ] || { tail -40 $OUT/pytest_ctx_$TAG.log; exit $rc; }
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/ctx_bench_$TAG.jsonl
for uf in 0 1 0 1; do
  for lens in "512" "200 150 100 62"; do
    LLMI_CTX_UNFUSED=$uf timeout -k 10 120 /tmp/cdb 32 3 $lens >> $OUT/ctx_bench_$TAG.jsonl || { echo "bench failed"; exit 1; }
  done
done
cat $OUT/ctx_bench_$TAG.jsonl
echo "[$(date +%T)] done"
