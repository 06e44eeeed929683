#!/bin/bash
# residual-norm block size A/B on the context decoder (LLMI_RN256=1: 256 threads)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_context_ops.py -k "residual" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_rn.log 2>&1
rc=$?; tail -2 $OUT/pytest_rn.log; [ $rc -eq 0 ] || exit $rc
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/ctx_bench_rn.jsonl
for v in 0 1 0 1 0 1; do
  LLMI_RN256=$v timeout -k 10 120 /tmp/cdb 32 3 200 150 100 62 | sed "s/^{/{\"rn256\": $v, /" >> $OUT/ctx_bench_rn.jsonl || exit 1
done
cat $OUT/ctx_bench_rn.jsonl
rm -rf /tmp/ctr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ctr -o ctr --output-format csv -- /tmp/cdb 32 1 200 150 100 62 > $OUT/ctx_trace_rn.log 2>&1 || exit 1
find /tmp/ctr -name '*kernel_stats.csv' -exec cp {} $OUT/ctx_kernel_stats_rn.csv \;
grep resid $OUT/ctx_kernel_stats_rn.csv | cut -d, -f1-4
