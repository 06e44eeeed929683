#!/bin/bash
# end-of-round prefill / context evidence: fp8-lo gate_up balance vs stream-K, prefill kernel
# traces (exact and fp8-lo), the context decoder bench fused vs unfused
set -o pipefail
TAG=${1:-fin}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/pf_skf8_$TAG.jsonl
for pass in 1 2; do
  for v in 0 1; do
    r=$(LLMI_SK_F8=$v timeout -k 10 200 python -u tools/prefill_probe.py 512 5 2> $OUT/pf_skf8.err) || { tail -5 $OUT/pf_skf8.err; exit 1; }
    echo "{\"sk_f8\": $v, \"r\": $r}" | tee -a $OUT/pf_skf8_$TAG.jsonl
  done
done
for mode in exact exact8; do
  rm -rf /tmp/pft
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pft -o pf --output-format csv -- python3 tools/prefill_probe.py 512 2 $mode > $OUT/pf_trace_${mode}_$TAG.log 2>&1 || { echo "trace $mode failed"; exit 1; }
  find /tmp/pft -name '*kernel_stats.csv' -exec cp {} $OUT/pf_kernel_stats_${mode}_$TAG.csv \;
done
g++ -std=c++17 -O2 -I include tools/ctx_decoder_bench.cpp -L llm-inference_amd/lib -lllmi -Wl,-rpath,$PWD/llm-inference_amd/lib -o /tmp/cdb || exit 1
: > $OUT/ctx_bench_$TAG.jsonl
for uf in 0 1 0; do
  for lens in "512" "200 150 100 62"; do
    LLMI_CTX_UNFUSED=$uf timeout -k 10 120 /tmp/cdb 32 3 $lens >> $OUT/ctx_bench_$TAG.jsonl || exit 1
  done
done
cat $OUT/ctx_bench_$TAG.jsonl
rm -rf /tmp/ctr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ctr -o ctr --output-format csv -- /tmp/cdb 32 1 200 150 100 62 > $OUT/ctx_trace_$TAG.log 2>&1 || exit 1
find /tmp/ctr -name '*kernel_stats.csv' -exec cp {} $OUT/ctx_kernel_stats_$TAG.csv \;
echo done
