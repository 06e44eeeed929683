#!/bin/bash
# Round-3 measurement session (one gpurun call): bench line, eager kernel trace of the
# bench, FETCH/WRITE PMC passes on the 7B fp16 and the 13B int8 decode kernels, the
# two-process one-shot exchange latency.   bash tools/gpu_r03.sh <tag>
set -o pipefail
TAG=${1:-r03}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step bench
timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
step "kernel trace (eager bench)"
rm -rf /tmp/prof_trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace -o trace --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-side --eager > $OUT/prof_trace_$TAG.log 2>&1 || { echo "trace failed $?"; tail -20 $OUT/prof_trace_$TAG.log; exit 1; }
find /tmp/prof_trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$TAG.csv \;
step "pmc fetch 7B"
rm -rf /tmp/pmc_f /tmp/pmc_w /tmp/pmc_fi /tmp/pmc_wi
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'gemv_kernel|attn_decode_kernel|attn_oproj_kernel' -d /tmp/pmc_f -o pmc --output-format csv -- python3 tools/kernel_probe.py --ctx 2048 --prefill --iters 8 --kernels gate_up,qkv,lm_head,attn,o,down > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed $?"; tail -20 $OUT/pmc_fetch_$TAG.log; exit 1; }
find /tmp/pmc_f -name '*counter_collection.csv' -exec cp {} $OUT/pmc_fetch_$TAG.csv \;
step "pmc write 7B"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'gemv_kernel|attn_decode_kernel|attn_oproj_kernel' -d /tmp/pmc_w -o pmc --output-format csv -- python3 tools/kernel_probe.py --ctx 2048 --prefill --iters 8 --kernels gate_up,qkv,lm_head,attn,o,down > $OUT/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed $?"; tail -20 $OUT/pmc_write_$TAG.log; exit 1; }
find /tmp/pmc_w -name '*counter_collection.csv' -exec cp {} $OUT/pmc_write_$TAG.csv \;
step "pmc fetch 13B int8"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'gemv_kernel|attn_oproj_kernel' -d /tmp/pmc_fi -o pmc --output-format csv -- python3 tools/int8_probe.py 8 i8 eager > $OUT/pmc_fetch_i8_$TAG.log 2>&1 || { echo "pmc fetch i8 failed $?"; tail -20 $OUT/pmc_fetch_i8_$TAG.log; exit 1; }
find /tmp/pmc_fi -name '*counter_collection.csv' -exec cp {} $OUT/pmc_fetch_i8_$TAG.csv \;
step "pmc write 13B int8"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'gemv_kernel|attn_oproj_kernel' -d /tmp/pmc_wi -o pmc --output-format csv -- python3 tools/int8_probe.py 8 i8 eager > $OUT/pmc_write_i8_$TAG.log 2>&1 || { echo "pmc write i8 failed $?"; tail -20 $OUT/pmc_write_i8_$TAG.log; exit 1; }
find /tmp/pmc_wi -name '*counter_collection.csv' -exec cp {} $OUT/pmc_write_i8_$TAG.csv \;
step "int8 probe (graph loop)"
timeout -k 10 200 python3 tools/int8_probe.py 8 > $OUT/int8_probe_$TAG.json 2>&1 || { echo "int8 probe failed"; exit 1; }
cat $OUT/int8_probe_$TAG.json
step "one-shot exchange, two processes on one GPU (7B width)"
timeout -k 10 300 python3 tools/xchg_probe.py llama2-7b 2 > $OUT/xchg_probe_$TAG.json 2> $OUT/xchg_probe_$TAG.err || { echo "xchg probe failed $?"; tail -20 $OUT/xchg_probe_$TAG.err; exit 1; }
cat $OUT/xchg_probe_$TAG.json
step done
