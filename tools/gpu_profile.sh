#!/bin/bash
# One GPU session: bench line, rocprofv3 kernel-trace stats of the same bench,
# separate FETCH_SIZE / WRITE_SIZE PMC passes on the gate_up GEMV.
# Usage (on the gpurun box): bash tools/gpu_profile.sh <tag>
#   SKIP_PROFILE=1: tests + bench only;  SKIP_TESTS=1: profiles only
set -o pipefail
TAG=${1:-r02}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -2 $OUT/pytest_gpu_$TAG.log
echo "[$(date +%T)] bench"
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
fi
[ -n "$SKIP_PROFILE" ] && exit 0
if [ -z "$FROM_PMC" ]; then
echo "[$(date +%T)] attention sweep"
timeout -k 10 300 python3 tools/kernel_probe.py --layers 2 --iters 100 --loop --attn-sweep 8,64,65,128,256,512,1024,2047 > $OUT/probe_$TAG.json 2> $OUT/probe_$TAG.err || { echo "probe failed $?"; tail -20 $OUT/probe_$TAG.err; exit 1; }
cat $OUT/probe_$TAG.json
echo "[$(date +%T)] kernel trace"
rm -rf /tmp/prof_trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/prof_trace -o trace --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-side --eager > $OUT/prof_trace_$TAG.log 2>&1 || { echo "trace failed $?"; tail -20 $OUT/prof_trace_$TAG.log; exit 1; }
find /tmp/prof_trace -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats_$TAG.csv \;
python3 tools/trace_summary.py $(find /tmp/prof_trace -name '*kernel_trace.csv' | head -1) > $OUT/trace_summary_$TAG.json || echo "trace summary failed"
fi
echo "[$(date +%T)] pmc fetch"
rm -rf /tmp/pmc_f /tmp/pmc_w
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'gemv_kernel|attn_decode_kernel|attn_oproj_kernel' -d /tmp/pmc_f -o pmc --output-format csv -- python3 tools/kernel_probe.py --ctx 2048 --prefill --iters 8 --kernels gate_up,qkv,lm_head,attn,o,down > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed $?"; tail -20 $OUT/pmc_fetch_$TAG.log; exit 1; }
find /tmp/pmc_f -name '*counter_collection.csv' -exec cp {} $OUT/pmc_fetch_$TAG.csv \;
echo "[$(date +%T)] pmc write"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'gemv_kernel|attn_decode_kernel|attn_oproj_kernel' -d /tmp/pmc_w -o pmc --output-format csv -- python3 tools/kernel_probe.py --ctx 2048 --prefill --iters 8 --kernels gate_up,qkv,lm_head,attn,o,down > $OUT/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed $?"; tail -20 $OUT/pmc_write_$TAG.log; exit 1; }
find /tmp/pmc_w -name '*counter_collection.csv' -exec cp {} $OUT/pmc_write_$TAG.csv \;
echo "[$(date +%T)] prefill trace"
rm -rf /tmp/prof_pf
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_pf -o pf --output-format csv -- python3 tools/prefill_probe.py 512 2 > $OUT/prof_prefill_$TAG.log 2>&1 || { echo "prefill trace failed $?"; tail -20 $OUT/prof_prefill_$TAG.log; exit 1; }
find /tmp/prof_pf -name '*kernel_stats.csv' -exec cp {} $OUT/prefill_kernel_stats_$TAG.csv \;
echo "[$(date +%T)] pmc mfma (prefill GEMM)"
rm -rf /tmp/pmc_m
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE --kernel-include-regex 'gemm[23]?_kernel|attn_prefill' -d /tmp/pmc_m -o pmc --output-format csv -- python3 tools/prefill_probe.py 512 1 > $OUT/pmc_mfma_$TAG.log 2>&1 || { echo "pmc mfma failed $?"; tail -20 $OUT/pmc_mfma_$TAG.log; exit 1; }
find /tmp/pmc_m -name '*counter_collection.csv' -exec cp {} $OUT/pmc_mfma_$TAG.csv \;
echo "[$(date +%T)] counters available"
timeout -k 10 120 rocprofv3 -L > $OUT/rocprof_counters_$TAG.txt 2>&1 || true
echo "[$(date +%T)] done"
ls -la $OUT
