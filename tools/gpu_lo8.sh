#!/bin/bash
# fp8 lo-plane prefill (gemm3 lo8): exact-data k-map check, shape timings vs the fp16
# planes, the prefill tests, the prefill probe.   bash tools/gpu_lo8.sh <tag>
set -o pipefail
TAG=${1:-lo8}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "gemm3 lo8, exact data (k-map check)"
for s in qkv_s2 gate_up down_s8 o_s8; do
  timeout -k 10 60 ./tools/gemm_bench/gemm_bench_lo8 512 5 1 $s 3 1 >> $OUT/gemm_lo8_$TAG.jsonl || { echo "lo8 exact failed $?"; exit 1; }
done
cat $OUT/gemm_lo8_$TAG.jsonl
step "gemm3 planes 1/2/lo8, random data"
for s in qkv_s2 gate_up down_s8 o_s8; do
  timeout -k 10 120 ./tools/gemm_bench/gemm_bench_lo8 512 20 1 $s 0 0 >> $OUT/gemm_all_$TAG.jsonl || { echo "gemm bench failed $?"; exit 1; }
done
cat $OUT/gemm_all_$TAG.jsonl
step "prefill tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_prefill.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_prefill_$TAG.log 2>&1 || { echo "prefill tests failed $?"; tail -40 $OUT/pytest_prefill_$TAG.log; exit 1; }
grep -E "rel-L2|passed|failed" $OUT/pytest_prefill_$TAG.log
step "prefill probe"
timeout -k 10 300 python3 tools/prefill_probe.py 512 5 > $OUT/prefill_probe_$TAG.json 2>&1 || { echo "probe failed $?"; tail $OUT/prefill_probe_$TAG.json; exit 1; }
cat $OUT/prefill_probe_$TAG.json
step done
