#!/bin/bash
# balanced gate_up in both two-plane modes vs plain; prefill tests; prefill probe.
set -o pipefail
TAG=${1:-bal2}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
step() { echo "[$(date +%T)] $*"; }
step "gate_up: planes 2 plain, fp16-lo balanced (exact data), fp16-lo balanced, lo8 balanced (random)"
timeout -k 10 60 ./tools/gemm_bench/gemm_bench_lo8 512 20 1 gate_up 2 0 > $OUT/bal2_$TAG.jsonl || { echo "p2 failed $?"; exit 1; }
timeout -k 10 60 ./tools/gemm_bench/gemm_bench_lo8 512 10 1 gate_up 5 1 >> $OUT/bal2_$TAG.jsonl || { echo "p5 exact failed $?"; cat $OUT/bal2_$TAG.jsonl; exit 1; }
timeout -k 10 60 ./tools/gemm_bench/gemm_bench_lo8 512 20 1 gate_up 5 0 >> $OUT/bal2_$TAG.jsonl || { echo "p5 failed $?"; cat $OUT/bal2_$TAG.jsonl; exit 1; }
timeout -k 10 60 ./tools/gemm_bench/gemm_bench_lo8 512 20 1 gate_up 4 0 >> $OUT/bal2_$TAG.jsonl || { echo "p4 failed $?"; cat $OUT/bal2_$TAG.jsonl; exit 1; }
cat $OUT/bal2_$TAG.jsonl
step "prefill tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_prefill.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_prefill_$TAG.log 2>&1 || { echo "prefill tests failed $?"; tail -40 $OUT/pytest_prefill_$TAG.log; exit 1; }
grep -E "rel-L2|passed|failed" $OUT/pytest_prefill_$TAG.log
step "prefill probe"
timeout -k 10 300 python3 tools/prefill_probe.py 512 5 > $OUT/prefill_probe_$TAG.json 2>&1 || { echo "probe failed $?"; tail $OUT/prefill_probe_$TAG.json; exit 1; }
cat $OUT/prefill_probe_$TAG.json
step done
