#!/bin/bash
# Quick GPU experiment: gpu suite (optional), kernel probe (attention sweep + 2-layer loop), bench.
#   gpurun -- bash tools/gpu_exp.sh <tag>     (SKIP_TESTS=1, SKIP_BENCH=1, PROBE_ARGS=...)
set -o pipefail
TAG=${1:-exp}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  echo "[$(date +%T)] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed $?"; tail -40 $OUT/pytest_gpu_$TAG.log; exit 1; }
  tail -2 $OUT/pytest_gpu_$TAG.log
fi
echo "[$(date +%T)] probe"
timeout -k 10 300 python3 tools/kernel_probe.py --layers 2 --iters 100 --loop --attn-sweep 8,64,65,128,256,512,1024,2047 $PROBE_ARGS > $OUT/probe_$TAG.json 2> $OUT/probe_$TAG.err || { echo "probe failed $?"; tail -20 $OUT/probe_$TAG.err; exit 1; }
cat $OUT/probe_$TAG.json
if [ -z "$SKIP_BENCH" ]; then
  echo "[$(date +%T)] bench"
  timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 $BENCH_ARGS > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed $?"; tail -20 $OUT/bench_$TAG.err; exit 1; }
  cat $OUT/bench_$TAG.json
fi
echo "[$(date +%T)] done"
